#!/bin/bash
# Per-role phase stamps, finishing-time spread and in-kernel clock of band_rs
# (scripts/rs_stamps.hip, built in-tree beforehand): cfg2 8 / 32 pairs and cfg4 4 / 32 pairs per
# launch, each after 3 launches and after about 2 s of back-to-back launches.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-stamps}; mkdir -p "$OUT"
for args in "8 64 192 540 960 0 3" "8 64 192 540 960 0 2000" "32 64 192 540 960 0 3" "32 64 192 540 960 0 500" \
            "4 16 256 1080 1920 1 3" "4 16 256 1080 1920 1 1000" "32 16 256 1080 1920 1 3" "32 16 256 1080 1920 1 150"; do
  echo "== $args" >> "$OUT/stamps.log"
  timeout -k 10 120 ./scripts/rs_stamps_bin $args >> "$OUT/stamps.log" 2>&1 || { echo "failed on $args"; exit 2; }
done
grep -E "^==|band_rs|compute lifetime" "$OUT/stamps.log"
