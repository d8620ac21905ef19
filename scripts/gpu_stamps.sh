#!/bin/bash
# Per-role phase stamps and finishing-time spread of band_rs (scripts/rs_stamps.hip, built
# in-tree beforehand) for the 8- / 32-pair cfg2 and 4- / 32-pair cfg4 launches.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-stamps}; mkdir -p "$OUT"
for args in "8 64 192" "32 64 192" "4 16 256 1080 1920 1" "32 16 256 1080 1920 1"; do
  echo "== $args" >> "$OUT/stamps.log"
  timeout -k 10 120 ./scripts/rs_stamps_bin $args >> "$OUT/stamps.log" 2>&1 || { echo "failed on $args"; exit 2; }
done
cat "$OUT/stamps.log"
