#!/bin/bash
# Warm per-pair cost of band_rs against pairs per launch (scripts/rs_stamps.hip, built in-tree):
# about 1.5 s of back-to-back launches before the stamped one.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-sweep}; mkdir -p "$OUT"
for args in "4 16 256 1080 1920 1 750" "8 16 256 1080 1920 1 400" "16 16 256 1080 1920 1 200" "32 16 256 1080 1920 1 110" \
            "2 64 192 540 960 0 5000" "8 64 192 540 960 0 1400" "16 64 192 540 960 0 700" "32 64 192 540 960 0 350" \
            "4 16 256 1080 1920 1 750" "32 64 192 540 960 0 350" "8 64 192 540 960 0 1400"; do
  echo "== $args" >> "$OUT/stamps.log"
  timeout -k 10 120 ./scripts/rs_stamps_bin $args >> "$OUT/stamps.log" 2>&1 || { echo "failed on $args"; exit 2; }
done
grep -E "^==|band_rs|compute lifetime" "$OUT/stamps.log"
