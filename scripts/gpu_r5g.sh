#!/bin/bash
# Round 5: footprint calibration -- the r03 band_rs-pattern micro (1 pair) and the sliding micro at 1 / 2 / 32 pairs
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5h; mkdir -p "$OUT"; export TMPDIR=/tmp
true
for np in 32; do
  timeout -k 10 300 ./scripts/micro/sl_pattern_bin $np > "$OUT/slp$np.jsonl" 2>&1 || { echo "micro failed"; exit 3; }
done
cat "$OUT"/slp*.jsonl
