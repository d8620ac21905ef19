#!/bin/bash
# Quick A/B call: band kernel variants (prebuilt bin/wsa_*), warp parity + timings.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-ca}; mkdir -p "$OUT"
for n in base z1 base z1 base z1; do
  echo -n "$n: " >> "$OUT/ab.log"
  timeout -k 10 60 bin/wsa_$n h2 >> "$OUT/ab.log" 2>&1 || exit 3
done
cat "$OUT/ab.log"
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -k "warp" --timeout 120 --timeout-method thread > "$OUT/warp_tests.log" 2>&1 || { tail -20 "$OUT/warp_tests.log"; exit 4; }
tail -2 "$OUT/warp_tests.log"
timeout -k 10 200 python scripts/bench_ops.py --only warp_disp_f32_540x960x32,warp_smooth_disp_f32_540x960x32,warp_flow2_f32_540x960x32 > "$OUT/warp_ops.log" 2>&1 || { tail -20 "$OUT/warp_ops.log"; exit 5; }
cat "$OUT/warp_ops.log"
exit 0
