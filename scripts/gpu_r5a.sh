#!/bin/bash
# Round 5, first sliding-window run: its parity on small shapes, then same-box A/B against
# band_rs on the bench launches, then the rest of the band parity tests.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5a; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_sp.py \
  -k "sl and not bench" > "$OUT/sl_small.log" 2>&1 || { echo "sl small FAILED"; tail -30 "$OUT/sl_small.log"; exit 2; }
echo "sl small ok"; tail -2 "$OUT/sl_small.log"
for r in 1 2; do
  timeout -k 10 300 python -u scripts/ab_time.py --ops cfg2_b32_rs,cfg2_b32_sl,cfg4_b32_rs,cfg4_b32,cfg4_rs,cfg4_b4_auto --reps 15 --tag lib >> "$OUT/ab.jsonl" 2>> "$OUT/ab.err" || { echo "ab failed"; tail -5 "$OUT/ab.err"; exit 3; }
done
for lib in var_so/nosl_fuse.so realtime_stereo_matcher_amd/libstereocv.so; do
  STEREOCV_LIB=$lib timeout -k 10 300 python -u scripts/ab_time.py --ops cfg2_fused_b32,cfg2_fused_nv_b32,cfg4_fused_nv_b32 --reps 15 >> "$OUT/ab_fused.jsonl" 2>> "$OUT/ab.err" || { echo "ab fused failed"; tail -5 "$OUT/ab.err"; exit 4; }
done
cat "$OUT/ab.jsonl" "$OUT/ab_fused.jsonl"
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_sp.py tests/test_gpu_parity.py > "$OUT/gpu_band.log" 2>&1
echo "band tests rc=$?"; grep -E "passed|failed" "$OUT/gpu_band.log" | tail -3; grep -E "^FAILED" "$OUT/gpu_band.log" | head -20
