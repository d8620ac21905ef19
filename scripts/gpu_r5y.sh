#!/bin/bash
# Round 5: the fused fold with 1/C and 2^kk in the exponent's FMA (var_so/foldfma.so, band_sl)
# against the library -- fused parity on the variant, then 32-pair A/B
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5y; mkdir -p "$OUT"; export TMPDIR=/tmp
STEREOCV_LIB=var_so/foldfma.so timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_sp.py -k "fused" > "$OUT/tests.log" 2>&1
rc=$?; grep -E "passed|failed" "$OUT/tests.log" | tail -1; grep -E "^FAILED" "$OUT/tests.log" | head; [ $rc -le 1 ] || exit $rc
for r in 1 2 3; do
  for lib in realtime_stereo_matcher_amd/libstereocv.so var_so/foldfma.so; do
    STEREOCV_LIB=$lib timeout -k 10 200 python -u scripts/ab_time.py --ops cfg2_fused_nv_b32,cfg4_fused_nv_b32,cfg2_fused_b32 --reps 10 >> "$OUT/ab.jsonl" 2>> "$OUT/ab.err" || { echo "ab failed"; tail -3 "$OUT/ab.err"; exit 2; }
  done
done
cut -c1-140 "$OUT/ab.jsonl"
