#!/bin/bash
# Round 5: autocast reference-semantics fused fold + cfg4 N=8 rank launch tests; cfg3 store policy A/B
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5l; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_autocast.py tests/test_gpu_sp.py tests/test_library_ops.py tests/test_gpu_parity.py > "$OUT/tests.log" 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" "$OUT/tests.log" | tail -2; grep -E "^FAILED|Error" "$OUT/tests.log" | head -20
[ $rc -le 1 ] || exit $rc
for r in 1 2; do
  for lib in realtime_stereo_matcher_amd/libstereocv.so var_so/rs_plainst.so var_so/nosl_half.so var_so/sl_nooffload.so; do
    STEREOCV_LIB=$lib timeout -k 10 200 python -u scripts/ab_time.py --ops cfg3,cfg2_b32,cfg2_fused_nv_f16_b32,cfg2_fused_nv_b32,cfg4_fused_nv_b32 --reps 10 >> "$OUT/ab.jsonl" 2>> "$OUT/ab.err" || { echo "ab failed"; tail -3 "$OUT/ab.err"; exit 2; }
  done
done
cat "$OUT/ab.jsonl"
