#!/bin/bash
# Round 5: fp16-rounded fused fold on packed converts + mixed FMA -- parity, then A/B against
# the previous build (var_so/base.so) on the 32-pair fp16 volume-free cfg2 launch
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5s; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_autocast.py tests/test_gpu_parity.py -k "autocast or fused" > "$OUT/tests.log" 2>&1
rc=$?; grep -E "passed|failed" "$OUT/tests.log" | tail -1; grep -E "^FAILED" "$OUT/tests.log" | head; [ $rc -le 1 ] || exit $rc
for r in 1 2 3; do
  for lib in realtime_stereo_matcher_amd/libstereocv.so var_so/base.so; do
    STEREOCV_LIB=$lib timeout -k 10 200 python -u scripts/ab_time.py --ops cfg2_fused_nv_f16_b32 --reps 10 >> "$OUT/ab.jsonl" 2>> "$OUT/ab.err" || { echo "ab failed"; tail -3 "$OUT/ab.err"; exit 2; }
  done
done
cut -c1-160 "$OUT/ab.jsonl"
