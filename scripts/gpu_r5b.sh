#!/bin/bash
# Round 5: ablations of the sliding-window kernel on the bench's 32-pair cfg2 launch (same box)
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5b; mkdir -p "$OUT"; export TMPDIR=/tmp
for r in 1 2; do
  for lib in realtime_stereo_matcher_amd/libstereocv.so var_so/sl_ab1.so var_so/sl_ab2.so var_so/sl_ab4.so var_so/sl_ab8.so \
             var_so/sl_ab16.so var_so/sl_ab32.so var_so/sl_ab64.so var_so/sl_ab6.so var_so/sl_ab20.so var_so/sl_sets8.so; do
    STEREOCV_LIB=$lib timeout -k 10 120 python -u scripts/ab_time.py --ops cfg2_b32_sl --reps 10 >> "$OUT/ab.jsonl" 2>> "$OUT/ab.err" || { echo "failed on $lib"; tail -5 "$OUT/ab.err"; exit 2; }
  done
done
cat "$OUT/ab.jsonl"
