#!/bin/bash
# Round 5: load / store cache policies of the sliding-window kernel, cfg2 32-pair launch, same box
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5c; mkdir -p "$OUT"; export TMPDIR=/tmp
for r in 1 2; do
  for lib in realtime_stereo_matcher_amd/libstereocv.so var_so/sl_ntl.so var_so/sl_plst.so var_so/sl_ntl_plst.so var_so/sl_ntl_s8.so; do
    STEREOCV_LIB=$lib timeout -k 10 200 python -u scripts/ab_time.py --ops cfg2_b32_sl,cfg4_b32,cfg2_fused_nv_b32 --reps 10 >> "$OUT/ab.jsonl" 2>> "$OUT/ab.err" || { echo "failed on $lib"; tail -5 "$OUT/ab.err"; exit 2; }
  done
done
cat "$OUT/ab.jsonl"
