#!/bin/bash
# Round 5: band_sl with two feature-load sets (var_so/sets2.so) against four, on the fused
# passes and the volume (32 pairs); then the SQ set of the final build's volume-free passes
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5aa; mkdir -p "$OUT"; export TMPDIR=/tmp
for r in 1 2 3; do
  for lib in realtime_stereo_matcher_amd/libstereocv.so var_so/sets2.so; do
    STEREOCV_LIB=$lib timeout -k 10 200 python -u scripts/ab_time.py --ops cfg2_fused_nv_b32,cfg2_fused_b32 --reps 10 >> "$OUT/ab.jsonl" 2>> "$OUT/ab.err" || { echo "ab failed"; tail -3 "$OUT/ab.err"; exit 2; }
  done
done
cut -c1-140 "$OUT/ab.jsonl"
bash scripts/gpu_sq.sh r5aa/sq "cfg2_fused_nv_b32 cfg4_fused_nv_b32" || exit 6
