#!/bin/bash
# Same-box A/B of variant library builds (var_so/*.so, scripts/build_variants.py) on one op:
#   bash scripts/gpu_ab_var.sh TAG OP "name1 name2 ..."   (2 alternating rounds)
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; OP=$2; NAMES=$3
OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
for r in 1 2; do
  for n in $NAMES; do
    lib=var_so/$n.so; [ "$n" = default ] && lib=realtime_stereo_matcher_amd/libstereocv.so
    STEREOCV_LIB=$lib timeout -k 10 120 python -u scripts/ab_time.py --ops "$OP" --reps 15 --tag $n >> "$OUT/ab.jsonl" 2>> "$OUT/ab.err" || { echo "failed on $n"; tail -5 "$OUT/ab.err"; exit 2; }
  done
done
cat "$OUT/ab.jsonl"
