#!/bin/bash
# Ablation timings of one op: bash scripts/gpu_ablate.sh TAG OP "bits..."
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-abl}; OP=${2:-inner_product_h2_cfg2}; BITS=${3:-0 1 2 4 8 16}
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
for ab in $BITS; do
  STEREOCV_ABLATE=$ab timeout -k 10 120 python scripts/prof_op.py $OP --reps 10 --time >> "$OUT/ablate.log" 2>&1 || exit 3
done
exit 0
