#!/bin/bash
# h2 experiments: stagger sweep (library, prof_op timings) and ablation stamps.
#   bash scripts/gpu_h2_exp.sh TAG "staggers" "ablate bits"
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-exp}; STAG=${2:-0 2 4 8}; ABS=${3:-0 2 8 10}
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
for sg in $STAG; do
  STEREOCV_H2_STAGGER=$sg timeout -k 10 120 python scripts/prof_op.py inner_product_h2_cfg2 --reps 20 --time >> "$OUT/stagger.log" 2>&1 || exit 3
  echo "stagger=$sg" >> "$OUT/stagger.log"
done
for ab in $ABS; do
  hipcc -O3 -std=c++17 --offload-arch=gfx950 -DSMCV_STAMPS -DSMCV_ABLATE=$ab -Iinclude scripts/ip_stamps.hip -o /tmp/ip_stamps_$ab > "$OUT/build_$ab.log" 2>&1 || exit 2
  echo "== ablate $ab" >> "$OUT/stamps.log"
  timeout -k 10 60 /tmp/ip_stamps_$ab 192 h2 >> "$OUT/stamps.log" 2>&1 || exit 4
done
exit 0
