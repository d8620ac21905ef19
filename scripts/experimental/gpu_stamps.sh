#!/bin/bash
# Build and run the phase-stamp diagnostic of the band kernels on the GPU box.
#   bash scripts/gpu_stamps.sh TAG "kernels" "ablate bits"   (kernels: ws f32 bf16x3)
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-stamps}; KS=${2:-ws f32 bf16x3}; ABS=${3:-0}; XF=${4:-}
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
for ab in $ABS; do
  hipcc -O3 -std=c++20 --offload-arch=gfx950 -fno-slp-vectorize -DSMCV_STAMPS -DSMCV_ABLATE=$ab $XF -Iinclude scripts/ip_stamps.hip -o /tmp/ip_stamps_$ab > "$OUT/build_$ab.log" 2>&1 || exit 2
done
for ab in $ABS; do
  for k in $KS; do
    echo "== ablate $ab" >> "$OUT/stamps_$k.log"
    timeout -k 10 120 /tmp/ip_stamps_$ab 192 $k >> "$OUT/stamps_$k.log" 2>&1 || exit 3
  done
done
exit 0
