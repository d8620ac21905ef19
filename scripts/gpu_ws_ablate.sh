#!/bin/bash
# Build the ws ablation variants and time them on the GPU box.
#   bash scripts/gpu_ws_ablate.sh TAG "ablate bits" "modes" "extra flags"
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-wsab}; ABS=${2:-0}; MODES=${3:-ws}; XF=${4:-}
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
for ab in $ABS; do
  hipcc -O3 -std=c++20 --offload-arch=gfx950 -DSMCV_ABLATE=$ab $XF -Iinclude scripts/ws_ablate.hip -o /tmp/wsa_$ab > "$OUT/build_$ab.log" 2>&1 || exit 2
done
for ab in $ABS; do
  for m in $MODES; do
    timeout -k 10 60 /tmp/wsa_$ab $m >> "$OUT/ablate.log" 2>&1 || exit 3
  done
done
exit 0
