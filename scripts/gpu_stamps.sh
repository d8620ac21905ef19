#!/bin/bash
# Build and run the phase-stamp diagnostic of the band kernels on the GPU box.
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-stamps}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
hipcc -O3 -std=c++17 --offload-arch=gfx950 -DSMCV_STAMPS -Iinclude scripts/ip_stamps.hip -o /tmp/ip_stamps > "$OUT/build.log" 2>&1 || exit 2
timeout -k 10 120 /tmp/ip_stamps 192 f32 > "$OUT/stamps_f32.log" 2>&1 || exit 3
timeout -k 10 120 /tmp/ip_stamps 192 bf16x3 > "$OUT/stamps_bf16x3.log" 2>&1 || exit 4
exit 0
