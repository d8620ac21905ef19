#!/bin/bash
# Iteration pass for the band kernels: filtered GPU parity tests, phase stamps, op timings.
#   bash scripts/gpu_h2.sh TAG [pytest -k expr] [ops]
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-h2}; K=${2:-"inner_product or correlation or cfg2 or cfg4 or noncontig or zero"}
OPS=${3:-inner_product_h2_cfg2,correlation_cfg4_pair,soft_argmin_cfg2}
OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "$K" > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc" >> "$OUT/pytest_gpu.log"
if [ $rc -ne 0 ]; then exit $rc; fi
hipcc -O3 -std=c++17 --offload-arch=gfx950 -DSMCV_STAMPS -Iinclude scripts/ip_stamps.hip -o /tmp/ip_stamps > "$OUT/build.log" 2>&1 || exit 2
timeout -k 10 60 /tmp/ip_stamps 192 h2 > "$OUT/stamps.log" 2>&1 || exit 3
timeout -k 10 300 python scripts/bench_ops.py --only "$OPS" > "$OUT/ops.log" 2>&1 || exit 4
exit 0
