#!/bin/bash
# parity subset + phase stamps + op timings
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-iter}; K=${2:-"inner_product or correlation or argext or cfg2 or cfg4 or noncontig or zero"}
OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q --timeout=300 -p no:cacheprovider -k "$K" > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc" >> "$OUT/pytest_gpu.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
hipcc -O3 -std=c++17 --offload-arch=gfx950 -DSMCV_STAMPS -Iinclude scripts/ip_stamps.hip -o /tmp/ip_stamps > "$OUT/build.log" 2>&1 || exit 2
timeout -k 10 120 /tmp/ip_stamps 192 > "$OUT/stamps.log" 2>&1 || exit 3
timeout -k 10 400 python scripts/bench_ops.py --only inner_product_mfma_cfg2,correlation_cfg4_pair,soft_argmin_cfg2 > "$OUT/ops.log" 2>&1 || exit 4
exit $rc
