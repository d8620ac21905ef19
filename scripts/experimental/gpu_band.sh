#!/bin/bash
# Iteration pass for the band kernels (inner product, correlation, groupwise, fused soft-argmin)
# and the regression kernels: filtered GPU parity tests, phase stamps, op timings.
#   bash scripts/gpu_band.sh TAG [pytest -k expr] [ops]
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-band}
K=${2:-"inner_product or correlation or groupwise or fused or cfg2 or cfg3 or cfg4 or noncontig or zero or regression or softargmin or argext"}
OPS=${3:-inner_product_h2_cfg2,fused_ip_softargmin_cfg2,fused_ip_softargmin_novol_cfg2,soft_argmin_cfg2,hard_argmax_cfg2,groupwise_bf16_cfg3,correlation_cfg4_pair,concat_fp16_cfg5}
OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "$K" > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc" >> "$OUT/pytest_gpu.log"
if [ $rc -ne 0 ]; then exit $rc; fi
hipcc -O3 -std=c++17 --offload-arch=gfx950 -DSMCV_STAMPS -Iinclude scripts/ip_stamps.hip -o /tmp/ip_stamps > "$OUT/build.log" 2>&1 || exit 2
for M in h2 fused fusednv gw; do
  timeout -k 10 60 /tmp/ip_stamps 192 $M > "$OUT/stamps_$M.log" 2>&1 || exit 3
done
hipcc -O3 -std=c++17 --offload-arch=gfx950 -DSMCV_STAMPS -DSMCV_PREFETCH=0 -Iinclude scripts/ip_stamps.hip -o /tmp/ip_stamps_nopf > "$OUT/build_nopf.log" 2>&1 || exit 2
timeout -k 10 60 /tmp/ip_stamps_nopf 192 h2 > "$OUT/stamps_h2_nopf.log" 2>&1 || exit 3
timeout -k 10 300 python scripts/bench_ops.py --only "$OPS" > "$OUT/ops.log" 2>&1 || exit 4
exit 0
