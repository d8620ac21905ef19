#!/bin/bash
# Fast iteration pass: GPU parity tests (optionally filtered), ablation timings of one op,
# per-op timings.   usage: bash scripts/gpu_iter.sh TAG OP [pytest -k expr]
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-iter}; OP=${2:-inner_product_mfma_cfg2}; K=${3:-}
OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
if [ -n "$K" ]; then
  timeout -k 10 600 python -m pytest tests -m gpu -q --timeout=300 -p no:cacheprovider -k "$K" > "$OUT/pytest_gpu.log" 2>&1
else
  timeout -k 10 600 python -m pytest tests -m gpu -q --timeout=300 -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
fi
rc=$?; echo "pytest rc=$rc" >> "$OUT/pytest_gpu.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for ab in 0 1 2 4 3 5 6 7; do
  STEREOCV_ABLATE=$ab timeout -k 10 120 python scripts/prof_op.py $OP --reps 10 --time >> "$OUT/ablate.log" 2>&1 || exit 3
done
timeout -k 10 400 python scripts/bench_ops.py > "$OUT/ops.log" 2>&1 || exit 4
exit $rc
