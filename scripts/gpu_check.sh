#!/bin/bash
# GPU pass: parity tests, smoke, per-op timings, bench, rocprofv3 kernel trace.
# usage: bash scripts/gpu_check.sh [tag] [quick]
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
rc=$?
echo "pytest rc=$rc" >> "$OUT/pytest_gpu.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit 3
timeout -k 10 400 python scripts/bench_ops.py > "$OUT/ops.log" 2>&1 || exit 4
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --cpu-baseline-seconds 5 > "$OUT/bench_auto.log" 2>&1 || exit 5
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o bench -- python3 bench.py --steps 20 --warmup 5 --cpu-baseline-seconds 0 > "$OUT/prof.log" 2>&1 || exit 6
exit $rc
