#!/bin/bash
# GPU-box run: -m gpu tests, then every bench config (one JSON line each) into gpurun_out/$TAG.
#   bash scripts/gpu_round.sh TAG [skip-tests]
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-round}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread \
    > "$OUT/gpu_tests.log" 2>&1 || { tail -30 "$OUT/gpu_tests.log"; exit 3; }
  tail -2 "$OUT/gpu_tests.log"
fi
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 240 python -u bench.py "$@" > "$OUT/bench_$n.json" 2> "$OUT/bench_$n.err" || {
    echo "bench $n failed"; tail -20 "$OUT/bench_$n.err"; exit 4; }
  echo "$n: $(python -c "import json,sys; r=json.load(open('$OUT/bench_$n.json')); print(round(r['value'],1), r['unit'], 'kernel_us', round(r['roofline']['avg_kernel_us'],1), 'frac', round(r['roofline']['frac'],3), r.get('numerics'))")"
}
run cfg2 --config cfg2
run cfg2_fused_novolume --config cfg2 --pipeline fused-novolume --cpu-baseline-seconds 0
run cfg2_fused --config cfg2 --pipeline fused --cpu-baseline-seconds 0
run cfg3 --config cfg3
run cfg4 --config cfg4
run cfg5 --config cfg5
run cfg5_interweave --config cfg5 --pipeline interweave
exit 0
