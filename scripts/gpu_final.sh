#!/bin/bash
# Round-end rehearsal of the driver's GPU steps: -m gpu tests, smoke(), the default bench line.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-final}; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || { tail -30 "$OUT/gpu_tests.log"; exit 3; }
tail -2 "$OUT/gpu_tests.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 4; }
tail -3 "$OUT/smoke.log"
timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 5; }
cat "$OUT/bench.json"
