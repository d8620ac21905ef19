#!/bin/bash
# After switching cfg2's volume-free pass to band_rs FUSE 2: the -m gpu suite, smoke, and the
# fused evidence (bench line, kernel trace, HBM counters) for cfg2 fused-novolume.
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-fuse2ev}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || { tail -30 "$OUT/gpu_tests.log"; exit 3; }
tail -1 "$OUT/gpu_tests.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 4; }
tail -1 "$OUT/smoke.log"
bash scripts/gpu_evidence.sh "$TAG/ev" "cfg2_fused_novolume:--config cfg2 --pipeline fused-novolume" || exit 5
timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 6
python3 -c "import json; r=json.load(open('$OUT/bench.json')); print('default bench', round(r['value'],1), round(r['roofline']['frac'],4))"
