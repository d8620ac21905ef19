#!/bin/bash
# band_h2ws on the GPU: its parity tests, then a same-box A/B of cfg2 (and the cfg4 split pass)
# against band_h2db.   bash scripts/gpu_h2ws.sh TAG
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-h2ws}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "h2ws" \
  --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 2; }
tail -2 "$OUT/pytest.log"
for r in 1 2 3; do
  timeout -k 10 200 python -u scripts/ab_time.py --ops cfg2_h2db,cfg2_h2ws >> "$OUT/ab.jsonl" 2>> "$OUT/ab.err" || { tail -5 "$OUT/ab.err"; exit 2; }
done
cat "$OUT/ab.jsonl"
