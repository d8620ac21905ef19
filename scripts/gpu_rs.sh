#!/bin/bash
# Role-split band kernel: parity (rs tests first, the rest of the file after), then same-box
# timing of cfg2 / cfg4 against band_h2db and band_sp.
#   bash scripts/gpu_rs.sh TAG [pytest -k expr]
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-rs}; K=${2:-rs}
OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_sp.py -x -v -k "$K" --timeout 150 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; tail -15 "$OUT/tests.log"
[ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  timeout -k 10 200 python -u scripts/ab_time.py --ops cfg2_h2db,cfg2_sp,cfg2_rs,cfg4,cfg4_rs --tag r$r >> "$OUT/ab.jsonl" 2>> "$OUT/ab.err" || { tail -5 "$OUT/ab.err"; exit 3; }
done
cat "$OUT/ab.jsonl"
