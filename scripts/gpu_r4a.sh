#!/bin/bash
# Round 4, first call: parity of the software-pipelined band kernel, then same-box timing of
# the cfg2 / cfg4 launches against band_h2db.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r4a; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_sp.py -x -v --timeout 150 --timeout-method thread > "$OUT/sp_tests.log" 2>&1
rc=$?; tail -25 "$OUT/sp_tests.log"
[ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  timeout -k 10 200 python -u scripts/ab_time.py --ops cfg2,cfg2_h2db,cfg4 --tag r$r >> "$OUT/ab.jsonl" 2>> "$OUT/ab.err" || { tail -5 "$OUT/ab.err"; exit 3; }
done
cat "$OUT/ab.jsonl"
