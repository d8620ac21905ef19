#!/bin/bash
# b16 band kernel: parity tests (b16 cases), then same-box timing against band_h2.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-b16}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "b16" -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -15 "$OUT/pytest.log"
[ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  timeout -k 10 200 python -u scripts/ab_time.py --ops cfg2_h2,cfg2_b16 >> "$OUT/ab.jsonl" 2>> "$OUT/ab.err" || { tail -5 "$OUT/ab.err"; exit 3; }
done
cat "$OUT/ab.jsonl"
