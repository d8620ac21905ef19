#!/bin/bash
# Same-box A/B of library builds on a list of ops: bash scripts/gpu_ab_ops.sh TAG OPS lib1.so lib2.so ...
# (3 alternating rounds; one JSON line per op and build)
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; OPS=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
for r in 1 2 3; do
  for lib in "$@"; do
    STEREOCV_LIB=$lib timeout -k 10 200 python -u scripts/ab_time.py --ops "$OPS" >> "$OUT/ab.jsonl" 2>> "$OUT/ab.err" || { echo "failed on $lib"; tail -5 "$OUT/ab.err"; exit 2; }
  done
done
cat "$OUT/ab.jsonl"
