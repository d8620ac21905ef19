#!/bin/bash
# Round bench + evidence: the bench line, a kernel-trace/stats profile of the same command,
# and the two HBM counter passes (FETCH_SIZE, WRITE_SIZE; one --pmc per run, kernel trace only).
# usage: bash scripts/gpu_bench_prof.sh TAG [extra bench args]
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-bench}; shift
OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 300 python bench.py "$@" > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o run --output-format csv -- \
  python3 bench.py --steps 20 --warmup 5 --cpu-baseline-seconds 0 "$@" > "$OUT/kt.json" 2> "$OUT/kt.err" || exit 3
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- \
  python3 bench.py --steps 5 --warmup 2 --cpu-baseline-seconds 0 "$@" > "$OUT/fetch.log" 2>&1 || exit 4
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- \
  python3 bench.py --steps 5 --warmup 2 --cpu-baseline-seconds 0 "$@" > "$OUT/write.log" 2>&1 || exit 5
exit 0
