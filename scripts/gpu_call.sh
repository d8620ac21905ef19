#!/bin/bash
# Round 6: one parametrised GPU call (replaces the one-shot gpu_r5*.sh launchers).
#   scripts/gpu_call.sh NAME STEP [STEP ...]
# STEP: tests:<pytest -k expression or file list, '+'-separated>  (GPU tests, one process)
#       ab:<lib specs, '+'-separated>:<cases>[:<extra args, '+'-separated>]  (scripts/ab_libs.py)
#       bench:<bench.py args, '+'-separated>                      (one JSON line -> NAME/bench.jsonl)
#       py:<script + args, '+'-separated>                         (any scripts/*.py, -> NAME/py.log)
#       bin:<program + args, '+'-separated>                       (a micro-benchmark, -> NAME/bin.log)
# Every step runs under its own time limit; the first failing step ends the call.
cd "$GRAFT_REPO_ROOT" || exit 1
NAME=$1; shift
OUT=gpurun_out/$NAME; mkdir -p "$OUT"
for step in "$@"; do
  kind=${step%%:*}; arg=${step#*:}
  case $kind in
    tests)
      timeout -k 10 900 python -u -m pytest ${arg//+/ } -m gpu -v --maxfail=5 --timeout 300 --timeout-method thread \
        -p no:cacheprovider > "$OUT/tests.log" 2>&1; rc=$?
      tail -4 "$OUT/tests.log"; [ $rc -eq 0 ] || { echo "tests rc $rc"; exit $rc; } ;;
    ab)
      libs=${arg%%:*}; rest=${arg#*:}; cases=${rest%%:*}; extra=""
      [ "$rest" != "$cases" ] && extra=${rest#*:}
      timeout -k 10 600 python -u scripts/ab_libs.py ${libs//+/ } --cases "$cases" ${extra//+/ } >> "$OUT/ab.jsonl" 2>> "$OUT/ab.err"; rc=$?
      [ $rc -eq 0 ] || { tail -5 "$OUT/ab.err"; exit $rc; } ;;
    bench)
      timeout -k 10 600 python -u bench.py ${arg//+/ } >> "$OUT/bench.jsonl" 2>> "$OUT/bench.err"; rc=$?
      [ $rc -eq 0 ] || { tail -5 "$OUT/bench.err"; exit $rc; } ;;
    py)
      timeout -k 10 600 python -u ${arg//+/ } >> "$OUT/py.log" 2>&1; rc=$?
      [ $rc -eq 0 ] || { tail -5 "$OUT/py.log"; exit $rc; } ;;
    bin)
      timeout -k 10 300 ${arg//+/ } >> "$OUT/bin.log" 2>&1; rc=$?
      [ $rc -eq 0 ] || { tail -5 "$OUT/bin.log"; exit $rc; } ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "all steps ok"
