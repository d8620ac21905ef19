#!/bin/bash
# Round 5: the sliding pattern under three workgroup -> row maps (scripts/micro/sl_pattern.hip)
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5e; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 300 ./scripts/micro/sl_pattern_bin 32 > "$OUT/slp32.jsonl" 2>&1 || { echo "micro failed"; cat "$OUT/slp32.jsonl"; exit 3; }
cat "$OUT/slp32.jsonl"
