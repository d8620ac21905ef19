#!/bin/bash
# Round 5: write schedules of the cfg2 traffic (scripts/micro/sl_pattern.hip), box identified
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5i; mkdir -p "$OUT"; export TMPDIR=/tmp
(hostname; rocm-smi --showuniqueid --showmemorypartition --showcomputepartition --showclocks 2>&1 | grep -v "^=\|^$") > "$OUT/box.txt" 2>&1
timeout -k 10 300 ./scripts/micro/sl_pattern_bin 32 > "$OUT/slp32.jsonl" 2>&1 || { echo "micro failed"; exit 3; }
timeout -k 10 200 python -u scripts/ab_time.py --ops cfg2_b32_sl,cfg2_b32_rs --reps 10 >> "$OUT/ab.jsonl" 2>> "$OUT/ab.err" || { echo "ab failed"; exit 2; }
cat "$OUT/box.txt" "$OUT/slp32.jsonl" "$OUT/ab.jsonl"
