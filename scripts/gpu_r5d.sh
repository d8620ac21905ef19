#!/bin/bash
# Round 5: the sliding kernel's memory pattern without arithmetic (scripts/micro/sl_pattern.hip)
# beside the kernel itself, same box
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5d; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/ab_time.py --ops cfg2_b32_sl,cfg2_b32_rs --reps 10 >> "$OUT/ab.jsonl" 2>> "$OUT/ab.err" || { echo "ab failed"; exit 2; }
timeout -k 10 240 ./scripts/micro/sl_pattern_bin 32 > "$OUT/slp32.jsonl" 2>&1 || { echo "micro failed"; cat "$OUT/slp32.jsonl"; exit 3; }
timeout -k 10 120 ./scripts/micro/sl_pattern_bin 8 > "$OUT/slp8.jsonl" 2>&1 || { echo "micro8 failed"; exit 4; }
timeout -k 10 200 python -u scripts/ab_time.py --ops cfg2_b32_sl,cfg2_b32_rs --reps 10 >> "$OUT/ab.jsonl" 2>> "$OUT/ab.err" || { echo "ab failed"; exit 2; }
cat "$OUT/ab.jsonl" "$OUT/slp32.jsonl" "$OUT/slp8.jsonl"
