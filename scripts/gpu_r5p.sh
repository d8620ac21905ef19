#!/bin/bash
# Round 5: cfg2 volume placement -- five 32-pair volume buffers allocated in a row, with the
# default caching allocator and with expandable segments
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5p; mkdir -p "$OUT"
timeout -k 10 200 python -u scripts/place_ab.py --seq 5 --reps 5 > "$OUT/seq_default.jsonl" 2> "$OUT/seq_default.err" || exit 2
PYTORCH_HIP_ALLOC_CONF=expandable_segments:True timeout -k 10 200 python -u scripts/place_ab.py --seq 5 --reps 5 > "$OUT/seq_expandable.jsonl" 2> "$OUT/seq_expandable.err" || exit 3
cut -c1-200 "$OUT"/seq_*.jsonl
