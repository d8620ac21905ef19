#!/bin/bash
# Round 5: cfg2 volume placement -- the slow and the fast buffer under a sequential fill and the
# regression's plane walk, beside the band kernel
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5r; mkdir -p "$OUT"
timeout -k 10 200 python -u scripts/place_ab.py --order "F,V,V" --patterns --reps 5 > "$OUT/o1.jsonl" 2> "$OUT/o1.err" || { tail -3 "$OUT/o1.err"; exit 2; }
cut -c1-150 "$OUT"/o*.jsonl
