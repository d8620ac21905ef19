#!/bin/bash
# Round 5: cfg2 volume placement -- torch, plain hipMalloc and contiguous (hipExtMallocWithFlags)
# volume buffers in three allocation orders
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5v; mkdir -p "$OUT"
i=0
for o in "F,V,H,C" "F,C,V,V" "F,V,V,C"; do
  i=$((i+1))
  timeout -k 10 200 python -u scripts/place_ab.py --order "$o" --reps 5 > "$OUT/o$i.jsonl" 2> "$OUT/o$i.err" || { tail -3 "$OUT/o$i.err"; exit 2; }
done
cut -c1-125 "$OUT"/o*.jsonl
