#!/bin/bash
# Round 5: cfg2 volume placement -- allocation order (features first / volumes first / spacers)
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5q; mkdir -p "$OUT"
i=0
for o in "F,V,V" "V,V,F" "F,S1024,V,V" "F,S64,V,V" "F,S13000,V"; do
  i=$((i+1))
  timeout -k 10 200 python -u scripts/place_ab.py --order "$o" --reps 5 > "$OUT/o$i.jsonl" 2> "$OUT/o$i.err" || { tail -3 "$OUT/o$i.err"; exit 2; }
done
cut -c1-150 "$OUT"/o*.jsonl
