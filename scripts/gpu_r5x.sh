#!/bin/bash
# Round 5: band_rs (algo 11) vs band_sl (algo 12) vs band_h2db (algo 8) on the slow (first) and
# a fast cfg2 volume buffer of one process each
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5x; mkdir -p "$OUT"
for r in 1 2; do
  for algo in 11 12 8; do
    echo "== algo $algo" >> "$OUT/place.jsonl"
    timeout -k 10 200 python -u scripts/place_ab.py --algo $algo --order "F,V,V" --reps 5 >> "$OUT/place.jsonl" 2>> "$OUT/place.err" || { tail -3 "$OUT/place.err"; exit 2; }
  done
done
cut -c1-125 "$OUT/place.jsonl"
