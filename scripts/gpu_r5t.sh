#!/bin/bash
# Round 5: XCD-interleaved segment chunks (SMCV_SCHED_IL, band_rs) against contiguous XCD ranges,
# on the slow (first) and a fast volume buffer of one process each
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r5t}; mkdir -p "$OUT"
for r in 1 2; do
  for lib in realtime_stereo_matcher_amd/libstereocv.so var_so/il64.so var_so/il16.so var_so/il8.so; do
    echo "== $lib" >> "$OUT/place.jsonl"
    STEREOCV_LIB=$lib timeout -k 10 200 python -u scripts/place_ab.py --order "F,V,V" --reps 5 >> "$OUT/place.jsonl" 2>> "$OUT/place.err" || { tail -3 "$OUT/place.err"; exit 2; }
  done
done
grep -v "zero_\|soft_argmin" "$OUT/place.jsonl" | cut -c1-130
