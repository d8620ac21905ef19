#!/bin/bash
# A/B of prebuilt bin/wsa_<name> variants in one mode, interleaved.   bash scripts/gpu_ab2.sh TAG MODE "names"
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$1; mkdir -p "$OUT"
for r in 1 2 3; do
  for n in $3; do
    echo -n "$n: " >> "$OUT/ab.log"
    timeout -k 10 60 bin/wsa_$n $2 >> "$OUT/ab.log" 2>&1 || exit 3
  done
done
cat "$OUT/ab.log"
