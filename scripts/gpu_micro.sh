#!/bin/bash
# Memory-pattern micro-benchmarks (prebuilt in bin/): store shapes, read+write floor, LDS-DMA mix.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-micro}; mkdir -p "$OUT"
for b in rw_patterns mlp_patterns; do
  echo "== $b"; timeout -k 10 120 bin/$b > "$OUT/$b.log" 2>&1 || { cat "$OUT/$b.log"; exit 3; }
  cat "$OUT/$b.log"
done
