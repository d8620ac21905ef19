#!/bin/bash
# b16 vs h2 diagnostics (binaries prebuilt by scripts/build_stamps.sh): phase stamps of both
# kernels at 8 cfg2 pairs per launch, ablation timings, and the store-pattern micro-benchmark.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-b16diag}; mkdir -p "$OUT"; export TMPDIR=/tmp
for m in h2 b16; do
  timeout -k 10 60 bin/stamps/ip_stamps 192 $m 8 > "$OUT/stamps_$m.log" 2>&1 || { cat "$OUT/stamps_$m.log"; exit 3; }
  cat "$OUT/stamps_$m.log"
done
for r in 1 2; do for ab in 0 1 4 8 16; do for m in h2 b16; do
  echo -n "ablate=$ab $m: "; timeout -k 10 60 bin/stamps/ip_ab$ab 192 $m 8 > "$OUT/ab.tmp" 2>&1 || { cat "$OUT/ab.tmp"; exit 5; }
  head -1 "$OUT/ab.tmp"
done; done; done
timeout -k 10 120 bin/store_patterns > "$OUT/store_patterns.log" 2>&1 || exit 6
cat "$OUT/store_patterns.log"
