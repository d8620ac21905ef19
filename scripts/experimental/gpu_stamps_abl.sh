#!/bin/bash
# Phase stamps of band_h2 and band_b16 (8 cfg2 pairs per launch) in the full build and in the
# stamped ablation builds (bin/stamps/st_ab<N>: -DSMCV_STAMPS -DSMCV_ABLATE=N).
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-stabl}; mkdir -p "$OUT"; export TMPDIR=/tmp
for b in ip_stamps st_ab4 st_ab1 st_ab16; do for m in h2 b16; do
  echo "== $b $m"
  timeout -k 10 60 bin/stamps/$b 192 $m 8 > "$OUT/$b.$m.log" 2>&1 || { cat "$OUT/$b.$m.log"; exit 3; }
  cat "$OUT/$b.$m.log"
done; done
