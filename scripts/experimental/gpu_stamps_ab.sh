#!/bin/bash
# Phase stamps (N-pair cfg2 launch) of the band kernel plus ablation timings; binaries prebuilt
# here into bin/stamps/ (scripts/ip_stamps.hip, -DSMCV_STAMPS / -DSMCV_ABLATE=n).
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-stamps}; N=${2:-8}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 120 bin/stamps/ip_stamps 192 h2 $N > "$OUT/stamps_h2.log" 2>&1 || exit 3
cat "$OUT/stamps_h2.log"
for r in 1 2; do for ab in 0 4 16 32 48 6 8 1; do
  echo -n "ablate=$ab: "; timeout -k 10 120 bin/stamps/ip_ab$ab 192 h2 $N > "$OUT/ab.tmp" 2>&1 || exit 5
  cat "$OUT/ab.tmp"
done; done
