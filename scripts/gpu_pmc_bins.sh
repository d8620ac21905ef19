#!/bin/bash
# HBM counters (separate --pmc passes) for prebuilt ablation binaries.
#   bash scripts/gpu_pmc_bins.sh TAG "bin:mode ..."
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-pmc}; SPECS=${2}
OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
for spec in $SPECS; do
  b=${spec%%:*}; m=${spec#*:}
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d "$OUT/${b}_${m}_$c" -o run -- bin/wsa_$b $m > "$OUT/${b}_${m}_$c.log" 2>&1 || exit 4
  done
done
exit 0
