#!/bin/bash
# Run the prebuilt ws ablation binaries (bin/wsa_*) on the GPU box.
#   bash scripts/run_ws_ablate.sh TAG "names" "modes"
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-wsab}; NAMES=${2}; MODES=${3:-ws}
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
for n in $NAMES; do
  for m in $MODES; do
    echo -n "$n: " >> "$OUT/ablate.log"
    timeout -k 10 60 bin/wsa_$n $m >> "$OUT/ablate.log" 2>&1 || exit 3
  done
done
exit 0
