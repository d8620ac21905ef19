#!/bin/bash
# Round 5 close: the driver's steps (-m gpu, smoke, default bench), then the evidence of the three
# fused configurations on the final build
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_final.sh r5z || exit $?
bash scripts/gpu_evidence.sh r05ev2 "cfg2_fused:--config cfg2 --pipeline fused" \
  "cfg2_fused_novolume:--config cfg2 --pipeline fused-novolume" \
  "cfg4_fused_novolume:--config cfg4 --pipeline fused-novolume" || exit 6
