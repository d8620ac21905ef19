#!/bin/bash
# Round 5 evidence, second half: cfg4 (32 pairs, and the 4-pair per-rank launch of the N = 8
# run), cfg4 volume-free fused, cfg5 / interweave, and the SQ sets of the volume kernel and of
# the two volume-free fused passes (fp32 band_sl, fp16 band_h2) on 32-pair cfg2 launches.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
bash scripts/gpu_evidence.sh r05ev "cfg4:--config cfg4" "cfg4_b4:--config cfg4 --batch 4" \
  "cfg4_fused_novolume:--config cfg4 --pipeline fused-novolume" \
  "cfg5:--config cfg5" "cfg5_interweave:--config cfg5 --pipeline interweave" || exit 5
bash scripts/gpu_sq.sh r05sq "cfg2_b32 cfg2_fused_nv_b32 cfg2_fused_nv_f16_b32" || exit 6
