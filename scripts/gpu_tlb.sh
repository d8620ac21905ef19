#!/bin/bash
# Translation (UTCL1) and TCP stall counters of band kernels, one --pmc pass per counter group.
#   bash scripts/gpu_tlb.sh TAG "ops..."
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-tlb}; OPS=${2:-inner_product_ws_cfg2 inner_product_bf16x3_cfg2}
OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
i=0
for op in $OPS; do
  while read -r pmc; do
    i=$((i+1))
    timeout -k 10 180 rocprofv3 --pmc $pmc --output-format csv -d "$OUT/p$i" -o p -- python3 scripts/prof_op.py $op --reps 3 > "$OUT/p$i.log" 2>&1 || exit 4
    echo "$op | $pmc | p$i" >> "$OUT/index.txt"
  done <<'PASSES'
TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum
TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_SERIALIZATION_STALL_sum TCP_UTCL1_THRASHING_STALL_sum
TCP_PENDING_STALL_CYCLES_sum TCP_UTCL1_STALL_INFLIGHT_MAX_sum
TA_BUSY_avr TA_BUSY_max
SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD
PASSES
done
exit 0
