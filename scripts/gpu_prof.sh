#!/bin/bash
# Counter passes (one rocprofv3 --pmc run per pass, kernel trace only) + ablation timings.
# usage: bash scripts/gpu_prof.sh TAG OP
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-prof}; OP=${2:-inner_product_mfma_cfg2}
OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
for ab in 0 1 2 4 3 5 6 7; do
  STEREOCV_ABLATE=$ab timeout -k 10 120 python scripts/prof_op.py $OP --reps 10 --time >> "$OUT/ablate.log" 2>&1 || exit 3
done
i=0
while read -r pmc; do
  i=$((i+1))
  timeout -k 10 180 rocprofv3 --pmc $pmc --output-format csv -d "$OUT/pmc$i" -o p -- python3 scripts/prof_op.py $OP --reps 3 > "$OUT/pmc$i.log" 2>&1 || exit 4
done <<'PASSES'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE
SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE
FETCH_SIZE
WRITE_SIZE
TCC_HIT_sum TCC_MISS_sum
SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC
PASSES
exit 0
