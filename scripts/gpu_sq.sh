#!/bin/bash
# SQ counters of the band kernels (scripts/ab_time.py ops; cfg2_b32 / cfg4_b32 = the bench launch): where the waves'
# cycles go (parked at waitcnt / barrier, issue-stalled, issuing by instruction class), MFMA
# busy, LDS conflicts, clock.   bash scripts/gpu_sq.sh TAG "op1 op2 ..."
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-sq}; OPS=${2:-cfg2_sp cfg2_h2db}
OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_SCA SQ_LDS_IDX_ACTIVE"
P3="GRBM_GUI_ACTIVE GRBM_COUNT"
for op in $OPS; do
  i=0
  for P in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d "$OUT/${op}_p$i" -o run -- python3 scripts/ab_time.py --ops $op --reps 6 > "$OUT/${op}_p$i.log" 2>&1 || { echo "pass $i of $op failed"; tail -5 "$OUT/${op}_p$i.log"; exit 4; }
  done
done
echo done
