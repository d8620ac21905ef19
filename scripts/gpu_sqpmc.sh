#!/bin/bash
# SQ counters of the cfg2 band kernel (harness bin/wsa_base, 8 pairs per launch): where the
# waves' cycles go (parked at waitcnt/barrier vs issue-stalled vs issuing), LDS conflicts.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-sq}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES --output-format csv -d "$OUT/p1" -o run -- bin/wsa_base ${2:-h2x8} > "$OUT/p1.log" 2>&1 || exit 4
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_SCA SQ_WAVES --output-format csv -d "$OUT/p2" -o run -- bin/wsa_base ${2:-h2x8} > "$OUT/p2.log" 2>&1 || exit 5
exit 0
