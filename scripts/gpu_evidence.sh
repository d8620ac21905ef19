#!/bin/bash
# Round evidence for every bench configuration: the bench line, a rocprofv3 kernel-trace/stats
# profile of the same command (the same steps and warm-up: the bench's steps alternate two volume
# buffers, which some boxes map at different speeds, so both runs see the same alternation), and the HBM counter passes (FETCH_SIZE, WRITE_SIZE: one --pmc per
# run, kernel trace only); for the groupwise MFMA path also SQ_VALU_MFMA_BUSY_CYCLES with
# SQ_BUSY_CYCLES / GRBM_GUI_ACTIVE.  Fold the result into profiles/ with scripts/evidence_summary.py.
#   bash scripts/gpu_evidence.sh TAG ["name:bench args" ...]
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-ev}; shift
OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
SPECS=("$@")
if [ ${#SPECS[@]} -eq 0 ]; then
  SPECS=("cfg2:--config cfg2" "cfg2_fused_novolume:--config cfg2 --pipeline fused-novolume"
         "cfg3:--config cfg3" "cfg4:--config cfg4" "cfg5:--config cfg5"
         "cfg5_interweave:--config cfg5 --pipeline interweave")
fi
for spec in "${SPECS[@]}"; do
  n=${spec%%:*}; args=${spec#*:}
  D="$OUT/$n"; mkdir -p "$D"
  echo "== $n: $args"
  timeout -k 10 300 python bench.py $args > "$D/bench.json" 2> "$D/bench.err" || { echo "bench $n failed"; exit 2; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$D/kt" -o run --output-format csv -- \
    python3 bench.py --cpu-baseline-seconds 0 --no-check $args > "$D/kt.json" 2> "$D/kt.err" || { echo "kt $n failed"; exit 3; }
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d "$D/$c" -o run -- \
      python3 bench.py --steps 3 --warmup 1 --cpu-baseline-seconds 0 --no-check $args > "$D/$c.log" 2>&1 || { echo "pmc $c $n failed"; exit 4; }
  done
  if [ "$n" = "cfg3" ]; then
    timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$D/MFMA" -o run -- \
      python3 bench.py --steps 3 --warmup 1 --cpu-baseline-seconds 0 --no-check $args > "$D/MFMA.log" 2>&1 || { echo "pmc mfma $n failed"; exit 5; }
  fi
  python3 -c "import json; r=json.load(open('$D/bench.json')); print('$n', round(r['value'],1), r['unit'], 'kernel_us/launch', round(r['roofline']['avg_kernel_us'],1), 'frac', round(r['roofline']['frac'],3))"
done
exit 0
