#!/bin/bash
# Round evidence in one call: the -m gpu suite, smoke, every bench configuration with its
# rocprofv3 kernel trace and HBM counter passes (scripts/gpu_evidence.sh), the SQ counter passes
# of the default volume kernel on cfg2 / cfg4 (scripts/gpu_sq.sh), and the V4 volume bench.
#   bash scripts/gpu_round_evidence.sh TAG
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-round}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || { tail -30 "$OUT/gpu_tests.log"; exit 3; }
tail -1 "$OUT/gpu_tests.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 4; }
tail -1 "$OUT/smoke.log"
bash scripts/gpu_evidence.sh "$TAG/ev" "cfg2:--config cfg2" "cfg2_fused:--config cfg2 --pipeline fused" \
  "cfg2_fused_novolume:--config cfg2 --pipeline fused-novolume" \
  "cfg2_fused_novolume_f16:--config cfg2 --pipeline fused-novolume --features f16" \
  "cfg3:--config cfg3" "cfg4:--config cfg4" "cfg4_fused_novolume:--config cfg4 --pipeline fused-novolume" \
  "cfg5:--config cfg5" "cfg5_interweave:--config cfg5 --pipeline interweave" || exit 5
bash scripts/gpu_sq.sh "$TAG/sq" "cfg2_b32 cfg4_b32" || exit 6
timeout -k 10 120 python scripts/v4_bench.py > "$OUT/v4.json" 2> "$OUT/v4.err" || exit 7
cat "$OUT/v4.json"
