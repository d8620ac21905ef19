#!/bin/bash
# cfg4 evidence at the bench's default launch (the rank's whole batch), the SQ passes of the
# 32-pair launches, the bench-launch parity tests, and a same-box pairs-per-launch A/B on cfg2.
#   bash scripts/gpu_b32.sh TAG
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-b32}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_sp.py -x -v -m gpu -k bench_launch --timeout 180 --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 3; }
tail -1 "$OUT/tests.log"
for c in 8 32 8 32; do
  timeout -k 10 200 python bench.py --config cfg2 --chunk $c --no-check --cpu-baseline-seconds 0 >> "$OUT/ab_chunk.jsonl" 2>> "$OUT/ab_chunk.err" || exit 4
  python3 -c "import json; r=[json.loads(l) for l in open('$OUT/ab_chunk.jsonl')][-1]; print('cfg2 chunk', r['config']['pairs_per_launch'], round(r['value'],1), round(r['roofline']['avg_kernel_us'],1), round(r['roofline']['frac'],4))"
done
bash scripts/gpu_evidence.sh "$TAG/ev" "cfg4:--config cfg4" "cfg4_fused_novolume:--config cfg4 --pipeline fused-novolume" || exit 5
bash scripts/gpu_sq.sh "$TAG/sq" "cfg2_b32 cfg4_b32" || exit 6
echo done
