#!/bin/bash
# Same-box A/B of the bench's warm-up length (cfg2 default workload): --warmup 5 against 60.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-warm}; mkdir -p "$OUT"
for w in 5 60 5 60; do
  timeout -k 10 200 python bench.py --warmup $w --no-check --cpu-baseline-seconds 0 >> "$OUT/warm.jsonl" 2>> "$OUT/warm.err" || exit 2
  python3 -c "import json; r=[json.loads(l) for l in open('$OUT/warm.jsonl')][-1]; print('warmup', r['warmup'], round(r['value'],1), round(r['roofline']['avg_kernel_us'],1), round(r['roofline']['frac'],4))"
done
