#!/bin/bash
# Same-box A/B of the V4 volume: var_so/v4old.so (bf16 hi/lo split) vs var_so/v4new.so (scaled
# fp16 split), then a kernel trace of the new one.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-v4ab}; mkdir -p "$OUT"; export TMPDIR=/tmp
for r in 1 2; do
  for n in v4old v4new; do
    STEREOCV_LIB=var_so/$n.so timeout -k 10 120 python scripts/v4_bench.py > "$OUT/$n.$r.json" 2> "$OUT/$n.err" || { tail -5 "$OUT/$n.err"; exit 2; }
    echo "$n $(python3 -c "import json;r=json.load(open('$OUT/$n.$r.json'));print(r['ms']['hip_fused'], r['max_abs_err_vs_reference_loop'], r['mfma']['frac_useful'])")"
  done
done
STEREOCV_LIB=var_so/v4new.so timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o run --output-format csv -- python3 scripts/v4_bench.py > "$OUT/kt.log" 2>&1 || { tail -5 "$OUT/kt.log"; exit 3; }
python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/kt/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "v4" in r["Name"]:
        print(r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
