#!/bin/bash
# Kernel traces of the V4 volume builds var_so/NAME.so (per-kernel averages).
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-v4kt}; mkdir -p "$OUT"; export TMPDIR=/tmp
for n in ${2:-v4old v4new}; do
  STEREOCV_LIB=var_so/$n.so timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$OUT/$n" -o run --output-format csv -- python3 scripts/v4_bench.py > "$OUT/$n.log" 2>&1 || { tail -5 "$OUT/$n.log"; exit 3; }
  python3 - "$OUT/$n" "$n" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "v4" in r["Name"]:
        print(sys.argv[2], r["Name"][:40], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
done
