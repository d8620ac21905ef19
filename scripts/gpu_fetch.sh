#!/bin/bash
# HBM fetch / write bytes per launch of the band kernels for library builds (rocprofv3 --pmc
# FETCH_SIZE and --pmc WRITE_SIZE, separate passes with the kernel trace), ops via ab_time.py.
#   bash scripts/gpu_fetch.sh TAG OPS lib1.so [lib2.so ...]
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; OPS=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
i=0
for lib in "$@"; do
  for c in FETCH_SIZE WRITE_SIZE; do
    STEREOCV_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$OUT/l$i/$c" -o run -- python3 scripts/ab_time.py --ops $OPS --reps 3 > "$OUT/l$i.$c.log" 2>&1 || { tail -5 "$OUT/l$i.$c.log"; exit 2; }
  done
  python3 - "$OUT/l$i" "$lib" <<'PY'
import csv, sys, glob, collections
d, lib = sys.argv[1], sys.argv[2]
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    f = glob.glob(d + "/" + c + "/**/*counter_collection.csv", recursive=True)[0]
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        per[r["Kernel_Name"][:60]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    for k, v in per.items():
        if "band" in k or "merge" in k:
            m = sum(v.values()) / len(v)
            print(lib.split("/")[-1], c, k, "KiB/launch", round(m), "GB/launch", round(m * 1024 * (2 if c == "FETCH_SIZE" else 1) / 1e9, 4))
PY
  i=$((i+1))
done
