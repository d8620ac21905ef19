#!/bin/bash
# Effective shader clock of the band kernels (GRBM_GUI_ACTIVE / 8 / duration) from a counter
# pass and a kernel-trace pass of scripts/ab_time.py.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-clock}; mkdir -p "$OUT"; export TMPDIR=/tmp
OPS=${2:-cfg2_h2,cfg2_h2db}
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --kernel-trace --output-format csv -d "$OUT/pmc" -o run -- python3 scripts/ab_time.py --ops $OPS --reps 5 > "$OUT/pmc.log" 2>&1 || { tail -5 "$OUT/pmc.log"; exit 2; }
python3 - "$OUT" <<'PY'
import csv, sys, collections, glob
out = sys.argv[1]
files = glob.glob(out + "/pmc/**/*.csv", recursive=True)
cc = [f for f in files if f.endswith("counter_collection.csv")][0]
rows = list(csv.DictReader(open(cc)))
print(list(rows[0].keys()))
per = collections.defaultdict(dict)
for r in rows:
    key = (r["Kernel_Name"][:50], r.get("Dispatch_Id"))
    per[key][r["Counter_Name"]] = float(r["Counter_Value"])
    for f in ("Start_Timestamp", "End_Timestamp"):
        if f in r: per[key][f] = float(r[f])
for (k, d), v in sorted(per.items(), key=lambda x: int(x[0][1] or 0)):
    if "band" not in k: continue
    dur = v.get("End_Timestamp", 0) - v.get("Start_Timestamp", 0)
    print(k, d, "GRBM", v.get("GRBM_GUI_ACTIVE"), "dur_ns", dur, "GHz", round(v["GRBM_GUI_ACTIVE"] / 8 / dur, 3) if dur > 0 else None)
PY
