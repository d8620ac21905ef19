#!/usr/bin/env python3
"""Fold a gpu_bench_prof.sh run into the committed evidence under profiles/.

    python scripts/pmc_summary.py gpurun_out/TAG ROUND   (e.g. gpurun_out/b1 r01)

Writes profiles/ROUND_kernel_stats.csv (the rocprofv3 --kernel-trace --stats summary of the
bench command, kernel names shortened), profiles/ROUND_bench.json (the bench line) and
profiles/pmc_traffic.json: HBM bytes per launch per kernel from the two --pmc passes,
corrected as MI355X_MICROARCH.md (HBM section) prescribes -- FETCH_SIZE is in KiB and counts
half the bytes of a 16-B/lane streaming read on gfx950 (x2), WRITE_SIZE (KiB) is exact for
16-B/lane stores.
"""
import csv
import json
import os
import re
import shutil
import sys


def short(name):
    m = re.search(r"(?:smcv::)?(?:\w+::)*?(\w+)<", name) or re.search(r"(\w+)\(", name)
    base = m.group(1) if m else name[:40]
    if "smcv::" in name:
        tpl = name[name.index("<") : name.index(">") + 1] if "<" in name else ""
        return base + tpl
    return base


def counters(path, counter):
    per = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != counter:
                continue
            per.setdefault(short(row["Kernel_Name"]), []).append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in per.items()}


def main():
    src, rnd = sys.argv[1], sys.argv[2]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    prof = os.path.join(root, "profiles")
    os.makedirs(prof, exist_ok=True)
    rows = []
    with open(os.path.join(src, "kt", "run_kernel_stats.csv")) as f:
        for row in csv.DictReader(f):
            row["Name"] = short(row["Name"])
            rows.append(row)
    with open(os.path.join(prof, f"{rnd}_kernel_stats.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
        w.writeheader()
        w.writerows(rows)
    shutil.copy(os.path.join(src, "bench.json"), os.path.join(prof, f"{rnd}_bench.json"))
    fetch = counters(os.path.join(src, "fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = counters(os.path.join(src, "write", "run_counter_collection.csv"), "WRITE_SIZE")
    out = {"source": f"{rnd}: rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate runs of "
                     "bench.py --steps 5 --warmup 2",
           "correction": "hbm_bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024 (gfx950)",
           "kernels": {}}
    for k in sorted(set(fetch) & set(write)):
        if "smcv" not in k and not k.startswith(("ip_", "band_", "softargmin", "argext", "dot_volume")):
            continue
        fb, wb = 2 * fetch[k] * 1024, write[k] * 1024
        rec = {"fetch_bytes": fb, "write_bytes": wb, "hbm_bytes_per_launch": fb + wb}
        out["kernels"][k] = rec
        base = k.split("<")[0]
        out["kernels"].setdefault(base, rec)
    with open(os.path.join(prof, "pmc_traffic.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))
    for r in rows[:4]:
        print(r["Name"], r["Calls"], r["AverageNs"])


if __name__ == "__main__":
    main()
