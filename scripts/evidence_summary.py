#!/usr/bin/env python3
"""Fold a scripts/gpu_evidence.sh run into the committed evidence under profiles/ROUND/.

    python scripts/evidence_summary.py gpurun_out/TAG r02

Per configuration NAME it writes profiles/ROUND/NAME/:
  bench.json          the bench line of the run (HIP-event kernel time, roofline, cpu_baseline)
  kernel_stats.csv    rocprofv3 --kernel-trace --stats of the same command (names shortened)
  pmc.json            HBM bytes per launch per kernel from the separate --pmc FETCH_SIZE and
                      --pmc WRITE_SIZE passes, corrected as MI355X_MICROARCH.md prescribes
                      (FETCH_SIZE KiB x2 on gfx950 for 16-B/lane streaming reads, WRITE_SIZE KiB
                      exact), plus (cfg3) the MFMA busy fraction from SQ_VALU_MFMA_BUSY_CYCLES
and profiles/ROUND/summary.json with one row per configuration (bench kernel time vs the
rocprofv3 average of the dominant kernel -- the profiled process's own HIP-event average beside
it, profiled_bench_avg_kernel_us -- algorithmic vs counted bytes).
"""
import csv
import glob
import json
import os
import re
import sys

KEEP = ("band_h2", "band_sl", "band_rs", "softargmin", "argext", "concat_kernel", "shifted_rows_kernel", "interweave_kernel",
        "dot_volume", "ip_", "warp")


def short(name):
    m = re.search(r"(?:\w+::)*?(\w+)<", name) or re.search(r"(\w+)\(", name)
    base = m.group(1) if m else name[:40]
    if "<" in name:
        return base + name[name.index("<"): name.index(">") + 1]
    return base


def find(d, pattern):
    hits = glob.glob(os.path.join(d, "**", pattern), recursive=True)
    return hits[0] if hits else None


def counter_means(path, names):
    per = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] not in names:
                continue
            k = short(row["Kernel_Name"])
            per.setdefault(k, {}).setdefault(row["Counter_Name"], {}).setdefault(row.get("Dispatch_Id", "0"), 0.0)
            # one row per dispatch and counter (summed over dimensions when split)
            per[k][row["Counter_Name"]][row.get("Dispatch_Id", "0")] += float(row["Counter_Value"])
    out = {}
    for k, cs in per.items():
        out[k] = {c: sum(v.values()) / len(v) for c, v in cs.items()}
    return out


def main():
    src, rnd = sys.argv[1], sys.argv[2]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    dst_root = os.path.join(root, "profiles", rnd)
    summary = {}
    spath = os.path.join(dst_root, "summary.json")
    if os.path.exists(spath):  # several evidence runs fold into one summary (rows replaced by name)
        with open(spath) as f:
            summary = json.load(f)
    for d in sorted(glob.glob(os.path.join(src, "*"))):
        if not os.path.isdir(d) or not os.path.exists(os.path.join(d, "bench.json")):
            continue
        name = os.path.basename(d)
        dst = os.path.join(dst_root, name)
        os.makedirs(dst, exist_ok=True)
        bench = json.load(open(os.path.join(d, "bench.json")))
        json.dump(bench, open(os.path.join(dst, "bench.json"), "w"))
        row = {"value": bench["value"], "unit": bench["unit"], "kernel": bench["roofline"]["kernel"],
               "bench_avg_kernel_us": bench["roofline"]["avg_kernel_us"], "frac": bench["roofline"]["frac"],
               "algorithmic_bytes_per_launch": bench["roofline"]["achieved"] * 1e3 * bench["roofline"]["avg_kernel_us"]}
        ks = find(os.path.join(d, "kt"), "*kernel_stats.csv")
        if ks:
            rows = []
            with open(ks) as f:
                for r in csv.DictReader(f):
                    r["Name"] = short(r["Name"])
                    rows.append(r)
            with open(os.path.join(dst, "kernel_stats.csv"), "w", newline="") as f:
                w = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
                w.writeheader()
                w.writerows(rows)
            top = max(rows, key=lambda r: float(r["TotalDurationNs"]))
            row["rocprof_top_kernel"] = top["Name"]
            row["rocprof_avg_us"] = float(top["AverageNs"]) / 1e3
            # the profiled process's own bench line (kt.json): the same launches, timed by the
            # bench's HIP events and by the kernel trace; a separate process may draw differently
            # mapped volume buffers (profiles/r05/placement/), so this is the like-for-like pair
            kt = os.path.join(d, "kt.json")
            if os.path.exists(kt) and os.path.getsize(kt) > 0:
                with open(kt) as f:
                    ktb = json.loads(f.read().strip().splitlines()[-1])
                row["profiled_bench_avg_kernel_us"] = ktb["roofline"]["avg_kernel_us"]
                row["profiled_bench_value"] = ktb["value"]
        pmc = {"correction": "hbm_bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024 (gfx950)", "kernels": {}}
        fp, wp = find(os.path.join(d, "FETCH_SIZE"), "*counter_collection.csv"), find(os.path.join(d, "WRITE_SIZE"), "*counter_collection.csv")
        if fp and wp:
            fetch = counter_means(fp, {"FETCH_SIZE"})
            write = counter_means(wp, {"WRITE_SIZE"})
            for k in sorted(set(fetch) & set(write)):
                if not k.startswith(KEEP):
                    continue
                fb, wb = 2 * fetch[k]["FETCH_SIZE"] * 1024, write[k]["WRITE_SIZE"] * 1024
                pmc["kernels"][k] = {"fetch_bytes": fb, "write_bytes": wb, "hbm_bytes_per_launch": fb + wb}
        mp = find(os.path.join(d, "MFMA"), "*counter_collection.csv")
        if mp:
            m = counter_means(mp, {"SQ_VALU_MFMA_BUSY_CYCLES", "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE"})
            for k, c in m.items():
                if not k.startswith(KEEP):
                    continue
                rec = pmc["kernels"].setdefault(k, {})
                rec.update(c)
                if c.get("GRBM_GUI_ACTIVE"):
                    # SQ_VALU_MFMA_BUSY_CYCLES is summed over all 1024 SIMDs (32 cycles per
                    # 32x32x16 MFMA, MI355X_MICROARCH.md); GRBM_GUI_ACTIVE is summed over the 8
                    # XCDs (8 x kernel cycles), so the busy fraction per SIMD is
                    # MFMA_BUSY / (1024 * GRBM_GUI_ACTIVE / 8)
                    rec["mfma_busy_frac"] = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (128.0 * c["GRBM_GUI_ACTIVE"])
        json.dump(pmc, open(os.path.join(dst, "pmc.json"), "w"), indent=1)
        for k, rec in pmc["kernels"].items():
            if row.get("rocprof_top_kernel") == k:
                row["pmc_hbm_bytes_per_launch"] = rec.get("hbm_bytes_per_launch")
                if "mfma_busy_frac" in rec:
                    row["mfma_busy_frac"] = rec["mfma_busy_frac"]
        summary[name] = row
    json.dump(summary, open(os.path.join(dst_root, "summary.json"), "w"), indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
