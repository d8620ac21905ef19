#!/usr/bin/env python3
"""Summarise a scripts/gpu_sq.sh run: per op, the band kernel's SQ counters averaged over its
dispatches, as fractions of wave cycles (SQ_WAVE_CYCLES and SQ_WAIT_* / SQ_ACTIVE_* count
quad-cycles; SQ_VALU_MFMA_BUSY_CYCLES counts cycles, MI355X_MICROARCH.md).

    python scripts/sq_summary.py gpurun_out/TAG [out.json]"""
import csv
import glob
import json
import os
import sys


def load(d):
    vals = {}
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                k = row["Kernel_Name"]
                if "band_" not in k:
                    continue
                vals.setdefault(row["Counter_Name"], []).append((float(row["Counter_Value"]),
                                                                  float(row["End_Timestamp"]) - float(row["Start_Timestamp"]),
                                                                  k.split("(")[0][-60:]))
    return vals


def main():
    root = sys.argv[1]
    out = {}
    ops = sorted({os.path.basename(p).rsplit("_p", 1)[0] for p in glob.glob(os.path.join(root, "*_p1"))})
    for op in ops:
        v = {}
        for i in (1, 2, 3):
            for c, rows in load(os.path.join(root, f"{op}_p{i}")).items():
                v[c] = sum(r[0] for r in rows) / len(rows)
                v["dur_ns_p%d" % i] = sum(r[1] for r in rows) / len(rows)
                v["kernel"] = rows[0][2]
        wc = v.get("SQ_WAVE_CYCLES", 0) or 1
        s = {"kernel": v.get("kernel"), "dur_us": round(v.get("dur_ns_p1", 0) / 1e3, 1),
             "waves": v.get("SQ_WAVES"),
             "wait_any": round(v.get("SQ_WAIT_ANY", 0) / wc, 3),
             "wait_inst_any": round(v.get("SQ_WAIT_INST_ANY", 0) / wc, 3),
             "active_any": round(v.get("SQ_ACTIVE_INST_ANY", 0) / wc, 3),
             "valu": round(v.get("SQ_ACTIVE_INST_VALU", 0) / wc, 3),
             "lds": round(v.get("SQ_ACTIVE_INST_LDS", 0) / wc, 3),
             "vmem": round(v.get("SQ_ACTIVE_INST_VMEM", 0) / wc, 3),
             "sca": round(v.get("SQ_ACTIVE_INST_SCA", 0) / wc, 3),
             "misc": round(v.get("SQ_ACTIVE_INST_MISC", 0) / wc, 3),
             "wait_inst_lds": round(v.get("SQ_WAIT_INST_LDS", 0) / wc, 3),
             "lds_bank_conflict_per_idx_active": round(v.get("SQ_LDS_BANK_CONFLICT", 0) / (v.get("SQ_LDS_IDX_ACTIVE", 0) or 1), 4),
             "raw": v}
        if "GRBM_GUI_ACTIVE" in v and v.get("dur_ns_p3"):
            s["clock_ghz"] = round(v["GRBM_GUI_ACTIVE"] / 8 / v["dur_ns_p3"], 3)
        if "SQ_VALU_MFMA_BUSY_CYCLES" in v and "GRBM_GUI_ACTIVE" in v:
            # per SIMD: busy cycles over (kernel cycles x 4 SIMDs x 256 CUs)
            s["mfma_busy"] = round(v["SQ_VALU_MFMA_BUSY_CYCLES"] / (v["GRBM_GUI_ACTIVE"] / 8 * 1024), 4)
        out[op] = s
        print(op, json.dumps({k: x for k, x in s.items() if k != "raw"}))
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
