#!/usr/bin/env python3
"""Instruction mix per barrier-delimited region of one kernel in a hipcc --save-temps .s file.
    python scripts/asm_regions.py file.s KERNEL_SYMBOL_REGEX"""
import re
import sys
from collections import Counter

text = open(sys.argv[1]).read().splitlines()
pat = re.compile(sys.argv[2])
body, on = [], False
for ln in text:
    if not on and pat.match(ln) and ln.endswith(":") or (not on and pat.match(ln.split(":")[0]) and ":" in ln and not ln.startswith("\t")):
        on = True
        continue
    if on:
        if ln.startswith(".Lfunc_end"):
            break
        body.append(ln)
classes = [("mfma", r"v_mfma"), ("ds_w32", r"ds_write_b32"), ("ds_w128", r"ds_write_b128"), ("ds_r128", r"ds_read_b128"),
           ("ds_other", r"ds_"), ("bstore", r"buffer_store"), ("gload", r"global_load"), ("gstore", r"global_store"),
           ("accrd", r"v_accvgpr_read"), ("accmv", r"v_accvgpr_(mov|write)"), ("lane", r"v_(read|write)lane"),
           ("waitcnt", r"s_waitcnt"), ("branch", r"s_cbranch|s_branch"), ("salu", r"s_"), ("valu", r"v_")]
regions, cur = [], Counter()
for ln in body:
    ins = ln.split(";")[0].strip()
    if not ins or ins.startswith(".") or ins.endswith(":"):
        continue
    if ins.startswith("s_barrier"):
        regions.append(cur)
        cur = Counter()
        continue
    for name, rx in classes:
        if re.match(rx, ins):
            cur[name] += 1
            break
    else:
        cur["other"] += 1
regions.append(cur)
names = [c[0] for c in classes] + ["other"]
print("region " + " ".join(f"{n:>8}" for n in names) + "    total")
for i, r in enumerate(regions):
    print(f"{i:6d} " + " ".join(f"{r[n]:8d}" for n in names) + f" {sum(r.values()):8d}")
