#!/usr/bin/env python3
"""Audit the inner-product band kernels' hand-counted loads: between each inline-asm
global_load and the inline-asm s_waitcnt that retires it, no instruction may read or copy the
load's destination registers (cdna_hip_programming.md §5.7 item 1).  Exit 1 on a violation."""
import re
import subprocess
import sys
import tempfile
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "realtime_stereo_matcher_amd", "csrc", "ip_mfma.hip")


def regs(text):
    out = set()
    for a, b in re.findall(r"v\[(\d+):(\d+)\]", text):
        out.update(range(int(a), int(b) + 1))
    for a in re.findall(r"\bv(\d+)\b", text):
        out.add(int(a))
    return out


def main():
    with tempfile.TemporaryDirectory() as td:
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-I",
                        os.path.join(ROOT, "include"), "-c", SRC, "-save-temps", "-o",
                        os.path.join(td, "x.o")], cwd=td, check=True, capture_output=True)
        asm = open(os.path.join(td, "ip_mfma-hip-amdgcn-amd-amdhsa-gfx950.s")).read()
    bad = 0
    kernels = re.findall(r"^(_ZN4smcv\S*ip_band_mfma\S*):", asm, re.M)
    for name in kernels:
        i = asm.index(name + ":")
        j = asm.index(".Lfunc_end", i)
        lines = [l.strip() for l in asm[i:j].splitlines()]
        pending = set()
        for n, l in enumerate(lines):
            if l.startswith("global_load_dwordx") and "off" in l:
                dst = regs(l.split(",")[0])
                if n > 0 and lines[n - 1] == ";;#ASMSTART":
                    pending |= dst
                continue
            if l.startswith("s_waitcnt") and "vmcnt" in l and n > 0 and lines[n - 1] == ";;#ASMSTART":
                pending.clear()
                continue
            if not pending or l.startswith((";", ".")) or l.endswith(":"):
                continue
            if l.startswith(("s_", "ds_write", "global_store")) and not (regs(l) & pending):
                continue
            ops = l.split(None, 1)
            srcs = regs(ops[1].split(",", 1)[1]) if len(ops) > 1 and "," in ops[1] else set()
            if l.startswith(("ds_write", "global_store")):
                srcs = regs(ops[1]) if len(ops) > 1 else set()
            if srcs & pending:
                print(f"{name[:60]}: line {n}: reads in-flight registers: {l}")
                bad += 1
            dsts = regs(ops[1].split(",", 1)[0]) if len(ops) > 1 else set()
            if dsts & pending and not l.startswith(("ds_", "global_store")):
                print(f"{name[:60]}: line {n}: overwrites in-flight registers: {l}")
                bad += 1
    print(f"checked {len(kernels)} kernels, {bad} violation(s)")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
