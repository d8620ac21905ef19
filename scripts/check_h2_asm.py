#!/usr/bin/env python3
"""Static check of the hand-counted vmcnt scheme of csrc/ip_h2.hip on the compiled gfx950 asm.

The feature loads are inline-asm `global_load_dwordx{2,4}` the compiler does not track, so the
kernel relies on two properties of the generated code, checked here for every instantiation:
  1. no instruction touches a load's destination registers between the load and the next
     `s_waitcnt vmcnt` (a register copy there would read data that has not landed);
  2. no wave ends (s_endpgm) with such a load still in flight (the L2 touches included);
  3. no `flat_*` memory instruction exists (flat ops count in vmcnt out of order, which would
     break the `vmcnt(4 (T-1))` wait that lets the output stores stay in flight);
  4. band_h2db (ip_h2db.hip), band_rs (ip_rs.hip) and band_sl (ip_sl.hip) have no scratch
     access at all: a spill reload counts in vmcnt (band_rs's and band_sl's loads are
     compiler-tracked; the other checks find no inline-asm loads in them, and the scratch check
     is what applies there) and would wait for the feature loads in flight.
A may-pending dataflow over the kernel's basic blocks carries each load to every instruction it
can reach before a vmcnt wait.

    python scripts/check_h2_asm.py [-DSMCV_ABLATE=N] [--stamps]   # hipcc --save-temps, then scan
Run it on every build that goes to the GPU (the library, and each diagnostic ablation build).
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "realtime_stereo_matcher_amd", "csrc")
SRCS = [os.path.join(CSRC, "ip_h2.hip"), os.path.join(CSRC, "ip_h2db.hip"), os.path.join(CSRC, "ip_rs.hip"),
        os.path.join(CSRC, "ip_sl.hip")]


def regs(tok):
    m = re.fullmatch(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.fullmatch(r"v(\d+)", tok)
    return {int(m.group(1))} if m else set()


def kernels(asm_text):
    """(name, [(line_no, instruction)]) per band_h2 instantiation.  Instructions that come from
    an inline-asm statement (between ;;#ASMSTART and ;;#ASMEND) are tagged with a leading '@':
    only those loads are hand-counted (the compiler waits for its own)."""
    out, cur, in_asm = [], None, False
    for ln, line in enumerate(asm_text.splitlines(), 1):
        if re.match(r"^_ZN4smcv6h2band(7band_h2|9band_h2db|7band_rs|7band_sl).*:", line):
            cur = (line.split(":")[0], [])
            out.append(cur)
            continue
        if cur is None:
            continue
        if ";;#ASMSTART" in line:
            in_asm = True
            continue
        if ";;#ASMEND" in line:
            in_asm = False
            continue
        ins = line.split(";")[0].strip()
        if in_asm and ins and not ins.startswith(".") and not ins.endswith(":"):
            ins = "@" + ins
        if ins.startswith(".Lfunc_end"):
            cur = None
            continue
        if not ins or ins.startswith("."):
            if re.match(r"^\.L\w+:$", ins):
                cur[1].append((ln, ins))
            continue
        cur[1].append((ln, ins))
    return out


def blocks_of(body):
    """Split into basic blocks; returns (blocks, label->index, successors)."""
    blocks, labels = [[]], {}
    for ln, ins in body:
        if ins.endswith(":"):
            if blocks[-1]:
                blocks.append([])
            labels[ins[:-1]] = len(blocks) - 1
            continue
        blocks[-1].append((ln, ins))
        op = ins.lstrip("@").split()[0]
        if op.startswith(("s_branch", "s_cbranch", "s_endpgm", "s_setpc")):
            blocks.append([])
    succ = []
    for i, b in enumerate(blocks):
        s = set()
        last = b[-1][1].lstrip("@").split() if b else []
        op = last[0] if last else ""
        if op.startswith(("s_branch", "s_cbranch")):
            s.add(labels[last[1]])
        if not op.startswith(("s_branch", "s_endpgm", "s_setpc")) and i + 1 < len(blocks):
            s.add(i + 1)
        succ.append(s)
    return blocks, succ


def transfer(block, pending, report=None, no_scratch=False):
    pending = set(pending)
    for ln, ins in block:
        hand = ins.startswith("@")  # from an inline-asm statement
        ins = ins.lstrip("@")
        op = ins.split()[0]
        if report is not None and op.startswith("flat_"):
            report.append(f"{ln}: flat memory op: {ins}")
        if op.startswith("s_waitcnt") and "vmcnt" in ins:
            pending = set()
            continue
        if op == "s_endpgm" and pending and report is not None:
            report.append(f"{ln}: wave ends with loads in flight into v{sorted(pending)[:4]}...")
        toks = [t.strip(",") for t in ins.split()[1:]]
        if no_scratch and op.startswith("scratch_") and report is not None:
            report.append(f"{ln}: scratch access (a spill counts in vmcnt): {ins}")
        if hand and op in ("global_load_dwordx4", "global_load_dwordx2", "global_load_dword"):
            srcs = set()
            for t in toks[1:]:
                srcs |= regs(t)
            if report is not None and srcs & pending:
                report.append(f"{ln}: address reads pending v{sorted(srcs & pending)}: {ins}")
            pending |= regs(toks[0])
            continue
        used = set()
        for t in toks:
            used |= regs(t)
        if report is not None and used & pending:
            report.append(f"{ln}: touches pending load regs v{sorted(used & pending)}: {ins}")
    return pending


def check(asm_text):
    bad = []
    for name, body in kernels(asm_text):
        blocks, succ = blocks_of(body)
        ins_state = [set() for _ in blocks]
        changed = True
        while changed:  # may-pending dataflow to a fixed point
            changed = False
            for i, b in enumerate(blocks):
                out = transfer(b, ins_state[i])
                for j in succ[i]:
                    if not out <= ins_state[j]:
                        ins_state[j] |= out
                        changed = True
        rep = []
        for i, b in enumerate(blocks):
            # no scratch at all in band_h2db (volume and fused), band_rs and band_sl
            no_scr = "9band_h2db" in name or "7band_rs" in name or "7band_sl" in name
            transfer(b, ins_state[i], rep, no_scratch=no_scr)
        bad += [f"{name}:{r}" for r in rep]
    return bad


def main():
    args = sys.argv[1:]
    srcs = SRCS
    if "--stamps" in args:  # the round-3 diagnostic driver (scripts/experimental/ip_stamps.hip) instead
        args.remove("--stamps")
        srcs = [os.path.join(ROOT, "scripts", "experimental", "ip_stamps.hip")]
        args.append("-DSMCV_STAMPS")
    bad, n = [], 0
    # the sources compile concurrently (device code only: the asm is all that is scanned)
    with tempfile.TemporaryDirectory() as td:
        procs = []
        for k, src in enumerate(srcs):
            out = os.path.join(td, f"k{k}.s")
            cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++20", "--offload-arch=gfx950", *args, "-I",
                   os.path.join(ROOT, "include"), "--cuda-device-only", "-S", src, "-o", out]
            procs.append((subprocess.Popen(cmd, cwd=td, stdout=subprocess.PIPE, stderr=subprocess.PIPE), out))
        for p, out in procs:
            _, err = p.communicate()
            if p.returncode != 0:
                raise SystemExit(err.decode()[-2000:])
            asm = open(out).read()
            bad += check(asm)
            n += len(kernels(asm))
    for b in bad[:int(os.environ.get("SHOW", 40))]:
        print(b)
    print(f"{n} kernels checked, {len(bad)} problems")
    if n == 0:
        print("no band kernels found in the asm (renamed?)")
        return 1
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
