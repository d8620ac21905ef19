#!/usr/bin/env python3
"""Static check of the hand-counted vmcnt scheme of csrc/ip_ws.hip on the compiled gfx950 asm.

The staging waves keep kRd channel stages of feature loads in flight: inline-asm
`global_load_dwordx{2,4}` the compiler does not track, consumed after a hand-placed
`s_waitcnt vmcnt(N)`.  The kernel relies on these properties of the generated code, checked here
for every band_ws instantiation:
  1. no instruction reads or writes a hand load's destination registers while that load may
     still be in flight (a register copy or spill there would move data that has not landed);
  2. no wave ends (s_endpgm) with a hand load in flight;
  3. no `flat_*` memory instruction exists (flat ops count in vmcnt out of order).
The vector-memory queue is modelled exactly: every global_/buffer_/scratch_ op enters it in
issue order, and `s_waitcnt vmcnt(N)` retires all but the N youngest.  A may-state dataflow
(the set of possible queues per basic block) runs to a fixed point over the kernel's CFG.

    python scripts/check_ws_asm.py [extra hipcc flags]
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "realtime_stereo_matcher_amd", "csrc", "ip_ws.hip")
KERNEL = re.compile(r"^(_ZN4smcv6wsband7band_ws\w*):")
QMAX = 64  # the hardware counter saturates at 63 outstanding operations
VMEM = ("global_", "buffer_", "scratch_", "flat_")


def regs(tok):
    m = re.fullmatch(r"([va])\[(\d+):(\d+)\]", tok)
    if m:
        return {f"{m.group(1)}{i}" for i in range(int(m.group(2)), int(m.group(3)) + 1)}
    m = re.fullmatch(r"([va])(\d+)", tok)
    return {tok} if m else set()


def kernels(asm_text):
    """(name, [(line_no, instruction)]) per instantiation; instructions that come from an
    inline-asm statement are tagged with a leading '@'."""
    out, cur, in_asm = [], None, False
    for ln, line in enumerate(asm_text.splitlines(), 1):
        m = KERNEL.match(line)
        if m:
            cur = (m.group(1), [])
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
        if ins.startswith(".Lfunc_end"):
            cur = None
            continue
        if not ins or (ins.startswith(".") and not re.match(r"^\.L\w+:$", ins)):
            continue
        if in_asm and not ins.endswith(":"):
            ins = "@" + ins
        cur[1].append((ln, ins))
    return out


def blocks_of(body):
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


def norm(q):
    """Canonical queue: entries older than the oldest hand load never matter (vmcnt(N) keeps
    the N youngest), so leading untracked entries are dropped."""
    q = q[-QMAX:]
    i = 0
    while i < len(q) and not q[i]:
        i += 1
    return q[i:]


def step(queue, ln, ins, report):
    """One instruction applied to one possible queue (a tuple of frozensets of registers; an
    empty set = an operation whose registers nobody hand-counts)."""
    hand = ins.startswith("@")
    ins = ins.lstrip("@")
    op = ins.split()[0]
    toks = [t.strip(",") for t in ins.split()[1:]]
    pending = set().union(*queue) if queue else set()
    if op.startswith("flat_") and report is not None:
        report.append(f"{ln}: flat memory op: {ins}")
    if op.startswith("s_waitcnt"):
        m = re.search(r"vmcnt\((\d+)\)", ins)
        if m:
            n = int(m.group(1))
            return norm(queue[len(queue) - n:]) if n < len(queue) else queue
        if ins.strip() == "s_waitcnt 0":
            return ()
        return queue
    if op == "s_endpgm" and pending and report is not None:
        report.append(f"{ln}: wave ends with hand loads in flight into {sorted(pending)[:4]}")
    used = set()
    for t in toks:
        used |= regs(t)
    if op.startswith(VMEM):
        is_load = "load" in op or "atomic" in op
        dst = regs(toks[0]) if (is_load and toks) else set()
        srcs = used - dst
        if report is not None and (used & pending):
            report.append(f"{ln}: vmem op touches pending hand-load regs "
                          f"{sorted(used & pending)[:4]}: {ins}")
        entry = frozenset(dst) if hand else frozenset()
        return norm(queue + (entry,))
    if report is not None and used & pending:
        report.append(f"{ln}: touches pending hand-load regs {sorted(used & pending)[:4]}: {ins}")
    return queue


def transfer(block, states, report=None):
    out = set()
    for q in states:
        for ln, ins in block:
            q = step(q, ln, ins, report)
        out.add(q)
    return out


def check(asm_text):
    bad = []
    for name, body in kernels(asm_text):
        blocks, succ = blocks_of(body)
        ins_state = [set() for _ in blocks]
        ins_state[0] = {()}
        work = [0]
        while work:
            i = work.pop()
            outs = transfer(blocks[i], ins_state[i])
            for j in succ[i]:
                new = outs - ins_state[j]
                if new:
                    ins_state[j] |= new
                    if len(ins_state[j]) > 4096:
                        bad.append(f"{name}: state explosion at block {j}")
                        return bad
                    work.append(j)
        rep = []
        for i, b in enumerate(blocks):
            transfer(b, ins_state[i], rep)
        bad += [f"{name}:{r}" for r in sorted(set(rep))]
    return bad


def main():
    args = sys.argv[1:]
    with tempfile.TemporaryDirectory() as td:
        cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++20", "--offload-arch=gfx950", *args, "-I",
               os.path.join(ROOT, "include"), "-c", SRC, "--save-temps", "-o",
               os.path.join(td, "ws.o")]
        subprocess.run(cmd, cwd=td, check=True, capture_output=True)
        asm = open(os.path.join(td, "ip_ws-hip-amdgcn-amd-amdhsa-gfx950.s")).read()
    only = os.environ.get("WS_KERNEL")
    if only:
        asm = "\n".join(l if not KERNEL.match(l) or only in l else l.replace(":", "_skip:", 1)
                         for l in asm.splitlines())
    bad = check(asm)
    for b in bad[:40]:
        print(b)
    n = len(kernels(asm))
    print(f"{n} kernels checked, {len(bad)} problems")
    if n == 0:
        print("no band_ws kernels found in the asm (renamed?)")
        return 1
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
