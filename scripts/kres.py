#!/usr/bin/env python3
"""Print per-kernel register / LDS / occupancy / spill figures of one HIP source (gfx950)."""
import re
import subprocess
import sys

src = sys.argv[1]
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-I", "include", "-c", src,
       "-o", "/tmp/_kres.o", "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = None
rows = []
for line in out.splitlines():
    m = re.search(r"remark: +(.*?): (\S+)", line)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2)
    if k == "Function Name":
        cur = {"name": v}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
for r in rows:
    name = subprocess.run(["c++filt"], input=r["name"], capture_output=True, text=True).stdout.strip()
    name = name.replace("smcv::(anonymous namespace)::", "").replace("void ", "")
    name = re.sub(r"\(.*", "", name)
    print(f"{name[:70]:70s} vgpr={r.get('VGPRs','?'):>4} agpr={r.get('AGPRs','?'):>3} "
          f"spill={r.get('VGPRs Spill','?')} scratch={r.get('ScratchSize [bytes/lane]','?')} "
          f"occ={r.get('Occupancy [waves/SIMD]','?')} lds={r.get('LDS Size [bytes/block]','?')}")
