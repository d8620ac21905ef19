#!/usr/bin/env python3
"""Per-kernel register / scratch / LDS summary of a hipcc --cuda-device-only -S asm file.
    python scripts/kres_asm.py file.s [name-substring]"""
import re
import sys

s = open(sys.argv[1]).read()
sub = sys.argv[2] if len(sys.argv) > 2 else ""
for m in re.finditer(r"\.amdhsa_kernel (\S+)\n(.*?)\.end_amdhsa_kernel", s, re.S):
    name, body = m.group(1), m.group(2)
    if sub not in name:
        continue
    g = lambda k: int(re.search(rf"\.{k} (\d+)", body).group(1)) if re.search(rf"\.{k} (\d+)", body) else -1  # noqa
    print(f"{name[:90]:90s} vgpr={g('amdhsa_next_free_vgpr'):4d} acc_off={g('amdhsa_accum_offset'):4d} "
          f"sgpr={g('amdhsa_next_free_sgpr'):3d} scratch={g('amdhsa_private_segment_fixed_size'):5d} "
          f"lds={g('amdhsa_group_segment_fixed_size')}")
