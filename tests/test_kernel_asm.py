"""Static checks of compiled gfx950 code (CPU only; needs hipcc).

The h2 band kernel issues its feature loads as inline asm and counts vmcnt by hand
(csrc/ip_h2.hip); scripts/check_h2_asm.py verifies on the generated asm that no instruction
touches a load's destination registers before its wait and that no flat memory op exists.
scripts/check_h2_bounds.py replays the kernel's load / ring / store indexing on the host."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"),
                    reason="hipcc not available")
def test_h2_asm_vmcnt_discipline():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "check_h2_asm.py")],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]


def test_h2_indexing_replay():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "check_h2_bounds.py")],
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
