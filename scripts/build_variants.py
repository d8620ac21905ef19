#!/usr/bin/env python3
"""Diagnostic library builds for same-box A/B: libstereocv.so with one source recompiled under
extra -D flags, written to var_so/NAME.so (select one with STEREOCV_LIB=...).

    python scripts/build_variants.py NAME SOURCE.hip -DFLAG=V [...]
    python scripts/build_variants.py NAME /path/other.hip:SOURCE.hip [...]   (another file in
                                                                             SOURCE.hip's place)"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from realtime_stereo_matcher_amd import build_lib as B  # noqa: E402


def main():
    name, src, flags = sys.argv[1], sys.argv[2], sys.argv[3:]
    B.build(verbose=False)  # the regular objects
    out_dir = os.path.join(ROOT, "build", "var")
    os.makedirs(out_dir, exist_ok=True)
    obj = os.path.join(out_dir, name + ".o")
    if ":" in src:  # another file compiled in place of a library source
        srcp, src = src.split(":")
    else:
        srcp = os.path.join(B.CSRC, src)
    subprocess.run([B.hipcc(), *B.CXXFLAGS, "-I", B.CSRC, *flags, "-c", srcp, "-o", obj], check=True)
    objs = [os.path.join(B.BUILD, os.path.basename(s)[:-4] + ".o") for s in B.sources() if os.path.basename(s) != src]
    so_dir = os.path.join(ROOT, "var_so")  # travels to the GPU box (build/ does not)
    os.makedirs(so_dir, exist_ok=True)
    so = os.path.join(so_dir, name + ".so")
    subprocess.run([B.hipcc(), "-shared", "-fPIC", f"--offload-arch={B.ARCH}", *objs, obj, "-o", so], check=True)
    print(so)


if __name__ == "__main__":
    main()
