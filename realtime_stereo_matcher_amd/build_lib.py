"""Build libstereocv.so (all HIP sources under csrc/) for gfx950 with hipcc, in-tree.

    python -m realtime_stereo_matcher_amd.build_lib [--jobs N]

Objects are compiled in parallel into build/ and linked into
realtime_stereo_matcher_amd/libstereocv.so (git-ignored; it travels to the GPU box).
"""
import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
BUILD = os.path.join(ROOT, "build", "stereocv")
LIB = os.path.join(PKG, "libstereocv.so")
ARCH = "gfx950"
CXXFLAGS = ["-O3", "-std=c++20", "-fPIC", f"--offload-arch={ARCH}", "-I", os.path.join(ROOT, "include"),
            "-Wall", "-Wno-unused-function", "-munsafe-fp-atomics"]


# per-source extra flags (none at present)
EXTRA = {}


def hipcc():
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm required to build libstereocv.so)")


def sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hip"))


def _compile(src):
    obj = os.path.join(BUILD, os.path.basename(src)[:-4] + ".o")
    deps = [src] + [os.path.join(CSRC, h) for h in os.listdir(CSRC) if h.endswith(".h")]
    deps.append(os.path.join(ROOT, "include", "stereocv.h"))
    if os.path.exists(obj) and all(os.path.getmtime(obj) >= os.path.getmtime(d) for d in deps):
        return obj
    cmd = [hipcc(), *CXXFLAGS, *EXTRA.get(os.path.basename(src), []), "-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed on {src}:\n{r.stdout}\n{r.stderr}")
    return obj


def build(jobs=8, verbose=True):
    os.makedirs(BUILD, exist_ok=True)
    srcs = sources()
    with cf.ThreadPoolExecutor(max_workers=max(1, min(jobs, 16))) as ex:
        objs = list(ex.map(_compile, srcs))
    if os.path.exists(LIB) and all(os.path.getmtime(LIB) >= os.path.getmtime(o) for o in objs):
        return LIB
    tmp = LIB + ".tmp"
    cmd = [hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", tmp]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, LIB)
    if verbose:
        print(f"built {LIB}")
    return LIB


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=8)
    a = ap.parse_args()
    try:
        build(a.jobs)
    except RuntimeError as e:
        print(e, file=sys.stderr)
        sys.exit(1)
