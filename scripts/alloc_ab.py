#!/usr/bin/env python3
"""Diagnostic: does the band kernel's speed depend on where its output volume lands in HBM?
Times the default cfg2 volume launch (sm_cv_inner_product_ex, algo auto) into output buffers
from torch's caching allocator, plain hipMalloc and hipExtMallocWithFlags(hipDeviceMallocContiguous),
a fresh buffer per trial.   python scripts/alloc_ab.py [--pairs 8,32] [--trials 3]"""
import argparse
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from realtime_stereo_matcher_amd import _lib, functional as F  # noqa: E402

HIP = ctypes.CDLL("libamdhip64.so")
CONTIGUOUS = 0x4  # hipDeviceMallocContiguous (hip_runtime_api.h)


def hip_alloc(nbytes, flags):
    p = ctypes.c_void_p()
    if flags is None:
        rc = HIP.hipMalloc(ctypes.byref(p), ctypes.c_size_t(nbytes))
    else:
        rc = HIP.hipExtMallocWithFlags(ctypes.byref(p), ctypes.c_size_t(nbytes), ctypes.c_uint(flags))
    return p.value if rc == 0 else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", default="8,32")
    ap.add_argument("--trials", type=int, default=3)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    lib = _lib.load()
    C, H, W, D = 64, 540, 960, 192
    for n in [int(x) for x in a.pairs.split(",")]:
        g = torch.Generator(device="cuda").manual_seed(5)
        L = torch.randn(n, C, H, W, device="cuda", generator=g)
        R = torch.randn(n, C, H, W, device="cuda", generator=g)
        nbytes = n * D * H * W * 4
        st = torch.cuda.current_stream().cuda_stream
        for trial in range(a.trials):
            for mode in ("torch", "hipMalloc", "contiguous"):
                keep = None
                if mode == "torch":
                    keep = torch.empty(n, D, H, W, device="cuda")
                    ptr = keep.data_ptr()
                else:
                    ptr = hip_alloc(nbytes, None if mode == "hipMalloc" else CONTIGUOUS)
                    if ptr is None:
                        print(json.dumps({"pairs": n, "mode": mode, "trial": trial, "alloc": "failed"}), flush=True)
                        continue

                def run():
                    _lib.check(lib.sm_cv_inner_product_ex(
                        L.data_ptr(), R.data_ptr(), ptr, F._dtype_code(L), n, C, H, W, D,
                        _lib.strides_arg(L), _lib.strides_arg(R), F._ALGOS["auto"], st), "alloc_ab")

                for _ in range(3):
                    run()
                torch.cuda.synchronize()
                ts = []
                for _ in range(a.reps):
                    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    s.record()
                    run()
                    e.record()
                    e.synchronize()
                    ts.append(s.elapsed_time(e) * 1e3)
                ts.sort()
                med = ts[len(ts) // 2]
                frac = (2 * n * C * H * W * 4 + nbytes) / (med * 1e-6) / 8e12
                print(json.dumps({"pairs": n, "mode": mode, "trial": trial, "median_us": round(med, 1),
                                  "us_per_pair": round(med / n, 2), "frac": round(frac, 4),
                                  "ptr_mod_2M": ptr % (1 << 21), "ptr_mod_1G": ptr % (1 << 30)}), flush=True)
                torch.cuda.synchronize()
                if keep is None:
                    HIP.hipFree(ctypes.c_void_p(ptr))
                del keep
        del L, R
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
