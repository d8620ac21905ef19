#!/usr/bin/env python3
"""Median kernel time (HIP events) of the inner-product volume at W % 4 != 0 widths next to
W = 960 (cfg2 otherwise): the band kernel serves fp32 rows of any width; algo "valu" is the
register-tiled VALU kernel that served them before.  Checks a few rows against fp64."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from realtime_stereo_matcher_amd import functional as F  # noqa: E402


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    g = torch.Generator(device="cuda").manual_seed(0)
    for W in (960, 958, 957, 959):
        L = torch.randn(1, 64, 540, W, device="cuda", generator=g)
        R = torch.randn(1, 64, 540, W, device="cuda", generator=g)
        nb = 2 * 64 * 540 * W * 4 + 192 * 540 * W * 4
        vol = F.inner_product_volume(L, R, 192)
        err = 0.0
        for y in (0, 269, 539):
            Ld, Rd = L[0, :, y].double(), R[0, :, y].double()
            for d in (0, 1, 2, 3, 97, 191):
                ref = (Ld[:, d:] * Rd[:, :W - d]).sum(0)
                err = max(err, (vol[0, d, y, d:].double() - ref).abs().max().item())
                err = max(err, vol[0, d, y, :d].abs().max().item() if d else 0.0)
        t = timeit(lambda: F.inner_product_volume(L, R, 192))
        tv = timeit(lambda: F.inner_product_volume(L, R, 192, algo="valu"), reps=5)
        print(f"W={W}: auto {t:.1f} us (frac {nb / t / 8e6:.3f}), valu {tv:.1f} us, max err {err:.3g}", flush=True)


if __name__ == "__main__":
    main()
