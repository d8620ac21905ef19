#!/usr/bin/env python3
"""Experiment: cfg2 volume + soft-argmin, whole image vs row chunks (does the chunk's volume come
back from the 256 MiB Infinity Cache?).  python scripts/exp_chunks.py"""
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
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


g = torch.Generator(device="cuda").manual_seed(0)
L = torch.randn(1, 64, 540, 960, device="cuda", generator=g)
R = torch.randn(1, 64, 540, 960, device="cuda", generator=g)
D = 192


def separate():
    return F.soft_argmin(F.inner_product_volume(L, R, D))


def chunked(k):
    bounds = [round(540 * i / k) for i in range(k + 1)]

    def fn():
        out = torch.empty(1, 1, 540, 960, device="cuda")
        for y0, y1 in zip(bounds[:-1], bounds[1:]):
            v = F.inner_product_volume(L[:, :, y0:y1], R[:, :, y0:y1], D)
            out[:, :, y0:y1] = F.soft_argmin(v)
        return out
    return fn


ref = separate()
print(f"separate         {timeit(separate):8.1f} us")
for k in (2, 3, 4, 6, 8):
    fn = chunked(k)
    assert torch.equal(fn(), ref)
    print(f"chunked k={k}      {timeit(fn):8.1f} us")
vol = F.inner_product_volume(L, R, D)
print(f"volume only      {timeit(lambda: F.inner_product_volume(L, R, D)):8.1f} us")
print(f"soft-argmin only {timeit(lambda: F.soft_argmin(vol)):8.1f} us")
half = F.inner_product_volume(L[:, :, :135], R[:, :, :135], D)
print(f"soft-argmin 1/4 (warm) {timeit(lambda: F.soft_argmin(half)):8.1f} us")
print(f"fused            {timeit(lambda: F.inner_product_soft_argmin(L, R, D)):8.1f} us")
