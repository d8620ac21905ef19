#!/usr/bin/env python3
"""Run one operator a few times (for rocprofv3 counter passes / ablation timing).
    python scripts/prof_op.py inner_product_mfma_cfg2 [--reps 5]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from realtime_stereo_matcher_amd import functional as F  # noqa: E402


def feats(shape, dtype):
    g = torch.Generator(device="cuda").manual_seed(0)
    return (torch.randn(*shape, device="cuda", generator=g).to(dtype),
            torch.randn(*shape, device="cuda", generator=g).to(dtype))


OPS = {
    "inner_product_mfma_cfg2": lambda: (lambda L, R: lambda: F.inner_product_volume(L, R, 192, algo="mfma"))(*feats((1, 64, 540, 960), torch.float32)),
    "inner_product_h2_cfg2": lambda: (lambda L, R: lambda: F.inner_product_volume(L, R, 192, algo="h2"))(*feats((1, 64, 540, 960), torch.float32)),
    "inner_product_valu_cfg2": lambda: (lambda L, R: lambda: F.inner_product_volume(L, R, 192, algo="valu"))(*feats((1, 64, 540, 960), torch.float32)),
    "soft_argmin_cfg2": lambda: (lambda v: lambda: F.soft_argmin(v))(torch.randn(1, 192, 540, 960, device="cuda")),
    "groupwise_bf16_cfg3": lambda: (lambda L, R: lambda: F.groupwise_volume(L, R, 8, 192))(*feats((1, 256, 540, 960), torch.bfloat16)),
    "correlation_cfg4_pair": lambda: (lambda L, R: lambda: F.correlation_volume(L, R, 256))(*feats((1, 16, 1080, 1920), torch.float32)),
    "concat_fp16_cfg5": lambda: (lambda L, R: lambda: F.concat_volume(L, R, 64))(*feats((1, 128, 540, 960), torch.float16)),
}

if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("op", choices=sorted(OPS))
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--time", action="store_true", help="print the median kernel time")
    a = ap.parse_args()
    fn = OPS[a.op]()
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(a.reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) * 1e3)
    if a.time:
        ts.sort()
        print(f"{a.op} ablate={os.environ.get('STEREOCV_ABLATE', '0')} median_us={ts[len(ts) // 2]:.1f}")
