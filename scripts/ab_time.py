#!/usr/bin/env python3
"""Median / min launch time of the hot-path kernels at the bench workloads, for same-box A/B of
library builds (STEREOCV_LIB=path selects the .so).  One JSON line per op.
    STEREOCV_LIB=... python scripts/ab_time.py [--ops cfg2,cfg3,...] [--reps 25] [--tag name]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from realtime_stereo_matcher_amd import functional as F  # noqa: E402


def feats(shape, dtype):
    g = torch.Generator(device="cuda").manual_seed(1234)
    return (torch.randn(*shape, device="cuda", generator=g).to(dtype),
            torch.randn(*shape, device="cuda", generator=g).to(dtype))


def _warp_nows(img, flow):
    """The warp without a workspace (sm_warp_by_flow: warp_kernel for two-channel flows)."""
    from realtime_stereo_matcher_amd import _lib
    N, C, Hi, Wi = img.shape
    _, c, h, w = flow.shape
    out = torch.empty((N, C, h, w), dtype=torch.float32, device="cuda")
    _lib.check(_lib.load().sm_warp_by_flow(img.data_ptr(), flow.data_ptr(), out.data_ptr(), _lib.SM_F32,
                                           N, C, Hi, Wi, h, w, c, None, None,
                                           torch.cuda.current_stream().cuda_stream), "warp")
    return out


def _autocast(f):
    with torch.autocast("cuda", dtype=torch.float16):
        return f()


def ops():
    return {
        # name: (setup -> callable, pairs per launch, algorithmic bytes per pair)
        "cfg2": (lambda: (lambda L, R: lambda: F.inner_product_volume(L, R, 192))(*feats((8, 64, 540, 960), torch.float32)),
                 8, 663552000),
        # the bench's launch since pairs per launch = the rank's whole batch (32 at N = 1)
        "cfg2_b32": (lambda: (lambda L, R: lambda: F.inner_product_volume(L, R, 192))(*feats((32, 64, 540, 960), torch.float32)),
                     32, 663552000),
        # round 5: the sliding-window kernel (AUTO) against the role-split one, bench shapes
        "cfg2_b32_rs": (lambda: (lambda L, R: lambda: F.inner_product_volume(L, R, 192, algo="rs"))(*feats((32, 64, 540, 960), torch.float32)),
                        32, 663552000),
        "cfg2_b32_sl": (lambda: (lambda L, R: lambda: F.inner_product_volume(L, R, 192, algo="sl"))(*feats((32, 64, 540, 960), torch.float32)),
                        32, 663552000),
        "cfg4_b32_rs": (lambda: (lambda L, R: lambda: F.correlation_volume(L, R, 256, algo="rs"))(*feats((32, 16, 1080, 1920), torch.float32)),
                        32, 2388787200),
        "cfg4_b4_auto": (lambda: (lambda L, R: lambda: F.correlation_volume(L, R, 256))(*feats((4, 16, 1080, 1920), torch.float32)),
                         4, 2388787200),
        "cfg2_fused_b32": (lambda: (lambda L, R: lambda: F.inner_product_soft_argmin(L, R, 192, keep_volume=True))(
            *feats((32, 64, 540, 960), torch.float32)), 32, 665625600),
        "cfg2_fused_nv_f16_b32": (lambda: (lambda L, R: lambda: _autocast(lambda: F.inner_product_soft_argmin(L, R, 192, keep_volume=False)))(
            *feats((32, 64, 540, 960), torch.float16)), 32, 134784000),
        "cfg4_fused_nv_f16_b32": (lambda: (lambda L, R: lambda: _autocast(lambda: F.inner_product_soft_argmin(L, R, 256, mean=True, keep_volume=False)))(
            *feats((32, 16, 1080, 1920), torch.float16)), 32, 74649600 + 8294400),
        "cfg4_b32": (lambda: (lambda L, R: lambda: F.correlation_volume(L, R, 256))(*feats((32, 16, 1080, 1920), torch.float32)),
                     32, 2388787200),
        "cfg2_fused_nv_b32": (lambda: (lambda L, R: lambda: F.inner_product_soft_argmin(L, R, 192, keep_volume=False))(
            *feats((32, 64, 540, 960), torch.float32)), 32, 267494400),
        "cfg4_fused_nv_b32": (lambda: (lambda L, R: lambda: F.inner_product_soft_argmin(L, R, 256, mean=True, keep_volume=False))(
            *feats((32, 16, 1080, 1920), torch.float32)), 32, 273715200),
        "cfg2_h2": (lambda: (lambda L, R: lambda: F.inner_product_volume(L, R, 192, algo="h2"))(*feats((8, 64, 540, 960), torch.float32)),
                    8, 663552000),
        "cfg2_h2db": (lambda: (lambda L, R: lambda: F.inner_product_volume(L, R, 192, algo="h2db"))(*feats((8, 64, 540, 960), torch.float32)),
                      8, 663552000),
        "cfg2_rs": (lambda: (lambda L, R: lambda: F.inner_product_volume(L, R, 192, algo="rs"))(*feats((8, 64, 540, 960), torch.float32)),
                    8, 663552000),
        "cfg2_fused": (lambda: (lambda L, R: lambda: F.inner_product_soft_argmin(L, R, 192, keep_volume=True))(
            *feats((8, 64, 540, 960), torch.float32)), 8, 665625600),
        "cfg2_fused_nv": (lambda: (lambda L, R: lambda: F.inner_product_soft_argmin(L, R, 192, keep_volume=False))(
            *feats((8, 64, 540, 960), torch.float32)), 8, 267494400),
        "cfg2_regress": (lambda: (lambda v: lambda: F.soft_argmin(v))(torch.randn(8, 192, 540, 960, device="cuda")),
                         8, 400204800),
        "cfg3": (lambda: (lambda L, R: lambda: F.groupwise_volume(L, R, 8, 192))(*feats((1, 256, 540, 960), torch.bfloat16)),
                 1, 3715891200),
        "cfg4": (lambda: (lambda L, R: lambda: F.correlation_volume(L, R, 256))(*feats((4, 16, 1080, 1920), torch.float32)),
                 4, 2388787200),
        "cfg4_rs": (lambda: (lambda L, R: lambda: F.correlation_volume(L, R, 256, algo="rs"))(*feats((4, 16, 1080, 1920), torch.float32)),
                    4, 2388787200),
        "cfg4_fused_nv": (lambda: (lambda L, R: lambda: F.inner_product_soft_argmin(L, R, 256, mean=True, keep_volume=False))(
            *feats((4, 16, 1080, 1920), torch.float32)), 4, 273715200),
        # f-4: 1x32x540x960 fp32 features warped by a 2-channel flow (sigma 4 px) / a disparity map
        "warp2": (lambda: (lambda img, fl: lambda: F.warp_by_flow_map(img, fl))(
            torch.randn(1, 32, 540, 960, device="cuda"), 4 * torch.randn(1, 2, 540, 960, device="cuda")),
            1, 136857600),
        "warp2_nows": (lambda: (lambda img, fl: lambda: _warp_nows(img, fl))(
            torch.randn(1, 32, 540, 960, device="cuda"), 4 * torch.randn(1, 2, 540, 960, device="cuda")),
            1, 136857600),
        "warp1": (lambda: (lambda img, fl: lambda: F.warp_by_flow_map(img, fl))(
            torch.randn(1, 32, 540, 960, device="cuda"), 192 * torch.rand(1, 1, 540, 960, device="cuda")),
            1, 134784000),
        "cfg5": (lambda: (lambda L, R: lambda: F.concat_volume(L, R, 64))(*feats((1, 128, 540, 960), torch.float16)),
                 1, 17252352000),
        # round 6: cfg5's output written by torch's sequential fill, the store-pattern ceiling
        "cfg5_fill": (lambda: (lambda o: lambda: o.zero_())(torch.empty(1, 256, 540, 960, 64, dtype=torch.float16, device="cuda")),
                      1, 17252352000),
        "cfg5_iw": (lambda: (lambda L, R: lambda: F.interweave_volume(L, R, 64))(*feats((1, 128, 540, 960), torch.float16)),
                    1, 17252352000),
        # round 6: the stale figures
        "cfg2_argext": (lambda: (lambda v: lambda: F.hard_argmax(v))(torch.randn(8, 192, 540, 960, device="cuda")),
                        8, 192 * 540 * 960 * 4 + 540 * 960 * 8),
        "cfg2_f32": (lambda: (lambda L, R: lambda: F.inner_product_volume(L, R, 192, algo="f32"))(*feats((8, 64, 540, 960), torch.float32)),
                     8, 663552000),
        "cfg2_valu": (lambda: (lambda L, R: lambda: F.inner_product_volume(L, R, 192, algo="valu"))(*feats((2, 64, 540, 960), torch.float32)),
                      2, 663552000),
        "cfg2_b32_auto": (lambda: (lambda L, R: lambda: F.inner_product_volume(L, R, 192))(*feats((32, 64, 540, 960), torch.float32)),
                          32, 663552000),
        **{f"ragged_{w}": (lambda w=w: (lambda L, R: lambda: F.inner_product_volume(L, R, 192))(*feats((8, 64, 540, w), torch.float32)),
                           8, (2 * 64 + 192) * 540 * w * 4) for w in (928, 944, 952, 956, 957, 958, 959, 960)},
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ops", default="cfg2")
    ap.add_argument("--reps", type=int, default=25)
    ap.add_argument("--tag", default=os.environ.get("STEREOCV_LIB", "default"))
    a = ap.parse_args()
    table = ops()
    for name in a.ops.split(","):
        setup, pairs, nbytes = table[name]
        fn = setup()
        for _ in range(5):
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
        ts.sort()
        med = ts[len(ts) // 2]
        print(json.dumps({"tag": os.path.basename(a.tag), "op": name, "median_us": round(med, 1),
                          "min_us": round(ts[0], 1), "us_per_pair": round(med / pairs, 2),
                          "frac": round(nbytes * pairs / (med * 1e-6) / 8e12, 4)}), flush=True)
        del fn
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
