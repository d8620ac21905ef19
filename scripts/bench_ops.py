#!/usr/bin/env python3
"""Per-operator timing at the BASELINE.json configs (HIP events, median of N launches).

Prints one JSON line per op: median kernel time, algorithmic bytes (read L + R,
write the output once) and the fraction of the 8 TB/s HBM roofline.
    python scripts/bench_ops.py [--reps 20] [--only name,...]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from realtime_stereo_matcher_amd import functional as F  # noqa: E402

PEAK = 8.0e12
MFMA_PEAK = 2.5e15  # dense bf16 / fp16 (MI355X_MICROARCH.md)


def timeit(fn, reps, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) * 1e-3)
    ts.sort()
    return ts[len(ts) // 2], ts[0]


def feats(shape, dtype, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    L = torch.randn(*shape, device="cuda", generator=g).to(dtype)
    R = torch.randn(*shape, device="cuda", generator=g).to(dtype)
    return L, R


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    only = set(filter(None, a.only.split(",")))
    rows = []

    def run(name, fn, nbytes, flops=None, **extra):
        if only and name not in only:
            return
        med, best = timeit(fn, a.reps)
        rec = {"op": name, "median_us": med * 1e6, "best_us": best * 1e6, "alg_bytes": nbytes,
               "GBps": nbytes / med / 1e9, "roofline_frac": nbytes / med / PEAK}
        if flops:  # valid-cell FLOPs against the dense bf16/fp16 MFMA peak
            rec.update(TFLOPs=flops / med / 1e12, mfma_peak_frac=flops / med / MFMA_PEAK)
        rec.update(extra)
        rows.append(rec)
        print(json.dumps(rec), flush=True)

    # cfg2: inner product fp32 1x64x540x960 D=192 (+ regression)
    L, R = feats((1, 64, 540, 960), torch.float32)
    n_in = 2 * L.numel() * 4
    vol_b = 192 * 540 * 960 * 4
    for algo in ("h2", "h2db", "rs", "sl", "f32", "valu"):
        run(f"inner_product_{algo}_cfg2", lambda: F.inner_product_volume(L, R, 192, algo=algo), n_in + vol_b)
    vol = F.inner_product_volume(L, R, 192)
    run("soft_argmin_cfg2", lambda: F.soft_argmin(vol), vol_b + 540 * 960 * 4)
    run("hard_argmax_cfg2", lambda: F.hard_argmax(vol), vol_b + 540 * 960 * 8)
    prob = torch.softmax(vol, 1)
    run("regression_presoftmax_cfg2", lambda: F.regression_presoftmax(prob), vol_b + 540 * 960 * 4)
    del vol, prob
    run("fused_ip_softargmin_cfg2", lambda: F.inner_product_soft_argmin(L, R, 192),
        n_in + vol_b + 540 * 960 * 4)
    run("fused_ip_softargmin_novol_cfg2",
        lambda: F.inner_product_soft_argmin(L, R, 192, keep_volume=False), n_in + 540 * 960 * 4)
    del L, R
    torch.cuda.empty_cache()

    # cfg3: groupwise bf16 1x256x540x960 G=8 D=192 -> fp32 (N,G,H,W,D)
    L, R = feats((1, 256, 540, 960), torch.bfloat16)
    run("groupwise_bf16_cfg3", lambda: F.groupwise_volume(L, R, 8, 192),
        2 * L.numel() * 2 + 8 * 540 * 960 * 192 * 4,
        flops=2 * 256 * 540 * sum(960 - d for d in range(192)))
    del L, R
    torch.cuda.empty_cache()

    # cfg4 per pair: correlation fp32 1x16x1080x1920 D=256 (mean)
    L, R = feats((1, 16, 1080, 1920), torch.float32)
    run("correlation_cfg4_pair", lambda: F.correlation_volume(L, R, 256),
        2 * L.numel() * 4 + 256 * 1080 * 1920 * 4)
    del L, R
    torch.cuda.empty_cache()

    # cfg5: concat / interweave fp16 1x128x540x960 D=64
    L, R = feats((1, 128, 540, 960), torch.float16)
    n_in = 2 * L.numel() * 2
    run("interweave_fp16_cfg5", lambda: F.interweave(L, R), 2 * n_in)
    run("concat_fp16_cfg5", lambda: F.concat_volume(L, R, 64), n_in + 256 * 540 * 960 * 64 * 2)
    run("interweave_shifted_fp16_cfg5", lambda: F.interweave_volume(L, R, 64),
        n_in + 256 * 540 * 960 * 64 * 2)
    run("diff_volume_fp16_cfg5", lambda: F.difference_volume(L, R, 64),
        n_in + 128 * 540 * 960 * 64 * 2)
    del L, R
    torch.cuda.empty_cache()
    # the in-model difference volume (v1-v3): 1x32x(H/8)x(W/8) at KITTI 1/8 res, D=24
    L, R = feats((1, 32, 68, 120), torch.float32)
    run("diff_volume_f32_model", lambda: F.difference_volume(L, R, 24),
        2 * L.numel() * 4 + 32 * 24 * 68 * 120 * 4)
    del L, R

    # §8f-4 warp: 1x32x540x960 fp32 features by a 0..192 disparity map (read image + flow,
    # write the warped map once)
    img, _ = feats((1, 32, 540, 960), torch.float32)
    disp = torch.rand(1, 1, 540, 960, device="cuda") * 192
    run("warp_disp_f32_540x960x32", lambda: F.warp_by_flow_map(img, disp),
        2 * img.numel() * 4 + disp.numel() * 4)
    ramp = torch.linspace(0, 192, 960, device="cuda").view(1, 1, 1, 960).expand(1, 1, 540, 960)
    smooth = (ramp + torch.rand(1, 1, 540, 960, device="cuda")).contiguous()  # slanted plane
    run("warp_smooth_disp_f32_540x960x32", lambda: F.warp_by_flow_map(img, smooth),
        2 * img.numel() * 4 + smooth.numel() * 4)
    flow2 = torch.randn(1, 2, 540, 960, device="cuda") * 4
    run("warp_flow2_f32_540x960x32", lambda: F.warp_by_flow_map(img, flow2),
        2 * img.numel() * 4 + flow2.numel() * 4)


if __name__ == "__main__":
    main()
