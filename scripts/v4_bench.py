#!/usr/bin/env python3
"""§8f-2 measurement: MobileStereoNetV4's cost volume (model/mobile_stereo_net_v4.py:443-461) at
the 1/4-resolution features of a KITTI frame (384x1248 -> 1x32x96x312, D = 48) three ways on one
MI355X: the reference's own loop (48 x interweave + Conv3d stack + volume11, torch eager on
MIOpen), the same arithmetic batched over the disparities (impl="torch"), and the fused HIP
operator (sm_v4_volume).  Prints one JSON line; max |HIP - reference loop| is checked.

    python scripts/v4_bench.py [--shape N C H W] [--reps 20]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from realtime_stereo_matcher_amd.model.mobile_stereo_net_v4 import interweave_conv_volume  # noqa: E402
from realtime_stereo_matcher_amd.model.stereo_net_v4 import MobileStereoNetV4HIP  # noqa: E402

MFMA_16BIT_PEAK_TF = 2500.0


def reference_loop(fL, fR, conv3d, volume11, D):
    """The reference's loop, op for op (mobile_stereo_net_v4.py:443-461, interweave :17-23)."""
    B, C, H, W = fL.shape
    volume = fL.new_zeros([B, 1, D, H, W])
    for i in range(D):
        l, r = (fL[:, :, :, i:], fR[:, :, :, :-i]) if i > 0 else (fL, fR)
        x = l.new_zeros([B, 2 * C, H, l.shape[3]])
        x[:, ::2] = l
        x[:, 1::2] = r
        x = volume11(torch.squeeze(conv3d(torch.unsqueeze(x.contiguous(), 1)), 2))
        volume[:, :, i, :, i:] = x
    return volume.squeeze(1)


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", type=int, nargs=4, default=[1, 32, 96, 312])
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    n, c, h, w = a.shape
    D = 48
    torch.manual_seed(0)
    net = MobileStereoNetV4HIP(192).cuda().eval()
    g = torch.Generator(device="cuda").manual_seed(0)
    fL = torch.randn(n, c, h, w, device="cuda", generator=g)
    fR = torch.randn(n, c, h, w, device="cuda", generator=g)
    with torch.no_grad():
        ref = reference_loop(fL, fR, net.conv3d, net.volume11, D)
        hip = interweave_conv_volume(fL, fR, net.conv3d, net.volume11, D)
        err = (hip - ref).abs().max().item()
        t_ref = timeit(lambda: reference_loop(fL, fR, net.conv3d, net.volume11, D), max(3, a.reps // 4))
        t_bat = timeit(lambda: interweave_conv_volume(fL, fR, net.conv3d, net.volume11, D, impl="torch"), a.reps)
        t_hip = timeit(lambda: interweave_conv_volume(fL, fR, net.conv3d, net.volume11, D), a.reps)
    cells = n * h * sum(max(0, w - i) for i in range(D))
    useful = cells * (2 * 32 * 576 * 2 + 16 * 576 * 2)  # layers 2 + 3 (the MFMA part), 2 flops/FMA
    rec = {"op": "v4_volume (interweave + Conv3d stack + volume11, D=48)",
           "shape": [n, c, h, w], "D": D, "max_abs_err_vs_reference_loop": err,
           "ms": {"reference_loop_torch": t_ref, "batched_torch_miopen": t_bat, "hip_fused": t_hip},
           "speedup_vs_reference_loop": t_ref / t_hip, "speedup_vs_batched": t_bat / t_hip,
           "mfma": {"useful_tflops": useful / (t_hip * 1e-3) / 1e12, "peak": MFMA_16BIT_PEAK_TF,
                    "frac_useful": useful / (t_hip * 1e-3) / 1e12 / MFMA_16BIT_PEAK_TF,
                    "frac_issued": 3 * useful * (34 * 32) / (30 * 32) / (t_hip * 1e-3) / 1e12 / MFMA_16BIT_PEAK_TF,
                    "note": "useful = layer-2/3 flops of valid cells; issued ~ 3x (scaled fp16 hi/lo split) x strip halo"}}
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
