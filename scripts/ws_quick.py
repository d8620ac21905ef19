#!/usr/bin/env python3
"""Quick GPU check of the band kernels: parity of the warp-specialised kernel against an fp64
reference on sampled shapes, then median kernel times (HIP events) of ws vs h2 on the BASELINE
shapes.    python scripts/ws_quick.py [--skip-parity] [--skip-time]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from realtime_stereo_matcher_amd import functional as F  # noqa: E402


def ref_ip(L, R, D, mean=False, rows=None):
    """fp64 inner product / correlation volume (N, D, H, W) on the GPU (rows: subset of y)."""
    L64, R64 = L.double(), R.double()
    n, c, h, w = L.shape
    ys = range(h) if rows is None else rows
    out = torch.zeros(n, D, len(ys), w, dtype=torch.float64, device=L.device)
    for i, y in enumerate(ys):
        for d in range(min(D, w)):
            out[:, d, i, d:] = (L64[:, :, y, d:] * R64[:, :, y, :w - d]).sum(1)
    return out / c if mean else out


def ref_gw(L, R, G, D):
    L64, R64 = L.double(), R.double()
    n, c, h, w = L.shape
    out = torch.zeros(n, G, h, w, D, dtype=torch.float64, device=L.device)
    cg = c // G
    for d in range(min(D, w)):
        p = (L64[..., d:] * R64[..., :w - d]).view(n, G, cg, h, w - d).mean(2)
        out[..., d:, d] = p
    return out


def ref_softargmin(vol):
    p = torch.softmax(vol.double(), dim=1)
    d = torch.arange(vol.shape[1], device=vol.device, dtype=torch.float64).view(1, -1, 1, 1)
    return (p * d).sum(1, keepdim=True)


def parity():
    g = torch.Generator(device="cuda").manual_seed(0)
    worst = 0.0
    ok = True
    for (n, c, h, w, D, scale) in [(1, 64, 3, 256, 192, 1.0), (2, 16, 2, 200, 40, 1.0), (1, 24, 2, 132, 9, 1.0),
                                    (1, 64, 2, 960, 192, 1.0), (1, 32, 2, 100, 64, 1e-6), (1, 32, 2, 128, 100, 1e5),
                                    (1, 8, 3, 64, 256, 1.0), (1, 48, 2, 4, 3, 1.0)]:
        L = torch.randn(n, c, h, w, device="cuda", generator=g) * scale
        R = torch.randn(n, c, h, w, device="cuda", generator=g) * scale
        for mean in (False, True):
            got = (F.correlation_volume(L, R, D) if mean else F.inner_product_volume(L, R, D, algo="ws")).double()
            ref = ref_ip(L, R, D, mean)
            bound = (ref_ip(L.abs(), R.abs(), D, mean) * 1e-5).clamp_min(1e-30)
            err = ((got - ref).abs() / bound).max().item()
            worst = max(worst, err)
            flag = "OK" if err <= 1.0 else "FAIL"
            ok &= err <= 1.0
            print(f"ip mean={mean} {n}x{c}x{h}x{w} D={D} scale={scale}: max err/bound {err:.3g} {flag}", flush=True)
        if D <= 192:
            vol, disp = F.inner_product_soft_argmin(L, R, D, keep_volume=True)
            _, disp2 = F.inner_product_soft_argmin(L, R, D, keep_volume=False)
            own = ref_softargmin(vol)  # fp64 soft-argmin of the kernel's own volume
            e = (disp.double() - own).abs().max().item()
            same = torch.equal(disp, disp2) and torch.equal(vol, F.inner_product_volume(L, R, D, algo="ws"))
            # context: the deviation of a torch-fp32 volume's disparity from the fp64 pipeline
            rd = ref_softargmin(ref_ip(L, R, D))
            e64 = (disp.double() - rd).abs().max().item()
            t32 = (ref_softargmin(ref_ip(L, R, D).float()) - rd).abs().max().item()
            ok &= e <= 1e-4 and same
            print(f"  fused: |disp - fp64 softargmin(own vol)| {e:.3g}, bit-identical volume/no-volume {same}; "
                  f"vs fp64 pipeline {e64:.3g} (fp32-rounded exact volume: {t32:.3g}) "
                  f"{'OK' if e <= 1e-4 and same else 'FAIL'}", flush=True)
    for (n, c, h, w, G, D, dt) in [(1, 64, 2, 256, 8, 192, torch.bfloat16), (1, 32, 2, 100, 2, 24, torch.float32),
                                   (1, 16, 2, 64, 4, 7, torch.float16), (1, 64, 2, 960, 8, 192, torch.bfloat16)]:
        L = torch.randn(n, c, h, w, device="cuda", generator=g).to(dt)
        R = torch.randn(n, c, h, w, device="cuda", generator=g).to(dt)
        got = F.groupwise_volume(L, R, G, D).double()
        ref = ref_gw(L, R, G, D)
        e = (got - ref).abs().max().item()
        ok &= e <= 1e-4
        print(f"gw {dt} {n}x{c}x{h}x{w} G={G} D={D}: max err {e:.3g} {'OK' if e <= 1e-4 else 'FAIL'}", flush=True)
    for dt in (torch.float16, torch.bfloat16):
        L = torch.randn(1, 32, 2, 256, device="cuda", generator=g).to(dt)
        R = torch.randn(1, 32, 2, 256, device="cuda", generator=g).to(dt)
        got = F.inner_product_volume(L, R, 96, algo="ws").double()
        ref = ref_ip(L, R, 96)
        e = ((got - ref).abs() / ref.abs().clamp_min(1.0)).max().item()
        ok &= e <= 2 ** -7
        print(f"ip {dt}: max rel err {e:.3g} {'OK' if e <= 2 ** -7 else 'FAIL'}", flush=True)
    # non-finite features take the exact path
    L = torch.randn(1, 16, 2, 256, device="cuda", generator=g)
    R = torch.randn(1, 16, 2, 256, device="cuda", generator=g)
    L[0, 3, 1, 77] = float("inf")
    R[0, 5, 0, 10] = float("nan")
    got = F.inner_product_volume(L, R, 64, algo="ws").double()
    ref = ref_ip(L, R, 64)
    same_nan = torch.equal(torch.isnan(got), torch.isnan(ref))
    fin = torch.isfinite(ref)
    e = (got[fin] - ref[fin]).abs().max().item()
    ok &= same_nan and e <= 1e-4 and torch.equal(torch.isinf(got), torch.isinf(ref))
    print(f"nonfinite: nan pattern {same_nan}, max err {e:.3g}", flush=True)
    print("PARITY", "OK" if ok else "FAIL", flush=True)
    return ok


def timeit(fn, reps=20):
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


def timing():
    g = torch.Generator(device="cuda").manual_seed(0)
    L = torch.randn(1, 64, 540, 960, device="cuda", generator=g)
    R = torch.randn(1, 64, 540, 960, device="cuda", generator=g)
    nb = 663552000
    for algo in ("ws", "h2", "ws", "h2"):
        t = timeit(lambda: F.inner_product_volume(L, R, 192, algo=algo))
        print(f"cfg2 ip {algo}: {t:.1f} us  frac {nb / t / 8e6:.3f}", flush=True)
    t = timeit(lambda: F.inner_product_soft_argmin(L, R, 192, keep_volume=False))
    print(f"cfg2 fused-novolume ws: {t:.1f} us  frac {267494400 / t / 8e6:.3f}", flush=True)
    t = timeit(lambda: F.inner_product_soft_argmin(L, R, 192, keep_volume=True))
    print(f"cfg2 fused (volume) ws: {t:.1f} us  frac {665625600 / t / 8e6:.3f}", flush=True)
    del L, R
    Lb = torch.randn(1, 256, 540, 960, device="cuda", generator=g).bfloat16()
    Rb = torch.randn(1, 256, 540, 960, device="cuda", generator=g).bfloat16()
    t = timeit(lambda: F.groupwise_volume(Lb, Rb, 8, 192))
    print(f"cfg3 groupwise ws: {t:.1f} us  frac {3715891200 / t / 8e6:.3f}", flush=True)
    del Lb, Rb
    L4 = torch.randn(1, 16, 1080, 1920, device="cuda", generator=g)
    R4 = torch.randn(1, 16, 1080, 1920, device="cuda", generator=g)
    t = timeit(lambda: F.correlation_volume(L4, R4, 256))
    print(f"cfg4 correlation ws (1 pair): {t:.1f} us  frac {2388787200 / t / 8e6:.3f}", flush=True)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--skip-parity", action="store_true")
    ap.add_argument("--skip-time", action="store_true")
    a = ap.parse_args()
    ok = True
    if not a.skip_parity:
        ok = parity()
    if not a.skip_time and ok:
        timing()
    sys.exit(0 if ok else 1)
