"""Same-process A/B of library builds on the bench's cfg2 / cfg4 launches (round 6).

Every library (libstereocv.so and var_so/*.so builds) is loaded with ctypes into ONE process, so
all of them write into the same two volume buffers: A, the process's first volume-sized torch
allocation (the one some boxes map slowly, profiles/r05/placement/), and B, a later one.  Cases
alternate A / B as the bench's steps do.

  python scripts/ab_libs.py LIB[=name] ... [--cases cfg2_rs,cfg2_sl,...] [--reps 6] [--rounds 2]

Cases: cfg2_<algo> (the 32-pair inner-product volume with algo rs / sl / auto), cfg2_fused /
cfg2_fusednv (the fused pass with / without the volume), cfg4_<algo> (32-pair correlation
volume D = 256), cfg4_fusednv, cfg3_auto (groupwise bf16, G = 8; use --pairs 1)."""
import argparse
import ctypes
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from realtime_stereo_matcher_amd import _lib  # noqa: E402

ALGO = {"auto": 0, "rs": 11, "sl": 12, "h2db": 8}


def load(path):
    lib = ctypes.CDLL(path)
    for name, args in _lib.SIGNATURES.items():
        f = getattr(lib, name, None)
        if f is not None:
            f.argtypes = args
            f.restype = _lib._RESTYPE.get(name, ctypes.c_int)
    return lib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--cases", default="cfg2_rs,cfg2_sl")
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--pairs", type=int, default=32)
    a = ap.parse_args()
    libs = []
    for spec in a.libs:
        path, _, name = spec.partition("=")
        libs.append((name or os.path.basename(path), load(os.path.join(ROOT, path))))
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream()
    cases = a.cases.split(",")
    g = torch.Generator(device=dev).manual_seed(0)
    n = a.pairs
    need4 = any(c.startswith("cfg4") for c in cases)
    need2 = any(c.startswith("cfg2") for c in cases)
    need3 = any(c.startswith("cfg3") for c in cases)
    data = {}
    if need3:  # groupwise bf16, G = 8, (N, G, H, W, D) fp32 out
        data["cfg3"] = (torch.randn(n, 256, 540, 960, device=dev, generator=g).bfloat16(),
                        torch.randn(n, 256, 540, 960, device=dev, generator=g).bfloat16(), 192, 540, 960)
    if need2:
        data["cfg2"] = (torch.randn(n, 64, 540, 960, device=dev, generator=g),
                        torch.randn(n, 64, 540, 960, device=dev, generator=g), 192, 540, 960)
    if need4:
        data["cfg4"] = (torch.randn(n, 16, 1080, 1920, device=dev, generator=g),
                        torch.randn(n, 16, 1080, 1920, device=dev, generator=g), 256, 1080, 1920)
    vols = {}
    for k, (L, R, D, h, w) in data.items():
        G = 8 if k == "cfg3" else 1
        vols[k] = (torch.empty(n, G * D, h, w, device=dev), torch.empty(n, G * D, h, w, device=dev))
    disp = {k: torch.empty(n, 1, v[3], v[4], device=dev) for k, v in data.items()}

    def launch(lib, case, vol):
        cfg, _, kind = case.partition("_")
        L, R, D, h, w = data[cfg]
        c = L.shape[1]
        ls, rs = _lib.strides_arg(L), _lib.strides_arg(R)
        mean = cfg == "cfg4"
        if cfg == "cfg3":
            rc = lib.sm_cv_groupwise(L.data_ptr(), R.data_ptr(), vol.data_ptr(), _lib.SM_BF16, n, c, h, w, D, 8,
                                     ls, rs, st.cuda_stream)
        elif kind.startswith("fused"):
            keep = kind == "fused"
            rc = lib.sm_cv_inner_product_softargmin_ws(L.data_ptr(), R.data_ptr(), vol.data_ptr() if keep else None,
                                                       disp[cfg].data_ptr(), _lib.SM_F32, n, c, h, w, D, ls, rs,
                                                       1 if mean else 0, None, 0, st.cuda_stream)
        elif mean:
            rc = lib.sm_cv_correlation_mean_ex(L.data_ptr(), R.data_ptr(), vol.data_ptr(), _lib.SM_F32, n, c, h, w,
                                               D, ls, rs, ALGO[kind], st.cuda_stream)
        else:
            rc = lib.sm_cv_inner_product_ex(L.data_ptr(), R.data_ptr(), vol.data_ptr(), _lib.SM_F32, n, c, h, w,
                                            D, ls, rs, ALGO[kind], st.cuda_stream)
        if rc != 0:
            raise RuntimeError(f"{case}: rc {rc}")

    def timed(lib, case, vol):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        launch(lib, case, vol)
        e1.record(st)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3

    alg = {"cfg2": 663552000, "cfg4": 2388787200, "cfg3": 3715891200}
    for rnd in range(a.rounds):
        for case in cases:
            for name, lib in libs:
                A, B = vols[case.split("_")[0]]
                timed(lib, case, A)
                ta, tb = [], []
                for _ in range(a.reps):
                    ta.append(timed(lib, case, A))
                    tb.append(timed(lib, case, B))
                for buf, ts in (("A", ta), ("B", tb)):
                    med = statistics.median(ts)
                    cfg = case.split("_")[0]
                    print(json.dumps({"round": rnd, "case": case, "lib": name, "buf": buf,
                                      "median_us": round(med, 1), "min_us": round(min(ts), 1),
                                      "frac_volume_bytes": round(n * alg[cfg] / (med * 1e-6) / 8e12, 4)}),
                          flush=True)


if __name__ == "__main__":
    main()
