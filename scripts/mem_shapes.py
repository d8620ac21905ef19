"""Round 6: the cfg2 write and read streams by the x-width a workgroup owns
(scripts/micro/mem_shapes.hip), beside band_rs and a sequential fill, on the first (A) and a later
(B) volume-sized torch buffer.   python scripts/mem_shapes.py [--pairs 32] [--reps 5]"""
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

CASES = [("w px128 nt (band_rs)", 0, "w"), ("w px256 nt", 1, "w"), ("w px512 nt", 2, "w"),
         ("w row nt", 3, "w"), ("w transposed nt", 4, "w"), ("w px128 plain", 5, "w"),
         ("w row plain", 6, "w"), ("w transposed plain", 7, "w"),
         ("r px128 +win (band_rs)", 10, "r"), ("r px128", 11, "r"), ("r px256", 12, "r"),
         ("r px512", 13, "r"), ("r row", 14, "r"), ("r px256 +win", 15, "r"),
         ("r px128 +hot win", 16, "r"), ("w rowwalk xcd", 20, "w"), ("w rowwalk global", 21, "w"),
         ("r rowwalk xcd", 22, "r"), ("r rowwalk global", 23, "r"), ("r rowwalk xcd +win", 24, "r"),
         ("rw units +win (band_rs)", 30, "rw"), ("rw units", 31, "rw"), ("rw rowwalk xcd +win", 32, "rw"),
         ("rw rowwalk xcd (band_sl)", 33, "rw"), ("band_sl", "sl", "rw"),
         ("w rowwalk xcd stagger wg", 25, "w"), ("w rowwalk xcd stagger wg+unit", 26, "w"),
         ("w units stagger wg", 27, "w"),
         ("gw w 4 waves nt (band_rs GW)", 40, "gw"), ("gw w 4 waves plain", 41, "gw"),
         ("gw w 8 waves nt", 42, "gw"), ("gw w 8 waves plain", 43, "gw"),
         ("gw w rowwalk 4 waves nt", 44, "gw"), ("gw w rowwalk 4 waves plain", 45, "gw")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=32)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--only", default="", help="comma-separated variant numbers")
    ap.add_argument("--gw-pairs", type=int, default=0, help="groupwise write cases only, with N pairs")
    a = ap.parse_args()
    n, c, h, w, D = a.pairs, 64, 540, 960, 192
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    L = torch.randn(n, c, h, w, device=dev, generator=g)
    R = torch.randn(n, c, h, w, device=dev, generator=g)
    A = torch.empty(n, D, h, w, device=dev)
    B = torch.empty(n, D, h, w, device=dev)
    micro = ctypes.CDLL(os.path.join(ROOT, "scripts", "micro", "libmem_shapes.so"))
    micro.mem_run.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 3 + [ctypes.c_int, ctypes.c_void_p]
    lib = _lib.load()
    st = torch.cuda.current_stream()
    nbytes = {"r": 2 * c * h * w * 4, "w": D * h * w * 4, "rw": 2 * c * h * w * 4 + D * h * w * 4,
              "gw": 8 * D * h * w * 4}
    if a.gw_pairs:  # the groupwise writes need G x the volume: their own buffers (A, B per cfg3 pair)
        n = a.gw_pairs

    def timed(variant, vol):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        if variant == "fill":
            vol.zero_()
        elif variant in ("rs", "sl"):
            _lib.check(lib.sm_cv_inner_product_ex(L.data_ptr(), R.data_ptr(), vol.data_ptr(), _lib.SM_F32, n, c, h,
                                                  w, D, _lib.strides_arg(L), _lib.strides_arg(R),
                                                  11 if variant == "rs" else 12, st.cuda_stream),
                       "sm_cv_inner_product_ex")
        else:
            rc = micro.mem_run(variant, L.data_ptr(), R.data_ptr(), vol.data_ptr(), n, st.cuda_stream)
            if rc:
                raise RuntimeError(f"mem_run({variant}) = {rc}")
        e1.record(st)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3

    for _ in range(3):
        timed("rs", A)
        timed("rs", B)
    for rnd in range(2):
        sel = [c for c in CASES if not a.only or str(c[1]) in a.only.split(",")]
        for name, variant, kind in [("band_rs", "rs", "rw"), ("zero_ fill", "fill", "w")] + sel:
            timed(variant, A)
            ta, tb = [], []
            for _ in range(a.reps):
                ta.append(timed(variant, A))
                tb.append(timed(variant, B))
            for buf, ts in (("A", ta), ("B", tb)):
                med = statistics.median(ts)
                print(json.dumps({"round": rnd, "case": name, "buf": buf, "median_us": round(med, 1),
                                  "TBps": round(n * nbytes[kind] / med / 1e6, 3),
                                  "frac": round(n * nbytes[kind] / (med * 1e-6) / 8e12, 4)}), flush=True)


if __name__ == "__main__":
    main()
