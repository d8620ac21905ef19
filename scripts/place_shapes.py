"""Round-6 placement experiment: the band kernel's memory pattern with three
volume-store shapes (scripts/micro/place_shapes.hip), on a process's first volume-sized torch
buffer (A) and a later one (B), allocated in the bench's order (features, then the volumes);
band_rs (libstereocv, algo 11) on the same two buffers beside it.

  python scripts/place_shapes.py [--pairs 32] [--reps 6]

One JSON line per (case, buffer): median / min µs per launch and the fraction of the 8 TB/s peak
for the case's algorithmic bytes."""
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

CASES = [  # (name, variant = MODE * 4 + SHAPE, bytes per pair)
    ("reads", 1 * 4 + 0, "r"),
    ("reads lds-dma", 33 * 4 + 0, "r"),
    ("writes 8x128B", 2 * 4 + 0, "w"),
    ("writes 4x256B", 2 * 4 + 1, "w"),
    ("writes 2x512B", 2 * 4 + 2, "w"),
    ("mixed 8x128B", 3 * 4 + 0, "rw"),
    ("mixed 4x256B", 3 * 4 + 1, "rw"),
    ("mixed 2x512B", 3 * 4 + 2, "rw"),
    ("mixed lds-dma 8x128B", 35 * 4 + 0, "rw"),
    ("mixed lds-dma 2x512B", 35 * 4 + 2, "rw"),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=32)
    ap.add_argument("--reps", type=int, default=6)
    a = ap.parse_args()
    n, c, h, w, D = a.pairs, 64, 540, 960, 192
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    L = torch.randn(n, c, h, w, device=dev, generator=g)
    R = torch.randn(n, c, h, w, device=dev, generator=g)
    A = torch.empty(n, D, h, w, device=dev)
    B = torch.empty(n, D, h, w, device=dev)
    micro = ctypes.CDLL(os.path.join(ROOT, "scripts", "micro", "libplace_shapes.so"))
    micro.pshape_run.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 3 + [ctypes.c_int, ctypes.c_void_p]
    lib = _lib.load()
    st = torch.cuda.current_stream()
    rd, wr = 2 * c * h * w * 4, D * h * w * 4
    nbytes = {"r": rd, "w": wr, "rw": rd + wr}

    def launch(variant, vol):
        if variant is None:
            _lib.check(lib.sm_cv_inner_product_ex(L.data_ptr(), R.data_ptr(), vol.data_ptr(), _lib.SM_F32, n, c, h,
                                                  w, D, _lib.strides_arg(L), _lib.strides_arg(R), 11,
                                                  st.cuda_stream), "sm_cv_inner_product_ex")
            return
        rc = micro.pshape_run(variant, L.data_ptr(), R.data_ptr(), vol.data_ptr(), n, st.cuda_stream)
        if rc != 0:
            raise RuntimeError(f"pshape_run({variant}) = {rc}")

    def timed(variant, vol):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        if variant == "fill":
            vol.zero_()
        else:
            launch(variant, vol)
        e1.record(st)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3

    for _ in range(3):
        timed(None, A)
        timed(None, B)
    for rnd in range(2):
        for name, variant, kind in [("band_rs", None, "rw"), ("zero_ fill", "fill", "w")] + CASES:
            timed(variant, A)
            ta, tb = [], []
            for _ in range(a.reps):  # alternating, as the bench's steps do
                ta.append(timed(variant, A))
                tb.append(timed(variant, B))
            for buf, ts in (("A", ta), ("B", tb)):
                med = statistics.median(ts)
                print(json.dumps({"round": rnd, "case": name, "buf": buf, "median_us": round(med, 1),
                                  "min_us": round(min(ts), 1),
                                  "frac": round(n * nbytes[kind] / (med * 1e-6) / 8e12, 4)}), flush=True)


if __name__ == "__main__":
    main()
