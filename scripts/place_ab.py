"""Where the cfg2 volume lands in HBM: the band_rs launch of 32 cfg2 pairs timed into different
output buffers (HIP events on the launch stream, medians).

  python scripts/place_ab.py [--pairs 32] [--reps 6]

1. two torch buffers A, B written alternately (the bench's pattern: the new volume is allocated
   while the previous step's is still referenced), volume kernel only and with the soft-argmin;
2. one pool, the output at offsets of 0 .. 64 MiB from its (2 MiB-aligned) start.
Prints one JSON line per case with the buffer's virtual address."""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from realtime_stereo_matcher_amd import _lib, functional as F


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=32)
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--seq", type=int, default=0, help="instead: time K buffers allocated in a row")
    ap.add_argument("--algo", type=int, default=0, help="sm_ip_algo for sm_cv_inner_product_ex (0 auto)")
    ap.add_argument("--patterns", action="store_true", help="--order: also zero_ and soft_argmin")
    ap.add_argument("--order", default="", help="instead: allocation order, e.g. F,S1024,V,V (F: the "
                    "features, V: a volume buffer (torch), H: one from hipMalloc, C: one from "
                    "hipExtMallocWithFlags(contiguous), S<MiB>: a spacer); every V / H / C timed")
    a = ap.parse_args()
    n, c, h, w, D = a.pairs, 64, 540, 960, 192
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    held, vols = [], []
    L = R = None
    raw = []  # (ptr) from hipMalloc / hipExtMallocWithFlags, freed at the end
    vb0 = n * D * h * w * 4

    class _Raw:  # a volume-sized buffer outside torch's allocator
        def __init__(self, flags):
            import ctypes
            self.hip = ctypes.CDLL("libamdhip64.so")
            self.p = ctypes.c_void_p()
            if flags < 0:
                rc = self.hip.hipMalloc(ctypes.byref(self.p), ctypes.c_size_t(vb0))
            else:
                rc = self.hip.hipExtMallocWithFlags(ctypes.byref(self.p), ctypes.c_size_t(vb0), ctypes.c_uint(flags))
            if rc != 0:
                raise RuntimeError(f"hip allocation failed ({rc})")
            raw.append(self)

        def data_ptr(self):
            return self.p.value

    for tok in (a.order.split(",") if a.order else ["F"]):
        if tok == "F":
            L = torch.randn(n, c, h, w, device=dev, generator=g)
            R = torch.randn(n, c, h, w, device=dev, generator=g)
        elif tok == "V":
            vols.append(torch.empty(n, D, h, w, device=dev))
        elif tok == "H":  # plain hipMalloc
            vols.append(_Raw(-1))
        elif tok == "C":  # hipExtMallocWithFlags(hipDeviceMallocContiguous)
            vols.append(_Raw(4))
        else:
            held.append(torch.empty(int(tok[1:]) << 20, dtype=torch.uint8, device=dev))
    lib = _lib.load()
    st = torch.cuda.current_stream()
    vb = n * D * h * w * 4

    def launch(ptr):
        _lib.check(lib.sm_cv_inner_product_ex(L.data_ptr(), R.data_ptr(), ptr, _lib.SM_F32, n, c, h, w, D,
                                              _lib.strides_arg(L), _lib.strides_arg(R), a.algo,
                                              st.cuda_stream),
                   "sm_cv_inner_product_ex")

    def timed(ptr, after=None):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        launch(ptr)
        e1.record(st)
        if after is not None:
            after()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3

    def rep(case, ts, addr):
        ts = ts[1:] if len(ts) > 2 else ts
        print(json.dumps({"case": case, "addr": hex(addr), "addr_mod_1g": hex(addr % (1 << 30)),
                          "median_us": round(statistics.median(ts), 1), "min_us": round(min(ts), 1),
                          "frac": round(n * 663552000 / (statistics.median(ts) * 1e-6) / 8e12, 4),
                          "all": [round(t) for t in ts]}), flush=True)

    if a.order:
        for _ in range(3):
            timed(vols[0].data_ptr())
        def op_time(f):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            f()
            e1.record(st)
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) * 1e3

        for r in range(2):
            for i, b in enumerate(vols):
                rep(f"{a.order}: V{i} round {r}", [timed(b.data_ptr()) for _ in range(a.reps)], b.data_ptr())
                if not a.patterns or isinstance(b, _Raw):
                    continue
                # the same buffer under a sequential fill and under the regression's plane walk
                rep(f"{a.order}: V{i} zero_", [op_time(b.zero_) for _ in range(a.reps)], b.data_ptr())
                rep(f"{a.order}: V{i} soft_argmin", [op_time(lambda: F.soft_argmin(b)) for _ in range(a.reps)],
                    b.data_ptr())
        return
    if a.seq:
        bufs = [torch.empty(n, D, h, w, device=dev) for _ in range(a.seq)]
        for _ in range(3):
            timed(bufs[0].data_ptr())
        for r in range(2):
            for i, b in enumerate(bufs):
                rep(f"seq {i} round {r}", [timed(b.data_ptr()) for _ in range(a.reps)], b.data_ptr())
        return
    A = torch.empty(n, D, h, w, device=dev)
    B = torch.empty(n, D, h, w, device=dev)
    for _ in range(4):
        timed(A.data_ptr())
    # 1. alternating A / B, volume only, then with the soft-argmin after each launch
    ta, tb = [], []
    for _ in range(a.reps):
        ta.append(timed(A.data_ptr()))
        tb.append(timed(B.data_ptr()))
    rep("A alternating", ta, A.data_ptr())
    rep("B alternating", tb, B.data_ptr())
    ta, tb = [], []
    for _ in range(a.reps):
        ta.append(timed(A.data_ptr(), lambda: F.soft_argmin(A)))
        tb.append(timed(B.data_ptr(), lambda: F.soft_argmin(B)))
    rep("A with soft-argmin", ta, A.data_ptr())
    rep("B with soft-argmin", tb, B.data_ptr())
    ta = [timed(A.data_ptr()) for _ in range(a.reps)]
    rep("A back to back", ta, A.data_ptr())
    tb = [timed(B.data_ptr()) for _ in range(a.reps)]
    rep("B back to back", tb, B.data_ptr())
    del A, B
    torch.cuda.empty_cache()
    # 2. one pool, offsets
    pool = torch.empty(vb + (130 << 20), dtype=torch.uint8, device=dev)
    base = (pool.data_ptr() + (2 << 20) - 1) // (2 << 20) * (2 << 20)
    for off_mb in (0, 1, 2, 4, 8, 16, 32, 64, 0):
        p = base + (off_mb << 20)
        rep(f"pool +{off_mb} MiB", [timed(p) for _ in range(a.reps)], p)


if __name__ == "__main__":
    main()
