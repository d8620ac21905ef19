"""CPU-baseline proxy check (CONTAINER-ONLY; never runs on the GPU box).

bench.py's ``cpu_baseline`` cannot time the reference on the GPU box (the reference does not
travel), so it times ``oracle/torch_port.py``: the same eager op sequence, restated.  This script
times the REAL reference (imported read-only from /root/reference, ``python3 -B``) and the port
on identical inputs and threads, per BASELINE config, and checks that the port's time is within
+-10 % of the reference's ("CPU baseline").  The result is written to
``tests/golden/time_ref_vs_port.json``.

Reference call sites timed (file:line under /root/reference):
  cfg2  TorchInnerProductCost.forward       cost_volume/inner_product.py:11-42
        + disparity_regression (softmax in)  model/mobile_disp_net_c.py:208-220
  cfg3  TorchGroupwiseCost.forward           cost_volume/groupwise.py:24-56
  cfg4  make_correlation_volume              model/mobile_disp_net_c.py:188-205
        + disparity_regression               model/mobile_disp_net_c.py:208-220
  cfg5  TorchConcatenateCost.forward         cost_volume/concatenate.py:11-41

Row bands of the full-size configs are timed (rows are independent; the per-disparity Python
loop is the same), so the whole check takes about a minute on 8 cores.

Usage:  cd /root/repo && python3 -B tests/golden/time_ref_vs_port.py
"""
import importlib.util
import json
import os
import statistics
import sys
import time

import torch

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
sys.dont_write_bytecode = True
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import torch_port as P  # noqa: E402


def _load(path, name):
    spec = importlib.util.spec_from_file_location(name, os.path.join(REF, path))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _median_time(fn, reps):
    fn()  # warm-up (allocator, thread pool)
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts)


def main():
    ip_mod = _load("cost_volume/inner_product.py", "ref_inner_product")
    gw_mod = _load("cost_volume/groupwise.py", "ref_groupwise")
    cc_mod = _load("cost_volume/concatenate.py", "ref_concatenate")
    dnc_mod = _load("model/mobile_disp_net_c.py", "ref_dispnetc")
    threads = os.cpu_count()
    torch.set_num_threads(threads)
    g = torch.Generator().manual_seed(0)

    def feats(c, h, w, dtype=torch.float32):
        return (torch.randn(1, c, h, w, generator=g).to(dtype),
                torch.randn(1, c, h, w, generator=g).to(dtype))

    cases = []
    L2, R2 = feats(64, 68, 960)
    ip = ip_mod.TorchInnerProductCost(192)
    cases.append(("cfg2", "1x64x68x960 f32 (68 of 540 rows), D=192, inner product + soft-argmin",
                  lambda: dnc_mod.disparity_regression(ip(L2, R2), 192),
                  lambda: P.cv_plus_regression(L2, R2, 192), 7))
    L3, R3 = feats(256, 8, 960, torch.bfloat16)
    gw = gw_mod.TorchGroupwiseCost(8, 192)
    cases.append(("cfg3", "1x256x8x960 bf16 (8 of 540 rows), G=8, D=192, groupwise",
                  lambda: gw(L3, R3), lambda: P.sweep_groupwise(L3, R3, 8, 192), 7))
    L4, R4 = feats(16, 68, 1920)
    cases.append(("cfg4", "1x16x68x1920 f32 (68 of 1080 rows), D=256, correlation + soft-argmin",
                  lambda: dnc_mod.disparity_regression(dnc_mod.make_correlation_volume(L4, R4, 256), 256),
                  lambda: P.correlation_plus_regression(L4, R4, 256), 7))
    L5, R5 = feats(128, 8, 960, torch.float16)
    cc = cc_mod.TorchConcatenateCost(64)
    cases.append(("cfg5", "1x128x8x960 f16 (8 of 540 rows), D=64, concatenate",
                  lambda: cc(L5, R5), lambda: P.sweep_concat(L5, R5, 64), 7))

    out = {"generator": "tests/golden/time_ref_vs_port.py", "torch": torch.__version__,
           "threads": threads, "bar": "port time within +-10% of the reference", "cases": []}
    ok = True
    for name, what, ref_fn, port_fn, reps in cases:
        same = torch.equal(ref_fn(), port_fn())
        # interleave the two to share any drift in machine load
        t_ref, t_port = [], []
        for _ in range(reps):
            t_ref.append(_median_time(ref_fn, 1))
            t_port.append(_median_time(port_fn, 1))
        tr, tp = statistics.median(t_ref), statistics.median(t_port)
        ratio = tp / tr
        good = same and abs(ratio - 1.0) <= 0.10
        ok &= good
        out["cases"].append({"config": name, "sample": what, "ref_s": tr, "port_s": tp,
                             "port_over_ref": ratio, "identical_outputs": same, "ok": good})
        print(f"{name}: ref {tr * 1e3:.1f} ms  port {tp * 1e3:.1f} ms  ratio {ratio:.3f}  "
              f"identical {same}  {'OK' if good else 'FAIL'}", flush=True)
    out["ok"] = ok
    with open(os.path.join(HERE, "time_ref_vs_port.json"), "w") as f:
        json.dump(out, f, indent=1)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
