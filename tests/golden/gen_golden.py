"""Golden-vector generator for the stereo cost-volume hot path (CONTAINER-ONLY).

This script imports the *reference* implementation from ``/root/reference`` at
run time (read-only, ``python3 -B`` so no bytecode is written there) and records
its outputs on small seeded inputs.  Nothing produced here contains reference
source: every fixture is data (inputs and the reference's outputs).  The GPU box
never runs this script; it only reads the committed ``*.npz`` + ``manifest.json``.

Reference call sites exercised (file:line under /root/reference):
  * TorchInnerProductCost     cost_volume/inner_product.py:5-45
  * TorchGroupwiseCost        cost_volume/groupwise.py:5-56
  * TorchConcatenateCost      cost_volume/concatenate.py:5-41
  * TorchInterweaveCost       cost_volume/interweave.py:5-25
  * make_cost_volume          model/mobile_stereo_net.py:8-27
  * make_correlation_volume   model/mobile_disp_net_c.py:188-205
  * disparity_regression      model/mobile_disp_net_c.py:208-220 (softmax inside, keepdim)
  * disparity_regression      model/mobile_stereo_net_v4.py:10-14 (pre-softmaxed, no keepdim)
  * interweave_tensors        model/mobile_stereo_net_v4.py:17-23 (+ shifted use :443-461)
  * inline soft-argmin        model/mobile_stereo_net.py:144-147
  * hard argmin/argmax        build-defined (torch.argmax/argmin over the reference volume)
  * warp_by_flow_map          tools/warp.py:5-42

Usage:  cd /root/repo && python3 -B tests/golden/gen_golden.py
"""
import importlib.util
import json
import os
import sys

import numpy as np
import torch

REF = "/root/reference"
OUT_DIR = os.path.dirname(os.path.abspath(__file__))
sys.dont_write_bytecode = True


def _load(path, name):
    spec = importlib.util.spec_from_file_location(name, os.path.join(REF, path))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


ip_mod = _load("cost_volume/inner_product.py", "ref_inner_product")
gw_mod = _load("cost_volume/groupwise.py", "ref_groupwise")
cc_mod = _load("cost_volume/concatenate.py", "ref_concatenate")
iw_mod = _load("cost_volume/interweave.py", "ref_interweave")
msn_mod = _load("model/mobile_stereo_net.py", "ref_msn")
v4_mod = _load("model/mobile_stereo_net_v4.py", "ref_msn_v4")
dnc_mod = _load("model/mobile_disp_net_c.py", "ref_dispnetc")
warp_mod = _load("tools/warp.py", "ref_warp")

DT = {"f32": torch.float32, "f16": torch.float16, "bf16": torch.bfloat16}

manifest = {"generator": "tests/golden/gen_golden.py", "torch": torch.__version__, "cases": []}


def to_np(t):
    """Store bf16 as its raw uint16 bits (numpy has no bfloat16)."""
    t = t.detach().cpu().contiguous()
    if t.dtype == torch.bfloat16:
        return t.view(torch.int16).numpy().view(np.uint16)
    return t.numpy()


def feats(seed, shape, dtype, kind="normal"):
    rng = np.random.default_rng(seed)
    if kind == "normal":
        a = rng.standard_normal(shape, dtype=np.float32)
        b = rng.standard_normal(shape, dtype=np.float32)
    elif kind == "int":
        a = rng.integers(-8, 9, size=shape).astype(np.float32)
        b = rng.integers(-8, 9, size=shape).astype(np.float32)
    elif kind == "tie":  # very few distinct values -> many argmin/argmax ties
        a = rng.integers(-1, 2, size=shape).astype(np.float32)
        b = rng.integers(-1, 2, size=shape).astype(np.float32)
    else:
        raise ValueError(kind)
    return torch.from_numpy(a).to(DT[dtype]), torch.from_numpy(b).to(DT[dtype])


def save(name, op, params, arrays, dtype, **extra):
    fn = f"{name}.npz"
    np.savez_compressed(os.path.join(OUT_DIR, fn), **{k: to_np(v) for k, v in arrays.items()})
    rec = {"name": name, "file": fn, "op": op, "params": params, "dtype": dtype}
    rec.update(extra)
    manifest["cases"].append(rec)


def main():
    torch.manual_seed(0)
    # ---------------- a-1 inner product --------------------------------------
    for D in (1, 9, 33, 40):
        L, R = feats(1, (2, 8, 5, 33), "f32")
        out = ip_mod.TorchInnerProductCost(D)(L, R)
        save(f"inner_product_n2c8h5w33_d{D}_f32", "inner_product", {"max_disparity": D},
             {"left": L, "right": R, "out": out}, "f32")
    L, R = feats(0, (1, 32, 64, 128), "f32")  # BASELINE configs[0] (cfg1)
    out = ip_mod.TorchInnerProductCost(24)(L, R)
    save("inner_product_cfg1_n1c32h64w128_d24_f32", "inner_product", {"max_disparity": 24},
         {"left": L, "right": R, "out": out}, "f32")
    L, R = feats(2, (2, 8, 5, 33), "f32", "int")
    out = ip_mod.TorchInnerProductCost(9)(L, R)
    save("inner_product_int_n2c8h5w33_d9_f32", "inner_product", {"max_disparity": 9},
         {"left": L, "right": R, "out": out}, "f32", exact=True)
    for dt in ("f16", "bf16"):
        L, R = feats(3, (1, 8, 4, 20), dt)
        out = ip_mod.TorchInnerProductCost(7)(L, R)
        save(f"inner_product_n1c8h4w20_d7_{dt}", "inner_product", {"max_disparity": 7},
             {"left": L, "right": R, "out": out}, dt, literal=True)
    # non-contiguous input (stride view) gives identical values in the reference
    L, R = feats(4, (2, 8, 5, 33), "f32")
    Lt = L.transpose(2, 3).contiguous().transpose(2, 3)
    out = ip_mod.TorchInnerProductCost(6)(Lt, R)
    save("inner_product_noncontig_n2c8h5w33_d6_f32", "inner_product", {"max_disparity": 6},
         {"left": L, "right": R, "out": out}, "f32")

    # ---------------- a-2 groupwise -------------------------------------------
    for G in (1, 2, 8):
        L, R = feats(10 + G, (2, 16, 4, 21), "f32")
        out = gw_mod.TorchGroupwiseCost(G, 7)(L, R)
        save(f"groupwise_n2c16h4w21_g{G}_d7_f32", "groupwise", {"n_groups": G, "max_disparity": 7},
             {"left": L, "right": R, "out": out}, "f32")
    L, R = feats(20, (1, 16, 4, 21), "bf16")
    out = gw_mod.TorchGroupwiseCost(8, 7)(L, R)
    save("groupwise_n1c16h4w21_g8_d7_bf16", "groupwise", {"n_groups": 8, "max_disparity": 7},
         {"left": L, "right": R, "out": out}, "bf16", literal=True)
    L, R = feats(21, (1, 64, 3, 40), "bf16")
    out = gw_mod.TorchGroupwiseCost(2, 24)(L, R)
    save("groupwise_n1c64h3w40_g2_d24_bf16", "groupwise", {"n_groups": 2, "max_disparity": 24},
         {"left": L, "right": R, "out": out}, "bf16", literal=True)
    L, R = feats(22, (1, 16, 3, 12), "f32")
    out = gw_mod.TorchGroupwiseCost(4, 20)(L, R)  # D > W
    save("groupwise_n1c16h3w12_g4_d20_f32", "groupwise", {"n_groups": 4, "max_disparity": 20},
         {"left": L, "right": R, "out": out}, "f32")
    try:
        gw_mod.TorchGroupwiseCost(3, 4)(*feats(23, (1, 16, 2, 8), "f32"))
        raise SystemExit("expected AssertionError")
    except AssertionError as e:
        manifest["groupwise_assert_message_c16_g3"] = str(e)

    # ---------------- a-3 concatenate -----------------------------------------
    for dt, shape, D in (("f32", (2, 4, 3, 17), 5), ("f16", (1, 4, 3, 17), 20), ("bf16", (1, 6, 2, 19), 8)):
        L, R = feats(30, shape, dt)
        out = cc_mod.TorchConcatenateCost(D)(L, R)
        save(f"concat_{'x'.join(map(str, shape))}_d{D}_{dt}", "concat", {"max_disparity": D},
             {"left": L, "right": R, "out": out}, dt, exact=True)

    # ---------------- a-4 interweave ------------------------------------------
    for dt, shape in (("f32", (2, 4, 3, 17)), ("f16", (1, 8, 3, 17)), ("bf16", (1, 5, 2, 9))):
        L, R = feats(40, shape, dt)
        out = iw_mod.TorchInterweaveCost()(L, R)
        out2 = v4_mod.interweave_tensors(L, R)
        assert torch.equal(out, out2)
        save(f"interweave_{'x'.join(map(str, shape))}_{dt}", "interweave", {},
             {"left": L, "right": R, "out": out}, dt, exact=True)
    # v4's shifted use (mobile_stereo_net_v4.py:443-461): volume[:, :, i, :, i:] gets the
    # interwoven slice for disparity i; zero elsewhere (new_zeros, :443).
    for dt, shape, D in (("f32", (1, 4, 3, 17), 6), ("f16", (2, 3, 2, 11), 13)):
        L, R = feats(41, shape, dt)
        n, c, h, w = shape
        vol = L.new_zeros([n, 2 * c, D, h, w])
        for i in range(D):
            if i == 0:
                vol[:, :, 0] = v4_mod.interweave_tensors(L, R)
            elif i < w:
                vol[:, :, i, :, i:] = v4_mod.interweave_tensors(L[:, :, :, i:], R[:, :, :, :-i])
        save(f"interweave_shifted_{'x'.join(map(str, shape))}_d{D}_{dt}", "interweave_shifted",
             {"max_disparity": D}, {"left": L, "right": R, "out": vol}, dt, exact=True)

    # ---------------- a-5 difference volume (fill 1.0) ------------------------
    for D, shape in ((9, (2, 8, 5, 33)), (40, (1, 4, 3, 33)), (24, (1, 32, 6, 10))):
        L, R = feats(50 + D, shape, "f32")
        out = msn_mod.make_cost_volume(L, R, D)
        save(f"diff_volume_{'x'.join(map(str, shape))}_d{D}_f32", "diff_volume", {"max_disp": D},
             {"left": L, "right": R, "out": out}, "f32", exact=True)
    L, R = feats(59, (1, 4, 3, 17), "f16")
    out = msn_mod.make_cost_volume(L, R, 6)
    save("diff_volume_1x4x3x17_d6_f16", "diff_volume", {"max_disp": 6},
         {"left": L, "right": R, "out": out}, "f16", exact=True)

    # ---------------- a-6 correlation (mean) ----------------------------------
    for D, shape in ((12, (2, 16, 5, 33)), (40, (1, 16, 3, 33)), (48, (1, 16, 4, 80))):
        L, R = feats(60 + D, shape, "f32")
        out = dnc_mod.make_correlation_volume(L, R, D)
        save(f"correlation_{'x'.join(map(str, shape))}_d{D}_f32", "correlation", {"max_disp": D},
             {"left": L, "right": R, "out": out}, "f32")

    # ---------------- a-7 soft-argmin regression ------------------------------
    for shape in ((2, 24, 5, 7), (1, 192, 4, 9), (1, 48, 3, 33)):
        rng = np.random.default_rng(70 + shape[1])
        cv = torch.from_numpy(rng.standard_normal(shape, dtype=np.float32) * 3.0)
        D = shape[1]
        out = dnc_mod.disparity_regression(cv, D)  # softmax inside, keepdim
        save(f"softargmin_{'x'.join(map(str, shape))}_f32", "softargmin", {"max_disp": D},
             {"volume": cv, "out": out}, "f32")
        # inline form of mobile_stereo_net.py:144-147 on the same volume (softmax -> sum p*d, keepdim)
        x = torch.nn.functional.softmax(cv, dim=1)
        d = torch.arange(0, D, dtype=x.dtype)
        inline = torch.sum(x * d.view(1, -1, 1, 1), dim=1, keepdim=True)
        assert torch.equal(inline, out)
        # v4 form: pre-softmaxed input, no keepdim (mobile_stereo_net_v4.py:10-14)
        p = torch.nn.functional.softmax(cv, dim=1)
        out4 = v4_mod.disparity_regression(p, D)
        save(f"regression_presoftmax_{'x'.join(map(str, shape))}_f32", "regression_presoftmax",
             {"maxdisp": D}, {"volume": p, "out": out4}, "f32")
    try:
        dnc_mod.disparity_regression(torch.zeros(1, 5, 2, 2), 4)
        raise SystemExit("expected AssertionError")
    except AssertionError as e:
        manifest["softargmin_assert_message_d5_vs_4"] = str(e)
    try:
        dnc_mod.disparity_regression(torch.zeros(5, 2, 2), 5)
        raise SystemExit("expected AssertionError")
    except AssertionError as e:
        manifest["softargmin_assert_message_ndim3"] = str(e)

    # ---------------- a-8 hard argmin / argmax (build-defined) ----------------
    for kind in ("int", "tie"):
        L, R = feats(80, (2, 8, 5, 33), "f32", kind)
        vol = ip_mod.TorchInnerProductCost(12)(L, R)
        save(f"argmax_{kind}_n2c8h5w33_d12_f32", "argext", {"max_disparity": 12, "mode": "max"},
             {"left": L, "right": R, "volume": vol, "out": torch.argmax(vol, dim=1)}, "f32", exact=True)
        dv = msn_mod.make_cost_volume(L, R, 12).abs().sum(dim=1)  # SAD-style cost (N,D,H,W)
        save(f"argmin_{kind}_n2c8h5w33_d12_f32", "argext", {"max_disparity": 12, "mode": "min"},
             {"volume": dv, "out": torch.argmin(dv, dim=1)}, "f32", exact=True)

    # ---------------- §8f-4 warp_by_flow_map (tools/warp.py:5-42) -------------
    rng = np.random.default_rng(90)
    warp_cases = [  # name, image shape, flow shape, flow generator
        ("disp_n1c3h12w40", (1, 3, 12, 40), (1, 1, 12, 40), lambda sh: rng.uniform(0, 20, sh)),
        ("flow2_n2c5h9w17", (2, 5, 9, 17), (2, 2, 9, 17), lambda sh: rng.standard_normal(sh) * 3),
        ("resize_n1c4h6w20_to_h12w40", (1, 4, 6, 20), (1, 1, 12, 40), lambda sh: rng.uniform(-5, 45, sh)),
        ("disp_n1c32h30w40", (1, 32, 30, 40), (1, 1, 30, 40), lambda sh: rng.uniform(0, 24, sh)),
        ("intdisp_n1c6h8w33", (1, 6, 8, 33), (1, 1, 8, 33), lambda sh: rng.integers(0, 12, sh)),
        # degenerate grids: h = 1 / w = 1 divide by zero in the reference's normalisation -> NaN
        ("degenerate_h1_n1c2h4w16", (1, 2, 4, 16), (1, 1, 1, 16), lambda sh: rng.uniform(0, 3, sh)),
        ("degenerate_w1_n1c2h4w16", (1, 2, 4, 16), (1, 1, 4, 1), lambda sh: rng.uniform(0, 3, sh)),
        ("nanflow_n1c3h6w20", (1, 3, 6, 20), (1, 2, 6, 20),
         lambda sh: np.where(rng.uniform(size=sh) < 0.05, np.nan, rng.uniform(-4, 4, sh))),
    ]
    for name, ish, fsh, gen in warp_cases:
        img = torch.from_numpy(rng.standard_normal(ish).astype(np.float32))
        flow = torch.from_numpy(np.asarray(gen(fsh), dtype=np.float32))
        out = warp_mod.warp_by_flow_map(img, flow)
        save(f"warp_{name}_f32", "warp", {}, {"image": img, "flow": flow, "out": out}, "f32")
    try:
        warp_mod.warp_by_flow_map(torch.zeros(1, 2, 3, 4), torch.zeros(1, 3, 3, 4))
    except AssertionError as e:
        manifest["warp_assert_message_c3"] = str(e)

    # shape-mismatch behaviour of the reference (RuntimeError from torch)
    try:
        ip_mod.TorchInnerProductCost(3)(torch.zeros(1, 4, 2, 8), torch.zeros(1, 5, 2, 8))
        manifest["shape_mismatch_raises"] = None
    except RuntimeError as e:
        manifest["shape_mismatch_raises"] = "RuntimeError"

    with open(os.path.join(OUT_DIR, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print(f"wrote {len(manifest['cases'])} cases to {OUT_DIR}")


if __name__ == "__main__":
    main()
