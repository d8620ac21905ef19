"""Golden vectors for float64 features (CONTAINER-ONLY; VERDICT r05 "missing 3").

The reference's operators take any floating dtype and torch computes an fp64 input in fp64.  This
script imports the reference modules from /root/reference (``python3 -B``: no bytecode written
there), runs them on seeded fp64 CPU tensors and records inputs and outputs only:

  f64_inner_product_n2c8h5w33_d12.npz   TorchInnerProductCost      cost_volume/inner_product.py:11-42
  f64_correlation_n1c16h4w40_d20.npz    make_correlation_volume    model/mobile_disp_net_c.py:188-205
  f64_groupwise_n1c16h3w21_g4_d9.npz    TorchGroupwiseCost (fp32)  cost_volume/groupwise.py:24-56
  f64_concat_n1c4h3w17_d6.npz           TorchConcatenateCost       cost_volume/concatenate.py:11-41
  f64_interweave_n1c4h3w17.npz          TorchInterweaveCost        cost_volume/interweave.py:10-22
  f64_diff_n1c4h3w17_d6.npz             make_cost_volume           model/mobile_stereo_net.py:8-27
  f64_softargmin_n2d24h5w7.npz          disparity_regression       model/mobile_disp_net_c.py:208-220
  f64_presoftmax_n1d24h4w9.npz          disparity_regression (v4)  model/mobile_stereo_net_v4.py:10-14
  f64_argmax_n2d12h5w33.npz             torch.argmax over the inner-product volume (build-defined)
  f64_manifest.json

Usage:  cd /root/repo && python3 -B tests/golden/gen_f64_golden.py
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


def main():
    ip = _load("cost_volume/inner_product.py", "ref_inner_product")
    gw = _load("cost_volume/groupwise.py", "ref_groupwise")
    cc = _load("cost_volume/concatenate.py", "ref_concatenate")
    iw = _load("cost_volume/interweave.py", "ref_interweave")
    msn = _load("model/mobile_stereo_net.py", "ref_msn")
    v4 = _load("model/mobile_stereo_net_v4.py", "ref_msn_v4")
    dnc = _load("model/mobile_disp_net_c.py", "ref_dispnetc")
    cases = []

    def feats(seed, shape):
        rng = np.random.default_rng(seed)
        return (torch.from_numpy(rng.standard_normal(shape)), torch.from_numpy(rng.standard_normal(shape)))

    def save(name, op, params, arrays):
        np.savez_compressed(os.path.join(OUT_DIR, name + ".npz"), **{k: v.numpy() for k, v in arrays.items()})
        cases.append({"name": name, "file": name + ".npz", "op": op, "params": params,
                      "dtypes": {k: str(v.dtype).replace("torch.", "") for k, v in arrays.items()}})

    L, R = feats(700, (2, 8, 5, 33))
    vol = ip.TorchInnerProductCost(12)(L, R)
    save("f64_inner_product_n2c8h5w33_d12", "inner_product", {"max_disparity": 12},
         {"left": L, "right": R, "out": vol})
    save("f64_argmax_n2d12h5w33", "argmax", {}, {"volume": vol, "out": torch.argmax(vol, dim=1)})
    L, R = feats(701, (1, 16, 4, 40))
    save("f64_correlation_n1c16h4w40_d20", "correlation", {"max_disp": 20},
         {"left": L, "right": R, "out": dnc.make_correlation_volume(L, R, 20)})
    L, R = feats(702, (1, 16, 3, 21))
    save("f64_groupwise_n1c16h3w21_g4_d9", "groupwise", {"n_groups": 4, "max_disparity": 9},
         {"left": L, "right": R, "out": gw.TorchGroupwiseCost(4, 9)(L, R)})
    L, R = feats(703, (1, 4, 3, 17))
    save("f64_concat_n1c4h3w17_d6", "concat", {"max_disparity": 6},
         {"left": L, "right": R, "out": cc.TorchConcatenateCost(6)(L, R)})
    save("f64_interweave_n1c4h3w17", "interweave", {}, {"left": L, "right": R, "out": iw.TorchInterweaveCost()(L, R)})
    save("f64_diff_n1c4h3w17_d6", "diff_volume", {"max_disp": 6},
         {"left": L, "right": R, "out": msn.make_cost_volume(L, R, 6)})
    cv = torch.from_numpy(np.random.default_rng(704).standard_normal((2, 24, 5, 7)) * 3.0)
    save("f64_softargmin_n2d24h5w7", "softargmin", {"max_disp": 24},
         {"volume": cv, "out": dnc.disparity_regression(cv, 24)})
    p = torch.softmax(torch.from_numpy(np.random.default_rng(705).standard_normal((1, 24, 4, 9)) * 3.0), dim=1)
    save("f64_presoftmax_n1d24h4w9", "regression_presoftmax", {"maxdisp": 24},
         {"volume": p, "out": v4.disparity_regression(p, 24)})
    with open(os.path.join(OUT_DIR, "f64_manifest.json"), "w") as f:
        json.dump({"generator": "tests/golden/gen_f64_golden.py", "torch": torch.__version__, "cases": cases},
                  f, indent=1)
    print(f"wrote {len(cases)} fp64 cases to {OUT_DIR}")


if __name__ == "__main__":
    main()
