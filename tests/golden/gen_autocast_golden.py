"""Golden vectors for the reference's fp16 (autocast) eval of the fused path (CONTAINER-ONLY).

VERDICT r05 "missing 2": the fused autocast disparity was only compared with the soft-argmin of
the engine's own fp16-rounded volume.  The reference's volume is different: under
``torch.cuda.amp.autocast`` (evaluate_stereo.py:25,48) ``left * right`` is not an autocast op, so
each product of the fp16 features is rounded to fp16 (cost_volume/inner_product.py:38-40;
``.mean`` in model/mobile_disp_net_c.py:196-202), ``torch.sum`` / ``.mean`` accumulate the fp16
products in fp32 and round the cell to fp16, and ``F.softmax`` (an autocast fp32 op) regresses
that fp16 volume in fp32 (mobile_disp_net_c.py:208-220).

This script imports the reference modules from /root/reference (``python3 -B``: no bytecode
written there) and runs their volume ops on fp16 CPU tensors (the same per-product fp16 rounding
and fp32 accumulation as on the GPU).  Autocast is a GPU mode, so the regression applies its one
effect explicitly: ``disparity_regression`` on the volume cast to fp32 (softmax is on autocast's
fp32 list; the fp16 disparity values 0..D-1 are exact).  It writes inputs and outputs only:

  autocast_inner_product_n1c32h4w128_d96_f16.npz   left, right (fp16), volume (fp16), disparity (fp32)
  autocast_correlation_n1c16h4w128_d48_f16.npz     the same for make_correlation_volume (mean)
  autocast_manifest.json

Usage:  cd /root/repo && python3 -B tests/golden/gen_autocast_golden.py
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
    ip_mod = _load("cost_volume/inner_product.py", "ref_inner_product")
    dnc_mod = _load("model/mobile_disp_net_c.py", "ref_dispnetc")
    cases = []
    for name, (n, c, h, w), D, seed, mean in (
            ("autocast_inner_product_n1c32h4w128_d96_f16", (1, 32, 4, 128), 96, 600, False),
            ("autocast_correlation_n1c16h4w128_d48_f16", (1, 16, 4, 128), 48, 601, True)):
        rng = np.random.default_rng(seed)
        L = torch.from_numpy(rng.standard_normal((n, c, h, w), dtype=np.float32)).half()
        R = torch.from_numpy(rng.standard_normal((n, c, h, w), dtype=np.float32)).half()
        vol = dnc_mod.make_correlation_volume(L, R, D) if mean else ip_mod.TorchInnerProductCost(D)(L, R)
        assert vol.dtype == torch.float16
        disp = dnc_mod.disparity_regression(vol.float(), D)  # autocast: fp32 softmax of the fp16 cells
        assert disp.dtype == torch.float32
        np.savez_compressed(os.path.join(OUT_DIR, name + ".npz"), left=L.numpy(), right=R.numpy(),
                            volume=vol.numpy(), disparity=disp.numpy())
        cases.append({"name": name, "file": name + ".npz", "max_disparity": D, "mean": mean,
                      "shape": [n, c, h, w]})
    with open(os.path.join(OUT_DIR, "autocast_manifest.json"), "w") as f:
        json.dump({"generator": "tests/golden/gen_autocast_golden.py", "torch": torch.__version__,
                   "cases": cases}, f, indent=1)
    print(f"wrote {len(cases)} autocast cases to {OUT_DIR}")


if __name__ == "__main__":
    main()
