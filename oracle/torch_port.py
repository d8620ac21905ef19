"""CPU baseline port of the reference's eager op sequence (TEST / BENCH INFRASTRUCTURE ONLY).

Only ``bench.py``'s ``cpu_baseline`` leg and ``tests/`` may use this module.  It
restates the *algorithm* of the reference's CPU path -- per-disparity
``mul -> reduce -> strided slice-assign`` into a pre-filled volume, then softmax and
a weighted sum over D -- in torch eager on the host cores, so that the GPU box (where
the reference itself cannot travel) can time a faithful proxy of the reference CPU
path.  ``tests/test_oracle_golden.py`` pins it against the golden vectors, and
``tests/golden/time_ref_vs_port.py`` (container-only) checks that its CPU time is
within ±10 % of the real reference on identical inputs.

Followed semantics (babiking/realtime_stereo_matcher):
  * inner product      cost_volume/inner_product.py:11-42
  * correlation mean   model/mobile_disp_net_c.py:188-205
  * soft-argmin        model/mobile_disp_net_c.py:208-220, model/mobile_stereo_net.py:144-147
"""
import torch
import torch.nn.functional as F


def sweep_dot_volume(left: torch.Tensor, right: torch.Tensor, num_disp: int, mean: bool = False):
    """Per-disparity eager sweep (the reference algorithm's structure, one temporary per d)."""
    n, c, h, w = left.shape
    vol = left.new_zeros((n, num_disp, h, w))
    reduce = torch.mean if mean else torch.sum
    for shift in range(num_disp):
        if shift >= w:
            break
        lhs = left if shift == 0 else left[..., shift:]
        rhs = right if shift == 0 else right[..., : w - shift]
        vol[:, shift, :, shift:] = reduce(lhs * rhs, dim=1)
    return vol


def soft_argmin_eager(volume: torch.Tensor):
    """softmax over D, then sum of p * d with keepdim (the reference's regression)."""
    num_disp = volume.shape[1]
    prob = F.softmax(volume, dim=1)
    levels = torch.arange(num_disp, dtype=prob.dtype).view(1, num_disp, 1, 1)
    return (prob * levels).sum(dim=1, keepdim=True)


def cv_plus_regression(left, right, num_disp):
    """cfg2's CPU path end-to-end: inner-product volume then soft-argmin."""
    return soft_argmin_eager(sweep_dot_volume(left, right, num_disp))
