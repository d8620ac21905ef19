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
  * groupwise          cost_volume/groupwise.py:12-22 (helper), :24-56 (forward)
  * concatenate        cost_volume/concatenate.py:11-41
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


def correlation_plus_regression(left, right, num_disp):
    """cfg4's CPU path: the mean-over-C correlation volume, then soft-argmin."""
    return soft_argmin_eager(sweep_dot_volume(left, right, num_disp, mean=True))


def sweep_groupwise(left, right, n_groups, num_disp):
    """cfg3's CPU path: per disparity, the product in the input dtype, viewed as
    (N, G, C/G, H, W') and averaged over the group's channels, slice-assigned into an fp32
    (N, G, H, W, D) volume (D innermost) allocated on the CPU."""
    n, c, h, w = left.shape
    vol = torch.zeros((n, n_groups, h, w, num_disp))
    for shift in range(min(num_disp, w)):
        lhs = left if shift == 0 else left[..., shift:]
        rhs = right if shift == 0 else right[..., : w - shift]
        prod = (lhs * rhs).view(n, n_groups, c // n_groups, h, w - shift)
        vol[:, :, :, shift:, shift] = prod.mean(dim=2)
    return vol


def sweep_concat(left, right, num_disp):
    """cfg5's CPU path: (N, 2C, H, W, D) in the left dtype, left half L, right half the
    shifted R, both zero where x < d."""
    n, c, h, w = left.shape
    vol = left.new_zeros((n, 2 * c, h, w, num_disp))
    for shift in range(min(num_disp, w)):
        vol[:, :c, :, shift:, shift] = left[..., shift:]
        vol[:, c:, :, shift:, shift] = right[..., : w - shift]
    return vol


def sweep_interweave_shifted(left, right, num_disp):
    """cfg5's v4 variant (model/mobile_stereo_net_v4.py:443-461 before the Conv3d): per disparity
    the interleaved (L[..., d:], R[..., :-d]) channels written into a zero (N, 2C, D, H, W) volume."""
    n, c, h, w = left.shape
    vol = left.new_zeros((n, 2 * c, num_disp, h, w))
    for shift in range(min(num_disp, w)):
        vol[:, 0::2, shift, :, shift:] = left[..., shift:]
        vol[:, 1::2, shift, :, shift:] = right[..., : w - shift]
    return vol
