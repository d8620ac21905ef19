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


# ---------------------------------------------------------------- eager restatements for the
# model-level isolation test (tests/test_model_isolation.py): the same networks run once with the
# engine's ops and once with these, on the same device and the same MIOpen trunk, so the
# difference is the engine's own contribution.  Device-agnostic torch code.
def sweep_diff_volume(left, right, num_disp):
    """make_cost_volume (model/mobile_stereo_net.py:8-27): L - R(x-d) at x >= d, 1.0 elsewhere,
    (N, C, D, H, W) in the left dtype."""
    n, c, h, w = left.shape
    vol = left.new_ones((n, c, num_disp, h, w))
    for shift in range(min(num_disp, w)):
        vol[:, :, shift, :, shift:] = left[..., shift:] - right[..., : w - shift]
    return vol


def soft_argmin_fp64(volume, keepdim=True):
    """The reference's softmax-then-weighted-sum over D (mobile_stereo_net.py:144-147) evaluated in
    fp64 and rounded once to fp32: the exact regression of the given volume."""
    v = volume.double()
    p = F.softmax(v, dim=1)
    d = torch.arange(v.shape[1], dtype=torch.float64, device=v.device).view(1, -1, 1, 1)
    return (p * d).sum(dim=1, keepdim=keepdim).float()


def regression_presoftmax_fp64(x, maxdisp):
    """mobile_stereo_net_v4.py:10-14 in fp64, rounded once to fp32."""
    d = torch.arange(maxdisp, dtype=torch.float64, device=x.device).view(1, maxdisp, 1, 1)
    return (x.double() * d).sum(dim=1).float()


def warp_grid_sample(image, flow):
    """tools/warp.py:5-42 restated: grid (x - fx, y - fy) normalised by (w - 1, h - 1), then
    F.grid_sample bilinear, zero padding, align_corners=False."""
    n, c, h, w = flow.shape
    gy, gx = torch.meshgrid(torch.arange(h, device=image.device, dtype=image.dtype),
                            torch.arange(w, device=image.device, dtype=image.dtype), indexing="ij")
    gx = (gx.view(1, 1, h, w) - flow[:, 0:1]).permute(0, 2, 3, 1)
    if c == 2:
        gy = (gy.view(1, 1, h, w) - flow[:, 1:2]).permute(0, 2, 3, 1)
    else:
        gy = gy.view(1, h, w, 1).expand(n, h, w, 1)
    grid = torch.cat((2.0 * gx / (w - 1.0) - 1.0, 2.0 * gy / (h - 1.0) - 1.0), dim=-1)
    return F.grid_sample(image, grid, mode="bilinear", padding_mode="zeros", align_corners=False)


def v4_volume_loop(featL, featR, conv3d, volume11, volume_size):
    """MobileStereoNetV4's per-disparity loop (model/mobile_stereo_net_v4.py:443-461): interleave
    L[..., i:] (even channels) and R[..., :-i] (odd), run the Conv3d stack and volume11 on the
    crop, place the result at x >= i of a zero (N, D, H, W) volume."""
    b, c, h, w = featL.shape
    vol = featL.new_zeros((b, volume_size, h, w))
    for i in range(min(volume_size, w)):
        lx, rx = featL[..., i:], featR[..., : w - i]
        x = torch.stack((lx, rx), dim=2).reshape(b, 2 * c, h, w - i)
        x = volume11(conv3d(x.unsqueeze(1)).squeeze(2))
        vol[:, i, :, i:] = x[:, 0]
    return vol
