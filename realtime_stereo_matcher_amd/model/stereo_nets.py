"""Model-level drop-in demo: MobileStereoNet v1 and v2 on PyTorch-ROCm with their
cost volume, disparity regression and (v2) refinement warp on the HIP engine.

Architecture and parameter names follow the reference networks ``MobileStereoNet``
(model/mobile_stereo_net.py:89-158, configure/stereo_net_config.json) and ``MobileStereoNetV2``
(model/mobile_stereo_net_v2.py:136-232, configure/stereo_net_config_v2.json), so a reference
``state_dict`` loads unchanged.  The convolution trunk, the 3-D cost filter and the refinement
convolutions stay on torch (MIOpen); the hot-path operators are this package's:

  * the difference cost volume ``make_cost_volume`` (reference :8-27)   -> ``sm_cv_diff``;
  * the inline soft-argmin (reference :144-147, v2 :217-220)           -> ``sm_regress_softargmin``;
  * v2's RefineNet warp ``warp_by_flow_map`` (v2 :59-96, used at :127)  -> ``sm_warp_by_flow``.

Forward / inference only (the engine's ops have no backward).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..functional import warp_by_flow_map
from .mobile_stereo_net import make_cost_volume, soft_argmin_regression


def _cbr(cin, cout, stride=1, dilation=1):
    """3x3 conv (no bias) -> BatchNorm -> ReLU; indices 0/1/2 as in the reference's conv_3x3."""
    return nn.Sequential(nn.Conv2d(cin, cout, 3, stride, dilation, dilation=dilation, bias=False),
                         nn.BatchNorm2d(cout), nn.ReLU())


class _Residual(nn.Module):
    """Two dilated 3x3 conv-bn-relu layers plus the identity (reference ResBlock, :44-54)."""

    def __init__(self, ch, dilation=1):
        super().__init__()
        self.conv = nn.Sequential(_cbr(ch, ch, dilation=dilation), _cbr(ch, ch, dilation=dilation))

    def forward(self, x):
        return x + self.conv(x)


class _Refine(nn.Module):
    """Disparity refinement at twice the input resolution (reference RefineNet, v1 :57-86; v2
    :97-134).  v1 guides with the left image (4 input channels); v2 also warps the right image
    by the upsampled disparity and guides with both (7 input channels)."""

    def __init__(self, in_dim=4, hidden=32, dilations=(1, 2, 4, 8, 1, 1), warp=False):
        super().__init__()
        self.warp = warp
        layers = [_cbr(in_dim, hidden)] + [_Residual(hidden, d) for d in dilations]
        layers.append(nn.Conv2d(hidden, 1, 3, 1, 1))
        self.conv0 = nn.Sequential(*layers)

    def forward(self, disp, l_rgb, r_rgb=None):
        up = 2 * F.interpolate(disp, scale_factor=2, mode="bilinear", align_corners=False)
        size = tuple(up.shape[2:])
        guide = [F.interpolate(l_rgb, size, mode="bilinear", align_corners=False)]
        if self.warp:
            r = F.interpolate(r_rgb, size, mode="bilinear", align_corners=False)
            guide.append(warp_by_flow_map(r, up))                       # HIP: sm_warp_by_flow
        residual = self.conv0(torch.cat([up] + guide, dim=1))
        return F.relu(up + residual)


class MobileStereoNetHIP(nn.Module):
    """MobileStereoNet v1 (``v2=False``) or v2 (``v2=True``, with the v2 constructor arguments)
    with the HIP cost volume, soft-argmin and warp."""

    def __init__(self, levels=3, max_disp=192, hidden_dim=32, v2=False, refine_dim=7,
                 refine_dilates=(1, 2, 4, 8, 1, 1)):
        super().__init__()
        self.k = levels
        self.v2 = v2
        self.align = 1 << levels
        self.max_disp = (max_disp + 1) >> levels
        hd = hidden_dim
        trunk = []
        for i in range(levels):
            trunk += [_cbr(3 if i == 0 else hd, hd, stride=2), _Residual(hd)]
        trunk.append(nn.Conv2d(hd, hd, 3, 1, 1))
        self.feature_extractor = nn.Sequential(*trunk)
        filt = []
        for _ in range(4):
            filt += [nn.Conv3d(hd, hd, 3, 1, 1), nn.BatchNorm3d(hd), nn.ReLU()]
        filt.append(nn.Conv3d(hd, 1, 3, 1, 1))
        self.cost_filter = nn.Sequential(*filt)
        self.refine_layer = nn.ModuleList(
            _Refine(refine_dim if v2 else 4, hd if v2 else 32, tuple(refine_dilates), warp=v2)
            for _ in range(levels))

    def forward(self, left_img, right_img):
        norm = lambda im: (2.0 * (im / 255.0) - 1.0).contiguous()  # noqa: E731
        left, right = norm(left_img), norm(right_img)
        h, w = left.shape[2:]
        pad = (0, (-w) % self.align, 0, (-h) % self.align)
        left, right = F.pad(left, pad), F.pad(right, pad)
        fl = self.feature_extractor(left)
        fr = self.feature_extractor(right)
        volume = make_cost_volume(fl, fr, self.max_disp)               # HIP: sm_cv_diff
        cost = self.cost_filter(volume).squeeze(1)
        disp = soft_argmin_regression(cost)                             # HIP: sm_regress_softargmin
        outs = []
        for refine in self.refine_layer:
            disp = refine(disp, left, right) if self.v2 else refine(disp, left)
            scale = left.shape[3] / disp.shape[3]
            full = F.interpolate(disp * scale, tuple(left.shape[2:]))[:, :, :h, :w]
            outs.append(-full)
        return outs
