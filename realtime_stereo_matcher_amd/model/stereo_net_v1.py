"""Model-level drop-in demo: MobileStereoNet (v1) on PyTorch-ROCm with its cost
volume and disparity regression on the HIP engine.

Architecture and parameter names follow the reference network ``MobileStereoNet``
(model/mobile_stereo_net.py:89-158, config configure/stereo_net_config.json), so a reference
``state_dict`` loads unchanged.  The convolution trunk, the 3-D cost filter and the refinement
stages stay on torch (MIOpen); the two hot-path operators are this package's:

  * the difference cost volume ``make_cost_volume`` (reference :8-27) -> ``sm_cv_diff``;
  * the inline soft-argmin (reference :144-147)                      -> ``sm_regress_softargmin``.

Forward / inference only (the engine's ops have no backward).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

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
    """Disparity refinement at twice the input resolution (reference RefineNet, :57-86)."""

    DILATIONS = (1, 2, 4, 8, 1, 1)

    def __init__(self):
        super().__init__()
        layers = [_cbr(4, 32)] + [_Residual(32, d) for d in self.DILATIONS]
        layers.append(nn.Conv2d(32, 1, 3, 1, 1))
        self.conv0 = nn.Sequential(*layers)

    def forward(self, disp, rgb):
        up = 2 * F.interpolate(disp, scale_factor=2, mode="bilinear", align_corners=False)
        guide = F.interpolate(rgb, tuple(up.shape[2:]), mode="bilinear", align_corners=False)
        residual = self.conv0(torch.cat((up, guide), dim=1))
        return F.relu(up + residual)


class MobileStereoNetHIP(nn.Module):
    """MobileStereoNet (v1) with the HIP cost volume and soft-argmin."""

    def __init__(self, levels=3):
        super().__init__()
        self.k = levels
        self.align = 1 << levels
        self.max_disp = (192 + 1) >> levels
        trunk = []
        for i in range(levels):
            trunk += [_cbr(3 if i == 0 else 32, 32, stride=2), _Residual(32)]
        trunk.append(nn.Conv2d(32, 32, 3, 1, 1))
        self.feature_extractor = nn.Sequential(*trunk)
        filt = []
        for _ in range(4):
            filt += [nn.Conv3d(32, 32, 3, 1, 1), nn.BatchNorm3d(32), nn.ReLU()]
        filt.append(nn.Conv3d(32, 1, 3, 1, 1))
        self.cost_filter = nn.Sequential(*filt)
        self.refine_layer = nn.ModuleList(_Refine() for _ in range(levels))

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
            disp = refine(disp, left)
            scale = left.shape[3] / disp.shape[3]
            full = F.interpolate(disp * scale, tuple(left.shape[2:]))[:, :, :h, :w]
            outs.append(-full)
        return outs
