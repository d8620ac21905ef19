"""Model-level drop-in demo, part 2: MobileStereoNetV4 on PyTorch-ROCm with its
cost-volume stage and disparity regression on the HIP engine.

Architecture and parameter names follow the reference ``MobileStereoNetV4``
(model/mobile_stereo_net_v4.py:291-524, configure/stereo_net_config_v4.json: max_disp 192), so a
reference ``state_dict`` loads unchanged.  The 2-D trunk, the 2-D hourglasses and the classifier
stay on torch (MIOpen); the hot-path operators are this package's:

  * the 48-iteration interweave -> Conv3d(8,3,3)/s8 -> (4,3,3)/s4 -> (2,3,3)/s2 -> 1x1 loop
    (reference :443-461) -> ``mobile_stereo_net_v4.interweave_conv_volume`` (one fused HIP pass,
    ``sm_v4_volume``);
  * ``disparity_regression`` over the softmaxed volume (reference :10-14) -> ``sm_regress_softargmin``
    with ``SM_REGRESS_PRESOFTMAXED``.

Forward / inference only (the engine's ops have no backward).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from .mobile_stereo_net_v4 import disparity_regression, interweave_conv_volume


def _bn_conv(cin, cout, k, stride=1, pad=0, dilation=1, groups=1):
    """Conv2d (no bias) + BatchNorm2d, the reference's ``convbn`` (:208-220) when groups == 1."""
    return [nn.Conv2d(cin, cout, k, stride, dilation if dilation > 1 else pad, dilation=dilation,
                      groups=groups, bias=False), nn.BatchNorm2d(cout)]


class _InvertedResidual(nn.Module):
    """MobileV2_Residual (:91-148): 1x1 expand -> 3x3 depthwise -> 1x1 project, each with BN
    (ReLU6 after the first two), identity shortcut when the shape is kept."""

    def __init__(self, inp, oup, stride, expand, dilation=1):
        super().__init__()
        hid = int(inp * expand)
        self.use_res_connect = stride == 1 and inp == oup
        dw = [nn.Conv2d(hid, hid, 3, stride, dilation, dilation=dilation, groups=hid, bias=False),
              nn.BatchNorm2d(hid), nn.ReLU6(inplace=True)]
        pw = _bn_conv(hid, oup, 1)
        expand_layers = [] if expand == 1 else _bn_conv(inp, hid, 1) + [nn.ReLU6(inplace=True)]
        self.conv = nn.Sequential(*(expand_layers + dw + pw))

    def forward(self, x):
        y = self.conv(x)
        return x + y if self.use_res_connect else y


def _dws(inp, oup, stride, pad, dilation, relu_out=True):
    """convbn_dws (:26-65): 3x3 depthwise + BN + ReLU6, 1x1 pointwise + BN (+ ReLU6)."""
    layers = _bn_conv(inp, inp, 3, stride, pad, dilation, groups=inp) + [nn.ReLU6(inplace=True)]
    layers += _bn_conv(inp, oup, 1)
    if relu_out:
        layers.append(nn.ReLU6(inplace=False))
    return nn.Sequential(*layers)


class _DwsResidual(nn.Module):
    """MobileV1_Residual (:68-88): two depthwise-separable blocks plus a (projected) shortcut."""

    def __init__(self, inp, oup, stride, downsample, pad, dilation):
        super().__init__()
        self.stride = stride
        self.downsample = downsample
        self.conv1 = _dws(inp, oup, stride, pad, dilation)
        self.conv2 = _dws(oup, oup, 1, pad, dilation, relu_out=False)

    def forward(self, x):
        y = self.conv2(self.conv1(x))
        return y + (x if self.downsample is None else self.downsample(x))


class _Features(nn.Module):
    """feature_extraction(add_relus=True) (:151-205): 1/4-resolution, 64 + 128 + 128 channels."""

    def __init__(self):
        super().__init__()
        self.firstconv = nn.Sequential(_InvertedResidual(3, 32, 2, 3), nn.ReLU(inplace=True),
                                       _InvertedResidual(32, 32, 1, 3), nn.ReLU(inplace=True),
                                       _InvertedResidual(32, 32, 1, 3), nn.ReLU(inplace=True))
        self._inp = 32
        self.layer1 = self._stack(32, 3, 1, 1)
        self.layer2 = self._stack(64, 16, 2, 1)
        self.layer3 = self._stack(128, 3, 1, 1)
        self.layer4 = self._stack(128, 3, 1, 2)

    def _stack(self, planes, blocks, stride, dilation):
        down = None
        if stride != 1 or self._inp != planes:
            down = nn.Sequential(nn.Conv2d(self._inp, planes, 1, stride, bias=False), nn.BatchNorm2d(planes))
        mods = [_DwsResidual(self._inp, planes, stride, down, 1, dilation)]
        self._inp = planes
        mods += [_DwsResidual(planes, planes, 1, None, 1, dilation) for _ in range(1, blocks)]
        return nn.Sequential(*mods)

    def forward(self, x):
        x = self.layer1(self.firstconv(x))
        l2 = self.layer2(x)
        l3 = self.layer3(l2)
        return torch.cat((l2, l3, self.layer4(l3)), dim=1)


class _Hourglass(nn.Module):
    """hourglass2D (:223-288): two stride-2 inverted residuals down, two transposed convs up,
    inverted-residual skips."""

    def __init__(self, c):
        super().__init__()
        self.conv1 = _InvertedResidual(c, 2 * c, 2, 2)
        self.conv2 = _InvertedResidual(2 * c, 2 * c, 1, 2)
        self.conv3 = _InvertedResidual(2 * c, 4 * c, 2, 2)
        self.conv4 = _InvertedResidual(4 * c, 4 * c, 1, 2)
        up = lambda a, b: nn.Sequential(  # noqa: E731
            nn.ConvTranspose2d(a, b, 3, padding=1, output_padding=1, stride=2, bias=False), nn.BatchNorm2d(b))
        self.conv5 = up(4 * c, 2 * c)
        self.conv6 = up(2 * c, c)
        self.redir1 = _InvertedResidual(c, c, 1, 2)
        self.redir2 = _InvertedResidual(2 * c, 2 * c, 1, 2)

    def forward(self, x):
        c2 = self.conv2(self.conv1(x))
        c4 = self.conv4(self.conv3(c2))
        c5 = F.relu(self.conv5(c4) + self.redir2(c2), inplace=True)
        return F.relu(self.conv6(c5) + self.redir1(x), inplace=True)


def _classifier(c):
    return nn.Sequential(nn.Sequential(*_bn_conv(c, c, 3, 1, 1)), nn.ReLU(inplace=True),
                         nn.Conv2d(c, c, 3, padding=1, stride=1, bias=False, dilation=1))


class MobileStereoNetV4HIP(nn.Module):
    """MobileStereoNetV4 (:291-524) with the fused HIP interweave/Conv3d volume and the HIP
    pre-softmaxed regression.  ``volume_impl``: "hip" (default, the fused kernel) or "torch" (the
    same volume with MIOpen Conv3d over all disparities at once, for comparison)."""

    def __init__(self, max_disp=192, volume_impl="hip"):
        super().__init__()
        self.maxdisp = max_disp
        self.num_groups = 1
        self.volume_size = 48
        self.hg_size = 48
        self.dres_expanse_ratio = 3
        self.volume_impl = volume_impl
        self.feature_extraction = _Features()
        pre = []
        for a, b in ((320, 256), (256, 128), (128, 64)):
            pre += [nn.Sequential(*_bn_conv(a, b, 1)), nn.ReLU(inplace=True)]
        self.preconv11 = nn.Sequential(*pre, nn.Conv2d(64, 32, 1, 1, 0, 1))
        c3d = []
        for cin, cout, kd in ((1, 16, 8), (16, 32, 4), (32, 16, 2)):
            c3d += [nn.Conv3d(cin, cout, (kd, 3, 3), stride=[kd, 1, 1], padding=[0, 1, 1]),
                    nn.BatchNorm3d(cout), nn.ReLU()]
        self.conv3d = nn.Sequential(*c3d)
        self.volume11 = nn.Sequential(nn.Sequential(*_bn_conv(16, 1, 1)), nn.ReLU(inplace=True))
        hg, r = self.hg_size, self.dres_expanse_ratio
        self.dres0 = nn.Sequential(_InvertedResidual(self.volume_size, hg, 1, r), nn.ReLU(inplace=True),
                                   _InvertedResidual(hg, hg, 1, r), nn.ReLU(inplace=True))
        self.dres1 = nn.Sequential(_InvertedResidual(hg, hg, 1, r), nn.ReLU(inplace=True),
                                   _InvertedResidual(hg, hg, 1, r))
        self.encoder_decoder1 = _Hourglass(hg)
        self.encoder_decoder2 = _Hourglass(hg)
        self.encoder_decoder3 = _Hourglass(hg)
        self.classif0 = _classifier(hg)
        self.classif1 = _classifier(hg)
        self.classif2 = _classifier(hg)
        self.classif3 = _classifier(hg)

    def forward(self, L, R):
        L = (2.0 * (L / 255.0) - 1.0).contiguous()
        R = (2.0 * (R / 255.0) - 1.0).contiguous()
        featL = self.preconv11(self.feature_extraction(L))
        featR = self.preconv11(self.feature_extraction(R))
        volume = interweave_conv_volume(featL, featR, self.conv3d, self.volume11, self.volume_size,
                                        impl=self.volume_impl)  # (B, 48, H, W); HIP: sm_v4_volume
        cost0 = self.dres0(volume)
        cost0 = self.dres1(cost0) + cost0
        out3 = self.encoder_decoder3(self.encoder_decoder2(self.encoder_decoder1(cost0)))
        cost3 = self.classif3(out3).unsqueeze(1)
        cost3 = F.interpolate(cost3, [self.maxdisp, L.size()[2], L.size()[3]], mode="trilinear").squeeze(1)
        pred3 = disparity_regression(F.softmax(cost3, dim=1), self.maxdisp)  # HIP: presoftmaxed regression
        return [-1.0 * pred3.unsqueeze(1)]
