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


# ------------------------------------------------------------------------------------ v3
class _SamePadConv(nn.Conv2d):
    """Strided conv with TensorFlow-style 'same' padding, extra pixel bottom/right (reference
    same_padding_conv / SameConv2d, model/mobile_stereo_net_v3.py:145-167)."""

    def forward(self, x):
        (kh, kw), (sh, sw) = self.kernel_size, self.stride
        ph = max((-(-x.shape[2] // sh) - 1) * sh + kh - x.shape[2], 0)
        pw = max((-(-x.shape[3] // sw) - 1) * sw + kw - x.shape[3], 0)
        x = F.pad(x, (pw // 2, pw - pw // 2, ph // 2, ph - ph // 2))
        return F.conv2d(x, self.weight, self.bias, stride=self.stride)


def _lrelu():
    return nn.LeakyReLU(0.2)


class _Up(nn.Module):
    """2x transposed-conv upsample merged with the skip connection (reference UpsampleBlock,
    v3 :170-190)."""

    def __init__(self, cin, cout):
        super().__init__()
        self.up_conv = nn.Sequential(nn.ConvTranspose2d(cin, cout, 2, 2), _lrelu())
        self.merge_conv = nn.Sequential(nn.Conv2d(2 * cout, cout, 1), _lrelu(),
                                        nn.Conv2d(cout, cout, 3, 1, 1), _lrelu(),
                                        nn.Conv2d(cout, cout, 3, 1, 1), _lrelu())

    def forward(self, x, skip):
        return self.merge_conv(torch.cat((self.up_conv(x), skip), dim=1))


class _UNet(nn.Module):
    """Feature pyramid, coarsest first (reference UNetFeatureExtractor, v3 :193-246)."""

    def __init__(self, dims):
        super().__init__()
        levels = len(dims) - 1
        self.down_layers = nn.ModuleList()
        for i in range(levels + 1):
            if i == 0:
                mods = [nn.Conv2d(3, dims[0], 3, 1, 1), _lrelu()]
            else:
                mods = [_SamePadConv(dims[i - 1], dims[i], 4, 2), _lrelu()]
                for _ in range(3 if i == levels else 1):
                    mods += [nn.Conv2d(dims[i], dims[i], 3, 1, 1), _lrelu()]
            self.down_layers.append(nn.Sequential(*mods))
        self.up_layers = nn.ModuleList(_Up(dims[j], dims[j - 1]) for j in range(levels, 0, -1))

    def forward(self, x):
        skips = []
        for layer in self.down_layers:
            x = layer(x)
            skips.append(x)
        pyramid = [x]
        for i, up in enumerate(self.up_layers):
            x = up(x, skips[len(skips) - 2 - i])
            pyramid.append(x)
        return pyramid


class _RefineFeat(nn.Module):
    """v3 refinement: the upsampled disparity, the left feature map and the right feature map
    warped by that disparity (reference RefineNet, v3 :100-140)."""

    def __init__(self, in_dim, hidden, dilations):
        super().__init__()
        layers = [_cbr(in_dim, hidden)] + [_Residual(hidden, d) for d in dilations]
        layers.append(nn.Conv2d(hidden, 1, 3, 1, 1))
        self.conv0 = nn.Sequential(*layers)

    def forward(self, disp, l_fmap, r_fmap):
        up = 2 * F.interpolate(disp, scale_factor=2, mode="bilinear", align_corners=False)
        size = tuple(up.shape[2:])
        if tuple(l_fmap.shape[2:]) != size or tuple(r_fmap.shape[2:]) != size:
            l_fmap = F.interpolate(l_fmap, size, mode="bilinear", align_corners=False)
            r_fmap = F.interpolate(r_fmap, size, mode="bilinear", align_corners=False)
        r_fmap = warp_by_flow_map(r_fmap, up)                          # HIP: sm_warp_by_flow
        residual = self.conv0(torch.cat((up, l_fmap, r_fmap), dim=1))
        return F.relu(up + residual)


class MobileStereoNetV3HIP(nn.Module):
    """MobileStereoNetV3 (reference v3 :249-336, configure/stereo_net_config_v3.json) with the HIP
    difference volume, soft-argmin and feature-map warp."""

    def __init__(self, down_factor=3, max_disp=192, refine_dilates=(1, 2, 4, 8, 1, 1), hidden_dim=32):
        super().__init__()
        self.down_factor = down_factor
        self.align = 1 << down_factor
        self.max_disp = (max_disp + 1) >> down_factor
        self.feature_extractor = _UNet([hidden_dim] * (down_factor + 1))
        hd = hidden_dim
        filt = []
        for _ in range(4):
            filt += [nn.Conv3d(hd, hd, 3, 1, 1), nn.BatchNorm3d(hd), nn.ReLU()]
        filt.append(nn.Conv3d(hd, 1, 3, 1, 1))
        self.cost_filter = nn.Sequential(*filt)
        self.refine_layers = nn.ModuleList(
            _RefineFeat(1 + 2 * hd, hd, tuple(refine_dilates)) for _ in range(down_factor))

    def forward(self, l_img, r_img):
        norm = lambda im: (2.0 * (im / 255.0) - 1.0).contiguous()  # noqa: E731
        left, right = norm(l_img), norm(r_img)
        h, w = left.shape[2:]
        pad = (0, (-w) % self.align, 0, (-h) % self.align)
        left, right = F.pad(left, pad), F.pad(right, pad)
        lp = self.feature_extractor(left)
        rp = self.feature_extractor(right)
        volume = make_cost_volume(lp[0], rp[0], self.max_disp)          # HIP: sm_cv_diff
        disp = soft_argmin_regression(self.cost_filter(volume).squeeze(1))  # HIP: soft-argmin
        outs = []
        for i, refine in enumerate(self.refine_layers):
            disp = refine(disp, lp[i + 1], rp[i + 1])
            scale = left.shape[3] / disp.shape[3]
            outs.append(-F.interpolate(disp * scale, tuple(left.shape[2:]))[:, :, :h, :w])
        return outs


# ------------------------------------------------------------------------------ DispNetC
class _Layer(nn.Module):
    """Holds one Sequential under the attribute name ``layer`` (the reference blocks' layout)."""

    def __init__(self, *mods):
        super().__init__()
        self.layer = nn.Sequential(*mods)

    def forward(self, x):
        return self.layer(x)


def _conv_block(cin, cout, k, stride=1, bn=True):
    """k x k conv (no bias, 'same' padding for odd k) [-> BN] -> LeakyReLU(0.1)
    (reference Conv2dBlock, model/mobile_disp_net_c.py:9-55)."""
    mods = [nn.Conv2d(cin, cout, k, stride, (k - 1) // 2, bias=False)]
    if bn:
        mods.append(nn.BatchNorm2d(cout))
    mods.append(nn.LeakyReLU(0.1))
    return _Layer(*mods)


def _deconv_block(cin, cout, k, stride, bn=True):
    """Transposed conv doubling the size [-> BN] -> LeakyReLU(0.1) (reference
    Conv2dTransposeBlock, :58-109)."""
    mods = [nn.ConvTranspose2d(cin, cout, k, stride, (k - 1) // 2,
                               output_padding=stride - 1 - int(k % 2 == 0), bias=False)]
    if bn:
        mods.append(nn.BatchNorm2d(cout))
    mods.append(nn.LeakyReLU(0.1))
    return _Layer(*mods)


class _ResDown(nn.Module):
    """Strided residual block with a projected shortcut (reference ResBlock, :112-141)."""

    def __init__(self, cin, cout, stride=1):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, cout, 3, stride, 1)
        self.bn1 = nn.BatchNorm2d(cout)
        self.relu = nn.ReLU()
        self.conv2 = nn.Conv2d(cout, cout, 3, 1, 1)
        self.bn2 = nn.BatchNorm2d(cout)
        self.shortcut = (nn.Sequential(nn.Conv2d(cin, cout, 1, stride), nn.BatchNorm2d(cout))
                         if stride != 1 or cin != cout else None)

    def forward(self, x):
        skip = x if self.shortcut is None else self.shortcut(x)
        y = self.bn2(self.conv2(self.relu(self.bn1(self.conv1(x)))))
        return self.relu(y + skip)


class _UpPredict(nn.Module):
    """Coarse disparity prediction plus 2x feature upsampling merged with the skip features
    (reference UpsampleBlock, :144-185)."""

    def __init__(self, cin, cskip, cout, bn=True):
        super().__init__()
        self.deconv = _deconv_block(cin, cout, 4, 2, bn)
        self.predict = nn.Conv2d(cin, 1, 3, 1, 1, bias=False)
        self.up_predict = nn.ConvTranspose2d(1, 1, 4, 2, 1, bias=False)
        self.concat = nn.Conv2d(cskip + cout + 1, cout, 3, 1, 1, bias=False)

    def forward(self, x, skip):
        disp = self.predict(x)
        merged = torch.cat((skip, self.deconv(x), self.up_predict(disp)), dim=1)
        return disp, self.concat(merged)


class MobileDispNetCHIP(nn.Module):
    """MobileDispNetC (reference model/mobile_disp_net_c.py:237-412, configure/disp_net_c_config.json)
    with the correlation volume (mean over channels, D = max_disp // 4) on the HIP band kernel
    (sm_cv_correlation_mean)."""

    def __init__(self, hidden_dim=32, max_disp=192, with_batch_norm=True):
        super().__init__()
        self.down_factor = 6
        self.max_disp = max_disp
        c, bn = hidden_dim, with_batch_norm
        self.conv1 = _conv_block(3, c, 7, 2, bn)
        self.conv2 = _conv_block(c, 2 * c, 5, 2, bn)
        self.conv_redir = _conv_block(2 * c, c, 1, 1, bn)
        self.conv3 = nn.Sequential(_conv_block(c + max_disp // 4, 4 * c, 5, 2, bn),
                                   _conv_block(4 * c, 4 * c, 3, 1, False))
        self.res4 = _ResDown(4 * c, 8 * c, 2)
        self.res5 = _ResDown(8 * c, 16 * c, 2)
        self.res6 = _ResDown(16 * c, 32 * c, 2)
        self.up5 = _UpPredict(32 * c, 16 * c, 16 * c, bn)
        self.up4 = _UpPredict(16 * c, 8 * c, 8 * c, bn)
        self.up3 = _UpPredict(8 * c, 4 * c, 4 * c, bn)
        self.up2 = _UpPredict(4 * c, 2 * c, 2 * c, bn)
        self.up1 = _UpPredict(2 * c, c, c, bn)
        self.predict = nn.Conv2d(c, 1, 3, 1, 1, bias=False)

    @staticmethod
    def _resize(disp, shape):
        """reference disparity_interpolate (:223-234): bilinear resize with the x-scale applied."""
        if tuple(disp.shape[2:]) != tuple(shape):
            disp = F.interpolate(disp * (float(shape[1]) / disp.shape[3]), tuple(shape),
                                 mode="bilinear", align_corners=False)
        return disp

    def forward(self, l_img, r_img):
        from .mobile_disp_net_c import make_correlation_volume

        norm = lambda im: (2.0 * (im / 255.0) - 1.0).contiguous()  # noqa: E731
        left, right = norm(l_img), norm(r_img)
        h, w = left.shape[2:]
        align = 1 << self.down_factor
        pad = (0, (-w) % align, 0, (-h) % align)
        left, right = F.pad(left, pad), F.pad(right, pad)
        l1, r1 = self.conv1(left), self.conv1(right)
        l2, r2 = self.conv2(l1), self.conv2(r1)
        corr = make_correlation_volume(l2, r2, self.max_disp // 4)     # HIP: sm_cv_correlation_mean
        c3 = self.conv3(torch.cat((self.conv_redir(l2), corr), dim=1))
        r4 = self.res4(c3)
        r5 = self.res5(r4)
        r6 = self.res6(r5)
        d6, u = self.up5(r6, r5)
        d5, u = self.up4(u, r4)
        d4, u = self.up3(u, c3)
        d3, u = self.up2(u, l2)
        d2, u = self.up1(u, l1)
        d1 = self.predict(u)
        size = tuple(left.shape[2:])
        return [-self._resize(d, size)[:, :, :h, :w] for d in (d6, d5, d4, d3, d2, d1)]
