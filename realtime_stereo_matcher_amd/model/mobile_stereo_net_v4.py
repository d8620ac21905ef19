"""Hot-path helpers of ``model/mobile_stereo_net_v4.py``."""
import torch

from .. import functional as F


def disparity_regression(x, maxdisp):
    """sum_d d * x[:, d] over an already-softmaxed (N,D,H,W) volume -> (N,H,W)
    (model/mobile_stereo_net_v4.py:10-14)."""
    assert len(x.shape) == 4
    if x.shape[1] != maxdisp:
        raise RuntimeError(f"disparity_regression: volume has {x.shape[1]} planes, maxdisp={maxdisp}")
    return F.regression_presoftmax(x)


def interweave_tensors(refimg_fea, targetimg_fea):
    """(N,C,H,W) x2 -> (N,2C,H,W), even = ref, odd = target (model/mobile_stereo_net_v4.py:17-23)."""
    return F.interweave(refimg_fea, targetimg_fea)


def interweave_volume(featL, featR, volume_size):
    """The per-disparity loop input of MobileStereoNetV4 (:443-461) materialised at once:
    (N,C,H,W) x2 -> (N,2C,D,H,W), slice d = interweave(L[..., d:], R[..., :-d]) placed at
    x >= d, zeros elsewhere."""
    return F.interweave_volume(featL, featR, volume_size)


def fold_v4_weights(conv3d, volume11):
    """Eval-mode folding of the V4 cost-volume stack (:317-335) into plain weights + biases:
    Conv3d(1,16,(8,3,3))+BN3d, Conv3d(16,32,(4,3,3))+BN3d, Conv3d(32,16,(2,3,3))+BN3d, then the
    1x1 Conv2d(16,1) (no bias) + BN2d.  Returns fp32 tensors (w1 (16,8,3,3), b1 (16),
    w2 (32,16,4,3,3), b2 (32), w3 (16,32,2,3,3), b3 (16), w4 (16), b4 (1))."""
    out = []
    for conv, bn in ((conv3d[0], conv3d[1]), (conv3d[3], conv3d[4]), (conv3d[6], conv3d[7]),
                     (volume11[0][0], volume11[0][1])):
        s = bn.weight / torch.sqrt(bn.running_var + bn.eps)
        w = conv.weight * s.view(-1, *([1] * (conv.weight.dim() - 1)))
        b = bn.bias - bn.running_mean * s
        if conv.bias is not None:
            b = b + conv.bias * s
        out += [w.detach().float().contiguous(), b.detach().float().contiguous()]
    w1, b1, w2, b2, w3, b3, w4, b4 = out
    return w1.reshape(16, 8, 3, 3), b1, w2, b2, w3, b3, w4.reshape(16), b4


def _volume_torch(featL, featR, conv3d, volume11, D):
    """The reference loop's arithmetic with every disparity as one batch entry (MIOpen Conv3d).
    Slice i of the reference convolves only x >= i with zero padding at the crop's edges; on the
    full-width zero-filled slice the same holds once every layer's output is re-zeroed at x < i."""
    B, C, H, W = featL.shape
    x = interweave_volume(featL, featR, D)                      # (B, 2C, D, H, W), 0 at x < d
    x = x.permute(0, 2, 1, 3, 4).reshape(B * D, 1, 2 * C, H, W)
    keep = (torch.arange(W, device=x.device).view(1, W) >=
            torch.arange(D, device=x.device).view(D, 1)).to(x.dtype)  # (D, W)
    keep = keep.repeat(B, 1).view(B * D, 1, 1, 1, W)
    for j in range(0, 9, 3):
        x = conv3d[j + 2](conv3d[j + 1](conv3d[j](x))) * keep
    x = volume11(x.squeeze(2)) * keep.squeeze(2)
    return x.view(B, D, H, W)


def interweave_conv_volume(featL, featR, conv3d, volume11, volume_size, impl="hip"):
    """MobileStereoNetV4's cost volume (:443-461): for every disparity i < volume_size,
    interweave(L[..., i:], R[..., :-i]) -> conv3d (8,3,3)/s8, (4,3,3)/s4, (2,3,3)/s2 with BN + ReLU
    -> squeeze -> volume11 (1x1 conv + BN + ReLU), placed at x >= i of a zero (N, D, H, W) volume.
    ``impl="hip"``: the HIP kernels (eval-mode BN folded); ``"torch"``: MIOpen."""
    if impl == "torch":
        return _volume_torch(featL, featR, conv3d, volume11, volume_size)
    if conv3d.training or volume11.training:
        raise RuntimeError("interweave_conv_volume(impl='hip') folds BatchNorm: eval mode only")
    return F.v4_volume(featL, featR, *fold_v4_weights(conv3d, volume11), volume_size)


__all__ = ["disparity_regression", "interweave_tensors", "interweave_volume",
           "interweave_conv_volume", "fold_v4_weights"]
