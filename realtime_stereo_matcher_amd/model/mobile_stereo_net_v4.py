"""Hot-path helpers of ``model/mobile_stereo_net_v4.py``."""
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
