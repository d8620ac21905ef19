"""Hot-path helpers of ``model/mobile_stereo_net.py``."""
from .. import functional as F


def make_cost_volume(left, right, max_disp):
    """Difference volume (model/mobile_stereo_net.py:8-27): (N,C,H,W) x2 -> (N,C,D,H,W),
    left - right(x-d) for x >= d and 1.0 for x < d."""
    return F.difference_volume(left, right, max_disp)


def soft_argmin_regression(cost_volume):
    """The inline regression of MobileStereoNet.forward (:144-147): softmax over D, then
    sum_d d * p with keepdim -> (N,1,H,W)."""
    return F.soft_argmin(cost_volume, keepdim=True)
