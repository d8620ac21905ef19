"""Hot-path helpers of ``model/mobile_disp_net_c.py``."""
from .. import functional as F


def make_correlation_volume(l_fmap, r_fmap, max_disp):
    """Mean-correlation volume (model/mobile_disp_net_c.py:188-205): (N,C,H,W) x2 -> (N,D,H,W)."""
    return F.correlation_volume(l_fmap, r_fmap, max_disp)


def disparity_regression(corr_volume, max_disp):
    """Soft-argmin with the softmax inside, keepdim -> (N,1,H,W)
    (model/mobile_disp_net_c.py:208-220, same assertion messages)."""
    assert len(corr_volume.shape) == 4, f"#dimensions of correlation volume != 4."
    assert (
        corr_volume.shape[1] == max_disp
    ), f"#channels of correlation volume != max_disparity ({max_disp})."
    return F.soft_argmin(corr_volume, keepdim=True)
