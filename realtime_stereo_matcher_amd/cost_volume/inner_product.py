"""Drop-in for ``cost_volume/inner_product.py`` (TorchInnerProductCost, :5-45)."""
import torch.nn as nn

from .. import functional as F


class TorchInnerProductCost(nn.Module):
    """Inner-product cost volume: (N,C,H,W) x2 -> (N, max_disparity, H, W).

    volume[n, d, y, x] = sum_c left[n,c,y,x] * right[n,c,y,x-d] for x >= d, 0 otherwise
    (reference forward: cost_volume/inner_product.py:11-42).  Runs one HIP kernel on the
    input's device; output dtype/device follow ``left``.
    """

    def __init__(self, max_disparity, *args, algo="auto", **kwargs) -> None:
        super().__init__(*args, **kwargs)
        self.max_disparity = max_disparity
        self.algo = algo

    def forward(self, left, right):
        return F.inner_product_volume(left, right, self.max_disparity, algo=self.algo)

    def __str__(self):
        # same description string as the reference (inner_product.py:44-45)
        return f"{self.__class__.__name__} | aijk,aijh->ajkh"
