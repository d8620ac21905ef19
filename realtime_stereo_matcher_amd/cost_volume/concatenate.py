"""Drop-in for ``cost_volume/concatenate.py`` (TorchConcatenateCost, :5-41)."""
import torch.nn as nn

from .. import functional as F


class TorchConcatenateCost(nn.Module):
    """Concatenation volume: (N,C,H,W) x2 -> (N, 2C, H, W, max_disparity).

    volume[:, :C, y, x, d] = left[..., x], volume[:, C:, y, x, d] = right[..., x-d] for x >= d,
    both 0 for x < d (reference: concatenate.py:11-41).  Bit-exact copy kernel.
    """

    def __init__(self, max_disparity, *args, **kwargs) -> None:
        super().__init__(*args, **kwargs)
        self.max_disparity = max_disparity

    def forward(self, left, right):
        return F.concat_volume(left, right, self.max_disparity)
