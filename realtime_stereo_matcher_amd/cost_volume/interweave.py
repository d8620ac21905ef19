"""Drop-in for ``cost_volume/interweave.py`` (TorchInterweaveCost, :5-25)."""
import torch.nn as nn

from .. import functional as F


class TorchInterweaveCost(nn.Module):
    """Channel interweave: (N,C,H,W) x2 -> (N, 2C, H, W), even channels left, odd right
    (reference: interweave.py:10-22).  Bit-exact copy kernel."""

    def __init__(self, *args, **kwargs) -> None:
        super().__init__(*args, **kwargs)

    def forward(self, left, right):
        return F.interweave(left, right)

    def __str__(self):
        return self.__class__.__name__
