"""Drop-in for ``cost_volume/groupwise.py`` (TorchGroupwiseCost, :5-56)."""
import torch.nn as nn

from .. import functional as F


class TorchGroupwiseCost(nn.Module):
    """Group-wise correlation volume: (N,C,H,W) x2 -> (N, n_groups, H, W, max_disparity) fp32.

    volume[n, g, y, x, d] = mean over the g-th contiguous block of C/G channels of
    left*right(x-d) for x >= d, 0 otherwise (reference: groupwise.py:24-56).  Asserts
    C % G == 0 with the reference's message (:15-17).  The output lives on the input's
    device (the reference always allocates it on the CPU, :39 -- documented deviation).
    """

    def __init__(self, n_groups, max_disparity, *args, **kwargs) -> None:
        super().__init__(*args, **kwargs)
        self.n_groups = n_groups
        self.max_disparity = max_disparity

    def groupwise(self, left, right, n_groups):
        """Zero-disparity group-wise mean, (N, G, H, W) in the input dtype -- the reference
        helper (:12-22), whose (left*right).view(...).mean(2) keeps left.dtype.  The kernel
        accumulates in fp32 and rounds once to that dtype (the reference rounds every product
        and the mean in fp16/bf16: within its last-bit rounding)."""
        return F.groupwise_volume(left, right, n_groups, 1)[..., 0].to(left.dtype)

    def forward(self, left, right):
        return F.groupwise_volume(left, right, self.n_groups, self.max_disparity)
