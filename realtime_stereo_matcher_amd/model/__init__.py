"""Mirror of the reference ``model`` package's cost-volume and regression helpers only.

The network bodies (feature extractors, 3-D/2-D cost filters, refinement) are out of scope:
they stay on PyTorch-ROCm / MIOpen.  A reference network is switched to this engine by
replacing the helper it imports, e.g. ``mobile_stereo_net.make_cost_volume``.
"""
from . import mobile_disp_net_c, mobile_stereo_net, mobile_stereo_net_v2, mobile_stereo_net_v3, mobile_stereo_net_v4  # noqa: F401
