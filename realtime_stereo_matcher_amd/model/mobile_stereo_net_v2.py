"""Hot-path helpers of ``model/mobile_stereo_net_v2.py`` (same ops as v1: :8-27, :217-220)."""
from .mobile_stereo_net import make_cost_volume, soft_argmin_regression  # noqa: F401
from ..functional import warp_by_flow_map  # noqa: F401,E402  (reference _v2.py:59-96, RefineNet warp)
