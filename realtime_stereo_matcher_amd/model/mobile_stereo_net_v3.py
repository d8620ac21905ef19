"""Hot-path helpers of ``model/mobile_stereo_net_v3.py`` (same ops as v1: :9-28, :321-324)."""
from .mobile_stereo_net import make_cost_volume, soft_argmin_regression  # noqa: F401
from ..functional import warp_by_flow_map  # noqa: F401,E402  (reference _v3.py:60-97, RefineNet warp)
