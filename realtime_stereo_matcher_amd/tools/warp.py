"""Drop-in for ``tools/warp.py`` (reference tools/warp.py:5-42): ``warp_by_flow_map`` on the
HIP warp kernel (csrc/warp.hip), same arguments, output and AssertionError."""
from ..functional import warp_by_flow_map  # noqa: F401
