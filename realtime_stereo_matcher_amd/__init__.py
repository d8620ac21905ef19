"""realtime_stereo_matcher_amd -- MI355X-native stereo cost-volume + disparity-regression engine.

Drop-in for the hot path of babiking/realtime_stereo_matcher:
  * ``realtime_stereo_matcher_amd.cost_volume``  mirrors ``cost_volume/*`` (the four nn.Modules)
  * ``realtime_stereo_matcher_amd.model``        mirrors the CV/regression helpers of ``model/*``
  * ``realtime_stereo_matcher_amd.functional``   the functional layer over libstereocv.so
  * ``realtime_stereo_matcher_amd.distributed``  batch sharding + RCCL gather of disparities

All compute runs in hand-written HIP kernels for gfx950 (``csrc/``, C ABI in
``include/stereocv.h``).  There is no CPU fallback.
"""
from . import functional  # noqa: F401
from ._lib import LIB_PATH, StereoCVError, load as load_library  # noqa: F401

__version__ = "0.1.0"
