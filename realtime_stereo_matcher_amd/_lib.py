"""ctypes binding of libstereocv.so (the C ABI in include/stereocv.h).

The library is required: there is no CPU or eager-PyTorch fallback anywhere in this
package.  If the shared object is missing or fails to load, every operator raises.
"""
import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("STEREOCV_LIB", os.path.join(_HERE, "libstereocv.so"))

SM_F32, SM_F16, SM_BF16, SM_F64 = 0, 1, 2, 3
SM_OK, SM_EINVAL, SM_EDTYPE, SM_ELAUNCH, SM_EUNSUPPORTED = 0, -1, -2, -3, -4
SM_ARGMIN, SM_ARGMAX = 0, 1
SM_REGRESS_SOFTMAX, SM_REGRESS_PRESOFTMAXED, SM_REGRESS_OUT_F32 = 0, 1, 2
SM_FUSED_DISP_F32 = 2
SM_FUSED_EXACT_ACC = 4
SM_IP_AUTO, SM_IP_VALU, SM_IP_MFMA_F32, SM_IP_MFMA_H2, SM_IP_MFMA_H2DB, SM_IP_MFMA_RS, SM_IP_MFMA_SL = 0, 1, 2, 5, 8, 11, 12

_p = ctypes.c_void_p
_i = ctypes.c_int
_l = ctypes.c_int64
_lp = ctypes.POINTER(ctypes.c_int64)

# name -> argtypes (restype is int unless listed in _RESTYPE)
SIGNATURES = {
    "sm_version": [],
    "sm_last_error": [],
    "sm_cv_inner_product": [_p, _p, _p, _i, _l, _l, _l, _l, _l, _lp, _lp, _p],
    "sm_cv_inner_product_ex": [_p, _p, _p, _i, _l, _l, _l, _l, _l, _lp, _lp, _i, _p],
    "sm_cv_correlation_mean": [_p, _p, _p, _i, _l, _l, _l, _l, _l, _lp, _lp, _p],
    "sm_cv_correlation_mean_ex": [_p, _p, _p, _i, _l, _l, _l, _l, _l, _lp, _lp, _i, _p],
    "sm_cv_groupwise": [_p, _p, _p, _i, _l, _l, _l, _l, _l, _l, _lp, _lp, _p],
    "sm_cv_inner_product_softargmin": [_p, _p, _p, _p, _i, _l, _l, _l, _l, _l, _lp, _lp, _i, _p],
    "sm_cv_inner_product_softargmin_workspace_bytes": [_l, _l, _l, _l],
    "sm_cv_inner_product_softargmin_ws": [_p, _p, _p, _p, _i, _l, _l, _l, _l, _l, _lp, _lp, _i, _p, _l, _p],
    "sm_cv_concat": [_p, _p, _p, _i, _l, _l, _l, _l, _l, _lp, _lp, _p],
    "sm_cv_interweave": [_p, _p, _p, _i, _l, _l, _l, _l, _lp, _lp, _p],
    "sm_cv_interweave_shifted": [_p, _p, _p, _i, _l, _l, _l, _l, _l, _lp, _lp, _p],
    "sm_cv_diff": [_p, _p, _p, _i, _l, _l, _l, _l, _l, _lp, _lp, _p],
    "sm_regress_softargmin": [_p, _p, _i, _l, _l, _l, _l, _i, _lp, _p],
    "sm_regress_argext": [_p, _p, _i, _l, _l, _l, _l, _i, _lp, _p],
    "sm_warp_by_flow": [_p, _p, _p, _i, _l, _l, _l, _l, _l, _l, _l, _lp, _lp, _p],
    "sm_warp_by_flow_workspace_bytes": [_l, _l, _l, _l, _l],
    "sm_warp_by_flow_ws": [_p, _p, _p, _i, _l, _l, _l, _l, _l, _l, _l, _lp, _lp, _p, _l, _p],
    "sm_v4_volume_workspace_bytes": [_l, _l, _l],
    "sm_v4_volume": [_p, _p, _p, _i, _l, _l, _l, _l, _l, _lp, _lp] + [_p] * 9 + [_l, _p],
}
_RESTYPE = {"sm_last_error": ctypes.c_char_p, "sm_v4_volume_workspace_bytes": ctypes.c_int64,
            "sm_warp_by_flow_workspace_bytes": ctypes.c_int64,
            "sm_cv_inner_product_softargmin_workspace_bytes": ctypes.c_int64}

_lock = threading.Lock()
_lib = None


class StereoCVError(RuntimeError):
    """A libstereocv call returned a non-zero status."""


def load():
    """Load (once) and return the ctypes handle; raise if the library is unavailable."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"libstereocv.so not found at {LIB_PATH}. Build it with "
                "`python -m realtime_stereo_matcher_amd.build_lib` (hipcc, gfx950). "
                "There is no CPU fallback.")
        lib = ctypes.CDLL(LIB_PATH)
        for name, args in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.argtypes = args
            fn.restype = _RESTYPE.get(name, ctypes.c_int)
        _lib = lib
        return lib


def check(rc, what):
    if rc != SM_OK:
        msg = load().sm_last_error().decode(errors="replace")
        raise StereoCVError(f"{what} failed (status {rc}): {msg}")


def strides_arg(t):
    """(N, C, H, W) element strides as an int64[4] for the C ABI."""
    return (ctypes.c_int64 * 4)(*[int(s) for s in t.stride()])
