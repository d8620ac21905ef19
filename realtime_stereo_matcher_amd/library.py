"""The engine's operators as PyTorch custom ops (``torch.ops.stereocv.*``) with fake kernels.

The reference networks are traced by ``torch.onnx.export`` (tools/convert.py:18-26) and by
thop / fvcore (tools/profiler.py:11-26).  A ctypes call is opaque to a tracer: ``torch.jit.trace``
would bake the call's output in as a constant and ``torch.export`` / ``torch.compile`` could
not see through it.  Registered here with ``torch.library.custom_op``, each operator is one node
of the traced graph: ``functional`` routes a call through ``torch.ops.stereocv.<name>`` whenever
it runs under ``torch.jit.trace`` or a compiler (dynamo / export), the fake kernel gives
FakeTensor tracing the output's shape, dtype and device, and the real kernel is the same
libstereocv call as the eager path (no CPU fallback).  The ops are forward-only like the rest
of the engine: their backward raises ``NotImplementedError``.
"""
from __future__ import annotations

import threading

import torch

from . import functional as F

_state = threading.local()


def tracing() -> bool:
    """True when a functional call should go through torch.ops.stereocv (a tracer or compiler
    is recording, and the call is not already the body of one of these ops)."""
    if getattr(_state, "inside", False):
        return False
    try:
        compiling = torch.compiler.is_compiling()
    except AttributeError:  # older torch
        compiling = False
    return torch.jit.is_tracing() or compiling


class _Inside:
    def __enter__(self):
        self.prev = getattr(_state, "inside", False)
        _state.inside = True

    def __exit__(self, *exc):
        _state.inside = self.prev


def _forward_only(ctx, *grads):
    raise NotImplementedError(
        "realtime_stereo_matcher_amd cost-volume kernels are forward/inference-only; "
        "backward is not implemented")


def _no_ctx(ctx, inputs, output):
    return None


def _register(name, impl, fake):
    op = torch.library.custom_op(f"stereocv::{name}", mutates_args=())(impl)
    op.register_fake(fake)
    torch.library.register_autograd(f"stereocv::{name}", _forward_only, setup_context=_no_ctx)
    return op


def _empty(shape, like, dtype=None):
    return like.new_empty(shape, dtype=dtype if dtype is not None else like.dtype)


# ------------------------------------------------------------------------------------- ops
def _inner_product(left: torch.Tensor, right: torch.Tensor, max_disparity: int,
                   algo: str) -> torch.Tensor:
    with _Inside():
        return F.inner_product_volume(left, right, max_disparity, algo=algo)


def _inner_product_fake(left, right, max_disparity, algo):
    n, _, h, w = left.shape
    return _empty((n, max_disparity, h, w), left)


def _correlation(left: torch.Tensor, right: torch.Tensor, max_disp: int,
                 algo: str = "auto") -> torch.Tensor:
    with _Inside():
        return F.correlation_volume(left, right, max_disp, algo=algo)


def _correlation_fake(left, right, max_disp, algo="auto"):
    n, _, h, w = left.shape
    return _empty((n, max_disp, h, w), left)


def _groupwise(left: torch.Tensor, right: torch.Tensor, n_groups: int,
               max_disparity: int) -> torch.Tensor:
    with _Inside():
        return F.groupwise_volume(left, right, n_groups, max_disparity)


def _groupwise_fake(left, right, n_groups, max_disparity):
    n, _, h, w = left.shape
    return _empty((n, n_groups, h, w, max_disparity), left, torch.float32)


def _concat(left: torch.Tensor, right: torch.Tensor, max_disparity: int) -> torch.Tensor:
    with _Inside():
        return F.concat_volume(left, right, max_disparity)


def _concat_fake(left, right, max_disparity):
    n, c, h, w = left.shape
    return _empty((n, 2 * c, h, w, max_disparity), left)


def _interweave(left: torch.Tensor, right: torch.Tensor) -> torch.Tensor:
    with _Inside():
        return F.interweave(left, right)


def _interweave_fake(left, right):
    n, c, h, w = left.shape
    return _empty((n, 2 * c, h, w), left)


def _interweave_volume(left: torch.Tensor, right: torch.Tensor, max_disparity: int) -> torch.Tensor:
    with _Inside():
        return F.interweave_volume(left, right, max_disparity)


def _interweave_volume_fake(left, right, max_disparity):
    n, c, h, w = left.shape
    return _empty((n, 2 * c, max_disparity, h, w), left)


def _difference(left: torch.Tensor, right: torch.Tensor, max_disp: int) -> torch.Tensor:
    with _Inside():
        return F.difference_volume(left, right, max_disp)


def _difference_fake(left, right, max_disp):
    n, c, h, w = left.shape
    return _empty((n, c, max_disp, h, w), left)


def _regress_dtype(volume, f32):
    # the autocast rule of functional._regress, decided when the graph was traced (f32: an
    # fp16 / bf16 volume under autocast gives fp32)
    return torch.float32 if f32 else volume.dtype


def _soft_argmin(volume: torch.Tensor, f32: bool = False) -> torch.Tensor:
    with _Inside(), F._F32Decided(f32):
        return F.soft_argmin(volume, keepdim=False)


def _soft_argmin_fake(volume, f32=False):
    n, _, h, w = volume.shape
    return _empty((n, h, w), volume, _regress_dtype(volume, f32))


def _presoftmax(prob: torch.Tensor, f32: bool = False) -> torch.Tensor:
    with _Inside(), F._F32Decided(f32):
        return F.regression_presoftmax(prob)


def _presoftmax_fake(prob, f32=False):
    n, _, h, w = prob.shape
    return _empty((n, h, w), prob, _regress_dtype(prob, f32))


def _argext_fake(volume):
    n, _, h, w = volume.shape
    return _empty((n, h, w), volume, torch.int64)


def _hard_argmin(volume: torch.Tensor) -> torch.Tensor:
    with _Inside():
        return F.hard_argmin(volume)


def _hard_argmax(volume: torch.Tensor) -> torch.Tensor:
    with _Inside():
        return F.hard_argmax(volume)


def _fused(left: torch.Tensor, right: torch.Tensor, max_disparity: int, mean: bool,
           f32: bool = False, exact: bool = False) -> tuple[torch.Tensor, torch.Tensor]:
    with _Inside(), F._F32Decided(f32):
        return F.inner_product_soft_argmin(left, right, max_disparity, mean=mean, keep_volume=True,
                                           exact_accumulators=exact)


def _fused_disp_dtype(left, f32):
    # autocast with half features (decided when the graph was traced): fp32 disparities
    return torch.float32 if f32 else left.dtype


def _fused_fake(left, right, max_disparity, mean, f32=False, exact=False):
    n, _, h, w = left.shape
    return (_empty((n, max_disparity, h, w), left),
            _empty((n, 1, h, w), left, _fused_disp_dtype(left, f32)))


def _fused_novolume(left: torch.Tensor, right: torch.Tensor, max_disparity: int, mean: bool,
                    f32: bool = False, exact: bool = False) -> torch.Tensor:
    with _Inside(), F._F32Decided(f32):
        return F.inner_product_soft_argmin(left, right, max_disparity, mean=mean,
                                           keep_volume=False, exact_accumulators=exact)[1]


def _fused_novolume_fake(left, right, max_disparity, mean, f32=False, exact=False):
    n, _, h, w = left.shape
    return _empty((n, 1, h, w), left, _fused_disp_dtype(left, f32))


def _warp(image: torch.Tensor, flow: torch.Tensor, f32: bool = False) -> torch.Tensor:
    with _Inside(), F._F32Decided(f32):
        return F.warp_by_flow_map(image, flow)


def _warp_fake(image, flow, f32=False):
    # the output dtype rule of functional.warp_by_flow_map: fp32 under autocast (grid_sample is
    # an autocast fp32 op; decided when the graph was traced), else the image dtype (fp32 for an
    # fp32 image)
    n, _, h, w = flow.shape
    odt = torch.float32 if f32 else image.dtype
    return _empty((n, image.shape[1], h, w), image, odt)


def _v4(featL: torch.Tensor, featR: torch.Tensor, w1: torch.Tensor, b1: torch.Tensor,
        w2: torch.Tensor, b2: torch.Tensor, w3: torch.Tensor, b3: torch.Tensor, w4: torch.Tensor,
        b4: torch.Tensor, volume_size: int) -> torch.Tensor:
    with _Inside():
        return F.v4_volume(featL, featR, w1, b1, w2, b2, w3, b3, w4, b4, volume_size)


def _v4_fake(featL, featR, w1, b1, w2, b2, w3, b3, w4, b4, volume_size):
    n, _, h, w = featL.shape
    return _empty((n, volume_size, h, w), featL, torch.float32)


inner_product_volume = _register("inner_product_volume", _inner_product, _inner_product_fake)
correlation_volume = _register("correlation_volume", _correlation, _correlation_fake)
groupwise_volume = _register("groupwise_volume", _groupwise, _groupwise_fake)
concat_volume = _register("concat_volume", _concat, _concat_fake)
interweave = _register("interweave", _interweave, _interweave_fake)
interweave_volume = _register("interweave_volume", _interweave_volume, _interweave_volume_fake)
difference_volume = _register("difference_volume", _difference, _difference_fake)
soft_argmin = _register("soft_argmin", _soft_argmin, _soft_argmin_fake)
regression_presoftmax = _register("regression_presoftmax", _presoftmax, _presoftmax_fake)
hard_argmin = _register("hard_argmin", _hard_argmin, _argext_fake)
hard_argmax = _register("hard_argmax", _hard_argmax, _argext_fake)
inner_product_soft_argmin = _register("inner_product_soft_argmin", _fused, _fused_fake)
inner_product_soft_argmin_novolume = _register("inner_product_soft_argmin_novolume",
                                               _fused_novolume, _fused_novolume_fake)
warp_by_flow_map = _register("warp_by_flow_map", _warp, _warp_fake)
v4_volume = _register("v4_volume", _v4, _v4_fake)
