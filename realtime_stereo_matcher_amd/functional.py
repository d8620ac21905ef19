"""Functional front-end of the MI355X stereo cost-volume engine.

Every function validates its arguments the way the reference does, allocates the output
with the caching allocator on the input's device and enqueues ONE libstereocv kernel on
the current HIP stream (no host sync).  There is no CPU / eager fallback: tensors must live
on a HIP device and the native library must load, otherwise the call raises.

Reference operators mirrored (babiking/realtime_stereo_matcher):
  inner_product_volume   cost_volume/inner_product.py:11-42
  groupwise_volume       cost_volume/groupwise.py:24-56
  concat_volume          cost_volume/concatenate.py:11-41
  interweave             cost_volume/interweave.py:10-22, model/mobile_stereo_net_v4.py:17-23
  interweave_volume      model/mobile_stereo_net_v4.py:443-461 (shifted interweave, materialised)
  difference_volume      model/mobile_stereo_net.py:8-27 (+ _v2.py:8-27, _v3.py:9-28)
  correlation_volume     model/mobile_disp_net_c.py:188-205
  inner_product_soft_argmin  either volume fused with soft_argmin
  soft_argmin            model/mobile_disp_net_c.py:208-220, model/mobile_stereo_net.py:144-147
  regression_presoftmax  model/mobile_stereo_net_v4.py:10-14
  hard_argmin/argmax     build-defined
  warp_by_flow_map       tools/warp.py:5-42, model/mobile_stereo_net_v2.py:59-96
"""
from __future__ import annotations

import numpy as np
import threading

import torch

from . import _lib

# float64 (round 6): the cost volumes and the regressions in fp64 (csrc/f64.hip), as torch
# computes an fp64 input; the warp and the V4 volume stay float32 / 16-bit
_DTYPES = {torch.float32: _lib.SM_F32, torch.float16: _lib.SM_F16, torch.bfloat16: _lib.SM_BF16,
           torch.float64: _lib.SM_F64}
_WARP_DTYPES = (torch.float32, torch.float16, torch.bfloat16)
_ALGOS = {"auto": _lib.SM_IP_AUTO, "valu": _lib.SM_IP_VALU, "mfma": _lib.SM_IP_MFMA_F32,
          "f32": _lib.SM_IP_MFMA_F32, "h2": _lib.SM_IP_MFMA_H2, "h2db": _lib.SM_IP_MFMA_H2DB,
          "rs": _lib.SM_IP_MFMA_RS, "sl": _lib.SM_IP_MFMA_SL}


# ----------------------------------------------------------------------------------- plumbing
def _traced():
    """Under torch.jit.trace or a compiler the call is routed through torch.ops.stereocv, so the
    traced graph holds the operator instead of its output as a constant (library.py)."""
    from . import library
    return library.tracing()


def _ops():
    from . import library  # noqa: F401  (registers the ops)
    return torch.ops.stereocv

def _device_check(*ts):
    dev = ts[0].device
    for t in ts:
        if t.device.type != "cuda":
            raise RuntimeError(
                "realtime_stereo_matcher_amd runs on HIP devices only (got a tensor on "
                f"'{t.device}'); there is no CPU fallback -- move the features with .cuda()")
        if t.device != dev:
            raise RuntimeError(f"tensors on different devices: {dev} vs {t.device}")
    return dev


def _dtype_code(t):
    code = _DTYPES.get(t.dtype)
    if code is None:
        raise TypeError(f"unsupported dtype {t.dtype}; expected float32, float16, bfloat16 or float64")
    return code


def _rows_contiguous(t):
    """The C ABI needs unit W stride; any other stride pattern is passed through."""
    return t if (t.dim() == 0 or t.stride(-1) == 1 or t.size(-1) <= 1) else t.contiguous()


def _stride_ok(t):
    # size-1 W can carry any stride in torch; normalise so the ABI sees 1
    if t.size(-1) <= 1 and t.stride(-1) != 1:
        t = t.contiguous()
    return t


def _pair(left, right, what):
    if not isinstance(left, torch.Tensor) or not isinstance(right, torch.Tensor):
        raise TypeError(f"{what}: left and right must be tensors")
    if left.dim() != 4 or right.dim() != 4:
        raise RuntimeError(f"{what}: expected 4-D (N, C, H, W) features, got {tuple(left.shape)} "
                           f"and {tuple(right.shape)}")
    if left.shape != right.shape:
        raise RuntimeError(f"{what}: left/right shape mismatch {tuple(left.shape)} vs "
                           f"{tuple(right.shape)}")
    if left.dtype != right.dtype:
        raise RuntimeError(f"{what}: left/right dtype mismatch {left.dtype} vs {right.dtype}")
    code = _dtype_code(left)
    dev = _device_check(left, right)
    left = _stride_ok(_rows_contiguous(left))
    right = _stride_ok(_rows_contiguous(right))
    return left, right, dev, code


def _stream(dev):
    return torch.cuda.current_stream(dev).cuda_stream


def _disp(max_disparity, what):
    d = int(max_disparity)
    if d < 0:
        raise RuntimeError(f"{what}: max disparity must be non-negative, got {d}")
    return d


class _ForwardOnly(torch.autograd.Function):
    """Marks outputs as produced by a forward-only native kernel (no autograd support yet)."""

    @staticmethod
    def forward(ctx, fn, *tensors):
        return fn()

    @staticmethod
    def backward(ctx, *grads):
        raise NotImplementedError(
            "realtime_stereo_matcher_amd cost-volume kernels are forward/inference-only; "
            "backward is not implemented")


def _run(fn, *inputs):
    # the entry points size persistent grids and set kernel attributes on the CURRENT HIP
    # device: make it the inputs' device for the call
    with torch.cuda.device(inputs[0].device):
        if torch.is_grad_enabled() and any(t.requires_grad for t in inputs):
            return _ForwardOnly.apply(fn, *inputs)
        return fn()


def _ptr(t):
    return t.data_ptr()


_HALF = (torch.float16, torch.bfloat16)


def _autocast_fp32(*ts):
    """True when torch autocast is active on the tensors' device and one of them is fp16 / bf16.

    The reference evaluates under ``torch.cuda.amp.autocast`` (``mixed_precision`` defaults to
    True: evaluate_stereo.py:48,124,182,231,320; test_stereo.py:117).  Its Conv3d outputs are
    then fp16, but ``F.softmax``, ``torch.sum`` and ``F.grid_sample`` are autocast fp32 ops, so
    the soft-argmin (mobile_stereo_net.py:144-147, mobile_disp_net_c.py:208-220) returns an fp32
    disparity from an fp16 volume and the RefineNet warp (tools/warp.py:39) samples in fp32.
    The engine follows: under autocast these ops return fp32 (one rounding, from fp64 / fp32
    arithmetic), never the volume's reduced dtype.
    """
    ov = getattr(_decided, "f32", None)
    if ov is not None:  # the body of a torch.ops.stereocv op: the decision made at trace time
        return ov
    return any(t.dtype in _HALF for t in ts) and torch.is_autocast_enabled(ts[0].device.type)


_decided = threading.local()


class _F32Decided:
    """Inside a torch.ops.stereocv op (library.py) the fp32-output decision is an op argument
    taken when the graph was traced, not the autocast state at run time: a compiled graph may run
    its ops after the compiler removed the autocast regions."""

    def __init__(self, value):
        self.value = bool(value)

    def __enter__(self):
        self.prev = getattr(_decided, "f32", None)
        _decided.f32 = self.value

    def __exit__(self, *exc):
        _decided.f32 = self.prev


# ----------------------------------------------------------------------------- a-1, a-6, a-2
def inner_product_volume(left, right, max_disparity, algo="auto"):
    """(N,C,H,W) x2 -> (N,D,H,W): sum_c L*R(x-d) for x >= d, 0 elsewhere (left dtype/device)."""
    if _traced():
        return _ops().inner_product_volume(left, right, int(max_disparity), algo)
    left, right, dev, code = _pair(left, right, "inner_product_volume")
    D = _disp(max_disparity, "inner_product_volume")
    if algo not in _ALGOS:
        raise ValueError(f"algo must be one of {sorted(_ALGOS)}")
    n, c, h, w = left.shape

    def fn():
        out = torch.empty((n, D, h, w), dtype=left.dtype, device=dev)
        if out.numel():
            lib = _lib.load()
            _lib.check(lib.sm_cv_inner_product_ex(
                _ptr(left), _ptr(right), _ptr(out), code, n, c, h, w, D,
                _lib.strides_arg(left), _lib.strides_arg(right), _ALGOS[algo], _stream(dev)),
                "sm_cv_inner_product")
        return out

    return _run(fn, left, right)


def correlation_volume(l_fmap, r_fmap, max_disp, algo="auto"):
    """(N,C,H,W) x2 -> (N,D,H,W): mean_c L*R(x-d) for x >= d, 0 elsewhere (``algo``: the band
    kernel, as for inner_product_volume)."""
    if algo not in _ALGOS:
        raise ValueError(f"algo must be one of {sorted(_ALGOS)}")
    if _traced():
        return _ops().correlation_volume(l_fmap, r_fmap, int(max_disp), algo)
    left, right, dev, code = _pair(l_fmap, r_fmap, "correlation_volume")
    D = _disp(max_disp, "correlation_volume")
    n, c, h, w = left.shape

    def fn():
        out = torch.empty((n, D, h, w), dtype=left.dtype, device=dev)
        if out.numel():
            lib = _lib.load()
            _lib.check(lib.sm_cv_correlation_mean_ex(
                _ptr(left), _ptr(right), _ptr(out), code, n, c, h, w, D,
                _lib.strides_arg(left), _lib.strides_arg(right), _ALGOS[algo], _stream(dev)),
                "sm_cv_correlation_mean_ex")
        return out

    return _run(fn, left, right)


def inner_product_soft_argmin(left, right, max_disparity, mean=False, keep_volume=True,
                              exact_accumulators=False):
    """Cost volume + soft-argmin in one kernel pass.

    The inner-product volume (cost_volume/inner_product.py:11-42; ``mean=True``: the
    correlation volume of model/mobile_disp_net_c.py:188-205) and its disparity regression
    sum_d d * softmax_d(volume) (model/mobile_disp_net_c.py:208-220, = the inline soft-argmin of
    model/mobile_stereo_net.py:144-147).  Returns ``(volume, disparity)``: the (N,D,H,W) volume
    (``None`` with ``keep_volume=False``: it is then never written) and the (N,1,H,W) disparity.

    Precision, per the reference's two calls:
    - fp32 features: the volume and the disparity are fp32.  For D <= 192 the disparity does
      not depend on ``keep_volume`` (one kernel folds the same accumulators either way; on the
      sliding-window kernel the fold scales the raw accumulators inside the exponent's FMA
      rather than reading the stored cells, so it is within 1e-4 of the soft-argmin of the
      volume returned, not bit-equal to it).  For C = 16 and D > 192 the volume-kept call runs
      the volume kernel and the regression kernel, the volume-free call one two-pass fold: the
      two disparities agree within 1e-4.
    - fp16 / bf16 features outside autocast: both in the feature dtype.
    - fp16 / bf16 features under ``torch.autocast`` (the reference's default eval,
      evaluate_stereo.py:48): the volume keeps the feature dtype and the disparity is fp32, the
      soft-argmin of the volume's cells as rounded to the feature dtype -- what the reference's
      ``disparity_regression(corr_volume)`` regresses -- on every shape.  ``exact_accumulators=
      True`` regresses the fp32 accumulators of the exact products instead (no rounding), on the
      shapes the fused kernel takes (4-element aligned rows; D <= 192 with the volume kept);
      the other shapes regress the rounded volume either way.

    fp32 features (W >= 4) run one fused band kernel for D <= 192 and, without the volume, for
    C = 16 and D <= 256 (two D passes per segment merged in registers) or other D > 192 (passes
    of <= 192 disparities whose partial softmax states a second kernel merges, in a workspace
    allocated here); other shapes run the volume and the regression kernels back to back.
    """
    if _traced():
        f32, ex = _autocast_fp32(left), bool(exact_accumulators)
        if keep_volume:
            return _ops().inner_product_soft_argmin(left, right, int(max_disparity), bool(mean), f32, ex)
        return None, _ops().inner_product_soft_argmin_novolume(left, right, int(max_disparity),
                                                               bool(mean), f32, ex)
    left, right, dev, code = _pair(left, right, "inner_product_soft_argmin")
    D = _disp(max_disparity, "inner_product_soft_argmin")
    n, c, h, w = left.shape
    mode = 1 if mean else 0
    # autocast eval with fp16 / bf16 features: the volume keeps the feature dtype (the reference
    # assigns into zeros of left.dtype) and the soft-argmin returns fp32 -- the fused kernel's
    # fp32-disparity mode, which rounds each cell to the feature dtype before the fold (the
    # volume the reference regresses); SM_FUSED_EXACT_ACC folds the fp32 accumulators instead
    f32disp = _autocast_fp32(left)
    if f32disp:
        mode |= _lib.SM_FUSED_DISP_F32
        if exact_accumulators:
            mode |= _lib.SM_FUSED_EXACT_ACC

    def call(vol, disp, ws=None, nws=0):
        lib = _lib.load()
        return lib.sm_cv_inner_product_softargmin_ws(
            _ptr(left), _ptr(right), None if vol is None else _ptr(vol), _ptr(disp), code,
            n, c, h, w, D, _lib.strides_arg(left), _lib.strides_arg(right), mode,
            None if ws is None else _ptr(ws), nws, _stream(dev))

    def fn(keep):
        vol = torch.empty((n, D, h, w), dtype=left.dtype, device=dev) if keep else None
        disp = torch.empty((n, 1, h, w), dtype=torch.float32 if f32disp else left.dtype, device=dev)
        if disp.numel():
            # first without a workspace: the volume-free shapes band_sl takes (C = 16, D <= 256)
            # merge their D passes in registers and need none (the cfg4 launch used
            # to allocate 2.6 GB it never read)
            rc = call(vol, disp)
            if rc == _lib.SM_EUNSUPPORTED and vol is None and (code == _lib.SM_F32 or f32disp):
                # several D passes on band_h2: their partial softmax states go to a workspace
                nws = int(_lib.load().sm_cv_inner_product_softargmin_workspace_bytes(n, h, w, D))
                if nws > 0:
                    rc = call(None, disp, torch.empty(nws, dtype=torch.uint8, device=dev), nws)
            if rc == _lib.SM_EUNSUPPORTED and vol is None:
                # not a fused shape: the two-kernel path needs the volume in HBM for a moment
                rc = call(torch.empty((n, D, h, w), dtype=left.dtype, device=dev), disp)
            _lib.check(rc, "sm_cv_inner_product_softargmin")
        return vol, disp

    if keep_volume:
        return _run(lambda: fn(True), left, right)
    return None, _run(lambda: fn(False)[1], left, right)


def groupwise_volume(left, right, n_groups, max_disparity):
    """(N,C,H,W) x2 -> (N,G,H,W,D) float32: per-group mean of L*R(x-d), 0 for x < d.

    Deviation (documented): the reference allocates its output on the CPU regardless of the
    input device (cost_volume/groupwise.py:39); this engine returns it on the input device.
    """
    if _traced():
        return _ops().groupwise_volume(left, right, int(n_groups), int(max_disparity))
    G = int(n_groups)
    D = _disp(max_disparity, "groupwise_volume")
    if isinstance(left, torch.Tensor) and left.dim() == 4 and D > 0:
        # the reference asserts inside groupwise(), reached once per disparity (groupwise.py:15-17)
        c = left.shape[1]
        assert c % G == 0, f"groupwise cost channel ({c}) % #groups ({G}) != 0."
    left, right, dev, code = _pair(left, right, "groupwise_volume")
    n, c, h, w = left.shape

    def fn():
        out = torch.empty((n, G, h, w, D), dtype=torch.float32, device=dev)
        if out.numel():
            lib = _lib.load()
            _lib.check(lib.sm_cv_groupwise(
                _ptr(left), _ptr(right), _ptr(out), code, n, c, h, w, D, G,
                _lib.strides_arg(left), _lib.strides_arg(right), _stream(dev)),
                "sm_cv_groupwise")
        return out

    return _run(fn, left, right)


# ----------------------------------------------------------------------------- a-3, a-4, a-5
def concat_volume(left, right, max_disparity):
    """(N,C,H,W) x2 -> (N,2C,H,W,D): [:C]=L, [C:]=R(x-d) for x >= d, 0 elsewhere (bit-exact)."""
    if _traced():
        return _ops().concat_volume(left, right, int(max_disparity))
    left, right, dev, code = _pair(left, right, "concat_volume")
    D = _disp(max_disparity, "concat_volume")
    n, c, h, w = left.shape

    def fn():
        out = torch.empty((n, 2 * c, h, w, D), dtype=left.dtype, device=dev)
        if out.numel():
            lib = _lib.load()
            _lib.check(lib.sm_cv_concat(
                _ptr(left), _ptr(right), _ptr(out), code, n, c, h, w, D,
                _lib.strides_arg(left), _lib.strides_arg(right), _stream(dev)), "sm_cv_concat")
        return out

    return _run(fn, left, right)


def interweave(left, right):
    """(N,C,H,W) x2 -> (N,2C,H,W): even channels L, odd channels R (bit-exact)."""
    if _traced():
        return _ops().interweave(left, right)
    left, right, dev, code = _pair(left, right, "interweave")
    n, c, h, w = left.shape

    def fn():
        out = torch.empty((n, 2 * c, h, w), dtype=left.dtype, device=dev)
        if out.numel():
            lib = _lib.load()
            _lib.check(lib.sm_cv_interweave(
                _ptr(left), _ptr(right), _ptr(out), code, n, c, h, w,
                _lib.strides_arg(left), _lib.strides_arg(right), _stream(dev)), "sm_cv_interweave")
        return out

    return _run(fn, left, right)


def interweave_volume(left, right, max_disparity):
    """(N,C,H,W) x2 -> (N,2C,D,H,W): the v4 per-disparity interweave, 0 for x < d (bit-exact)."""
    if _traced():
        return _ops().interweave_volume(left, right, int(max_disparity))
    left, right, dev, code = _pair(left, right, "interweave_volume")
    D = _disp(max_disparity, "interweave_volume")
    n, c, h, w = left.shape

    def fn():
        out = torch.empty((n, 2 * c, D, h, w), dtype=left.dtype, device=dev)
        if out.numel():
            lib = _lib.load()
            _lib.check(lib.sm_cv_interweave_shifted(
                _ptr(left), _ptr(right), _ptr(out), code, n, c, h, w, D,
                _lib.strides_arg(left), _lib.strides_arg(right), _stream(dev)),
                "sm_cv_interweave_shifted")
        return out

    return _run(fn, left, right)


def v4_volume(featL, featR, w1, b1, w2, b2, w3, b3, w4, b4, volume_size=48):
    """MobileStereoNetV4's cost volume (model/mobile_stereo_net_v4.py:443-461):
    (N,32,H,W) fp32 x2 -> (N,D,H,W) fp32, slice i = volume11(conv3d(interweave(L[..., i:],
    R[..., :-i]))) at x >= i, 0 elsewhere, from eval-mode-folded weights
    (``model.mobile_stereo_net_v4.fold_v4_weights``)."""
    if _traced():
        return _ops().v4_volume(featL, featR, w1, b1, w2, b2, w3, b3, w4, b4, int(volume_size))
    left, right, dev, code = _pair(featL, featR, "v4_volume")
    if code != _lib.SM_F32:
        raise TypeError("v4_volume: float32 features only")
    D = _disp(volume_size, "v4_volume")
    n, c, h, w = left.shape
    ws = [t.detach().to(device=dev, dtype=torch.float32).contiguous() for t in (w1, b1, w2, b2, w3, b3, w4, b4)]
    shapes = [(16, 8, 3, 3), (16,), (32, 16, 4, 3, 3), (32,), (16, 32, 2, 3, 3), (16,), (16,), (1,)]
    for t, shp in zip(ws, shapes):
        if t.numel() != int(np.prod(shp)):
            raise ValueError(f"v4_volume: weight of {t.numel()} elements, expected shape {shp}")

    def fn():
        out = torch.empty((n, D, h, w), dtype=torch.float32, device=dev)
        if out.numel():
            lib = _lib.load()
            nbytes = int(lib.sm_v4_volume_workspace_bytes(n, h, w))
            scratch = torch.empty(nbytes, dtype=torch.uint8, device=dev)
            _lib.check(lib.sm_v4_volume(
                _ptr(left), _ptr(right), _ptr(out), code, n, c, h, w, D,
                _lib.strides_arg(left), _lib.strides_arg(right), *[_ptr(t) for t in ws],
                _ptr(scratch), nbytes, _stream(dev)), "sm_v4_volume")
        return out

    return _run(fn, left, right)


def difference_volume(left, right, max_disp):
    """(N,C,H,W) x2 -> (N,C,D,H,W): L - R(x-d) for x >= d, 1.0 elsewhere (bit-exact)."""
    if _traced():
        return _ops().difference_volume(left, right, int(max_disp))
    left, right, dev, code = _pair(left, right, "difference_volume")
    D = _disp(max_disp, "difference_volume")
    n, c, h, w = left.shape

    def fn():
        out = torch.empty((n, c, D, h, w), dtype=left.dtype, device=dev)
        if out.numel():
            lib = _lib.load()
            _lib.check(lib.sm_cv_diff(
                _ptr(left), _ptr(right), _ptr(out), code, n, c, h, w, D,
                _lib.strides_arg(left), _lib.strides_arg(right), _stream(dev)), "sm_cv_diff")
        return out

    return _run(fn, left, right)


# ----------------------------------------------------------------------------- a-7, a-8
def _volume(volume, what):
    if not isinstance(volume, torch.Tensor):
        raise TypeError(f"{what}: volume must be a tensor")
    if volume.dim() != 4:
        raise RuntimeError(f"{what}: expected a 4-D (N, D, H, W) volume, got {tuple(volume.shape)}")
    code = _dtype_code(volume)
    dev = _device_check(volume)
    return _stride_ok(_rows_contiguous(volume)), dev, code


def _regress(volume, flags, what):
    vol, dev, code = _volume(volume, what)
    n, d, h, w = vol.shape
    odt = vol.dtype
    if _autocast_fp32(vol):  # autocast: F.softmax / torch.sum run in fp32 (see _autocast_fp32)
        flags |= _lib.SM_REGRESS_OUT_F32
        odt = torch.float32

    def fn():
        out = torch.empty((n, h, w), dtype=odt, device=dev)
        if out.numel():
            lib = _lib.load()
            _lib.check(lib.sm_regress_softargmin(
                _ptr(vol), _ptr(out), code, n, d, h, w, flags, _lib.strides_arg(vol), _stream(dev)),
                "sm_regress_softargmin")
        return out

    return _run(fn, vol)


def soft_argmin(volume, keepdim=True):
    """sum_d d * softmax_d(volume) -> (N,1,H,W) (keepdim) or (N,H,W); fp64 accumulation.
    The output has the volume's dtype; under torch autocast an fp16 / bf16 volume gives fp32
    (the reference's autocast F.softmax + torch.sum)."""
    if _traced():
        out = _ops().soft_argmin(volume, _autocast_fp32(volume))
        return out.unsqueeze(1) if keepdim else out
    out = _regress(volume, _lib.SM_REGRESS_SOFTMAX, "soft_argmin")
    return out.unsqueeze(1) if keepdim else out


def regression_presoftmax(prob):
    """sum_d d * prob[:, d] over an already-softmaxed (N,D,H,W) volume -> (N,H,W) (fp32 under
    autocast for an fp16 / bf16 input, the reference's autocast torch.sum)."""
    if _traced():
        return _ops().regression_presoftmax(prob, _autocast_fp32(prob))
    return _regress(prob, _lib.SM_REGRESS_PRESOFTMAXED, "regression_presoftmax")


def _argext(volume, mode, what):
    vol, dev, code = _volume(volume, what)
    n, d, h, w = vol.shape
    if d == 0 and n * h * w > 0:
        raise IndexError(f"{what}: cannot reduce over an empty disparity axis")
    out = torch.empty((n, h, w), dtype=torch.int64, device=dev)
    if out.numel():
        lib = _lib.load()
        _lib.check(lib.sm_regress_argext(_ptr(vol), _ptr(out), code, n, d, h, w, mode,
                                         _lib.strides_arg(vol), _stream(dev)), "sm_regress_argext")
    return out


def hard_argmin(volume):
    """First index of the minimum over D -> (N,H,W) int64 (ties -> lowest d, NaN wins)."""
    if _traced():
        return _ops().hard_argmin(volume)
    return _argext(volume, _lib.SM_ARGMIN, "hard_argmin")


def hard_argmax(volume):
    """First index of the maximum over D -> (N,H,W) int64 (ties -> lowest d, NaN wins)."""
    if _traced():
        return _ops().hard_argmax(volume)
    return _argext(volume, _lib.SM_ARGMAX, "hard_argmax")


# ------------------------------------------------------------------------------ §8f-4 warp
def warp_by_flow_map(image, flow):
    """Warp ``image`` (N,C,Hi,Wi) by a disparity / flow map ``flow`` (N,1|2,H,W) -> (N,C,H,W).

    Mirrors ``warp_by_flow_map`` (tools/warp.py:5-42, model/mobile_stereo_net_v2.py:59-96,
    _v3.py:60-97): grid (x - fx, y - fy) normalised by (w - 1, h - 1), bilinear grid_sample with
    zero padding and align_corners=False, evaluated by ONE HIP kernel (csrc/warp.hip) in fp32;
    the same AssertionError as the reference for a flow with 3+ channels.

    Dtypes: float32 image and flow as they are.  fp16 / bf16 are read as fp32 and sampled in
    fp32: under torch autocast (grid_sample is an autocast fp32 op, so the reference's RefineNet
    warps an fp16 v3 feature map by an fp32 disparity and gets fp32) the output is fp32; without
    autocast image and flow must share one dtype (as grid_sample requires) and the fp32 result is
    rounded once to it.
    """
    if not isinstance(image, torch.Tensor) or not isinstance(flow, torch.Tensor):
        raise TypeError("warp_by_flow_map: image and flow must be tensors")
    if _traced():
        return _ops().warp_by_flow_map(image, flow, _autocast_fp32(image, flow))
    if flow.dim() != 4:
        raise ValueError(f"warp_by_flow_map: expected a 4-D flow map, got {tuple(flow.shape)}")
    n, c, h, w = flow.shape
    assert c == 1 or c == 2, f"invalid flow map dimension 1 or 2 ({c})!"  # tools/warp.py:18
    if image.dim() != 4:
        raise RuntimeError(f"warp_by_flow_map: expected a 4-D image, got {tuple(image.shape)}")
    if image.shape[0] != n:
        raise RuntimeError(f"warp_by_flow_map: image batch {image.shape[0]} != flow batch {n}")
    for t in (image, flow):
        if t.dtype not in _WARP_DTYPES:
            raise TypeError(f"warp_by_flow_map: unsupported dtype {t.dtype}; expected float32, "
                            "float16 or bfloat16")
    dev = _device_check(image, flow)
    if _autocast_fp32(image, flow):
        odt = torch.float32
    elif image.dtype != flow.dtype:
        raise RuntimeError(f"warp_by_flow_map: image ({image.dtype}) and flow ({flow.dtype}) must "
                           "have the same dtype outside autocast (grid_sample's rule)")
    else:
        odt = image.dtype
    # reduced-precision inputs are widened once on the device (exact); the kernel samples fp32
    image = image.float() if image.dtype != torch.float32 else image
    flow = flow.float() if flow.dtype != torch.float32 else flow
    image = _stride_ok(_rows_contiguous(image))
    flow = _stride_ok(_rows_contiguous(flow))
    N, C, Hi, Wi = image.shape
    out = torch.empty((N, C, h, w), dtype=torch.float32, device=dev)
    if out.numel():
        lib = _lib.load()
        # two-channel flows sample a channel-last copy of the image (csrc/warp.hip)
        nws = int(lib.sm_warp_by_flow_workspace_bytes(N, C, Hi, Wi, c))
        ws = torch.empty(nws, dtype=torch.uint8, device=dev) if nws > 0 else None
        _lib.check(lib.sm_warp_by_flow_ws(_ptr(image), _ptr(flow), _ptr(out), _lib.SM_F32, N, C, Hi,
                                          Wi, h, w, c, _lib.strides_arg(image),
                                          _lib.strides_arg(flow), _ptr(ws) if ws is not None else None,
                                          nws, _stream(dev)), "sm_warp_by_flow_ws")
    return out if odt == torch.float32 else out.to(odt)
