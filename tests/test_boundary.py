"""CPU-side tests of the drop-in boundary: the C ABI library loads and exports every symbol
declared in include/stereocv.h, host-side validation mirrors the reference's error
behaviour, and the product path refuses to run on the CPU (no fallback)."""
import ctypes
import os
import re

import pytest
import torch

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "stereocv.h")


def declared_symbols():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const char\*|int64_t|int)\s+(sm_[a-z0-9_]+)\s*\(", src, re.M)))


def test_header_declares_the_abi():
    syms = declared_symbols()
    for s in ("sm_cv_inner_product", "sm_cv_groupwise", "sm_cv_concat", "sm_cv_interweave",
              "sm_cv_interweave_shifted", "sm_cv_diff", "sm_cv_correlation_mean",
              "sm_regress_softargmin", "sm_regress_argext", "sm_last_error", "sm_version"):
        assert s in syms


def test_library_loads_and_exports_every_declared_symbol():
    from realtime_stereo_matcher_amd import _lib

    lib = _lib.load()
    for s in declared_symbols():
        assert hasattr(lib, s), f"libstereocv.so does not export {s}"
        assert s in _lib.SIGNATURES, f"_lib.SIGNATURES lacks {s}"
    assert lib.sm_version() >= 100
    # the binding table matches the header one-for-one
    assert sorted(_lib.SIGNATURES) == declared_symbols()


def test_library_is_gfx950_code_object():
    from realtime_stereo_matcher_amd import _lib

    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_error_path_without_gpu_work():
    """Invalid arguments are rejected on the host before any launch (no device needed)."""
    from realtime_stereo_matcher_amd import _lib

    lib = _lib.load()
    bad_strides = (ctypes.c_int64 * 4)(10, 5, 2, 2)  # W stride != 1
    rc = lib.sm_cv_inner_product(1, 1, 1, _lib.SM_F32, 1, 2, 3, 4, 5, bad_strides, None, None)
    assert rc == _lib.SM_EINVAL
    assert b"W stride" in lib.sm_last_error()
    rc = lib.sm_cv_groupwise(1, 1, 1, _lib.SM_F32, 1, 16, 2, 8, 4, 3, None, None, None)
    assert rc == _lib.SM_EINVAL and b"C % G" in lib.sm_last_error()
    rc = lib.sm_cv_inner_product_softargmin(1, 1, 1, 1, _lib.SM_F32, 1, 2, 3, 4, 5, None, None, 8,
                                            None)
    assert rc == _lib.SM_EINVAL and b"mode" in lib.sm_last_error()
    rc = lib.sm_cv_concat(1, 1, 1, 7, 1, 2, 3, 4, 5, None, None, None)
    assert rc == _lib.SM_EDTYPE
    rc = lib.sm_regress_argext(1, 1, _lib.SM_F32, 1, 4, 2, 2, 9, None, None)
    assert rc == _lib.SM_EINVAL
    # empty problems are a no-op success
    assert lib.sm_cv_inner_product(None, None, None, _lib.SM_F32, 0, 2, 3, 4, 5, None, None, None) == 0
    lib.sm_cv_diff(None, None, None, _lib.SM_F32, 1, 2, 3, 0, 5, None, None, None)


def test_reference_module_surface():
    from realtime_stereo_matcher_amd.cost_volume import (TorchConcatenateCost, TorchGroupwiseCost,
                                                         TorchInnerProductCost, TorchInterweaveCost)
    from realtime_stereo_matcher_amd.model import mobile_disp_net_c, mobile_stereo_net, mobile_stereo_net_v4

    m = TorchInnerProductCost(24)
    assert m.max_disparity == 24 and isinstance(m, torch.nn.Module)
    assert str(m) == "TorchInnerProductCost | aijk,aijh->ajkh"
    assert str(TorchInterweaveCost()) == "TorchInterweaveCost"
    g = TorchGroupwiseCost(8, 48)
    assert (g.n_groups, g.max_disparity) == (8, 48)
    assert TorchConcatenateCost(12).max_disparity == 12
    for fn in (mobile_stereo_net.make_cost_volume, mobile_disp_net_c.make_correlation_volume,
               mobile_disp_net_c.disparity_regression, mobile_stereo_net_v4.disparity_regression,
               mobile_stereo_net_v4.interweave_tensors):
        assert callable(fn)


def test_cpu_tensors_fail_loudly():
    from realtime_stereo_matcher_amd.cost_volume import TorchInnerProductCost
    from realtime_stereo_matcher_amd import functional as F

    l = torch.randn(1, 4, 2, 8)
    with pytest.raises(RuntimeError, match="HIP devices only"):
        TorchInnerProductCost(3)(l, l)
    with pytest.raises(RuntimeError, match="HIP devices only"):
        F.soft_argmin(torch.randn(1, 4, 2, 2))


def test_reference_error_conventions(manifest):
    from realtime_stereo_matcher_amd.cost_volume import TorchGroupwiseCost, TorchInnerProductCost
    from realtime_stereo_matcher_amd.model import mobile_disp_net_c

    with pytest.raises(AssertionError) as e:
        TorchGroupwiseCost(3, 4)(torch.zeros(1, 16, 2, 8), torch.zeros(1, 16, 2, 8))
    assert str(e.value) == manifest["groupwise_assert_message_c16_g3"]
    with pytest.raises(AssertionError) as e:
        mobile_disp_net_c.disparity_regression(torch.zeros(1, 5, 2, 2), 4)
    assert str(e.value) == manifest["softargmin_assert_message_d5_vs_4"]
    with pytest.raises(AssertionError) as e:
        mobile_disp_net_c.disparity_regression(torch.zeros(5, 2, 2), 5)
    assert str(e.value) == manifest["softargmin_assert_message_ndim3"]
    assert manifest["shape_mismatch_raises"] == "RuntimeError"
    with pytest.raises(RuntimeError, match="shape mismatch"):
        TorchInnerProductCost(3)(torch.zeros(1, 4, 2, 8), torch.zeros(1, 5, 2, 8))
    with pytest.raises(TypeError):  # integer features: no floating dtype the engine takes
        TorchInnerProductCost(3)(torch.zeros(1, 4, 2, 8, dtype=torch.int32),
                                 torch.zeros(1, 4, 2, 8, dtype=torch.int32))
    # float64 is accepted (round 6) and, on the CPU, refused as any CPU tensor is
    with pytest.raises(RuntimeError, match="HIP devices only"):
        TorchInnerProductCost(3)(torch.zeros(1, 4, 2, 8, dtype=torch.float64),
                                 torch.zeros(1, 4, 2, 8, dtype=torch.float64))


def test_product_package_never_imports_oracle():
    pkg = os.path.join(ROOT, "realtime_stereo_matcher_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith(".py"):
                src = open(os.path.join(dirpath, f)).read()
                assert "oracle" not in re.sub(r'""".*?"""', "", src, flags=re.S), f


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    """No CPU fallback: without the shared object every operator raises ImportError."""
    from realtime_stereo_matcher_amd import _lib

    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "libstereocv.so"))
    with pytest.raises(ImportError, match="no CPU fallback|There is no CPU fallback"):
        _lib.load()
