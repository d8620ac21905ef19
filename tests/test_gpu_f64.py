"""float64 features and volumes (VERDICT r05 "missing 3"): the reference's operators take any
floating dtype and torch computes an fp64 input in fp64 (cost_volume/*.py, model/*.py).  The engine
runs them in fp64 (csrc/f64.hip; the copy volumes as 8-byte elements in csrc/cv_copy.hip).

Pinned against the reference's own fp64 outputs (tests/golden/gen_f64_golden.py): sums within
1e-12 of sum_c |L R| (fp64 summation order), copies and argmax bit-exact, the groupwise float32
volume within one float32 ulp (the fp64 mean rounded once), the regressions within 1e-12.
"""
import json
import os

import numpy as np
import pytest
import torch

from oracle import stereo_oracle as O

pytestmark = pytest.mark.gpu
GD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _cases():
    with open(os.path.join(GD, "f64_manifest.json")) as f:
        return json.load(f)["cases"]


def _abs_norm(l, r, D):
    return O._dot_volume(np.abs(l), np.abs(r), D)


@pytest.mark.parametrize("rec", _cases(), ids=[c["name"] for c in _cases()])
def test_f64_golden(rec):
    from realtime_stereo_matcher_amd import functional as F

    a = np.load(os.path.join(GD, rec["file"]))
    p = rec["params"]
    g = {k: torch.from_numpy(a[k]).cuda() for k in a.files if k != "out"}
    want = a["out"]
    op = rec["op"]
    if op == "inner_product":
        got = F.inner_product_volume(g["left"], g["right"], p["max_disparity"])
        bound = 1e-12 * (_abs_norm(a["left"], a["right"], p["max_disparity"]) + 1)
    elif op == "correlation":
        got = F.correlation_volume(g["left"], g["right"], p["max_disp"])
        bound = 1e-12 * (_abs_norm(a["left"], a["right"], p["max_disp"]) / a["left"].shape[1] + 1)
    elif op == "groupwise":
        got = F.groupwise_volume(g["left"], g["right"], p["n_groups"], p["max_disparity"])
        assert got.dtype == torch.float32
        np.testing.assert_allclose(got.cpu().numpy(), want, rtol=2 ** -23, atol=1e-30)
        return
    elif op in ("concat", "interweave", "diff_volume"):
        got = {"concat": lambda: F.concat_volume(g["left"], g["right"], p["max_disparity"]),
               "interweave": lambda: F.interweave(g["left"], g["right"]),
               "diff_volume": lambda: F.difference_volume(g["left"], g["right"], p["max_disp"])}[op]()
        assert got.dtype == torch.float64
        np.testing.assert_array_equal(got.cpu().numpy(), want)
        return
    elif op == "softargmin":
        got = F.soft_argmin(g["volume"])
        bound = 1e-12
    elif op == "regression_presoftmax":
        got = F.regression_presoftmax(g["volume"])
        bound = 1e-12
    elif op == "argmax":
        got = F.hard_argmax(g["volume"])
        np.testing.assert_array_equal(got.cpu().numpy(), want)
        return
    else:
        raise AssertionError(op)
    assert got.dtype == torch.float64
    err = np.abs(got.cpu().numpy() - want)
    assert (err <= bound).all(), float(err.max())


def test_f64_sweep_strided_fused_and_specials():
    """Oracle sweep (fp64 oracle sums): a strided view, D > W, the mean over zero channels
    (NaN, as torch), the fused call (two kernels: the fp64 volume, then the fp64 soft-argmin;
    without the volume it is allocated for a moment), argmin with NaN and ties."""
    from realtime_stereo_matcher_amd import functional as F

    rng = np.random.default_rng(9)
    big = rng.standard_normal((2, 24, 6, 70))
    l, r = big[:, ::2], big[:, 1::2]  # channel-strided views
    L, R = torch.from_numpy(big).cuda()[:, ::2], torch.from_numpy(big).cuda()[:, 1::2]
    for D in (1, 30, 90):  # D > W for the last
        got = F.inner_product_volume(L, R, D).cpu().numpy()
        want = O._dot_volume(l, r, D)
        assert (np.abs(got - want) <= 1e-12 * (_abs_norm(l, r, D) + 1)).all()
    vol, disp = F.inner_product_soft_argmin(L, R, 40)
    assert vol.dtype == torch.float64 and disp.dtype == torch.float64
    v = O._dot_volume(l, r, 40)
    q = np.exp(v - v.max(axis=1, keepdims=True))
    ref = (q * np.arange(40).reshape(1, -1, 1, 1)).sum(axis=1, keepdims=True) / q.sum(axis=1, keepdims=True)
    assert np.abs(disp.cpu().numpy() - ref).max() <= 1e-9
    none, disp2 = F.inner_product_soft_argmin(L, R, 40, keep_volume=False)
    assert none is None and torch.equal(disp2, disp)
    z = torch.zeros(1, 0, 2, 8, dtype=torch.float64, device="cuda")
    assert torch.isnan(F.correlation_volume(z, z, 3)[:, :, :, 3:]).all()  # 0 / 0, as torch
    cv = torch.from_numpy(rng.integers(-2, 3, (1, 9, 3, 5)).astype(np.float64)).cuda()
    cv[0, 4, 1, 2] = float("nan")
    got = F.hard_argmin(cv).cpu().numpy()
    np.testing.assert_array_equal(got, torch.argmin(cv.cpu(), dim=1).numpy())
