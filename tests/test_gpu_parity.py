"""GPU parity of the HIP kernels (through the C ABI) against the golden vectors recorded from
the reference and against the CPU oracle (oracle/stereo_oracle.py).

Tolerances (north star, BASELINE.json): fp32 volumes / regression within 1e-4 absolute;
copy volumes (concat, interweave, difference) and argmin/argmax indices bit-exact.
"""
import numpy as np
import pytest
import torch

from conftest import cases, load_case
from oracle import stereo_oracle as O

pytestmark = pytest.mark.gpu

TOL = 1e-4
TDT = {"f32": torch.float32, "f16": torch.float16, "bf16": torch.bfloat16}


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def dev(a, dt="f32"):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).to("cuda").to(TDT[dt])


def host(t):
    return t.float().cpu().numpy() if t.dtype != torch.int64 else t.cpu().numpy()


def _ids(cs):
    return [c["name"] for c in cs]


# =============================================================================== golden vectors
@pytest.mark.parametrize("algo", ["auto", "h2", "h2db", "rs", "sl", "f32", "valu"])
@pytest.mark.parametrize("rec", cases("inner_product"), ids=_ids(cases("inner_product")))
def test_golden_inner_product(rec, algo):
    from realtime_stereo_matcher_amd.cost_volume import TorchInnerProductCost

    a = load_case(rec)
    dt = rec["dtype"]
    D = rec["params"]["max_disparity"]
    L, R = dev(a["left"], dt), dev(a["right"], dt)
    if "noncontig" in rec["name"]:
        L = L.transpose(2, 3).contiguous().transpose(2, 3)  # W stride != 1 -> wrapper re-lays rows
    out = TorchInnerProductCost(D, algo=algo)(L, R)
    assert out.shape == a["out"].shape and out.dtype == TDT[dt] and out.device == L.device
    got = host(out)
    if rec.get("exact"):
        np.testing.assert_array_equal(got, a["out"])
    elif dt == "f32":
        np.testing.assert_allclose(got, a["out"], atol=TOL, rtol=0)
    else:
        # fp32 accumulation of exact products vs torch's per-product rounding: compare with
        # the exact-product oracle to one output ulp, and with the literal golden loosely.
        ref = O.inner_product(a["left"], a["right"], D, out_dtype=dt).astype(np.float32)
        ulp = 2.0 ** -10 if dt == "f16" else 2.0 ** -7
        np.testing.assert_allclose(got, ref, rtol=ulp, atol=1e-3)
        np.testing.assert_allclose(got, a["out"], rtol=4 * ulp, atol=4e-2)


@pytest.mark.parametrize("rec", cases("correlation"), ids=_ids(cases("correlation")))
def test_golden_correlation(rec):
    from realtime_stereo_matcher_amd.model.mobile_disp_net_c import make_correlation_volume

    a = load_case(rec)
    out = make_correlation_volume(dev(a["left"]), dev(a["right"]), rec["params"]["max_disp"])
    np.testing.assert_allclose(host(out), a["out"], atol=TOL, rtol=0)


@pytest.mark.parametrize("rec", cases("groupwise"), ids=_ids(cases("groupwise")))
def test_golden_groupwise(rec):
    from realtime_stereo_matcher_amd.cost_volume import TorchGroupwiseCost

    a = load_case(rec)
    p = rec["params"]
    dt = rec["dtype"]
    out = TorchGroupwiseCost(p["n_groups"], p["max_disparity"])(dev(a["left"], dt), dev(a["right"], dt))
    assert out.dtype == torch.float32 and out.shape == a["out"].shape
    got = host(out)
    if dt == "f32":
        np.testing.assert_allclose(got, a["out"], atol=TOL, rtol=0)
    else:
        # parity bar: the fp32 oracle on the same bf16-representable inputs
        ref = O.groupwise(a["left"], a["right"], p["n_groups"], p["max_disparity"])
        np.testing.assert_allclose(got, ref, atol=TOL, rtol=0)
        # the reference rounds every product and the mean to bf16 (groupwise.py:21 in bf16):
        # |exact - literal| <= 2^-9 * (mean_c |L*R| + |mean|) per element; allow 2x that.
        scale = O.groupwise(np.abs(a["left"]), np.abs(a["right"]), p["n_groups"], p["max_disparity"])
        bound = 2.0 ** -8 * (scale + np.abs(got)) + 1e-6
        assert np.all(np.abs(got - a["out"]) <= bound)


@pytest.mark.parametrize("rec", cases("concat"), ids=_ids(cases("concat")))
def test_golden_concat(rec):
    from realtime_stereo_matcher_amd.cost_volume import TorchConcatenateCost

    a = load_case(rec)
    dt = rec["dtype"]
    out = TorchConcatenateCost(rec["params"]["max_disparity"])(dev(a["left"], dt), dev(a["right"], dt))
    np.testing.assert_array_equal(host(out), a["out"].astype(np.float32))


@pytest.mark.parametrize("rec", cases("interweave"), ids=_ids(cases("interweave")))
def test_golden_interweave(rec):
    from realtime_stereo_matcher_amd.cost_volume import TorchInterweaveCost
    from realtime_stereo_matcher_amd.model.mobile_stereo_net_v4 import interweave_tensors

    a = load_case(rec)
    dt = rec["dtype"]
    L, R = dev(a["left"], dt), dev(a["right"], dt)
    np.testing.assert_array_equal(host(TorchInterweaveCost()(L, R)), a["out"].astype(np.float32))
    np.testing.assert_array_equal(host(interweave_tensors(L, R)), a["out"].astype(np.float32))


@pytest.mark.parametrize("rec", cases("interweave_shifted"), ids=_ids(cases("interweave_shifted")))
def test_golden_interweave_shifted(rec):
    from realtime_stereo_matcher_amd.model.mobile_stereo_net_v4 import interweave_volume

    a = load_case(rec)
    dt = rec["dtype"]
    out = interweave_volume(dev(a["left"], dt), dev(a["right"], dt), rec["params"]["max_disparity"])
    np.testing.assert_array_equal(host(out), a["out"].astype(np.float32))


@pytest.mark.parametrize("rec", cases("diff_volume"), ids=_ids(cases("diff_volume")))
def test_golden_diff_volume(rec):
    from realtime_stereo_matcher_amd.model.mobile_stereo_net import make_cost_volume

    a = load_case(rec)
    dt = rec["dtype"]
    out = make_cost_volume(dev(a["left"], dt), dev(a["right"], dt), rec["params"]["max_disp"])
    np.testing.assert_array_equal(host(out), a["out"].astype(np.float32))


@pytest.mark.parametrize("rec", cases("softargmin"), ids=_ids(cases("softargmin")))
def test_golden_softargmin(rec):
    from realtime_stereo_matcher_amd.model.mobile_disp_net_c import disparity_regression
    from realtime_stereo_matcher_amd.model.mobile_stereo_net import soft_argmin_regression

    a = load_case(rec)
    v = dev(a["volume"])
    for out in (disparity_regression(v, rec["params"]["max_disp"]), soft_argmin_regression(v)):
        assert out.shape == a["out"].shape
        np.testing.assert_allclose(host(out), a["out"], atol=TOL, rtol=0)
        np.testing.assert_allclose(host(out), O.softargmin(a["volume"]), atol=2e-5, rtol=0)


@pytest.mark.parametrize("rec", cases("regression_presoftmax"), ids=_ids(cases("regression_presoftmax")))
def test_golden_regression_presoftmax(rec):
    from realtime_stereo_matcher_amd.model.mobile_stereo_net_v4 import disparity_regression

    a = load_case(rec)
    out = disparity_regression(dev(a["volume"]), rec["params"]["maxdisp"])
    assert out.shape == a["out"].shape
    np.testing.assert_allclose(host(out), a["out"], atol=TOL, rtol=0)


@pytest.mark.parametrize("rec", cases("argext"), ids=_ids(cases("argext")))
def test_golden_argext(rec):
    from realtime_stereo_matcher_amd import functional as F
    from realtime_stereo_matcher_amd.cost_volume import TorchInnerProductCost

    a = load_case(rec)
    fn = F.hard_argmax if rec["params"]["mode"] == "max" else F.hard_argmin
    np.testing.assert_array_equal(host(fn(dev(a["volume"]))), a["out"])
    if "left" in a:  # end to end: integer features -> exact volume -> bit-exact argmax
        for algo in ("auto", "h2", "h2db", "rs", "sl", "f32", "valu"):
            vol = TorchInnerProductCost(rec["params"]["max_disparity"], algo=algo)(dev(a["left"]), dev(a["right"]))
            np.testing.assert_array_equal(host(vol), a["volume"])
            np.testing.assert_array_equal(host(F.hard_argmax(vol)), a["out"])


# =============================================================================== oracle sweeps
SHAPES = [  # (N, C, H, W, D)
    (1, 1, 1, 1, 1), (1, 3, 2, 7, 5), (2, 17, 3, 65, 24), (1, 64, 2, 200, 192), (1, 16, 3, 130, 256),
    (1, 32, 2, 100, 300), (1, 8, 2, 64, 64), (1, 5, 1, 33, 0), (3, 64, 1, 97, 65), (1, 128, 2, 70, 48),
    # W % 4 == 0 shapes for the 16-B staging paths: channel tails, partial bands, D passes, W < 128
    (2, 20, 3, 260, 100), (1, 48, 2, 132, 33), (1, 16, 1, 1000, 256), (1, 7, 2, 36, 40),
    (1, 64, 2, 960, 192), (1, 33, 2, 512, 31),
    # fp32 rows of width W % 4 != 0 on the band kernel: misaligned 16-B loads / stores, the
    # row-end group loaded from W - 4, full tiles (plain stores) and a partial last quad
    (1, 64, 2, 958, 192), (2, 24, 2, 257, 100), (1, 64, 1, 957, 64),
]


def _feats(seed, shape, kind="normal"):
    rng = np.random.default_rng(seed)
    if kind == "int":
        return (rng.integers(-8, 9, size=shape).astype(np.float32),
                rng.integers(-8, 9, size=shape).astype(np.float32))
    return rng.standard_normal(shape, dtype=np.float32), rng.standard_normal(shape, dtype=np.float32)


@pytest.mark.parametrize("algo", ["auto", "h2", "h2db", "rs", "sl", "f32", "valu"])
@pytest.mark.parametrize("shape", SHAPES, ids=[str(s) for s in SHAPES])
def test_inner_product_vs_oracle(shape, algo):
    from realtime_stereo_matcher_amd import functional as F

    n, c, h, w, D = shape
    l, r = _feats(hash(shape) % 1000, (n, c, h, w))
    got = host(F.inner_product_volume(dev(l), dev(r), D, algo=algo))
    np.testing.assert_allclose(got, O.inner_product(l, r, D), atol=TOL, rtol=0)
    li, ri = _feats(7, (n, c, h, w), "int")
    np.testing.assert_array_equal(host(F.inner_product_volume(dev(li), dev(ri), D, algo=algo)),
                                  O.inner_product(li, ri, D))


def _cell_norm(l, r, D):
    """sum_c |L||R(x-d)| per volume cell: the magnitude an fp32 sum's rounding scales with."""
    return O.inner_product(np.abs(l), np.abs(r), D)


@pytest.mark.parametrize("algo", ["auto", "h2", "h2db", "rs", "sl", "f32"])
@pytest.mark.parametrize("scale", [1e-15, 1e-6, 1e-3, 1e3, 1e6, 1e15])
def test_inner_product_feature_scales(scale, algo):
    """Uniformly tiny or huge features: the fp16 split rescales each segment by a power of two
    (a recomputed first segment, then the carried scale), so accuracy is relative, as in fp32."""
    from realtime_stereo_matcher_amd import functional as F

    l, r = _feats(21, (1, 64, 3, 512))
    l, r = (l * scale).astype(np.float32), (r * scale).astype(np.float32)
    got = host(F.inner_product_volume(dev(l), dev(r), 192, algo=algo))
    err = np.abs(got - O.inner_product(l, r, 192))
    assert (err <= 1e-5 * _cell_norm(l, r, 192) + 1e-37).all(), float((err / (_cell_norm(l, r, 192) + 1e-37)).max())
    corr = host(F.correlation_volume(dev(l), dev(r), 192))
    err = np.abs(corr - O.correlation_mean(l, r, 192))
    assert (err <= 1e-5 * _cell_norm(l, r, 192) / 64 + 1e-37).all()


@pytest.mark.parametrize("algo", ["auto", "h2", "h2db", "rs", "sl"])
def test_inner_product_mixed_scales(algo):
    """Feature scale changing from row to row (10^-8 .. 10^8, L and R independently) and within
    a row (10^-2 .. 10^2 per pixel): every segment must land in a safe fp16 range."""
    from realtime_stereo_matcher_amd import functional as F

    rng = np.random.default_rng(5)
    n, c, h, w, D = 2, 48, 6, 640, 160
    l, r = _feats(22, (n, c, h, w))
    l = (l * 10.0 ** rng.uniform(-8, 8, (n, 1, h, 1)) * 10.0 ** rng.uniform(-2, 2, (n, 1, h, w))).astype(np.float32)
    r = (r * 10.0 ** rng.uniform(-8, 8, (n, 1, h, 1)) * 10.0 ** rng.uniform(-2, 2, (n, 1, h, w))).astype(np.float32)
    got = host(F.inner_product_volume(dev(l), dev(r), D, algo=algo))
    err = np.abs(got - O.inner_product(l, r, D))
    bound = 1e-5 * _cell_norm(l, r, D) + 1e-30
    assert (err <= bound).all(), float((err / bound).max())


@pytest.mark.parametrize("dt", ["f16", "bf16"])
@pytest.mark.parametrize("shape", [(2, 20, 3, 260, 100), (1, 64, 2, 960, 192), (1, 16, 2, 512, 256),
                                   (1, 33, 2, 128, 31)], ids=str)
def test_inner_product_half_vs_oracle(shape, dt):
    """fp16 / bf16 features through the default (two-plane band) kernel: fp32 accumulation of
    exact products, rounded once to the output dtype (one output ulp of the exact oracle)."""
    from realtime_stereo_matcher_amd import functional as F

    n, c, h, w, D = shape
    l, r = _feats(31, (n, c, h, w))
    l, r = O.round_to_dtype(l, dt).astype(np.float32), O.round_to_dtype(r, dt).astype(np.float32)
    got = F.inner_product_volume(dev(l, dt), dev(r, dt), D)
    assert got.dtype == TDT[dt]
    ulp = 2.0 ** -10 if dt == "f16" else 2.0 ** -7
    ref = O.inner_product(l, r, D, out_dtype=dt).astype(np.float32)
    np.testing.assert_allclose(host(got), ref, rtol=ulp, atol=1e-3)
    corr = F.correlation_volume(dev(l, dt), dev(r, dt), D)
    np.testing.assert_allclose(host(corr), O.correlation_mean(l, r, D, out_dtype=dt).astype(np.float32),
                               rtol=ulp, atol=1e-4)


@pytest.mark.parametrize("algo,dt", [("auto", "f32"), ("h2", "f32"), ("h2db", "f32"), ("rs", "f32"), ("sl", "f32"), ("f32", "f32"), ("valu", "f32"),
                                     ("auto", "f16"), ("auto", "bf16")])
def test_inner_product_nonfinite(algo, dt):
    """+-inf and NaN features give the reference's inf / NaN cells, and x < d cells stay 0."""
    from realtime_stereo_matcher_amd import functional as F

    l, r = _feats(23, (1, 16, 3, 256))
    l, r = O.round_to_dtype(l, dt).astype(np.float32), O.round_to_dtype(r, dt).astype(np.float32)
    l[0, 5, 0, 130] = np.inf
    l[0, 0, 1, 7] = -np.inf
    r[0, 3, 1, 100] = np.nan
    r[0, 9, 2, 3] = np.inf
    D = 64
    got = host(F.inner_product_volume(dev(l, dt), dev(r, dt), D, algo=algo))
    want = O.inner_product(l, r, D, out_dtype=dt).astype(np.float32)
    np.testing.assert_array_equal(np.isnan(got), np.isnan(want))
    np.testing.assert_array_equal(np.isposinf(got), np.isposinf(want))
    np.testing.assert_array_equal(np.isneginf(got), np.isneginf(want))
    fin = np.isfinite(want)
    ulp = {"f32": 0.0, "f16": 2.0 ** -10, "bf16": 2.0 ** -7}[dt]
    np.testing.assert_allclose(got[fin], want[fin], atol=TOL if dt == "f32" else 1e-3, rtol=ulp)


@pytest.mark.parametrize("shape", SHAPES, ids=[str(s) for s in SHAPES])
def test_correlation_and_groupwise_vs_oracle(shape):
    from realtime_stereo_matcher_amd import functional as F

    n, c, h, w, D = shape
    l, r = _feats(11, (n, c, h, w))
    np.testing.assert_allclose(host(F.correlation_volume(dev(l), dev(r), D)),
                               O.correlation_mean(l, r, D), atol=TOL, rtol=0)
    for G in {1, c} | ({c // 2} if c % 2 == 0 else set()):
        got = host(F.groupwise_volume(dev(l), dev(r), G, D))
        np.testing.assert_allclose(got, O.groupwise(l, r, G, D), atol=TOL, rtol=0)


@pytest.mark.parametrize("dt", ["f32", "f16", "bf16"])
@pytest.mark.parametrize("shape", [(1, 3, 2, 7, 5), (2, 5, 3, 33, 40), (1, 4, 2, 64, 64), (1, 6, 2, 19, 8)])
def test_copy_volumes_vs_oracle(shape, dt):
    from realtime_stereo_matcher_amd import functional as F

    n, c, h, w, D = shape
    l, r = _feats(3, (n, c, h, w))
    l, r = O.round_to_dtype(l, dt).astype(np.float32), O.round_to_dtype(r, dt).astype(np.float32)
    L, R = dev(l, dt), dev(r, dt)
    np.testing.assert_array_equal(host(F.concat_volume(L, R, D)), O.concatenate(l, r, D))
    np.testing.assert_array_equal(host(F.interweave(L, R)), O.interweave(l, r))
    np.testing.assert_array_equal(host(F.interweave_volume(L, R, D)), O.interweave_shifted(l, r, D))
    want = O.round_to_dtype(O.diff_volume(l, r, D), dt).astype(np.float32) if dt != "f32" else O.diff_volume(l, r, D)
    np.testing.assert_array_equal(host(F.difference_volume(L, R, D)), want)


def test_noncontiguous_inputs():
    """Strided (but row-contiguous) views go through the strides of the C ABI untouched."""
    from realtime_stereo_matcher_amd import functional as F

    l, r = _feats(5, (2, 24, 6, 40))
    L, R = dev(l), dev(r)
    Ls, Rs = L[:, ::2, 1::2], R[:, ::2, 1::2]  # channel and row strides
    ls, rs = l[:, ::2, 1::2], r[:, ::2, 1::2]
    np.testing.assert_allclose(host(F.inner_product_volume(Ls, Rs, 17)), O.inner_product(ls, rs, 17), atol=TOL)
    np.testing.assert_allclose(host(F.correlation_volume(Ls, Rs, 9)), O.correlation_mean(ls, rs, 9), atol=TOL)
    np.testing.assert_allclose(host(F.groupwise_volume(Ls, Rs, 3, 9)), O.groupwise(ls, rs, 3, 9), atol=TOL)
    np.testing.assert_array_equal(host(F.concat_volume(Ls, Rs, 7)), O.concatenate(ls, rs, 7))
    np.testing.assert_array_equal(host(F.interweave(Ls, Rs)), O.interweave(ls, rs))
    np.testing.assert_array_equal(host(F.difference_volume(Ls, Rs, 7)), O.diff_volume(ls, rs, 7))
    vol = dev(np.random.default_rng(1).standard_normal((2, 30, 5, 12), dtype=np.float32))
    vs = vol[:, :, ::2]
    np.testing.assert_allclose(host(F.soft_argmin(vs)), O.softargmin(host(vs)), atol=2e-5)
    np.testing.assert_array_equal(host(F.hard_argmin(vs)), O.argext(host(vs), "min"))


@pytest.mark.parametrize("shape", [(1, 192, 3, 257), (2, 24, 5, 7), (1, 1, 2, 3), (1, 300, 2, 64), (1, 48, 1, 1000)])
@pytest.mark.parametrize("scale", [1.0, 30.0])
def test_regression_vs_oracle(shape, scale):
    from realtime_stereo_matcher_amd import functional as F

    v = np.random.default_rng(9).standard_normal(shape, dtype=np.float32) * scale
    V = dev(v)
    np.testing.assert_allclose(host(F.soft_argmin(V, keepdim=False)), O.softargmin(v, keepdim=False), atol=2e-5, rtol=0)
    prob = torch.softmax(V, dim=1)
    np.testing.assert_allclose(host(F.regression_presoftmax(prob)),
                               O.regression_presoftmax(host(prob), shape[1]), atol=TOL, rtol=0)
    vi = np.round(v).astype(np.float32)  # ties
    for mode, fn in (("min", F.hard_argmin), ("max", F.hard_argmax)):
        np.testing.assert_array_equal(host(fn(dev(vi))), O.argext(vi, mode))


def test_regression_special_values():
    from realtime_stereo_matcher_amd import functional as F

    v = np.zeros((1, 20, 1, 6), np.float32)
    v[0, :, 0, 0] = -np.inf                      # all -inf column -> NaN (torch)
    v[0, 3, 0, 1] = np.nan                       # a NaN -> NaN; argmin/argmax pick it
    v[0, :10, 0, 2] = -np.inf                    # leading -inf chunk then finite values
    v[0, 5, 0, 3] = np.inf                       # +inf -> NaN in softmax
    v[0, 7, 0, 4] = 80.0                         # large spread
    t = torch.from_numpy(v)
    ref = torch.sum(torch.softmax(t.double(), 1) * torch.arange(20.).view(1, -1, 1, 1), 1).float().numpy()
    got = host(F.soft_argmin(dev(v), keepdim=False))
    np.testing.assert_allclose(got, ref, atol=2e-5, equal_nan=True)
    np.testing.assert_array_equal(host(F.hard_argmax(dev(v))), torch.argmax(t, 1).numpy())
    np.testing.assert_array_equal(host(F.hard_argmin(dev(v))), torch.argmin(t, 1).numpy())


@pytest.mark.parametrize("W", [8, 6])  # H*W % 4 == 0: the flat fp32 kernel; else the generic one
def test_regression_special_values_flat(W):
    """Special columns through the flat-plane fp32 soft-argmin (regress.hip), D = 37 so every
    disparity quarter ends in a partial chunk."""
    from realtime_stereo_matcher_amd import functional as F

    D = 37
    v = np.random.default_rng(4).standard_normal((2, D, 2, W)).astype(np.float32)
    v[0, :, 0, 0] = -np.inf                      # all -inf -> NaN
    v[0, :, 0, 1] = -np.inf
    v[0, 12, 0, 1] = np.nan                      # NaN inside an all -inf chunk -> NaN
    v[0, 3, 1, 1] = np.inf                       # +inf -> NaN
    v[0, 30, 1, 2] = np.inf
    v[0, 2, 1, 2] = -np.inf                      # +inf and -inf in one column -> NaN
    v[1, :20, 1, 3] = -np.inf                    # leading -inf quarters, finite tail
    v[1, 36, 0, 4] = 90.0                        # last disparity dominates
    v[1, :, 1, 5] = np.linspace(-200, 200, D)    # steep ramp, rescales every chunk
    t = torch.from_numpy(v)
    ref = torch.sum(torch.softmax(t.double(), 1) * torch.arange(float(D)).view(1, -1, 1, 1), 1).float().numpy()
    got = host(F.soft_argmin(dev(v), keepdim=False))
    np.testing.assert_allclose(got, ref, atol=2e-5, equal_nan=True)
    np.testing.assert_array_equal(np.isnan(got), np.isnan(ref))
    # hard argext on the same columns (flat fp32 kernel for W = 8): NaN wins, first index on ties
    vt = v.copy()
    vt[1, :, 0, 0] = 3.0                         # all tied -> 0
    vt[1, 10:, 0, 1] = 5.0                       # tie from d = 10 on
    np.testing.assert_array_equal(host(F.hard_argmax(dev(vt))), torch.argmax(torch.from_numpy(vt), 1).numpy())
    np.testing.assert_array_equal(host(F.hard_argmin(dev(vt))), torch.argmin(torch.from_numpy(vt), 1).numpy())


@pytest.mark.parametrize("hw", [(2, 8), (3, 5)])  # H*W % 4 == 0: the flat fp32 kernel; else generic
@pytest.mark.parametrize("D", [37, 48])
def test_regression_presoftmax_special_values(hw, D):
    """The v4 regression over already-softmaxed input (model/mobile_stereo_net_v4.py:10-14) on
    the flat one-wave kernel and its generic twin: inf * 0 at d = 0 gives NaN (torch), a NaN entry
    propagates, +inf elsewhere gives inf, D % 8 != 0 leaves a partial chunk -- against
    torch.sum(x * arange(D)) on the CPU, and flat vs generic agree."""
    from realtime_stereo_matcher_amd import functional as F

    H, W = hw
    x = np.random.default_rng(6).random((2, D, H, W)).astype(np.float32)
    x /= x.sum(1, keepdims=True)
    x[0, 0, 0, 0] = np.inf                       # inf * 0 -> NaN
    x[0, 5, 0, 1] = np.nan                       # NaN propagates
    x[1, D - 1, H - 1, W - 1] = np.inf           # inf * (D - 1) -> inf
    x[1, 3, 0, 2] = -np.inf
    x[1, 9, 0, 2] = np.inf                       # -inf and +inf -> NaN
    t = torch.from_numpy(x)
    ref = torch.sum(t * torch.arange(D, dtype=torch.float32).view(1, -1, 1, 1), 1).numpy()
    got = host(F.regression_presoftmax(dev(x)))
    np.testing.assert_array_equal(np.isnan(got), np.isnan(ref))
    np.testing.assert_array_equal(np.isinf(got), np.isinf(ref))
    fin = np.isfinite(ref)
    np.testing.assert_allclose(got[fin], ref[fin], atol=TOL, rtol=1e-6)
    # the same planes at a 4-byte (not 16-byte) aligned offset take the generic kernel
    big = torch.zeros(2 * D * H * W + 1, device="cuda")
    xs = big[1:].view(2, D, H, W)
    xs.copy_(dev(x))
    got2 = host(F.regression_presoftmax(xs))
    np.testing.assert_array_equal(np.isnan(got2), np.isnan(got))
    np.testing.assert_allclose(got2[fin], got[fin], atol=TOL, rtol=1e-6)


def test_zero_channels_and_empty():
    from realtime_stereo_matcher_amd import functional as F

    z = torch.zeros(1, 0, 2, 9, device="cuda")
    assert torch.equal(F.inner_product_volume(z, z, 4).cpu(), torch.zeros(1, 4, 2, 9))
    corr = F.correlation_volume(z, z, 4).cpu()  # mean over empty C = NaN where x >= d
    ref = torch.zeros(1, 4, 2, 9)
    for d in range(4):
        ref[:, d, :, d:] = float("nan")
    assert torch.equal(torch.isnan(corr), torch.isnan(ref))
    e = torch.zeros(0, 4, 2, 9, device="cuda")
    assert F.inner_product_volume(e, e, 3).shape == (0, 3, 2, 9)
    assert F.concat_volume(e, e, 3).shape == (0, 8, 2, 9, 3)


# =============================================================================== full-size configs
def _rows_check(full, fn_oracle, rows, atol, exact=False):
    for y in rows:
        want = fn_oracle(y)
        got = host(full(y))
        if exact:
            np.testing.assert_array_equal(got, want)
        else:
            np.testing.assert_allclose(got, want, atol=atol, rtol=0)


@pytest.mark.parametrize("algo", ["auto", "h2", "h2db", "rs", "sl", "f32", "valu"])
def test_cfg2_inner_product_full_size(algo):
    """BASELINE configs[1]: 1x64x540x960 fp32, D=192 -- every row depends only on the same
    row of L and R (inner_product.py:38-40), so rows sampled from the full-size launch are
    compared with the oracle on the same rows; plus the soft-argmin of the full volume."""
    from realtime_stereo_matcher_amd import functional as F

    g = torch.Generator(device="cuda").manual_seed(0)
    L = torch.randn(1, 64, 540, 960, device="cuda", generator=g)
    R = torch.randn(1, 64, 540, 960, device="cuda", generator=g)
    vol = F.inner_product_volume(L, R, 192, algo=algo)
    disp = F.soft_argmin(vol)
    torch.cuda.synchronize()
    from oracle.torch_port import soft_argmin_eager, sweep_dot_volume

    ln, rn = host(L), host(R)
    worst = worst_torch = 0.0
    mean_dev = []
    for y in (0, 1, 269, 538, 539):
        ref = O.inner_product(ln[:, :, y:y + 1], rn[:, :, y:y + 1], 192)
        got_v = host(vol[:, :, y:y + 1])
        np.testing.assert_allclose(got_v, ref, atol=TOL, rtol=0)
        # the regression kernel on this volume vs the fp64 regression of the same volume
        got_d = host(disp[:, :, y:y + 1])
        np.testing.assert_allclose(got_d, O.softargmin(got_v), atol=TOL, rtol=0)
        # end to end, per pixel: |disp - fp64 pipeline| against the same deviation of torch's
        # own fp32 pipeline (the reference's arithmetic) on these rows.  fp32-volume rounding is
        # amplified by sharp / bimodal softmaxes at a few pixels, for torch as for the kernel
        # (same amplification, different rounding).  Two bars, both written here:
        #   EPE level (north star "EPE identical within 1e-4"): the MEAN per-pixel |disp - fp64
        #     pipeline| over the sampled rows <= 1e-4 -- it bounds |EPE_kernel - EPE_exact| for
        #     ANY ground truth;
        #   per pixel (a relaxation of 1e-4, stated in DESIGN §4): max |disp - fp64 pipeline|
        #     <= max(1e-4, 2 x torch fp32's own per-pixel deviation on the same rows).
        exact = O.softargmin(ref).astype(np.float64)
        t32 = soft_argmin_eager(sweep_dot_volume(torch.from_numpy(ln[:, :, y:y + 1]),
                                                 torch.from_numpy(rn[:, :, y:y + 1]), 192))
        worst_torch = max(worst_torch, np.abs(t32.numpy().astype(np.float64) - exact).max())
        dd = np.abs(got_d.astype(np.float64) - exact)
        worst = max(worst, dd.max())
        mean_dev.append(dd.mean())
    mean_abs = float(np.mean(mean_dev))
    print(f"cfg2 {algo}: per-pixel |disp - fp64 pipeline|: max kernel {worst:.3g}, "
          f"torch fp32 {worst_torch:.3g}; mean kernel {mean_abs:.3g}")
    assert mean_abs <= TOL, mean_abs
    assert worst <= max(TOL, 2 * worst_torch), (worst, worst_torch)
    # x < d triangle is exactly zero everywhere
    tri = torch.arange(960, device="cuda")[None, :] < torch.arange(192, device="cuda")[:, None]
    assert not vol[0].permute(1, 0, 2)[:, tri].any()


def test_cfg3_groupwise_bf16_full_size():
    """BASELINE configs[2]: 1x256x540x960 bf16, G=8, D=192, fp32 (N,G,H,W,D) output."""
    from realtime_stereo_matcher_amd import functional as F

    g = torch.Generator(device="cuda").manual_seed(0)
    L = torch.randn(1, 256, 540, 960, device="cuda", generator=g).bfloat16()
    R = torch.randn(1, 256, 540, 960, device="cuda", generator=g).bfloat16()
    vol = F.groupwise_volume(L, R, 8, 192)
    assert vol.shape == (1, 8, 540, 960, 192) and vol.dtype == torch.float32
    ln, rn = host(L), host(R)
    for y in (0, 300, 539):
        ref = O.groupwise(ln[:, :, y:y + 1], rn[:, :, y:y + 1], 8, 192)
        np.testing.assert_allclose(host(vol[:, :, y:y + 1]), ref, atol=TOL, rtol=0)


def test_cfg4_correlation_full_res_pair():
    """BASELINE configs[3] per pair: 16x1080x1920 fp32, D=256 (mean over C)."""
    from realtime_stereo_matcher_amd import functional as F

    g = torch.Generator(device="cuda").manual_seed(0)
    L = torch.randn(1, 16, 1080, 1920, device="cuda", generator=g)
    R = torch.randn(1, 16, 1080, 1920, device="cuda", generator=g)
    vol = F.correlation_volume(L, R, 256)
    ln, rn = host(L), host(R)
    for y in (0, 777, 1079):
        ref = O.correlation_mean(ln[:, :, y:y + 1], rn[:, :, y:y + 1], 256)
        np.testing.assert_allclose(host(vol[:, :, y:y + 1]), ref, atol=TOL, rtol=0)


def test_cfg5_concat_interweave_fp16_full_size():
    """BASELINE configs[4]: 1x128x540x960 fp16, concat D=64 (17 GB) and interweave."""
    from realtime_stereo_matcher_amd import functional as F

    g = torch.Generator(device="cuda").manual_seed(0)
    L = torch.randn(1, 128, 540, 960, device="cuda", generator=g).half()
    R = torch.randn(1, 128, 540, 960, device="cuda", generator=g).half()
    iw = F.interweave(L, R)
    assert torch.equal(iw[:, 0::2], L) and torch.equal(iw[:, 1::2], R)
    del iw
    vol = F.concat_volume(L, R, 64)
    assert vol.shape == (1, 256, 540, 960, 64)
    ln, rn = host(L), host(R)
    for y in (0, 123, 539):
        ref = O.concatenate(ln[:, :, y:y + 1], rn[:, :, y:y + 1], 64)
        np.testing.assert_array_equal(host(vol[:, :, y:y + 1]), ref)
    # checksum of checksums: every d-slice of the left half sums to the shifted left plane
    for d in (0, 17, 63):
        assert torch.equal(vol[0, :128, :, d:, d], L[0, :, :, d:])
        assert torch.equal(vol[0, 128:, :, d:, d], R[0, :, :, :960 - d])
    del vol
    # the v4 shifted interweave at the full C = 128 (a 17 GB volume): every d slice
    sv = F.interweave_volume(L, R, 64)
    assert sv.shape == (1, 256, 64, 540, 960)
    for d in range(64):
        assert torch.equal(sv[0, 0::2, d, :, d:], L[0, :, :, d:])
        assert torch.equal(sv[0, 1::2, d, :, d:], R[0, :, :, :960 - d])
        assert not sv[0, :, d, :, :d].any()
    for y in (0, 539):
        np.testing.assert_array_equal(host(sv[:, :, :, y:y + 1]),
                                      O.interweave_shifted(ln[:, :, y:y + 1], rn[:, :, y:y + 1], 64))


# =============================================================================== band kernel: groupwise + fused
GW_SHAPES = [(1, 32, 3, 260, 100, 4), (2, 48, 2, 132, 33, 3), (1, 64, 2, 512, 192, 8),
             (1, 16, 2, 64, 256, 2), (1, 24, 2, 200, 40, 8), (1, 40, 2, 128, 7, 5)]


@pytest.mark.parametrize("dt", ["f32", "f16", "bf16"])
@pytest.mark.parametrize("shape", GW_SHAPES, ids=str)
def test_groupwise_band_vs_oracle(shape, dt):
    """The groupwise MFMA band kernel (D-innermost epilogue ring): fp32 (N,G,H,W,D) within 1e-4
    of the fp64 oracle on the same dtype-rounded features -- channel tails (C/G not a multiple
    of 16), two D passes, D % 4 != 0 (scalar d stores) and a partial last x tile."""
    from realtime_stereo_matcher_amd import functional as F

    n, c, h, w, D, G = shape
    l, r = _feats(51, (n, c, h, w))
    l, r = O.round_to_dtype(l, dt).astype(np.float32), O.round_to_dtype(r, dt).astype(np.float32)
    got = F.groupwise_volume(dev(l, dt), dev(r, dt), G, D)
    assert got.dtype == torch.float32 and got.shape == (n, G, h, w, D)
    np.testing.assert_allclose(host(got), O.groupwise(l, r, G, D), atol=TOL, rtol=0)


def test_groupwise_band_nonfinite():
    """+-inf / NaN in one group's channels give inf / NaN only in that group's cells."""
    from realtime_stereo_matcher_amd import functional as F

    l, r = _feats(52, (1, 32, 3, 256))
    l[0, 5, 0, 130] = np.inf   # group 0 (8 channels per group)
    r[0, 19, 1, 100] = np.nan  # group 2
    r[0, 30, 2, 3] = -np.inf   # group 3
    got = host(F.groupwise_volume(dev(l), dev(r), 4, 48))
    want = O.groupwise(l, r, 4, 48)
    np.testing.assert_array_equal(np.isnan(got), np.isnan(want))
    np.testing.assert_array_equal(np.isposinf(got), np.isposinf(want))
    np.testing.assert_array_equal(np.isneginf(got), np.isneginf(want))
    fin = np.isfinite(want)
    np.testing.assert_allclose(got[fin], want[fin], atol=TOL, rtol=0)


FUSED_SHAPES = [(1, 64, 3, 512, 192), (2, 20, 3, 260, 100), (1, 33, 2, 132, 31), (1, 16, 2, 64, 64),
                (1, 8, 3, 100, 24), (1, 7, 2, 36, 40), (1, 16, 2, 64, 256), (1, 5, 2, 33, 9),
                (1, 64, 2, 958, 192), (2, 20, 2, 259, 100),
                # C = 16 one channel step, both band geometries (the fused C = 16
                # instantiations of the sliding-window / role-split kernels), and more rows than
                # workgroups (the sliding window's row changes), C = 16 and 64
                (2, 16, 3, 260, 100), (1, 16, 2, 388, 192), (1, 16, 300, 196, 160),
                (2, 64, 150, 260, 192)]


@pytest.mark.parametrize("mean", [False, True])
@pytest.mark.parametrize("shape", FUSED_SHAPES, ids=str)
def test_fused_soft_argmin(shape, mean):
    """Volume + soft-argmin in one pass: the volume is bit-identical to the
    volume op's, the disparity is the fp64 soft-argmin of that volume within 1e-4, and the
    volume-free call returns the same disparity (D > 192: two kernels; fp32 rows of any width
    take the fused kernel)."""
    from realtime_stereo_matcher_amd import functional as F

    n, c, h, w, D = shape
    l, r = _feats(41, (n, c, h, w))
    L, R = dev(l), dev(r)
    vol, disp = F.inner_product_soft_argmin(L, R, D, mean=mean)
    ref = F.correlation_volume(L, R, D) if mean else F.inner_product_volume(L, R, D)
    assert torch.equal(vol, ref)
    assert disp.shape == (n, 1, h, w) and disp.dtype == torch.float32
    np.testing.assert_allclose(host(disp), O.softargmin(host(vol)), atol=TOL, rtol=0)
    none, disp2 = F.inner_product_soft_argmin(L, R, D, mean=mean, keep_volume=False)
    assert none is None
    if D <= 192:  # the same band-kernel fold, bit for bit
        assert torch.equal(disp2, disp)
    else:  # volume-free D > 192: per-pass states merged by a second kernel
        np.testing.assert_allclose(host(disp2), host(disp), atol=TOL, rtol=0)


@pytest.mark.parametrize("mean", [False, True])
@pytest.mark.parametrize("shape", [(1, 16, 2, 320, 256), (2, 24, 2, 257, 300), (1, 8, 3, 64, 200),
                                   (1, 16, 300, 260, 256), (2, 16, 3, 132, 200)], ids=str)
def test_fused_soft_argmin_multipass(shape, mean):
    """Volume-free fused pass for D > 192 (MobileDispNetC's D = 256): C = 16 takes the
    sliding-window kernel's two passes with the states merged in registers; other shapes per-pass
    partial softmax states in a workspace, merged by a second kernel.  The disparity is the fp64
    soft-argmin of the volume op's volume within 1e-4."""
    from realtime_stereo_matcher_amd import _lib
    from realtime_stereo_matcher_amd import functional as F

    n, c, h, w, D = shape
    assert _lib.load().sm_cv_inner_product_softargmin_workspace_bytes(n, h, w, D) > 0
    l, r = _feats(43, (n, c, h, w))
    L, R = dev(l), dev(r)
    none, disp = F.inner_product_soft_argmin(L, R, D, mean=mean, keep_volume=False)
    vol = F.correlation_volume(L, R, D) if mean else F.inner_product_volume(L, R, D)
    assert none is None and disp.shape == (n, 1, h, w)
    np.testing.assert_allclose(host(disp), O.softargmin(host(vol)), atol=TOL, rtol=0)
    # the same through the two-kernel path (volume kept)
    _, disp2 = F.inner_product_soft_argmin(L, R, D, mean=mean)
    np.testing.assert_allclose(host(disp), host(disp2), atol=TOL, rtol=0)


def test_cfg4_fused_volume_free_full_res():
    """BASELINE configs[3] shape (1x16x1080x1920, correlation D = 256) through the volume-free
    fused path (band_sl: two passes per segment, merged in registers): the disparity matches the two-kernel pipeline's (volume,
    then soft-argmin) within 1e-4 everywhere, and sampled rows match the fp64 soft-argmin of
    the volume."""
    from realtime_stereo_matcher_amd import functional as F

    g = torch.Generator(device="cuda").manual_seed(3)
    L = torch.randn(1, 16, 1080, 1920, device="cuda", generator=g)
    R = torch.randn(1, 16, 1080, 1920, device="cuda", generator=g)
    _, disp = F.inner_product_soft_argmin(L, R, 256, mean=True, keep_volume=False)
    vol = F.correlation_volume(L, R, 256)
    ref = F.soft_argmin(vol)
    assert (disp - ref.view_as(disp)).abs().max().item() <= TOL
    for y in (0, 540, 1079):
        np.testing.assert_allclose(host(disp[:, :, y:y + 1]), O.softargmin(host(vol[:, :, y:y + 1])),
                                   atol=TOL, rtol=0)


def test_fused_soft_argmin_nonfinite_and_empty():
    from realtime_stereo_matcher_amd import functional as F

    l, r = _feats(23, (1, 16, 3, 256))
    l[0, 5, 0, 130] = np.inf
    l[0, 0, 1, 7] = -np.inf
    r[0, 3, 1, 100] = np.nan
    r[0, 9, 2, 3] = np.inf
    vol, disp = F.inner_product_soft_argmin(dev(l), dev(r), 64)
    v = host(vol)
    np.testing.assert_array_equal(np.isnan(v), np.isnan(O.inner_product(l, r, 64)))
    np.testing.assert_allclose(host(disp), O.softargmin(v), atol=TOL, rtol=0, equal_nan=True)
    z = torch.zeros(1, 4, 2, 8, device="cuda")
    vol0, disp0 = F.inner_product_soft_argmin(z, z, 0)
    assert vol0.shape == (1, 0, 2, 8) and torch.equal(disp0, torch.zeros(1, 1, 2, 8, device="cuda"))


@pytest.mark.parametrize("mean", [False, True])
@pytest.mark.parametrize("kind", ["nonfinite", "tiny"])
def test_fused_volume_free_multipass_exact_segments(kind, mean):
    """D = 256 without the volume (band_sl's two passes merged in registers) on segments that
    take the band kernel's exact fp32 path: +-inf / NaN features, or a feature scale the fp16
    split cannot reach (max |L| ~ 2^-91).  NaN is carried as NaN, so the merged disparity equals
    the two-kernel pipeline's."""
    from realtime_stereo_matcher_amd import functional as F

    l, r = _feats(24 if kind == "nonfinite" else 25, (1, 16, 3, 320))
    if kind == "nonfinite":
        l[0, 5, 0, 300] = np.inf     # pass 0 and pass 1 cells of row 0
        l[0, 0, 1, 7] = -np.inf
        r[0, 3, 1, 100] = np.nan     # NaN in one pass only for some pixels
        r[0, 9, 2, 3] = np.inf
    else:
        l, r = (l * 1e-28).astype(np.float32), (r * 1e-8).astype(np.float32)
    L, R = dev(l), dev(r)
    _, disp = F.inner_product_soft_argmin(L, R, 256, mean=mean, keep_volume=False)
    vol = F.correlation_volume(L, R, 256) if mean else F.inner_product_volume(L, R, 256)
    want = O.softargmin(host(vol))
    got = host(disp)
    np.testing.assert_array_equal(np.isnan(got), np.isnan(want))
    np.testing.assert_allclose(got, want, atol=TOL, rtol=0, equal_nan=True)


@pytest.mark.parametrize("mean", [False, True])
@pytest.mark.parametrize("kind", ["nonfinite", "tiny"])
def test_fused_volume_free_one_pass_exact_segments(kind, mean):
    """One D pass (D = 160, C = 64: the role-split kernel's volume-free form) on segments that
    take the exact fp32 path: +-inf / NaN features, or a scale the fp16 split cannot reach.  The
    volume-free disparity equals the volume-kept call's bit for bit (NaN where it is NaN), and
    that one is the fp64 soft-argmin of its volume."""
    from realtime_stereo_matcher_amd import functional as F

    l, r = _feats(26 if kind == "nonfinite" else 27, (2, 64, 3, 320))
    if kind == "nonfinite":
        l[0, 5, 0, 300] = np.inf
        l[1, 0, 1, 7] = -np.inf
        r[0, 3, 1, 100] = np.nan
        r[1, 9, 2, 3] = np.inf
    else:
        l, r = (l * 1e-28).astype(np.float32), (r * 1e-8).astype(np.float32)
    L, R = dev(l), dev(r)
    vol, disp = F.inner_product_soft_argmin(L, R, 160, mean=mean)
    none, disp2 = F.inner_product_soft_argmin(L, R, 160, mean=mean, keep_volume=False)
    assert none is None
    np.testing.assert_array_equal(host(disp2), host(disp))
    np.testing.assert_allclose(host(disp), O.softargmin(host(vol)), atol=TOL, rtol=0, equal_nan=True)


def test_cfg2_fused_full_size():
    """cfg2 through the fused kernel: the volume equals the volume op's bit for bit, the
    disparity is the fp64 soft-argmin of that volume, with or without the volume written."""
    from realtime_stereo_matcher_amd import functional as F

    g = torch.Generator(device="cuda").manual_seed(0)
    L = torch.randn(1, 64, 540, 960, device="cuda", generator=g)
    R = torch.randn(1, 64, 540, 960, device="cuda", generator=g)
    vol, disp = F.inner_product_soft_argmin(L, R, 192)
    assert torch.equal(vol, F.inner_product_volume(L, R, 192))
    _, disp2 = F.inner_product_soft_argmin(L, R, 192, keep_volume=False)
    assert torch.equal(disp2, disp)
    for y in (0, 1, 269, 539):
        np.testing.assert_allclose(host(disp[:, :, y:y + 1]), O.softargmin(host(vol[:, :, y:y + 1])),
                                   atol=TOL, rtol=0)


# ================================================================================ §8f-4 warp
@pytest.mark.parametrize("rec", cases("warp"), ids=_ids(cases("warp")))
def test_golden_warp(rec):
    from realtime_stereo_matcher_amd.tools.warp import warp_by_flow_map

    a = load_case(rec)
    out = warp_by_flow_map(dev(a["image"]), dev(a["flow"]))
    assert out.shape == a["out"].shape and out.dtype == torch.float32
    np.testing.assert_allclose(host(out), a["out"], atol=TOL, rtol=0)


@pytest.mark.parametrize("ish,fsh", [((2, 7, 33, 65), (2, 1, 33, 65)), ((1, 3, 17, 30), (1, 2, 40, 61)),
                                     ((1, 5, 1, 9), (1, 1, 2, 9)), ((3, 1, 8, 8), (3, 2, 8, 8)),
                                     ((1, 9, 6, 1100), (1, 1, 6, 1100)), ((1, 2, 3, 5000), (1, 1, 3, 5000))])
def test_warp_vs_oracle(ish, fsh):
    from realtime_stereo_matcher_amd.functional import warp_by_flow_map

    rng = np.random.default_rng(11)
    img = rng.standard_normal(ish).astype(np.float32)
    flow = (rng.standard_normal(fsh) * 8 + 4).astype(np.float32)
    flow[..., 0, :3] = 1e9       # far outside: all corners padded -> 0
    flow[..., -1, -2:] = -3.0    # exact integer shift
    np.testing.assert_allclose(host(warp_by_flow_map(dev(img), dev(flow))),
                               O.warp_by_flow_map(img, flow), atol=TOL, rtol=0)


def test_warp_strided_and_errors():
    from realtime_stereo_matcher_amd.functional import warp_by_flow_map

    rng = np.random.default_rng(12)
    img = rng.standard_normal((2, 6, 10, 24)).astype(np.float32)
    flow = rng.uniform(0, 6, (2, 2, 10, 24)).astype(np.float32)
    I, Fl = dev(img), dev(flow)
    got = warp_by_flow_map(I[:, ::2], Fl[:, :1])         # channel-strided image, 1-ch flow view
    np.testing.assert_allclose(host(got), O.warp_by_flow_map(img[:, ::2], flow[:, :1]), atol=TOL, rtol=0)
    assert warp_by_flow_map(I[:, :0], Fl[:, :1]).shape == (2, 0, 10, 24)
    with pytest.raises(AssertionError, match="invalid flow map dimension"):
        warp_by_flow_map(I, torch.zeros(2, 3, 10, 24, device="cuda"))
    with pytest.raises(TypeError):
        warp_by_flow_map(I.double(), Fl[:, :1].double())
    with pytest.raises(RuntimeError):  # mixed dtypes outside autocast, as grid_sample
        warp_by_flow_map(I.half(), Fl[:, :1])
    # fp16 image and flow outside autocast: sampled in fp32 from the fp16 values, rounded once
    ih, fh = I.half(), Fl[:, :1].half()
    got = warp_by_flow_map(ih, fh)
    assert got.dtype == torch.float16
    want = O.warp_by_flow_map(host(ih), host(fh))
    np.testing.assert_allclose(host(got), want, atol=2e-3, rtol=2.0 ** -10)
    with pytest.raises(RuntimeError):
        warp_by_flow_map(I.cpu(), Fl[:, :1].cpu())


def test_warp_full_size_rows():
    """1x32x540x960 features warped by a 0..192 disparity map (RefineNet-style, full KITTI
    quarter-res plane): sampled rows, the border rows included, against the oracle."""
    from realtime_stereo_matcher_amd.functional import warp_by_flow_map

    g = torch.Generator(device="cuda").manual_seed(5)
    I = torch.randn(1, 32, 540, 960, device="cuda", generator=g)
    Fl = torch.rand(1, 1, 540, 960, device="cuda", generator=g) * 192
    out = warp_by_flow_map(I, Fl)
    rows = [0, 1, 269, 538, 539]
    ref = O.warp_by_flow_map(host(I), host(Fl), rows=rows)
    np.testing.assert_allclose(host(out[:, :, rows]), ref, atol=TOL, rtol=0)


def _warp_no_workspace(img, flow):
    """The warp through sm_warp_by_flow (no workspace: warp_kernel / warp_rows_kernel)."""
    from realtime_stereo_matcher_amd import _lib

    N, C, Hi, Wi = img.shape
    _, c, h, w = flow.shape
    out = torch.empty((N, C, h, w), dtype=torch.float32, device="cuda")
    _lib.check(_lib.load().sm_warp_by_flow(img.data_ptr(), flow.data_ptr(), out.data_ptr(), _lib.SM_F32,
                                           N, C, Hi, Wi, h, w, c, _lib.strides_arg(img),
                                           _lib.strides_arg(flow), torch.cuda.current_stream().cuda_stream),
               "sm_warp_by_flow")
    return out


@pytest.mark.parametrize("C", [1, 3, 4, 5, 32, 64, 65])
def test_warp_channel_last_path_bit_identical(C):
    """Two-channel flows take the channel-last gather (warp_to_nhwc + warp_gather_nhwc, C <= 64)
    when functional passes its workspace: bit-identical to warp_kernel, padding, NaN flows,
    a channel-strided image and a resized output grid included; and within TOL of the oracle."""
    from realtime_stereo_matcher_amd import _lib
    from realtime_stereo_matcher_amd.functional import warp_by_flow_map

    g = torch.Generator(device="cuda").manual_seed(100 + C)
    img = torch.randn(2, 2 * C, 19, 70, device="cuda", generator=g)[:, ::2]  # channel-strided
    flow = torch.randn(2, 2, 23, 67, device="cuda", generator=g) * 6
    flow[0, 0, 0, :5] = float("nan")
    flow[1, 1, 3, :4] = 1e9
    flow[1, :, -1, -3:] = 2.0
    got = warp_by_flow_map(img, flow)
    assert (int(_lib.load().sm_warp_by_flow_workspace_bytes(2, C, 19, 70, 2)) > 0) == (C <= 64)
    want = _warp_no_workspace(img, flow)
    assert torch.equal(torch.nan_to_num(got, nan=7.0), torch.nan_to_num(want, nan=7.0))
    assert torch.equal(torch.isnan(got), torch.isnan(want))
    if C in (3, 32):
        ref = O.warp_by_flow_map(host(img), host(flow))
        np.testing.assert_allclose(host(got), ref, atol=TOL, rtol=0)


def test_warp_full_size_two_channel_flow():
    """1x32x540x960 features, a sigma-4 two-channel flow (the bench's warp2 shape) through the
    channel-last path: sampled rows against the oracle and the whole plane against warp_kernel."""
    from realtime_stereo_matcher_amd.functional import warp_by_flow_map

    g = torch.Generator(device="cuda").manual_seed(6)
    I = torch.randn(1, 32, 540, 960, device="cuda", generator=g)
    Fl = torch.randn(1, 2, 540, 960, device="cuda", generator=g) * 4
    out = warp_by_flow_map(I, Fl)
    assert torch.equal(out, _warp_no_workspace(I, Fl))
    rows = [0, 1, 270, 539]
    ref = O.warp_by_flow_map(host(I), host(Fl), rows=rows)
    np.testing.assert_allclose(host(out[:, :, rows]), ref, atol=TOL, rtol=0)
