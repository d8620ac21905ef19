"""GPU parity of the role-split band kernel (algo "rs", csrc/ip_rs.hip) and the sliding-window
band kernel (algo "sl", csrc/ip_sl.hip; AUTO's choice) against the CPU oracle, on the shapes they
take (fp32, 4-element aligned rows, C = 16 or 64, D > 64 per pass), including the bench's own
launch shapes (cfg2 and cfg4: the whole 32-pair batch per launch; cfg4 also the 4-pair launch of
each rank at N = 8) and shapes with several rows per workgroup (the sliding window's row
changes).

Reference op: TorchInnerProductCost.forward (cost_volume/inner_product.py:11-42) and
make_correlation_volume (model/mobile_disp_net_c.py:188-205).  Tolerance: 1e-4 absolute for
fp32 volumes (north star), bit-exact for integer-valued features, relative 1e-5 of
sum_c |L||R| for scaled features.
"""
import numpy as np
import pytest
import torch

from oracle import stereo_oracle as O

pytestmark = pytest.mark.gpu
TOL = 1e-4
ALGOS = ["rs", "sl"]


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).to("cuda")


def host(t):
    return t.float().cpu().numpy()


def _feats(seed, shape, kind="normal"):
    rng = np.random.default_rng(seed)
    if kind == "int":
        return (rng.integers(-8, 9, size=shape).astype(np.float32),
                rng.integers(-8, 9, size=shape).astype(np.float32))
    return rng.standard_normal(shape, dtype=np.float32), rng.standard_normal(shape, dtype=np.float32)


# (N, C, H, W, D): every segment pattern -- the 64-pixel last tile of a 960 row, rows shorter
# than one segment, W = 4, odd item counts per workgroup, D one disparity past a block, two
# balanced D passes of 128 (D = 256), D > W
SP_SHAPES = [(1, 64, 3, 512, 192), (2, 64, 5, 260, 100), (3, 64, 2, 132, 128), (2, 64, 3, 960, 191),
             (1, 64, 2, 16, 96), (1, 64, 1, 4, 80), (1, 16, 4, 388, 192), (1, 16, 3, 1000, 256),
             (2, 16, 2, 200, 65), (1, 64, 2, 64, 192), (5, 16, 1, 900, 160),
             # more rows than workgroups: each sliding-window workgroup walks several rows
             (2, 64, 300, 324, 192), (3, 16, 200, 260, 256), (1, 16, 700, 132, 100),
             (1, 64, 520, 196, 128)]


@pytest.mark.parametrize("algo", ALGOS)
@pytest.mark.parametrize("shape", SP_SHAPES, ids=[str(s) for s in SP_SHAPES])
def test_sp_inner_product_and_correlation(shape, algo):
    from realtime_stereo_matcher_amd import functional as F

    n, c, h, w, D = shape
    l, r = _feats(hash(shape) % 997, (n, c, h, w))
    got = host(F.inner_product_volume(dev(l), dev(r), D, algo=algo))
    np.testing.assert_allclose(got, O.inner_product(l, r, D), atol=TOL, rtol=0)
    # identical to the double-buffered kernel's volume up to fp32 summation order: both use the
    # same split; compare loosely, and exactly on integer-valued features
    li, ri = _feats(7, (n, c, h, w), "int")
    np.testing.assert_array_equal(host(F.inner_product_volume(dev(li), dev(ri), D, algo=algo)),
                                  O.inner_product(li, ri, D))
    corr = host(F.correlation_volume(dev(l), dev(r), D, algo=algo))
    np.testing.assert_allclose(corr, O.correlation_mean(l, r, D), atol=TOL, rtol=0)


def _cell_norm(l, r, D):
    return O.inner_product(np.abs(l), np.abs(r), D)


@pytest.mark.parametrize("algo", ALGOS)
@pytest.mark.parametrize("scale", [1e-15, 1e-6, 1e6, 1e15])
def test_sp_feature_scales(scale, algo):
    """Uniformly tiny or huge features: the first segment is recomputed with a new power-of-two
    scale (the pipeline restart), later ones carry it."""
    from realtime_stereo_matcher_amd import functional as F

    l, r = _feats(21, (1, 64, 3, 512))
    l, r = (l * scale).astype(np.float32), (r * scale).astype(np.float32)
    got = host(F.inner_product_volume(dev(l), dev(r), 192, algo=algo))
    err = np.abs(got - O.inner_product(l, r, 192))
    assert (err <= 1e-5 * _cell_norm(l, r, 192) + 1e-37).all()


@pytest.mark.parametrize("algo", ALGOS)
def test_sp_mixed_scales(algo):
    """Scale changing from row to row and pixel to pixel: restarts and carried scales mixed
    with the drain of the previous segment (its own scale)."""
    from realtime_stereo_matcher_amd import functional as F

    rng = np.random.default_rng(5)
    n, c, h, w, D = 2, 64, 6, 640, 160
    l, r = _feats(22, (n, c, h, w))
    l = (l * 10.0 ** rng.uniform(-8, 8, (n, 1, h, 1)) * 10.0 ** rng.uniform(-2, 2, (n, 1, h, w))).astype(np.float32)
    r = (r * 10.0 ** rng.uniform(-8, 8, (n, 1, h, 1)) * 10.0 ** rng.uniform(-2, 2, (n, 1, h, w))).astype(np.float32)
    got = host(F.inner_product_volume(dev(l), dev(r), D, algo=algo))
    err = np.abs(got - O.inner_product(l, r, D))
    bound = 1e-5 * _cell_norm(l, r, D) + 1e-30
    assert (err <= bound).all(), float((err / bound).max())


@pytest.mark.parametrize("algo", ALGOS)
@pytest.mark.parametrize("c", [16, 64])
def test_sp_nonfinite(c, algo):
    """+-inf features take the exact path; NaN reaches the band (max|x| does not see it) and the
    x < d cells are still forced to 0; the drained neighbours are unaffected."""
    from realtime_stereo_matcher_amd import functional as F

    l, r = _feats(23, (1, c, 4, 512))
    l[0, 5, 0, 130] = np.inf
    l[0, 0, 1, 7] = -np.inf
    r[0, 3, 1, 100] = np.nan
    r[0, 9, 2, 3] = np.inf
    l[0, 2, 3, 1] = np.nan  # NaN in L next to the x < d triangle
    r[0, 1, 3, 0] = np.nan  # NaN at R pixel 0: the pad groups of the row read it
    D = 128
    got = host(F.inner_product_volume(dev(l), dev(r), D, algo=algo))
    want = O.inner_product(l, r, D)
    np.testing.assert_array_equal(np.isnan(got), np.isnan(want))
    np.testing.assert_array_equal(np.isposinf(got), np.isposinf(want))
    np.testing.assert_array_equal(np.isneginf(got), np.isneginf(want))
    fin = np.isfinite(want)
    np.testing.assert_allclose(got[fin], want[fin], atol=TOL, rtol=0)


@pytest.mark.parametrize("algo", ALGOS)
def test_sp_strided_inputs(algo):
    """Channel- and batch-strided views (rows contiguous) go through the ABI strides."""
    from realtime_stereo_matcher_amd import functional as F

    l, r = _feats(9, (2, 128, 3, 320))
    L, R = dev(l)[:, ::2], dev(r)[:, 1::2]  # C = 64 with channel stride 2 H W
    got = host(F.inner_product_volume(L, R, 192, algo=algo))
    np.testing.assert_allclose(got, O.inner_product(l[:, ::2], r[:, 1::2], 192), atol=TOL, rtol=0)


def _check_rows(vol, L, R, D, rows, mean=False):
    """Rows of every pair of ``vol`` against the oracle; copies only those rows to the host."""
    for n in range(vol.shape[0]):
        for y in rows:
            fn = O.correlation_mean if mean else O.inner_product
            ref = fn(host(L[n:n + 1, :, y:y + 1]), host(R[n:n + 1, :, y:y + 1]), D)
            np.testing.assert_allclose(host(vol[n:n + 1, :, y:y + 1]), ref, atol=TOL, rtol=0,
                                       err_msg=f"pair {n} row {y}")


# bench.py CONFIGS: cfg2 and cfg4 launch the rank's whole batch (32 pairs at N = 1) at once
BENCH_PAIRS = 32


@pytest.mark.parametrize("algo", ALGOS)
def test_sp_cfg2_bench_launch_shape(algo):
    """The bench's launch: the whole cfg2 global batch, 32 pairs (32x64x540x960 fp32, D = 192;
    a 12.7 GB volume) in ONE launch.  Rows of
    EVERY pair (first, last and the pair boundaries of the persistent schedule) against the
    oracle, the x < d triangle exactly zero, and the soft-argmin of every sampled row."""
    from realtime_stereo_matcher_amd import functional as F

    g = torch.Generator(device="cuda").manual_seed(3)
    L = torch.randn(BENCH_PAIRS, 64, 540, 960, device="cuda", generator=g)
    R = torch.randn(BENCH_PAIRS, 64, 540, 960, device="cuda", generator=g)
    vol = F.inner_product_volume(L, R, 192, algo=algo)
    disp = F.soft_argmin(vol)
    torch.cuda.synchronize()
    _check_rows(vol, L, R, 192, (0, 1, 270, 538, 539))
    for n in range(BENCH_PAIRS):
        got = host(vol[n:n + 1, :, 100:101])
        np.testing.assert_allclose(host(disp[n:n + 1, :, 100:101]).reshape(-1),
                                   O.softargmin(got).reshape(-1), atol=TOL, rtol=0)
    tri = torch.arange(960, device="cuda")[None, :] < torch.arange(192, device="cuda")[:, None]
    for n in range(BENCH_PAIRS):
        assert not vol[n].permute(1, 0, 2)[:, tri].any()


@pytest.mark.parametrize("algo", ALGOS)
def test_sp_cfg4_bench_launch_shape(algo):
    """The bench's cfg4 launch: the whole global batch, 32 pairs of 16x1080x1920 fp32, correlation
    D = 256 (two passes of 128 per segment; a 68 GB volume, element offsets past 2^32) in one
    launch; rows of every pair against the oracle."""
    from realtime_stereo_matcher_amd import functional as F

    g = torch.Generator(device="cuda").manual_seed(4)
    L = torch.randn(BENCH_PAIRS, 16, 1080, 1920, device="cuda", generator=g)
    R = torch.randn(BENCH_PAIRS, 16, 1080, 1920, device="cuda", generator=g)
    vol = F.correlation_volume(L, R, 256, algo=algo)
    torch.cuda.synchronize()
    _check_rows(vol, L, R, 256, (0, 541, 1079), mean=True)
    del vol
    torch.cuda.empty_cache()


@pytest.mark.parametrize("algo", ALGOS)
def test_sp_cfg4_rank_launch_at_n8(algo):
    """The per-rank cfg4 launch at N = 8 (global batch 32 sharded over 8 GPUs: 4 pairs of
    16x1080x1920 fp32, correlation D = 256, mobile_disp_net_c.py:365-367): rows of every pair
    (first, middle, last, and the rows around each XCD range boundary of the schedule) against
    the oracle."""
    from realtime_stereo_matcher_amd import functional as F

    g = torch.Generator(device="cuda").manual_seed(5)
    L = torch.randn(4, 16, 1080, 1920, device="cuda", generator=g)
    R = torch.randn(4, 16, 1080, 1920, device="cuda", generator=g)
    vol = F.correlation_volume(L, R, 256, algo=algo)
    torch.cuda.synchronize()
    _check_rows(vol, L, R, 256, (0, 539, 540, 1079), mean=True)
    del vol
    torch.cuda.empty_cache()


# groupwise volumes of 16-bit features on the role-split kernel ((N, G, H, W, D) fp32 output,
# the ring in pixel-record layout): group steps of 16 / 32 / 64 channels, D = 68..192 (D < DMAX
# takes the masked readout), ragged W, several pairs; exact products, so within 1e-4 of the
# fp64 oracle on the dtype-rounded features
GW_SHAPES = [(1, 256, 3, 960, 192, 8), (2, 64, 2, 260, 100, 4), (1, 128, 2, 200, 68, 4),
             (1, 64, 3, 132, 128, 1), (1, 32, 2, 388, 160, 2), (3, 128, 1, 64, 192, 2)]


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16], ids=["bf16", "f16"])
@pytest.mark.parametrize("shape", GW_SHAPES, ids=[str(s) for s in GW_SHAPES])
def test_rs_groupwise_16bit(shape, dt):
    from realtime_stereo_matcher_amd import functional as F

    n, c, h, w, D, G = shape
    l, r = _feats(hash(shape) % 991, (n, c, h, w))
    L = torch.from_numpy(l).cuda().to(dt)
    R = torch.from_numpy(r).cuda().to(dt)
    got = host(F.groupwise_volume(L, R, G, D))
    assert got.shape == (n, G, h, w, D)
    want = O.groupwise(host(L), host(R), G, D)
    np.testing.assert_allclose(got, want, atol=TOL, rtol=0)


def _softargmin_bound(vol64, eps):
    """Rigorous per-pixel bound on the soft-argmin change under cell errors |delta_k| <= eps_k
    (test_autocast._disp_bound's form): e^max(eps) * sum_k |k - disp| q_k (e^eps_k - 1)."""
    q = np.exp(vol64 - vol64.max(axis=1, keepdims=True))
    q /= q.sum(axis=1, keepdims=True)
    k = np.arange(vol64.shape[1], dtype=np.float64).reshape(1, -1, 1, 1)
    disp = (k * q).sum(axis=1, keepdims=True)
    s = (np.abs(k - disp) * q * np.expm1(eps)).sum(axis=1, keepdims=True)
    return disp, np.exp(eps.max(axis=1, keepdims=True)) * s


@pytest.mark.parametrize("D", [160, 256])
def test_sl_mixed_scales_c16(D):
    """band_sl's one-channel-step (C = 16) restart path -- the range check before a
    segment's steps, the window re-staged -- under row-to-row and pixel-to-pixel scale changes,
    for the volume (both kernels, one and two D passes) and for the volume-free fused call
    (D = 256: the two-pass f_m / f_s register carry across restarts, cfg4's production shape).
    L's row scale is the inverse of R's, so the features span 1e-8 .. 1e8 while the cells stay
    O(10) and the softmax is well conditioned.  Volume: relative 1e-5 of sum_c |L R| (the other
    scale tests' bar).  Disparity: the fp64 soft-argmin of the oracle volume within the rigorous
    softmax bound for cell errors of 4e-6 sum_c |L R| (the split's three dropped terms, 2^-22
    each, and fp32 accumulation over 16 products), plus 1e-4."""
    from realtime_stereo_matcher_amd import functional as F

    rng = np.random.default_rng(D)
    n, c, h, w = 2, 16, 6, 640
    l, r = _feats(31, (n, c, h, w))
    row = 10.0 ** rng.uniform(-8, 8, (n, 1, h, 1))
    l = (l * row * 10.0 ** rng.uniform(-0.5, 0.5, (n, 1, h, w))).astype(np.float32)
    r = (r / row * 10.0 ** rng.uniform(-0.5, 0.5, (n, 1, h, w))).astype(np.float32)
    want = O.inner_product(l, r, D)
    cn = _cell_norm(l, r, D)
    for algo in ALGOS:
        got = host(F.inner_product_volume(dev(l), dev(r), D, algo=algo))
        err = np.abs(got - want)
        assert (err <= 1e-5 * cn + 1e-30).all(), (algo, float((err / (1e-5 * cn + 1e-30)).max()))
    _, disp = F.inner_product_soft_argmin(dev(l), dev(r), D, keep_volume=False)
    ex, bound = _softargmin_bound(O._dot_volume(l.astype(np.float64), r.astype(np.float64), D),
                                  4e-6 * O._dot_volume(np.abs(l).astype(np.float64), np.abs(r).astype(np.float64), D))
    err = np.abs(host(disp).astype(np.float64) - ex)
    assert (err <= bound + TOL).all(), float((err / (bound + TOL)).max())


@pytest.mark.parametrize("D,keep", [(96, True), (96, False), (256, False)])
def test_fused_cells_near_flt_max(D, keep):
    """the sliding-window kernel's fused fold takes 1/C and the segment scale into the
    exponent's FMA, whose shift is clamped at 2e38; a block whose largest cell is above that must
    not overflow exp2.  C = 16, |L| = |R| = a with R = L, 16 a^2 = 3.2e38: every pixel's d = 0 cell
    is 3.2e38 and the others at least 2 a^2 lower, so the soft-argmin is 0 (ties give their mean),
    finite; the oracle's fp64 soft-argmin of the fp32 volume says the same."""
    from realtime_stereo_matcher_amd import functional as F

    rng = np.random.default_rng(7)
    a = np.float32(np.sqrt(3.2e38 / 16))
    l = (np.where(rng.uniform(size=(1, 16, 2, 128)) < 0.5, -a, a)).astype(np.float32)
    r = l.copy()
    vol, disp = F.inner_product_soft_argmin(dev(l), dev(r), D, keep_volume=keep)
    want_vol = O.inner_product(l, r, D)
    assert np.isfinite(want_vol).all() and want_vol.max() >= 3.0e38
    got = host(disp)
    assert np.isfinite(got).all()
    np.testing.assert_allclose(got, O.softargmin(want_vol), atol=TOL, rtol=0)
    if keep:
        np.testing.assert_allclose(host(vol), want_vol, rtol=1e-5, atol=0)
