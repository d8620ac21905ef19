"""Pin the CPU oracle (oracle/stereo_oracle.py) and the eager CPU port (oracle/torch_port.py)
against the golden vectors recorded from the reference's own modules (CPU-only tests)."""
import os

import numpy as np
import pytest
import torch

from conftest import cases, load_case
from oracle import stereo_oracle as O
from oracle import torch_port as P

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

TOL_F32 = 1e-4  # north-star fp32 bar (BASELINE.json)


def _ids(cs):
    return [c["name"] for c in cs]


@pytest.mark.parametrize("rec", cases("inner_product"), ids=_ids(cases("inner_product")))
def test_inner_product(rec):
    a = load_case(rec)
    D = rec["params"]["max_disparity"]
    got = O.inner_product(a["left"], a["right"], D, out_dtype=rec["dtype"], literal=rec.get("literal", False))
    ref = a["out"].astype(np.float32)
    if rec.get("exact"):
        np.testing.assert_array_equal(got, ref)
    elif rec["dtype"] == "f32":
        np.testing.assert_allclose(got, ref, atol=TOL_F32, rtol=0)
    else:  # f16 / bf16: literal product rounding, fp64 sum -> within 1 output ulp
        np.testing.assert_allclose(got.astype(np.float32), ref, rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("rec", cases("groupwise"), ids=_ids(cases("groupwise")))
def test_groupwise(rec):
    a = load_case(rec)
    p = rec["params"]
    lit = "bf16" if rec["dtype"] == "bf16" else None
    got = O.groupwise(a["left"], a["right"], p["n_groups"], p["max_disparity"], literal_dtype=lit)
    assert got.dtype == np.float32 and got.shape == a["out"].shape
    if lit:
        # literal bf16 product + bf16 mean: agree within one bf16 ulp of the value
        np.testing.assert_allclose(got, a["out"], rtol=2 ** -7, atol=1e-6)
    else:
        np.testing.assert_allclose(got, a["out"], atol=TOL_F32, rtol=0)


def test_groupwise_assert_message(manifest):
    with pytest.raises(AssertionError) as e:
        O.groupwise(np.zeros((1, 16, 2, 8), np.float32), np.zeros((1, 16, 2, 8), np.float32), 3, 4)
    assert str(e.value) == manifest["groupwise_assert_message_c16_g3"]


@pytest.mark.parametrize("rec", cases("concat"), ids=_ids(cases("concat")))
def test_concat(rec):
    a = load_case(rec)
    got = O.concatenate(a["left"], a["right"], rec["params"]["max_disparity"])
    np.testing.assert_array_equal(got, a["out"])


@pytest.mark.parametrize("rec", cases("interweave"), ids=_ids(cases("interweave")))
def test_interweave(rec):
    a = load_case(rec)
    np.testing.assert_array_equal(O.interweave(a["left"], a["right"]), a["out"])


@pytest.mark.parametrize("rec", cases("interweave_shifted"), ids=_ids(cases("interweave_shifted")))
def test_interweave_shifted(rec):
    a = load_case(rec)
    got = O.interweave_shifted(a["left"], a["right"], rec["params"]["max_disparity"])
    np.testing.assert_array_equal(got, a["out"])


@pytest.mark.parametrize("rec", cases("diff_volume"), ids=_ids(cases("diff_volume")))
def test_diff_volume(rec):
    a = load_case(rec)
    got = O.diff_volume(a["left"], a["right"], rec["params"]["max_disp"])
    np.testing.assert_array_equal(got, a["out"])


@pytest.mark.parametrize("rec", cases("correlation"), ids=_ids(cases("correlation")))
def test_correlation(rec):
    a = load_case(rec)
    got = O.correlation_mean(a["left"], a["right"], rec["params"]["max_disp"])
    np.testing.assert_allclose(got, a["out"], atol=TOL_F32, rtol=0)


@pytest.mark.parametrize("rec", cases("softargmin"), ids=_ids(cases("softargmin")))
def test_softargmin(rec):
    a = load_case(rec)
    got = O.softargmin(a["volume"], rec["params"]["max_disp"])
    assert got.shape == a["out"].shape
    np.testing.assert_allclose(got, a["out"], atol=TOL_F32, rtol=0)


@pytest.mark.parametrize("rec", cases("regression_presoftmax"), ids=_ids(cases("regression_presoftmax")))
def test_regression_presoftmax(rec):
    a = load_case(rec)
    got = O.regression_presoftmax(a["volume"], rec["params"]["maxdisp"])
    assert got.shape == a["out"].shape
    np.testing.assert_allclose(got, a["out"], atol=TOL_F32, rtol=0)


def test_softargmin_assert_messages(manifest):
    with pytest.raises(AssertionError) as e:
        O.softargmin(np.zeros((1, 5, 2, 2), np.float32), 4)
    assert str(e.value) == manifest["softargmin_assert_message_d5_vs_4"]
    with pytest.raises(AssertionError) as e:
        O.softargmin(np.zeros((5, 2, 2), np.float32), 5)
    assert str(e.value) == manifest["softargmin_assert_message_ndim3"]


@pytest.mark.parametrize("rec", cases("argext"), ids=_ids(cases("argext")))
def test_argext(rec):
    a = load_case(rec)
    got = O.argext(a["volume"], rec["params"]["mode"])
    np.testing.assert_array_equal(got, a["out"])
    if "left" in a:  # the integer-valued volume itself is exact in the oracle
        vol = O.inner_product(a["left"], a["right"], rec["params"]["max_disparity"])
        np.testing.assert_array_equal(vol, a["volume"])


def test_argext_nan_first_index():
    v = np.zeros((1, 4, 1, 3), np.float32)
    v[0, 2, 0, 0] = np.nan
    v[0, 3, 0, 0] = np.nan
    v[0, 1, 0, 1] = 5.0
    t = torch.from_numpy(v)
    for mode, fn in (("max", torch.argmax), ("min", torch.argmin)):
        np.testing.assert_array_equal(O.argext(v, mode), fn(t, dim=1).numpy())


# --------------------------------------------------------------------------- the eager CPU port
def test_torch_port_inner_product_cfg1():
    rec = next(c for c in cases("inner_product") if "cfg1" in c["name"])
    a = load_case(rec)
    got = P.sweep_dot_volume(torch.from_numpy(a["left"]), torch.from_numpy(a["right"]), 24)
    np.testing.assert_allclose(got.numpy(), a["out"], atol=TOL_F32, rtol=0)


@pytest.mark.parametrize("rec", cases("correlation"), ids=_ids(cases("correlation")))
def test_torch_port_correlation(rec):
    a = load_case(rec)
    got = P.sweep_dot_volume(torch.from_numpy(a["left"]), torch.from_numpy(a["right"]),
                             rec["params"]["max_disp"], mean=True)
    np.testing.assert_allclose(got.numpy(), a["out"], atol=TOL_F32, rtol=0)


@pytest.mark.parametrize("rec", cases("softargmin"), ids=_ids(cases("softargmin")))
def test_torch_port_softargmin(rec):
    a = load_case(rec)
    np.testing.assert_array_equal(P.soft_argmin_eager(torch.from_numpy(a["volume"])).numpy(), a["out"])


# ------------------------------------------------------------------------------ §8f-4 warp
@pytest.mark.parametrize("rec", cases("warp"), ids=_ids(cases("warp")))
def test_warp(rec):
    a = load_case(rec)
    got = O.warp_by_flow_map(a["image"], a["flow"])
    assert got.shape == a["out"].shape and got.dtype == np.float32
    np.testing.assert_allclose(got, a["out"], atol=TOL_F32, rtol=0)


def test_warp_assert_message(manifest):
    with pytest.raises(AssertionError) as e:
        O.warp_by_flow_map(np.zeros((1, 2, 3, 4), np.float32), np.zeros((1, 3, 3, 4), np.float32))
    assert str(e.value) == manifest["warp_assert_message_c3"]


def test_warp_rows_subset_matches_full():
    """The oracle's row-subset mode (used at full size on the GPU) equals the full evaluation."""
    rng = np.random.default_rng(3)
    img = rng.standard_normal((2, 3, 9, 21)).astype(np.float32)
    for fch in (1, 2):
        flow = rng.uniform(-3, 8, (2, fch, 9, 21)).astype(np.float32)
        full = O.warp_by_flow_map(img, flow)
        rows = [0, 4, 8]
        np.testing.assert_array_equal(O.warp_by_flow_map(img, flow, rows=rows), full[:, :, rows])


def test_model_weights_deterministic():
    """tests/model_weights.seeded_state is a pure function of (layout, seed)."""
    from model_weights import seeded_state

    layout = {"a.weight": torch.zeros(4, 3, 3, 3), "a.bias": torch.zeros(4),
              "bn.weight": torch.zeros(4), "bn.bias": torch.zeros(4),
              "bn.running_mean": torch.zeros(4), "bn.running_var": torch.zeros(4),
              "bn.num_batches_tracked": torch.zeros((), dtype=torch.int64)}
    s1, s2 = seeded_state(layout, 5), seeded_state(layout, 5)
    assert all(torch.equal(s1[k], s2[k]) for k in layout)
    assert not torch.equal(seeded_state(layout, 6)["a.weight"], s1["a.weight"])
    assert float(s1["bn.running_var"].min()) >= 0.75


V4_FILES = sorted(f for f in os.listdir(GOLDEN_DIR) if f.startswith("v4_volume_"))


def v4_case(name):
    """A §8f-2 fixture: inputs, the conv3d / volume11 parameters (``p/`` keys) and the volume
    the reference loop produced (tests/golden/gen_model_golden.py)."""
    a = np.load(os.path.join(GOLDEN_DIR, name))  # allow_pickle=False: data only
    return a, {k[2:]: a[k] for k in a.files if k.startswith("p/")}


@pytest.mark.parametrize("name", V4_FILES)
def test_v4_volume(name):
    """The V4 interweave + Conv3d cost-volume restatement (model/mobile_stereo_net_v4.py:443-461)
    against the reference loop's own output."""
    a, p = v4_case(name)
    np.testing.assert_allclose(O.v4_volume(a["featL"], a["featR"], p, 48), a["volume"], atol=1e-5, rtol=0)


# ------------------------------------------------- eager restatements of the isolation test
@pytest.mark.parametrize("rec", cases("diff_volume"), ids=_ids(cases("diff_volume")))
def test_torch_port_diff_volume(rec):
    a = load_case(rec)
    dt = {"f32": torch.float32, "f16": torch.float16, "bf16": torch.bfloat16}[rec["dtype"]]
    got = P.sweep_diff_volume(torch.from_numpy(a["left"]).to(dt), torch.from_numpy(a["right"]).to(dt),
                              rec["params"]["max_disp"])
    np.testing.assert_array_equal(got.float().numpy(), a["out"].astype(np.float32))


@pytest.mark.parametrize("rec", cases("softargmin"), ids=_ids(cases("softargmin")))
def test_torch_port_softargmin_fp64(rec):
    a = load_case(rec)
    got = P.soft_argmin_fp64(torch.from_numpy(a["volume"])).numpy()
    np.testing.assert_allclose(got, O.softargmin(a["volume"]), atol=1e-6, rtol=0)
    np.testing.assert_allclose(got, a["out"], atol=TOL_F32, rtol=0)


@pytest.mark.parametrize("rec", cases("regression_presoftmax"), ids=_ids(cases("regression_presoftmax")))
def test_torch_port_presoftmax_fp64(rec):
    a = load_case(rec)
    got = P.regression_presoftmax_fp64(torch.from_numpy(a["volume"]), rec["params"]["maxdisp"]).numpy()
    np.testing.assert_allclose(got, a["out"], atol=TOL_F32, rtol=0)


@pytest.mark.parametrize("rec", cases("warp"), ids=_ids(cases("warp")))
def test_torch_port_warp(rec):
    a = load_case(rec)
    got = P.warp_grid_sample(torch.from_numpy(a["image"]), torch.from_numpy(a["flow"])).numpy()
    np.testing.assert_allclose(got, a["out"], atol=TOL_F32, rtol=0, equal_nan=True)


@pytest.mark.parametrize("name", V4_FILES)
def test_torch_port_v4_volume_loop(name):
    """The eager V4 loop on modules loaded with the fixture's parameters reproduces the reference
    loop's output (the isolation test swaps it in for the HIP operator)."""
    from realtime_stereo_matcher_amd.model.stereo_net_v4 import MobileStereoNetV4HIP

    a, p = v4_case(name)
    net = MobileStereoNetV4HIP(192)
    net.conv3d.load_state_dict({k[7:]: torch.from_numpy(v) for k, v in p.items() if k.startswith("conv3d.")})
    net.volume11.load_state_dict({k[9:]: torch.from_numpy(v) for k, v in p.items() if k.startswith("volume11.")})
    net.eval()
    with torch.no_grad():
        got = P.v4_volume_loop(torch.from_numpy(a["featL"]), torch.from_numpy(a["featR"]),
                               net.conv3d, net.volume11, 48).numpy()
    np.testing.assert_allclose(got, a["volume"], atol=1e-5, rtol=0)


def _autocast_cases():
    import json
    with open(os.path.join(GOLDEN_DIR, "autocast_manifest.json")) as f:
        return json.load(f)["cases"]


@pytest.mark.parametrize("rec", _autocast_cases(), ids=[c["name"] for c in _autocast_cases()])
def test_autocast_fixture(rec):
    """The reference's fp16 eval (tests/golden/gen_autocast_golden.py): the oracle's literal form
    (each product rounded to fp16, fp64 sum, one fp16 rounding) is within one fp16 ulp of the
    reference's fp16 volume (its sums are fp32), and the fp64 soft-argmin of that fp16 volume is
    the reference's fp32 disparity within the fp32 bar (its CPU fp32 softmax deviates by up to
    8.4e-5 at disparities of ~90 px)."""
    a = np.load(os.path.join(GOLDEN_DIR, rec["file"]))
    D = rec["max_disparity"]
    f = O.correlation_mean if rec["mean"] else O.inner_product
    got = f(a["left"], a["right"], D, out_dtype="f16", literal=True).astype(np.float64)
    ref = a["volume"].astype(np.float64)
    ulp = np.spacing(np.abs(ref).astype(np.float16)).astype(np.float64)
    assert (np.abs(got - ref) <= ulp).all()
    # the literal rounding matters: the exact-product volume differs from the reference's
    exact = f(a["left"], a["right"], D, out_dtype="f16").astype(np.float64)
    assert (exact != ref).any()
    np.testing.assert_allclose(O.softargmin(a["volume"].astype(np.float32)), a["disparity"],
                               atol=TOL_F32, rtol=0)


def _f64_cases():
    import json
    with open(os.path.join(GOLDEN_DIR, "f64_manifest.json")) as f:
        return json.load(f)["cases"]


@pytest.mark.parametrize("rec", _f64_cases(), ids=[c["name"] for c in _f64_cases()])
def test_f64_fixture(rec):
    """The oracle's fp64 restatement against the reference's fp64 outputs
    (tests/golden/gen_f64_golden.py): sums within 1e-12 of sum |L R|, copies bit-exact."""
    a = np.load(os.path.join(GOLDEN_DIR, rec["file"]))
    p, op, want = rec["params"], rec["op"], a["out"]
    if op in ("inner_product", "correlation"):
        D = p.get("max_disparity", p.get("max_disp"))
        got = O._dot_volume(a["left"], a["right"], D) / (a["left"].shape[1] if op == "correlation" else 1)
        norm = O._dot_volume(np.abs(a["left"]), np.abs(a["right"]), D)
        assert (np.abs(got - want) <= 1e-12 * (norm + 1)).all()
    elif op == "groupwise":
        got = O.groupwise(a["left"], a["right"], p["n_groups"], p["max_disparity"])
        np.testing.assert_allclose(got, want, rtol=2 ** -23, atol=1e-30)
    elif op == "concat":
        np.testing.assert_array_equal(O.concatenate(a["left"], a["right"], p["max_disparity"]), want)
    elif op == "interweave":
        np.testing.assert_array_equal(O.interweave(a["left"], a["right"]), want)
    elif op == "diff_volume":
        np.testing.assert_array_equal(O.diff_volume(a["left"], a["right"], p["max_disp"]), want)
    elif op == "argmax":
        np.testing.assert_array_equal(O.argext(a["volume"], "max"), want)
    elif op in ("softargmin", "regression_presoftmax"):
        v = a["volume"]
        d = np.arange(v.shape[1], dtype=np.float64).reshape(1, -1, 1, 1)
        if op == "softargmin":
            q = np.exp(v - v.max(axis=1, keepdims=True))
            got = (q * d).sum(axis=1, keepdims=True) / q.sum(axis=1, keepdims=True)
        else:
            got = (v * d).sum(axis=1)
        np.testing.assert_allclose(got, want, atol=1e-12, rtol=0)
    else:
        raise AssertionError(op)
