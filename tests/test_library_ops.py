"""torch.ops.stereocv: the engine's operators as traceable custom ops (library.py).

The reference traces its networks with torch.onnx.export (tools/convert.py:18-26) and with
thop / fvcore (tools/profiler.py:11-26).  Under a tracer the functional layer routes every call
through torch.ops.stereocv, so the traced graph holds the operator, not a baked constant."""
import pytest
import torch

from realtime_stereo_matcher_amd import library  # noqa: F401  (registers the ops)

OPS = ["inner_product_volume", "correlation_volume", "groupwise_volume", "concat_volume",
       "interweave", "interweave_volume", "difference_volume", "soft_argmin",
       "regression_presoftmax", "hard_argmin", "hard_argmax", "inner_product_soft_argmin",
       "inner_product_soft_argmin_novolume", "warp_by_flow_map", "v4_volume"]


def test_ops_registered():
    for name in OPS:
        assert hasattr(torch.ops.stereocv, name), name


def test_fake_kernels_shapes():
    """FakeTensor tracing (torch.export / torch.compile) sees each output's shape and dtype."""
    from torch._subclasses.fake_tensor import FakeTensorMode

    with FakeTensorMode():
        l, r = torch.empty(2, 8, 4, 16), torch.empty(2, 8, 4, 16)
        ops = torch.ops.stereocv
        assert ops.inner_product_volume(l, r, 5, "auto").shape == (2, 5, 4, 16)
        assert ops.correlation_volume(l, r, 6).shape == (2, 6, 4, 16)
        g = ops.groupwise_volume(l, r, 2, 5)
        assert g.shape == (2, 2, 4, 16, 5) and g.dtype == torch.float32
        assert ops.concat_volume(l, r, 3).shape == (2, 16, 4, 16, 3)
        assert ops.interweave(l, r).shape == (2, 16, 4, 16)
        assert ops.interweave_volume(l, r, 3).shape == (2, 16, 3, 4, 16)
        assert ops.difference_volume(l, r, 3).shape == (2, 8, 3, 4, 16)
        v = torch.empty(2, 5, 4, 16)
        assert ops.soft_argmin(v).shape == (2, 4, 16)
        assert ops.regression_presoftmax(v).shape == (2, 4, 16)
        a = ops.hard_argmax(v)
        assert a.shape == (2, 4, 16) and a.dtype == torch.int64
        vol, d = ops.inner_product_soft_argmin(l, r, 5, False)
        assert vol.shape == (2, 5, 4, 16) and d.shape == (2, 1, 4, 16)
        assert ops.inner_product_soft_argmin_novolume(l, r, 5, True).shape == (2, 1, 4, 16)
        img, fl = torch.empty(2, 3, 8, 20), torch.empty(2, 1, 4, 16)
        wp = ops.warp_by_flow_map(img, fl)
        assert wp.shape == (2, 3, 4, 16) and wp.dtype == torch.float32
        ws = [torch.empty(s) for s in ((16, 8, 3, 3), (16,), (32, 16, 4, 3, 3), (32,),
                                       (16, 32, 2, 3, 3), (16,), (16,), (1,))]
        f32 = torch.empty(2, 32, 4, 16)
        assert ops.v4_volume(f32, f32, *ws, 12).shape == (2, 12, 4, 16)


def test_eager_path_not_routed():
    assert not library.tracing()


@pytest.mark.gpu
def test_jit_trace_inner_product_network():
    """torch.jit.trace of the reference-style CV + regression: the graph holds the ops and
    reproduces the eager outputs on NEW inputs (a baked constant would not)."""
    from realtime_stereo_matcher_amd.cost_volume import TorchInnerProductCost
    from realtime_stereo_matcher_amd.model.mobile_disp_net_c import disparity_regression

    class Net(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.cv = TorchInnerProductCost(24)

        def forward(self, l, r):
            return disparity_regression(self.cv(l, r), 24)

    g = torch.Generator(device="cuda").manual_seed(3)
    l0, r0 = (torch.randn(1, 32, 16, 64, device="cuda", generator=g) for _ in range(2))
    net = Net().eval()
    with torch.no_grad():
        traced = torch.jit.trace(net, (l0, r0))
    assert "stereocv::inner_product_volume" in str(traced.inlined_graph)
    assert "stereocv::soft_argmin" in str(traced.inlined_graph)
    l1, r1 = (torch.randn(1, 32, 16, 64, device="cuda", generator=g) for _ in range(2))
    with torch.no_grad():
        torch.testing.assert_close(traced(l1, r1), net(l1, r1), rtol=0, atol=0)


@pytest.mark.gpu
def test_torch_export_groupwise_and_correlation():
    """torch.export through the fake kernels; the exported program runs the HIP kernels."""
    from realtime_stereo_matcher_amd.cost_volume import TorchGroupwiseCost
    from realtime_stereo_matcher_amd.model.mobile_disp_net_c import make_correlation_volume

    class Net(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.gw = TorchGroupwiseCost(4, 16)

        def forward(self, l, r):
            return self.gw(l, r).sum(-1), make_correlation_volume(l, r, 16)

    g = torch.Generator(device="cuda").manual_seed(4)
    l0, r0 = (torch.randn(1, 16, 8, 64, device="cuda", generator=g) for _ in range(2))
    net = Net().eval()
    ep = torch.export.export(net, (l0, r0))
    s = str(ep.graph)
    assert "stereocv.groupwise_volume" in s and "stereocv.correlation_volume" in s
    l1, r1 = (torch.randn(1, 16, 8, 64, device="cuda", generator=g) for _ in range(2))
    for a, b in zip(ep.module()(l1, r1), net(l1, r1)):
        torch.testing.assert_close(a, b, rtol=0, atol=0)


@pytest.mark.gpu
@pytest.mark.parametrize("v", ["v2", "v3", "v4"])
def test_jit_trace_refine_and_v4_networks(v):
    """torch.jit.trace of the demo networks whose forward calls the warp (v2 / v3 RefineNet,
    model/mobile_stereo_net_v2.py:127, _v3.py:136) or the V4 volume (mobile_stereo_net_v4.py:
    443-461): the graph holds stereocv::warp_by_flow_map / stereocv::v4_volume and reproduces
    the eager network on NEW inputs (a baked constant would not)."""
    import numpy as np
    from test_model_demo import _fixture, _net

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    net = _net(_fixture(v), v).cuda()
    g = torch.Generator(device="cuda").manual_seed(11)
    x0 = [torch.rand(1, 3, 64, 96, device="cuda", generator=g) for _ in range(2)]
    with torch.no_grad():
        traced = torch.jit.trace(net, tuple(x0), check_trace=False)
    graph = str(traced.inlined_graph)
    assert ("stereocv::v4_volume" if v == "v4" else "stereocv::warp_by_flow_map") in graph
    x1 = [torch.rand(1, 3, 64, 96, device="cuda", generator=g) for _ in range(2)]
    with torch.no_grad():
        got, want = traced(*x1), net(*x1)
    got = got if isinstance(got, (list, tuple)) else [got]
    want = want if isinstance(want, (list, tuple)) else [want]
    for a, b in zip(got, want):
        torch.testing.assert_close(a, b, rtol=0, atol=0)
    with torch.no_grad():
        first = traced(*x0)
    first = first if isinstance(first, (list, tuple)) else [first]
    assert not np.array_equal(got[-1].cpu().numpy(), first[-1].cpu().numpy())  # not a constant


@pytest.mark.gpu
@pytest.mark.parametrize("keep", [True, False])
def test_jit_trace_fused_volume_regression(keep):
    """The fused volume + soft-argmin as one traced node, volume kept or not."""
    from realtime_stereo_matcher_amd import functional as F

    class Net(torch.nn.Module):
        def forward(self, l, r):
            vol, disp = F.inner_product_soft_argmin(l, r, 96, keep_volume=keep)
            return disp if vol is None else (vol, disp)

    g = torch.Generator(device="cuda").manual_seed(5)
    l0, r0 = (torch.randn(1, 64, 8, 256, device="cuda", generator=g) for _ in range(2))
    with torch.no_grad():
        traced = torch.jit.trace(Net(), (l0, r0))
    name = "inner_product_soft_argmin" if keep else "inner_product_soft_argmin_novolume"
    assert f"stereocv::{name}" in str(traced.inlined_graph)
    l1, r1 = (torch.randn(1, 64, 8, 256, device="cuda", generator=g) for _ in range(2))
    with torch.no_grad():
        got, want = traced(l1, r1), Net()(l1, r1)
    got = got if isinstance(got, tuple) else (got,)
    want = want if isinstance(want, tuple) else (want,)
    for a, b in zip(got, want):
        torch.testing.assert_close(a, b, rtol=0, atol=0)


@pytest.mark.gpu
def test_autocast_decision_fixed_at_trace_time():
    """the fp32-output choice of the regression / fused / warp ops under autocast is
    an op argument taken when the graph is traced, so a graph traced under autocast returns what
    its fake kernels promised even when it later runs with autocast off (as a compiler that
    removed the autocast regions would run it)."""
    from realtime_stereo_matcher_amd import functional as F

    class Net(torch.nn.Module):
        def forward(self, l, r, v, img, fl):
            _, d = F.inner_product_soft_argmin(l, r, 96, keep_volume=False)
            return F.soft_argmin(v), d, F.warp_by_flow_map(img, fl)

    g = torch.Generator(device="cuda").manual_seed(9)
    args = (torch.randn(1, 32, 4, 128, device="cuda", generator=g).half(),
            torch.randn(1, 32, 4, 128, device="cuda", generator=g).half(),
            torch.randn(1, 24, 4, 40, device="cuda", generator=g).half(),
            torch.randn(1, 8, 4, 40, device="cuda", generator=g).half(),
            torch.rand(1, 1, 4, 40, device="cuda", generator=g).half())
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.float16):
        traced = torch.jit.trace(Net(), args)
        want = Net()(*args)
    assert all(t.dtype == torch.float32 for t in want)
    with torch.no_grad():  # autocast off at run time
        got = traced(*args)
    for a, b in zip(got, want):
        assert a.dtype == torch.float32
        torch.testing.assert_close(a, b, rtol=0, atol=0)
