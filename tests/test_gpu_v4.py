"""§8f-2 / §8f-3: MobileStereoNetV4's interweave + Conv3d cost volume as one HIP operator
(csrc/v4_volume.hip) against the reference loop's own outputs (tests/golden/v4_volume_*.npz,
model/mobile_stereo_net_v4.py:443-461) and the fp64 oracle restatement
(oracle/stereo_oracle.py:v4_volume)."""
import os

import numpy as np
import pytest
import torch

from oracle import stereo_oracle as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
V4_FILES = sorted(f for f in os.listdir(GOLDEN) if f.startswith("v4_volume_"))
TOL = 1e-4

pytestmark = pytest.mark.gpu


def _stacks(params=None, seed=0):
    """conv3d / volume11 modules in the reference layout (mobile_stereo_net_v4.py:317-335), loaded
    from a fixture's parameters or seeded (random BatchNorm statistics), in eval mode."""
    from realtime_stereo_matcher_amd.model.stereo_net_v4 import MobileStereoNetV4HIP

    net = MobileStereoNetV4HIP(192)
    c3d, v11 = net.conv3d, net.volume11
    if params is not None:
        c3d.load_state_dict({k[7:]: torch.from_numpy(v) for k, v in params.items() if k.startswith("conv3d.")})
        v11.load_state_dict({k[9:]: torch.from_numpy(v) for k, v in params.items() if k.startswith("volume11.")})
    else:
        g = torch.Generator().manual_seed(seed)
        with torch.no_grad():
            for m in list(c3d.modules()) + list(v11.modules()):
                if isinstance(m, (torch.nn.Conv3d, torch.nn.Conv2d)):
                    m.weight.copy_(torch.randn(m.weight.shape, generator=g) * (2.0 / m.weight[0].numel()) ** 0.5)
                    if m.bias is not None:
                        m.bias.copy_(torch.randn(m.bias.shape, generator=g) * 0.05)
                elif isinstance(m, (torch.nn.BatchNorm2d, torch.nn.BatchNorm3d)):
                    m.running_mean.copy_(torch.randn(m.running_mean.shape, generator=g) * 0.1)
                    m.running_var.copy_(torch.rand(m.running_var.shape, generator=g) * 0.5 + 0.75)
                    m.weight.copy_(torch.rand(m.weight.shape, generator=g) * 0.5 + 0.75)
                    m.bias.copy_(torch.randn(m.bias.shape, generator=g) * 0.1 + 0.05)
    return c3d.cuda().eval(), v11.cuda().eval()


def _params(c3d, v11):
    p = {f"conv3d.{k}": v.detach().cpu().numpy() for k, v in c3d.state_dict().items()}
    p.update({f"volume11.{k}": v.detach().cpu().numpy() for k, v in v11.state_dict().items()})
    return p


@pytest.mark.parametrize("name", V4_FILES)
def test_v4_volume_golden(name):
    """The fused HIP volume and the MIOpen batched form against the reference loop's output."""
    from realtime_stereo_matcher_amd.model.mobile_stereo_net_v4 import interweave_conv_volume

    a = np.load(os.path.join(GOLDEN, name))
    p = {k[2:]: a[k] for k in a.files if k.startswith("p/")}
    c3d, v11 = _stacks(p)
    L, R = torch.from_numpy(a["featL"]).cuda(), torch.from_numpy(a["featR"]).cuda()
    with torch.no_grad():
        got = interweave_conv_volume(L, R, c3d, v11, 48)
        ref_t = interweave_conv_volume(L, R, c3d, v11, 48, impl="torch")
    assert got.shape == a["volume"].shape and got.dtype == torch.float32
    np.testing.assert_allclose(got.cpu().numpy(), a["volume"], atol=TOL, rtol=0)
    np.testing.assert_allclose(ref_t.cpu().numpy(), a["volume"], atol=TOL, rtol=0)


V4_SHAPES = [(1, 32, 1, 31, 48), (2, 32, 3, 64, 48), (1, 32, 50, 47, 48), (1, 32, 4, 40, 48),
             (1, 32, 2, 100, 7), (1, 32, 7, 91, 60)]


@pytest.mark.parametrize("shape", V4_SHAPES, ids=str)
def test_v4_volume_vs_oracle(shape):
    """Single rows, many row bands (H = 50), W < D (empty planes), partial strips, D != 48."""
    from realtime_stereo_matcher_amd import functional as F
    from realtime_stereo_matcher_amd.model.mobile_stereo_net_v4 import fold_v4_weights

    n, c, h, w, D = shape
    c3d, v11 = _stacks(seed=hash(shape) % 1000)
    rng = np.random.default_rng(5)
    fl = rng.standard_normal((n, c, h, w)).astype(np.float32)
    fr = rng.standard_normal((n, c, h, w)).astype(np.float32)
    with torch.no_grad():
        got = F.v4_volume(torch.from_numpy(fl).cuda(), torch.from_numpy(fr).cuda(),
                          *fold_v4_weights(c3d, v11), D).cpu().numpy()
    want = O.v4_volume(fl, fr, _params(c3d, v11), D)
    np.testing.assert_allclose(got, want, atol=TOL, rtol=0)
    tri = np.arange(w)[None, :] < np.arange(D)[:, None]
    assert not got.transpose(0, 2, 1, 3)[:, :, tri].any()


def test_v4_volume_strided_and_errors():
    from realtime_stereo_matcher_amd import functional as F
    from realtime_stereo_matcher_amd.model.mobile_stereo_net_v4 import fold_v4_weights

    c3d, v11 = _stacks(seed=3)
    ws = fold_v4_weights(c3d, v11)
    big = torch.randn(2, 40, 3, 70, device="cuda")
    L, R = big[:, :32], big[:, 8:]  # channel-sliced views (non-contiguous N stride)
    with torch.no_grad():
        got = F.v4_volume(L, R, *ws, 48)
        ref = F.v4_volume(L.contiguous(), R.contiguous(), *ws, 48)
    assert torch.equal(got, ref)
    with pytest.raises(RuntimeError, match="C = 32"):
        F.v4_volume(big[:, :16], big[:, :16], *ws, 48)
    with pytest.raises(TypeError):
        F.v4_volume(L.half(), R.half(), *ws, 48)


def test_v4_volume_network_shape_sampled_rows():
    """The V4 network's own volume shape (1x32x96x312, D = 48: KITTI-like 384x1248 input at 1/4
    resolution, model/mobile_stereo_net_v4.py:443-461): sampled rows against the fp64 oracle.
    Row y depends on feature rows y-3 .. y+3 (three 3x3 layers), so the oracle runs on that band;
    the band's own edges are the image's edges only at y = 0 and y = H-1, where that is exact."""
    from realtime_stereo_matcher_amd import functional as F
    from realtime_stereo_matcher_amd.model.mobile_stereo_net_v4 import fold_v4_weights

    n, c, h, w, D = 1, 32, 96, 312, 48
    c3d, v11 = _stacks(seed=17)
    g = torch.Generator(device="cuda").manual_seed(9)
    L = torch.randn(n, c, h, w, device="cuda", generator=g)
    R = torch.randn(n, c, h, w, device="cuda", generator=g)
    with torch.no_grad():
        got = F.v4_volume(L, R, *fold_v4_weights(c3d, v11), D).cpu().numpy()
    fl, fr = L.cpu().numpy(), R.cpu().numpy()
    p = _params(c3d, v11)
    for y in (0, 1, 47, 94, 95):
        y0, y1 = max(0, y - 3), min(h, y + 4)
        want = O.v4_volume(fl[:, :, y0:y1], fr[:, :, y0:y1], p, D)[:, :, y - y0]
        np.testing.assert_allclose(got[:, :, y], want, atol=TOL, rtol=0)
