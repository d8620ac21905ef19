"""§8f-3 model-level drop-in demo: MobileStereoNet (v1) with the HIP cost volume and soft-argmin
(realtime_stereo_matcher_amd/model/stereo_net_v1.py) against the reference network's own eval
outputs, recorded from a seeded-init reference model (tests/golden/gen_model_golden.py)."""
import os

import numpy as np
import pytest
import torch

FIX = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "model_msn_v1.npz")


def _fixture():
    return np.load(FIX)  # allow_pickle=False (default): data only


def _net(a):
    from realtime_stereo_matcher_amd.model.stereo_net_v1 import MobileStereoNetHIP

    net = MobileStereoNetHIP()
    sd = {k[3:]: torch.from_numpy(a[k]) for k in a.files if k.startswith("sd/")}
    net.load_state_dict(sd, strict=True)
    return net.eval()


def test_state_dict_matches_reference_layout():
    """CPU: the demo network takes the reference network's state_dict unchanged."""
    _net(_fixture())


@pytest.mark.gpu
def test_model_outputs_match_reference():
    """GPU: all three refinement outputs within 2e-3 px of the reference's (|disp| ~ 65..105 px
    at full resolution; the difference is MIOpen-vs-CPU convolution rounding through 3 stages)."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    a = _fixture()
    net = _net(a).cuda()
    with torch.no_grad():
        outs = net(torch.from_numpy(a["left"]).cuda(), torch.from_numpy(a["right"]).cuda())
    assert len(outs) == 3
    for i, o in enumerate(outs):
        ref = a[f"out{i}"]
        assert tuple(o.shape) == ref.shape
        np.testing.assert_allclose(o.float().cpu().numpy(), ref, atol=2e-3, rtol=0)
