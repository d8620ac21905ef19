"""Model-level golden vectors for the §8f-3 drop-in demo (CONTAINER-ONLY).

Imports the reference networks ``MobileStereoNet`` (model/mobile_stereo_net.py:89-158) and
``MobileStereoNetV2`` (model/mobile_stereo_net_v2.py:136-232), ``MobileStereoNetV3``
(model/mobile_stereo_net_v3.py:249-336), ``MobileDispNetC`` (model/mobile_disp_net_c.py:237-412)
and ``MobileStereoNetV4`` (model/mobile_stereo_net_v4.py:291-524; plus its cost-volume loop alone,
:443-461, in ``v4_volume_*.npz``),
with the parameters of their configure/*.json, from
``/root/reference`` at run time (``python3 -B``), builds it with a seeded random init (no
checkpoint ships with the reference), randomises the BatchNorm statistics so eval mode is not an
identity, and records in ``model_msn_v{1,2,3}.npz`` / ``model_dispnetc.npz``: the state_dict (``sd/<key>``), a left/right image
pair of 1x3x60x90 (not a multiple of 8: exercises the reference padding) and the reference's
three eval-mode outputs on CPU.  Only data is written.

Usage:  cd /root/repo && python3 -B tests/golden/gen_model_golden.py
"""
import importlib.util
import os
import sys

import numpy as np
import torch

REF = "/root/reference"
OUT_DIR = os.path.dirname(os.path.abspath(__file__))
V2_PARAMS = {"down_factor": 3, "max_disp": 192, "refine_dim": 7,
             "refine_dilates": [1, 2, 4, 8, 1, 1], "hidden_dim": 32}  # stereo_net_config_v2.json
DNC_PARAMS = {"hidden_dim": 8, "max_disp": 192, "with_batch_norm": True}  # disp_net_c_config.json
V3_PARAMS = {"down_factor": 3, "max_disp": 192, "refine_dilates": [1, 2, 4, 8, 1, 1],
             "hidden_dim": 32}  # stereo_net_config_v3.json
sys.dont_write_bytecode = True


def _load(path, name):
    spec = importlib.util.spec_from_file_location(name, os.path.join(REF, path))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def record(net, out_name, hw=(60, 90), weight_seed=None):
    """weight_seed: load synthetic weights from tests/model_weights.seeded_state instead of
    storing the state_dict (keeps the larger networks' fixtures small)."""
    torch.manual_seed(0)
    g = torch.Generator().manual_seed(1)
    if weight_seed is not None:
        sys.path.insert(0, os.path.dirname(OUT_DIR))
        from model_weights import seeded_state

        net.load_state_dict(seeded_state(net.state_dict(), weight_seed))
    with torch.no_grad():
        for m in net.modules() if weight_seed is None else ():
            if isinstance(m, (torch.nn.BatchNorm2d, torch.nn.BatchNorm3d)):
                m.running_mean.copy_(torch.randn(m.running_mean.shape, generator=g) * 0.1)
                m.running_var.copy_(torch.rand(m.running_var.shape, generator=g) * 0.5 + 0.75)
                m.weight.copy_(torch.rand(m.weight.shape, generator=g) * 0.5 + 0.75)
                m.bias.copy_(torch.randn(m.bias.shape, generator=g) * 0.1)
    net.eval()
    rng = np.random.default_rng(7)
    left = rng.uniform(0, 255, (1, 3) + tuple(hw)).astype(np.float32)
    right = np.roll(left, -5, axis=3) + rng.normal(0, 2, left.shape).astype(np.float32)  # ~5 px shift
    with torch.no_grad():
        outs = net(torch.from_numpy(left), torch.from_numpy(right))
    arrays = ({f"sd/{k}": v.detach().numpy() for k, v in net.state_dict().items()}
              if weight_seed is None else {"weight_seed": np.array(weight_seed)})
    arrays.update(left=left, right=right.astype(np.float32))
    for i, o in enumerate(outs):
        arrays[f"out{i}"] = o.numpy()
    out = os.path.join(OUT_DIR, out_name)
    np.savez_compressed(out, **arrays)
    print(f"wrote {out}: {len(arrays)} arrays, outputs {[tuple(o.shape) for o in outs]}")


def record_v4_volume(v4_mod, shape, seed, out_name):
    """§8f-2 fixture: the reference V4 cost-volume loop (model/mobile_stereo_net_v4.py:443-461)
    on seeded (N, 32, H, W) features with the seeded-init conv3d / volume11 stacks (:317-335,
    BatchNorm statistics randomised); stores their parameters (``p/<module>.<key>``), the inputs
    and the (N, 48, H, W) volume."""
    torch.manual_seed(seed)
    net = v4_mod.MobileStereoNetV4(192)
    g = torch.Generator().manual_seed(seed + 1)
    with torch.no_grad():
        for m in list(net.conv3d.modules()) + list(net.volume11.modules()):
            if isinstance(m, (torch.nn.BatchNorm2d, torch.nn.BatchNorm3d)):
                m.running_mean.copy_(torch.randn(m.running_mean.shape, generator=g) * 0.1)
                m.running_var.copy_(torch.rand(m.running_var.shape, generator=g) * 0.5 + 0.75)
                m.weight.copy_(torch.rand(m.weight.shape, generator=g) * 0.5 + 0.75)
                m.bias.copy_(torch.randn(m.bias.shape, generator=g) * 0.1 + 0.05)
    net.eval()
    rng = np.random.default_rng(seed)
    fl = rng.standard_normal(shape).astype(np.float32)
    fr = rng.standard_normal(shape).astype(np.float32)
    L, R = torch.from_numpy(fl), torch.from_numpy(fr)
    B, C, H, W = shape
    vol = L.new_zeros([B, 1, net.volume_size, H, W])
    with torch.no_grad():
        for i in range(net.volume_size):  # the reference loop, verbatim semantics
            x = v4_mod.interweave_tensors(L[:, :, :, i:], R[:, :, :, :-i]) if i > 0 else \
                v4_mod.interweave_tensors(L, R)
            x = net.volume11(torch.squeeze(net.conv3d(torch.unsqueeze(x, 1)), 2))
            vol[:, :, i, :, i:] = x
    arrays = {f"p/conv3d.{k}": v.numpy() for k, v in net.conv3d.state_dict().items()}
    arrays.update({f"p/volume11.{k}": v.numpy() for k, v in net.volume11.state_dict().items()})
    arrays.update(featL=fl, featR=fr, volume=vol.squeeze(1).numpy())
    out = os.path.join(OUT_DIR, out_name)
    np.savez_compressed(out, **arrays)
    print(f"wrote {out}: volume {tuple(vol.squeeze(1).shape)}, "
          f"{float((vol > 0).float().mean()):.2f} of the cells positive")


def main():
    torch.manual_seed(0)
    record(_load("model/mobile_stereo_net.py", "ref_msn").MobileStereoNet(), "model_msn_v1.npz")
    torch.manual_seed(0)
    record(_load("model/mobile_stereo_net_v2.py", "ref_msn_v2").MobileStereoNetV2(**V2_PARAMS),
           "model_msn_v2.npz")
    torch.manual_seed(0)
    record(_load("model/mobile_stereo_net_v3.py", "ref_msn_v3").MobileStereoNetV3(**V3_PARAMS),
           "model_msn_v3.npz")
    torch.manual_seed(0)
    # 100 x 200 pads to 128 x 256: conv2 features 16 x 32 x 64, correlation D = 48 < W = 64
    record(_load("model/mobile_disp_net_c.py", "ref_dnc").MobileDispNetC(**DNC_PARAMS),
           "model_dispnetc.npz", hw=(100, 200), weight_seed=11)
    v4 = _load("model/mobile_stereo_net_v4.py", "ref_msn_v4")
    torch.manual_seed(0)
    # 64 x 256 input: 1/4-res features 16 x 64 (W > volume_size 48, H and W divisible by 16)
    record(v4.MobileStereoNetV4(192), "model_msn_v4.npz", hw=(64, 256), weight_seed=13)
    record_v4_volume(v4, (1, 32, 6, 70), 21, "v4_volume_1x32x6x70_d48_f32.npz")
    record_v4_volume(v4, (2, 32, 5, 53), 22, "v4_volume_2x32x5x53_d48_f32.npz")


if __name__ == "__main__":
    main()
