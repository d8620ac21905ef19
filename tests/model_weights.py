"""Deterministic synthetic weights for the model-level demo fixtures (tests/test_model_demo.py,
tests/golden/gen_model_golden.py).  Written from a numpy PCG64 stream in sorted state_dict key
order, so the fixture only needs the seed, not the tensors (numpy's PCG64 output is stable)."""
import numpy as np
import torch


def seeded_state(state_dict, seed):
    """A state_dict of the same keys / shapes / dtypes: conv weights N(0, 1/fan_in), biases
    N(0, 0.05^2), BatchNorm weight U(0.75, 1.25), bias N(0, 0.1^2), running_mean N(0, 0.1^2),
    running_var U(0.75, 1.25); integer buffers copied."""
    rng = np.random.default_rng(seed)
    out = {}
    for k in sorted(state_dict):
        t = state_dict[k]
        if not t.is_floating_point():
            out[k] = t.clone()
            continue
        shape = tuple(t.shape)
        name = k.rsplit(".", 1)[-1]
        if name == "running_var" or (name == "weight" and len(shape) == 1):
            a = rng.uniform(0.75, 1.25, shape)
        elif name in ("running_mean", "bias") and len(shape) == 1 and ("bn" in k or _is_bn(state_dict, k)):
            a = rng.normal(0.0, 0.1, shape)
        elif name == "bias":
            a = rng.normal(0.0, 0.05, shape)
        else:
            fan_in = int(np.prod(shape[1:])) if len(shape) > 1 else 1
            a = rng.standard_normal(shape) / np.sqrt(fan_in)
        out[k] = torch.from_numpy(np.asarray(a, dtype=np.float32)).reshape(shape)
    return out


def _is_bn(sd, key):
    return key.rsplit(".", 1)[0] + ".running_mean" in sd
