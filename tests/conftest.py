import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN_DIR = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")


def load_manifest():
    with open(os.path.join(GOLDEN_DIR, "manifest.json")) as f:
        return json.load(f)


def load_case(rec):
    """Return {name: np.ndarray}; bf16 arrays are converted to float32 values."""
    from oracle.stereo_oracle import bf16_bits_to_f32

    z = np.load(os.path.join(GOLDEN_DIR, rec["file"]))  # allow_pickle=False (default)
    out = {}
    for k in z.files:
        a = z[k]
        if a.dtype == np.uint16 and rec["dtype"] == "bf16":
            a = bf16_bits_to_f32(a)
        out[k] = a
    return out


def cases(op):
    return [c for c in load_manifest()["cases"] if c["op"] == op]


@pytest.fixture(scope="session")
def manifest():
    return load_manifest()
