import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "conformer-nemo_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests", "golden"),
          ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X); run with -m gpu")
    config.addinivalue_line("markers", "slow: multi-second CPU work")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


def rel_l2(a, b):
    import numpy as np
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def max_rel(a, b):
    import numpy as np
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


def summary_err(key, a, z, prefix, floor_norm=0.0):
    """Compare a full tensor with a fixture summary written by tests/golden/gen_large_goldens.py
    (L2 norm, values at seeded positions, dot products with 2 seeded directions).  Errors are taken
    relative to N = max(ref norm, floor_norm) (floor_norm: for analytically ~zero tensors, e.g. the
    depthwise-conv bias gradient under train-mode BatchNorm): returns (||sampled err|| / max(||ref
    samples||, 1e-2 N sqrt(samples / n)), |norm - ref| / N, max |proj - ref| / N)."""
    import numpy as np
    from gen_large_goldens import summary_spec
    flat = np.asarray(a, dtype=np.float64).reshape(-1)
    idx, dirs = summary_spec(key, flat.size)
    samp, norm, proj = z[f"{prefix}{key}__samp"].astype(np.float64), float(z[f"{prefix}{key}__norm"]), z[f"{prefix}{key}__proj"]
    N = max(norm, floor_norm, 1e-30)
    floor = 1e-2 * N * np.sqrt(len(idx) / flat.size)
    e_s = float(np.linalg.norm(flat[idx] - samp) / max(np.linalg.norm(samp), floor, 1e-30))
    e_n = abs(float(np.linalg.norm(flat)) - norm) / N
    e_p = float(np.abs(dirs.astype(np.float64) @ flat - proj).max() / N)
    return e_s, e_n, e_p
