"""CPU: the RNN-T loss oracle (GPU-kernel formulas, oracle/rnnt_loss_oracle.py) reproduces the
reference's numpy RNN-T loss costs and gradients (tests/golden/rnnt_loss_*.npz)."""
import glob
import os

import numpy as np
import pytest

import rnnt_loss_oracle as RO
from conftest import GOLDEN

FILES = sorted(glob.glob(os.path.join(GOLDEN, "rnnt_loss_*.npz")))


@pytest.mark.parametrize("path", FILES, ids=[os.path.basename(f) for f in FILES])
def test_oracle_matches_reference(path):
    z = np.load(path)
    c, g = RO.rnnt_loss(z["acts"], z["labels"], z["act_lens"], z["label_lens"], int(z["blank"]),
                        float(z["fastemit_lambda"]), float(z["clamp"]))
    # the reference keeps its lattices in float32 (rnnt_numpy.py:127, 158): measured cost rel. error
    # <= 2.9e-5 at U=11, T=13; gradient abs. error <= 2.8e-5
    np.testing.assert_allclose(c, z["costs"], rtol=1e-4, atol=0)
    np.testing.assert_allclose(g, z["grads"], rtol=0, atol=5e-5 * max(1.0, np.abs(z["grads"]).max()))
