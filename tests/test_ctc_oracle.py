"""The CTC oracle (oracle/ctc_oracle.py) against the reference's own CTCLoss / ConvASRDecoder
expression (tests/golden/ctc_*.npz, from tests/golden/gen_ctc_goldens.py)."""
import glob
import os

import numpy as np
import pytest

import ctc_oracle as CO
from conftest import GOLDEN, rel_l2

CASES = sorted(glob.glob(os.path.join(GOLDEN, "ctc_*.npz")))


@pytest.mark.parametrize("path", CASES, ids=[os.path.basename(p)[:-4] for p in CASES])
def test_ctc_oracle_matches_reference(path):
    z = np.load(path)
    lp, greedy = CO.head_forward(z["enc"], z["w"], z["b"])
    assert rel_l2(lp, z["log_probs"]) < 1e-6
    np.testing.assert_array_equal(greedy, z["greedy"])
    nll, g = CO.ctc_loss(z["log_probs"], z["targets"], z["in_len"], z["tgt_len"], int(z["blank"]))
    np.testing.assert_allclose(nll, z["nll"], rtol=1e-5, atol=1e-4)
    B = lp.shape[0]
    np.testing.assert_allclose(nll.mean(), float(z["loss"]), rtol=1e-5)
    assert rel_l2(g / B, z["grad_lp"]) < 1e-5
    denc, dw, db = CO.head_backward(z["enc"], z["w"], z["log_probs"], z["grad_lp"].astype(np.float64))
    assert rel_l2(denc, z["grad_enc"]) < 1e-5
    assert rel_l2(dw, z["grad_w"]) < 1e-5
    assert rel_l2(db, z["grad_b"]) < 1e-5


def test_golden_covers_edge_cases():
    z = np.load(os.path.join(GOLDEN, "ctc_small.npz"))
    assert (z["tgt_len"] == 0).any()                       # empty target
    assert float(z["nll"].min()) == 0.0                    # an infeasible utterance, zero_infinity'd
    assert (z["in_len"] < z["log_probs"].shape[1]).any()   # ragged inputs
