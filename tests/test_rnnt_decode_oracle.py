"""CPU: the prediction-network / greedy-decoding oracle (oracle/rnnt_decode_oracle.py) against the
REFERENCE RNNTDecoder / GreedyBatchedRNNTInfer outputs (tests/golden/rnnt_decode_*.npz)."""
import glob
import os

import numpy as np
import pytest

import rnnt_decode_oracle as RD

FILES = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "rnnt_decode_*.npz")))


def _sds(z):
    d = {k[4:]: z[k] for k in z.files if k.startswith("dec/")}
    j = {k[6:]: z[k] for k in z.files if k.startswith("joint/")}
    return d, j


@pytest.mark.parametrize("path", FILES, ids=[os.path.basename(f)[:-4] for f in FILES])
def test_predict_matches_reference(path):
    z = np.load(path)
    d, _ = _sds(z)
    L = int(z["L"])
    g, (h, c) = RD.predict(d, L, z["y"])
    np.testing.assert_allclose(g.transpose(0, 2, 1), z["pred_g"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(h, z["pred_h"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(c, z["pred_c"], rtol=1e-5, atol=1e-6)
    g2, (h2, c2) = RD.predict(d, L, z["y"], z["h0"], z["c0"], add_sos=False)
    np.testing.assert_allclose(g2, z["pred2_g"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(h2, z["pred2_h"], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("path", FILES, ids=[os.path.basename(f)[:-4] for f in FILES])
def test_greedy_matches_reference(path):
    z = np.load(path)
    d, j = _sds(z)
    V = int(z["V"])
    res, has_state = RD.greedy_decode(d, j, int(z["L"]), str(z["activation"]), z["enc"], z["enc_len"], V,
                                      int(z["max_symbols"]), log_normalize=True)   # CPU reference log-normalises
    assert has_state == bool(z["has_state"])
    for b, (toks, steps, score, h, c) in enumerate(res):
        n = int(z["ntok"][b])
        assert toks == z["tokens"][b, :n].tolist() and steps == z["timesteps"][b, :n].tolist()
        assert abs(score - z["scores"][b]) <= 1e-4 * max(1.0, abs(z["scores"][b]))
        if has_state:
            np.testing.assert_allclose(h, z["final_h"][:, b], rtol=1e-5, atol=1e-6)
            np.testing.assert_allclose(c, z["final_c"][:, b], rtol=1e-5, atol=1e-6)
