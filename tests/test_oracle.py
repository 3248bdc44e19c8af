"""Pins the numpy oracle (oracle/conformer_oracle.py) to the reference's own outputs.

The fixtures under tests/golden/ were produced by running the reference encoder
(tests/golden/gen_goldens.py).  The reference ships no tests or golden vectors of its own
(SURVEY §4), so these reference-generated fixtures are the only pin.
"""
import glob
import json
import os

import numpy as np
import pytest

import conformer_oracle as O
from conftest import GOLDEN, rel_l2
from recipe import encoder_param_shapes, make_state_dict

ENC_FILES = sorted(glob.glob(os.path.join(GOLDEN, "enc_*.npz")))
FAST = [f for f in ENC_FILES if "large17.npz" not in f]


def test_calc_length_matches_reference():
    z = np.load(os.path.join(GOLDEN, "calc_length.npz"))
    np.testing.assert_array_equal(O.calc_length(z["lengths"]), z["out"])


def test_rel_shift_matches_reference():
    z = np.load(os.path.join(GOLDEN, "rel_shift.npz"))
    np.testing.assert_array_equal(O.rel_shift(z["x"]), z["out"])


def test_rel_shift_is_the_skewed_gather():
    """rel_shift(x)[..., i, j] == x[..., i, T-1-i+j] for j < T (the identity the fused kernel uses)."""
    rng = np.random.default_rng(0)
    for T in (1, 2, 5, 17):
        x = rng.standard_normal((2, 3, T, 2 * T - 1)).astype(np.float32)
        y = O.rel_shift(x)[..., :T]
        i = np.arange(T)[:, None]
        j = np.arange(T)[None, :]
        np.testing.assert_array_equal(y, x[..., i, T - 1 - i + j])


def test_rel_positional_encoding_matches_reference():
    z = np.load(os.path.join(GOLDEN, "rel_pe.npz"))
    pe, center = O.rel_pe_table(5000, 64)
    x, pos = O.rel_positional_encoding(z["x"], pe, center, 8.0)
    assert rel_l2(x, z["x_out"]) < 1e-7
    assert rel_l2(pos, z["pos_emb"]) < 1e-6


def test_recipe_reproduces_stored_weights():
    for name in ("enc_tiny.npz", "enc_tiny_dk10.npz"):
        z = np.load(os.path.join(GOLDEN, name))
        cfg = json.loads(str(z["cfg_json"]))
        sd = make_state_dict(cfg, int(z["seed"]))
        for k, v in sd.items():
            np.testing.assert_array_equal(v, z["w/" + k])


@pytest.mark.parametrize("path", FAST, ids=[os.path.basename(f) for f in FAST])
def test_oracle_encoder_matches_reference(path):
    z = np.load(path)
    cfg = json.loads(str(z["cfg_json"]))
    sd = make_state_dict(cfg, int(z["seed"]))
    y, yl = O.encoder_forward(z["x"], z["lengths"], sd, cfg)
    np.testing.assert_array_equal(yl, z["y_len"])
    assert y.shape == z["y"].shape
    assert rel_l2(y, z["y"]) < 2e-6


@pytest.mark.slow
def test_oracle_large17_matches_reference():
    z = np.load(os.path.join(GOLDEN, "enc_large17.npz"))
    cfg = json.loads(str(z["cfg_json"]))
    y, yl = O.encoder_forward(z["x"], z["lengths"], make_state_dict(cfg, int(z["seed"])), cfg)
    np.testing.assert_array_equal(yl, z["y_len"])
    assert rel_l2(y, z["y"]) < 2e-6


def test_flop_formula():
    """Large-17 B=32 T=1000 = 2632.6 GFLOP; cfg1 = 7.4 GFLOP."""
    assert abs(O.encoder_flops(32, 1000, 512, 17) / 1e9 - 2632.6) < 0.1
    assert abs(O.encoder_flops(4, 200, 176, 16) / 1e9 - 7.4) < 0.05


def test_recipe_keys_cover_reference_layout():
    keys = [k for k, _ in encoder_param_shapes(dict(d_model=512, n_heads=8, n_layers=17))]
    assert len(keys) == 686
