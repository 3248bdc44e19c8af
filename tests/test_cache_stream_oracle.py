"""CPU checks of the cache-aware streaming definition (oracle/cache_aware_oracle.py).
Parity unpinned (no reference counterpart): these tests pin the DEFINITION's own consistency -
the chunked computation with carried state equals the full-sequence causal forward for several
chunk sizes / left contexts, the model is causal, and with infinite context and a 1-frame kernel
the causal changes reduce to the pinned oracle's arithmetic where they must."""
import numpy as np
import pytest

import cache_aware_oracle as CA
from conftest import rel_l2
from recipe import make_state_dict

CFG = dict(feat_in=16, n_layers=2, d_model=32, n_heads=4, conv_kernel_size=7, xscaling=True, pos_emb_max_len=512)


def _inputs(B, T, seed=3):
    return np.random.default_rng(seed).standard_normal((B, CFG["feat_in"], T)).astype(np.float32)


@pytest.mark.parametrize("chunk,left", [(1, 3), (2, 5), (4, 4), (3, 16)])
def test_chunked_equals_full_causal(chunk, left):
    sd = make_state_dict(CFG, 5)
    x = _inputs(2, 4 * chunk * 4)
    full = CA.causal_forward(x, sd, CFG, left, dtype=np.float64)
    ch = CA.chunked_forward(x, sd, CFG, left, chunk, dtype=np.float64)
    assert full.shape == ch.shape == (2, 32, 4 * chunk)
    assert rel_l2(ch, full) <= 1e-12


def test_layer_norm_conv_variant():
    cfg = dict(CFG, conv_norm_type="layer_norm")
    sd = make_state_dict(cfg, 6)
    x = _inputs(1, 32)
    assert rel_l2(CA.chunked_forward(x, sd, cfg, 6, 2, dtype=np.float64),
                  CA.causal_forward(x, sd, cfg, 6, dtype=np.float64)) <= 1e-12


def test_causal_future_frames_do_not_matter():
    sd = make_state_dict(CFG, 5)
    x = _inputs(1, 48)
    y = CA.causal_forward(x, sd, CFG, 8, dtype=np.float64)
    x2 = x.copy()
    x2[:, :, 24:] = _inputs(1, 24, seed=9)          # change input frames >= 24 (encoder frames >= 6)
    y2 = CA.causal_forward(x2, sd, CFG, 8, dtype=np.float64)
    np.testing.assert_array_equal(y[:, :, :6], y2[:, :, :6])
    assert np.abs(y[:, :, 6:] - y2[:, :, 6:]).max() > 1e-3


def test_left_context_limits_history():
    sd = make_state_dict(CFG, 5)
    x = _inputs(1, 64)
    y = CA.causal_forward(x, sd, CFG, 2, dtype=np.float64)
    x2 = x.copy()
    x2[:, :, :4] += 1.0                                 # perturb encoder frame 0's input only
    y2 = CA.causal_forward(x2, sd, CFG, 2, dtype=np.float64)
    # receptive field of frame t: conv taps (K-1 = 6 frames back per layer, 2 layers) and 2 frames of
    # attention per layer -> frames >= 1 + 2 * (6 + 2) + 1 are unaffected
    np.testing.assert_array_equal(y[:, :, 18:], y2[:, :, 18:])
    assert np.abs(y[:, :, 0] - y2[:, :, 0]).max() > 1e-3
