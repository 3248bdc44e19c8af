"""CPU: the augmentation oracle (oracle/augment_oracle.py) and the product's host-side rectangle
tables (conformer_amd/augment.py) against the reference modules' outputs (tests/golden/augment_*.npz)."""
import json
import os
import random

import numpy as np
import pytest

import augment_oracle as AO

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _case(name):
    z = np.load(os.path.join(GOLD, name + ".npz"))
    return z, json.loads(str(z["kwargs_json"]))


@pytest.mark.parametrize("name", ["augment_ctc_bpe", "augment_int_width"])
def test_oracle_spec_augment(name):
    z, kw = _case(name)
    y = AO.spec_augment(z["x"], z["lengths"], random.Random(int(z["seed"])), **kw)
    np.testing.assert_array_equal(y, z["y"])


def test_oracle_spec_cutout():
    z, kw = _case("augment_cutout")
    y = AO.spec_cutout(z["x"], random.Random(int(z["seed"])), **kw)
    np.testing.assert_array_equal(y, z["y"])


def _apply_rects(x, rects, value):
    y = x.copy()
    for b in range(rects.shape[0]):
        for f0, f1, t0, t1 in rects[b]:
            y[b, f0:f1, t0:t1] = value
    return y


@pytest.mark.parametrize("name", ["augment_ctc_bpe", "augment_int_width", "augment_cutout"])
def test_host_rectangle_tables(name):
    """The product draws mask geometry on the host (same random.Random call order) and ships one
    rectangle table; painting those rectangles must give the reference output exactly."""
    import torch
    from conformer_amd.augment import cutout_rects, spec_augment_rects
    z, kw = _case(name)
    rng = random.Random(int(z["seed"]))
    x = z["x"]
    if str(z["kind"]) == "SpecCutout":
        rects, value = cutout_rects(x.shape, rng, **kw), 0.0
    else:
        value = kw.pop("mask_value", 0.0)
        rects = spec_augment_rects(x.shape, torch.from_numpy(z["lengths"]), rng, **kw)
    assert rects.dtype == np.int32 and rects.shape[:1] == (x.shape[0],) and rects.shape[2] == 4
    np.testing.assert_array_equal(_apply_rects(x, rects, value), z["y"])


from hypothesis import given, settings, strategies as st  # noqa: E402


@settings(max_examples=60, deadline=None)
@given(B=st.integers(1, 4), F=st.integers(8, 96), T=st.integers(1, 300), fm=st.integers(0, 3), tm=st.integers(0, 6),
       fw=st.integers(0, 30), tw_int=st.integers(0, 40), tw_frac=st.floats(0.0, 1.0), use_frac=st.booleans(),
       seed=st.integers(0, 2 ** 31), data=st.data())
def test_host_rectangles_match_oracle_property(B, F, T, fm, tm, fw, tw_int, tw_frac, use_frac, seed, data):
    """For any SpecAugment configuration the host-drawn rectangle table paints exactly what the
    reference's slice-assignment loop writes (same random.Random call order), including the
    ValueError the reference raises when freq_width exceeds the feature count."""
    import torch
    from conformer_amd.augment import spec_augment_rects
    lengths = np.array(data.draw(st.lists(st.integers(0, T), min_size=B, max_size=B)), dtype=np.int64)
    x = np.random.default_rng(seed % 1000).standard_normal((B, F, T)).astype(np.float32)
    tw = float(tw_frac) if use_frac else tw_int
    try:
        want = AO.spec_augment(x, lengths, random.Random(seed), fm, tm, fw, tw, mask_value=-3.0)
    except ValueError:
        with pytest.raises(ValueError):
            spec_augment_rects(x.shape, torch.from_numpy(lengths), random.Random(seed), fm, tm, fw, tw)
        return
    rects = spec_augment_rects(x.shape, torch.from_numpy(lengths), random.Random(seed), fm, tm, fw, tw)
    np.testing.assert_array_equal(_apply_rects(x, rects, -3.0), want)
