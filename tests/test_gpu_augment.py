"""GPU parity of the on-device spectrogram augmentation (include/cfm_augment.h)
against the REFERENCE modules' outputs (tests/golden/augment_*.npz, gen_augment_goldens.py):
bit-exact for SpecAugment / SpecCutout / SpectrogramAugmentation under the same seeds."""
import json
import os
import random

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _case(name):
    z = np.load(os.path.join(GOLD, name + ".npz"))
    return z, json.loads(str(z["kwargs_json"]))


@pytest.mark.parametrize("name", ["augment_ctc_bpe", "augment_int_width"])
def test_spec_augment_matches_reference(name):
    from nemo.collections.asr.parts.submodules.spectr_augment import SpecAugment
    z, kw = _case(name)
    m = SpecAugment(rng=random.Random(int(z["seed"])), **kw)
    x = torch.from_numpy(z["x"]).cuda()
    y = m(input_spec=x, length=torch.from_numpy(z["lengths"]).cuda())
    assert y is x                                   # in place, as the reference
    np.testing.assert_array_equal(y.cpu().numpy(), z["y"])


def test_spec_cutout_matches_reference():
    from nemo.collections.asr.parts.submodules.spectr_augment import SpecCutout
    z, kw = _case("augment_cutout")
    m = SpecCutout(rng=random.Random(int(z["seed"])), **kw)
    x = torch.from_numpy(z["x"]).cuda()
    np.testing.assert_array_equal(m(input_spec=x).cpu().numpy(), z["y"])


def test_spectrogram_augmentation_choice_sequence():
    from nemo.collections.asr.modules import SpectrogramAugmentation
    z, kw = _case("augment_choice")
    seed = int(z["seed"])
    random.seed(seed)
    m = SpectrogramAugmentation(rng=random.Random(seed), **kw)
    ln = torch.from_numpy(z["lengths"]).cuda()
    for i in range(z["y"].shape[0]):
        x = torch.from_numpy(z["x"]).cuda()
        np.testing.assert_array_equal(m(input_spec=x, length=ln).cpu().numpy(), z["y"][i])


def test_non_contiguous_input_is_masked_in_place():
    from nemo.collections.asr.parts.submodules.spectr_augment import SpecAugment
    z, kw = _case("augment_int_width")
    base = torch.from_numpy(np.ascontiguousarray(z["x"].transpose(0, 2, 1))).cuda()
    x = base.transpose(1, 2)                        # (B, F, T) view, not contiguous
    m = SpecAugment(rng=random.Random(int(z["seed"])), **kw)
    m(input_spec=x, length=torch.from_numpy(z["lengths"]).cuda())
    np.testing.assert_array_equal(base.transpose(1, 2).cpu().numpy(), z["y"])


def test_spec_shot_distribution_and_determinism():
    from nemo.collections.asr.parts.submodules.spectr_augment import SpecShot
    g = np.load(os.path.join(GOLD, "augment_specshot.npz"))
    ratio = float(g["mask_ratio"])
    x = torch.randn(8, 80, 501, device="cuda")      # odd element count exercises the tail
    torch.manual_seed(0)
    y = SpecShot(mask_ratio=ratio)(input_spec=x)
    torch.manual_seed(0)
    y2 = SpecShot(mask_ratio=ratio)(input_spec=x)
    assert torch.equal(y, y2)
    kept = (y != 0).double().mean().item()
    # the reference's kept fraction at the same ratio (torch CPU generator) is g["kept"]; both are
    # Binomial(n, 0.7)/n with n = 320k: 5 sigma ~ 0.004
    assert abs(kept - (1 - ratio)) < 4e-3 and abs(kept - float(g["kept"])) < 6e-3
    keep = y != 0
    assert torch.equal(y[keep], x[keep])
    tail = (y[..., -1] != 0).double().mean().item()  # the tail elements are masked too
    assert 0.5 < tail < 0.9


def test_empty_config_is_identity_and_cpu_is_refused():
    from nemo.collections.asr.modules import SpectrogramAugmentation
    from nemo.collections.asr.parts.submodules.spectr_augment import SpecCutout
    x = torch.randn(2, 80, 50, device="cuda")
    assert SpectrogramAugmentation()(input_spec=x, length=torch.tensor([50, 40], device="cuda")) is x
    with pytest.raises(RuntimeError):
        SpecCutout(rect_masks=2)(input_spec=torch.zeros(1, 80, 50))
