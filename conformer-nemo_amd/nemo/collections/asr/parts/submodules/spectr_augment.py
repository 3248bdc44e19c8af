"""Drop-in SpecAugment / SpecCutout / SpecShot (reference
nemo/collections/asr/parts/submodules/spectr_augment.py:24-184), SURVEY §8 row f4.

Same constructors and keyword-only forwards.  The masks are painted on the device by libcfm.so
(include/cfm_augment.h); the mask geometry comes from the module's `random.Random` in the
reference's call order, so a seeded rng reproduces the reference's masks bit for bit
(tests/golden/augment_*.npz).  SpecAugment and SpecCutout modify `input_spec` in place and return
it, as the reference does; SpecShot returns a new tensor.  Differences by design: SpecShot's
per-element uniforms come from a device counter hash seeded from torch's default CPU generator
(the reference draws them with torch.rand on the CPU), so it matches the reference in distribution
only; inputs must be float32 CUDA tensors (there is no CPU path).
"""
from __future__ import annotations

import random

import torch
import torch.nn as nn

from conformer_amd import augment as _aug
from nemo.core.classes.common import Typing, typecheck
from nemo.core.neural_types import LengthsType, NeuralType, SpectrogramType

__all__ = ["SpecAugment", "SpecCutout", "SpecShot"]


class SpecAugment(nn.Module, Typing):
    """Frequency and time masks (spectr_augment.py:24-105); time_width int = absolute, float in
    [0, 1] = fraction of each utterance's length."""

    @property
    def input_types(self):
        return {"input_spec": NeuralType(("B", "D", "T"), SpectrogramType()),
                "length": NeuralType(tuple("B"), LengthsType())}

    @property
    def output_types(self):
        return {"augmented_spec": NeuralType(("B", "D", "T"), SpectrogramType())}

    def __init__(self, freq_masks=0, time_masks=0, freq_width=10, time_width=10, rng=None, mask_value=0.0):
        super().__init__()
        self._rng = random.Random() if rng is None else rng
        self.freq_masks = freq_masks
        self.time_masks = time_masks
        self.freq_width = freq_width
        self.time_width = time_width
        self.mask_value = mask_value
        if isinstance(time_width, int):
            self.adaptive_temporal_width = False
        else:
            if time_width > 1.0 or time_width < 0.0:
                raise ValueError("If `time_width` is a float value, must be in range [0, 1]")
            self.adaptive_temporal_width = True

    @typecheck()
    @torch.no_grad()
    def forward(self, input_spec, length):
        lengths = length.detach().cpu() if self.time_masks > 0 else None   # one host copy per batch
        rects = _aug.spec_augment_rects(input_spec.shape, lengths, self._rng, self.freq_masks, self.time_masks,
                                        self.freq_width, self.time_width)
        return _aug.mask_rects_(input_spec, rects, self.mask_value)


class SpecCutout(nn.Module, Typing):
    """Random rectangles zeroed (spectr_augment.py:108-152)."""

    @property
    def input_types(self):
        return {"input_spec": NeuralType(("B", "D", "T"), SpectrogramType())}

    @property
    def output_types(self):
        return {"augmented_spec": NeuralType(("B", "D", "T"), SpectrogramType())}

    def __init__(self, rect_masks=0, rect_time=5, rect_freq=20, rng=None):
        super().__init__()
        self._rng = random.Random() if rng is None else rng
        self.rect_masks = rect_masks
        self.rect_time = rect_time
        self.rect_freq = rect_freq

    @typecheck()
    @torch.no_grad()
    def forward(self, input_spec):
        rects = _aug.cutout_rects(input_spec.shape, self._rng, self.rect_masks, self.rect_time, self.rect_freq)
        return _aug.mask_rects_(input_spec, rects, 0.0)


class SpecShot(nn.Module, Typing):
    """Element-wise random masking with probability mask_ratio (spectr_augment.py:154-184)."""

    @property
    def input_types(self):
        return {"input_spec": NeuralType(("B", "D", "T"), SpectrogramType())}

    @property
    def output_types(self):
        return {"augmented_spec": NeuralType(("B", "D", "T"), SpectrogramType())}

    def __init__(self, mask_ratio=0.3, mask_value=0.0):
        super().__init__()
        self.mask_ratio = mask_ratio
        self.mask_value = mask_value

    @typecheck()
    @torch.no_grad()
    def forward(self, input_spec):
        seed = int(torch.randint(0, 2 ** 62, (1,)).item())   # from torch's default CPU generator
        return _aug.spec_shot(input_spec, self.mask_ratio, seed)
