"""Oracle (TEST INFRASTRUCTURE ONLY — imported by tests/, never by the product path) for the
spectrogram augmentation row (include/cfm_augment.h).

A numpy restatement of the reference's masking loops, drawing from a `random.Random` in exactly the
reference's call order:
  spec_augment   spectr_augment.py:80-105   (freq masks, then time masks, per utterance; in place)
  spec_cutout    spectr_augment.py:138-152  (rectangles, value 0.0; in place)
  choice         audio_preprocessing.py:511-521 (global random.choice over the configured types)
Pinned to outputs of the reference modules themselves: tests/golden/augment_*.npz
(tests/golden/gen_augment_goldens.py).
"""
from __future__ import annotations

import random

import numpy as np


def _time_width(length: int, time_width) -> int:
    """spectr_augment.py:94-97: adaptive width = max(1, int(length * time_width)) where the product
    is a float32 tensor (int64 length tensor x python float -> float32)."""
    if isinstance(time_width, int):
        return time_width
    return max(1, int(np.float32(length) * np.float32(time_width)))


def spec_augment(x: np.ndarray, lengths, rng: random.Random, freq_masks: int, time_masks: int, freq_width: int,
                 time_width, mask_value: float = 0.0) -> np.ndarray:
    y = x.copy()
    B, F, _ = y.shape
    for idx in range(B):
        for _ in range(freq_masks):
            x_left = rng.randint(0, F - freq_width)
            w = rng.randint(0, freq_width)
            y[idx, x_left:x_left + w, :] = mask_value
        for _ in range(time_masks):
            L = int(lengths[idx])
            tw = _time_width(L, time_width)
            y_left = rng.randint(0, max(1, L - tw))
            w = rng.randint(0, tw)
            y[idx, :, y_left:y_left + w] = mask_value
    return y


def spec_cutout(x: np.ndarray, rng: random.Random, rect_masks: int, rect_time: int, rect_freq: int) -> np.ndarray:
    y = x.copy()
    B, F, T = y.shape
    for idx in range(B):
        for _ in range(rect_masks):
            rx = rng.randint(0, F - rect_freq)
            ry = rng.randint(0, T - rect_time)
            wx = rng.randint(0, rect_freq)
            wy = rng.randint(0, rect_time)
            y[idx, rx:rx + wx, ry:ry + wy] = 0.0
    return y
