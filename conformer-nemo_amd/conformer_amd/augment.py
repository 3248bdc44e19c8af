"""Host runtime of the on-device spectrogram augmentation (include/cfm_augment.h), SURVEY §8 f4.

The reference (spectr_augment.py:80-152) loops over utterances in Python and writes every mask
with a separate slice assignment, reading `length[idx]` from the device once per time mask.  Here
the mask geometry is drawn on the host with the SAME random.Random call sequence (so a seeded rng
gives the reference's masks exactly), from ONE host copy of the lengths, into one int32 rectangle
table [f0, f1, t0, t1) per mask; one kernel launch then paints every rectangle on the device.
"""
from __future__ import annotations

import ctypes
import random
from typing import Sequence

import numpy as np
import torch

from . import _lib


def spec_augment_rects(shape: Sequence[int], length: torch.Tensor, rng: random.Random, freq_masks: int,
                       time_masks: int, freq_width: int, time_width) -> np.ndarray:
    """SpecAugment.forward's draws (spectr_augment.py:85-103) -> (B, freq_masks + time_masks, 4) int32.
    `length` is a CPU tensor; the adaptive width keeps the reference's tensor arithmetic
    (int64 length * python float -> float32, then int())."""
    B, F, T = (int(s) for s in shape)
    adaptive = not isinstance(time_width, int)
    rects = np.zeros((B, freq_masks + time_masks, 4), dtype=np.int32)
    for idx in range(B):
        k = 0
        for _ in range(freq_masks):
            x_left = rng.randint(0, F - freq_width)
            w = rng.randint(0, freq_width)
            rects[idx, k] = (x_left, x_left + w, 0, T)
            k += 1
        for _ in range(time_masks):
            tw = max(1, int(length[idx] * time_width)) if adaptive else time_width
            y_left = rng.randint(0, max(1, length[idx] - tw))
            w = rng.randint(0, tw)
            y_left = int(y_left)
            rects[idx, k] = (0, F, y_left, y_left + int(w))
            k += 1
    return rects


def cutout_rects(shape: Sequence[int], rng: random.Random, rect_masks: int, rect_time: int,
                 rect_freq: int) -> np.ndarray:
    """SpecCutout.forward's draws (spectr_augment.py:142-150) -> (B, rect_masks, 4) int32."""
    B, F, T = (int(s) for s in shape)
    rects = np.zeros((B, rect_masks, 4), dtype=np.int32)
    for idx in range(B):
        for i in range(rect_masks):
            rx = rng.randint(0, F - rect_freq)
            ry = rng.randint(0, T - rect_time)
            wx = rng.randint(0, rect_freq)
            wy = rng.randint(0, rect_time)
            rects[idx, i] = (rx, rx + wx, ry, ry + wy)
    return rects


def _check_spec(spec: torch.Tensor, what: str) -> None:
    if not spec.is_cuda:
        raise _lib.CfmError(f"{what}: the native path needs a CUDA (ROCm) tensor")
    if spec.dtype != torch.float32 or spec.dim() != 3:
        raise _lib.CfmError(f"{what}: expected a (B, F, T) float32 spectrogram, got {tuple(spec.shape)} {spec.dtype}")


def mask_rects_(spec: torch.Tensor, rects: np.ndarray, value: float) -> torch.Tensor:
    """spec[b, f0:f1, t0:t1] = value for every rectangle, in place on the device (one launch)."""
    _check_spec(spec, "mask_rects_")
    B, F, T = spec.shape
    if rects.size == 0 or spec.numel() == 0:
        return spec
    n = rects.shape[1]
    table = torch.from_numpy(np.ascontiguousarray(rects, dtype=np.int32)).pin_memory()
    table = table.to(spec.device, non_blocking=True)
    work = spec if spec.is_contiguous() else spec.contiguous()
    st = ctypes.c_void_p(torch.cuda.current_stream(spec.device).cuda_stream)
    _lib.check(_lib.load().cfm_spec_mask_rects(work.data_ptr(), B, F, T, table.data_ptr(), n, float(value), st),
               "cfm_spec_mask_rects")
    if work is not spec:
        spec.copy_(work)
    return spec


def spec_shot(spec: torch.Tensor, mask_ratio: float, seed: int) -> torch.Tensor:
    """SpecShot.forward (spectr_augment.py:177-184): a new tensor keeping elements where
    1 - U(0,1) > mask_ratio; the uniforms come from a counter hash of (seed, element index)."""
    _check_spec(spec, "spec_shot")
    x = spec.contiguous()
    out = torch.empty_like(x)
    st = ctypes.c_void_p(torch.cuda.current_stream(spec.device).cuda_stream)
    _lib.check(_lib.load().cfm_spec_shot(x.data_ptr(), out.data_ptr(), x.numel(), float(mask_ratio),
                                         int(seed) & (2 ** 64 - 1), st), "cfm_spec_shot")
    return out
