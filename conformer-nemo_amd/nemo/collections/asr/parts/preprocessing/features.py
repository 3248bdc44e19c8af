"""Drop-in `FilterbankFeatures` and `normalize_batch` (reference
nemo/collections/asr/parts/preprocessing/features.py:54-83, 196-453), SURVEY §8 row f1.

Same constructor arguments, the same registered buffers (`window` (win_length,) and `fb`
(1, nfilt, n_fft//2+1), so `featurizer.window` / `featurizer.fb` load from a checkpoint
unchanged), `get_seq_len`, `filter_banks` and forward(x, seq_len) -> (features, seq_len).  The
arithmetic runs in libcfm.so (include/cfm_mel.h) on the input's GPU: one STFT/mel kernel and one
normalise/mask kernel.  CPU tensors are refused (no fallback).

Deviations (documented, not silent): training-mode dither draws its N(0,1) noise from the
library's counter-based generator, not torch.randn (same distribution, different samples);
`frame_splicing > 1` and fixed_mean/fixed_std normalisation raise NotImplementedError; the
reference's ValueError for a length-1 per_feature slice is raised only when the lengths are
host tensors (on device tensors the output is NaN, as torch.std of one value is).
"""
from __future__ import annotations

import math
import random

import torch
import torch.nn as nn

CONSTANT = 1e-5


def normalize_batch(x, seq_len, normalize_type):
    """features.py:54-83 on the GPU (per_feature / all_features); other types return x unchanged."""
    from conformer_amd.mel import normalize_batch as _nb
    return _nb(x, seq_len, normalize_type)


def _window(name, length):
    fns = {"hann": torch.hann_window, "hamming": torch.hamming_window, "blackman": torch.blackman_window,
           "bartlett": torch.bartlett_window, "none": None}
    fn = fns.get(name, None)
    return fn(length, periodic=False) if fn else None


class FilterbankFeatures(nn.Module):
    """Raw audio (B, N) -> log-mel features (B, nfilt, T) (features.py:196-453)."""

    def __init__(self, sample_rate=16000, n_window_size=320, n_window_stride=160, window="hann",
                 normalize="per_feature", n_fft=None, preemph=0.97, nfilt=64, lowfreq=0, highfreq=None, log=True,
                 log_zero_guard_type="add", log_zero_guard_value=2 ** -24, dither=CONSTANT, pad_to=16,
                 max_duration=16.7, frame_splicing=1, exact_pad=False, pad_value=0, mag_power=2.0, use_grads=False,
                 rng=None, nb_augmentation_prob=0.0, nb_max_freq=4000, stft_exact_pad=False, stft_conv=False):
        super().__init__()
        if stft_conv or stft_exact_pad:      # features.py:232-240: forcibly disabled
            stft_conv = False
            stft_exact_pad = False
        if exact_pad and n_window_stride % 2 == 1:
            raise NotImplementedError(f"{self} received exact_pad == True, but hop_size was odd.")
        if (n_window_size is None or n_window_stride is None or not isinstance(n_window_size, int)
                or not isinstance(n_window_stride, int) or n_window_size <= 0 or n_window_stride <= 0):
            raise ValueError(f"{self} got an invalid value for either n_window_size or n_window_stride. "
                             f"Both must be positive ints.")
        if log_zero_guard_type not in ["add", "clamp"]:
            raise ValueError(f"{self} received {log_zero_guard_type} for the log_zero_guard_type parameter. "
                             f"It must be either 'add' or 'clamp'.")
        if frame_splicing > 1:
            raise NotImplementedError("frame_splicing > 1 is not on the native path")
        self.log_zero_guard_value = log_zero_guard_value
        self.win_length = n_window_size
        self.hop_length = n_window_stride
        self.n_fft = n_fft or 2 ** math.ceil(math.log2(self.win_length))
        self.stft_pad_amount = (self.n_fft - self.hop_length) // 2 if exact_pad else None
        self.stft_exact_pad = stft_exact_pad
        self.stft_conv = stft_conv
        self.exact_pad = exact_pad
        self.window_name = window
        self.register_buffer("window", _window(window, self.win_length))
        self.normalize = normalize
        self.log = log
        self.dither = dither
        self.frame_splicing = frame_splicing
        self.nfilt = nfilt
        self.preemph = preemph
        self.pad_to = pad_to
        highfreq = highfreq or sample_rate / 2
        from conformer_amd.mel import slaney_filterbank
        self.register_buffer("fb", slaney_filterbank(sample_rate, self.n_fft, nfilt, lowfreq, highfreq).unsqueeze(0))
        max_length = self.get_seq_len(torch.tensor(max_duration * sample_rate, dtype=torch.float))
        max_pad = pad_to - (max_length % pad_to) if (pad_to != "max" and pad_to > 0) else 0
        self.max_length = int(max_length + max_pad)
        self.pad_value = pad_value
        self.mag_power = mag_power
        self.log_zero_guard_type = log_zero_guard_type
        self.use_grads = use_grads
        self._rng = random.Random() if rng is None else rng
        self.nb_augmentation_prob = nb_augmentation_prob
        if self.nb_augmentation_prob > 0.0:
            if nb_max_freq >= sample_rate / 2:
                self.nb_augmentation_prob = 0.0
            else:
                self._nb_max_fft_bin = int((nb_max_freq / sample_rate) * n_fft)
        self._native = {}
        self._synced = {}
        self._seed = random.Random(0x6d656c).getrandbits(63)

    def log_zero_guard_value_fn(self, x):
        if isinstance(self.log_zero_guard_value, str):
            if self.log_zero_guard_value == "tiny":
                return torch.finfo(x.dtype).tiny
            if self.log_zero_guard_value == "eps":
                return torch.finfo(x.dtype).eps
            raise ValueError(f"{self} received {self.log_zero_guard_value} for the log_zero_guard_type parameter. "
                             f"It must be either a number, 'tiny', or 'eps'")
        return self.log_zero_guard_value

    def get_seq_len(self, seq_len):
        pad_amount = self.stft_pad_amount * 2 if self.stft_pad_amount is not None else self.n_fft // 2 * 2
        seq_len = torch.floor((seq_len + pad_amount - self.n_fft) / self.hop_length) + 1
        return seq_len.to(dtype=torch.long)

    @property
    def filter_banks(self):
        return self.fb

    def _native_for(self, dev):
        from conformer_amd.mel import NativeMel
        nat = self._native.get(dev.index)
        if nat is None:
            nat = NativeMel(self.win_length, self.hop_length, self.n_fft, self.nfilt, self.exact_pad, self.preemph,
                            self.mag_power, self.log, self.log_zero_guard_type,
                            float(self.log_zero_guard_value_fn(torch.zeros(1))), self.normalize, self.pad_value,
                            self.pad_to, self.max_length, dev)
            self._native[dev.index] = nat
        snap = tuple((t.data_ptr(), t._version) if t is not None else None for t in (self.window, self.fb))
        if self._synced.get(dev.index) != snap:
            nat.set_tables(self.window, self.fb)
            self._synced[dev.index] = snap
        return nat

    def forward(self, x, seq_len):
        if not x.is_cuda:
            raise RuntimeError("FilterbankFeatures (MI355X-native) needs a GPU tensor")
        if self.normalize == "per_feature" and not seq_len.is_cuda:
            if int(self.get_seq_len(seq_len.float()).min()) == 1:       # features.py:59-63
                raise ValueError("normalize_batch with `per_feature` normalize_type received a tensor of length 1. "
                                 "This will result in torch.std() returning nan")
        dither = float(self.dither) if (self.training and self.dither > 0) else 0.0
        nb_mask, nb_bin = None, 0
        if self.training and self.nb_augmentation_prob > 0.0:
            nb_mask = torch.tensor([self._rng.random() < self.nb_augmentation_prob for _ in range(x.shape[0])],
                                   dtype=torch.uint8)
            nb_bin = self._nb_max_fft_bin
        seed = 0
        if dither > 0:
            self._seed = (self._seed * 6364136223846793005 + 1442695040888963407) % (1 << 64)
            seed = self._seed
        with torch.no_grad():
            return self._native_for(x.device).forward(x, seq_len, dither, seed, nb_mask, nb_bin)
