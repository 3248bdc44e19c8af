"""Drop-in `AudioToMelSpectrogramPreprocessor` and `SpectrogramAugmentation` (reference
nemo/collections/asr/modules/audio_preprocessing.py:63-281), SURVEY §8 row f1: the yaml
`preprocessor._target_` of conformer_ctc_bpe.yaml:78-92 resolves here with the same kwargs, the
same `featurizer.window` / `featurizer.fb` buffers, and keyword-only forward(input_signal, length)
-> (processed_signal (B, features, T), processed_length (B,)).  The featurizer runs in
libcfm.so (include/cfm_mel.h).

`SpectrogramAugmentation` (audio_preprocessing.py:416-521) composes the drop-in
SpecCutout / SpecAugment / SpecShot (on-device masking, include/cfm_augment.h) and picks one per
call with the global `random.choice`, as the reference does.
"""
from __future__ import annotations

import random
from collections import OrderedDict

import torch

from nemo.collections.asr.parts.preprocessing.features import FilterbankFeatures
from nemo.collections.asr.parts.submodules.spectr_augment import SpecAugment, SpecCutout, SpecShot
from nemo.core.classes.common import typecheck
from nemo.core.classes.module import NeuralModule
from nemo.core.neural_types import AudioSignal, LengthsType, MelSpectrogramType, NeuralType, SpectrogramType


class AudioPreprocessor(NeuralModule):
    """audio_preprocessing.py:63-95: forward -> get_features under no_grad."""

    def __init__(self, win_length, hop_length):
        super().__init__()
        self.win_length = win_length
        self.hop_length = hop_length
        self.torch_windows = {"hann": torch.hann_window, "hamming": torch.hamming_window,
                              "blackman": torch.blackman_window, "bartlett": torch.bartlett_window,
                              "ones": torch.ones, None: torch.ones}

    @typecheck()
    def forward(self, input_signal, length):
        with torch.no_grad():
            return self.get_features(input_signal, length)

    def get_features(self, input_signal, length):
        raise NotImplementedError


class AudioToMelSpectrogramPreprocessor(AudioPreprocessor):
    @property
    def input_types(self):
        return OrderedDict({"input_signal": NeuralType(("B", "T"), AudioSignal(freq=self._sample_rate)),
                            "length": NeuralType(tuple("B"), LengthsType())})

    @property
    def output_types(self):
        return OrderedDict({"processed_signal": NeuralType(("B", "D", "T"), MelSpectrogramType()),
                            "processed_length": NeuralType(tuple("B"), LengthsType())})

    def __init__(self, sample_rate=16000, window_size=0.02, window_stride=0.01, n_window_size=None,
                 n_window_stride=None, window="hann", normalize="per_feature", n_fft=None, preemph=0.97, features=64,
                 lowfreq=0, highfreq=None, log=True, log_zero_guard_type="add", log_zero_guard_value=2 ** -24,
                 dither=1e-5, pad_to=16, frame_splicing=1, exact_pad=False, stft_exact_pad=False, stft_conv=False,
                 pad_value=0, mag_power=2.0, rng=None, nb_augmentation_prob=0.0, nb_max_freq=4000):
        super().__init__(n_window_size, n_window_stride)
        self._sample_rate = sample_rate
        if window_size and n_window_size:
            raise ValueError(f"{self} received both window_size and n_window_size. Only one should be specified.")
        if window_stride and n_window_stride:
            raise ValueError(f"{self} received both window_stride and n_window_stride. Only one should be specified.")
        if window_size:
            n_window_size = int(window_size * self._sample_rate)
        if window_stride:
            n_window_stride = int(window_stride * self._sample_rate)
        self.featurizer = FilterbankFeatures(
            sample_rate=self._sample_rate, n_window_size=n_window_size, n_window_stride=n_window_stride,
            window=window, normalize=normalize, n_fft=n_fft, preemph=preemph, nfilt=features, lowfreq=lowfreq,
            highfreq=highfreq, log=log, log_zero_guard_type=log_zero_guard_type,
            log_zero_guard_value=log_zero_guard_value, dither=dither, pad_to=pad_to, frame_splicing=frame_splicing,
            exact_pad=exact_pad, stft_exact_pad=stft_exact_pad, stft_conv=stft_conv, pad_value=pad_value,
            mag_power=mag_power, rng=rng, nb_augmentation_prob=nb_augmentation_prob, nb_max_freq=nb_max_freq)

    def get_features(self, input_signal, length):
        return self.featurizer(input_signal, length)

    @property
    def filter_banks(self):
        return self.featurizer.filter_banks


class SpectrogramAugmentation(NeuralModule):
    """audio_preprocessing.py:416-521: one of SpecCutout / SpecAugment / SpecShot per call."""

    @property
    def input_types(self):
        return {"input_spec": NeuralType(("B", "D", "T"), SpectrogramType()),
                "length": NeuralType(tuple("B"), LengthsType())}

    @property
    def output_types(self):
        return {"augmented_spec": NeuralType(("B", "D", "T"), SpectrogramType())}

    def __init__(self, freq_masks=0, time_masks=0, freq_width=10, time_width=10, rect_masks=0, rect_time=5,
                 rect_freq=20, specshot_ratio=0, rng=None, augmask_value=0.0, use_numba_spec_augment: bool = True):
        super().__init__()
        self.augment_type = []
        if rect_masks > 0:
            self.spec_cutout = SpecCutout(rect_masks=rect_masks, rect_time=rect_time, rect_freq=rect_freq, rng=rng)
            self.augment_type.append("spec_cutout")
        if freq_masks + time_masks > 0:
            self.spec_augment = SpecAugment(freq_masks=freq_masks, time_masks=time_masks, freq_width=freq_width,
                                            time_width=time_width, rng=rng, mask_value=augmask_value)
            self.augment_type.append("spec_augment")
        if specshot_ratio > 0.0:
            self.spec_shot = SpecShot(mask_ratio=specshot_ratio, mask_value=augmask_value)
            self.augment_type.append("spec_shot")

    @typecheck()
    def forward(self, input_spec, length):
        if len(self.augment_type) == 0:
            return input_spec
        augment = random.choice(self.augment_type)
        if augment == "spec_augment":
            return self.spec_augment(input_spec=input_spec, length=length)
        elif augment == "spec_shot":
            return self.spec_shot(input_spec=input_spec)
        return self.spec_cutout(input_spec=input_spec)
