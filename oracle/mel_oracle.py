"""CPU oracle (TEST INFRASTRUCTURE ONLY) for the log-mel front end, SURVEY §8 row f1.

numpy restatement of FilterbankFeatures.forward (nemo/collections/asr/parts/preprocessing/features.py
:382-453) in eval mode (no dither / narrow-band augmentation), normalize_batch (54-83) and
get_seq_len (368-376), plus librosa.filters.mel (third-party, unpinned in
requirements/requirements_asr.txt:5 and absent here; its published Slaney algorithm is restated in
`mel_filterbank`).  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module.  Pinned by tests/golden/mel_*.npz, made by running the reference FilterbankFeatures
itself (tests/golden/gen_mel_goldens.py); the filterbank is cross-checked against
transformers.audio_utils.mel_filter_bank (an independent implementation of the same algorithm).
"""
from __future__ import annotations

import math
from typing import Optional

import numpy as np


def hz_to_mel(f, htk=False):
    f = np.asanyarray(f, dtype=np.float64)
    if htk:
        return 2595.0 * np.log10(1.0 + f / 700.0)
    f_sp, min_log_hz = 200.0 / 3, 1000.0
    min_log_mel, logstep = min_log_hz / f_sp, np.log(6.4) / 27.0
    return np.where(f >= min_log_hz, min_log_mel + np.log(np.maximum(f, 1e-300) / min_log_hz) / logstep, f / f_sp)


def mel_to_hz(m, htk=False):
    m = np.asanyarray(m, dtype=np.float64)
    if htk:
        return 700.0 * (10.0 ** (m / 2595.0) - 1.0)
    f_sp, min_log_hz = 200.0 / 3, 1000.0
    min_log_mel, logstep = min_log_hz / f_sp, np.log(6.4) / 27.0
    return np.where(m >= min_log_mel, min_log_hz * np.exp(logstep * (m - min_log_mel)), f_sp * m)


def mel_filterbank(sr, n_fft, n_mels, fmin=0.0, fmax=None, htk=False, norm="slaney"):
    """librosa.filters.mel: triangular filters on the mel scale, Slaney area normalisation."""
    fmax = sr / 2.0 if fmax is None else fmax
    fft = np.arange(1 + n_fft // 2) * (sr / n_fft)
    mel_f = mel_to_hz(np.linspace(hz_to_mel(fmin, htk), hz_to_mel(fmax, htk), n_mels + 2), htk)
    fdiff = np.diff(mel_f)
    ramps = mel_f[:, None] - fft[None, :]
    w = np.zeros((n_mels, 1 + n_fft // 2), dtype=np.float32)
    for i in range(n_mels):
        w[i] = np.maximum(0, np.minimum(-ramps[i] / fdiff[i], ramps[i + 2] / fdiff[i + 1]))
    if norm == "slaney":
        w *= (2.0 / (mel_f[2:n_mels + 2] - mel_f[:n_mels]))[:, None]
    return w


def window(name, n):
    """torch.{hann,hamming,blackman,bartlett}_window(n, periodic=False) (features.py:279-287)."""
    k = np.arange(n, dtype=np.float64)
    x = 2 * np.pi * k / (n - 1)
    if name == "hann":
        w = 0.5 - 0.5 * np.cos(x)
    elif name == "hamming":
        w = 0.54 - 0.46 * np.cos(x)
    elif name == "blackman":
        w = 0.42 - 0.5 * np.cos(x) + 0.08 * np.cos(2 * x)
    elif name == "bartlett":
        w = 1 - np.abs(2 * k / (n - 1) - 1)
    else:
        return None
    return w.astype(np.float32)


def seq_len(length, n_fft, hop, exact_pad=False):
    """get_seq_len (features.py:368-376) in float32."""
    pad = ((n_fft - hop) // 2) * 2 if exact_pad else n_fft // 2 * 2
    L = np.asarray(length, dtype=np.float32)
    return (np.floor((L + np.float32(pad) - np.float32(n_fft)) / np.float32(hop)) + 1).astype(np.int64)


def normalize_batch(x, sl, normalize_type):
    """features.py:54-83 (float64 statistics, torch's unbiased std)."""
    x = np.asarray(x, dtype=np.float32)
    if normalize_type == "per_feature":
        out = np.empty_like(x)
        for i in range(x.shape[0]):
            seg = x[i, :, : sl[i]].astype(np.float64)
            m, s = seg.mean(axis=1), seg.std(axis=1, ddof=1)
            out[i] = (x[i] - m[:, None].astype(np.float32)) / (s[:, None].astype(np.float32) + np.float32(1e-5))
        return out
    if normalize_type == "all_features":
        out = np.empty_like(x)
        for i in range(x.shape[0]):
            seg = x[i, :, : sl[i]].astype(np.float64)
            out[i] = (x[i] - np.float32(seg.mean())) / (np.float32(seg.std(ddof=1)) + np.float32(1e-5))
        return out
    return x


def filterbank_features(x, length, fb, win, n_fft=512, hop=160, preemph: Optional[float] = 0.97, mag_power=2.0,
                        log=True, guard_type="add", guard=2 ** -24, normalize="per_feature", pad_value=0.0, pad_to=0,
                        exact_pad=False):
    """FilterbankFeatures.forward, eval mode (features.py:382-453).  x (B, N) float32."""
    x = np.asarray(x, dtype=np.float32)
    sl = seq_len(length, n_fft, hop, exact_pad)
    if exact_pad:
        P = (n_fft - hop) // 2
        x = np.pad(x, ((0, 0), (P, P)), mode="reflect")
    if preemph is not None:
        x = np.concatenate([x[:, :1], x[:, 1:] - np.float32(preemph) * x[:, :-1]], axis=1)
    if not exact_pad:
        x = np.pad(x, ((0, 0), (n_fft // 2, n_fft // 2)), mode="reflect")
    T = 1 + (x.shape[1] - n_fft) // hop
    wfull = np.zeros(n_fft, dtype=np.float32)
    woff = (n_fft - len(win)) // 2
    wfull[woff:woff + len(win)] = win if win is not None else 1.0
    idx = np.arange(T)[:, None] * hop + np.arange(n_fft)[None, :]
    frames = x[:, idx] * wfull                                    # (B, T, n_fft)
    spec = np.fft.rfft(frames.astype(np.float64), axis=-1)
    mag = np.sqrt(spec.real ** 2 + spec.imag ** 2)
    if mag_power != 1.0:
        mag = mag ** mag_power
    mel = np.einsum("mk,btk->bmt", fb.astype(np.float64), mag)
    if log:
        mel = np.log(mel + guard) if guard_type == "add" else np.log(np.maximum(mel, guard))
    mel = normalize_batch(mel.astype(np.float32), sl, normalize)
    t = np.arange(mel.shape[-1])[None, :]
    mel = np.where((t >= sl[:, None])[:, None, :], np.float32(pad_value), mel)
    if pad_to and pad_to > 0 and mel.shape[-1] % pad_to:
        mel = np.pad(mel, ((0, 0), (0, 0), (0, pad_to - mel.shape[-1] % pad_to)), constant_values=pad_value)
    return mel.astype(np.float32), sl
