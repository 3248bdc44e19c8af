"""Golden fixtures for the log-mel front end (include/cfm_mel.h), from the REFERENCE
FilterbankFeatures (nemo/collections/asr/parts/preprocessing/features.py:196-453), eval mode,
float32 on CPU.  Only where /root/reference exists:

    python tests/golden/gen_mel_goldens.py   # writes tests/golden/mel_*.npz

features.py imports librosa (unpinned, requirements_asr.txt:5) and torch_stft, absent here.  The
module is loaded with stubs: `librosa.filters.mel` = transformers.audio_utils.mel_filter_bank
(norm='slaney', mel_scale='slaney', an independent implementation of librosa's published
algorithm), `torch_stft.STFT` (only used when stft_conv=True, which the reference forcibly
disables, features.py:232-240), perturb/segment/logging (no arithmetic on this path).  The
filterbank the reference used is stored with each case so the GPU test feeds the same table.
Inputs: seeded sums of sinusoids + noise at speech-like amplitude, ragged lengths.
"""
import importlib.util
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from gen_goldens import REF, load_reference  # noqa: E402


def load_features():
    load_reference()
    from transformers.audio_utils import mel_filter_bank

    def mel(sr, n_fft, n_mels=128, fmin=0.0, fmax=None, htk=False, norm="slaney", dtype=np.float32):
        fmax = sr / 2.0 if fmax is None else fmax
        fb = mel_filter_bank(num_frequency_bins=1 + n_fft // 2, num_mel_filters=n_mels, min_frequency=float(fmin),
                             max_frequency=float(fmax), sampling_rate=sr, norm=norm,
                             mel_scale="htk" if htk else "slaney")
        return fb.T.astype(dtype)

    lib = types.ModuleType("librosa")
    lib.filters = types.SimpleNamespace(mel=mel)
    util = types.ModuleType("librosa.util")
    util.tiny = lambda x: np.finfo(np.float32).tiny
    lib.util = util
    sys.modules["librosa"] = lib
    sys.modules["librosa.util"] = util
    ts = types.ModuleType("torch_stft")
    ts.STFT = type("STFT", (torch.nn.Module,), {})
    sys.modules["torch_stft"] = ts

    class _Log:
        def __getattr__(self, _n):
            return lambda *a, **k: None

    u = types.ModuleType("nemo.utils")
    u.logging = _Log()
    sys.modules["nemo.utils"] = u
    for n, attrs in {"nemo.collections.asr.parts.preprocessing": {},
                     "nemo.collections.asr.parts.preprocessing.perturb": {"AudioAugmentor": object},
                     "nemo.collections.asr.parts.preprocessing.segment": {"AudioSegment": object}}.items():
        m = types.ModuleType(n)
        m.__dict__.update(attrs)
        m.__path__ = []
        sys.modules[n] = m
    name = "nemo.collections.asr.parts.preprocessing.features"
    spec = importlib.util.spec_from_file_location(name, f"{REF}/nemo/collections/asr/parts/preprocessing/features.py")
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def audio(g, B, N, lengths):
    t = np.arange(N) / 16000.0
    x = np.zeros((B, N), dtype=np.float64)
    for b in range(B):
        for _ in range(6):
            x[b] += g.uniform(0.02, 0.3) * np.sin(2 * np.pi * g.uniform(60, 7800) * t + g.uniform(0, 6.3))
        x[b] += 0.01 * g.standard_normal(N)
        x[b, lengths[b]:] = 0.0        # padded batch: zeros past each utterance
    return x.astype(np.float32)


CASES = {
    # conformer_ctc_bpe.yaml:78-92 (window 0.025 s, stride 0.01 s, n_fft 512, 80 mels, per_feature, pad_to 0)
    "mel_ctc_bpe": dict(kw=dict(sample_rate=16000, n_window_size=400, n_window_stride=160, window="hann",
                                normalize="per_feature", n_fft=512, nfilt=80, dither=1e-5, pad_to=0, pad_value=0.0),
                        B=3, N=16000, lengths=[16000, 12345, 4321], seed=1),
    # reference defaults: 20 ms window (320) -> n_fft 512, 64 mels, pad_to 16, all_features, hamming
    "mel_allfeat_pad16": dict(kw=dict(sample_rate=16000, n_window_size=320, n_window_stride=160, window="hamming",
                                      normalize="all_features", nfilt=64, pad_to=16, pad_value=-1.5),
                              B=2, N=9000, lengths=[9000, 5000], seed=2),
    # exact_pad (center=False + reflect pad), clamp guard, magnitude spectrum, no normalisation, no pre-emphasis
    "mel_exactpad_clamp": dict(kw=dict(sample_rate=16000, n_window_size=256, n_window_stride=128, window="blackman",
                                       normalize=None, n_fft=256, nfilt=40, preemph=None, exact_pad=True,
                                       log_zero_guard_type="clamp", log_zero_guard_value=1e-6, mag_power=1.0,
                                       pad_to=8),
                               B=2, N=4000, lengths=[4000, 2500], seed=3),
}


def main():
    feat = load_features()
    for name, c in CASES.items():
        fe = feat.FilterbankFeatures(**c["kw"]).eval()
        g = np.random.default_rng(c["seed"])
        x = audio(g, c["B"], c["N"], c["lengths"])
        L = torch.tensor(c["lengths"], dtype=torch.int64)
        y, yl = fe(torch.from_numpy(x), L)
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), x=x, lengths=np.array(c["lengths"], dtype=np.int64),
                            kw=np.array(repr(sorted(c["kw"].items()))), fb=fe.fb.numpy()[0],
                            window=(fe.window.numpy() if fe.window is not None else np.zeros(0, np.float32)),
                            y=y.numpy(), y_len=yl.numpy())
        print(name, tuple(y.shape), yl.tolist())


if __name__ == "__main__":
    main()
