"""CPU: the log-mel oracle (oracle/mel_oracle.py) reproduces the reference FilterbankFeatures
(tests/golden/mel_*.npz); the library's host-side librosa.filters.mel restatement agrees with the
oracle's and with transformers' independent implementation; frame counts / seq_len rules."""
import ast
import glob
import os

import numpy as np
import pytest

import mel_oracle as MO
from conftest import GOLDEN, rel_l2

FILES = sorted(glob.glob(os.path.join(GOLDEN, "mel_*.npz")))


def _kw(z):
    return dict(ast.literal_eval(str(z["kw"])))


def oracle_run(z):
    kw = _kw(z)
    n_fft = kw.get("n_fft") or 2 ** int(np.ceil(np.log2(kw["n_window_size"])))
    win = z["window"] if z["window"].size else None
    return MO.filterbank_features(
        z["x"], z["lengths"], z["fb"], win, n_fft=n_fft, hop=kw["n_window_stride"], preemph=kw.get("preemph", 0.97),
        mag_power=kw.get("mag_power", 2.0), guard_type=kw.get("log_zero_guard_type", "add"),
        guard=kw.get("log_zero_guard_value", 2 ** -24), normalize=kw.get("normalize", "per_feature"),
        pad_value=kw.get("pad_value", 0.0), pad_to=kw.get("pad_to", 16), exact_pad=kw.get("exact_pad", False))


@pytest.mark.parametrize("path", FILES, ids=[os.path.basename(f) for f in FILES])
def test_oracle_matches_reference(path):
    z = np.load(path)
    y, yl = oracle_run(z)
    np.testing.assert_array_equal(yl, z["y_len"])
    assert y.shape == z["y"].shape
    # the reference's STFT runs in float32 (torch.stft), the oracle's in float64: measured relL2
    # 2e-7 .. 1.9e-5, max |err| 1.2e-5 .. 2.8e-4 on normalised features
    assert rel_l2(y, z["y"]) <= 5e-5
    assert np.abs(y - z["y"]).max() <= 2e-3


@pytest.mark.parametrize("path", FILES, ids=[os.path.basename(f) for f in FILES])
def test_window_matches_reference(path):
    z = np.load(path)
    kw = _kw(z)
    w = MO.window(kw.get("window", "hann"), kw["n_window_size"])
    np.testing.assert_allclose(w, z["window"], rtol=0, atol=2e-7)


def test_filterbank_restatements_agree():
    from transformers.audio_utils import mel_filter_bank
    from conformer_amd.mel import slaney_filterbank
    for sr, n_fft, n_mels, fmin, fmax in [(16000, 512, 80, 0.0, 8000.0), (16000, 512, 64, 0.0, 8000.0),
                                          (16000, 256, 40, 20.0, 7600.0), (22050, 1024, 128, 0.0, 11025.0)]:
        o = MO.mel_filterbank(sr, n_fft, n_mels, fmin, fmax)
        t = mel_filter_bank(num_frequency_bins=1 + n_fft // 2, num_mel_filters=n_mels, min_frequency=fmin,
                            max_frequency=fmax, sampling_rate=sr, norm="slaney", mel_scale="slaney").T
        lib = slaney_filterbank(sr, n_fft, n_mels, fmin, fmax).numpy()
        assert np.abs(o - t).max() <= 1e-7 * max(1.0, np.abs(t).max())
        assert np.abs(lib - o).max() <= 2e-9
        assert ((lib != 0) == (o != 0)).all()
    for path in FILES:                         # and the table the reference actually used
        z = np.load(path)
        kw = _kw(z)
        n_fft = kw.get("n_fft") or 2 ** int(np.ceil(np.log2(kw["n_window_size"])))
        lib = slaney_filterbank(kw["sample_rate"], n_fft, kw["nfilt"]).numpy()
        assert np.abs(lib - z["fb"]).max() <= 1e-7 * np.abs(z["fb"]).max()


def test_seq_len_and_frames():
    from nemo.collections.asr.parts.preprocessing.features import FilterbankFeatures
    import torch
    for exact in (False, True):
        fe = FilterbankFeatures(n_window_size=400, n_window_stride=160, n_fft=512, nfilt=80, exact_pad=exact)
        L = np.arange(1, 40000, 97)
        np.testing.assert_array_equal(fe.get_seq_len(torch.tensor(L, dtype=torch.float)).numpy(),
                                      MO.seq_len(L, 512, 160, exact))
    for path in FILES:
        z = np.load(path)
        kw = _kw(z)
        n_fft = kw.get("n_fft") or 2 ** int(np.ceil(np.log2(kw["n_window_size"])))
        np.testing.assert_array_equal(MO.seq_len(z["lengths"], n_fft, kw["n_window_stride"],
                                                 kw.get("exact_pad", False)), z["y_len"])


def test_preprocessor_plugin_surface():
    from nemo.collections.asr.modules import AudioToMelSpectrogramPreprocessor
    from nemo.core.classes.common import Serialization
    cfg = {"_target_": "nemo.collections.asr.modules.AudioToMelSpectrogramPreprocessor", "sample_rate": 16000,
           "normalize": "per_feature", "window_size": 0.025, "window_stride": 0.01, "window": "hann",
           "features": 80, "n_fft": 512, "log": True, "frame_splicing": 1, "dither": 0.00001, "pad_to": 0,
           "pad_value": 0.0}                      # conformer_ctc_bpe.yaml:78-92
    p = Serialization.from_config_dict(cfg)
    assert isinstance(p, AudioToMelSpectrogramPreprocessor)
    assert sorted(p.state_dict()) == ["featurizer.fb", "featurizer.window"]
    assert tuple(p.filter_banks.shape) == (1, 80, 257)
    import torch
    with pytest.raises(TypeError):
        p(torch.zeros(1, 16000), torch.tensor([16000]))
    with pytest.raises(RuntimeError):            # no CPU fallback
        p(input_signal=torch.zeros(1, 16000), length=torch.tensor([16000]))
