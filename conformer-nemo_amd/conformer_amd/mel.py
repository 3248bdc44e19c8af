"""Host runtime around the C-ABI log-mel front end (include/cfm_mel.h), SURVEY §8 row f1.

`NativeMel` owns one `cfm_mel*` (twiddles, zero-padded window and the compacted mel filterbank on
one GPU); `forward` runs cfm_mel_forward on torch's current stream: raw (B, N) samples ->
(B, nfilt, T) log-mel features + int64 frame lengths, in one STFT/mel launch and one
normalise/mask launch.  `slaney_filterbank` is librosa.filters.mel restated in the library
(host code), used for the module's initial `fb` buffer.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import torch

from . import _lib

NORMALIZE = {"per_feature": 1, "all_features": 2}
LOG_GUARD = {"add": 0, "clamp": 1}


def slaney_filterbank(sample_rate: int, n_fft: int, n_mels: int, fmin: float = 0.0, fmax: Optional[float] = None,
                      htk: bool = False, norm: Optional[str] = "slaney") -> torch.Tensor:
    """librosa.filters.mel(sr, n_fft, n_mels, fmin, fmax, htk, norm) as a (n_mels, n_fft//2+1) fp32 tensor."""
    lib = _lib.load()
    fmax = float(sample_rate) / 2 if fmax is None else float(fmax)
    out = torch.empty((int(n_mels), int(n_fft) // 2 + 1), dtype=torch.float32)
    ptr = ctypes.cast(out.data_ptr(), ctypes.POINTER(ctypes.c_float))
    _lib.check(lib.cfm_mel_filterbank_slaney(int(sample_rate), int(n_fft), int(n_mels), float(fmin), fmax,
                                             1 if htk else 0, 1 if norm == "slaney" else 0, ptr),
               "cfm_mel_filterbank_slaney")
    return out


def normalize_batch(x: torch.Tensor, seq_len: torch.Tensor, normalize_type: str) -> torch.Tensor:
    """features.py:54-83 (per_feature / all_features) on the GPU; other types return x."""
    if normalize_type not in NORMALIZE:
        if isinstance(normalize_type, dict):
            raise NotImplementedError("fixed_mean / fixed_std normalisation is not on the native path")
        return x
    if not x.is_cuda:
        raise _lib.CfmError("normalize_batch: the native path needs CUDA tensors")
    xc = x.float().contiguous()
    out = torch.empty_like(xc)
    sl = seq_len.to(x.device, torch.int64).contiguous()
    B, F, T = xc.shape
    st = ctypes.c_void_p(torch.cuda.current_stream(x.device).cuda_stream)
    _lib.check(_lib.load().cfm_normalize_batch(xc.data_ptr(), sl.data_ptr(), B, F, T, NORMALIZE[normalize_type],
                                               out.data_ptr(), st), "cfm_normalize_batch")
    return out


class NativeMel:
    def __init__(self, n_window_size: int, n_window_stride: int, n_fft: int, nfilt: int, exact_pad: bool,
                 preemph: Optional[float], mag_power: float, log: bool, log_zero_guard_type: str,
                 log_zero_guard_value: float, normalize, pad_value: float, pad_to, max_length: int, device=None):
        self.lib = _lib.load()
        if not torch.cuda.is_available():
            raise _lib.CfmError("the native mel front end needs a ROCm GPU (torch.cuda.is_available() is False)")
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None else torch.device(device).index)
        c = _lib.CfmMelCfg()
        c.n_window_size, c.n_window_stride, c.n_fft, c.nfilt = int(n_window_size), int(n_window_stride), int(n_fft), int(nfilt)
        c.exact_pad = 1 if exact_pad else 0
        c.use_preemph = 0 if preemph is None else 1
        c.preemph = 0.0 if preemph is None else float(preemph)
        c.mag_power = float(mag_power)
        c.log = 1 if log else 0
        c.log_zero_guard_type = LOG_GUARD[log_zero_guard_type]
        c.log_zero_guard_value = float(log_zero_guard_value)
        if isinstance(normalize, dict):
            raise NotImplementedError("fixed_mean / fixed_std normalisation is not on the native path")
        c.normalize = NORMALIZE.get(normalize, 0) if normalize else 0
        c.pad_value = float(pad_value)
        c.pad_to = -1 if pad_to == "max" else int(pad_to)
        c.max_length = int(max_length)
        self.cfg = c
        h = ctypes.c_void_p()
        _lib.check(self.lib.cfm_mel_create(ctypes.byref(c), self.device.index, ctypes.byref(h)), "cfm_mel_create")
        self.handle = h
        self._tables = None

    def __del__(self):
        h = getattr(self, "handle", None)
        if h:
            self.lib.cfm_mel_destroy(h)
            self.handle = None

    def set_tables(self, window: Optional[torch.Tensor], fb: torch.Tensor) -> None:
        w = None if window is None else window.detach().to(self.device, torch.float32).contiguous()
        f = fb.detach().to(self.device, torch.float32).reshape(self.cfg.nfilt, -1).contiguous()
        if f.shape[1] != self.cfg.n_fft // 2 + 1:
            raise ValueError(f"filterbank has {f.shape[1]} bins, expected {self.cfg.n_fft // 2 + 1}")
        st = ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        _lib.check(self.lib.cfm_mel_set_tables(self.handle, None if w is None else w.data_ptr(), f.data_ptr(), st),
                   "cfm_mel_set_tables")
        self._tables = (w, f)

    def output_frames(self, n_samples: int) -> int:
        return int(self.lib.cfm_mel_output_frames(self.handle, int(n_samples)))

    def forward(self, x: torch.Tensor, length: torch.Tensor, dither: float = 0.0, seed: int = 0,
                nb_mask: Optional[torch.Tensor] = None, nb_max_bin: int = 0):
        xs = x.detach().to(self.device, torch.float32).contiguous()
        if xs.dim() != 2:
            raise ValueError(f"input_signal must be (B, T) samples, got {tuple(xs.shape)}")
        B, N = xs.shape
        ln = length.to(self.device).to(torch.int64).contiguous()
        Tout = self.output_frames(N)
        out = torch.empty((B, self.cfg.nfilt, Tout), dtype=torch.float32, device=self.device)
        out_len = torch.empty((B,), dtype=torch.int64, device=self.device)
        nbm = None if nb_mask is None else nb_mask.to(self.device, torch.uint8).contiguous()
        st = ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        _lib.check(self.lib.cfm_mel_forward(self.handle, xs.data_ptr(), ln.data_ptr(), B, N, ctypes.c_float(dither),
                                            ctypes.c_uint64(seed & (2 ** 64 - 1)),
                                            None if nbm is None else nbm.data_ptr(), int(nb_max_bin),
                                            out.data_ptr(), out_len.data_ptr(), st), "cfm_mel_forward")
        return out, out_len
