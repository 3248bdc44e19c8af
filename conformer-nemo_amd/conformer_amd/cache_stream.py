"""Host runtime of the cache-aware chunked streaming encoder (include/cfm_cache_stream.h).

`NativeCacheStream` owns the device state (subsampling caches, per-layer key/value and GLU rings)
of `batch` streams for one NativeEncoder and advances it one chunk per `step` on torch's current
stream.  The computed model is the causal variant of the reference encoder that the header defines
(causal subsampling / depthwise padding, attention context [left_context, 0]); parity is unpinned
(no reference counterpart) and checked against a full-sequence forward of that causal model
(oracle/cache_aware_oracle.py, tests/test_gpu_cache_stream.py).
"""
from __future__ import annotations

import ctypes
from typing import Optional

import torch

from . import _lib

SYMBOLS = ("cfm_cache_stream_create", "cfm_cache_stream_destroy", "cfm_cache_stream_reset",
           "cfm_cache_stream_workspace_size", "cfm_cache_stream_step", "cfm_cache_stream_position")


def _bind(lib) -> None:
    if getattr(lib, "_cache_stream_bound", False):
        return
    vp, ci, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
    sig = {
        "cfm_cache_stream_create": (ci, [vp, ci, ci, ci, ctypes.POINTER(vp)]),
        "cfm_cache_stream_destroy": (ci, [vp]),
        "cfm_cache_stream_reset": (ci, [vp, vp]),
        "cfm_cache_stream_workspace_size": (sz, [vp]),
        "cfm_cache_stream_step": (ci, [vp, vp, vp, vp, sz, vp]),
        "cfm_cache_stream_position": (ctypes.c_int64, [vp]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    lib._cache_stream_bound = True


class NativeCacheStream:
    """batch streams, `chunk` encoder frames (4 * chunk input frames) per step, `left_context` frames
    of attention history.  `encoder` is a conformer_amd.NativeEncoder whose weights are set."""

    def __init__(self, encoder, batch: int, chunk: int, left_context: int):
        self.lib = encoder.lib            # the encoder handle's own build (bf16 or fp16)
        _bind(self.lib)
        self.encoder = encoder            # keeps the weights alive
        self.device = encoder.device
        self.B, self.c, self.left = int(batch), int(chunk), int(left_context)
        self.feat_in = int(encoder.cfg.feat_in)
        d = int(encoder.cfg.d_model)
        self.d_out = int(encoder.cfg.feat_out) if int(encoder.cfg.feat_out) > 0 else d
        h = ctypes.c_void_p()
        _lib.check(self.lib.cfm_cache_stream_create(encoder.handle, self.B, self.c, self.left, ctypes.byref(h)),
                   "cfm_cache_stream_create", lib=self.lib)
        self.handle = h
        ws = int(self.lib.cfm_cache_stream_workspace_size(h))
        self._ws = torch.empty(ws, dtype=torch.uint8, device=f"cuda:{self.device}")
        self.reset()

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and h.value:
            try:
                self.lib.cfm_cache_stream_destroy(h)
            except Exception:
                pass
            self.handle = None

    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def reset(self) -> None:
        """Zero the caches, restart at frame 0, rebuild the position projections from the weights."""
        _lib.check(self.lib.cfm_cache_stream_reset(self.handle, self._stream()), "cfm_cache_stream_reset", lib=self.lib)

    @property
    def position(self) -> int:
        return int(self.lib.cfm_cache_stream_position(self.handle))

    def step(self, x_bft: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """x (batch, feat_in, 4 * chunk) -> (batch, d_out, chunk) fp32."""
        x = x_bft.to(f"cuda:{self.device}", torch.float32).contiguous()
        if x.shape != (self.B, self.feat_in, 4 * self.c):
            raise ValueError(f"chunk input {tuple(x.shape)} must be ({self.B}, {self.feat_in}, {4 * self.c})")
        if out is None:
            out = torch.empty((self.B, self.d_out, self.c), dtype=torch.float32, device=x.device)
        elif out.shape != (self.B, self.d_out, self.c) or out.dtype != torch.float32 or not out.is_contiguous():
            raise ValueError(f"out must be a contiguous fp32 ({self.B}, {self.d_out}, {self.c}) tensor")
        _lib.check(self.lib.cfm_cache_stream_step(self.handle, x.data_ptr(), out.data_ptr(), self._ws.data_ptr(),
                                                  self._ws.numel(), self._stream()), "cfm_cache_stream_step", lib=self.lib)
        return out
