"""Host runtime around the C-ABI streaming front end (include/cfm_stream.h), SURVEY §8 row a-ext5.

`NativeFrameBuffer` keeps S per-stream feature buffers (F, Tbuf) resident on one GPU and advances
them with cfm_frame_buffer_step on torch's current stream: shift-and-append of the new chunk(s),
per-feature mean / population-std normalisation, and the normalised buffers written in the
encoder's (B, F, T) input layout, so a streaming step is one small kernel + one encoder call with
no host round trip.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import torch

from . import _lib

ZERO_LEVEL_SPEC_DB_VAL = -16.635  # streaming_utils.py:469 (log-mel of a zero signal)


class NativeFrameBuffer:
    def __init__(self, streams: int, n_feat: int, n_frame: int, total_len: int, eps: float, device=None):
        self.lib = _lib.load()
        if not torch.cuda.is_available():
            raise _lib.CfmError("the native streaming buffer needs a ROCm GPU (torch.cuda.is_available() is False)")
        if not (1 <= n_frame <= total_len):
            raise ValueError(f"need 1 <= n_frame ({n_frame}) <= total buffer length ({total_len})")
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None else torch.device(device).index)
        self.S, self.F, self.n, self.T, self.eps = int(streams), int(n_feat), int(n_frame), int(total_len), float(eps)
        self.buffer = torch.empty((self.S, self.F, self.T), dtype=torch.float32, device=self.device)
        self.reset()

    def reset(self) -> None:
        self.buffer.fill_(ZERO_LEVEL_SPEC_DB_VAL)

    def step(self, frames: torch.Tensor, active: Optional[torch.Tensor] = None,
             out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """frames (S, F, k*n_frame) -> normalised buffers (S*k, F, Tbuf); buffer advanced by k chunks.
        `active` (S,) bool/uint8: streams with 0 are zeroed (the batched reference's `None` frame)."""
        fr = frames.to(self.device, torch.float32).contiguous()
        if fr.dim() != 3 or fr.shape[0] != self.S or fr.shape[1] != self.F or fr.shape[2] % self.n:
            raise ValueError(f"frames {tuple(fr.shape)} must be ({self.S}, {self.F}, k*{self.n})")
        k = fr.shape[2] // self.n
        if out is None:
            out = torch.empty((self.S * k, self.F, self.T), dtype=torch.float32, device=self.device)
        elif out.shape != (self.S * k, self.F, self.T) or out.dtype != torch.float32 or not out.is_contiguous():
            raise ValueError(f"out must be a contiguous fp32 ({self.S * k}, {self.F}, {self.T}) tensor")
        act = None
        if active is not None:
            act = active.to(self.device, torch.uint8).contiguous()
            if act.numel() != self.S:
                raise ValueError(f"active has {act.numel()} flags for {self.S} streams")
        st = ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        _lib.check(self.lib.cfm_frame_buffer_step(self.buffer.data_ptr(), fr.data_ptr(),
                                                  None if act is None else act.data_ptr(), self.S, self.F, self.T,
                                                  self.n, k, ctypes.c_float(self.eps), out.data_ptr(), st),
                   "cfm_frame_buffer_step")
        return out
