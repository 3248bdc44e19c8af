"""Host runtime around the C-ABI encoder handle (include/cfm_encoder.h).

`NativeEncoder` owns one `cfm_encoder*` (packed weights + positional table on one GPU) and a
grow-only device workspace, and runs `cfm_encoder_forward` on torch's current HIP stream.
Tensors are passed as raw device pointers; torch is used only for device memory and streams.
"""
from __future__ import annotations

import ctypes
from typing import Dict, Iterable, Optional, Tuple

import torch

from . import _lib

COMPUTE_MODES = {"fp32": _lib.CFM_COMPUTE_FP32, "bf16": _lib.CFM_COMPUTE_BF16, "fp16": _lib.CFM_COMPUTE_FP16}


def encoded_length(T: int) -> int:
    """calc_length (subsampling.py:272-282) via the library (host side)."""
    return _lib.load().cfm_encoded_length(int(T))


def make_cfg(feat_in: int, n_layers: int, d_model: int, feat_out: int = -1, subsampling_factor: int = 4,
             subsampling_conv_channels: int = -1, ff_expansion_factor: int = 4, n_heads: int = 4,
             att_context_size=None, xscaling: bool = True, pos_emb_max_len: int = 5000,
             conv_kernel_size: int = 31, conv_norm_type: str = "batch_norm") -> _lib.CfmEncoderCfg:
    ctx = list(att_context_size) if att_context_size else [-1, -1]
    c = _lib.CfmEncoderCfg()
    c.feat_in, c.n_layers, c.d_model, c.feat_out = int(feat_in), int(n_layers), int(d_model), int(feat_out)
    c.subsampling_factor = int(subsampling_factor)
    c.subsampling_conv_channels = int(subsampling_conv_channels)
    c.ff_expansion_factor = int(ff_expansion_factor)
    c.n_heads = int(n_heads)
    c.att_context_left, c.att_context_right = int(ctx[0]), int(ctx[1])
    c.xscaling = 1 if xscaling else 0
    c.pos_emb_max_len = int(pos_emb_max_len)
    c.conv_kernel_size = int(conv_kernel_size)
    if conv_norm_type not in ("batch_norm", "layer_norm"):
        raise ValueError(f"conv_norm_type={conv_norm_type} is not valid!")
    c.conv_norm_type = 0 if conv_norm_type == "batch_norm" else 1
    return c


class NativeEncoder:
    """One encoder instance on one GPU."""

    def __init__(self, cfg: _lib.CfmEncoderCfg, device: Optional[int] = None, compute: str = "bf16"):
        if compute not in COMPUTE_MODES:
            raise ValueError(f"compute must be one of {list(COMPUTE_MODES)}")
        self.lib = _lib.load(_lib.variant_of(compute))   # fp16: the libcfm_f16.so build
        if not torch.cuda.is_available():
            raise _lib.CfmError("the native Conformer encoder needs a ROCm GPU (torch.cuda.is_available() is False)")
        if compute not in COMPUTE_MODES:
            raise ValueError(f"compute must be one of {list(COMPUTE_MODES)}")
        self.device = torch.cuda.current_device() if device is None else int(device)
        self.compute = compute
        self.cfg = cfg
        h = ctypes.c_void_p()
        _lib.check(self.lib.cfm_encoder_create(ctypes.byref(cfg), self.device, COMPUTE_MODES[compute], ctypes.byref(h)),
                   "cfm_encoder_create", lib=self.lib)
        self.handle = h
        self._ws: Optional[torch.Tensor] = None

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and h.value:
            try:
                self.lib.cfm_encoder_destroy(h)
            except Exception:
                pass
            self.handle = None

    # ---- weights ------------------------------------------------------------------------------
    def param_names(self) -> Dict[str, int]:
        n = self.lib.cfm_encoder_param_count(self.handle)
        return {self.lib.cfm_encoder_param_name(self.handle, i).decode(): int(self.lib.cfm_encoder_param_numel(self.handle, i))
                for i in range(n)}

    def set_weights(self, tensors: Dict[str, torch.Tensor]) -> None:
        """Pack every tensor of the reference state_dict (fp32 copies are made as needed)."""
        keep, views = [], []
        for name, t in tensors.items():
            if not torch.is_floating_point(t):
                continue
            t = t.detach()
            if t.dtype != torch.float32 or not t.is_contiguous():
                t = t.float().contiguous()
            keep.append(t)
            v = _lib.CfmTensorView()
            v.name = name.encode()
            v.data = t.data_ptr()
            v.numel = t.numel()
            v.on_device = 1 if t.is_cuda else 0
            views.append(v)
        arr = (_lib.CfmTensorView * len(views))(*views)
        stream = torch.cuda.current_stream(self.device).cuda_stream
        _lib.check(self.lib.cfm_encoder_set_weights(self.handle, arr, len(views), ctypes.c_void_p(stream)),
                   "cfm_encoder_set_weights", lib=self.lib)
        del keep

    # ---- forward ------------------------------------------------------------------------------
    @property
    def max_audio_length(self) -> int:
        return int(self.lib.cfm_encoder_max_audio_length(self.handle))

    def set_max_audio_length(self, n: int) -> None:
        _lib.check(self.lib.cfm_encoder_set_max_audio_length(self.handle, int(n)), "set_max_audio_length", lib=self.lib)

    def set_pad_mask(self, on: bool) -> None:
        """enable_pad_mask (conformer_encoder.py:301-305): off -> conv module runs with pad_mask=None."""
        _lib.check(self.lib.cfm_encoder_set_pad_mask(self.handle, 1 if on else 0), "set_pad_mask", lib=self.lib)

    def set_abs_pos(self, on: bool) -> None:
        """self_attention_model='abs_pos': absolute sinusoids added after the xscale and plain
        MultiHeadAttention in the layers (cfm_encoder_set_abs_pos).  Clears the weights."""
        _lib.check(self.lib.cfm_encoder_set_abs_pos(self.handle, 1 if on else 0), "set_abs_pos", lib=self.lib)

    @property
    def abs_pos(self) -> bool:
        return bool(self.lib.cfm_encoder_abs_pos(self.handle))

    def set_microbatches(self, n: int) -> None:
        """Split each forward's batch over up to n concurrent streams (bitwise-identical results)."""
        _lib.check(self.lib.cfm_encoder_set_microbatches(self.handle, int(n)), "set_microbatches", lib=self.lib)

    def workspace_size(self, B: int, T: int) -> int:
        return int(self.lib.cfm_encoder_workspace_size(self.handle, int(B), int(T)))

    def _workspace(self, nbytes: int) -> torch.Tensor:
        if self._ws is None or self._ws.numel() < nbytes:
            self._ws = None
            self._ws = torch.empty(nbytes, dtype=torch.uint8, device=f"cuda:{self.device}")
        return self._ws

    def forward(self, x_bft: torch.Tensor, lengths: Optional[torch.Tensor] = None,
                out: Optional[torch.Tensor] = None, out_len: Optional[torch.Tensor] = None
                ) -> Tuple[torch.Tensor, torch.Tensor]:
        if not x_bft.is_cuda or x_bft.dim() != 3:
            raise ValueError("audio_signal must be a (B, feat_in, T) tensor on the GPU")
        if x_bft.dtype != torch.float32 or not x_bft.is_contiguous():
            x_bft = x_bft.float().contiguous()
        B, F, T = x_bft.shape
        if F != self.cfg.feat_in:
            raise ValueError(f"expected feat_in={self.cfg.feat_in}, got {F}")
        if T > self.max_audio_length:      # set_max_audio_length (conformer_encoder.py:240-241)
            torch.cuda.synchronize(self.device)
            self.set_max_audio_length(T)
        Tp = encoded_length(T)
        dout = self.cfg.feat_out if (self.cfg.feat_out > 0 and self.cfg.feat_out != self.cfg.d_model) else self.cfg.d_model
        dev = x_bft.device
        if out is None:
            out = torch.empty((B, dout, Tp), dtype=torch.float32, device=dev)
        if out_len is None:
            out_len = torch.empty((B,), dtype=torch.int32, device=dev)
        len_ptr = None
        if lengths is not None:
            lengths = lengths.to(device=dev, dtype=torch.int32).contiguous()
            len_ptr = lengths.data_ptr()
        nbytes = self.workspace_size(B, T)
        ws = self._workspace(nbytes)
        stream = torch.cuda.current_stream(dev).cuda_stream
        _lib.check(self.lib.cfm_encoder_forward(self.handle, x_bft.data_ptr(), len_ptr, B, T, out.data_ptr(),
                                                out_len.data_ptr(), ws.data_ptr(), nbytes, ctypes.c_void_p(stream)),
                   "cfm_encoder_forward", lib=self.lib)
        return out, out_len

    def layers_forward(self, x_btd: torch.Tensor, lengths: Optional[torch.Tensor] = None,
                       pos_emb: Optional[torch.Tensor] = None) -> torch.Tensor:
        """The ConformerLayer stack alone (cfm_encoder_layers_forward): x (B, T', d) -> (B, T', d) fp32.
        lengths: valid frames per utterance (pad / attention masks); pos_emb: (2T'-1, d) relative
        positions (None = the handle's table)."""
        if not x_btd.is_cuda or x_btd.dim() != 3 or x_btd.shape[-1] != self.cfg.d_model:
            raise ValueError(f"x must be a (B, T, {self.cfg.d_model}) tensor on the GPU")
        x = x_btd.detach().float().contiguous()
        B, Tp, d = x.shape
        dev = x.device
        len_ptr = None
        if lengths is not None:
            lengths = lengths.to(device=dev, dtype=torch.int32).contiguous()
            len_ptr = lengths.data_ptr()
        pe_ptr = None
        if pos_emb is not None:
            pos_emb = pos_emb.detach().to(device=dev, dtype=torch.float32).reshape(-1, d).contiguous()
            if pos_emb.shape[0] != 2 * Tp - 1:
                raise ValueError(f"pos_emb must hold 2T'-1 = {2 * Tp - 1} rows, got {pos_emb.shape[0]}")
            pe_ptr = pos_emb.data_ptr()
        elif Tp > self.max_audio_length:
            torch.cuda.synchronize(self.device)
            self.set_max_audio_length(Tp)
        y = torch.empty_like(x)
        nbytes = int(self.lib.cfm_encoder_layers_workspace_size(self.handle, B, Tp))
        ws = self._workspace(nbytes)
        stream = torch.cuda.current_stream(dev).cuda_stream
        _lib.check(self.lib.cfm_encoder_layers_forward(self.handle, x.data_ptr(), len_ptr, B, Tp, pe_ptr, y.data_ptr(),
                                                       ws.data_ptr(), nbytes, ctypes.c_void_p(stream)),
                   "cfm_encoder_layers_forward", lib=self.lib)
        return y

    def forward_timed(self, x_bft: torch.Tensor, lengths: Optional[torch.Tensor] = None):
        """Per-stage kernel timing (cfm_encoder_forward_timed): one production forward in which every
        kernel carries a start and a stop event in its own dispatch packet, so a kernel's time is its
        packet's begin -> end, the duration rocprofv3's kernel trace reports (CFM_STAGE_CLOCK=chain:
        stop events only, chained; =burst: each launch replayed 8x between stream events).
        Returns {stage: (device ms per forward, launches per forward)}."""
        B, F, T = x_bft.shape
        Tp = encoded_length(T)
        dout = self.cfg.feat_out if (self.cfg.feat_out > 0 and self.cfg.feat_out != self.cfg.d_model) else self.cfg.d_model
        out = torch.empty((B, dout, Tp), dtype=torch.float32, device=x_bft.device)
        out_len = torch.empty((B,), dtype=torch.int32, device=x_bft.device)
        len_ptr = None
        if lengths is not None:
            lengths = lengths.to(device=x_bft.device, dtype=torch.int32).contiguous()
            len_ptr = lengths.data_ptr()
        n = self.lib.cfm_num_stages()
        ms = (ctypes.c_float * n)()
        cnt = (ctypes.c_int * n)()
        nbytes = self.workspace_size(B, T)
        ws = self._workspace(nbytes)
        stream = torch.cuda.current_stream(x_bft.device).cuda_stream
        _lib.check(self.lib.cfm_encoder_forward_timed(self.handle, x_bft.data_ptr(), len_ptr, B, T, out.data_ptr(),
                                                      out_len.data_ptr(), ws.data_ptr(), nbytes, ctypes.c_void_p(stream),
                                                      ms, cnt), "cfm_encoder_forward_timed", lib=self.lib)
        return {self.lib.cfm_stage_name(i).decode(): (float(ms[i]), int(cnt[i])) for i in range(n)}

    def stage_clock_overhead_us(self, n: int = 200) -> float:
        """The stage clock's own cost per kernel (cfm_stage_clock_overhead): the mean begin -> end of n
        empty one-wave kernels timed the way forward_timed times each kernel."""
        us = ctypes.c_float(0.0)
        stream = torch.cuda.current_stream(self.device).cuda_stream
        _lib.check(self.lib.cfm_stage_clock_overhead(ctypes.c_void_p(stream), int(n), ctypes.byref(us)),
                   "cfm_stage_clock_overhead", lib=self.lib)
        return float(us.value)
