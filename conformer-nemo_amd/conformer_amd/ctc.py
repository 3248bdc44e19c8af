"""Host runtime around the C-ABI CTC head and CTC loss (include/cfm_ctc.h).

`NativeCtcHead` owns one `cfm_ctc_head*` (packed W and W^T on one GPU) and a grow-only device
workspace; `ctc_loss` runs `cfm_ctc_loss` on torch's current stream.  Tensors are passed as raw
device pointers; torch provides device memory and streams only.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Tuple

import torch

from . import _lib
from .runtime import COMPUTE_MODES


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else t.data_ptr()


def _stream(dev: torch.device):
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


class NativeCtcHead:
    """ConvASRDecoder arithmetic (conv_asr.py:442-444) and its backward on one GPU."""

    def __init__(self, feat_in: int, num_classes: int, device=None, compute: str = "bf16"):
        self.lib = _lib.load()
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None else device)
        self.feat_in, self.num_classes = int(feat_in), int(num_classes)
        h = ctypes.c_void_p()
        _lib.check(self.lib.cfm_ctc_head_create(self.feat_in, self.num_classes, self.device.index,
                                                COMPUTE_MODES[compute], ctypes.byref(h)), "cfm_ctc_head_create")
        self.handle = h
        self._ws = None

    def __del__(self):
        h = getattr(self, "handle", None)
        if h:
            self.lib.cfm_ctc_head_destroy(h)
            self.handle = None

    def set_weights(self, weight: torch.Tensor, bias: Optional[torch.Tensor]) -> None:
        w = weight.detach().to(self.device, torch.float32).reshape(self.num_classes, self.feat_in).contiguous()
        b = None if bias is None else bias.detach().to(self.device, torch.float32).contiguous()
        _lib.check(self.lib.cfm_ctc_head_set_weights(self.handle, w.data_ptr(), _ptr(b), _stream(self.device)),
                   "cfm_ctc_head_set_weights")
        # stream-ordered: a temporary w / b freed here is only reused by work queued after the pack

    def _workspace(self, B: int, T: int) -> torch.Tensor:
        n = self.lib.cfm_ctc_head_workspace_size(self.handle, B, T)
        if self._ws is None or self._ws.numel() < n:
            self._ws = torch.empty(n, dtype=torch.uint8, device=self.device)
        return self._ws

    def forward(self, enc_bdt: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """(B, D, T) fp32 -> log_probs (B, T, C) fp32, greedy predictions (B, T) int64."""
        x = enc_bdt.detach().to(torch.float32).contiguous()
        B, D, T = x.shape
        if D != self.feat_in:
            raise ValueError(f"encoder_output has {D} features, the head expects {self.feat_in}")
        lp = torch.empty((B, T, self.num_classes), dtype=torch.float32, device=x.device)
        greedy = torch.empty((B, T), dtype=torch.int32, device=x.device)
        ws = self._workspace(B, T)
        _lib.check(self.lib.cfm_ctc_head_forward(self.handle, x.data_ptr(), B, T, lp.data_ptr(), greedy.data_ptr(),
                                                 ws.data_ptr(), ws.numel(), _stream(x.device)), "cfm_ctc_head_forward")
        return lp, greedy.long()

    def backward(self, enc_bdt: torch.Tensor, log_probs: torch.Tensor, grad_lp: torch.Tensor,
                 need_input: bool = True, need_weight: bool = True):
        x = enc_bdt.detach().to(torch.float32).contiguous()
        B, D, T = x.shape
        lp = log_probs.detach().contiguous()
        g = grad_lp.detach().to(torch.float32).contiguous()
        genc = torch.empty_like(x) if need_input else None
        gw = torch.empty((self.num_classes, D), dtype=torch.float32, device=x.device) if need_weight else None
        gb = torch.empty((self.num_classes,), dtype=torch.float32, device=x.device) if need_weight else None
        ws = self._workspace(B, T)
        _lib.check(self.lib.cfm_ctc_head_backward(self.handle, x.data_ptr(), B, T, lp.data_ptr(), g.data_ptr(),
                                                  _ptr(genc), _ptr(gw), _ptr(gb), ws.data_ptr(), ws.numel(),
                                                  _stream(x.device)), "cfm_ctc_head_backward")
        return genc, gw, gb


def ctc_loss(log_probs: torch.Tensor, targets: torch.Tensor, input_lengths: torch.Tensor,
             target_lengths: torch.Tensor, blank: int, zero_infinity: bool, grad_scale: float = 1.0,
             want_grad: bool = True) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    """cfm_ctc_loss: per-utterance nll (B,) and grad_scale * d nll / d log_probs (torch convention)."""
    lib = _lib.load()
    lp = log_probs.detach().to(torch.float32).contiguous()
    B, T, C = lp.shape
    dev = lp.device
    tl = target_lengths.to(device=dev, dtype=torch.int32).contiguous()
    tg = targets.to(device=dev, dtype=torch.int32)
    if tg.dim() == 1:
        # torch's 1-D form: the utterances' targets concatenated (length sum(target_lengths)) ->
        # padded (B, max(target_lengths)) through the cumulative offsets
        tl64 = tl.to(torch.int64)
        U1 = int(tl64.max().item()) if B > 0 else 0
        if tg.numel() != int(tl64.sum().item()):
            raise ValueError(f"1-D targets hold {tg.numel()} labels but target_lengths sum to {int(tl64.sum())}")
        start = torch.cumsum(tl64, 0) - tl64
        col = torch.arange(max(U1, 1), device=dev, dtype=torch.int64)
        idx = (start[:, None] + col[None, :]).clamp_(max=max(tg.numel() - 1, 0))
        tg = torch.where(col[None, :] < tl64[:, None], tg[idx] if tg.numel() else torch.zeros_like(idx, dtype=torch.int32),
                         torch.zeros((), dtype=torch.int32, device=dev))[:, :U1]
    tg = tg.contiguous()
    U = tg.shape[1]
    il = input_lengths.to(device=dev, dtype=torch.int32).contiguous()
    nll = torch.empty(B, dtype=torch.float32, device=dev)
    grad = torch.empty_like(lp) if want_grad else None
    n = lib.cfm_ctc_loss_workspace_size(B, T, C, U)
    ws = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
    _lib.check(lib.cfm_ctc_loss(lp.data_ptr(), tg.data_ptr() if U > 0 else None, il.data_ptr(), tl.data_ptr(), B, T,
                                C, U, int(blank), 1 if zero_infinity else 0, float(grad_scale), nll.data_ptr(),
                                _ptr(grad), ws.data_ptr(), ws.numel(), _stream(dev)), "cfm_ctc_loss")
    return nll, grad
