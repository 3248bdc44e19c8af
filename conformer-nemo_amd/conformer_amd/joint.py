"""Host runtime around the C-ABI RNN-T joint (include/cfm_joint.h).

`NativeJoint` owns one `cfm_rnnt_joint*` (packed enc / pred / joint_net weights on one GPU) and a
grow-only workspace; `forward` runs cfm_rnnt_joint_forward on torch's current stream.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import torch

from . import _lib
from .runtime import COMPUTE_MODES

ACTIVATIONS = {"relu": 0, "sigmoid": 1, "tanh": 2}


class NativeJoint:
    """RNNTJoint.joint arithmetic (rnnt.py:951-1008) on one GPU."""

    def __init__(self, encoder_hidden: int, pred_hidden: int, joint_hidden: int, num_classes: int,
                 activation: str = "relu", device=None, compute: str = "bf16"):
        self.lib = _lib.load()
        if not torch.cuda.is_available():
            raise _lib.CfmError("the native RNN-T joint needs a ROCm GPU (torch.cuda.is_available() is False)")
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None else device)
        self.dims = (int(encoder_hidden), int(pred_hidden), int(joint_hidden), int(num_classes))
        h = ctypes.c_void_p()
        _lib.check(self.lib.cfm_rnnt_joint_create(*self.dims, ACTIVATIONS[activation.lower()], self.device.index,
                                                  COMPUTE_MODES[compute], ctypes.byref(h)), "cfm_rnnt_joint_create")
        self.handle = h
        self._ws: Optional[torch.Tensor] = None

    def __del__(self):
        h = getattr(self, "handle", None)
        if h:
            self.lib.cfm_rnnt_joint_destroy(h)
            self.handle = None

    def set_weights(self, w_enc, b_enc, w_pred, b_pred, w_out, b_out) -> None:
        ts = [None if t is None else t.detach().to(self.device, torch.float32).contiguous()
              for t in (w_enc, b_enc, w_pred, b_pred, w_out, b_out)]
        st = ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        _lib.check(self.lib.cfm_rnnt_joint_set_weights(self.handle, *[None if t is None else t.data_ptr() for t in ts],
                                                       st), "cfm_rnnt_joint_set_weights")

    def forward(self, enc_bdt: torch.Tensor, dec_bdu: torch.Tensor, log_softmax: bool = False,
                out: Optional[torch.Tensor] = None) -> torch.Tensor:
        e = enc_bdt.detach().to(self.device, torch.float32).contiguous()
        g = dec_bdu.detach().to(self.device, torch.float32).contiguous()
        B, H1, T = e.shape
        B2, H2, U = g.shape
        if B2 != B or H1 != self.dims[0] or H2 != self.dims[1]:
            raise ValueError(f"joint inputs {tuple(e.shape)} / {tuple(g.shape)} do not match dims {self.dims}")
        C = self.dims[3]
        if out is None:
            out = torch.empty((B, T, U, C), dtype=torch.float32, device=self.device)
        n = int(self.lib.cfm_rnnt_joint_workspace_size(self.handle, B, T, U))
        if self._ws is None or self._ws.numel() < n:
            self._ws = None
            self._ws = torch.empty(n, dtype=torch.uint8, device=self.device)
        st = ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        _lib.check(self.lib.cfm_rnnt_joint_forward(self.handle, e.data_ptr(), g.data_ptr(), B, T, U,
                                                   1 if log_softmax else 0, out.data_ptr(), self._ws.data_ptr(), n, st),
                   "cfm_rnnt_joint_forward")
        return out

    # ---- training (cfm_rnnt_joint_forward_train / cfm_rnnt_joint_backward) ------------------------
    def forward_train(self, enc_bdt: torch.Tensor, dec_bdu: torch.Tensor, dropout: float, seed: int) -> torch.Tensor:
        e = enc_bdt.detach().to(self.device, torch.float32).contiguous()
        g = dec_bdu.detach().to(self.device, torch.float32).contiguous()
        B, _, T = e.shape
        U = g.shape[2]
        out = torch.empty((B, T, U, self.dims[3]), dtype=torch.float32, device=self.device)
        n = int(self.lib.cfm_rnnt_joint_workspace_size(self.handle, B, T, U))
        ws = self._grow(n)
        st = ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        _lib.check(self.lib.cfm_rnnt_joint_forward_train(self.handle, e.data_ptr(), g.data_ptr(), B, T, U,
                                                         ctypes.c_float(dropout), ctypes.c_uint64(seed), out.data_ptr(),
                                                         ws.data_ptr(), n, st), "cfm_rnnt_joint_forward_train")
        return out

    def backward(self, enc_bdt, dec_bdu, dlogits, dropout: float, seed: int, w_enc, w_pred, w_out, want):
        """want = (d_enc, d_dec, w_enc, b_enc, w_pred, b_pred, w_out, b_out) -> the same tuple of tensors / None."""
        e = enc_bdt.detach().to(self.device, torch.float32).contiguous()
        g = dec_bdu.detach().to(self.device, torch.float32).contiguous()
        dl = dlogits.detach().to(self.device, torch.float32).contiguous()
        B, H1, T = e.shape
        _, H2, U = g.shape
        H, C = self.dims[2], self.dims[3]
        f = lambda t: t.detach().to(self.device, torch.float32).contiguous()  # noqa: E731
        shapes = [(B, H1, T), (B, H2, U), (H, H1), (H,), (H, H2), (H,), (C, H), (C,)]
        outs = [torch.empty(sh, device=self.device) if w else None for sh, w in zip(shapes, want)]
        n = int(self.lib.cfm_rnnt_joint_backward_workspace_size(self.handle, B, T, U))
        ws = torch.empty(n, dtype=torch.uint8, device=self.device)
        st = ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        we, wp, wo = f(w_enc), f(w_pred), f(w_out)
        ptr = lambda t: None if t is None else t.data_ptr()  # noqa: E731
        _lib.check(self.lib.cfm_rnnt_joint_backward(self.handle, e.data_ptr(), g.data_ptr(), B, T, U,
                                                    ctypes.c_float(dropout), ctypes.c_uint64(seed), dl.data_ptr(),
                                                    we.data_ptr(), wp.data_ptr(), wo.data_ptr(), *[ptr(t) for t in outs],
                                                    ws.data_ptr(), n, st), "cfm_rnnt_joint_backward")
        return outs

    def _grow(self, n: int) -> torch.Tensor:
        if self._ws is None or self._ws.numel() < n:
            self._ws = None
            self._ws = torch.empty(n, dtype=torch.uint8, device=self.device)
        return self._ws
