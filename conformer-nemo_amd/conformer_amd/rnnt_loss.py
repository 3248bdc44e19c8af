"""Host runtime around the C-ABI RNN-T loss (include/cfm_rnnt_loss.h), SURVEY §8 row f2.

`rnnt_loss(acts, labels, act_lens, label_lens, ...)` runs the three-kernel loss on torch's current
stream and returns per-utterance costs and (optionally) the gradient w.r.t. the raw joint logits,
as the reference's GPU numba loss produces them (gpu_rnnt.py:122-238).
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib


def rnnt_loss(acts: torch.Tensor, labels: torch.Tensor, act_lens: torch.Tensor, label_lens: torch.Tensor, blank: int,
              fastemit_lambda: float = 0.0, clamp: float = 0.0, want_grads: bool = True):
    lib = _lib.load()
    if not acts.is_cuda:
        raise _lib.CfmError("the native RNN-T loss needs CUDA tensors")
    dev = acts.device
    a = acts.detach().float().contiguous()
    if a.dim() != 4:
        raise ValueError(f"acts must be (B, T, U+1, V+1), got {tuple(a.shape)}")
    B, T, U, V = a.shape
    lab = labels.to(dev, torch.int32).contiguous()
    if lab.dim() != 2 or lab.shape[0] != B:
        raise ValueError("labels must be (B, L)")
    if lab.shape[1] == 0:
        lab = torch.zeros((B, 1), dtype=torch.int32, device=dev)
    al = act_lens.to(dev, torch.int32).contiguous()
    ll = label_lens.to(dev, torch.int32).contiguous()
    costs = torch.empty(B, dtype=torch.float32, device=dev)
    grads = torch.empty_like(a) if want_grads else None
    n = int(lib.cfm_rnnt_loss_workspace_size(B, T, U))
    ws = torch.empty(n, dtype=torch.uint8, device=dev)
    st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    _lib.check(lib.cfm_rnnt_loss(a.data_ptr(), lab.data_ptr(), lab.shape[1], al.data_ptr(), ll.data_ptr(), B, T, U, V,
                                 int(blank), ctypes.c_float(fastemit_lambda), ctypes.c_float(clamp), costs.data_ptr(),
                                 None if grads is None else grads.data_ptr(), ws.data_ptr(), n, st), "cfm_rnnt_loss")
    return costs, grads
