"""Host runtime around the C-ABI RNN-T loss (include/cfm_rnnt_loss.h), SURVEY §8 row f2.

`rnnt_loss(acts, labels, act_lens, label_lens, ...)` runs the three-kernel loss on torch's current
stream and returns per-utterance costs and (optionally) the gradient w.r.t. the raw joint logits,
as the reference's GPU numba loss produces them (gpu_rnnt.py:122-238).
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib


def _prepare(acts, labels, act_lens, label_lens):
    if not acts.is_cuda:
        raise _lib.CfmError("the native RNN-T loss needs CUDA tensors")
    dev = acts.device
    a = acts.detach().float().contiguous()
    if a.dim() != 4:
        raise ValueError(f"acts must be (B, T, U+1, V+1), got {tuple(a.shape)}")
    B = a.shape[0]
    lab = labels.to(dev, torch.int32).contiguous()
    if lab.dim() != 2 or lab.shape[0] != B:
        raise ValueError("labels must be (B, L)")
    if lab.shape[1] == 0:
        lab = torch.zeros((B, 1), dtype=torch.int32, device=dev)
    al = act_lens.to(dev, torch.int32).contiguous()
    ll = label_lens.to(dev, torch.int32).contiguous()
    return a, lab, al, ll


def rnnt_loss(acts: torch.Tensor, labels: torch.Tensor, act_lens: torch.Tensor, label_lens: torch.Tensor, blank: int,
              fastemit_lambda: float = 0.0, clamp: float = 0.0, want_grads: bool = True, keep_state: bool = False):
    """costs (B) and grads (acts' shape, or None).  keep_state (with want_grads False): also return the
    state rnnt_loss_grad needs to produce the gradient later, in the backward."""
    lib = _lib.load()
    a, lab, al, ll = _prepare(acts, labels, act_lens, label_lens)
    dev = a.device
    B, T, U, V = a.shape
    costs = torch.empty(B, dtype=torch.float32, device=dev)
    if keep_state and want_grads:
        raise ValueError("keep_state computes the gradient later: want_grads must be False")
    grads = torch.empty_like(a) if want_grads else None
    n = int(lib.cfm_rnnt_loss_workspace_size(B, T, U))
    ws = torch.empty(n, dtype=torch.uint8, device=dev)
    st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    if keep_state:   # costs + both lattices, the gradient later (rnnt_loss_grad)
        _lib.check(lib.cfm_rnnt_loss_costs(a.data_ptr(), lab.data_ptr(), lab.shape[1], al.data_ptr(), ll.data_ptr(), B,
                                           T, U, V, int(blank), ctypes.c_float(fastemit_lambda), costs.data_ptr(),
                                           ws.data_ptr(), n, st), "cfm_rnnt_loss_costs")
    else:
        _lib.check(lib.cfm_rnnt_loss(a.data_ptr(), lab.data_ptr(), lab.shape[1], al.data_ptr(), ll.data_ptr(), B, T, U,
                                     V, int(blank), ctypes.c_float(fastemit_lambda), ctypes.c_float(clamp),
                                     costs.data_ptr(), None if grads is None else grads.data_ptr(), ws.data_ptr(), n,
                                     st), "cfm_rnnt_loss")
    if keep_state:
        return costs, grads, (a, lab, al, ll, ws, int(blank), float(fastemit_lambda), float(clamp))
    return costs, grads


def rnnt_loss_grad(state, pre_scale: float = 1.0, scale: torch.Tensor = None) -> torch.Tensor:
    """The gradient w.r.t. acts from a rnnt_loss(..., want_grads=False, keep_state=True) state, times
    pre_scale and the per-utterance scale (B) - the reference's forward gradient after its in-place
    multiplies (cfm_rnnt_loss_grad)."""
    lib = _lib.load()
    a, lab, al, ll, ws, blank, fastemit_lambda, clamp = state
    B, T, U, V = a.shape
    sc = None
    if scale is not None:
        sc = scale.detach().to(a.device, torch.float32).reshape(-1)
        sc = (sc.expand(B) if sc.numel() == 1 else sc).contiguous()
        if sc.numel() != B:
            raise ValueError(f"scale must have 1 or B={B} elements")
    grads = torch.empty_like(a)
    st = ctypes.c_void_p(torch.cuda.current_stream(a.device).cuda_stream)
    _lib.check(lib.cfm_rnnt_loss_grad(a.data_ptr(), lab.data_ptr(), lab.shape[1], al.data_ptr(), ll.data_ptr(), B, T,
                                      U, V, blank, ctypes.c_float(fastemit_lambda), ctypes.c_float(clamp),
                                      ctypes.c_float(pre_scale), None if sc is None else sc.data_ptr(), grads.data_ptr(),
                                      ws.data_ptr(), ws.numel(), st), "cfm_rnnt_loss_grad")
    return grads
