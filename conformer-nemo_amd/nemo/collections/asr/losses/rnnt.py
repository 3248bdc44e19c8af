"""Drop-in `RNNTLoss` (reference nemo/collections/asr/losses/rnnt.py:163-306) and the loss it resolves
to by default, `RNNTLossNumba` (numba/rnnt_loss/rnnt_pytorch.py:36-219), SURVEY §8 row f2.

Same constructor (num_classes -> blank = num_classes, reduction 'mean_batch' | 'mean' | 'sum' |
None, loss_name 'default' | 'warprnnt_numba', loss_kwargs fastemit_lambda / clamp), the same
keyword-only forward(log_probs=, targets=, input_lengths=, target_lengths=) taking the joint's raw
logits (B, T, U+1, V+1), the same input checks (certify_inputs) and narrowing.  The log-softmax,
alpha/beta lattices and the gradient w.r.t. the logits run in libcfm.so (include/cfm_rnnt_loss.h);
like the reference GPU path, the gradient is computed in forward and scaled in backward.
"""
from __future__ import annotations

import os

import torch

from nemo.core.classes.common import typecheck
from nemo.core.neural_types import LabelsType, LengthsType, LogprobsType, LossType, NeuralType

RNNT_LOSS_NAMES = ("default", "warprnnt_numba")


def resolve_rnnt_default_loss_name() -> str:
    return "warprnnt_numba"


def certify_inputs(log_probs, labels, lengths, label_lengths):
    """rnnt_pytorch.py:179-219"""
    for t, name in ((labels, "labels"), (label_lengths, "label_lengths"), (lengths, "lengths")):
        if t.dtype is not torch.int32:
            raise TypeError(f"{name} must be {torch.int32}")
    for t, name in ((log_probs, "log_probs"), (labels, "labels"), (label_lengths, "label_lengths"),
                    (lengths, "lengths")):
        if not t.is_contiguous():
            raise ValueError(f"{name} must be contiguous")
    if lengths.shape[0] != log_probs.shape[0]:
        raise ValueError(f"Must have a length per example. Given lengths dim: {lengths.shape[0]}, "
                         f"Log probs dim : {log_probs.shape[0]}")
    if label_lengths.shape[0] != log_probs.shape[0]:
        raise ValueError(f"Must have a label length per example. Given label lengths dim : {label_lengths.shape[0]}, "
                         f"Log probs dim : {log_probs.shape[0]}")
    for t, dim, name in ((log_probs, 4, "log_probs"), (labels, 2, "labels"), (lengths, 1, "lenghts"),
                         (label_lengths, 1, "label_lenghts")):
        if len(t.shape) != dim:
            raise ValueError(f"{name} must be {dim}D")
    max_T, max_U = int(torch.max(lengths)), int(torch.max(label_lengths))
    T, U = log_probs.shape[1:3]
    if T != max_T:
        raise ValueError(f"Input length mismatch! Given T: {T}, Expected max T from input lengths: {max_T}")
    if U != max_U + 1:
        raise ValueError(f"Output length mismatch! Given U: {U}, Expected max U from target lengths: {max_U} + 1")


class _RNNTNative(torch.autograd.Function):
    """_RNNTNumba (rnnt_pytorch.py:36-84) on the native kernels."""

    @staticmethod
    def forward(ctx, acts, labels, act_lens, label_lens, blank, reduction, fastemit_lambda, clamp):
        from conformer_amd.rnnt_loss import rnnt_loss
        certify_inputs(acts, labels, act_lens, label_lens)
        if clamp < 0:
            raise ValueError("`clamp` must be 0.0 or positive float value.")
        # The reference writes the gradient here and scales it in place in the backward.  Deferred (default):
        # the backward writes it once, already scaled (cfm_rnnt_loss_grad, the same fp32 roundings) - one
        # pass over the (B, T, U, V) tensor instead of three.  CFM_RNNT_DEFER_GRAD=0: the reference order.
        defer = acts.requires_grad and os.environ.get("CFM_RNNT_DEFER_GRAD", "1") != "0"
        ctx.state, ctx.pre, ctx.alias = None, 1.0, False
        if defer:
            costs, grads, ctx.state = rnnt_loss(acts, labels, act_lens, label_lens, blank, fastemit_lambda, clamp,
                                                want_grads=False, keep_state=True)
            if ctx.state[0].data_ptr() == acts.data_ptr():
                # the kept logits ARE acts: save them through autograd, so that an in-place change of acts
                # before the backward raises (version check) and a second backward through a freed graph
                # raises as usual, while a retained graph can be differentiated again
                ctx.save_for_backward(acts)
                ctx.state = (None,) + tuple(ctx.state[1:])
                ctx.alias = True
        else:
            costs, grads = rnnt_loss(acts, labels, act_lens, label_lens, blank, fastemit_lambda, clamp,
                                     want_grads=acts.requires_grad)
        costs = costs.to(acts.dtype)
        if reduction in ["sum", "mean"]:
            costs = costs.sum().unsqueeze_(-1)
            if reduction == "mean":
                costs /= acts.shape[0]
                if grads is not None:
                    grads /= acts.shape[0]
                ctx.pre = float(torch.tensor(1.0, dtype=torch.float32) / acts.shape[0])   # ATen's reciprocal
        ctx.grads = grads
        return costs

    @staticmethod
    def backward(ctx, grad_output):
        if grad_output is not None and ctx.state is not None:
            from conformer_amd.rnnt_loss import rnnt_loss_grad
            state = ctx.state
            if ctx.alias:
                state = (ctx.saved_tensors[0],) + tuple(state[1:])
            # the state stays with the node: a retained graph gets the same gradient on every backward
            grads = rnnt_loss_grad(state, ctx.pre, grad_output)
            return grads, None, None, None, None, None, None, None
        if grad_output is not None and ctx.grads is not None:
            grad_output = grad_output.view(-1, 1, 1, 1).to(ctx.grads)
            return ctx.grads.mul_(grad_output), None, None, None, None, None, None, None
        return None, None, None, None, None, None, None, None


class RNNTLossNumba(torch.nn.Module):
    """rnnt_pytorch.py:158-219 (GPU path: the log-softmax is folded into the loss)."""

    def __init__(self, blank=0, reduction="mean", fastemit_lambda: float = 0.0, clamp: float = -1):
        super().__init__()
        self.blank = blank
        self.fastemit_lambda = fastemit_lambda
        self.clamp = float(clamp) if clamp > 0 else 0.0
        self.reduction = reduction

    def forward(self, acts, labels, act_lens, label_lens):
        if not acts.is_cuda:
            raise RuntimeError("RNNTLoss (MI355X-native) needs GPU tensors")
        return _RNNTNative.apply(acts, labels, act_lens, label_lens, self.blank, self.reduction,
                                 self.fastemit_lambda, self.clamp)


def resolve_rnnt_loss(loss_name: str, blank_idx: int, loss_kwargs: dict = None) -> torch.nn.Module:
    """losses/rnnt.py:94-160 for the losses this build provides."""
    if loss_name not in RNNT_LOSS_NAMES:
        raise ValueError(f"Provided `loss_name` {loss_name} not in list of available RNNT losses \n{list(RNNT_LOSS_NAMES)}")
    kw = dict(loss_kwargs or {})
    fastemit_lambda = kw.pop("fastemit_lambda", 0.0)
    clamp = kw.pop("clamp", -1.0)
    return RNNTLossNumba(blank=blank_idx, reduction="none", fastemit_lambda=fastemit_lambda, clamp=clamp)


class RNNTLoss(torch.nn.Module):
    @property
    def input_types(self):
        return {"log_probs": NeuralType(("B", "T", "T", "D"), LogprobsType()),
                "targets": NeuralType(("B", "T"), LabelsType()),
                "input_lengths": NeuralType(tuple("B"), LengthsType()),
                "target_lengths": NeuralType(tuple("B"), LengthsType())}

    @property
    def output_types(self):
        return {"loss": NeuralType(elements_type=LossType())}

    def __init__(self, num_classes, reduction: str = "mean_batch", loss_name: str = "default", loss_kwargs=None):
        super().__init__()
        if reduction not in [None, "mean", "sum", "mean_batch"]:
            raise ValueError("`reduction` must be one of [mean, sum, mean_batch]")
        self._blank = num_classes
        self.reduction = reduction
        self._loss = resolve_rnnt_loss(loss_name, blank_idx=self._blank, loss_kwargs=loss_kwargs)

    @typecheck()
    def forward(self, log_probs, targets, input_lengths, target_lengths):
        """losses/rnnt.py:252-306"""
        targets = targets.int()
        input_lengths = input_lengths.int()
        target_lengths = target_lengths.int()
        max_logit_len = input_lengths.max()
        max_targets_len = target_lengths.max()
        if log_probs.dtype != torch.float32:
            log_probs = log_probs.float()
        if log_probs.shape[1] != max_logit_len:
            log_probs = log_probs.narrow(dim=1, start=0, length=int(max_logit_len)).contiguous()
        if targets.shape[1] != max_targets_len:
            targets = targets.narrow(dim=1, start=0, length=int(max_targets_len))
        targets = targets.contiguous()
        if self.reduction != "mean_batch":
            self._loss.reduction = self.reduction
        loss = self._loss(acts=log_probs, labels=targets, act_lens=input_lengths, label_lens=target_lengths)
        if self.reduction != "mean_batch":
            self._loss.reduction = "none"
        if self.reduction == "mean_batch":
            loss = torch.mean(loss)
        return loss
