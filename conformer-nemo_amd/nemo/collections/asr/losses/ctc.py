"""Drop-in `CTCLoss` (reference nemo/collections/asr/losses/ctc.py:25-70): same constructor
(blank = num_classes, reductions 'mean_batch' | 'sum' | 'mean' | 'none', zero_infinity), the
keyword-only forward(log_probs=, targets=, input_lengths=, target_lengths=) on (B, T, C) log-probs;
the alpha-beta recursion and its gradient run in libcfm.so (include/cfm_ctc.h, cfm_ctc_loss).
"""
from __future__ import annotations

import torch

from nemo.core.classes.common import typecheck
from nemo.core.neural_types import LabelsType, LengthsType, LogprobsType, LossType, NeuralType


class _CtcFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, log_probs, targets, input_lengths, target_lengths, blank, zero_infinity):
        from conformer_amd.ctc import ctc_loss
        nll, grad = ctc_loss(log_probs, targets, input_lengths, target_lengths, blank, zero_infinity,
                             want_grad=ctx.needs_input_grad[0])
        ctx.save_for_backward(grad if grad is not None else nll)
        return nll

    @staticmethod
    def backward(ctx, grad_nll):
        (grad,) = ctx.saved_tensors
        # d sum_b g_b * nll_b / d lp = g_b * (per-utterance gradient)
        return grad * grad_nll.view(-1, 1, 1), None, None, None, None, None


class CTCLoss(torch.nn.Module):
    @property
    def input_types(self):
        return {"log_probs": NeuralType(('B', 'T', 'D'), LogprobsType()),
                "targets": NeuralType(('B', 'T'), LabelsType()),
                "input_lengths": NeuralType(tuple('B'), LengthsType()),
                "target_lengths": NeuralType(tuple('B'), LengthsType())}

    @property
    def output_types(self):
        return {"loss": NeuralType(elements_type=LossType())}

    def __init__(self, num_classes, zero_infinity=False, reduction='mean_batch'):
        super().__init__()
        self._blank = num_classes
        if reduction == 'mean_batch':
            self.reduction, self._apply_batch_mean = 'none', True
        elif reduction in ['sum', 'mean', 'none']:
            self.reduction, self._apply_batch_mean = reduction, False
        else:
            raise ValueError(f"reduction {reduction}")
        self.blank = self._blank
        self.zero_infinity = zero_infinity

    @typecheck()
    def forward(self, log_probs, targets, input_lengths, target_lengths):
        if not log_probs.is_cuda:
            raise RuntimeError("CTCLoss (MI355X-native) needs GPU tensors")
        nll = _CtcFn.apply(log_probs, targets, input_lengths, target_lengths, self._blank, self.zero_infinity)
        if self.reduction == 'sum':
            loss = nll.sum()
        elif self.reduction == 'mean':      # torch: divide by target lengths, then mean
            loss = (nll / target_lengths.to(nll.device).clamp(min=1).to(nll.dtype)).mean()
        else:
            loss = nll
        if self._apply_batch_mean:
            loss = torch.mean(loss)
        return loss
