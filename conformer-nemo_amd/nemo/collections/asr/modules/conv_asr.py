"""Drop-in `ConvASRDecoder` (reference nemo/collections/asr/modules/conv_asr.py:397-472): the CTC
head.  Same constructor, `decoder_layers.0.{weight,bias}` state_dict, keyword-only forward and
`num_classes_with_blank`; the arithmetic (and its backward) runs in libcfm.so
(include/cfm_ctc.h) on the module's GPU.  CPU tensors are refused (no fallback).
"""
from __future__ import annotations

import os
from collections import OrderedDict

import torch

from nemo.core.classes.common import typecheck
from nemo.core.classes.module import NeuralModule
from nemo.core.neural_types import AcousticEncodedRepresentation, LogprobsType, NeuralType


class _HeadFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, enc, weight, bias, native):
        lp, greedy = native.forward(enc)
        ctx.native = native
        ctx.save_for_backward(enc, lp)
        ctx.mark_non_differentiable(greedy)
        return lp, greedy

    @staticmethod
    def backward(ctx, grad_lp, _grad_greedy):
        enc, lp = ctx.saved_tensors
        genc, gw, gb = ctx.native.backward(enc, lp, grad_lp, need_input=ctx.needs_input_grad[0],
                                           need_weight=ctx.needs_input_grad[1] or ctx.needs_input_grad[2])
        if gw is not None:
            gw = gw.view(gw.shape[0], gw.shape[1], 1)
        return genc, gw, gb, None


class ConvASRDecoder(NeuralModule):
    """log_softmax(Conv1d(feat_in, num_classes + 1, k=1)(encoder_output).transpose(1, 2), -1)."""

    @property
    def input_types(self):
        return OrderedDict({"encoder_output": NeuralType(('B', 'D', 'T'), AcousticEncodedRepresentation())})

    @property
    def output_types(self):
        return OrderedDict({"logprobs": NeuralType(('B', 'T', 'D'), LogprobsType())})

    def __init__(self, feat_in, num_classes, init_mode="xavier_uniform", vocabulary=None):
        super().__init__()
        if vocabulary is None and num_classes < 0:
            raise ValueError("Neither of the vocabulary and num_classes are set! At least one of them need to be set.")
        if num_classes <= 0:
            num_classes = len(vocabulary)
        if vocabulary is not None and num_classes != len(vocabulary):
            raise ValueError(f"If vocabulary is specified, it's length should be equal to the num_classes. "
                             f"Instead got: num_classes={num_classes} and len(vocabulary)={len(vocabulary)}")
        self.__vocabulary = vocabulary
        self._feat_in = feat_in
        self._num_classes = num_classes + 1          # + blank (conv_asr.py:430-431)
        self.decoder_layers = torch.nn.Sequential(torch.nn.Conv1d(self._feat_in, self._num_classes, kernel_size=1,
                                                                  bias=True))
        if init_mode == "xavier_uniform":            # jasper.init_weights for Conv1d (jasper.py:94-100)
            torch.nn.init.xavier_uniform_(self.decoder_layers[0].weight, gain=1.0)
        elif init_mode == "xavier_normal":
            torch.nn.init.xavier_normal_(self.decoder_layers[0].weight, gain=1.0)
        elif init_mode == "kaiming_uniform":
            torch.nn.init.kaiming_uniform_(self.decoder_layers[0].weight, nonlinearity="relu")
        elif init_mode == "kaiming_normal":
            torch.nn.init.kaiming_normal_(self.decoder_layers[0].weight, nonlinearity="relu")
        elif init_mode is not None:
            raise ValueError(f"Unknown Initialization mode: {init_mode}")
        self._compute = os.environ.get("CFM_COMPUTE", "bf16")
        self._native = {}
        self._synced = {}

    @property
    def vocabulary(self):
        return self.__vocabulary

    @property
    def num_classes_with_blank(self):
        return self._num_classes

    def set_compute_mode(self, mode: str):
        if mode not in ("bf16", "fp32"):
            raise ValueError(mode)
        self._compute = mode
        self._native.clear()
        self._synced.clear()

    def _native_for(self, dev):
        from conformer_amd.ctc import NativeCtcHead
        key = (dev.index, self._compute)
        nat = self._native.get(key)
        if nat is None:
            nat = NativeCtcHead(self._feat_in, self._num_classes, dev.index, self._compute)
            self._native[key] = nat
        conv = self.decoder_layers[0]
        snap = (conv.weight.data_ptr(), conv.weight._version, conv.bias.data_ptr(), conv.bias._version)
        if self._synced.get(key) != snap:
            nat.set_weights(conv.weight, conv.bias)
            self._synced[key] = snap
        return nat

    @typecheck()
    def forward(self, encoder_output):
        return self.forward_with_predictions(encoder_output)[0]

    def forward_with_predictions(self, encoder_output):
        """log_probs and the greedy argmax (ctc_models.py:594) from one launch sequence."""
        if not encoder_output.is_cuda:
            raise RuntimeError("ConvASRDecoder (MI355X-native) needs a GPU tensor")
        conv = self.decoder_layers[0]
        return _HeadFn.apply(encoder_output, conv.weight, conv.bias, self._native_for(encoder_output.device))

    def input_example(self, max_batch=1, max_dim=256):
        p = next(self.parameters())
        return tuple([torch.randn(max_batch, self._feat_in, max_dim, device=p.device)])
