"""Drop-in `nemo.collections.asr.modules.RNNTJoint` (reference nemo/collections/asr/modules/rnnt.py:613-1038)
backed by the MI355X-native joint (include/cfm_joint.h).

Same constructor (jointnet dict with encoder_hidden / pred_hidden / joint_hidden / activation /
dropout, num_classes, vocabulary, log_softmax, preserve_memory, fuse_loss_wer, fused_batch_size),
same `pred` / `enc` / `joint_net` parameter names (state_dicts load unchanged), keyword-only
forward(encoder_outputs=(B, H1, T), decoder_outputs=(B, H2, U)) -> (B, T, U, V + 1).

log_softmax semantics follow rnnt.py:998-1006: None -> logits on a GPU (the native path only runs
on a GPU), True -> log-probs, False -> logits.  Differences by design: inference only (the joint's
backward and the fused joint+RNNT-loss+WER path need the RNNT loss, SURVEY §8f2, which is not
built: `fuse_loss_wer=True`, or a forward that requires grad, raises NotImplementedError).
"""
from __future__ import annotations

import os
from collections import OrderedDict
from typing import Any, Dict, List, Optional

import torch

from nemo.core.classes.common import typecheck
from nemo.core.classes.module import NeuralModule
from nemo.core.neural_types import AcousticEncodedRepresentation, LogprobsType, NeuralType

__all__ = ["RNNTJoint"]


class RNNTJoint(NeuralModule):
    @property
    def input_types(self):
        return OrderedDict({"encoder_outputs": NeuralType(("B", "D", "T"), AcousticEncodedRepresentation()),
                            "decoder_outputs": NeuralType(("B", "D", "T"), AcousticEncodedRepresentation())})

    @property
    def output_types(self):
        return OrderedDict({"outputs": NeuralType(("B", "T", "T", "D"), LogprobsType())})

    def __init__(self, jointnet: Dict[str, Any], num_classes: int, vocabulary: Optional[List] = None,
                 log_softmax: Optional[bool] = None, preserve_memory: bool = False, fuse_loss_wer: bool = False,
                 fused_batch_size: Optional[int] = None, experimental_fuse_loss_wer: Any = None):
        super().__init__()
        self.vocabulary = vocabulary
        self._vocab_size = num_classes
        self._num_classes = num_classes + 1            # + blank (rnnt.py:729)
        if experimental_fuse_loss_wer is not None:
            fuse_loss_wer = experimental_fuse_loss_wer
        if fuse_loss_wer and fused_batch_size is None:
            raise ValueError("If `fuse_loss_wer` is set, then `fused_batch_size` cannot be None!")
        self._fuse_loss_wer = fuse_loss_wer
        self._fused_batch_size = fused_batch_size
        self.log_softmax = log_softmax
        self.preserve_memory = preserve_memory
        self.encoder_hidden = jointnet["encoder_hidden"]
        self.pred_hidden = jointnet["pred_hidden"]
        self.joint_hidden = jointnet["joint_hidden"]
        self.activation = jointnet["activation"]
        dropout = jointnet.get("dropout", 0.0)
        if self.activation not in ["relu", "sigmoid", "tanh"]:
            raise ValueError("Unsupported activation for joint step - please pass one of [relu, sigmoid, tanh]")
        # module tree of _joint_net_modules (rnnt.py:1010-1038): pred, enc, joint_net = [act, (dropout), Linear]
        self.pred = torch.nn.Linear(self.pred_hidden, self.joint_hidden)
        self.enc = torch.nn.Linear(self.encoder_hidden, self.joint_hidden)
        act = {"relu": torch.nn.ReLU(inplace=True), "sigmoid": torch.nn.Sigmoid(), "tanh": torch.nn.Tanh()}[
            self.activation.lower()]
        layers = [act] + ([torch.nn.Dropout(p=dropout)] if dropout else []) + [
            torch.nn.Linear(self.joint_hidden, self._num_classes)]
        self.joint_net = torch.nn.Sequential(*layers)
        self.compute = os.environ.get("CFM_COMPUTE", "bf16")
        self._native = {}
        self._native_versions = {}

    @property
    def num_classes_with_blank(self):
        return self._num_classes

    def set_compute_mode(self, compute: str):
        if compute not in ("bf16", "fp32"):
            raise ValueError("compute must be 'bf16' or 'fp32'")
        self.compute = compute

    def _apply(self, fn, *args, **kwargs):
        self._native_versions = {}
        return super()._apply(fn, *args, **kwargs)

    def _native_for(self, dev: torch.device):
        from conformer_amd.joint import NativeJoint
        key = (dev.index if dev.index is not None else torch.cuda.current_device(), self.compute)
        nat = self._native.get(key)
        if nat is None:
            nat = NativeJoint(self.encoder_hidden, self.pred_hidden, self.joint_hidden, self._num_classes,
                              self.activation, key[0], self.compute)
            self._native[key] = nat
        out = self.joint_net[-1]
        ts = (self.enc.weight, self.enc.bias, self.pred.weight, self.pred.bias, out.weight, out.bias)
        version = tuple((t.data_ptr(), t._version) for t in ts)
        if self._native_versions.get(key) != version:
            nat.set_weights(*ts)
            self._native_versions[key] = version
        return nat

    def joint(self, f: torch.Tensor, g: torch.Tensor) -> torch.Tensor:
        """f (B, T, H1), g (B, U, H2) -> (B, T, U, V + 1)  (rnnt.py:951-1008)."""
        return self._run(f.transpose(1, 2), g.transpose(1, 2))

    def _run(self, enc_bdt, dec_bdu):
        if not enc_bdt.is_cuda:
            raise RuntimeError("RNNTJoint (MI355X-native) expects its inputs on a ROCm GPU")
        if torch.is_grad_enabled() and (enc_bdt.requires_grad or dec_bdu.requires_grad or
                                        any(p.requires_grad for p in self.parameters())) and self.training:
            raise NotImplementedError("the native RNN-T joint is inference-only (its backward needs the RNNT loss, "
                                      "which is not built); use torch.no_grad() or .eval()")
        nat = self._native_for(enc_bdt.device)
        return nat.forward(enc_bdt, dec_bdu, log_softmax=bool(self.log_softmax))

    @typecheck()
    def forward(self, encoder_outputs: torch.Tensor, decoder_outputs: Optional[torch.Tensor],
                encoder_lengths: Optional[torch.Tensor] = None, transcripts: Optional[torch.Tensor] = None,
                transcript_lengths: Optional[torch.Tensor] = None, compute_wer: bool = False):
        if self._fuse_loss_wer:
            raise NotImplementedError("fuse_loss_wer needs the RNNT loss (SURVEY §8f2), which is not built")
        if decoder_outputs is None:
            raise ValueError("decoder_outputs passed is None, and `fuse_loss_wer` is not set. "
                             "decoder_outputs can only be None for fused step!")
        return self._run(encoder_outputs, decoder_outputs)

    def input_example(self, max_batch=1, max_dim=8192):
        dev = next(self.parameters()).device
        return (torch.randn(max_batch, self.encoder_hidden, max_dim, device=dev),
                torch.randn(max_batch, self.pred_hidden, max_batch, device=dev))
