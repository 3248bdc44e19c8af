"""Drop-in `nemo.collections.asr.modules.RNNTDecoder` (reference rnnt.py:50-610, backed by
include/cfm_rnnt_decode.h) and `RNNTJoint` (reference nemo/collections/asr/modules/rnnt.py:613-1038,
backed by the MI355X-native joint, include/cfm_joint.h).

RNNTDecoder: same constructor (prednet dict, vocab_size, normalization_mode, random_state_sampling,
blank_as_pad), the same `prediction.embed` / `prediction.dec_rnn.lstm` parameters (state_dicts load
unchanged; init as rnn.py:151-237: forget-gate bias, chrono init, weights_init_scale), keyword-only
forward(targets, target_length, states) -> (g (B, H, U+1), target_length, states), `predict`, and the
state bookkeeping helpers the decoders use.  The embedding + LSTM recurrence runs in libcfm.so (fp32).
Under autograd (training) `predict` runs the native teacher-forced forward with LSTMDropout's output
dropout and a tape, and the native backpropagation through time (include/cfm_rnnt_decode.h, training
section) fills the embedding / LSTM gradients.  Differences by design: training starts from the zero
state (the reference's training call, rnnt.py:190-283 with state=None); normalization_mode must be None
and blank_as_pad True (the reference's defaults and the transducer configs' values); rnn_hidden_size >
pred_hidden (LSTM projection) is not built.

Same constructor (jointnet dict with encoder_hidden / pred_hidden / joint_hidden / activation /
dropout, num_classes, vocabulary, log_softmax, preserve_memory, fuse_loss_wer, fused_batch_size),
same `pred` / `enc` / `joint_net` parameter names (state_dicts load unchanged), keyword-only
forward(encoder_outputs=(B, H1, T), decoder_outputs=(B, H2, U)) -> (B, T, U, V + 1).

log_softmax semantics follow rnnt.py:998-1006: None -> logits on a GPU (the native path only runs
on a GPU), True -> log-probs, False -> logits.

`fuse_loss_wer=True` (conformer_transducer_bpe.yaml:164) runs the reference's fused step
(rnnt.py:824-949): per `fused_batch_size` sub-batch, the native joint on the sub-batch's own
(T', U') extent, the loss module set by `set_loss` (the native RNN-T loss, losses/rnnt.py) with its
reduction forced to None, optional WER through `set_wer`; returns (mean loss, wer, wer_num,
wer_denom).  Under autograd the joint runs cfm_rnnt_joint_forward_train (joint_net's Dropout in training
mode) and its backward (cfm_rnnt_joint_backward) gives the encoder-output, decoder-output and parameter
gradients, so the fused step trains as the reference's does (rnnt_models.py:673-739).
"""
from __future__ import annotations

import os
from collections import OrderedDict
from typing import Any, Dict, List, Optional

import torch

from nemo.core.classes.common import typecheck
from nemo.core.classes.module import NeuralModule
from nemo.core.neural_types import (AcousticEncodedRepresentation, ElementType, EmbeddedTextType, LabelsType,
                                    LengthsType, LogprobsType, NeuralType)

__all__ = ["RNNTDecoder", "RNNTJoint"]


class _LSTMDropout(torch.nn.Module):
    """Parameter container of rnn.LSTMDropout (nemo/collections/common/parts/rnn.py:151-237): an
    nn.LSTM under `.lstm` (the arithmetic runs natively) with the reference's initialisation."""

    def __init__(self, input_size, hidden_size, num_layers, dropout, forget_gate_bias, t_max=None,
                 weights_init_scale=1.0, hidden_hidden_bias_scale=0.0):
        super().__init__()
        self.lstm = torch.nn.LSTM(input_size=input_size, hidden_size=hidden_size, num_layers=num_layers,
                                  dropout=dropout)
        with torch.no_grad():
            if t_max is not None:                                   # chrono init (rnn.py:194-205)
                for name, p in self.lstm.named_parameters():
                    if "bias" in name:
                        n = p.nelement() // 4
                        p.fill_(0)
                        p[n:2 * n] = torch.log(torch.nn.init.uniform_(p[0:n], 1, t_max - 1))
                        p[0:n] = -p[n:2 * n]
            elif forget_gate_bias is not None:                      # rnn.py:206-213
                for name, p in self.lstm.named_parameters():
                    if "bias_ih" in name:
                        p[hidden_size:2 * hidden_size].fill_(forget_gate_bias)
                    if "bias_hh" in name:
                        p[hidden_size:2 * hidden_size] *= float(hidden_hidden_bias_scale)
            for name, p in self.named_parameters():
                if "weight" in name or "bias" in name:
                    p *= float(weights_init_scale)
        self.dropout = torch.nn.Dropout(dropout) if dropout else None


def _seed() -> int:
    return int(torch.randint(0, 2 ** 62, (1,)).item())


class _PredictTrainFn(torch.autograd.Function):
    """RNNTDecoder.predict under autograd: native teacher-forced forward + BPTT (cfm_rnnt_decode.h)."""

    @staticmethod
    def forward(ctx, nat, y, add_sos, dropout, seed, emb, *lstm):
        g, tape = nat.train_forward(y, add_sos, dropout, seed)
        L = len(lstm) // 4
        ctx.nat, ctx.y, ctx.add_sos, ctx.dropout, ctx.seed, ctx.tape, ctx.L = nat, y, add_sos, dropout, seed, tape, L
        ctx.save_for_backward(*lstm[:2 * L])
        ctx.mark_non_differentiable(tape)
        return g, tape

    @staticmethod
    def backward(ctx, dg, _dtape):
        L = ctx.L
        w = ctx.saved_tensors
        need = ctx.needs_input_grad
        want = (need[5], any(need[6:6 + L]), any(need[6 + L:6 + 2 * L]), any(need[6 + 2 * L:6 + 3 * L]),
                any(need[6 + 3 * L:6 + 4 * L]))
        if dg is None:
            dg = torch.zeros((ctx.y.shape[0], ctx.y.shape[1] + (1 if ctx.add_sos else 0), ctx.nat.H),
                             device=ctx.nat.device)
        demb, dwi, dwh, dbi, dbh = ctx.nat.backward(ctx.y, ctx.add_sos, ctx.dropout, ctx.seed, ctx.tape, dg,
                                                    list(w[:L]), list(w[L:2 * L]), want)
        ctx.tape = None
        per = lambda lst: list(lst) if lst is not None else [None] * L  # noqa: E731
        return (None, None, None, None, None, demb, *per(dwi), *per(dwh), *per(dbi), *per(dbh))


class _JointTrainFn(torch.autograd.Function):
    """RNNTJoint.joint under autograd: cfm_rnnt_joint_forward_train + cfm_rnnt_joint_backward."""

    @staticmethod
    def forward(ctx, nat, dropout, seed, enc_bdt, dec_bdu, w_enc, b_enc, w_pred, b_pred, w_out, b_out):
        out = nat.forward_train(enc_bdt, dec_bdu, dropout, seed)
        ctx.nat, ctx.dropout, ctx.seed = nat, dropout, seed
        ctx.save_for_backward(enc_bdt, dec_bdu, w_enc, w_pred, w_out)
        return out

    @staticmethod
    def backward(ctx, dlogits):
        enc, dec, w_enc, w_pred, w_out = ctx.saved_tensors
        want = tuple(bool(x) for x in ctx.needs_input_grad[3:11])
        outs = ctx.nat.backward(enc, dec, dlogits, ctx.dropout, ctx.seed, w_enc, w_pred, w_out, want)
        return (None, None, None, *outs)


class RNNTDecoder(NeuralModule):
    """Stateful LSTM prediction network (rnnt.py:50-610)."""

    @property
    def input_types(self):
        return {"targets": NeuralType(("B", "T"), LabelsType()),
                "target_length": NeuralType(tuple("B"), LengthsType()),
                "states": [NeuralType(("D", "B", "D"), ElementType(), optional=True)]}

    @property
    def output_types(self):
        return {"outputs": NeuralType(("B", "D", "T"), EmbeddedTextType()),
                "prednet_lengths": NeuralType(tuple("B"), LengthsType()),
                "states": [NeuralType(("D", "B", "D"), ElementType(), optional=True)]}

    def __init__(self, prednet: Dict[str, Any], vocab_size: int, normalization_mode: Optional[str] = None,
                 random_state_sampling: bool = False, blank_as_pad: bool = True):
        super().__init__()
        self.pred_hidden = prednet["pred_hidden"]
        self.pred_rnn_layers = prednet["pred_rnn_layers"]
        self.blank_idx = vocab_size
        self.vocab_size = vocab_size
        self.blank_as_pad = blank_as_pad
        if not blank_as_pad:
            raise NotImplementedError("blank_as_pad=False (masked greedy decoding) is not on the native path")
        if normalization_mode is not None:
            raise NotImplementedError("normalization_mode 'batch' / 'layer' LSTMs are not on the native path")
        rnn_hidden_size = prednet.get("rnn_hidden_size", -1)
        if rnn_hidden_size > 0 and rnn_hidden_size != self.pred_hidden:
            raise NotImplementedError("rnn_hidden_size != pred_hidden (projected LSTM) is not on the native path")
        self.random_state_sampling = random_state_sampling
        dropout = prednet.get("dropout", 0.0)
        self.prediction = torch.nn.ModuleDict({
            "embed": torch.nn.Embedding(vocab_size + 1, self.pred_hidden, padding_idx=self.blank_idx),
            "dec_rnn": _LSTMDropout(self.pred_hidden, self.pred_hidden, self.pred_rnn_layers, dropout,
                                    prednet.get("forget_gate_bias", 1.0), prednet.get("t_max", None),
                                    prednet.get("weights_init_scale", 1.0),
                                    prednet.get("hidden_hidden_bias_scale", 0.0)),
        })
        self._native = {}
        self._native_versions = {}
        self._rnnt_export = False

    def _apply(self, fn, *args, **kwargs):
        self._native_versions = {}
        return super()._apply(fn, *args, **kwargs)

    def _lstm_tensors(self):
        lstm = self.prediction["dec_rnn"].lstm
        L = self.pred_rnn_layers
        return ([getattr(lstm, f"weight_ih_l{l}") for l in range(L)], [getattr(lstm, f"weight_hh_l{l}") for l in range(L)],
                [getattr(lstm, f"bias_ih_l{l}") for l in range(L)], [getattr(lstm, f"bias_hh_l{l}") for l in range(L)])

    def native_for(self, dev: torch.device):
        from conformer_amd.rnnt_decode import NativePredictionNet
        key = dev.index if dev.index is not None else torch.cuda.current_device()
        nat = self._native.get(key)
        if nat is None:
            nat = NativePredictionNet(self.vocab_size, self.pred_hidden, self.pred_rnn_layers, key)
            self._native[key] = nat
        emb = self.prediction["embed"].weight
        lists = self._lstm_tensors()
        ts = [emb] + [t for ts in lists for t in ts]
        version = tuple((t.data_ptr(), t._version) for t in ts)
        if self._native_versions.get(key) != version:
            nat.set_weights(emb, *lists)
            self._native_versions[key] = version
        return nat

    @typecheck()
    def forward(self, targets, target_length, states=None):
        y = targets.type(torch.int64)                               # rnn.label_collate
        g, states = self.predict(y, state=states, add_sos=not self._rnnt_export)
        return g.transpose(1, 2), target_length, states

    def predict(self, y: Optional[torch.Tensor] = None, state: Optional[List[torch.Tensor]] = None,
                add_sos: bool = True, batch_size: Optional[int] = None):
        """rnnt.py:190-283: (g (B, U(+1), H), [h, c] each (L, B, H))."""
        _p = next(self.parameters())
        if _p.device.type != "cuda":
            raise RuntimeError("RNNTDecoder (MI355X-native) needs its parameters on a ROCm GPU")
        train = torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters())
        if y is not None:
            y = y.to(_p.device)
            if y.numel() and (int(y.min()) < 0 or int(y.max()) > self.blank_idx):
                raise IndexError("index out of range in self")       # nn.Embedding's error
            B = y.shape[0]
        else:
            B = (1 if state is None else state[0].size(1)) if batch_size is None else batch_size
        if state is None and self.random_state_sampling and self.training:
            state = self.initialize_state(torch.empty(B, 1, device=_p.device))
        h0, c0 = (None, None) if state is None else (state[0], state[1])
        if train and y is not None and state is None:
            return self._predict_train(y, add_sos)
        if train:
            raise NotImplementedError("the native prediction-net backward starts from the zero state with labels "
                                      "(the training call); use torch.no_grad() for stateful decoding")
        g, (h, c) = self.native_for(_p.device).predict(y, h0, c0, add_sos, B)
        return g, [h, c]

    def _predict_train(self, y: torch.Tensor, add_sos: bool):
        nat = self.native_for(y.device)
        drop = self.prediction["dec_rnn"].dropout
        p = float(drop.p) if (drop is not None and self.training) else 0.0
        lists = self._lstm_tensors()
        g, tape = _PredictTrainFn.apply(nat, y, bool(add_sos), p, _seed() if p > 0 else 0, self.prediction["embed"].weight,
                                        *[t for ts in lists for t in ts])
        # final states (detached): the top of every layer's last step on the tape
        B, S, H, L = y.shape[0], g.shape[1], self.pred_hidden, self.pred_rnn_layers
        # (cfm_rnnt_decode.h: per layer and step one block [gates (B, 4H) | c (B, H) | h (B, H)])
        tf = tape[: L * S * B * 6 * H * 4].view(torch.float32).view(L, S, 6 * B, H)
        h = tf[:, S - 1, 5 * B:6 * B].clone()
        c = tf[:, S - 1, 4 * B:5 * B].clone()
        return g, [h, c]

    def initialize_state(self, y: torch.Tensor) -> List[torch.Tensor]:
        batch = y.size(0)
        shape = (self.pred_rnn_layers, batch, self.pred_hidden)
        if self.random_state_sampling and self.training:
            return [torch.randn(shape, dtype=y.dtype, device=y.device), torch.randn(shape, dtype=y.dtype, device=y.device)]
        return [torch.zeros(shape, dtype=y.dtype, device=y.device), torch.zeros(shape, dtype=y.dtype, device=y.device)]

    def batch_select_state(self, batch_states: List[torch.Tensor], idx: int) -> List[List[torch.Tensor]]:
        """rnnt.py:514-531."""
        if batch_states is None:
            return None
        return [[batch_states[s][layer][idx] for layer in range(self.pred_rnn_layers)] for s in range(len(batch_states))]

    def batch_copy_states(self, old_states: List[torch.Tensor], new_states: List[torch.Tensor], ids: List[int],
                          value: Optional[float] = None) -> List[torch.Tensor]:
        """rnnt.py:579-610."""
        for s in range(len(old_states)):
            if value is None:
                old_states[s][:, ids, :] = new_states[s][:, ids, :]
            else:
                old_states[s][:, ids, :] *= 0.0
                old_states[s][:, ids, :] += value
        return old_states

    def batch_concat_states(self, batch_states: List[List[torch.Tensor]]) -> List[torch.Tensor]:
        """rnnt.py:533-555: B x ([L x (H)], [L x (H)]) -> [(L, B, H), (L, B, H)]."""
        return [torch.stack([torch.stack(b[s]) for b in batch_states], 0).transpose(1, 0)
                for s in range(len(batch_states[0]))]

    def batch_initialize_states(self, batch_states: List[torch.Tensor], decoder_states: List[List[torch.Tensor]]):
        """rnnt.py:485-512."""
        return [torch.stack([torch.stack([d[s][layer] for d in decoder_states]) for layer in range(self.pred_rnn_layers)])
                for s in range(len(decoder_states[0]))]



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
        self._loss = None
        self._wer = None

    # --- fused-step plumbing (rnnt_abstract.py: AbstractRNNTJoint) ----------------------------
    @property
    def loss(self):
        return self._loss

    def set_loss(self, loss):
        if not self._fuse_loss_wer:
            raise ValueError("Attempting to set loss module even though `fuse_loss_wer` is not set!")
        self._loss = loss

    @property
    def wer(self):
        return self._wer

    def set_wer(self, wer):
        if not self._fuse_loss_wer:
            raise ValueError("Attempting to set WER module even though `fuse_loss_wer` is not set!")
        self._wer = wer

    @property
    def fuse_loss_wer(self):
        return self._fuse_loss_wer

    def set_fuse_loss_wer(self, fuse_loss_wer, loss=None, metric=None):
        self._fuse_loss_wer = fuse_loss_wer
        self._loss = loss
        self._wer = metric

    @property
    def fused_batch_size(self):
        return self._fused_batch_size

    def set_fused_batch_size(self, fused_batch_size):
        self._fused_batch_size = fused_batch_size

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
        nat = self._native_for(enc_bdt.device)
        if torch.is_grad_enabled() and (enc_bdt.requires_grad or dec_bdu.requires_grad or
                                        any(p.requires_grad for p in self.parameters())):
            if self.log_softmax:
                raise NotImplementedError("the native joint backward takes raw logits (log_softmax None / False, the "
                                          "GPU training configuration)")
            drop = [m for m in self.joint_net if isinstance(m, torch.nn.Dropout)]
            p = float(drop[0].p) if (drop and self.training) else 0.0
            out = self.joint_net[-1]
            return _JointTrainFn.apply(nat, p, _seed() if p > 0 else 0, enc_bdt, dec_bdu, self.enc.weight, self.enc.bias,
                                       self.pred.weight, self.pred.bias, out.weight, out.bias)
        return nat.forward(enc_bdt, dec_bdu, log_softmax=bool(self.log_softmax))

    @typecheck()
    def forward(self, encoder_outputs: torch.Tensor, decoder_outputs: Optional[torch.Tensor],
                encoder_lengths: Optional[torch.Tensor] = None, transcripts: Optional[torch.Tensor] = None,
                transcript_lengths: Optional[torch.Tensor] = None, compute_wer: bool = False):
        if not self._fuse_loss_wer:
            if decoder_outputs is None:
                raise ValueError("decoder_outputs passed is None, and `fuse_loss_wer` is not set. "
                                 "decoder_outputs can only be None for fused step!")
            return self._run(encoder_outputs, decoder_outputs)
        return self._fused_step(encoder_outputs, decoder_outputs, encoder_lengths, transcripts, transcript_lengths,
                                compute_wer)

    def _fused_step(self, enc_bdt, dec_bdu, encoder_lengths, transcripts, transcript_lengths, compute_wer):
        """rnnt.py:812-949: sub-batches of fused_batch_size, each narrowed to its own max T' / U'."""
        if self._loss is None or self._wer is None:
            raise ValueError("`fuse_loss_wer` flag is set, but `loss` and `wer` modules were not provided! ")
        if self._fused_batch_size is None:
            raise ValueError("If `fuse_loss_wer` is set, then `fused_batch_size` cannot be None!")
        if encoder_lengths is None or transcript_lengths is None:
            raise ValueError("`fuse_loss_wer` is set, therefore encoder and target lengths must be provided as well!")
        losses, wer_num_l, wer_den_l = [], [], []
        wer = None
        B = int(enc_bdt.size(0))
        for b0 in range(0, B, self._fused_batch_size):
            n = min(b0 + self._fused_batch_size, B) - b0
            sub_enc = enc_bdt.narrow(0, b0, n)                     # (b, D, T)
            sub_tr = transcripts.narrow(0, b0, n)
            sub_el = encoder_lengths[b0:b0 + n]
            sub_tl = transcript_lengths[b0:b0 + n]
            t_max, u_max = int(sub_el.max()), int(sub_tl.max())
            if dec_bdu is not None:
                if sub_enc.shape[2] != t_max:
                    sub_enc = sub_enc.narrow(2, 0, t_max)
                sub_dec = dec_bdu.narrow(0, b0, n)
                if sub_dec.shape[2] != u_max + 1:
                    sub_dec = sub_dec.narrow(2, 0, u_max + 1)
                sub_joint = self._run(sub_enc, sub_dec)             # (b, T', U'+1, V+1)
                if sub_tr.shape[1] != u_max:
                    sub_tr = sub_tr.narrow(1, 0, u_max)
                red = self._loss.reduction
                self._loss.reduction = None
                try:
                    losses.append(self._loss(log_probs=sub_joint, targets=sub_tr.contiguous(), input_lengths=sub_el,
                                             target_lengths=sub_tl))
                finally:
                    self._loss.reduction = red
                del sub_joint
            else:
                losses = None
            if compute_wer:
                orig = getattr(self._wer, "log_prediction", False)
                self._wer.log_prediction = bool(orig and b0 == 0)
                self._wer.update(sub_enc.detach(), sub_el, sub_tr.detach(), sub_tl)
                wer, wn, wd = self._wer.compute()
                self._wer.reset()
                wer_num_l.append(wn)
                wer_den_l.append(wd)
                self._wer.log_prediction = orig
        loss = torch.cat(losses, 0).mean() if losses is not None else None
        if compute_wer:
            wer_num = torch.tensor([float(x) for x in wer_num_l]).sum().long()
            wer_denom = torch.tensor([float(x) for x in wer_den_l]).sum().long()
        else:
            wer_num = wer_denom = None
        return loss, wer, wer_num, wer_denom

    def input_example(self, max_batch=1, max_dim=8192):
        dev = next(self.parameters()).device
        return (torch.randn(max_batch, self.encoder_hidden, max_dim, device=dev),
                torch.randn(max_batch, self.pred_hidden, max_batch, device=dev))
