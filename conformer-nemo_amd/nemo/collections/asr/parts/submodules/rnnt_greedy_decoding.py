"""Drop-in greedy RNN-T decoders (reference
nemo/collections/asr/parts/submodules/rnnt_greedy_decoding.py:43-616), SURVEY §8 row f2.

`GreedyBatchedRNNTInfer` and `GreedyRNNTInfer` keep the reference constructors
(decoder_model, joint_model, blank_index, max_symbols_per_step, preserve_alignments) and
`forward(encoder_output (B, D, T), encoded_lengths (B,))` -> `(hypotheses,)` with the same
`Hypothesis` fields (y_sequence as a LongTensor, timestep, score, dec_state, length).  The whole
decode loop runs on the device (include/cfm_rnnt_decode.h): each utterance advances independently,
which reproduces the reference's lock-step batch loop exactly because masked utterances keep their
state and last label (:557-575).  Scores follow the reference's GPU behaviour: raw logits, or
log-probabilities when the joint's `log_softmax` is True.

Differences by design: `preserve_alignments=True` and `partial_hypotheses` raise
NotImplementedError; `max_symbols_per_step=None` (unbounded in the reference, which can then loop
forever) is capped at 100 labels per frame; inputs must live on a ROCm GPU.
"""
from __future__ import annotations

from typing import List, Optional

import torch

from nemo.collections.asr.parts.utils import rnnt_utils
from nemo.core.classes.common import Typing, typecheck
from nemo.core.neural_types import AcousticEncodedRepresentation, HypothesisType, LengthsType, NeuralType

UNBOUNDED_SYMBOLS_CAP = 100


def pack_hypotheses(hypotheses: List[rnnt_utils.Hypothesis], logitlen: torch.Tensor) -> List[rnnt_utils.Hypothesis]:
    """:43-57."""
    logitlen_cpu = logitlen.to("cpu") if hasattr(logitlen, "cpu") else logitlen
    for idx, hyp in enumerate(hypotheses):
        hyp.y_sequence = torch.tensor(hyp.y_sequence, dtype=torch.long)
        hyp.length = logitlen_cpu[idx]
        if hyp.dec_state is not None:
            hyp.dec_state = _states_to_device(hyp.dec_state)
    return hypotheses


def _states_to_device(dec_state, device="cpu"):
    if torch.is_tensor(dec_state):
        return dec_state.to(device)
    if isinstance(dec_state, (list, tuple)):
        return tuple(_states_to_device(d, device) for d in dec_state)
    return dec_state


class _GreedyRNNTInfer(Typing):
    """:70-188."""

    per_utterance = False

    @property
    def input_types(self):
        return {"encoder_output": NeuralType(("B", "D", "T"), AcousticEncodedRepresentation()),
                "encoded_lengths": NeuralType(tuple("B"), LengthsType()),
                "partial_hypotheses": [NeuralType(elements_type=HypothesisType(), optional=True)]}

    @property
    def output_types(self):
        return {"predictions": [NeuralType(elements_type=HypothesisType())]}

    def __init__(self, decoder_model, joint_model, blank_index: int, max_symbols_per_step: Optional[int] = None,
                 preserve_alignments: bool = False):
        super().__init__()
        self.decoder = decoder_model
        self.joint = joint_model
        self._blank_index = blank_index
        self._SOS = blank_index
        self.max_symbols = max_symbols_per_step
        self.preserve_alignments = preserve_alignments
        if blank_index != decoder_model.blank_idx:
            raise NotImplementedError("the native decoder needs blank_index == decoder.blank_idx (vocab_size)")

    def __call__(self, *args, **kwargs):
        return self.forward(*args, **kwargs)

    @typecheck()
    def forward(self, encoder_output: torch.Tensor, encoded_lengths: torch.Tensor,
                partial_hypotheses: Optional[List[rnnt_utils.Hypothesis]] = None):
        if partial_hypotheses is not None:
            raise NotImplementedError("`partial_hypotheses` support is not supported")
        if self.preserve_alignments:
            raise NotImplementedError("preserve_alignments is not on the native path")
        if not encoder_output.is_cuda:
            raise RuntimeError("greedy RNN-T decoding (MI355X-native) expects its inputs on a ROCm GPU")
        with torch.no_grad():
            dec, joint = self.decoder, self.joint
            out = joint.joint_net[-1]
            params = (joint.enc.weight, joint.enc.bias, joint.pred.weight, joint.pred.bias, out.weight, out.bias)
            ms = UNBOUNDED_SYMBOLS_CAP if self.max_symbols is None else int(self.max_symbols)
            nat = dec.native_for(encoder_output.device)
            tokens, tsteps, ntok, scores, h, c = nat.greedy(
                encoder_output, encoded_lengths, params, joint.activation, ms, bool(joint.log_softmax),
                sos_until_label=self.per_utterance)
            ntok_c = ntok.cpu().tolist()
            n = max(ntok_c) if ntok_c else 0
            tok_c = tokens[:, :n].cpu().tolist()
            ts_c = tsteps[:, :n].cpu().tolist()
            sc_c = scores.cpu().tolist()
            any_state = any(k > 0 for k in ntok_c)
            hyps = []
            for b, k in enumerate(ntok_c):
                hyp = rnnt_utils.Hypothesis(score=sc_c[b], y_sequence=tok_c[b][:k], timestep=ts_c[b][:k], dec_state=None)
                # batched: the batch state exists once any utterance emitted (:586-595, :613-614);
                # per utterance: once this utterance emitted (:333, :355)
                if (k > 0) if self.per_utterance else any_state:
                    hyp.dec_state = dec.batch_select_state([h, c], b)
                hyps.append(hyp)
            packed = pack_hypotheses(hyps, encoded_lengths)
        return (packed,)


class GreedyRNNTInfer(_GreedyRNNTInfer):
    """Per-utterance greedy decoding (:191-362)."""

    per_utterance = True


class GreedyBatchedRNNTInfer(_GreedyRNNTInfer):
    """Batch greedy decoding, blank-as-pad variant (:365-616)."""

    per_utterance = False
