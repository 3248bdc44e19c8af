"""WER metrics the model shells log (reference nemo/collections/asr/metrics/wer.py:27-275,
rnnt_wer.py:490-590), host-side (they run on decoded token lists, outside the hot path).

* `word_error_rate` (wer.py:27-60): Levenshtein distance over words (or characters with use_cer)
  summed over the batch / reference word count (`editdistance` is absent here: a plain DP).
* `WER` (wer.py:68-275): CTC greedy decoding of argmax predictions (collapse repeats, drop blanks;
  wer.py:149-172), tokens -> text through the vocabulary (char models) or a tokenizer (BPE), then
  update / compute / reset of (scores, words).
* `RNNTWER` (rnnt_wer.py:490-590): the same bookkeeping on hypotheses from the native greedy
  RNN-T decoder (`GreedyBatchedRNNTInfer`).
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence

import torch


def _edit_distance(a: Sequence, b: Sequence) -> int:
    prev = list(range(len(b) + 1))
    for i, x in enumerate(a, 1):
        cur = [i] + [0] * len(b)
        for j, y in enumerate(b, 1):
            cur[j] = min(prev[j] + 1, cur[j - 1] + 1, prev[j - 1] + (x != y))
        prev = cur
    return prev[-1]


def word_error_rate(hypotheses: List[str], references: List[str], use_cer: bool = False) -> float:
    if len(hypotheses) != len(references):
        raise ValueError("In word error rate calculation, hypotheses and reference lists must have the same number "
                         f"of elements. But I got:{len(hypotheses)} and {len(references)} correspondingly")
    scores = words = 0
    for h, r in zip(hypotheses, references):
        hl, rl = (list(h), list(r)) if use_cer else (h.split(), r.split())
        words += len(rl)
        scores += _edit_distance(hl, rl)
    return 1.0 * scores / words if words else float("inf")


def _move_batch_front(t: torch.Tensor, dim: int) -> torch.Tensor:
    dims = list(range(t.ndim))
    return t.permute(*([dim] + dims[:dim] + dims[dim + 1:]))


class _WERBase:
    def __init__(self, decode_tokens: Callable[[List[int]], str], batch_dim_index: int = 0, use_cer: bool = False,
                 log_prediction: bool = True, dist_sync_on_step: bool = False):
        self.decode_tokens_to_str = decode_tokens
        self.batch_dim_index = batch_dim_index
        self.use_cer = use_cer
        self.log_prediction = log_prediction
        self.dist_sync_on_step = dist_sync_on_step
        self.reset()

    def reset(self):
        self.scores = torch.tensor(0)
        self.words = torch.tensor(0)

    def _references(self, targets, target_lengths) -> List[str]:
        tg = _move_batch_front(targets.long().cpu(), self.batch_dim_index)
        tl = target_lengths.long().cpu()
        return [self.decode_tokens_to_str(tg[i][: int(tl[i])].tolist()) for i in range(tg.shape[0])]

    def _accumulate(self, hyps: List[str], refs: List[str]):
        words = scores = 0
        for h, r in zip(hyps, refs):
            hl, rl = (list(h), list(r)) if self.use_cer else (h.split(), r.split())
            words += len(rl)
            scores += _edit_distance(hl, rl)
        self.scores = self.scores + scores
        self.words = self.words + words

    def compute(self):
        scores, words = self.scores.detach().float(), self.words.detach().float()
        return scores / words, scores, words


class WER(_WERBase):
    """CTC greedy WER (wer.py:68-275).  vocabulary: the decoder's label list (blank = len(vocabulary))."""

    def __init__(self, vocabulary=None, tokenizer=None, batch_dim_index=0, use_cer=False, ctc_decode=True,
                 log_prediction=True, dist_sync_on_step=False):
        if tokenizer is not None:
            decode = lambda ids: tokenizer.ids_to_text(ids)   # noqa: E731  (WERBPE, wer_bpe.py)
            self.blank_id = tokenizer.vocab_size
        else:
            labels = list(vocabulary or [])
            decode = lambda ids: "".join(labels[i] for i in ids)   # noqa: E731
            self.blank_id = len(labels)
        self.ctc_decode = ctc_decode
        super().__init__(decode, batch_dim_index, use_cer, log_prediction, dist_sync_on_step)

    def ctc_decoder_predictions_tensor(self, predictions: torch.Tensor,
                                       predictions_len: Optional[torch.Tensor] = None) -> List[str]:
        pred = _move_batch_front(predictions, self.batch_dim_index).long().cpu()
        out = []
        for i in range(pred.shape[0]):
            p = pred[i].tolist()
            if predictions_len is not None:
                p = p[: int(predictions_len[i])]
            dec, prev = [], self.blank_id
            for t in p:                       # collapse repeats, drop blanks (wer.py:160-165)
                if (t != prev or prev == self.blank_id) and t != self.blank_id:
                    dec.append(t)
                prev = t
            out.append(self.decode_tokens_to_str(dec))
        return out

    def update(self, predictions, targets, target_lengths, predictions_lengths=None):
        with torch.no_grad():
            refs = self._references(targets, target_lengths)
            hyps = self.ctc_decoder_predictions_tensor(predictions, predictions_lengths)
            self._accumulate(hyps, refs)


class RNNTWER(_WERBase):
    """rnnt_wer.py:490-590 over the native greedy decoding (`decoding` = GreedyBatchedRNNTInfer)."""

    def __init__(self, decoding, vocabulary=None, tokenizer=None, batch_dim_index=0, use_cer=False,
                 log_prediction=True, dist_sync_on_step=False):
        self.decoding = decoding
        if tokenizer is not None:
            decode = lambda ids: tokenizer.ids_to_text(ids)   # noqa: E731
        else:
            labels = list(vocabulary or [])
            decode = lambda ids: "".join(labels[i] for i in ids)   # noqa: E731
        super().__init__(decode, batch_dim_index, use_cer, log_prediction, dist_sync_on_step)

    def update(self, encoder_output, encoded_lengths, targets, target_lengths):
        with torch.no_grad():
            refs = self._references(targets, target_lengths)
            (hyps,) = self.decoding(encoder_output=encoder_output, encoded_lengths=encoded_lengths)
            texts = [self.decode_tokens_to_str([int(t) for t in h.y_sequence]) for h in hyps]
            self._accumulate(texts, refs)
