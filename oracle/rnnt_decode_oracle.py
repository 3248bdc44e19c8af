"""Oracle (TEST INFRASTRUCTURE ONLY — imported by tests/, never by the product path) for the RNN-T
prediction network and greedy batch decoding (SURVEY §8 a-ext4 / f2, include/cfm_rnnt_decode.h).

float64 numpy restatement of
  torch.nn.LSTM (gate order i, f, g, o)        via LSTMDropout, nemo/collections/common/parts/rnn.py:151-237
  RNNTDecoder.predict                           nemo/collections/asr/modules/rnnt.py:190-283
  RNNTJoint.joint                               rnnt.py:951-1008 (act(enc(f) + pred(g)) -> joint_net)
  GreedyBatchedRNNTInfer._greedy_decode_blank_as_pad
                                                nemo/collections/asr/parts/submodules/rnnt_greedy_decoding.py:453-616
The batched greedy loop is restated per utterance: an utterance's tokens never depend on its batch
neighbours (masked utterances keep their state and last label, rnnt_greedy_decoding.py:557-575), so
at each frame it emits labels until the argmax is blank or max_symbols labels were emitted.  The
first step of an utterance feeds the zero "start of sequence" vector (`_pred_step(self._SOS)`,
:517-518); later steps embed the last label (the blank row while nothing was emitted).
Pinned to the reference modules' own outputs: tests/golden/rnnt_decode_*.npz.
"""
from __future__ import annotations

from typing import Dict, List, Tuple

import numpy as np


def _sig(x):
    return 1.0 / (1.0 + np.exp(-x))


def lstm_step(x, h, c, w_ih, w_hh, b_ih, b_hh):
    """One torch.nn.LSTM cell step on rows: x (B, I), h/c (B, H) -> (h', c')."""
    gates = x @ w_ih.T + b_ih + h @ w_hh.T + b_hh
    H = h.shape[1]
    i, f, g, o = _sig(gates[:, :H]), _sig(gates[:, H:2 * H]), np.tanh(gates[:, 2 * H:3 * H]), _sig(gates[:, 3 * H:])
    c2 = f * c + i * g
    return o * np.tanh(c2), c2


def lstm_params(sd: Dict[str, np.ndarray], L: int, prefix: str = "prediction.dec_rnn.lstm.") -> List[Tuple]:
    return [tuple(np.asarray(sd[f"{prefix}{n}_l{l}"], np.float64) for n in ("weight_ih", "weight_hh", "bias_ih",
                                                                               "bias_hh")) for l in range(L)]


def predict(sd, L: int, y, h0=None, c0=None, add_sos: bool = True):
    """RNNTDecoder.predict(y (B, U) int, state, add_sos) -> g (B, U(+1), H), (h, c) (L, B, H)."""
    emb = np.asarray(sd["prediction.embed.weight"], np.float64)
    B, U = y.shape
    H = emb.shape[1]
    x = emb[y]                                                    # (B, U, H)
    if add_sos:
        x = np.concatenate([np.zeros((B, 1, H)), x], 1)
    ps = lstm_params(sd, L)
    h = np.zeros((L, B, H)) if h0 is None else np.asarray(h0, np.float64).copy()
    c = np.zeros((L, B, H)) if c0 is None else np.asarray(c0, np.float64).copy()
    out = np.zeros((B, x.shape[1], H))
    for t in range(x.shape[1]):
        inp = x[:, t]
        for l, (wi, wh, bi, bh) in enumerate(ps):
            h[l], c[l] = lstm_step(inp, h[l], c[l], wi, wh, bi, bh)
            inp = h[l]
        out[:, t] = inp
    return out, (h, c)


ACT = {"relu": lambda z: np.maximum(z, 0.0), "sigmoid": _sig, "tanh": np.tanh}


def joint_logits(jsd, act: str, f, g):
    """RNNTJoint.joint on single frames / single label states: f (B, D1), g (B, H) -> (B, V + 1)."""
    fe = f @ np.asarray(jsd["enc.weight"], np.float64).T + jsd["enc.bias"]
    ge = g @ np.asarray(jsd["pred.weight"], np.float64).T + jsd["pred.bias"]
    last = max(int(k.split(".")[1]) for k in jsd if k.startswith("joint_net.") and k.endswith(".weight"))
    w, b = np.asarray(jsd[f"joint_net.{last}.weight"], np.float64), jsd[f"joint_net.{last}.bias"]
    return ACT[act](fe + ge) @ w.T + b


def greedy_decode(dsd, jsd, L: int, act: str, enc_bdt, enc_len, blank: int, max_symbols: int,
                  log_normalize: bool = False):
    """Per-utterance greedy RNN-T decoding.  Returns per utterance (tokens, timesteps, score, h, c)
    with h, c (L, H) the final committed state, and `has_state` (False when no utterance emitted:
    the reference then returns dec_state None)."""
    emb = np.asarray(dsd["prediction.embed.weight"], np.float64)
    ps = lstm_params(dsd, L)
    B, _, T = enc_bdt.shape
    H = emb.shape[1]
    res = []
    for b in range(B):
        h = np.zeros((L, 1, H))
        c = np.zeros((L, 1, H))
        last, toks, steps, score = blank, [], [], 0.0
        first = True
        for t in range(int(enc_len[b])):
            f = np.asarray(enc_bdt[b, :, t], np.float64)[None]
            for _ in range(max_symbols):
                inp = np.zeros((1, H)) if first else emb[[last]]
                first = False
                h2, c2 = h.copy(), c.copy()
                for l, (wi, wh, bi, bh) in enumerate(ps):
                    h2[l], c2[l] = lstm_step(inp, h[l], c[l], wi, wh, bi, bh)
                    inp = h2[l]
                z = joint_logits(jsd, act, f, inp)[0]
                if log_normalize:
                    m = z.max()
                    z = z - (m + np.log(np.exp(z - m).sum()))
                k = int(np.argmax(z))
                if k == blank:
                    break
                toks.append(k)
                steps.append(t)
                score += float(z[k])
                last, h, c = k, h2, c2
        res.append((toks, steps, score, h[:, 0], c[:, 0]))
    has_state = any(len(r[0]) > 0 for r in res)
    return res, has_state
