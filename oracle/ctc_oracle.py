"""CPU restatement (numpy, float64) of the CTC head and CTC loss — TEST INFRASTRUCTURE ONLY.

Imported by tests/ (and nothing on the product path).  Pinned by tests/golden/ctc_*.npz, which
tests/golden/gen_ctc_goldens.py produced by running the reference's own CTCLoss class
(nemo/collections/asr/losses/ctc.py) and the ConvASRDecoder forward expression with torch autograd.

Reference behaviour restated here:
  * ConvASRDecoder.forward, conv_asr.py:442-444:
        log_softmax(Conv1d(feat_in, C, kernel_size=1, bias=True)(encoder_output).transpose(1, 2), -1)
  * EncDecCTCModel greedy predictions, ctc_models.py:594: argmax over classes.
  * CTCLoss.forward, ctc.py:56-70: torch.nn.functional.ctc_loss on log_probs (T, B, C) with
    blank = num_classes (the last class, ctc.py:45), reduction 'none' then mean over the batch
    ('mean_batch', ctc.py:47-49); EncDecCTCModel passes zero_infinity=True (ctc_models.py:190-194).
    The loss is third-party arithmetic (PyTorch's ctc_loss, torch==1.13.0 pinned in
    requirements/requirements.txt:1): alpha-beta recursion over the extended label sequence
    (blank, l1, blank, ..., lU, blank) in log space; the gradient torch returns for log_probs is
    exp(lp[t][c]) - exp(log sum_{s: l'_s = c} alpha_t(s) beta_t(s) + nll - lp[t][c]), zero beyond
    the input length and for zero_infinity'd (infinite) losses.
"""
import numpy as np

NEG = -np.inf


def log_softmax(x, axis=-1):
    m = x.max(axis=axis, keepdims=True)
    return x - (m + np.log(np.exp(x - m).sum(axis=axis, keepdims=True)))


def head_forward(enc_bdt, w, b):
    """conv_asr.py:444 -> (log_probs (B, T, C), greedy (B, T))."""
    logits = np.einsum("bdt,cd->btc", enc_bdt.astype(np.float64), w.reshape(w.shape[0], -1).astype(np.float64))
    logits = logits + b.astype(np.float64)
    lp = log_softmax(logits)
    return lp, lp.argmax(-1)


def head_backward(enc_bdt, w, lp, dlp):
    """Backward of log_softmax(Conv1d_k1(enc)): (d enc (B, D, T), d W (C, D), d b (C))."""
    dlogits = dlp - np.exp(lp) * dlp.sum(-1, keepdims=True)            # (B, T, C)
    w2 = w.reshape(w.shape[0], -1).astype(np.float64)
    denc = np.einsum("btc,cd->bdt", dlogits, w2)
    dw = np.einsum("btc,bdt->cd", dlogits, enc_bdt.astype(np.float64))
    db = dlogits.sum((0, 1))
    return denc, dw, db


def _lse(*xs):
    m = max(xs)
    if m == NEG:
        return NEG
    return m + np.log(sum(np.exp(x - m) for x in xs))


def ctc_loss(lp_btc, targets, in_len, tgt_len, blank, zero_infinity=True):
    """Per-utterance nll (B,) and d nll_b / d log_probs (B, T, C) in torch's convention."""
    lp_btc = np.asarray(lp_btc, dtype=np.float64)
    B, T, C = lp_btc.shape
    nll = np.zeros(B)
    grad = np.zeros_like(lp_btc)
    for b in range(B):
        Tb, Ub = int(in_len[b]), int(tgt_len[b])
        lab = [int(v) for v in targets[b][:Ub]]
        ext = [blank]
        for c in lab:
            ext += [c, blank]
        S = len(ext)
        lp = lp_btc[b]
        alpha = np.full((Tb, S), NEG)
        alpha[0, 0] = lp[0, ext[0]]
        if S > 1:
            alpha[0, 1] = lp[0, ext[1]]
        for t in range(1, Tb):
            for s in range(S):
                a = alpha[t - 1, s]
                a1 = alpha[t - 1, s - 1] if s >= 1 else NEG
                a2 = alpha[t - 1, s - 2] if (s >= 2 and ext[s] != blank and ext[s] != ext[s - 2]) else NEG
                alpha[t, s] = lp[t, ext[s]] + _lse(a, a1, a2)
        ll = _lse(alpha[Tb - 1, S - 1], alpha[Tb - 1, S - 2] if S > 1 else NEG)
        if ll == NEG:
            nll[b] = 0.0 if zero_infinity else np.inf
            continue                                                   # gradient stays 0
        nll[b] = -ll
        beta = np.full((Tb, S), NEG)
        beta[Tb - 1, S - 1] = lp[Tb - 1, ext[S - 1]]
        if S > 1:
            beta[Tb - 1, S - 2] = lp[Tb - 1, ext[S - 2]]
        for t in range(Tb - 2, -1, -1):
            for s in range(S):
                b0 = beta[t + 1, s]
                b1 = beta[t + 1, s + 1] if s + 1 < S else NEG
                b2 = beta[t + 1, s + 2] if (s + 2 < S and ext[s] != blank and ext[s] != ext[s + 2]) else NEG
                beta[t, s] = lp[t, ext[s]] + _lse(b0, b1, b2)
        for t in range(Tb):
            lcab = {}
            for s in range(S):
                lcab[ext[s]] = _lse(lcab.get(ext[s], NEG), alpha[t, s] + beta[t, s])
            grad[b, t] = np.exp(lp[t])
            for c, v in lcab.items():
                grad[b, t, c] = np.exp(lp[t, c]) - np.exp(v + nll[b] - lp[t, c])
    return nll, grad
