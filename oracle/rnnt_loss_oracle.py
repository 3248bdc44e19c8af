"""CPU oracle (TEST INFRASTRUCTURE ONLY) for the RNN-T loss, SURVEY §8 row f2.

float64 numpy restatement of the reference's GPU RNN-T loss (warp-transducer semantics, numba):
  * log-softmax denominators per (b, t, u)        gpu_rnnt.py:90-120 (reduce.py reduce_max / reduce_exp)
  * alphas / betas lattices, log-likelihoods       gpu_rnnt_kernel.py:66-260 (rnnt_helper.log_sum_exp)
  * gradients w.r.t. the raw logits, FastEmit and clamp    gpu_rnnt_kernel.py:262-399
  * costs = -ll_forward * (1 + fastemit_lambda)   rnnt_helper.py:106-115
Only tests/ (and bench.py's cpu_baseline leg) may import this module.  Pinned by
tests/golden/rnnt_loss_*.npz, produced by the reference's own numpy implementation (rnnt_numpy.py).
"""
from __future__ import annotations

import numpy as np


def _lse(a, b):
    if a == -np.inf:
        return b
    if b == -np.inf:
        return a
    return np.log1p(np.exp(-abs(a - b))) + max(a, b)


def rnnt_loss(acts, labels, act_lens, label_lens, blank, fastemit_lambda=0.0, clamp=-1.0, want_grads=True):
    acts = np.asarray(acts, dtype=np.float64)
    B, T, U, V = acts.shape
    m = acts.max(-1, keepdims=True)
    denom = -(m[..., 0] + np.log(np.exp(acts - m).sum(-1)))           # (B, T, U)
    costs = np.zeros(B)
    grads = np.zeros_like(acts) if want_grads else None
    for b in range(B):
        Tb, Ub = int(act_lens[b]), int(label_lens[b]) + 1
        lab = labels[b]
        lp = lambda t, u, v: denom[b, t, u] + acts[b, t, u, v]         # noqa: E731
        al = np.full((T, U), -np.inf)
        al[0, 0] = 0.0
        for t in range(1, Tb):
            al[t, 0] = al[t - 1, 0] + lp(t - 1, 0, blank)
        for u in range(1, Ub):
            al[0, u] = al[0, u - 1] + lp(0, u - 1, lab[u - 1])
        for t in range(1, Tb):
            for u in range(1, Ub):
                al[t, u] = _lse(al[t, u - 1] + lp(t, u - 1, lab[u - 1]), al[t - 1, u] + lp(t - 1, u, blank))
        ll = al[Tb - 1, Ub - 1] + lp(Tb - 1, Ub - 1, blank)
        costs[b] = -ll * (1.0 + fastemit_lambda)
        if not want_grads:
            continue
        be = np.full((T, U), -np.inf)
        be[Tb - 1, Ub - 1] = lp(Tb - 1, Ub - 1, blank)
        for t in range(Tb - 2, -1, -1):
            be[t, Ub - 1] = be[t + 1, Ub - 1] + lp(t, Ub - 1, blank)
        for u in range(Ub - 2, -1, -1):
            be[Tb - 1, u] = be[Tb - 1, u + 1] + lp(Tb - 1, u, lab[u])
        for t in range(Tb - 2, -1, -1):
            for u in range(Ub - 2, -1, -1):
                be[t, u] = _lse(be[t, u + 1] + lp(t, u, lab[u]), be[t + 1, u] + lp(t, u, blank))
        for t in range(Tb):
            for u in range(Ub):
                logpk = denom[b, t, u] + acts[b, t, u]                 # (V,)
                g = np.exp(al[t, u] + be[t, u] + logpk - ll)
                if fastemit_lambda > 0.0 and u < Ub - 1:
                    g = g + fastemit_lambda * np.exp(al[t, u] + lp(t, u, lab[u]) + be[t, u + 1] + logpk - ll)
                if t == Tb - 1 and u == Ub - 1:
                    g[blank] -= np.exp(al[t, u] + logpk[blank] - ll)
                if t < Tb - 1:
                    g[blank] -= np.exp(al[t, u] + logpk[blank] - ll + be[t + 1, u])
                if u < Ub - 1:
                    g[lab[u]] -= np.exp(np.log1p(fastemit_lambda) + al[t, u] + logpk[lab[u]] - ll + be[t, u + 1])
                if clamp > 0.0:
                    g = np.clip(g, -clamp, clamp)
                grads[b, t, u] = g
    return costs, grads
