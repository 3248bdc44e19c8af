"""CPU restatement (numpy) of the cache-aware streaming encoder's DEFINITION.

TEST INFRASTRUCTURE ONLY (imported by tests/ and nothing in the product path).

PARITY UNPINNED: the reference (NeMo 1.8.2) has no cache-aware streaming encoder; it streams by
re-encoding overlapping buffers (streaming_utils.py:455-683).  include/cfm_cache_stream.h defines
what the chunked encoder computes, and this file states it as one full-sequence forward: the
reference ConformerEncoder (oracle/conformer_oracle.py, pinned to the reference's own outputs) with
  (1) both subsampling convolutions padding time by (2, 0) instead of (1, 1) (frequency (1, 1)),
  (2) attention context [left_context, 0] (make_masks' triu / tril, conformer_encoder.py:296-299),
  (3) the depthwise convolution padding time by (kernel_size - 1, 0) (conformer_modules.py:144-151
      pads (k-1)/2 on both sides).
Under (1)-(3) frame t depends on frames <= t only, so a chunked computation with carried state can
reproduce it exactly: `chunked_forward` below is that computation in numpy (state = the last input
frames / conv1 frames / keys+values / GLU outputs), and tests/test_cache_stream_oracle.py checks the
two against each other on the CPU before the GPU kernels are compared with either.
"""
from __future__ import annotations

import math
from typing import Dict, Optional

import numpy as np

from conformer_oracle import (feed_forward, layer_norm, linear, make_masks, rel_pe_table, rel_pos_mha, swish)


def conv2d_causal_t(x: np.ndarray, w: np.ndarray, b: np.ndarray, stride: int = 2) -> np.ndarray:
    """Conv2d on (B, Cin, T, F) with time padding (2, 0) and frequency padding (1, 1)."""
    B, Cin, T, F = x.shape
    Cout, _, KT, KF = w.shape
    xp = np.zeros((B, Cin, T + KT - 1, F + 2), dtype=x.dtype)
    xp[:, :, KT - 1:, 1:F + 1] = x
    To = (T + KT - 1 - KT) // stride + 1
    Fo = (F + 2 - KF) // stride + 1
    wm = w.reshape(Cout, Cin * KT * KF)
    out = np.empty((B, Cout, To, Fo), dtype=x.dtype)
    for bi in range(B):
        cols = np.empty((Cin, KT, KF, To, Fo), dtype=x.dtype)
        for kt in range(KT):
            for kf in range(KF):
                cols[:, kt, kf] = xp[bi, :, kt:kt + stride * To:stride, kf:kf + stride * Fo:stride]
        out[bi] = (wm @ cols.reshape(-1, To * Fo)).reshape(Cout, To, Fo)
    return out + b.reshape(1, Cout, 1, 1)


def causal_subsampling(x_btf: np.ndarray, sd, prefix: str = "pre_encode.") -> np.ndarray:
    h = x_btf[:, None]
    for i in (0, 2):
        h = np.maximum(conv2d_causal_t(h, sd[f"{prefix}conv.{i}.weight"], sd[f"{prefix}conv.{i}.bias"]), 0)
    b, c, t, f = h.shape
    h = h.transpose(0, 2, 1, 3).reshape(b, t, c * f)
    return h @ sd[f"{prefix}out.weight"].T + sd[f"{prefix}out.bias"]


def causal_conv_module(x: np.ndarray, sd, p: str, norm_type: str = "batch_norm",
                       cache: Optional[np.ndarray] = None) -> np.ndarray:
    """ConformerConvolution with the depthwise conv padded (K-1, 0); `cache` (B, K-1, D) replaces
    the left zero padding (the previous chunk's GLU outputs)."""
    B, T, D = x.shape
    h = linear(x, sd[p + "pointwise_conv1.weight"][:, :, 0], sd[p + "pointwise_conv1.bias"])
    h = h[..., :D] * (1 / (1 + np.exp(-h[..., D:])))
    w = sd[p + "depthwise_conv.weight"][:, 0, :]
    K = w.shape[1]
    left = np.zeros((B, K - 1, D), dtype=h.dtype) if cache is None else cache
    hp = np.concatenate([left, h], axis=1)
    out = np.zeros((B, T, D), dtype=h.dtype)
    for kk in range(K):
        out += hp[:, kk:kk + T, :] * w[:, kk]
    out += sd[p + "depthwise_conv.bias"]
    if norm_type == "batch_norm":
        rm, rv = sd[p + "batch_norm.running_mean"], sd[p + "batch_norm.running_var"]
        out = (out - rm) / np.sqrt(rv + out.dtype.type(1e-5)) * sd[p + "batch_norm.weight"] + sd[p + "batch_norm.bias"]
    else:
        out = layer_norm(out, sd[p + "batch_norm.weight"], sd[p + "batch_norm.bias"])
    out = swish(out)
    y = linear(out, sd[p + "pointwise_conv2.weight"][:, :, 0], sd[p + "pointwise_conv2.bias"])
    return y, hp[:, -(K - 1):] if K > 1 else hp[:, :0]


def _prep(sd, dtype):
    return {k: (v.astype(dtype) if np.issubdtype(np.asarray(v).dtype, np.floating) else v) for k, v in sd.items()}


def causal_forward(x_bft: np.ndarray, sd: Dict[str, np.ndarray], cfg: dict, left_context: int,
                   dtype=np.float32) -> np.ndarray:
    """Full-sequence forward of the causal encoder: (B, F, T) -> (B, d_out, T/4); T % 4 == 0."""
    sd = _prep(sd, dtype)
    x = np.asarray(x_bft, dtype=dtype).transpose(0, 2, 1)
    B, T, _ = x.shape
    assert T % 4 == 0
    d = cfg["d_model"]
    x = causal_subsampling(x, sd)
    if cfg.get("xscaling", True):
        x = x * x.dtype.type(math.sqrt(d))
    Tp = x.shape[1]
    pe, center = rel_pe_table(max(int(cfg.get("pos_emb_max_len", 5000)), T), d, dtype)
    pos_emb = pe[:, center - Tp: center + Tp - 1]
    _, att_mask = make_masks(Tp, np.full((B,), Tp), (left_context, 0))
    norm = cfg.get("conv_norm_type", "batch_norm")
    half = x.dtype.type(0.5)
    for i in range(cfg["n_layers"]):
        p = f"layers.{i}."
        x = x + half * feed_forward(layer_norm(x, sd[p + "norm_feed_forward1.weight"], sd[p + "norm_feed_forward1.bias"]),
                                    sd, p + "feed_forward1.")
        x = x + rel_pos_mha(layer_norm(x, sd[p + "norm_self_att.weight"], sd[p + "norm_self_att.bias"]), att_mask,
                            pos_emb, sd, p + "self_attn.", cfg["n_heads"])
        x = x + causal_conv_module(layer_norm(x, sd[p + "norm_conv.weight"], sd[p + "norm_conv.bias"]), sd, p + "conv.",
                                   norm)[0]
        x = x + half * feed_forward(layer_norm(x, sd[p + "norm_feed_forward2.weight"], sd[p + "norm_feed_forward2.bias"]),
                                    sd, p + "feed_forward2.")
        x = layer_norm(x, sd[p + "norm_out.weight"], sd[p + "norm_out.bias"])
    if "out_proj.weight" in sd:
        x = linear(x, sd["out_proj.weight"], sd["out_proj.bias"])
    return x.transpose(0, 2, 1)


def _chunk_mha(xq, k_all, v_all, t0, c, left, sd, p, H, pe_row):
    """Attention of chunk frames t0 .. t0+c-1 over keys/values of frames t0-len(k_all)+c .. t0+c-1."""
    B, _, D = xq.shape
    dk = D // H
    q = linear(xq, sd[p + "linear_q.weight"], sd[p + "linear_q.bias"]).reshape(B, c, H, dk)
    nk = k_all.shape[1]
    first = t0 + c - nk                       # global frame of k_all[:, 0]
    out = np.zeros((B, c, H, dk), dtype=xq.dtype)
    for i in range(c):
        t = t0 + i
        js = np.arange(max(0, t - left), t + 1)
        kk = k_all[:, js - first].reshape(B, len(js), H, dk)
        vv = v_all[:, js - first].reshape(B, len(js), H, dk)
        pp = linear(pe_row(t - js), sd[p + "linear_pos.weight"]).reshape(len(js), H, dk)
        qu = q[:, i] + sd[p + "pos_bias_u"]
        qv = q[:, i] + sd[p + "pos_bias_v"]
        s = (np.einsum("bhk,bjhk->bhj", qu, kk) + np.einsum("bhk,jhk->bhj", qv, pp)) / xq.dtype.type(math.sqrt(dk))
        e = np.exp(s - s.max(-1, keepdims=True))
        a = e / e.sum(-1, keepdims=True)
        out[:, i] = np.einsum("bhj,bjhk->bhk", a, vv)
    return linear(out.reshape(B, c, D), sd[p + "linear_out.weight"], sd[p + "linear_out.bias"])


def chunked_forward(x_bft: np.ndarray, sd: Dict[str, np.ndarray], cfg: dict, left_context: int, chunk: int,
                    dtype=np.float32) -> np.ndarray:
    """The same model computed chunk by chunk with carried state (what cfm_cache_stream_step does):
    4*chunk input frames per step; caches = last 2 input frames, last 2 conv1 frames, per layer the
    keys / values of the last `left_context` frames and the last K-1 GLU outputs."""
    sd = _prep(sd, dtype)
    x = np.asarray(x_bft, dtype=dtype)
    B, F, T = x.shape
    assert T % (4 * chunk) == 0
    d, H, L = cfg["d_model"], cfg["n_heads"], cfg["n_layers"]
    pe, center = rel_pe_table(max(int(cfg.get("pos_emb_max_len", 5000)), T), d, dtype)
    pe_row = lambda dist: pe[0, center - 1 - dist]          # pe row of position `dist` (>= 0)
    norm = cfg.get("conv_norm_type", "batch_norm")
    half = np.dtype(dtype).type(0.5)
    w1, b1 = sd["pre_encode.conv.0.weight"], sd["pre_encode.conv.0.bias"]
    w2, b2 = sd["pre_encode.conv.2.weight"], sd["pre_encode.conv.2.bias"]
    C = w1.shape[0]
    F1 = (F - 1) // 2 + 1
    mel_c = np.zeros((B, 1, 2, F), dtype=dtype)
    c1_c = np.zeros((B, C, 2, F1), dtype=dtype)
    kc = [np.zeros((B, 0, d), dtype=dtype) for _ in range(L)]
    vc = [np.zeros((B, 0, d), dtype=dtype) for _ in range(L)]
    gc = [None] * L
    outs = []
    for s0 in range(0, T, 4 * chunk):
        t0 = s0 // 4
        xin = np.concatenate([mel_c, x[:, None, :, s0:s0 + 4 * chunk].transpose(0, 1, 3, 2)], axis=2)
        mel_c = xin[:, :, -2:]
        h1 = np.maximum(_valid_conv(xin, w1, b1), 0)                    # (B, C, 2*chunk, F1)
        hin = np.concatenate([c1_c, h1], axis=2)
        c1_c = hin[:, :, -2:]
        h2 = np.maximum(_valid_conv(hin, w2, b2), 0)                    # (B, C, chunk, F2)
        b_, c_, t_, f_ = h2.shape
        xc = h2.transpose(0, 2, 1, 3).reshape(b_, t_, c_ * f_) @ sd["pre_encode.out.weight"].T + sd["pre_encode.out.bias"]
        if cfg.get("xscaling", True):
            xc = xc * xc.dtype.type(math.sqrt(d))
        for i in range(L):
            p = f"layers.{i}."
            xc = xc + half * feed_forward(layer_norm(xc, sd[p + "norm_feed_forward1.weight"],
                                                     sd[p + "norm_feed_forward1.bias"]), sd, p + "feed_forward1.")
            hn = layer_norm(xc, sd[p + "norm_self_att.weight"], sd[p + "norm_self_att.bias"])
            a = p + "self_attn."
            kc[i] = np.concatenate([kc[i], linear(hn, sd[a + "linear_k.weight"], sd[a + "linear_k.bias"])], 1)[:, -(left_context + chunk):]
            vc[i] = np.concatenate([vc[i], linear(hn, sd[a + "linear_v.weight"], sd[a + "linear_v.bias"])], 1)[:, -(left_context + chunk):]
            xc = xc + _chunk_mha(hn, kc[i], vc[i], t0, chunk, left_context, sd, a, H, pe_row)
            y, gc[i] = causal_conv_module(layer_norm(xc, sd[p + "norm_conv.weight"], sd[p + "norm_conv.bias"]), sd,
                                          p + "conv.", norm, gc[i])
            xc = xc + y
            xc = xc + half * feed_forward(layer_norm(xc, sd[p + "norm_feed_forward2.weight"],
                                                     sd[p + "norm_feed_forward2.bias"]), sd, p + "feed_forward2.")
            xc = layer_norm(xc, sd[p + "norm_out.weight"], sd[p + "norm_out.bias"])
        if "out_proj.weight" in sd:
            xc = linear(xc, sd["out_proj.weight"], sd["out_proj.bias"])
        outs.append(xc)
    return np.concatenate(outs, axis=1).transpose(0, 2, 1)


def _valid_conv(x: np.ndarray, w: np.ndarray, b: np.ndarray) -> np.ndarray:
    """Conv2d, stride 2, time unpadded (the caller prepends the 2 cached frames), frequency pad (1, 1)."""
    B, Cin, T, F = x.shape
    Cout = w.shape[0]
    xp = np.zeros((B, Cin, T, F + 2), dtype=x.dtype)
    xp[..., 1:F + 1] = x
    To = (T - 3) // 2 + 1
    Fo = (F + 2 - 3) // 2 + 1
    wm = w.reshape(Cout, -1)
    out = np.empty((B, Cout, To, Fo), dtype=x.dtype)
    for bi in range(B):
        cols = np.empty((Cin, 3, 3, To, Fo), dtype=x.dtype)
        for kt in range(3):
            for kf in range(3):
                cols[:, kt, kf] = xp[bi, :, kt:kt + 2 * To:2, kf:kf + 2 * Fo:2]
        out[bi] = (wm @ cols.reshape(-1, To * Fo)).reshape(Cout, To, Fo)
    return out + b.reshape(1, Cout, 1, 1)
