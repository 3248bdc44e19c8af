"""CPU restatement (numpy) of the reference Conformer encoder forward path.

TEST INFRASTRUCTURE ONLY.  This module is the parity *checker*: it may be imported only by
`tests/`, `__graft_entry__.smoke()` and the `cpu_baseline` leg of `bench.py`.  The product path
(`conformer-nemo_amd/`) never imports it and has no CPU fallback.

It restates, function by function, the arithmetic of the four reference files on the hot path
(all paths relative to the reference checkout):

  nemo/collections/asr/modules/conformer_encoder.py            (ConformerEncoder)
  nemo/collections/asr/parts/submodules/conformer_modules.py   (ConformerLayer / Convolution / FeedForward)
  nemo/collections/asr/parts/submodules/multi_head_attention.py (RelPositionMultiHeadAttention, RelPositionalEncoding)
  nemo/collections/asr/parts/submodules/subsampling.py          (ConvSubsampling 'striding', calc_length)

The reference dispatches every op to PyTorch ATen; this file re-derives each op from its
definition in plain numpy (float32 by default, float64 on request) in the reference's op order.

Pinning: `tests/test_oracle.py` checks this module against golden vectors produced by running the
reference itself (`tests/golden/gen_goldens.py`, committed with its outputs under `tests/golden/`).
Measured gate there: relL2 <= 1e-6 (fp32) against the reference encoder.

Weights are passed as a flat dict keyed exactly like the reference `state_dict()`.
Eval-mode semantics only (dropout = identity, BatchNorm uses running statistics), which is the
north-star inference path.
"""
from __future__ import annotations

import math
from typing import Dict, Optional, Sequence, Tuple

import numpy as np

__all__ = [
    "calc_length", "conv2d", "conv_subsampling", "create_pe", "rel_positional_encoding",
    "layer_norm", "swish", "feed_forward", "rel_shift", "rel_pos_mha", "conv_module",
    "conformer_layer", "make_masks", "encoder_forward", "encoder_flops",
]


# ----------------------------------------------------------------------------------------------
# subsampling.py
# ----------------------------------------------------------------------------------------------
def calc_length(lengths, padding: int = 1, kernel_size: int = 3, stride: int = 2,
                ceil_mode: bool = False, repeat_num: int = 2) -> np.ndarray:
    """`calc_length` (subsampling.py:272-282): float32 arithmetic, floor, cast to int32."""
    add_pad = np.float32(padding * 2 - kernel_size)
    one = np.float32(1.0)
    lengths = np.asarray(lengths)
    for _ in range(repeat_num):
        lengths = (lengths.astype(np.float32) + add_pad) / np.float32(stride) + one
        lengths = np.ceil(lengths) if ceil_mode else np.floor(lengths)
    return lengths.astype(np.int32)


def conv2d(x: np.ndarray, w: np.ndarray, b: Optional[np.ndarray], stride: int, pad: int) -> np.ndarray:
    """torch.nn.Conv2d semantics (cross-correlation, zero padding) for (B, Cin, H, W) input.

    Used by ConvSubsampling 'striding' (subsampling.py:99-116): kernel 3, stride 2, padding 1.
    """
    B, Cin, H, W = x.shape
    Cout, Cin2, KH, KW = w.shape
    assert Cin == Cin2
    Ho = (H + 2 * pad - KH) // stride + 1
    Wo = (W + 2 * pad - KW) // stride + 1
    xp = np.zeros((B, Cin, H + 2 * pad, W + 2 * pad), dtype=x.dtype)
    xp[:, :, pad:pad + H, pad:pad + W] = x
    out = np.zeros((B, Cout, Ho, Wo), dtype=x.dtype)
    wm = w.reshape(Cout, Cin * KH * KW)
    for bi in range(B):
        cols = np.empty((Cin, KH, KW, Ho, Wo), dtype=x.dtype)
        for kh in range(KH):
            for kw in range(KW):
                cols[:, kh, kw] = xp[bi, :, kh:kh + stride * Ho:stride, kw:kw + stride * Wo:stride]
        out[bi] = (wm @ cols.reshape(Cin * KH * KW, Ho * Wo)).reshape(Cout, Ho, Wo)
    if b is not None:
        out += b.reshape(1, Cout, 1, 1)
    return out


def conv_subsampling(x_btf: np.ndarray, lengths: np.ndarray, sd: Dict[str, np.ndarray],
                     prefix: str = "pre_encode.") -> Tuple[np.ndarray, np.ndarray]:
    """ConvSubsampling.forward, striding mode (subsampling.py:163-176).

    x.unsqueeze(1) -> [Conv2d(3, s2, p1) -> ReLU] x 2 -> (b,c,t,f) -> transpose(1,2).reshape(b,t,c*f)
    (feature index c*F2 + f) -> Linear.
    """
    lengths = calc_length(lengths)
    h = x_btf[:, None, :, :]
    n_conv = 0
    while f"{prefix}conv.{2 * n_conv}.weight" in sd:
        h = conv2d(h, sd[f"{prefix}conv.{2 * n_conv}.weight"], sd[f"{prefix}conv.{2 * n_conv}.bias"], 2, 1)
        h = np.maximum(h, 0)                     # activation=nn.ReLU() (conformer_encoder.py:158)
        n_conv += 1
    b, c, t, f = h.shape
    h = h.transpose(0, 2, 1, 3).reshape(b, t, c * f)
    y = h @ sd[f"{prefix}out.weight"].T + sd[f"{prefix}out.bias"]
    return y, lengths


# ----------------------------------------------------------------------------------------------
# multi_head_attention.py
# ----------------------------------------------------------------------------------------------
def create_pe(positions: np.ndarray, d_model: int, dtype=np.float32) -> np.ndarray:
    """PositionalEncoding.create_pe (multi_head_attention.py:235-248), float32 like the reference."""
    positions = positions.astype(np.float32).reshape(-1, 1)
    div_term = np.exp(np.arange(0, d_model, 2, dtype=np.float32) * np.float32(-(math.log(10000.0) / d_model)))
    pe = np.zeros((positions.shape[0], d_model), dtype=np.float32)
    pe[:, 0::2] = np.sin(positions * div_term)
    pe[:, 1::2] = np.cos(positions * div_term)
    return pe[None].astype(dtype)


def rel_pe_table(max_len: int, d_model: int, dtype=np.float32) -> Tuple[np.ndarray, int]:
    """RelPositionalEncoding.extend_pe (multi_head_attention.py:285-294): positions L-1 ... -(L-1)."""
    positions = np.arange(max_len - 1, -max_len, -1, dtype=np.float32)
    pe = create_pe(positions, d_model, dtype)
    center_pos = pe.shape[1] // 2 + 1
    return pe, center_pos


def rel_positional_encoding(x: np.ndarray, pe: np.ndarray, center_pos: int,
                            xscale: Optional[float]) -> Tuple[np.ndarray, np.ndarray]:
    """RelPositionalEncoding.forward (multi_head_attention.py:296-316), eval mode."""
    if xscale:
        x = x * x.dtype.type(xscale)
    T = x.shape[1]
    pos_emb = pe[:, center_pos - T: center_pos + T - 1]
    return x, pos_emb


def abs_positional_encoding(x: np.ndarray, pe: np.ndarray, xscale: Optional[float]) -> Tuple[np.ndarray, np.ndarray]:
    """PositionalEncoding.forward (multi_head_attention.py:257-271), eval mode: x * xscale + pe[:, :T]."""
    if xscale:
        x = x * x.dtype.type(xscale)
    pos_emb = pe[:, :x.shape[1]]
    return x + pos_emb, pos_emb


def layer_norm(x: np.ndarray, w: np.ndarray, b: np.ndarray, eps: float = 1e-5) -> np.ndarray:
    """torch.nn.LayerNorm over the last dim (biased variance, eps inside the sqrt)."""
    mu = x.mean(axis=-1, keepdims=True)
    var = ((x - mu) ** 2).mean(axis=-1, keepdims=True)
    return (x - mu) / np.sqrt(var + x.dtype.type(eps)) * w + b


def swish(x: np.ndarray) -> np.ndarray:
    """Swish == nn.SiLU (activations.py:20): x * sigmoid(x)."""
    return x / (1 + np.exp(-x))


def linear(x, w, b=None):
    y = x @ w.T
    return y if b is None else y + b


def feed_forward(x: np.ndarray, sd, p: str) -> np.ndarray:
    """ConformerFeedForward.forward (conformer_modules.py:195-200): Linear -> Swish -> Linear."""
    h = swish(linear(x, sd[p + "linear1.weight"], sd[p + "linear1.bias"]))
    return linear(h, sd[p + "linear2.weight"], sd[p + "linear2.bias"])


def rel_shift(x: np.ndarray) -> np.ndarray:
    """RelPositionMultiHeadAttention.rel_shift (multi_head_attention.py:159-170), literally:
    pad one zero column on the left, view as (b,h,t2+1,t1), drop the first row, view back."""
    b, h, qlen, pos_len = x.shape
    x = np.concatenate([np.zeros((b, h, qlen, 1), dtype=x.dtype), x], axis=-1)
    x = x.reshape(b, h, -1, qlen)
    x = x[:, :, 1:].reshape(b, h, qlen, pos_len)
    return x


def rel_pos_mha(x: np.ndarray, mask: Optional[np.ndarray], pos_emb: np.ndarray, sd, p: str,
                n_heads: int) -> np.ndarray:
    """RelPositionMultiHeadAttention.forward (multi_head_attention.py:172-210) with
    forward_qkv (69-92) and forward_attention (94-115); mask True = masked (-10000 fill, then 0)."""
    B, T, D = x.shape
    dk = D // n_heads
    q = linear(x, sd[p + "linear_q.weight"], sd[p + "linear_q.bias"]).reshape(B, T, n_heads, dk)
    k = linear(x, sd[p + "linear_k.weight"], sd[p + "linear_k.bias"]).reshape(B, T, n_heads, dk).transpose(0, 2, 1, 3)
    v = linear(x, sd[p + "linear_v.weight"], sd[p + "linear_v.bias"]).reshape(B, T, n_heads, dk).transpose(0, 2, 1, 3)
    nbp = pos_emb.shape[0]
    pp = linear(pos_emb, sd[p + "linear_pos.weight"]).reshape(nbp, -1, n_heads, dk).transpose(0, 2, 1, 3)
    q_u = (q + sd[p + "pos_bias_u"]).transpose(0, 2, 1, 3)
    q_v = (q + sd[p + "pos_bias_v"]).transpose(0, 2, 1, 3)
    ac = q_u @ k.transpose(0, 1, 3, 2)
    bd = q_v @ pp.transpose(0, 1, 3, 2)
    bd = rel_shift(bd)[:, :, :, :ac.shape[-1]]
    scores = (ac + bd) / x.dtype.type(math.sqrt(dk))
    return _attend(scores, mask, v, sd, p)


def mha(x: np.ndarray, mask: Optional[np.ndarray], sd, p: str, n_heads: int) -> np.ndarray:
    """MultiHeadAttention.forward (multi_head_attention.py:117-129), the abs_pos layers' attention:
    scores = q.k^T / sqrt(d_k), then forward_attention (94-115)."""
    B, T, D = x.shape
    dk = D // n_heads
    q = linear(x, sd[p + "linear_q.weight"], sd[p + "linear_q.bias"]).reshape(B, T, n_heads, dk).transpose(0, 2, 1, 3)
    k = linear(x, sd[p + "linear_k.weight"], sd[p + "linear_k.bias"]).reshape(B, T, n_heads, dk).transpose(0, 2, 1, 3)
    v = linear(x, sd[p + "linear_v.weight"], sd[p + "linear_v.bias"]).reshape(B, T, n_heads, dk).transpose(0, 2, 1, 3)
    scores = (q @ k.transpose(0, 1, 3, 2)) / x.dtype.type(math.sqrt(dk))
    return _attend(scores, mask, v, sd, p)


def _attend(scores, mask, v, sd, p):
    """forward_attention (multi_head_attention.py:94-115) + linear_out."""
    B, _, T, _ = scores.shape
    x = scores
    if mask is not None:
        m = mask[:, None]
        scores = np.where(m, x.dtype.type(-10000.0), scores)
        e = np.exp(scores - scores.max(-1, keepdims=True))
        attn = e / e.sum(-1, keepdims=True)
        attn = np.where(m, x.dtype.type(0.0), attn)
    else:
        e = np.exp(scores - scores.max(-1, keepdims=True))
        attn = e / e.sum(-1, keepdims=True)
    o = (attn @ v).transpose(0, 2, 1, 3).reshape(B, T, -1)
    return linear(o, sd[p + "linear_out.weight"], sd[p + "linear_out.bias"])


def conv_module(x: np.ndarray, pad_mask: Optional[np.ndarray], sd, p: str,
                norm_type: str = "batch_norm") -> np.ndarray:
    """ConformerConvolution.forward (conformer_modules.py:160-180), eval mode.

    pointwise_conv1 (k=1) -> GLU(dim=channels) -> masked_fill(pad, 0) -> depthwise conv (k, pad (k-1)/2,
    groups=d) -> BatchNorm1d(running stats) | LayerNorm -> Swish -> pointwise_conv2.
    Works in (B, T, C) layout; the reference's (B, C, T) transposes carry no arithmetic.
    """
    B, T, D = x.shape
    h = linear(x, sd[p + "pointwise_conv1.weight"][:, :, 0], sd[p + "pointwise_conv1.bias"])
    h = h[..., :D] * (1 / (1 + np.exp(-h[..., D:])))       # nn.functional.glu(x, dim=1)
    if pad_mask is not None:
        h = np.where(pad_mask[:, :, None], h.dtype.type(0.0), h)
    w = sd[p + "depthwise_conv.weight"][:, 0, :]             # (D, K)
    K = w.shape[1]
    pad = (K - 1) // 2
    hp = np.zeros((B, T + 2 * pad, D), dtype=h.dtype)
    hp[:, pad:pad + T] = h
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
    return linear(out, sd[p + "pointwise_conv2.weight"][:, :, 0], sd[p + "pointwise_conv2.bias"])


def conformer_layer(x, att_mask, pos_emb, pad_mask, sd, p: str, n_heads: int,
                    norm_type: str = "batch_norm", self_attention_model: str = "rel_pos") -> np.ndarray:
    """ConformerLayer.forward (conformer_modules.py:88-121), eval mode (dropout = identity);
    self_attention_model 'abs_pos' attends with MultiHeadAttention (conformer_modules.py:106-107)."""
    half = x.dtype.type(0.5)
    residual = x
    h = feed_forward(layer_norm(x, sd[p + "norm_feed_forward1.weight"], sd[p + "norm_feed_forward1.bias"]),
                     sd, p + "feed_forward1.")
    residual = residual + h * half
    h = layer_norm(residual, sd[p + "norm_self_att.weight"], sd[p + "norm_self_att.bias"])
    if self_attention_model == "abs_pos":
        h = mha(h, att_mask, sd, p + "self_attn.", n_heads)
    else:
        h = rel_pos_mha(h, att_mask, pos_emb, sd, p + "self_attn.", n_heads)
    residual = residual + h
    h = layer_norm(residual, sd[p + "norm_conv.weight"], sd[p + "norm_conv.bias"])
    h = conv_module(h, pad_mask, sd, p + "conv.", norm_type)
    residual = residual + h
    h = feed_forward(layer_norm(residual, sd[p + "norm_feed_forward2.weight"], sd[p + "norm_feed_forward2.bias"]),
                     sd, p + "feed_forward2.")
    residual = residual + h * half
    return layer_norm(residual, sd[p + "norm_out.weight"], sd[p + "norm_out.bias"])


# ----------------------------------------------------------------------------------------------
# conformer_encoder.py
# ----------------------------------------------------------------------------------------------
def make_masks(T: int, lengths: np.ndarray, att_context_size: Sequence[int] = (-1, -1)):
    """make_pad_mask + att_mask (conformer_encoder.py:260-272, 296-299). Returns (pad, att),
    both True = masked, like the reference after its inversion."""
    pad_valid = np.arange(T)[None, :] < np.asarray(lengths).reshape(-1, 1)
    att = pad_valid[:, None, :] & pad_valid[:, :, None]
    if att_context_size[0] >= 0:
        att = np.triu(att, k=-att_context_size[0])
    if att_context_size[1] >= 0:
        att = np.tril(att, k=att_context_size[1])
    return ~pad_valid, ~att


def encoder_forward(x_bft: np.ndarray, lengths: Optional[np.ndarray], sd: Dict[str, np.ndarray],
                    cfg: dict, dtype=np.float32) -> Tuple[np.ndarray, np.ndarray]:
    """ConformerEncoder.forward_for_export (conformer_encoder.py:236-281), eval mode.

    cfg keys follow the reference constructor (conformer_encoder.py:111-132): d_model, n_heads,
    n_layers, xscaling, att_context_size, pos_emb_max_len, conv_norm_type, feat_out.
    Returns (outputs (B, D, T'), encoded_lengths (B,) int32).
    """
    sd = {k: (v.astype(dtype) if np.issubdtype(np.asarray(v).dtype, np.floating) else v) for k, v in sd.items()}
    x = np.asarray(x_bft, dtype=dtype)
    B, F, T = x.shape
    d = cfg["d_model"]
    max_len = max(int(cfg.get("pos_emb_max_len", 5000)), T)      # set_max_audio_length (218-229, 240-241)
    if lengths is None:
        lengths = np.full((B,), T, dtype=np.int32)
    x = x.transpose(0, 2, 1)
    x, lengths = conv_subsampling(x, lengths, sd)
    xscale = math.sqrt(d) if cfg.get("xscaling", True) else None
    sam = cfg.get("self_attention_model", "rel_pos")
    if sam == "abs_pos":
        x, pos_emb = abs_positional_encoding(x, create_pe(np.arange(max_len), d, dtype), xscale)
    else:
        pe, center = rel_pe_table(max_len, d, dtype)
        x, pos_emb = rel_positional_encoding(x, pe, center, xscale)
    Tp = x.shape[1]
    pad_mask, att_mask = make_masks(Tp, lengths, cfg.get("att_context_size") or (-1, -1))
    if not cfg.get("use_pad_mask", True):   # enable_pad_mask(False): pad_mask = None (conformer_encoder.py:269-272)
        pad_mask = None
    for i in range(cfg["n_layers"]):
        x = conformer_layer(x, att_mask, pos_emb, pad_mask, sd, f"layers.{i}.", cfg["n_heads"],
                            cfg.get("conv_norm_type", "batch_norm"), sam)
    if "out_proj.weight" in sd:
        x = linear(x, sd["out_proj.weight"], sd["out_proj.bias"])
    return x.transpose(0, 2, 1), lengths


def encoder_flops(B: int, T: int, d: int, n_layers: int, F: int = 80, K: int = 31,
                  conv_channels: Optional[int] = None, ff_expansion: int = 4) -> float:
    """Algorithmic FLOPs of one encoder forward (SURVEY §8d formula, which matches torch
    FlopCounterMode on the reference exactly). 2 FLOPs per multiply-add."""
    C = conv_channels or d
    T1 = int(calc_length([T], repeat_num=1)[0])
    Tp = int(calc_length([T], repeat_num=2)[0])
    F1 = (F - 1) // 2 + 1
    F2 = (F1 - 1) // 2 + 1
    dff = ff_expansion * d
    sub = 2 * B * T1 * F1 * C * 9 + 2 * B * Tp * F2 * C * C * 9 + 2 * B * Tp * (C * F2) * d
    per_layer = (2 * B * Tp * d * dff * 2 * 2          # two FFNs, two GEMMs each
                 + 2 * B * Tp * d * d * 4              # q, k, v, out
                 + 2 * B * Tp * d * 2 * d              # pointwise_conv1 (d -> 2d)
                 + 2 * B * Tp * d * d                  # pointwise_conv2
                 + 2 * (2 * Tp - 1) * d * d            # linear_pos
                 + 2 * B * Tp * d * (4 * Tp - 1)       # ac (T'), bd (2T'-1), AV (T')
                 + 2 * B * Tp * d * K)                 # depthwise conv
    return float(sub + n_layers * per_layer)
