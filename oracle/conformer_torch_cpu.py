"""PyTorch-CPU restatement of the reference Conformer encoder forward (eval mode).

TEST / BASELINE INFRASTRUCTURE ONLY.  Imported by `tests/` and by the `cpu_baseline` leg of
`bench.py` (the reference's own Python never ships to the GPU box, so this restatement stands in
for it as the timed CPU baseline).  The product path (`conformer-nemo_amd/`) never
imports it.

Same arithmetic as `conformer_oracle.py` (which is pinned to reference-generated goldens), but on
torch CPU ops in the reference's op order and layout, so that its speed is the reference's speed:
  ConvSubsampling 'striding'       subsampling.py:99-116, 151-176 (Conv2d -> ReLU -> Conv2d -> ReLU,
                                   (b,c,t,f) -> (b,t,c*f) flatten, Linear); calc_length :272-282
  RelPositionalEncoding            multi_head_attention.py:235-248, 285-316 (x * sqrt(d), PE window)
  ConformerLayer                   conformer_modules.py:88-121 (macaron FFNs with 1/2 residual,
                                   rel-pos MHSA, convolution module, norm_out)
  RelPositionMultiHeadAttention    multi_head_attention.py:69-115, 159-210 (u/v biases, rel_shift,
                                   -10000 mask fill, softmax, zeroed masked probabilities)
  ConformerConvolution             conformer_modules.py:160-180 ((B,C,T) layout: Conv1d k=1, GLU,
                                   pad-mask fill, depthwise Conv1d, BatchNorm1d eval, Swish, Conv1d)
Weights: a dict keyed exactly like the reference state_dict (fp32 torch tensors).
Validated against the reference-generated goldens in tests/test_torch_cpu_baseline.py (relL2 1e-6)
and timed against the reference itself in this container by tools/cpu_baseline_check.py.
"""
from __future__ import annotations

import math
from typing import Dict, Optional, Sequence, Tuple

import torch
import torch.nn.functional as F

Tensor = torch.Tensor


def calc_length(lengths: Tensor, repeat_num: int = 2) -> Tensor:
    """subsampling.py:272-282 (padding 1, kernel 3, stride 2, floor) in float32, cast to int32."""
    L = lengths.to(torch.float32)
    for _ in range(repeat_num):
        L = torch.floor((L + (2 * 1 - 3)) / 2.0 + 1.0)
    return L.to(torch.int32)


def rel_pe(T: int, d: int, max_len: int = 5000) -> Tensor:
    """extend_pe + create_pe + the forward window (multi_head_attention.py:235-248, 285-316):
    the (2T-1, d) table of positions T-1 ... -(T-1)."""
    positions = torch.arange(T - 1, -T, -1, dtype=torch.float32).unsqueeze(1)
    div_term = torch.exp(torch.arange(0, d, 2, dtype=torch.float32) * -(math.log(10000.0) / d))
    pe = torch.zeros(positions.size(0), d)
    pe[:, 0::2] = torch.sin(positions * div_term)
    pe[:, 1::2] = torch.cos(positions * div_term)
    return pe.unsqueeze(0)


def abs_pe(T: int, d: int) -> Tensor:
    """PositionalEncoding create_pe + forward window (multi_head_attention.py:235-271): positions 0 ... T-1."""
    positions = torch.arange(0, T, dtype=torch.float32).unsqueeze(1)
    div_term = torch.exp(torch.arange(0, d, 2, dtype=torch.float32) * -(math.log(10000.0) / d))
    pe = torch.zeros(T, d)
    pe[:, 0::2] = torch.sin(positions * div_term)
    pe[:, 1::2] = torch.cos(positions * div_term)
    return pe.unsqueeze(0)


def rel_shift(x: Tensor) -> Tensor:
    """multi_head_attention.py:159-170."""
    b, h, qlen, pos_len = x.size()
    x = F.pad(x, pad=(1, 0))
    x = x.view(b, h, -1, qlen)
    return x[:, :, 1:].view(b, h, qlen, pos_len)


def masks(T: int, lengths: Tensor, ctx: Sequence[int] = (-1, -1)) -> Tuple[Tensor, Tensor]:
    """conformer_encoder.py:260-272, 296-299: (pad_mask, att_mask), True = masked."""
    pad = torch.arange(T).expand(lengths.size(0), -1) < lengths.unsqueeze(-1)
    att = pad.unsqueeze(1).repeat([1, T, 1])
    att = torch.logical_and(att, att.transpose(1, 2))
    if ctx[0] >= 0:
        att = att.triu(diagonal=-ctx[0])
    if ctx[1] >= 0:
        att = att.tril(diagonal=ctx[1])
    return ~pad, ~att


def mhsa(x: Tensor, att_mask: Tensor, pos_emb: Tensor, sd: Dict[str, Tensor], p: str, H: int) -> Tensor:
    """RelPositionMultiHeadAttention.forward (multi_head_attention.py:172-210) in eval mode."""
    B, T, D = x.shape
    dk = D // H
    q = F.linear(x, sd[p + "linear_q.weight"], sd[p + "linear_q.bias"]).view(B, -1, H, dk)
    k = F.linear(x, sd[p + "linear_k.weight"], sd[p + "linear_k.bias"]).view(B, -1, H, dk).transpose(1, 2)
    v = F.linear(x, sd[p + "linear_v.weight"], sd[p + "linear_v.bias"]).view(B, -1, H, dk).transpose(1, 2)
    if pos_emb is None:   # MultiHeadAttention.forward (multi_head_attention.py:117-129), abs_pos layers
        scores = torch.matmul(q.transpose(1, 2), k.transpose(-2, -1)) / math.sqrt(dk)
    else:
        pp = F.linear(pos_emb, sd[p + "linear_pos.weight"]).view(pos_emb.size(0), -1, H, dk).transpose(1, 2)
        q_u = (q + sd[p + "pos_bias_u"]).transpose(1, 2)
        q_v = (q + sd[p + "pos_bias_v"]).transpose(1, 2)
        ac = torch.matmul(q_u, k.transpose(-2, -1))
        bd = rel_shift(torch.matmul(q_v, pp.transpose(-2, -1)))[:, :, :, :ac.size(-1)]
        scores = (ac + bd) / math.sqrt(dk)
    m = att_mask.unsqueeze(1)
    attn = torch.softmax(scores.masked_fill(m, -10000.0), dim=-1).masked_fill(m, 0.0)
    o = torch.matmul(attn, v).transpose(1, 2).reshape(B, -1, D)
    return F.linear(o, sd[p + "linear_out.weight"], sd[p + "linear_out.bias"])


def conv_module(x: Tensor, pad_mask: Optional[Tensor], sd: Dict[str, Tensor], p: str, norm: str) -> Tensor:
    """ConformerConvolution.forward (conformer_modules.py:160-180), eval mode, (B, C, T) layout."""
    h = x.transpose(1, 2)
    h = F.conv1d(h, sd[p + "pointwise_conv1.weight"], sd[p + "pointwise_conv1.bias"])
    h = F.glu(h, dim=1)
    if pad_mask is not None:
        h = h.float().masked_fill(pad_mask.unsqueeze(1), 0.0)
    K = sd[p + "depthwise_conv.weight"].shape[-1]
    h = F.conv1d(h, sd[p + "depthwise_conv.weight"], sd[p + "depthwise_conv.bias"], padding=(K - 1) // 2,
                 groups=h.size(1))
    if norm == "batch_norm":
        h = F.batch_norm(h, sd[p + "batch_norm.running_mean"], sd[p + "batch_norm.running_var"],
                         sd[p + "batch_norm.weight"], sd[p + "batch_norm.bias"], False, 0.0, 1e-5)
    else:
        h = F.layer_norm(h.transpose(1, 2), (h.size(1),), sd[p + "batch_norm.weight"],
                         sd[p + "batch_norm.bias"], 1e-5).transpose(1, 2)
    h = F.silu(h)
    h = F.conv1d(h, sd[p + "pointwise_conv2.weight"], sd[p + "pointwise_conv2.bias"])
    return h.transpose(1, 2)


def ffn(x: Tensor, sd: Dict[str, Tensor], p: str) -> Tensor:
    """ConformerFeedForward.forward (conformer_modules.py:195-200)."""
    h = F.silu(F.linear(x, sd[p + "linear1.weight"], sd[p + "linear1.bias"]))
    return F.linear(h, sd[p + "linear2.weight"], sd[p + "linear2.bias"])


def layer(x, att_mask, pos_emb, pad_mask, sd, p: str, H: int, norm: str) -> Tensor:
    """ConformerLayer.forward (conformer_modules.py:88-121), eval mode."""
    d = x.size(-1)
    ln = lambda t, n: F.layer_norm(t, (d,), sd[p + n + ".weight"], sd[p + n + ".bias"], 1e-5)  # noqa: E731
    residual = x
    residual = residual + ffn(ln(x, "norm_feed_forward1"), sd, p + "feed_forward1.") * 0.5
    residual = residual + mhsa(ln(residual, "norm_self_att"), att_mask, pos_emb, sd, p + "self_attn.", H)
    residual = residual + conv_module(ln(residual, "norm_conv"), pad_mask, sd, p + "conv.", norm)
    residual = residual + ffn(ln(residual, "norm_feed_forward2"), sd, p + "feed_forward2.") * 0.5
    return ln(residual, "norm_out")


@torch.no_grad()
def encoder_forward(x_bft: Tensor, lengths: Optional[Tensor], sd: Dict[str, Tensor], cfg: dict) -> Tuple[Tensor, Tensor]:
    """ConformerEncoder.forward_for_export (conformer_encoder.py:236-281), eval mode."""
    B, _, T = x_bft.shape
    d = cfg["d_model"]
    if lengths is None:
        lengths = torch.full((B,), T, dtype=torch.int32)
    x = x_bft.transpose(1, 2).unsqueeze(1)                            # (B, 1, T, F)
    x = F.relu(F.conv2d(x, sd["pre_encode.conv.0.weight"], sd["pre_encode.conv.0.bias"], stride=2, padding=1))
    x = F.relu(F.conv2d(x, sd["pre_encode.conv.2.weight"], sd["pre_encode.conv.2.bias"], stride=2, padding=1))
    b, c, t, f = x.size()
    x = F.linear(x.transpose(1, 2).reshape(b, t, -1), sd["pre_encode.out.weight"], sd["pre_encode.out.bias"])
    lengths = calc_length(lengths)
    if cfg.get("xscaling", True):
        x = x * math.sqrt(d)
    if cfg.get("self_attention_model", "rel_pos") == "abs_pos":   # PositionalEncoding.forward, :257-271
        x = x + abs_pe(x.size(1), d)
        pos_emb = None
    else:
        pos_emb = rel_pe(x.size(1), d)
    pad_mask, att_mask = masks(x.size(1), lengths, cfg.get("att_context_size") or (-1, -1))
    if not cfg.get("use_pad_mask", True):
        pad_mask = None
    for i in range(cfg["n_layers"]):
        x = layer(x, att_mask, pos_emb, pad_mask, sd, f"layers.{i}.", cfg["n_heads"],
                  cfg.get("conv_norm_type", "batch_norm"))
    if "out_proj.weight" in sd:
        x = F.linear(x, sd["out_proj.weight"], sd["out_proj.bias"])
    return x.transpose(1, 2), lengths
