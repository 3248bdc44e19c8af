"""Attention / positional-encoding modules (reference multi_head_attention.py).

RelPositionMultiHeadAttention's arithmetic (Transformer-XL scores with rel_shift, masked softmax,
P.V) is the fused HIP kernel csrc/attention.hip; inside the encoder linear_q/k/v are one packed MFMA
GEMM and linear_pos of all layers is one GEMM per forward.  Called on their own, the attention modules
run the projections on cfm_op_linear and the core on cfm_op_rel_attention (conformer_amd.submodule_ops);
MultiHeadAttention is the same core with zero positional scores and biases.  Inference only.
"""
from __future__ import annotations

import math

import torch
from torch import nn


class MultiHeadAttention(nn.Module):
    def __init__(self, n_head, n_feat, dropout_rate):
        super().__init__()
        assert n_feat % n_head == 0
        self.d_k = n_feat // n_head
        self.s_d_k = math.sqrt(self.d_k)
        self.h = n_head
        self.linear_q = nn.Linear(n_feat, n_feat)
        self.linear_k = nn.Linear(n_feat, n_feat)
        self.linear_v = nn.Linear(n_feat, n_feat)
        self.linear_out = nn.Linear(n_feat, n_feat)
        self.dropout = nn.Dropout(p=dropout_rate)

    def forward(self, query, key, value, mask, pos_emb=None):
        """Scaled dot-product attention (multi_head_attention.py:94-128): (B, T, n_feat) -> (B, T, n_feat)."""
        return self._native_attention(query, key, value, mask, None)

    def set_compute_mode(self, compute: str):
        if compute not in ("bf16", "fp16", "fp32"):
            raise ValueError("compute must be 'bf16', 'fp16' or 'fp32'")
        self.compute = compute

    def _native_attention(self, query, key, value, mask, pos_emb):
        from conformer_amd import submodule_ops as ops
        ops.check_inference(self, query, key, value)
        B, T, d = query.shape
        if key.shape[1] != T or value.shape[1] != T:
            raise NotImplementedError("the native attention core is self-attention shaped (time1 == time2)")
        compute = ops.compute_mode(self)
        dt = ops.COMPUTE_DTYPE[compute]
        dev = query.device
        lengths, ctx = ops.masks_to_lengths(mask, None, B, T, dev)
        proj = lambda x, lin: ops.linear(x.detach().reshape(B * T, d).to(dt).contiguous(), lin.weight, lin.bias, 0,  # noqa: E731
                                         compute)
        q, k, v = proj(query, self.linear_q), proj(key, self.linear_k), proj(value, self.linear_v)
        if pos_emb is None:   # MultiHeadAttention: no positional scores, no biases
            p = torch.zeros((2 * T - 1, d), dtype=dt, device=dev)
            u = vb = torch.zeros((self.h, self.d_k), device=dev)
        else:
            if pos_emb.shape[0] != 1 or pos_emb.shape[1] != 2 * T - 1:
                raise ValueError(f"pos_emb must be (1, 2T-1, n_feat) = (1, {2 * T - 1}, {d})")
            p = ops.linear(pos_emb.detach().reshape(2 * T - 1, d).to(dt).contiguous(), self.linear_pos.weight, None, 0,
                           compute)
            u, vb = self.pos_bias_u, self.pos_bias_v
        ctxv = ops.rel_attention(q, k, v, p, u, vb, lengths, B, T, self.h, self.d_k, ctx, compute)
        y = ops.linear(ctxv, self.linear_out.weight, self.linear_out.bias, 0, compute)
        return y.float().reshape(B, T, d)


class RelPositionMultiHeadAttention(MultiHeadAttention):
    def __init__(self, n_head, n_feat, dropout_rate, pos_bias_u=None, pos_bias_v=None):
        super().__init__(n_head, n_feat, dropout_rate)
        self.linear_pos = nn.Linear(n_feat, n_feat, bias=False)
        if pos_bias_u is None or pos_bias_v is None:
            self.pos_bias_u = nn.Parameter(torch.zeros(self.h, self.d_k))
            self.pos_bias_v = nn.Parameter(torch.zeros(self.h, self.d_k))
        else:
            self.pos_bias_u = pos_bias_u
            self.pos_bias_v = pos_bias_v

    def forward(self, query, key, value, mask, pos_emb):
        """Transformer-XL attention with relative positions (multi_head_attention.py:172-210):
        (B, T, n_feat) -> (B, T, n_feat); mask (B, T, T) True = masked; pos_emb (1, 2T-1, n_feat)."""
        return self._native_attention(query, key, value, mask, pos_emb)


class PositionalEncoding(nn.Module):
    def __init__(self, d_model, dropout_rate, max_len=5000, xscale=None, dropout_rate_emb=0.0):
        super().__init__()
        self.d_model = d_model
        self.xscale = xscale
        self.max_len = max_len
        self.dropout = nn.Dropout(p=dropout_rate)
        self.dropout_emb = nn.Dropout(dropout_rate_emb) if dropout_rate_emb > 0 else None

    def extend_pe(self, length, device=None):
        """The native library owns the table (cfm_encoder_set_max_audio_length)."""
        self.max_len = max(self.max_len, int(length))


class RelPositionalEncoding(PositionalEncoding):
    pass
