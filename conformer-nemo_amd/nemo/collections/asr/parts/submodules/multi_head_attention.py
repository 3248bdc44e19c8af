"""Attention / positional-encoding parameter containers (reference multi_head_attention.py).

RelPositionMultiHeadAttention's arithmetic (Transformer-XL scores with rel_shift, masked softmax,
P.V) is the fused HIP kernel csrc/attention.hip; linear_q/k/v are one packed MFMA GEMM whose
epilogue writes V pre-transposed, linear_pos of all layers is one GEMM per forward.
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

    def forward(self, *args, **kwargs):
        raise NotImplementedError("attention runs inside ConformerEncoder's native forward")


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
