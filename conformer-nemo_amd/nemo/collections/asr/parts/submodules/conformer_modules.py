"""ConformerLayer / ConformerConvolution / ConformerFeedForward parameter containers
(reference conformer_modules.py:28-200).  Attribute names and shapes are the reference's, so
state_dicts load unchanged; the arithmetic is the native layer loop of csrc/encoder.hip.
"""
from __future__ import annotations

from torch import nn
from torch.nn import LayerNorm

from nemo.collections.asr.parts.submodules.multi_head_attention import (
    MultiHeadAttention,
    RelPositionMultiHeadAttention,
)
from nemo.collections.asr.parts.utils.activations import Swish

__all__ = ["ConformerConvolution", "ConformerFeedForward", "ConformerLayer"]


class ConformerLayer(nn.Module):
    def __init__(self, d_model, d_ff, self_attention_model="rel_pos", n_heads=4, conv_kernel_size=31,
                 conv_norm_type="batch_norm", dropout=0.1, dropout_att=0.1, pos_bias_u=None, pos_bias_v=None):
        super().__init__()
        self.self_attention_model = self_attention_model
        self.n_heads = n_heads
        self.fc_factor = 0.5
        self.norm_feed_forward1 = LayerNorm(d_model)
        self.feed_forward1 = ConformerFeedForward(d_model=d_model, d_ff=d_ff, dropout=dropout)
        self.norm_conv = LayerNorm(d_model)
        self.conv = ConformerConvolution(d_model=d_model, kernel_size=conv_kernel_size, norm_type=conv_norm_type)
        self.norm_self_att = LayerNorm(d_model)
        if self_attention_model == "rel_pos":
            self.self_attn = RelPositionMultiHeadAttention(n_head=n_heads, n_feat=d_model, dropout_rate=dropout_att,
                                                           pos_bias_u=pos_bias_u, pos_bias_v=pos_bias_v)
        elif self_attention_model == "abs_pos":
            self.self_attn = MultiHeadAttention(n_head=n_heads, n_feat=d_model, dropout_rate=dropout_att)
        else:
            raise ValueError(f"'{self_attention_model}' is not not a valid value for 'self_attention_model', "
                             f"valid values can be from ['rel_pos', 'abs_pos']")
        self.norm_feed_forward2 = LayerNorm(d_model)
        self.feed_forward2 = ConformerFeedForward(d_model=d_model, d_ff=d_ff, dropout=dropout)
        self.dropout = nn.Dropout(dropout)
        self.norm_out = LayerNorm(d_model)

    def forward(self, *args, **kwargs):
        raise NotImplementedError("ConformerLayer runs inside ConformerEncoder's native forward")


class ConformerConvolution(nn.Module):
    def __init__(self, d_model, kernel_size, norm_type="batch_norm"):
        super().__init__()
        assert (kernel_size - 1) % 2 == 0
        self.d_model = d_model
        self.pointwise_conv1 = nn.Conv1d(d_model, d_model * 2, kernel_size=1, stride=1, padding=0, bias=True)
        self.depthwise_conv = nn.Conv1d(d_model, d_model, kernel_size=kernel_size, stride=1,
                                        padding=(kernel_size - 1) // 2, groups=d_model, bias=True)
        if norm_type == "batch_norm":
            self.batch_norm = nn.BatchNorm1d(d_model)
        elif norm_type == "layer_norm":
            self.batch_norm = nn.LayerNorm(d_model)
        else:
            raise ValueError(f"conv_norm_type={norm_type} is not valid!")
        self.activation = Swish()
        self.pointwise_conv2 = nn.Conv1d(d_model, d_model, kernel_size=1, stride=1, padding=0, bias=True)

    def forward(self, *args, **kwargs):
        raise NotImplementedError("ConformerConvolution runs inside ConformerEncoder's native forward")


class ConformerFeedForward(nn.Module):
    def __init__(self, d_model, d_ff, dropout, activation=None):
        super().__init__()
        self.linear1 = nn.Linear(d_model, d_ff)
        self.activation = activation if activation is not None else Swish()
        self.dropout = nn.Dropout(p=dropout)
        self.linear2 = nn.Linear(d_ff, d_model)

    def forward(self, *args, **kwargs):
        raise NotImplementedError("ConformerFeedForward runs inside ConformerEncoder's native forward")
