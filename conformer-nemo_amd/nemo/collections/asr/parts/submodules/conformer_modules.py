"""ConformerLayer / ConformerConvolution / ConformerFeedForward (reference conformer_modules.py:28-200).
Attribute names and shapes are the reference's, so state_dicts load unchanged.  Inside ConformerEncoder
the arithmetic is the native layer loop of csrc/encoder.hip; called on their own, the modules run
natively too (conformer_amd.submodule_ops): ConformerLayer through the same layer stack
(cfm_encoder_layers_forward), the feed-forward and convolution modules through the kernel-level
entry points.  Standalone calls are inference-only (eval mode, no autograd)."""
from __future__ import annotations

import torch
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

    def forward(self, x, att_mask=None, pos_emb=None, pad_mask=None):
        """x (B, T, d_model) -> (B, T, d_model) (conformer_modules.py:88-121): macaron FFN, rel-pos MHSA
        (or MultiHeadAttention for abs_pos), convolution module, FFN, norm_out, on the native layer stack.
        att_mask (B, T, T) / pad_mask (B, T) (True = masked) as ConformerEncoder builds them; pos_emb
        (1, 2T-1, d_model) from RelPositionalEncoding (ignored for abs_pos)."""
        from conformer_amd import submodule_ops as ops
        ops.check_inference(self, x)
        abs_pos = self.self_attention_model == "abs_pos"
        if abs_pos:
            pos_emb = None   # MultiHeadAttention takes no positional input (conformer_modules.py:106-107)
        elif pos_emb is None:
            raise ValueError("rel_pos ConformerLayer needs pos_emb (RelPositionalEncoding's output)")
        B, T, _ = x.shape
        lengths, ctx = ops.masks_to_lengths(att_mask, pad_mask, B, T, x.device)
        if not hasattr(self, "_runner"):
            self._runner = ops.LayerRunner()
        return self._runner.forward(self, x, lengths, pos_emb, ctx, pad_mask is not None, ops.compute_mode(self),
                                    abs_pos=abs_pos)

    def set_compute_mode(self, compute: str):
        if compute not in ("bf16", "fp16", "fp32"):
            raise ValueError("compute must be 'bf16', 'fp16' or 'fp32'")
        self.compute = compute


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

    def forward(self, x, pad_mask=None):
        """x (B, T, d_model) -> (B, T, d_model) (conformer_modules.py:160-180): pointwise_conv1, GLU, pad mask,
        depthwise conv, Batch/LayerNorm, Swish, pointwise_conv2.  pad_mask (B, T), True = padded frame."""
        from conformer_amd import submodule_ops as ops
        ops.check_inference(self, x)
        compute = ops.compute_mode(self)
        B, T, d = x.shape
        lengths = None
        if pad_mask is not None:
            lengths, _ = ops.masks_to_lengths(None, pad_mask, B, T, x.device)
        x2 = x.detach().reshape(B * T, d).to(ops.COMPUTE_DTYPE[compute]).contiguous()
        pre = ops.linear(x2, self.pointwise_conv1.weight, self.pointwise_conv1.bias, 0, compute)
        mid = ops.conv_glu_dwconv(pre, lengths, B, T, d, self, compute)
        y = ops.linear(mid, self.pointwise_conv2.weight, self.pointwise_conv2.bias, 0, compute)
        return y.float().reshape(B, T, d)


class ConformerFeedForward(nn.Module):
    def __init__(self, d_model, d_ff, dropout, activation=None):
        super().__init__()
        self.linear1 = nn.Linear(d_model, d_ff)
        self.activation = activation if activation is not None else Swish()
        self.dropout = nn.Dropout(p=dropout)
        self.linear2 = nn.Linear(d_ff, d_model)

    def forward(self, x):
        """linear1 -> Swish -> linear2 (conformer_modules.py:195-200; dropout is the identity in eval)."""
        from conformer_amd import submodule_ops as ops
        ops.check_inference(self, x)
        if not isinstance(self.activation, (Swish, nn.SiLU)):
            raise NotImplementedError("the native feed-forward fuses Swish; other activations are not implemented")
        compute = ops.compute_mode(self)
        shape = x.shape
        x2 = x.detach().reshape(-1, shape[-1]).to(ops.COMPUTE_DTYPE[compute]).contiguous()
        h = ops.linear(x2, self.linear1.weight, self.linear1.bias, 2, compute)
        y = ops.linear(h, self.linear2.weight, self.linear2.bias, 0, compute)
        return y.float().reshape(*shape[:-1], y.shape[-1])
