"""Deterministic weight / input recipe shared by the golden generator and the parity tests.

Weights are regenerated from a seed instead of being committed (the Small config alone is 52 MB).
Every tensor gets its own PCG64 stream seeded from (seed, crc32(key)), so the values do not depend
on iteration order or on which other keys exist.  Distributions are chosen to exercise every term
(SURVEY §8c): non-zero pos_bias_u/v (the reference inits them to zero, which would hide bugs),
randomised BatchNorm running stats and affine, LayerNorm affine away from identity.

Key names and shapes follow the reference ConformerEncoder.state_dict().
"""
from __future__ import annotations

import math
import zlib
from typing import Dict, List, Tuple

import numpy as np


def _rng(seed: int, key: str) -> np.random.Generator:
    return np.random.Generator(np.random.PCG64([seed, zlib.crc32(key.encode())]))


def _uniform(seed, key, shape, lo, hi):
    return (_rng(seed, key).random(size=shape, dtype=np.float64) * (hi - lo) + lo).astype(np.float32)


def encoder_param_shapes(cfg: dict) -> List[Tuple[str, tuple]]:
    """(key, shape) of every state_dict entry of the reference ConformerEncoder for `cfg`
    (conformer_encoder.py:111-216, conformer_modules.py:40-86,131-158,188-193,
    multi_head_attention.py:55-67,141-157, subsampling.py:99-116,151-160)."""
    d = cfg["d_model"]
    H = cfg["n_heads"]
    F = cfg.get("feat_in", 80)
    C = cfg.get("subsampling_conv_channels", -1)
    C = d if C in (-1, None) else C
    dff = d * cfg.get("ff_expansion_factor", 4)
    K = cfg.get("conv_kernel_size", 31)
    F1 = (F - 1) // 2 + 1
    F2 = (F1 - 1) // 2 + 1
    out = [("pre_encode.conv.0.weight", (C, 1, 3, 3)), ("pre_encode.conv.0.bias", (C,)),
           ("pre_encode.conv.2.weight", (C, C, 3, 3)), ("pre_encode.conv.2.bias", (C,)),
           ("pre_encode.out.weight", (d, C * F2)), ("pre_encode.out.bias", (d,))]
    for i in range(cfg["n_layers"]):
        p = f"layers.{i}."
        ln = lambda n: [(p + n + ".weight", (d,)), (p + n + ".bias", (d,))]
        ff = lambda n: [(p + n + ".linear1.weight", (dff, d)), (p + n + ".linear1.bias", (dff,)),
                        (p + n + ".linear2.weight", (d, dff)), (p + n + ".linear2.bias", (d,))]
        out += ln("norm_feed_forward1") + ff("feed_forward1") + ln("norm_conv")
        out += [(p + "conv.pointwise_conv1.weight", (2 * d, d, 1)), (p + "conv.pointwise_conv1.bias", (2 * d,)),
                (p + "conv.depthwise_conv.weight", (d, 1, K)), (p + "conv.depthwise_conv.bias", (d,))]
        if cfg.get("conv_norm_type", "batch_norm") == "batch_norm":
            out += [(p + "conv.batch_norm.weight", (d,)), (p + "conv.batch_norm.bias", (d,)),
                    (p + "conv.batch_norm.running_mean", (d,)), (p + "conv.batch_norm.running_var", (d,)),
                    (p + "conv.batch_norm.num_batches_tracked", ())]
        else:
            out += [(p + "conv.batch_norm.weight", (d,)), (p + "conv.batch_norm.bias", (d,))]
        out += [(p + "conv.pointwise_conv2.weight", (d, d, 1)), (p + "conv.pointwise_conv2.bias", (d,))]
        out += ln("norm_self_att")
        for n in ("linear_q", "linear_k", "linear_v", "linear_out"):
            out += [(p + f"self_attn.{n}.weight", (d, d)), (p + f"self_attn.{n}.bias", (d,))]
        if cfg.get("self_attention_model", "rel_pos") == "rel_pos":   # abs_pos: MultiHeadAttention, no pos terms
            out += [(p + "self_attn.linear_pos.weight", (d, d)),
                    (p + "self_attn.pos_bias_u", (H, d // H)), (p + "self_attn.pos_bias_v", (H, d // H))]
        out += ln("norm_feed_forward2") + ff("feed_forward2") + ln("norm_out")
    fo = cfg.get("feat_out", -1)
    if fo and fo > 0 and fo != d:
        out += [("out_proj.weight", (fo, d)), ("out_proj.bias", (fo,))]
    return out


def make_state_dict(cfg: dict, seed: int = 0) -> Dict[str, np.ndarray]:
    sd = {}
    for key, shape in encoder_param_shapes(cfg):
        leaf = key.rsplit(".", 1)[-1]
        if leaf == "num_batches_tracked":
            sd[key] = np.array(0, dtype=np.int64)
            continue
        if key.endswith("running_mean"):
            sd[key] = _uniform(seed, key, shape, -0.5, 0.5)
        elif key.endswith("running_var"):
            sd[key] = _uniform(seed, key, shape, 0.5, 1.5)
        elif leaf in ("pos_bias_u", "pos_bias_v"):
            sd[key] = _uniform(seed, key, shape, -0.2, 0.2)
        elif len(shape) == 1 and (".norm_" in key or "batch_norm" in key) and leaf == "weight":
            sd[key] = _uniform(seed, key, shape, 0.8, 1.2)
        elif len(shape) == 1:                              # biases (incl. norm biases)
            sd[key] = _uniform(seed, key, shape, -0.1, 0.1)
        else:                                              # weights: U(-1/sqrt(fan_in), 1/sqrt(fan_in))
            fan_in = int(np.prod(shape[1:]))
            a = 1.0 / math.sqrt(fan_in)
            sd[key] = _uniform(seed, key, shape, -a, a)
    return sd


def make_inputs(B: int, T: int, feat_in: int = 80, seed: int = 0, lengths=None):
    """x ~ N(0,1) (like per_feature-normalised mel, features.py:54-68) and ragged lengths
    [T, 0.9T, 0.75T, 0.5T+1, ...] to exercise the masks."""
    g = np.random.Generator(np.random.PCG64([seed, 12345]))
    x = g.standard_normal(size=(B, feat_in, T), dtype=np.float32)
    if lengths is None:
        fr = [1.0, 0.9, 0.75, 0.5]
        lengths = [max(1, int(T * fr[i % 4]) + (1 if i % 4 == 3 else 0)) for i in range(B)]
        lengths = [min(T, l) for l in lengths]
    return x, np.asarray(lengths, dtype=np.int64)
