"""Native forwards of the Conformer submodules called on their own (reference conformer_modules.py:88-200,
multi_head_attention.py:43-210): ConformerLayer, ConformerFeedForward, ConformerConvolution,
RelPositionMultiHeadAttention and MultiHeadAttention.

* `ConformerLayer` runs the encoder's own layer stack (cfm_encoder_layers_forward) on a one-layer handle
  built from the layer's parameters: the same fused kernels, LayerNorm folding and masks as inside
  ConformerEncoder.
* The others compose the kernel-level entry points of include/cfm_encoder.h: cfm_op_linear (MFMA GEMM +
  bias / Swish), cfm_op_rel_attention (fused rel-pos attention core) and cfm_op_conv_glu_dwconv (GLU, pad
  mask, depthwise conv, Batch/LayerNorm, Swish).

Masks: the encoder's masks are functions of the utterance lengths and att_context_size
(conformer_encoder.py:257-270); the native kernels derive them from those, so the (B, T, T) att_mask and
(B, T) pad_mask given here are converted back into lengths and a context window, and a mask of any other
form is refused (NotImplementedError).  Inference only: the standalone modules have no native backward
(training runs through ConformerEncoder.train()), so train mode or inputs that require grad are refused.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional, Tuple

import torch

from . import _lib

COMPUTE_DTYPE = {"bf16": torch.bfloat16, "fp32": torch.float32, "fp16": torch.float16}
COMPUTE_ID = {"fp32": 0, "bf16": 1, "fp16": 2}


def compute_mode(module) -> str:
    c = getattr(module, "compute", None) or os.environ.get("CFM_COMPUTE", "bf16")
    if c not in COMPUTE_ID:
        raise ValueError("compute must be 'bf16', 'fp16' or 'fp32'")
    return c


def check_inference(module, *tensors) -> None:
    if module.training:
        raise NotImplementedError(f"{type(module).__name__}: standalone native forward is eval-mode only "
                                  "(the native training step runs through ConformerEncoder.train())")
    if torch.is_grad_enabled() and any(t is not None and t.requires_grad for t in tensors):
        raise RuntimeError(f"{type(module).__name__}: the standalone native forward does not propagate "
                           "gradients; call it under torch.no_grad()/inference_mode()")
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise RuntimeError(f"{type(module).__name__} (MI355X-native) expects its inputs on a ROCm GPU")


def _stream(dev) -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


# ---- masks -> (lengths, context) ------------------------------------------------------------------
def canonical_att_mask(lengths: torch.Tensor, T: int, left: int, right: int) -> torch.Tensor:
    """The encoder's attention mask (conformer_encoder.py:262-270), True = masked."""
    rng = torch.arange(T, device=lengths.device)
    valid = rng.unsqueeze(0) < lengths.unsqueeze(-1)
    m = valid.unsqueeze(1) & valid.unsqueeze(2)
    if left >= 0:
        m = m.triu(diagonal=-left)
    if right >= 0:
        m = m.tril(diagonal=right)
    return ~m


def masks_to_lengths(att_mask: Optional[torch.Tensor], pad_mask: Optional[torch.Tensor], B: int, T: int,
                     dev) -> Tuple[torch.Tensor, Tuple[int, int]]:
    """Lengths (B,) int32 and the (left, right) context window that reproduce the given masks."""
    if pad_mask is not None:
        if pad_mask.shape != (B, T):
            raise ValueError(f"pad_mask must be (B, T) = ({B}, {T}), got {tuple(pad_mask.shape)}")
        valid = ~pad_mask.to(dev, torch.bool)
        lengths = valid.sum(-1).to(torch.int32)
        if not torch.equal(valid, torch.arange(T, device=dev).unsqueeze(0) < lengths.unsqueeze(-1)):
            raise NotImplementedError("pad_mask must mark a suffix of padded frames per utterance")
    elif att_mask is not None:
        lengths = (~att_mask.to(dev, torch.bool)).any(-1).sum(-1).to(torch.int32)
    else:
        lengths = torch.full((B,), T, dtype=torch.int32, device=dev)
    if att_mask is None:
        return lengths, (-1, -1)
    att_mask = att_mask.to(dev, torch.bool)
    if att_mask.shape != (B, T, T):
        raise ValueError(f"att_mask must be (B, T, T) = ({B}, {T}, {T}), got {tuple(att_mask.shape)}")
    # the context window: the widest band of allowed keys around the diagonal in the longest utterance
    b = int(torch.argmax(lengths).item())
    L = int(lengths[b].item())
    left = right = -1
    if L > 0:
        allowed = ~att_mask[b, :L, :L]
        i = torch.arange(L, device=dev)
        j = torch.arange(L, device=dev)
        dist = j.unsqueeze(0) - i.unsqueeze(1)                    # key - query
        far_left = int((-dist).masked_fill(~allowed, -1).max().item())
        far_right = int(dist.masked_fill(~allowed, -1).max().item())
        left = -1 if far_left >= L - 1 else far_left
        right = -1 if far_right >= L - 1 else far_right
    if not torch.equal(att_mask, canonical_att_mask(lengths, T, left, right)):
        raise NotImplementedError("att_mask must be the encoder's length / att_context_size mask "
                                  "(conformer_encoder.py:262-270); arbitrary masks are not supported natively")
    return lengths, (left, right)


# ---- kernel-level ops ------------------------------------------------------------------------------
# packed weights of `linear`, per (weight, bias, compute): reused while neither tensor changed (same
# storage and autograd version), re-packed on the device otherwise (cfm_op_linear_pack, stream-ordered)
_LINEAR_PACKS: "dict" = {}


def _linear_pack(lib, mode, compute, weight, bias, dev):
    key = (id(weight), id(bias) if bias is not None else None, compute, str(dev))
    ver = (weight.data_ptr(), weight._version, tuple(weight.shape), str(weight.dtype),
           None if bias is None else (bias.data_ptr(), bias._version))
    hit = _LINEAR_PACKS.get(key)
    if hit is not None and hit[0] == ver:
        return hit[1], hit[2], hit[3]
    w = weight.detach().reshape(weight.shape[0], -1).to(dev, torch.float32).contiguous()
    N, K = w.shape
    b = None if bias is None else bias.detach().to(dev, torch.float32).contiguous()
    need = ctypes.c_size_t(0)
    _lib.check(lib.cfm_op_linear_pack(mode, None, None, N, K, None, ctypes.byref(need), _stream(dev)),
               "cfm_op_linear_pack", lib)
    ws = torch.empty(need.value, dtype=torch.uint8, device=dev)
    _lib.check(lib.cfm_op_linear_pack(mode, w.data_ptr(), None if b is None else b.data_ptr(), N, K, ws.data_ptr(),
                                      ctypes.byref(need), _stream(dev)), "cfm_op_linear_pack", lib)
    if len(_LINEAR_PACKS) > 256:
        _LINEAR_PACKS.clear()
    # w / b are kept alive with the pack so the device copy above never reads freed memory, and weight /
    # bias themselves so that their id() (the key) cannot be reused by another tensor while cached
    _LINEAR_PACKS[key] = (ver, ws, N, K, w, b, weight, bias)
    return ws, N, K


def linear(x2d: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor], act: int, compute: str) -> torch.Tensor:
    """x2d (M, K) in the compute dtype -> (M, N) compute dtype; act 0 none, 1 relu, 2 swish
    (cfm_op_linear_pack once per weight version, then cfm_op_linear_packed)."""
    lib = _lib.load(_lib.variant_of(compute))
    dev = x2d.device
    M, K = x2d.shape
    mode = COMPUTE_ID[compute]
    ws, N, Kw = _linear_pack(lib, mode, compute, weight, bias, dev)
    if Kw != K:
        raise ValueError(f"weight has {Kw} input features, x has {K}")
    y = torch.empty((M, N), dtype=COMPUTE_DTYPE[compute], device=dev)
    if M == 0:
        return y
    _lib.check(lib.cfm_op_linear_packed(mode, x2d.data_ptr(), M, K, ws.data_ptr(), N, act, y.data_ptr(), _stream(dev)),
               "cfm_op_linear_packed", lib)
    return y


def rel_attention(q, k, v, p, pos_u, pos_v, lengths, B, T, H, dk, ctx, compute) -> torch.Tensor:
    """Fused attention core (cfm_op_rel_attention) on projected q, k, v (B*T, H*dk) and p (2T-1, H*dk)."""
    lib = _lib.load(_lib.variant_of(compute))
    dev = q.device
    mode = COMPUTE_ID[compute]
    out = torch.empty((B * T, H * dk), dtype=COMPUTE_DTYPE[compute], device=dev)
    ws = torch.empty(int(lib.cfm_op_rel_attention_ws_size(mode, B, T, H, dk)), dtype=torch.uint8, device=dev)
    u = pos_u.detach().to(dev, torch.float32).contiguous()
    vb = pos_v.detach().to(dev, torch.float32).contiguous()
    _lib.check(lib.cfm_op_rel_attention(mode, q.data_ptr(), k.data_ptr(), v.data_ptr(), p.data_ptr(), u.data_ptr(),
                                        vb.data_ptr(), lengths.data_ptr(), B, T, H, dk, int(ctx[0]), int(ctx[1]),
                                        out.data_ptr(), ws.data_ptr(), _stream(dev)), "cfm_op_rel_attention", lib)
    return out


def conv_glu_dwconv(pre, lengths, B, T, d, conv, compute) -> torch.Tensor:
    """GLU + pad mask + depthwise conv + Batch/LayerNorm + Swish (cfm_op_conv_glu_dwconv) on pointwise_conv1's
    output pre (B*T, 2d); `conv` is the ConformerConvolution holding the weights."""
    lib = _lib.load(_lib.variant_of(compute))
    dev = pre.device
    mode = COMPUTE_ID[compute]
    K = conv.depthwise_conv.kernel_size[0]
    f32 = lambda t: None if t is None else t.detach().to(dev, torch.float32).contiguous()   # noqa: E731
    norm = conv.batch_norm
    is_bn = isinstance(norm, torch.nn.BatchNorm1d)
    dw_w, dw_b, nw, nb = f32(conv.depthwise_conv.weight), f32(conv.depthwise_conv.bias), f32(norm.weight), f32(norm.bias)
    mean = f32(norm.running_mean) if is_bn else None
    var = f32(norm.running_var) if is_bn else None
    out = torch.empty((B * T, d), dtype=COMPUTE_DTYPE[compute], device=dev)
    nbytes = int(lib.cfm_op_conv_glu_dwconv_ws_size(mode, B, T, d, K))
    ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    _lib.check(lib.cfm_op_conv_glu_dwconv(mode, pre.data_ptr(), None if lengths is None else lengths.data_ptr(), B, T,
                                          d, K, dw_w.data_ptr(), dw_b.data_ptr(), 0 if is_bn else 1, nw.data_ptr(),
                                          nb.data_ptr(), None if mean is None else mean.data_ptr(),
                                          None if var is None else var.data_ptr(), out.data_ptr(), ws.data_ptr(),
                                          nbytes, _stream(dev)), "cfm_op_conv_glu_dwconv", lib)
    return out


# ---- ConformerLayer through the encoder's layer stack -----------------------------------------------
_FRONT_FEAT, _FRONT_CH = 8, 64    # shape of the unused subsampling weights of the one-layer handle


class LayerRunner:
    """A one-layer native encoder handle holding one ConformerLayer's parameters (per device, compute
    mode and context window); re-packed when a parameter changes."""

    def __init__(self):
        self._handles = {}
        self._versions = {}

    def forward(self, layer, x: torch.Tensor, lengths: torch.Tensor, pos_emb: Optional[torch.Tensor],
                ctx: Tuple[int, int], use_pad_mask: bool, compute: str, abs_pos: bool = False) -> torch.Tensor:
        from .runtime import NativeEncoder, make_cfg
        d = layer.norm_out.normalized_shape[0]
        d_ff = layer.feed_forward1.linear1.out_features
        if d_ff % d:
            raise NotImplementedError(f"d_ff={d_ff} is not a multiple of d_model={d} (the native layer's FFN width "
                                      "is d_model * ff_expansion_factor)")
        dev = x.device
        key = (dev.index, compute, ctx, abs_pos)
        enc = self._handles.get(key)
        norm_type = "batch_norm" if isinstance(layer.conv.batch_norm, torch.nn.BatchNorm1d) else "layer_norm"
        if enc is None:
            with torch.cuda.device(dev):
                cfg = make_cfg(_FRONT_FEAT, 1, d, n_heads=layer.n_heads, ff_expansion_factor=d_ff // d,
                               subsampling_conv_channels=_FRONT_CH, att_context_size=list(ctx),
                               conv_kernel_size=layer.conv.depthwise_conv.kernel_size[0], conv_norm_type=norm_type)
                enc = NativeEncoder(cfg, device=dev.index, compute=compute)
                if abs_pos:   # MultiHeadAttention: positional projection and biases packed as zeros
                    enc.set_abs_pos(True)
            self._handles[key] = enc
        sd = layer.state_dict(keep_vars=True)
        version = tuple((t.data_ptr(), t._version) for t in sd.values())
        if self._versions.get(key) != version:
            tensors = {"layers.0." + k: v for k, v in sd.items() if torch.is_floating_point(v)}
            f2 = ((_FRONT_FEAT - 1) // 2 + 1 - 1) // 2 + 1
            for name, shape in (("pre_encode.conv.0.weight", (_FRONT_CH, 1, 3, 3)), ("pre_encode.conv.0.bias", (_FRONT_CH,)),
                                ("pre_encode.conv.2.weight", (_FRONT_CH, _FRONT_CH, 3, 3)),
                                ("pre_encode.conv.2.bias", (_FRONT_CH,)), ("pre_encode.out.weight", (d, _FRONT_CH * f2)),
                                ("pre_encode.out.bias", (d,))):
                tensors[name] = torch.zeros(shape, device=dev)
            with torch.cuda.device(dev):
                enc.set_weights(tensors)
            self._versions[key] = version
        enc.set_pad_mask(use_pad_mask)
        pe = None if pos_emb is None else pos_emb.reshape(-1, d)
        return enc.layers_forward(x, lengths, pe)


def _heads_for(d: int) -> int:
    """A head count the zero-layer handle accepts (d % h == 0, d / h <= 128); heads are unused there."""
    h = max(1, -(-d // 128))
    while d % h:
        h += 1
    return h


class SubsamplingRunner:
    """ConvSubsampling ('striding', factor 4) on a zero-layer native encoder handle without xscaling:
    cfm_encoder_forward then runs exactly conv.0 + ReLU, conv.2 + ReLU (implicit-GEMM MFMA) and the
    output Linear - the encoder's own front-end kernels (subsampling.py:163-176)."""

    def __init__(self):
        self._handles = {}
        self._versions = {}

    def forward(self, module, x: torch.Tensor, lengths: torch.Tensor, compute: str):
        from .runtime import NativeEncoder, make_cfg
        B, T, F = x.shape
        C = module.conv[0].out_channels
        d = module.out.out_features
        dev = x.device
        key = (dev.index, compute, F, C, d)
        enc = self._handles.get(key)
        if enc is None:
            with torch.cuda.device(dev):
                cfg = make_cfg(F, 0, d, n_heads=_heads_for(d), subsampling_conv_channels=C, xscaling=False)
                enc = NativeEncoder(cfg, device=dev.index, compute=compute)
            self._handles[key] = enc
        sd = module.state_dict(keep_vars=True)
        version = tuple((t.data_ptr(), t._version) for t in sd.values())
        if self._versions.get(key) != version:
            with torch.cuda.device(dev):
                enc.set_weights({"pre_encode." + k: v for k, v in sd.items()})
            self._versions[key] = version
        x_bft = x.detach().transpose(1, 2).to(torch.float32).contiguous()
        y, ylen = enc.forward(x_bft, lengths)
        return y.transpose(1, 2), ylen


SUBSAMPLING = SubsamplingRunner()
