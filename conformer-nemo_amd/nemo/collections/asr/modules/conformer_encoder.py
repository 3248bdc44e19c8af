"""Drop-in `nemo.collections.asr.modules.ConformerEncoder` backed by the MI355X-native library.

Same constructor kwargs (reference conformer_encoder.py:111-132), same module tree / state_dict keys
(SURVEY §8b), same keyword-only forward contract (:231-234, typecheck) returning
(outputs (B, d_model | feat_out, T') fp32, encoded_lengths (B,) int32).  The forward runs entirely in
libcfm.so (include/cfm_encoder.h): one stream-ordered C call per forward on torch's current stream.

Training mode (`.train()`) runs the native training step (include/cfm_train.h): a train-mode
forward with dropout (embedding, FFN inner, residual branches) and batch-statistics BatchNorm
(SyncBatchNorm across ranks after `set_sync_batchnorm(group)`), differentiable through
torch.autograd — gradients land in each parameter's `.grad`, running stats update in place.

Differences from the reference, by design:
  * training mode requires dropout_att == 0 and dropout_emb == 0 (attention-probability and
    positional-embedding dropout are not built) and conv_norm_type='batch_norm';
  * update_max_seq_length's distributed MAX all_reduce (:283-294) is dropped: it only decides
    whether to regrow the positional table, which is regrown per process on demand instead;
  * compute precision is selectable: 'bf16' (default, MFMA bf16 operands / fp32 accumulation and
    fp32 residual stream) or 'fp32' (exact-fp32 MFMA, the 1e-3 parity mode).  Set with the
    `compute` attribute, `set_compute_mode()`, or the CFM_COMPUTE environment variable.
"""
from __future__ import annotations

import math
import os
from collections import OrderedDict
from typing import Optional

import torch
from torch import nn

from nemo.collections.asr.parts.submodules.conformer_modules import ConformerLayer
from nemo.collections.asr.parts.submodules.multi_head_attention import PositionalEncoding, RelPositionalEncoding
from nemo.collections.asr.parts.submodules.subsampling import ConvSubsampling, calc_length
from nemo.core.classes.common import typecheck
from nemo.core.classes import Exportable
from nemo.core.classes.module import NeuralModule
from nemo.core.neural_types import AcousticEncodedRepresentation, LengthsType, NeuralType, SpectrogramType

# Structural generation: bumped whenever any module registers or replaces a parameter or buffer
# (torch's global registration hooks), and by ConformerEncoder.load_state_dict / _apply.  The
# encoder's cached parameter list is rebuilt only when it changes.
_STRUCT_GEN = [0]


def _bump_struct_gen(*_args):
    _STRUCT_GEN[0] += 1


nn.modules.module.register_module_parameter_registration_hook(_bump_struct_gen)
nn.modules.module.register_module_buffer_registration_hook(_bump_struct_gen)
nn.modules.module.register_module_module_registration_hook(_bump_struct_gen)

__all__ = ["ConformerEncoder"]


class ConformerEncoder(NeuralModule, Exportable):
    def input_example(self, max_batch=1, max_dim=256):
        dev = next(self.parameters()).device
        x = torch.randn(max_batch, self._feat_in, max_dim, device=dev)
        lengths = torch.randint(1, max_dim, (max_batch,), device=dev, dtype=torch.int64)
        return tuple([x, lengths])

    @property
    def input_types(self):
        return OrderedDict({"audio_signal": NeuralType(("B", "D", "T"), SpectrogramType()),
                            "length": NeuralType(tuple("B"), LengthsType())})

    @property
    def output_types(self):
        return OrderedDict({"outputs": NeuralType(("B", "D", "T"), AcousticEncodedRepresentation()),
                            "encoded_lengths": NeuralType(tuple("B"), LengthsType())})

    def __init__(self, feat_in, n_layers, d_model, feat_out=-1, subsampling="striding", subsampling_factor=4,
                 subsampling_conv_channels=-1, ff_expansion_factor=4, self_attention_model="rel_pos", n_heads=4,
                 att_context_size=None, xscaling=True, untie_biases=True, pos_emb_max_len=5000, conv_kernel_size=31,
                 conv_norm_type="batch_norm", dropout=0.1, dropout_emb=0.1, dropout_att=0.0):
        super().__init__()
        if self_attention_model != "rel_pos":
            raise NotImplementedError(f"self_attention_model='{self_attention_model}': only 'rel_pos' is native")
        d_ff = d_model * ff_expansion_factor
        self.d_model = d_model
        self._feat_in = feat_in
        self.scale = math.sqrt(self.d_model)
        self.att_context_size = list(att_context_size) if att_context_size else [-1, -1]
        self.xscale = math.sqrt(d_model) if xscaling else None
        if subsampling_conv_channels == -1:
            subsampling_conv_channels = d_model
        if not (subsampling and subsampling_factor > 1):
            raise NotImplementedError("the native path requires conv subsampling")
        self.pre_encode = ConvSubsampling(subsampling=subsampling, subsampling_factor=subsampling_factor,
                                          feat_in=feat_in, feat_out=d_model, conv_channels=subsampling_conv_channels,
                                          activation=nn.ReLU())
        self._feat_out = d_model
        pos_bias_u = pos_bias_v = None
        if not untie_biases:
            d_head = d_model // n_heads
            pos_bias_u = nn.Parameter(torch.zeros(n_heads, d_head))
            pos_bias_v = nn.Parameter(torch.zeros(n_heads, d_head))
        self.pos_emb_max_len = pos_emb_max_len
        self.pos_enc = RelPositionalEncoding(d_model=d_model, dropout_rate=dropout, max_len=pos_emb_max_len,
                                             xscale=self.xscale, dropout_rate_emb=dropout_emb)
        self.layers = nn.ModuleList([
            ConformerLayer(d_model=d_model, d_ff=d_ff, self_attention_model=self_attention_model, n_heads=n_heads,
                           conv_kernel_size=conv_kernel_size, conv_norm_type=conv_norm_type, dropout=dropout,
                           dropout_att=dropout_att, pos_bias_u=pos_bias_u, pos_bias_v=pos_bias_v)
            for _ in range(n_layers)])
        if feat_out > 0 and feat_out != self._feat_out:
            self.out_proj = nn.Linear(self._feat_out, feat_out)
            self._feat_out = feat_out
        else:
            self.out_proj = None
            self._feat_out = d_model
        self._native_cfg = dict(feat_in=feat_in, n_layers=n_layers, d_model=d_model, feat_out=feat_out,
                                subsampling_factor=subsampling_factor,
                                subsampling_conv_channels=subsampling_conv_channels,
                                ff_expansion_factor=ff_expansion_factor, n_heads=n_heads,
                                att_context_size=self.att_context_size, xscaling=xscaling,
                                pos_emb_max_len=pos_emb_max_len, conv_kernel_size=conv_kernel_size,
                                conv_norm_type=conv_norm_type)
        self.compute = os.environ.get("CFM_COMPUTE", "bf16")
        self._native = {}           # (device, compute) -> NativeEncoder
        self._native_versions = {}  # (device, compute) -> weight version snapshot
        self.max_audio_length = pos_emb_max_len
        self.use_pad_mask = True
        self._dropout, self._dropout_emb, self._dropout_att = float(dropout), float(dropout_emb), float(dropout_att)
        self._trainers = {}         # (device, compute) -> EncoderTrainer
        self._sync_bn_group = None
        self._sync_bn = False

    # ---- reference API ---------------------------------------------------------------------
    def set_max_audio_length(self, max_audio_length):
        """Regrow the relative positional table (conformer_encoder.py:218-229)."""
        self.max_audio_length = max(int(max_audio_length), self.max_audio_length)
        self.pos_enc.extend_pe(self.max_audio_length)
        for enc in self._native.values():
            enc.set_max_audio_length(self.max_audio_length)

    def update_max_seq_length(self, seq_length: int, device=None):
        if seq_length > self.max_audio_length:
            self.set_max_audio_length(seq_length)

    def make_pad_mask(self, max_audio_length, seq_lens):
        return torch.arange(max_audio_length, device=seq_lens.device).expand(seq_lens.size(0), -1) < seq_lens.unsqueeze(-1)

    def enable_pad_mask(self, on=True):
        mask = self.use_pad_mask
        self.use_pad_mask = on
        return mask

    def set_sync_batchnorm(self, group=None):
        """SyncBatchNorm over `group` (torch.distributed; RCCL on ROCm) in training mode."""
        self._sync_bn = True
        self._sync_bn_group = group

    def set_compute_mode(self, compute: str):
        if compute not in ("bf16", "fp32"):
            raise ValueError("compute must be 'bf16' or 'fp32'")
        self.compute = compute

    @staticmethod
    def calc_encoded_length(length):
        return calc_length(length, padding=1, kernel_size=3, stride=2, ceil_mode=False, repeat_num=2)

    # ---- native plumbing -----------------------------------------------------------------------
    def _weight_tensors(self):
        """Name -> tensor of every floating-point parameter / buffer, cached: the state_dict walk
        (~3.4 ms at Large-17) runs only after a structural change (a parameter or buffer registered
        or replaced anywhere, load_state_dict, .to()/.cuda()); each forward then checks only the
        (data_ptr, _version) pairs of the cached tensors (~0.2 ms)."""
        gen = _STRUCT_GEN[0]
        cache = self.__dict__.get("_wcache")
        if cache is None or cache[0] != gen:
            tensors = {k: v for k, v in self.state_dict(keep_vars=True).items() if torch.is_floating_point(v)}
            cache = (gen, tensors, tuple(tensors.values()))
            self.__dict__["_wcache"] = cache
        return cache[1]

    def _weight_version(self):
        self._weight_tensors()
        return tuple((t.data_ptr(), t._version) for t in self.__dict__["_wcache"][2])

    def load_state_dict(self, *args, **kwargs):
        _STRUCT_GEN[0] += 1
        self._native_versions = {}
        return super().load_state_dict(*args, **kwargs)

    def _native_for(self, device: torch.device):
        from conformer_amd import NativeEncoder, make_cfg

        key = (device.index if device.index is not None else torch.cuda.current_device(), self.compute)
        enc = self._native.get(key)
        if enc is None:
            with torch.cuda.device(key[0]):
                enc = NativeEncoder(make_cfg(**self._native_cfg), device=key[0], compute=self.compute)
                if self.max_audio_length > enc.max_audio_length:
                    enc.set_max_audio_length(self.max_audio_length)
            self._native[key] = enc
        tensors = self._weight_tensors()
        version = self._weight_version()
        if self._native_versions.get(key) != version:
            with torch.cuda.device(key[0]):
                enc.set_weights(tensors)
            self._native_versions[key] = version
        return enc

    def _trainer_for(self, device: torch.device):
        from conformer_amd import NativeEncoder, make_cfg
        from conformer_amd.train import EncoderTrainer

        key = (device.index if device.index is not None else torch.cuda.current_device(), self.compute)
        tr = self._trainers.get(key)
        if tr is None:
            with torch.cuda.device(key[0]):
                native = NativeEncoder(make_cfg(**self._native_cfg), device=key[0], compute=self.compute)
                if self.max_audio_length > native.max_audio_length:
                    native.set_max_audio_length(self.max_audio_length)
            tr = EncoderTrainer(native)
            self._trainers[key] = tr
        if self._sync_bn:
            import torch.distributed as dist
            if dist.is_available() and dist.is_initialized() and dist.get_world_size(self._sync_bn_group) > 1:
                tr.set_sync_group(self._sync_bn_group)
        return tr

    def _train_forward(self, audio_signal, length):
        from conformer_amd.train import encoder_train_forward

        if self._dropout_att != 0.0 or self._dropout_emb != 0.0:
            raise NotImplementedError("native training needs dropout_att == 0 and dropout_emb == 0")
        tr = self._trainer_for(audio_signal.device)
        if audio_signal.size(2) > tr.native.max_audio_length:
            tr.native.set_max_audio_length(audio_signal.size(2))
        sd = self.state_dict(keep_vars=True)
        params = [sd[n] for n in tr.names]
        seed = int(torch.randint(0, 2 ** 62, (1,)).item()) if self._dropout > 0 else 0
        y, ylen = encoder_train_forward(tr, audio_signal, length, params, self._dropout, seed, True, 0.1)
        for m in self.modules():   # BatchNorm1d bookkeeping done by the reference module in train mode
            if isinstance(m, nn.BatchNorm1d) and m.num_batches_tracked is not None:
                m.num_batches_tracked.add_(1)
        self._native_versions = {}   # running stats changed in place: repack before the next eval forward
        return y, ylen

    def _apply(self, fn, *args, **kwargs):
        _STRUCT_GEN[0] += 1
        self._native_versions = {}
        return super()._apply(fn, *args, **kwargs)

    # ---- forward ---------------------------------------------------------------------------------
    @typecheck()
    def forward(self, audio_signal, length=None):
        self.update_max_seq_length(seq_length=audio_signal.size(2), device=audio_signal.device)
        return self.forward_for_export(audio_signal=audio_signal, length=length)

    @typecheck()
    def forward_for_export(self, audio_signal, length=None):
        if not audio_signal.is_cuda:
            raise RuntimeError("ConformerEncoder (MI355X-native) expects audio_signal on a ROCm GPU")
        if self.training:
            if not self.use_pad_mask:
                raise NotImplementedError("enable_pad_mask(False) is an inference switch (conformer_encoder.py:301-302); "
                                          "the native training step always applies the pad mask")
            return self._train_forward(audio_signal, length)
        if torch.is_grad_enabled() and audio_signal.requires_grad:
            # eval-mode native forward builds no autograd graph: refuse rather than drop upstream gradients
            raise RuntimeError("ConformerEncoder eval forward does not propagate gradients to audio_signal; "
                               "use .train() for the differentiable native path or torch.no_grad() for inference")
        enc = self._native_for(audio_signal.device)
        enc.set_pad_mask(self.use_pad_mask)
        return enc.forward(audio_signal, length)
