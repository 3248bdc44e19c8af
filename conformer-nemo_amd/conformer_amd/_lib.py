"""ctypes binding of libcfm.so (the C-ABI declared in include/cfm_encoder.h, cfm_ctc.h, cfm_train.h,
cfm_joint.h, cfm_stream.h, cfm_mel.h,
cfm_rnnt_loss.h, cfm_augment.h, cfm_rnnt_decode.h and cfm_comm.h).

The library is built in-tree by `conformer-nemo_amd/csrc/Makefile` (or `__graft_entry__.build()`).
There is deliberately no fallback: if the shared object is missing or fails to load, importing
the native path raises immediately.
"""
from __future__ import annotations

import ctypes
import os
from typing import Dict, Optional

# CFM_LIB_PATH: load another build of the library (same-process A/B timing in tools/)
LIB_PATH = os.environ.get("CFM_LIB_PATH") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libcfm.so")
# the fp16 build (same sources, IEEE fp16 as the 16-bit compute type): compute='fp16'
LIB16_PATH = os.environ.get("CFM_LIB16_PATH") or os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                              "libcfm_f16.so")

CFM_COMPUTE_FP32 = 0
CFM_COMPUTE_BF16 = 1
CFM_COMPUTE_FP16 = 2

STATUS_NAMES = {0: "OK", 1: "INVALID_ARG", 2: "UNSUPPORTED", 3: "HIP", 4: "WORKSPACE", 5: "WEIGHTS", 6: "NOMEM"}

# every symbol include/cfm_encoder.h declares (checked by tests/test_abi.py)
EXPORTED_SYMBOLS = (
    "cfm_last_error", "cfm_version", "cfm_half_mode", "cfm_encoded_length", "cfm_encoder_create", "cfm_encoder_destroy",
    "cfm_encoder_set_weights", "cfm_encoder_param_count", "cfm_encoder_param_name", "cfm_encoder_param_numel",
    "cfm_encoder_set_max_audio_length", "cfm_encoder_set_pad_mask", "cfm_encoder_set_abs_pos", "cfm_encoder_abs_pos", "cfm_encoder_set_microbatches", "cfm_encoder_max_audio_length", "cfm_encoder_workspace_size",
    "cfm_encoder_forward", "cfm_num_stages", "cfm_stage_name", "cfm_encoder_forward_timed", "cfm_stage_clock_overhead", "cfm_op_layernorm", "cfm_op_linear", "cfm_op_linear_pack", "cfm_op_linear_packed", "cfm_op_rel_attention_ws_size",
    "cfm_op_rel_attention", "cfm_bench_gemm", "cfm_encoder_layers_workspace_size", "cfm_encoder_layers_forward",
    "cfm_op_conv_glu_dwconv_ws_size", "cfm_op_conv_glu_dwconv",
)
# every symbol include/cfm_train.h declares
TRAIN_SYMBOLS = (
    "cfm_op_layernorm_backward_ws_size", "cfm_op_layernorm_backward", "cfm_op_linear_backward_ws_size",
    "cfm_op_linear_backward", "cfm_op_swish_backward", "cfm_op_glu_backward", "cfm_op_dwconv_backward_ws_size",
    "cfm_op_dwconv_backward", "cfm_op_batchnorm_train_ws_size", "cfm_op_batchnorm_train_forward",
    "cfm_op_batchnorm_train_backward", "cfm_op_rel_attention_backward_ws_size", "cfm_op_rel_attention_backward",
    "cfm_train_tape_size", "cfm_train_workspace_size", "cfm_train_forward", "cfm_train_backward",
)
# every symbol include/cfm_joint.h declares
JOINT_SYMBOLS = (
    "cfm_rnnt_joint_create", "cfm_rnnt_joint_destroy", "cfm_rnnt_joint_set_weights", "cfm_rnnt_joint_workspace_size",
    "cfm_rnnt_joint_forward", "cfm_rnnt_joint_forward_train", "cfm_rnnt_joint_backward_workspace_size",
    "cfm_rnnt_joint_backward",
)
# every symbol include/cfm_stream.h declares
STREAM_SYMBOLS = ("cfm_frame_buffer_step",)
# every symbol include/cfm_mel.h declares
MEL_SYMBOLS = ("cfm_mel_create", "cfm_mel_destroy", "cfm_mel_set_tables", "cfm_mel_num_frames", "cfm_mel_output_frames",
               "cfm_mel_forward", "cfm_normalize_batch", "cfm_mel_filterbank_slaney")
# every symbol include/cfm_rnnt_loss.h declares
RNNT_LOSS_SYMBOLS = ("cfm_rnnt_loss_workspace_size", "cfm_rnnt_loss", "cfm_rnnt_loss_costs", "cfm_rnnt_loss_grad")
# every symbol include/cfm_augment.h declares
AUGMENT_SYMBOLS = ("cfm_spec_mask_rects", "cfm_spec_shot")
# every symbol include/cfm_rnnt_decode.h declares (bound in conformer_amd/rnnt_decode.py)
RNNT_DECODE_SYMBOLS = ("cfm_rnnt_decoder_create", "cfm_rnnt_decoder_destroy", "cfm_rnnt_decoder_set_weights",
                       "cfm_rnnt_decoder_predict_workspace_size", "cfm_rnnt_decoder_predict",
                       "cfm_rnnt_greedy_workspace_size", "cfm_rnnt_greedy_decode", "cfm_rnnt_decoder_train_tape_size",
                       "cfm_rnnt_decoder_train_forward", "cfm_rnnt_decoder_backward_workspace_size",
                       "cfm_rnnt_decoder_backward")
# every symbol include/cfm_comm.h declares (bound in conformer_amd/comm.py)
COMM_SYMBOLS = ("cfm_comm_get_unique_id", "cfm_comm_init", "cfm_comm_destroy", "cfm_comm_world", "cfm_allreduce_grads",
                "cfm_comm_allreduce_cb", "cfm_grad_buckets_create", "cfm_grad_buckets_ready_cb",
                "cfm_grad_buckets_finish", "cfm_grad_buckets_issued", "cfm_grad_buckets_destroy")
# every symbol include/cfm_cache_stream.h declares (bound in conformer_amd/cache_stream.py)
CACHE_STREAM_SYMBOLS = ("cfm_cache_stream_create", "cfm_cache_stream_destroy", "cfm_cache_stream_reset",
                        "cfm_cache_stream_workspace_size", "cfm_cache_stream_step", "cfm_cache_stream_position")
# every symbol include/cfm_ctc.h declares
CTC_SYMBOLS = (
    "cfm_ctc_head_create", "cfm_ctc_head_destroy", "cfm_ctc_head_set_weights", "cfm_ctc_head_workspace_size",
    "cfm_ctc_head_forward", "cfm_ctc_head_backward", "cfm_ctc_loss_workspace_size", "cfm_ctc_loss",
)


class CfmEncoderCfg(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in (
        "feat_in", "n_layers", "d_model", "feat_out", "subsampling_factor", "subsampling_conv_channels",
        "ff_expansion_factor", "n_heads", "att_context_left", "att_context_right", "xscaling", "pos_emb_max_len",
        "conv_kernel_size", "conv_norm_type")]


class CfmMelCfg(ctypes.Structure):
    _fields_ = [("n_window_size", ctypes.c_int), ("n_window_stride", ctypes.c_int), ("n_fft", ctypes.c_int),
                ("nfilt", ctypes.c_int), ("exact_pad", ctypes.c_int), ("use_preemph", ctypes.c_int),
                ("preemph", ctypes.c_float), ("mag_power", ctypes.c_float), ("log", ctypes.c_int),
                ("log_zero_guard_type", ctypes.c_int), ("log_zero_guard_value", ctypes.c_float),
                ("normalize", ctypes.c_int), ("pad_value", ctypes.c_float), ("pad_to", ctypes.c_int),
                ("max_length", ctypes.c_int)]


class CfmTensorView(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char_p), ("data", ctypes.c_void_p), ("numel", ctypes.c_int64),
                ("on_device", ctypes.c_int)]


class CfmError(RuntimeError):
    pass


_libs: Dict[str, ctypes.CDLL] = {}


ABI_VERSION = 3   # include/cfm_encoder.h CFM_ABI_VERSION: the struct layouts these bindings declare


def variant_of(compute: str) -> str:
    """The library build a compute mode runs in: 'fp16' -> libcfm_f16.so, else libcfm.so."""
    return "fp16" if compute == "fp16" else "bf16"


def load(variant: str = "bf16") -> ctypes.CDLL:
    """Load libcfm.so (variant 'bf16', the default) or libcfm_f16.so ('fp16') once.  torch must be
    imported first so the process shares torch's HIP runtime."""
    lib = _libs.get(variant)
    if lib is not None:
        return lib
    import torch  # noqa: F401  (HIP runtime first: libcfm resolves libamdhip64.so.7 to torch's copy)
    path = LIB16_PATH if variant == "fp16" else LIB_PATH
    if not os.path.exists(path):
        raise CfmError(f"native library not built: {path} (run `make -C conformer-nemo_amd/csrc` "
                       f"or __graft_entry__.build())")
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
    vp, ci, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
    sig = {
        "cfm_last_error": (ctypes.c_char_p, []),
        "cfm_version": (ci, []),
        "cfm_half_mode": (ci, []),
        "cfm_encoded_length": (ci, [ci]),
        "cfm_encoder_create": (ci, [ctypes.POINTER(CfmEncoderCfg), ci, ci, ctypes.POINTER(vp)]),
        "cfm_encoder_destroy": (None, [vp]),
        "cfm_encoder_set_weights": (ci, [vp, ctypes.POINTER(CfmTensorView), ci, vp]),
        "cfm_encoder_param_count": (ci, [vp]),
        "cfm_encoder_param_name": (ctypes.c_char_p, [vp, ci]),
        "cfm_encoder_param_numel": (ctypes.c_int64, [vp, ci]),
        "cfm_encoder_set_max_audio_length": (ci, [vp, ci]),
        "cfm_encoder_max_audio_length": (ci, [vp]),
        "cfm_encoder_set_microbatches": (ci, [vp, ci]),
        "cfm_encoder_set_pad_mask": (ci, [vp, ci]),
        "cfm_encoder_set_abs_pos": (ci, [vp, ci]),
        "cfm_encoder_abs_pos": (ci, [vp]),
        "cfm_encoder_workspace_size": (sz, [vp, ci, ci]),
        "cfm_encoder_forward": (ci, [vp, vp, vp, ci, ci, vp, vp, vp, sz, vp]),
        "cfm_num_stages": (ci, []),
        "cfm_stage_name": (ctypes.c_char_p, [ci]),
        "cfm_stage_clock_overhead": (ci, [vp, ci, ctypes.POINTER(ctypes.c_float)]),
        "cfm_encoder_forward_timed": (ci, [vp, vp, vp, ci, ci, vp, vp, vp, sz, vp, ctypes.POINTER(ctypes.c_float),
                                          ctypes.POINTER(ci)]),
        "cfm_op_layernorm": (ci, [ci, vp, ci, ci, vp, vp, vp, vp, vp]),
        "cfm_encoder_layers_workspace_size": (sz, [vp, ci, ci]),
        "cfm_encoder_layers_forward": (ci, [vp, vp, vp, ci, ci, vp, vp, vp, sz, vp]),
        "cfm_op_conv_glu_dwconv_ws_size": (sz, [ci, ci, ci, ci, ci]),
        "cfm_op_conv_glu_dwconv": (ci, [ci, vp, vp, ci, ci, ci, ci, vp, vp, ci, vp, vp, vp, vp, vp, vp, sz, vp]),
        "cfm_op_linear": (ci, [ci, vp, ci, ci, vp, vp, ci, ci, vp, vp, ctypes.POINTER(sz), vp]),
        "cfm_op_linear_pack": (ci, [ci, vp, vp, ci, ci, vp, ctypes.POINTER(sz), vp]),
        "cfm_op_linear_packed": (ci, [ci, vp, ci, ci, vp, ci, ci, vp, vp]),
        "cfm_op_rel_attention_ws_size": (sz, [ci, ci, ci, ci, ci]),
        "cfm_bench_gemm": (ci, [ci, ci, ci, ci, ci, ci, ci, ctypes.POINTER(ctypes.c_float)]),
        "cfm_op_rel_attention": (ci, [ci, vp, vp, vp, vp, vp, vp, vp, ci, ci, ci, ci, ci, ci, vp, vp, vp]),
        "cfm_op_layernorm_backward_ws_size": (sz, [ci, ci]),
        "cfm_op_layernorm_backward": (ci, [vp, ci, ci, vp, vp, vp, ci, vp, vp, vp, sz, vp]),
        "cfm_op_linear_backward_ws_size": (sz, [ci, ci, ci, ci]),
        "cfm_op_linear_backward": (ci, [ci, vp, ci, ci, vp, ci, vp, vp, vp, vp, vp, sz, vp]),
        "cfm_op_swish_backward": (ci, [vp, vp, vp, ctypes.c_int64, vp]),
        "cfm_op_glu_backward": (ci, [vp, vp, vp, ci, ci, ci, vp, vp]),
        "cfm_op_dwconv_backward_ws_size": (sz, [ci, ci, ci, ci]),
        "cfm_op_dwconv_backward": (ci, [vp, vp, vp, ci, ci, ci, ci, vp, vp, vp, vp, sz, vp]),
        "cfm_op_batchnorm_train_ws_size": (sz, [ci, ci]),
        "cfm_op_batchnorm_train_forward": (ci, [vp, ci, ci, vp, vp, ctypes.c_float, vp, vp, vp, vp, vp, vp, vp, sz, vp]),
        "cfm_op_batchnorm_train_backward": (ci, [vp, vp, ci, ci, vp, vp, vp, vp, vp, vp, sz, vp]),
        "cfm_op_rel_attention_backward_ws_size": (sz, [ci, ci, ci, ci, ci]),
        "cfm_op_rel_attention_backward": (ci, [ci, vp, vp, vp, vp, vp, vp, vp, ci, ci, ci, ci, ci, ci, vp, vp, vp, vp,
                                               vp, vp, vp, vp, sz, vp]),
        "cfm_rnnt_joint_create": (ci, [ci, ci, ci, ci, ci, ci, ci, ctypes.POINTER(vp)]),
        "cfm_rnnt_joint_destroy": (None, [vp]),
        "cfm_rnnt_joint_set_weights": (ci, [vp, vp, vp, vp, vp, vp, vp, vp]),
        "cfm_rnnt_joint_workspace_size": (sz, [vp, ci, ci, ci]),
        "cfm_rnnt_joint_forward": (ci, [vp, vp, vp, ci, ci, ci, ci, vp, vp, sz, vp]),
        "cfm_rnnt_joint_forward_train": (ci, [vp, vp, vp, ci, ci, ci, ctypes.c_float, ctypes.c_uint64, vp, vp, sz, vp]),
        "cfm_rnnt_joint_backward_workspace_size": (sz, [vp, ci, ci, ci]),
        "cfm_rnnt_joint_backward": (ci, [vp, vp, vp, ci, ci, ci, ctypes.c_float, ctypes.c_uint64, vp, vp, vp, vp, vp, vp,
                                         vp, vp, vp, vp, vp, vp, vp, sz, vp]),
        "cfm_frame_buffer_step": (ci, [vp, vp, vp, ci, ci, ci, ci, ci, ctypes.c_float, vp, vp]),
        "cfm_mel_create": (ci, [ctypes.POINTER(CfmMelCfg), ci, ctypes.POINTER(vp)]),
        "cfm_mel_destroy": (None, [vp]),
        "cfm_mel_set_tables": (ci, [vp, vp, vp, vp]),
        "cfm_mel_num_frames": (ctypes.c_long, [vp, ctypes.c_long]),
        "cfm_mel_output_frames": (ctypes.c_long, [vp, ctypes.c_long]),
        "cfm_mel_forward": (ci, [vp, vp, vp, ci, ctypes.c_long, ctypes.c_float, ctypes.c_uint64, vp, ci, vp, vp, vp]),
        "cfm_normalize_batch": (ci, [vp, vp, ci, ci, ci, ci, vp, vp]),
        "cfm_mel_filterbank_slaney": (ci, [ci, ci, ci, ctypes.c_double, ctypes.c_double, ci, ci,
                                           ctypes.POINTER(ctypes.c_float)]),
        "cfm_rnnt_loss_workspace_size": (sz, [ci, ci, ci]),
        "cfm_rnnt_loss": (ci, [vp, vp, ci, vp, vp, ci, ci, ci, ci, ci, ctypes.c_float, ctypes.c_float, vp, vp, vp, sz,
                               vp]),
        "cfm_rnnt_loss_costs": (ci, [vp, vp, ci, vp, vp, ci, ci, ci, ci, ci, ctypes.c_float, vp, vp, sz, vp]),
        "cfm_rnnt_loss_grad": (ci, [vp, vp, ci, vp, vp, ci, ci, ci, ci, ci, ctypes.c_float, ctypes.c_float,
                                    ctypes.c_float, vp, vp, vp, sz, vp]),
        "cfm_spec_mask_rects": (ci, [vp, ci, ci, ci, vp, ci, ctypes.c_float, vp]),
        "cfm_spec_shot": (ci, [vp, vp, ctypes.c_int64, ctypes.c_float, ctypes.c_uint64, vp]),
        "cfm_ctc_head_create": (ci, [ci, ci, ci, ci, ctypes.POINTER(vp)]),
        "cfm_ctc_head_destroy": (None, [vp]),
        "cfm_ctc_head_set_weights": (ci, [vp, vp, vp, vp]),
        "cfm_ctc_head_workspace_size": (sz, [vp, ci, ci]),
        "cfm_ctc_head_forward": (ci, [vp, vp, ci, ci, vp, vp, vp, sz, vp]),
        "cfm_ctc_head_backward": (ci, [vp, vp, ci, ci, vp, vp, vp, vp, vp, vp, sz, vp]),
        "cfm_ctc_loss_workspace_size": (sz, [ci, ci, ci, ci]),
        "cfm_ctc_loss": (ci, [vp, vp, vp, vp, ci, ci, ci, ci, ci, ci, ctypes.c_float, vp, vp, vp, sz, vp]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.cfm_version() != ABI_VERSION:
        raise CfmError(f"{path}: ABI version {lib.cfm_version()}, these bindings expect {ABI_VERSION} "
                       f"(include/cfm_encoder.h CFM_ABI_VERSION): rebuild the library")
    want = CFM_COMPUTE_FP16 if variant == "fp16" else CFM_COMPUTE_BF16
    if lib.cfm_half_mode() != want:
        raise CfmError(f"{path}: 16-bit compute mode {lib.cfm_half_mode()}, expected {want}")
    _libs[variant] = lib
    return lib


def check(status: int, what: str = "", lib: Optional[ctypes.CDLL] = None) -> None:
    """Raise CfmError for a non-OK status; the message is the failing library's cfm_last_error (`lib`,
    default libcfm.so: each build keeps its own)."""
    if status != 0:
        msg = (lib or load()).cfm_last_error().decode(errors="replace")
        raise CfmError(f"{what}: {STATUS_NAMES.get(status, status)}: {msg}")
