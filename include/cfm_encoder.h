/*
 * cfm_encoder.h — C-ABI of the MI355X-native Conformer encoder forward (libcfm.so).
 *
 * Drop-in boundary: this library replaces the arithmetic behind
 *   nemo.collections.asr.modules.ConformerEncoder.forward()        (conformer_encoder.py:231-234)
 *   ConformerEncoder.forward_for_export()                          (conformer_encoder.py:236-281)
 * of the reference (nghiahuynh-ai/Conformer-NeMo, a NeMo 1.8.2 fork).  The reference has no native
 * code on this path; its only "FFI" is the Python plugin contract (yaml `_target_` ->
 * ConformerEncoder(**kwargs), keyword-only forward(audio_signal=, length=)).  The Python mirror in
 * conformer-nemo_amd/nemo/collections/asr/modules/conformer_encoder.py binds these entry points
 * with ctypes.
 *
 * Conventions
 *   - Plain pointers and sizes only; no torch types.  All tensor pointers passed to
 *     cfm_encoder_forward are DEVICE pointers; `stream` is a hipStream_t passed as void*.
 *   - Every call returns cfm_status; on failure cfm_last_error() returns a thread-local message.
 *     No C++ exception crosses the ABI.
 *   - cfm_encoder_forward is stream-ordered and host-sync free (graph-capturable): it allocates
 *     nothing; all scratch lives in the caller-owned workspace.
 *   - Threading: one handle per device; concurrent calls on distinct handles are safe.
 */
#ifndef CFM_ENCODER_H_
#define CFM_ENCODER_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef int cfm_status;
#define CFM_OK 0
#define CFM_ERR_INVALID_ARG 1
#define CFM_ERR_UNSUPPORTED 2
#define CFM_ERR_HIP 3
#define CFM_ERR_WORKSPACE 4
#define CFM_ERR_WEIGHTS 5
#define CFM_ERR_NOMEM 6

/* Compute modes.  FP32: every contraction on v_mfma_f32_32x32x2_f32 (exact fp32 products).
 * BF16: operands in bf16 on v_mfma_f32_32x32x16_bf16 with fp32 accumulation, fp32 residual stream /
 * norms / softmax — the performance mode (libcfm.so).  FP16: the same kernels with IEEE fp16
 * operands on v_mfma_f32_32x32x16_f16 at the same rate (3 more mantissa bits: within the north-star
 * 1e-3 relative gate where bf16 is not), from libcfm_f16.so — the same sources built with the other
 * 16-bit format; inference only (its training entries refuse the 16-bit mode).  A library accepts
 * FP32 and its own 16-bit mode (cfm_half_mode()); every other entry point's `dtype` /
 * compute-mode argument that is not CFM_COMPUTE_FP32 means that 16-bit mode. */
#define CFM_COMPUTE_FP32 0
#define CFM_COMPUTE_BF16 1
#define CFM_COMPUTE_FP16 2

/* Constructor arguments of ConformerEncoder.__init__ (conformer_encoder.py:111-132).
 * Eval-mode forward only: dropout / dropout_emb / dropout_att are identities and are not passed. */
typedef struct cfm_encoder_cfg {
  int feat_in;                   /* feat_in (80)                                     */
  int n_layers;                  /* n_layers                                         */
  int d_model;                   /* d_model                                          */
  int feat_out;                  /* feat_out (-1: none)  -> out_proj if >0 and != d  */
  int subsampling_factor;        /* must be 4 ('striding', 2 x Conv2d s2)            */
  int subsampling_conv_channels; /* -1 -> d_model                                    */
  int ff_expansion_factor;       /* d_ff = d_model * ff_expansion_factor             */
  int n_heads;                   /* n_heads (self_attention_model must be 'rel_pos') */
  int att_context_left;          /* att_context_size[0] (-1 = unlimited)             */
  int att_context_right;         /* att_context_size[1] (-1 = unlimited)             */
  int xscaling;                  /* 1: x *= sqrt(d_model) (conformer_encoder.py:144) */
  int pos_emb_max_len;           /* pos_emb_max_len (5000)                           */
  int conv_kernel_size;          /* conv_kernel_size (31), odd                       */
  int conv_norm_type;            /* 0 = batch_norm, 1 = layer_norm                   */
} cfm_encoder_cfg;

/* One named fp32 tensor of the reference state_dict (keys as in SURVEY §8b, without the
 * `encoder.` prefix).  `on_device` = 1 for device pointers, 0 for host pointers. */
typedef struct cfm_tensor_view {
  const char* name;
  const float* data;
  int64_t numel;
  int on_device;
} cfm_tensor_view;

typedef struct cfm_encoder cfm_encoder;

const char* cfm_last_error(void);
/* ABI revision of every cfm_*.h struct and entry point.  A host checks it against the value it was
 * built with before passing any struct:
 *   1  round 1;
 *   2  cfm_train_opts (cfm_train.h) gained grad_ready / grad_ready_user, and dropout_emb / dropout_att
 *      became active (an older host's shorter struct would leave the callback pointer unset);
 *   3  the *_set_weights of cfm_ctc.h / cfm_joint.h / cfm_rnnt_decode.h are stream-ordered (they no
 *      longer synchronise the stream: a host must keep the sources valid until the stream passes the
 *      call); new entry points cfm_encoder_layers_forward, cfm_op_conv_glu_dwconv,
 *      cfm_encoder_set_abs_pos, cfm_half_mode (and the fp16 build libcfm_f16.so), the transducer
 *      training entries of cfm_joint.h / cfm_rnnt_decode.h. */
#define CFM_ABI_VERSION 3
int cfm_version(void);
/* This library's 16-bit compute mode: CFM_COMPUTE_BF16 (libcfm.so) or CFM_COMPUTE_FP16 (libcfm_f16.so). */
int cfm_half_mode(void);

/* calc_length (subsampling.py:272-282) on the host: encoder frames for `len` input frames. */
int cfm_encoded_length(int len);

cfm_status cfm_encoder_create(const cfm_encoder_cfg* cfg, int device, int compute_mode, cfm_encoder** out);
void cfm_encoder_destroy(cfm_encoder* h);

/* Copy + pack every parameter / buffer of the reference state_dict.  All keys listed by
 * cfm_encoder_param_count/cfm_encoder_param_name must be present (num_batches_tracked is optional).
 * May allocate and synchronises `stream`.  Call again whenever the weights change. */
cfm_status cfm_encoder_set_weights(cfm_encoder* h, const cfm_tensor_view* table, int n, void* stream);
int cfm_encoder_param_count(const cfm_encoder* h);
const char* cfm_encoder_param_name(const cfm_encoder* h, int i);
int64_t cfm_encoder_param_numel(const cfm_encoder* h, int i);

/* set_max_audio_length (conformer_encoder.py:218-229): regrow the relative positional table so
 * inputs of up to `max_audio_length` frames are accepted.  Allocates; not stream-ordered. */
cfm_status cfm_encoder_set_max_audio_length(cfm_encoder* h, int max_audio_length);
int cfm_encoder_max_audio_length(const cfm_encoder* h);

/* enable_pad_mask (conformer_encoder.py:301-305): on = 0 runs the layers with pad_mask = None, i.e.
 * the convolution module does not zero padded frames after the GLU (conformer_modules.py:165-166);
 * the attention mask is unchanged.  Default on. */
cfm_status cfm_encoder_set_pad_mask(cfm_encoder* h, int on);

/* self_attention_model='abs_pos' (conformer_encoder.py:184-189, conformer_modules.py:73-74, 106-107):
 * on = 1 adds PositionalEncoding's absolute sinusoids (positions 0 .. T'-1, fp32,
 * multi_head_attention.py:235-271) after the xscale, in the forward and the training step, and the
 * layers attend with MultiHeadAttention (multi_head_attention.py:94-129): the linear_pos /
 * pos_bias_u / pos_bias_v entries become optional in set_weights and are packed as zeros whatever
 * is passed (the rel-pos scores then reduce exactly to q.k / sqrt(d_k)).  Clears the weights: call
 * set_weights after it.  Not stream-ordered (synchronises the device).  Default off (rel_pos).
 * cfm_cache_stream_create refuses an abs_pos handle. */
cfm_status cfm_encoder_set_abs_pos(cfm_encoder* h, int on);
int cfm_encoder_abs_pos(const cfm_encoder* h);

/* Micro-batch concurrency (default 1, env CFM_MICROBATCH): the batch is split into up to n parts
 * (each >= 4 utterances) that run on library-owned streams forked from / joined into `stream`.
 * Outputs are bitwise identical for any n. */
cfm_status cfm_encoder_set_microbatches(cfm_encoder* h, int n);

/* Bytes of caller-owned device workspace needed by cfm_encoder_forward for (B, T). */
size_t cfm_encoder_workspace_size(const cfm_encoder* h, int B, int T);

/* forward_for_export (conformer_encoder.py:236-281), eval mode.
 *   x_bft      (B, feat_in, T) fp32, device
 *   len_b      (B,) int32 device, or NULL (every utterance has T frames: conformer_encoder.py:243-246)
 *   y_bdt      (B, feat_out or d_model, T') fp32 device, T' = cfm_encoded_length(T)
 *   out_len_b  (B,) int32 device: encoded lengths
 * Requires T <= cfm_encoder_max_audio_length(h). */
cfm_status cfm_encoder_forward(cfm_encoder* h, const float* x_bft, const int32_t* len_b, int B, int T, float* y_bdt,
                               int32_t* out_len_b, void* workspace, size_t workspace_bytes, void* stream);

/* The ConformerLayer stack alone (ConformerLayer.forward, conformer_modules.py:88-121, applied for
 * every layer of the handle as ConformerEncoder.forward_for_export :262-271 does): x_btd (B, T', d) fp32
 * is layer 0's input (after the positional encoding's xscale), y_btd (B, T', d) fp32 the last layer's
 * norm_out.  len_b (B) int32 valid frames per utterance (the pad and attention masks, as in the
 * encoder; NULL = all T'); pos_emb (2T'-1, d) fp32 relative positions T'-1 ... -(T'-1) as
 * RelPositionalEncoding.forward returns them (NULL = the handle's own table).  Stream-ordered;
 * workspace of cfm_encoder_layers_workspace_size bytes.  The subsampling weights are not used. */
size_t cfm_encoder_layers_workspace_size(const cfm_encoder* h, int B, int Tp);
cfm_status cfm_encoder_layers_forward(cfm_encoder* h, const float* x_btd, const int32_t* len_b, int B, int Tp,
                                      const float* pos_emb, float* y_btd, void* workspace, size_t workspace_bytes,
                                      void* stream);

/* Per-stage kernel timing on `stream` (single stream, no micro-batch split): one production forward
 * in which every kernel carries a start and a stop event in its own dispatch packet; each kernel's
 * begin -> end time (what rocprofv3's kernel trace reports) is ADDED into stage_ms[stage] and
 * stage_launches[stage] += kernels per forward.  The outputs are the forward's.  Synchronises; not
 * graph-capturable; used for the per-kernel roofline in bench.py.  CFM_STAGE_CLOCK=chain: stop events
 * only, a kernel's time = its stop - the previous stop (adds the dispatch gap and the event overhead);
 * =burst: every launch replayed 8x between two stream events (outputs then not the forward's). */
int cfm_num_stages(void);
const char* cfm_stage_name(int i);
cfm_status cfm_encoder_forward_timed(cfm_encoder* h, const float* x_bft, const int32_t* len_b, int B, int T,
                                     float* y_bdt, int32_t* out_len_b, void* workspace, size_t workspace_bytes,
                                     void* stream, float* stage_ms, int* stage_launches);
/* The stage clock's own cost: n empty one-wave kernels timed exactly as forward_timed times a kernel
 * (same CFM_STAGE_CLOCK mode); *us_per_kernel = their mean begin -> end (us).  Synchronises. */
cfm_status cfm_stage_clock_overhead(void* stream, int n, float* us_per_kernel);

/* ---- kernel-level entry points (used by the per-kernel parity tests) ---------------------- */
/* All buffers are device pointers; `dtype` is CFM_COMPUTE_FP32 (float) or CFM_COMPUTE_BF16 (uint16 bf16). */

/* y = LayerNorm(x) (eps 1e-5) rows x d fp32 -> compute type (and optionally fp32 in y_f32). */
cfm_status cfm_op_layernorm(int dtype, const float* x, int rows, int d, const float* w, const float* b, float* y_f32,
                            void* y_t, void* stream);
/* y[M,N] = x[M,K] . w[N,K]^T + bias (fp32 weights, packed internally into `pack_ws`).
 * act: 0 none, 1 relu, 2 swish.  Returns the pack workspace size when pack_ws == NULL.
 * Equivalent to cfm_op_linear_pack followed by cfm_op_linear_packed (nn.Linear.forward, used by the
 * ConformerFeedForward / MultiHeadAttention projections run standalone, conformer_modules.py:195-200,
 * multi_head_attention.py:71-75, 115). */
cfm_status cfm_op_linear(int dtype, const void* x, int M, int K, const float* w, const float* bias, int N, int act,
                         void* y, void* pack_ws, size_t* pack_ws_bytes, void* stream);
/* Pack w (N, K) fp32 and bias (N, or NULL) into pack_ws on the device, ordered on `stream` (no host
 * synchronisation): pack_ws == NULL returns its size in *pack_ws_bytes.  A packed buffer stays valid
 * for every later cfm_op_linear_packed call until the weights change (cache it per weight version). */
cfm_status cfm_op_linear_pack(int dtype, const float* w, const float* bias, int N, int K, void* pack_ws,
                              size_t* pack_ws_bytes, void* stream);
/* y[M,N] = x[M,K] . W^T + bias (+ act) from a cfm_op_linear_pack buffer of the same dtype, N, K. */
cfm_status cfm_op_linear_packed(int dtype, const void* x, int M, int K, const void* pack_ws, int N, int act, void* y,
                                void* stream);
/* Fused rel-pos attention core on projected q,k,v (M = B*T' rows, d = H*dk, compute type):
 * out[M, d] = softmax_mask(((q+u)k^T + rel_shift((q+v)p^T)) / sqrt(dk)) v, p = pos projection
 * rows (2T'-1, d).  Scratch `ws` of cfm_op_rel_attention_ws_size bytes. */
size_t cfm_op_rel_attention_ws_size(int dtype, int B, int Tp, int H, int dk);
cfm_status cfm_op_rel_attention(int dtype, const void* q, const void* k, const void* v, const void* p,
                                const float* pos_u, const float* pos_v, const int32_t* lens, int B, int Tp, int H,
                                int dk, int ctx_left, int ctx_right, void* out, void* ws, void* stream);

/* ConformerConvolution between its pointwise convolutions (conformer_modules.py:164-176): pre (B*T', 2d)
 * compute type = pointwise_conv1's output [a | gate] -> GLU -> pad mask (frames t >= lens[b] zeroed;
 * lens NULL = no mask) -> depthwise conv (k = K, zero padding (K-1)/2; dw_w (d, 1, K), dw_b (d), fp32) ->
 * norm_type 0: BatchNorm1d with running statistics (eps 1e-5) | 1: LayerNorm(d) -> Swish -> out (B*T', d)
 * compute type.  Synchronises the stream (host-side weight relayout).  Scratch of
 * cfm_op_conv_glu_dwconv_ws_size bytes. */
size_t cfm_op_conv_glu_dwconv_ws_size(int dtype, int B, int Tp, int d, int K);
cfm_status cfm_op_conv_glu_dwconv(int dtype, const void* pre, const int32_t* lens, int B, int Tp, int d, int K,
                                  const float* dw_w, const float* dw_b, int norm_type, const float* norm_w,
                                  const float* norm_b, const float* bn_mean, const float* bn_var, void* out, void* ws,
                                  size_t ws_bytes, void* stream);

/* GEMM microbenchmark on synthetic data: average device ms of `iters` launches of the encoder's
 * GEMM (M x N x K, epilogue id as in csrc/cfm_kernels.h, tile -1 = automatic choice).  Allocates. */
cfm_status cfm_bench_gemm(int dtype, int tile, int epilogue, int M, int N, int K, int iters, float* avg_ms);

#ifdef __cplusplus
}
#endif
#endif /* CFM_ENCODER_H_ */
