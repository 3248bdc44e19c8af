/*
 * cfm_train.h — backward building blocks of the Conformer layer (libcfm.so), SURVEY §8 row a16.
 *
 * Kernel-level entry points, each the backward of one reference op, tested against torch autograd
 * through the reference modules (tests/golden/bwd_*.npz):
 *   LayerNorm  (conformer_modules.py:73-77 norm_* = nn.LayerNorm(d_model), eps 1e-5)
 *   nn.Linear  (ConformerFeedForward.linear1/2, conformer_modules.py:189-191; attention projections)
 *   Swish      (activations.py:20: x * sigmoid(x))
 *   ConformerConvolution pieces (conformer_modules.py:160-180): GLU + pad mask, depthwise Conv1d,
 *   BatchNorm1d in training mode
 * All tensors are fp32 device pointers; the gradient GEMMs run in `dtype` (CFM_COMPUTE_FP32 or
 * CFM_COMPUTE_BF16 operands, fp32 accumulation).  Weight/bias gradients are deterministic
 * (fixed-order reductions).  Conventions as in cfm_encoder.h.
 */
#ifndef CFM_TRAIN_H_
#define CFM_TRAIN_H_

#include <stddef.h>
#include <stdint.h>

#include "cfm_encoder.h"

#ifdef __cplusplus
extern "C" {
#endif

/* dx (rows, d) = dLN/dx^T dy (+= into dx if accumulate: the residual-stream gradient);
 * dw, db (d) = sum over rows of dy * xhat and dy (NULL to skip). */
size_t cfm_op_layernorm_backward_ws_size(int rows, int d);
cfm_status cfm_op_layernorm_backward(const float* x, int rows, int d, const float* w, const float* dy, float* dx,
                                     int accumulate, float* dw, float* db, void* ws, size_t ws_bytes, void* stream);

/* y = x W^T + b with x (M, K), W (N, K):  dx = dy W (M, K), dw = dy^T x (N, K), db = sum dy (N);
 * any output may be NULL.  K % 4 == 0. */
size_t cfm_op_linear_backward_ws_size(int dtype, int M, int K, int N);
cfm_status cfm_op_linear_backward(int dtype, const float* x, int M, int K, const float* w, int N, const float* dy,
                                  float* dx, float* dw, float* db, void* ws, size_t ws_bytes, void* stream);

/* ---- convolution module (ConformerConvolution.forward, conformer_modules.py:160-180) ---- */
/* GLU(dim=1) + pad-mask backward: pre (B*T', 2d) = pointwise_conv1 output [a | g] (channels-last),
 * dy (B*T', d); frames t >= lens[b] get zero gradient (lens may be NULL).  -> dpre (B*T', 2d). */
cfm_status cfm_op_glu_backward(const float* pre, const float* dy, const int32_t* lens, int B, int Tp, int d, float* dpre,
                               void* stream);
/* Depthwise Conv1d(k=31, pad 15, groups=d) backward on channels-last (B, T', d) tensors; w is the
 * reference (d, 1, K) weight.  dx, dw (d, 1, K), db (d) may each be NULL. */
size_t cfm_op_dwconv_backward_ws_size(int B, int Tp, int d, int K);
cfm_status cfm_op_dwconv_backward(const float* x, const float* w, const float* dy, int B, int Tp, int d, int K,
                                  float* dx, float* dw, float* db, void* ws, size_t ws_bytes, void* stream);
/* BatchNorm1d in training mode over rows = B*T' frames (padded frames included, as the reference):
 * y = xhat * gamma + beta with batch statistics; saves xhat (rows, d), mean, rstd (d); updates
 * run_mean / run_var (momentum, unbiased variance) unless NULL.  Backward from xhat and rstd. */
size_t cfm_op_batchnorm_train_ws_size(int rows, int d);
cfm_status cfm_op_batchnorm_train_forward(const float* x, int rows, int d, const float* gamma, const float* beta,
                                          float momentum, float* run_mean, float* run_var, float* y, float* xhat,
                                          float* mean, float* rstd, void* ws, size_t ws_bytes, void* stream);
cfm_status cfm_op_batchnorm_train_backward(const float* dy, const float* xhat, int rows, int d, const float* gamma,
                                           const float* rstd, float* dx, float* dgamma, float* dbeta, void* ws,
                                           size_t ws_bytes, void* stream);

/* RelPositionMultiHeadAttention backward (multi_head_attention.py:172-210, dropout off), from the
 * same operands as cfm_op_rel_attention (cfm_encoder.h): q, k, v (B*T', H*dk) and p = linear_pos(pos_emb)
 * (2T'-1, H*dk) in the compute type, pos_u / pos_v (H*dk) fp32, pad lengths and context window.
 * dctx (B*T', H*dk) fp32 is the gradient of the attention context (the input of linear_out).
 * Outputs fp32: dq, dkey, dv (B*T', H*dk), dp (2T'-1, H*dk), du, dvb (H*dk; dp/du/dvb may be NULL). */
size_t cfm_op_rel_attention_backward_ws_size(int dtype, int B, int Tp, int H, int dk);
cfm_status cfm_op_rel_attention_backward(int dtype, const void* q, const void* k, const void* v, const void* p,
                                         const float* pos_u, const float* pos_v, const int32_t* lens, int B, int Tp,
                                         int H, int dk, int ctx_left, int ctx_right, const float* dctx, float* dq,
                                         float* dkey, float* dv, float* dp, float* du, float* dvb, void* ws,
                                         size_t ws_bytes, void* stream);

/* dz = du * swish'(z) elementwise (n elements). */
cfm_status cfm_op_swish_backward(const float* z, const float* du, float* dz, int64_t n, void* stream);

/* ---- whole-encoder training step (csrc/train.hip) -------------------------------------------
 * Replaces the autograd graph of ConformerEncoder.forward() in training mode
 * (conformer_encoder.py:236-281 -> ConformerLayer.forward conformer_modules.py:88-121 with
 * nn.Dropout active and BatchNorm1d on batch statistics) and its backward, as driven by
 * EncDecCTCModel.training_step (ctc_models.py:485-514) through Lightning's loss.backward().
 *
 * `params` / `grads` are host arrays of DEVICE pointers with one entry per parameter-table row
 * (cfm_encoder_param_name order, fp32, reference layouts).  Weights are read from `params` on
 * every call (nothing is cached: update them in place between steps freely).  The train forward
 * updates the batch_norm running_mean / running_var entries in place (momentum, unbiased variance,
 * like nn.BatchNorm1d) when opts->update_running_stats != 0.  grads[i] may be NULL (gradient not
 * wanted); non-NULL entries are overwritten (not accumulated); running-stat rows are ignored.
 * An abs_pos handle (cfm_encoder_set_abs_pos) adds the absolute sinusoids before the embedding
 * dropout; its linear_pos / pos_bias_u / pos_bias_v rows must point at zero-filled tensors (pass
 * NULL grads for them): MultiHeadAttention has no such parameters.
 *
 * The tape (caller-owned, cfm_train_tape_size bytes) carries the activations from the forward to
 * the backward; it must be passed unmodified to cfm_train_backward with the same B, T and opts.
 * The workspace (cfm_train_workspace_size) is scratch for either call.  Both calls are
 * stream-ordered and host-sync free.
 *
 * SyncBatchNorm (conformer_ctc_bpe.yaml:175 sync_batchnorm: true): with world > 1 the library calls
 * `allreduce(user, buf, n, stream)` on the host while enqueueing, to SUM n floats at `buf` (device,
 * inside the workspace) over all ranks, stream-ordered on `stream` (e.g. an RCCL all-reduce); every
 * rank must hold the same B and T.  Return 0 on success.
 */
typedef int (*cfm_allreduce_fn)(void* user, float* buf, int64_t n, void* stream);

/* Gradient readiness (data parallelism, SURVEY §8e: the gradient all-reduce overlapped with the
 * backward): when set, cfm_train_backward calls `grad_ready(user, first, n, stream)` on the host
 * right after it has ENQUEUED the last kernel writing the gradients of parameter-table rows
 * [first, first + n) - once per Conformer layer, last layer first, then once for the pre_encode
 * rows.  A collective issued from the callback and ordered after `stream` (e.g. an RCCL all-reduce
 * on a view of those gradients) then overlaps the rest of the backward.  Return 0 on success. */
typedef int (*cfm_grad_ready_fn)(void* user, int first_param, int n_params, void* stream);

typedef struct cfm_train_opts {
  float dropout;               /* ConformerEncoder(dropout=): embedding, FFN inner and residual-branch dropout */
  float dropout_emb;           /* dropout_emb on the positional window (multi_head_attention.py:316)        */
  float dropout_att;           /* dropout_att on the attention probabilities (multi_head_attention.py:111)   */
  float bn_momentum;           /* nn.BatchNorm1d momentum (0.1)                                               */
  int update_running_stats;    /* 1: update running_mean / running_var in place                              */
  int world;                   /* ranks sharing the BatchNorm statistics (1 = plain BatchNorm1d)             */
  uint64_t seed;               /* dropout mask seed; use a fresh one per step                                */
  cfm_allreduce_fn allreduce;  /* required when world > 1                                                    */
  void* allreduce_user;
  cfm_grad_ready_fn grad_ready;  /* optional (NULL): per-layer gradient readiness, backward only              */
  void* grad_ready_user;
} cfm_train_opts;

size_t cfm_train_tape_size(const cfm_encoder* h, int B, int T);
size_t cfm_train_workspace_size(const cfm_encoder* h, int B, int T);
/* x_bft (B, feat_in, T) fp32, len_b (B,) int32 or NULL -> y_bdt (B, d_model, T') fp32, out_len_b (B,) int32 */
cfm_status cfm_train_forward(cfm_encoder* h, const float* const* params, int n_params, const float* x_bft,
                             const int32_t* len_b, int B, int T, const cfm_train_opts* opts, float* y_bdt,
                             int32_t* out_len_b, void* tape, size_t tape_bytes, void* ws, size_t ws_bytes,
                             void* stream);
/* dy_bdt (B, d_model, T') fp32 = dLoss/dy -> grads (see above).  No input gradient (audio_signal
 * is a leaf without grad in every reference training path). */
cfm_status cfm_train_backward(cfm_encoder* h, const float* const* params, int n_params, const float* dy_bdt, int B,
                              int T, const cfm_train_opts* opts, float* const* grads, const void* tape,
                              size_t tape_bytes, void* ws, size_t ws_bytes, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* CFM_TRAIN_H_ */
