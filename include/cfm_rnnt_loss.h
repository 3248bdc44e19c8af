/*
 * cfm_rnnt_loss.h — C-ABI of the MI355X-native RNN-T loss (libcfm.so), SURVEY §8 row f2: the step
 * after the joint in BASELINE config-4 training.
 *
 * Replaces the arithmetic behind
 *   nemo.collections.asr.losses.rnnt.RNNTLoss.forward()           (losses/rnnt.py:252-306)
 *   RNNTLossNumba / _RNNTNumba.forward()                          (numba/rnnt_loss/rnnt_pytorch.py:36-84, 191-219)
 *   GPURNNT.compute_cost_and_score(): log-softmax denominators,   (numba/rnnt_loss/utils/cuda_utils/gpu_rnnt.py:122-238)
 *     compute_alphas_kernel / compute_betas_kernel /              (gpu_rnnt_kernel.py:66-399)
 *     compute_grad_kernel (FastEmit, clamp), compute_costs_data   (rnnt_helper.py:106-115)
 * acts are the joint's raw logits (B, T, U, V) fp32 (the log-softmax is folded in, as the GPU
 * reference does); costs[b] = -log P(y_b | x_b) * (1 + fastemit_lambda); grads (optional) =
 * d costs[b] / d acts[b], zero outside each utterance's (act_len, label_len + 1) lattice.
 *
 * Conventions as in cfm_encoder.h: device pointers, status codes + cfm_last_error(),
 * stream-ordered (void* = hipStream_t), caller-owned workspace, no host synchronisation.
 */
#ifndef CFM_RNNT_LOSS_H_
#define CFM_RNNT_LOSS_H_

#include <stddef.h>
#include <stdint.h>

#include "cfm_encoder.h"

#ifdef __cplusplus
extern "C" {
#endif

size_t cfm_rnnt_loss_workspace_size(int B, int T, int U);
/* labels (B, labels_ld) int32 (entries past label_lens[b] ignored); act_lens / label_lens (B) int32
 * with act_lens[b] <= T and label_lens[b] + 1 <= U (clamped on device otherwise); clamp <= 0 = off. */
cfm_status cfm_rnnt_loss(const float* acts, const int32_t* labels, int labels_ld, const int32_t* act_lens,
                         const int32_t* label_lens, int B, int T, int U, int V, int blank, float fastemit_lambda,
                         float clamp, float* costs, float* grads, void* workspace, size_t workspace_bytes,
                         void* stream);
/* The gradient in the backward pass instead of the forward.  The reference computes it in the forward and
 * scales it in place by the incoming gradient in the backward (rnnt_pytorch.py:36-84).  Here the forward
 * is cfm_rnnt_loss_costs (costs, plus both lattices kept in `workspace`), and the backward's
 * cfm_rnnt_loss_grad writes grads = g * pre_scale * scale[b] in one pass, with the same fp32 roundings as
 * the multiply-after.  scale: (B) fp32 or NULL (= 1); pre_scale: 1, or the fp32 reciprocal of a mean's
 * divisor.  Saves the backward's full re-read and re-write of the (B, T, U, V) gradient. */
cfm_status cfm_rnnt_loss_costs(const float* acts, const int32_t* labels, int labels_ld, const int32_t* act_lens,
                               const int32_t* label_lens, int B, int T, int U, int V, int blank, float fastemit_lambda,
                               float* costs, void* workspace, size_t workspace_bytes, void* stream);
cfm_status cfm_rnnt_loss_grad(const float* acts, const int32_t* labels, int labels_ld, const int32_t* act_lens,
                              const int32_t* label_lens, int B, int T, int U, int V, int blank, float fastemit_lambda,
                              float clamp, float pre_scale, const float* scale, float* grads, const void* workspace,
                              size_t workspace_bytes, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* CFM_RNNT_LOSS_H_ */
