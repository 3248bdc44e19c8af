/*
 * cfm_ctc.h — C-ABI of the MI355X-native CTC head and CTC loss (libcfm.so), SURVEY §8 row a17.
 *
 * Replaces the arithmetic behind
 *   nemo.collections.asr.modules.ConvASRDecoder.forward()      (conv_asr.py:442-444:
 *       log_softmax(Conv1d(feat_in, num_classes + 1, k=1)(encoder_output).transpose(1, 2), -1))
 *   EncDecCTCModel.forward greedy predictions                  (ctc_models.py:594: argmax over classes)
 *   nemo.collections.asr.losses.ctc.CTCLoss.forward()          (ctc.py:56-70 over
 *       torch.nn.functional.ctc_loss, blank = num_classes, reduction 'mean_batch' = mean of the
 *       per-utterance losses; EncDecCTCModel builds it with zero_infinity=True, ctc_models.py:190-194)
 * and their backward passes (the training step of BASELINE config 3).
 *
 * Conventions as in cfm_encoder.h: device pointers, fp32 tensors, int32 lengths/labels, status codes
 * with cfm_last_error(), stream-ordered (void* = hipStream_t), caller-owned workspace.
 */
#ifndef CFM_CTC_H_
#define CFM_CTC_H_

#include <stddef.h>
#include <stdint.h>

#include "cfm_encoder.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct cfm_ctc_head cfm_ctc_head;

/* num_classes = vocabulary size + 1 (the blank is the last class, conv_asr.py:431). */
cfm_status cfm_ctc_head_create(int feat_in, int num_classes, int device, int compute_mode, cfm_ctc_head** out);
void cfm_ctc_head_destroy(cfm_ctc_head* h);
/* weight (num_classes, feat_in) [the Conv1d (C, D, 1) weight], bias (num_classes): device fp32.
 * Packs private copies (W and W^T in the compute type) on `stream`; call again after an update.
 * Stream-ordered (no host synchronisation): the sources must stay valid until `stream` reaches the call. */
cfm_status cfm_ctc_head_set_weights(cfm_ctc_head* h, const float* weight, const float* bias, void* stream);
size_t cfm_ctc_head_workspace_size(const cfm_ctc_head* h, int B, int T);

/* enc_bdt (B, feat_in, T) -> logprobs_btc (B, T, num_classes); greedy_bt (B, T) argmax or NULL. */
cfm_status cfm_ctc_head_forward(cfm_ctc_head* h, const float* enc_bdt, int B, int T, float* logprobs_btc,
                                int32_t* greedy_bt, void* workspace, size_t workspace_bytes, void* stream);

/* Backward of log_softmax(Conv1d(enc)): grad_lp_btc = dL/dlogprobs (B, T, C) ->
 *   grad_enc_bdt (B, feat_in, T), grad_weight (C, feat_in), grad_bias (C)  (each may be NULL).
 * logprobs_btc is the forward output.  Overwrites (does not accumulate). */
cfm_status cfm_ctc_head_backward(cfm_ctc_head* h, const float* enc_bdt, int B, int T, const float* logprobs_btc,
                                 const float* grad_lp_btc, float* grad_enc_bdt, float* grad_weight, float* grad_bias,
                                 void* workspace, size_t workspace_bytes, void* stream);

/* CTC loss (torch.nn.functional.ctc_loss semantics, reduction 'none'):
 *   logprobs_btc (B, T, C) log-softmax outputs, targets_bu (B, U) padded labels in [0, C) \ {blank},
 *   input_lengths (B) <= T, target_lengths (B) <= U.
 *   nll_b (B): -log p(target | input), 0 where infinite if zero_infinity.
 *   grad_btc (B, T, C) or NULL: grad_scale * d nll_b / d logprobs in torch's convention
 *   (exp(lp) - posterior, 0 beyond input_lengths and for zero_infinity'd utterances).  For the
 *   reference's 'mean_batch' reduction pass grad_scale = 1/B and average nll_b.
 * Supports 2*U+1 <= 1024 extended states. */
size_t cfm_ctc_loss_workspace_size(int B, int T, int C, int U);
cfm_status cfm_ctc_loss(const float* logprobs_btc, const int32_t* targets_bu, const int32_t* input_lengths,
                        const int32_t* target_lengths, int B, int T, int C, int U, int blank, int zero_infinity,
                        float grad_scale, float* nll_b, float* grad_btc, void* workspace, size_t workspace_bytes,
                        void* stream);

#ifdef __cplusplus
}
#endif
#endif /* CFM_CTC_H_ */
