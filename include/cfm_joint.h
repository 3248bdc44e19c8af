/*
 * cfm_joint.h — C-ABI of the MI355X-native RNN-T joint network (libcfm.so), SURVEY §8 row a-ext4
 * (BASELINE config 4: Conformer-Transducer encoder + joint).
 *
 * Replaces the arithmetic behind
 *   nemo.collections.asr.modules.RNNTJoint.forward()   (rnnt.py:793-815, non-fused path)
 *   RNNTJoint.joint()                                   (rnnt.py:951-1008):
 *       out[b,t,u,:] = W_out . act(W_enc f[b,t] + b_enc + W_pred g[b,u] + b_pred) + b_out
 *       with act in {relu, sigmoid, tanh} (rnnt.py:1010-1038), dropout = identity (eval), and
 *       log_softmax over the classes only when requested (log_softmax=None on a GPU returns logits).
 *
 * Conventions as in cfm_encoder.h: device pointers, fp32 tensors, status codes + cfm_last_error(),
 * stream-ordered (void* = hipStream_t), caller-owned workspace, no host synchronisation.
 */
#ifndef CFM_JOINT_H_
#define CFM_JOINT_H_

#include <stddef.h>
#include <stdint.h>

#include "cfm_encoder.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct cfm_rnnt_joint cfm_rnnt_joint;

#define CFM_JOINT_RELU 0
#define CFM_JOINT_SIGMOID 1
#define CFM_JOINT_TANH 2

/* num_classes = vocabulary + 1 (blank last, rnnt.py:729). */
cfm_status cfm_rnnt_joint_create(int encoder_hidden, int pred_hidden, int joint_hidden, int num_classes,
                                 int activation, int device, int compute_mode, cfm_rnnt_joint** out);
void cfm_rnnt_joint_destroy(cfm_rnnt_joint* h);
/* Reference parameters (device fp32): enc.weight (H, H1), enc.bias (H), pred.weight (H, H2),
 * pred.bias (H), joint_net[-1].weight (C, H), joint_net[-1].bias (C).  Packs private copies. */
cfm_status cfm_rnnt_joint_set_weights(cfm_rnnt_joint* h, const float* w_enc, const float* b_enc, const float* w_pred,
                                      const float* b_pred, const float* w_out, const float* b_out, void* stream);
size_t cfm_rnnt_joint_workspace_size(const cfm_rnnt_joint* h, int B, int T, int U);
/* enc_bdt (B, H1, T), dec_bdu (B, H2, U) -> out (B, T, U, num_classes) fp32 (logits, or log-probs
 * when log_softmax != 0). */
cfm_status cfm_rnnt_joint_forward(cfm_rnnt_joint* h, const float* enc_bdt, const float* dec_bdu, int B, int T, int U,
                                  int log_softmax, float* out, void* workspace, size_t workspace_bytes, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* CFM_JOINT_H_ */
