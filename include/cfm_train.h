/*
 * cfm_train.h — backward building blocks of the Conformer layer (libcfm.so), SURVEY §8 row a16.
 *
 * Kernel-level entry points, each the backward of one reference op, tested against torch autograd
 * through the reference modules (tests/golden/bwd_*.npz):
 *   LayerNorm  (conformer_modules.py:73-77 norm_* = nn.LayerNorm(d_model), eps 1e-5)
 *   nn.Linear  (ConformerFeedForward.linear1/2, conformer_modules.py:189-191; attention projections)
 *   Swish      (activations.py:20: x * sigmoid(x))
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

/* dz = du * swish'(z) elementwise (n elements). */
cfm_status cfm_op_swish_backward(const float* z, const float* du, float* dz, int64_t n, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* CFM_TRAIN_H_ */
