// Encoder handle layout shared by the forward (encoder.hip) and the training step (train.hip).
// Internal: not part of the C-ABI (include/cfm_encoder.h declares the opaque handle).
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <utility>
#include <vector>

#include "../../include/cfm_encoder.h"
#include "cfm_abi.h"

namespace cfm {
struct LayerW {
  long ff1_w1, ff1_b1, ff1_w2, ff1_b2, ff2_w1, ff2_b1, ff2_w2, ff2_b2;
  long qkv_w, qkv_b, out_w, out_b, uv;   // uv: pos_bias_u | pos_bias_v, [H][dkp] each, zero-padded
  long pw1_w, pw1_b, dw_w, dw_b, bn_mean, bn_inv, bn_w, bn_b, pw2_w, pw2_b;
  long ln_w[5], ln_b[5];   // ff1, self_att, conv, ff2, out
  // LayerNorm-folded copies (cfm_encoder::ln_fold): W' = W * diag(gamma) of norm_self_att (q|k|v),
  // norm_conv (pointwise_conv1, GLU-packed) and norm_feed_forward2 (linear1), with the epilogue's
  // column terms c[n] = sum_k W'[n][k] and d[n] = sum_k beta[k] W[n][k] + bias[n] (fp32, [Npad]).
  long qkv_wf = -1, qkv_lc = -1, qkv_ld = -1;
  long pw1_wf = -1, pw1_lc = -1, pw1_ld = -1;
  long ff2_w1f = -1, ff2_lc = -1, ff2_ld = -1;
};

}  // namespace cfm

struct cfm_encoder {
  cfm_encoder_cfg cfg;
  int device, dtype, es;
  int d, H, dk, dkp, dff, C, F, F1, F2, K, L, dout, vt_rows;
  int bke;                   // K padding granule in elements (GEMM_BK_BYTES / es)
  bool has_out_proj;
  // packed weights (one device allocation)
  char* wbuf = nullptr;
  size_t wbytes = 0;
  bool weights_set = false;
  long conv1_w, conv1_b, conv2_w, conv2_b, sub_w, sub_b, pos_w, outp_w, outp_b;
  std::vector<cfm::LayerW> layers;
  // relative positional table (compute type), rows = 2*max_len - 1
  char* pe = nullptr;
  int max_len = 0;
  // self_attention_model='abs_pos' (cfm_encoder_set_abs_pos): PositionalEncoding adds pe_abs rows
  // 0 .. T'-1 (fp32, max_len x d) to the scaled embedding, and the layers' linear_pos / pos_bias_u /
  // pos_bias_v are packed as zeros, which turns the rel-pos attention into MultiHeadAttention exactly
  bool abs_pos = false;
  float* pe_abs = nullptr;
  // micro-batch concurrency: the batch is split into `microbatches` parts run on their own streams
  int microbatches = 1;
  // enable_pad_mask (conformer_encoder.py:301-305): false -> the conv module's GLU output is not
  // zeroed at padded frames (pad_mask=None, conformer_modules.py:165-166); attention masks stay.
  bool use_pad_mask = true;
  // Eval forward, bf16 mode: norm_self_att / norm_conv / norm_feed_forward2 are folded into the
  // following GEMM (the residual GEMM before each writes the compute-type rows and per-row granule
  // statistics); off in the fp32 parity mode (CFM_LN_FOLD=0/1 overrides for A/B).
  bool ln_fold = false;
  // bf16 eval forward with T' <= 678: pointwise_conv1 + GLU + depthwise conv + BatchNorm + Swish as
  // one launch (gemm_glu_dw); CFM_GLU_DW=0 keeps the two launches (A/B)
  bool fuse_glu_dw = true;
  bool fuse_conv12 = true;     // conv.0 on the matrix cores inside conv.2's implicit GEMM (CFM_CONV12=0: two kernels)
  // bf16 eval forward with the LayerNorm fold, dkp = 64, T' <= 256: each head's q | k | v projection
  // and its attention in one launch (qkv_rel_attention_fused); CFM_QKV_ATTN=0 keeps the QKV GEMM +
  // attention pair (A/B)
  bool fuse_qkv_attn = true;
  std::vector<hipStream_t> sub_streams;
  std::vector<hipEvent_t> sub_events;   // [0] fork, [1 + i] join of part i
  void* zero_page = nullptr;
  std::vector<std::pair<std::string, int64_t>> params;

  template <typename P = char>
  P* w(long off) const { return (P*)(wbuf + off); }
  long kpad(int k) const { return cfm::round_up(k, bke); }
};

