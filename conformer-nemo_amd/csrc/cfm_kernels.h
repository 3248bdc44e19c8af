// Internal launcher interface between the encoder orchestration (encoder.hip) and the kernels.
// Not part of the public C-ABI (that is include/cfm_encoder.h).
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cfm {

// Kernel clock for cfm_encoder_forward_timed.  When installed on the calling thread, every launch
// goes through it:
//   * packet mode (default): each kernel carries a start AND a stop event in its own dispatch packet
//     (hipExtLaunchKernel); a kernel's time is the packet's begin -> end timestamps, the duration
//     rocprofv3's kernel trace reports (no dispatch gap), measured inside a normal forward;
//   * chain mode: a stop event only; a kernel's time is the gap between its stop and the previous
//     kernel's stop on the stream (its execution + the dispatch gap + the event's own overhead);
//   * burst mode: each launch is replayed reps() times back-to-back between two stream events
//     (steady state, warm caches); the timed call's outputs are then not the forward's.
struct KernelClock {
  virtual int reps() = 0;
  virtual void begin(hipStream_t st) = 0;
  virtual hipEvent_t stop_event() = 0;
  virtual hipEvent_t start_event() { return nullptr; }
  virtual void end(hipStream_t st) = 0;
  virtual ~KernelClock() = default;
};
extern thread_local KernelClock* g_kclock;

template <typename F, typename... Args>
inline void cfm_launch(F kernel, dim3 grid, dim3 block, uint32_t lds_bytes, hipStream_t st, Args... args) {
  KernelClock* c = g_kclock;
  if (!c) {
    hipExtLaunchKernelGGL(kernel, grid, block, lds_bytes, st, nullptr, nullptr, 0, args...);
    return;
  }
  c->begin(st);
  for (int r = 1; r < c->reps(); ++r)
    hipExtLaunchKernelGGL(kernel, grid, block, lds_bytes, st, nullptr, nullptr, 0, args...);
  hipEvent_t e0 = c->start_event();
  hipEvent_t e1 = c->stop_event();
  hipExtLaunchKernelGGL(kernel, grid, block, lds_bytes, st, e0, e1, 0, args...);
  c->end(st);
}

enum Dtype { DT_F32 = 0, DT_BF16 = 1 };
inline int dtype_size(int dt) { return dt == DT_F32 ? 4 : 2; }

// GEMM geometry shared with the weight packer: packed weights are [Npad][Kpad] in the compute
// type, Npad a multiple of GEMM_BN (the widest N tile), Kpad a multiple of GEMM_BK_BYTES / elem_size.
constexpr int GEMM_BN = 256;
constexpr int GEMM_BK_BYTES = 128;
inline int round_up_int(int v, int m) { return (v + m - 1) / m * m; }

enum Epilogue {
  EPI_STORE = 0,       // C[m,n] = acc + bias[n]                        (compute type)
  EPI_RELU = 1,        // C = relu(acc + bias)
  EPI_SWISH = 2,       // C = swish(acc + bias)
  EPI_RESID = 3,       // X[m,n] (fp32) += alpha * (acc + bias)
  EPI_SCALE_F32 = 4,   // X[m,n] (fp32)  = (acc + bias) * alpha
  EPI_GLU_MASK = 5,    // C[m, c] = (a + ba) * sigmoid(g + bg), zero for padded frames (GLU-packed W)
  EPI_QKV = 6,         // packed cols [q | k | v]: C = [q+u | q+v | k] (ldc = 3*H*dkp), v -> Vt[(b*H+h)][d][t]
  EPI_GLU_DW = 7,      // EPI_GLU_MASK + depthwise conv (k 31) + BatchNorm (running stats) + Swish on an
                       // utterance-aligned 256-row tile (one per utterance at T' <= 256, else tiles of 226
                       // output frames with 15 context frames either side): C = conv module's S rows
  EPI_SWISH_BWD = 8,   // training: C (compute type) = acc * dropout'(m*ldz + n) * swish'(zin[m][n]), the
                       // FFN hidden's backward through Swish and its dropout (conformer_modules.py:196-198)
  EPI_SWISH_Z = 9,     // training: C = z = acc + bias and C2 = dropout(swish(z)) (mask index m*ldc + n), both
                       // compute type, ld ldc: the FFN hidden and its pre-activation tape in one pass
};

// Dropout masks (training): keep element e iff hash(key, e) >= thr, thr = p * 2^32; kept values are
// scaled by 1 / (1 - p).  The hash is a function of the element index only, so a mask is recomputed
// wherever it is needed (forward epilogue, backward) instead of being stored.
struct Drop {
  uint32_t thr;    // 0 = no dropout
  uint32_t key;    // per (step, site)
  float scale;     // 1 / (1 - p)
  uint32_t k0;     // mix32(key): the element-independent half of the hash for indices below 2^32
};
__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}
__device__ __forceinline__ float drop_mul(const Drop& d, uint64_t e) {
  if (d.thr == 0) return 1.0f;
  // the inner mix depends only on e >> 32, which is 0 for every index below 2^32: taken from d.k0, and
  // computed only when some lane of the wave has a larger index (a wave-uniform branch)
  const uint32_t hi = (uint32_t)(e >> 32);
  uint32_t km = d.k0;
  if (__builtin_amdgcn_ballot_w64(hi != 0)) km = mix32(d.key ^ hi * 0x9e3779b9u);
  const uint32_t h = mix32((uint32_t)e ^ km);
  return h >= d.thr ? d.scale : 0.0f;
}

// host: keep(e) iff hash(seed, site, e) >= thr, thr = p * 2^32; kept values scaled by 1/(1-p)
inline uint32_t host_mix32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}
inline Drop make_drop(float p, uint64_t seed, int site) {
  Drop d{0u, 0u, 1.0f};
  if (p <= 0.0f) return d;
  const double t = (p < 1.0f ? (double)p : 1.0) * 4294967296.0;
  d.thr = (uint32_t)(t > 4294967295.0 ? 4294967295.0 : (t < 1.0 ? 1.0 : t));
  d.key = host_mix32((uint32_t)seed ^ host_mix32((uint32_t)(seed >> 32) + 0x632be5abu * (uint32_t)site));
  d.k0 = host_mix32(d.key);
  d.scale = p < 1.0f ? 1.0f / (1.0f - p) : 0.0f;
  return d;
}

struct GemmEpi {
  int mode;
  const float* bias;   // [Npad] fp32 (may be null)
  float alpha;
  void* C; long ldc;   // elements
  float* X; long ldx;  // fp32 residual / output
  const int32_t* lens; int Tp;          // pad mask (EPI_GLU_MASK) and row -> (b, t) for EPI_QKV
  void* Vt; int H; int dkp; int vt_rows; int Tpad;  // EPI_QKV: Vt [(B*H) * vt_rows][Tpad]
  int qk_cols;         // EPI_QKV: columns < qk_cols (= 2*H*dkp) are q and k, the rest are V
  const float* uv;     // EPI_QKV: pos_bias_u then pos_bias_v, each [H][dkp] zero-padded
  float qscale;        // EPI_QKV: (q + u), (q + v) are written pre-multiplied by log2(e) / sqrt(dk)
  int out_scalar;      // EPI_SCALE_F32: element stores (fp32 rows whose stride is not a multiple of 4)
  int nt_store;        // EPI_SCALE_F32 with out_scalar: non-temporal body stores (output read by no later kernel soon)
  int wt;              // set by gemm(): 16-byte output stores write-through (sc1), see store16_wt
  const float* Xin;    // EPI_RESID: residual input (null: X, updated in place)
  Drop drop;           // EPI_RESID: dropout on the branch, mask index m * ldx + n (thr 0: none)
  // LayerNorm folded into the next GEMM (eval forward, bf16 mode; DESIGN.md §4 "LayerNorm fold").
  // Producer (EPI_RESID): also writes the new X rows in the compute type to xb (ld ldx) and, per row
  // and 128-column granule g, the granule's (mean, M2) to ln_out[m * ln_parts + g].
  void* xb;
  float2* ln_out;
  int ln_parts;        // granules per row = ceil(N / 128)
  // Consumer (any compute-type epilogue): the GEMM ran on A = xb with W' = W * diag(gamma); the
  // epilogue forms LayerNorm(x) . W^T + b = rstd * (acc - mean * ln_c[n]) + ln_d[n] from the row's
  // granule partials (ln_in, ln_parts per row, ln_width = d columns in all); bias must be null.
  const float2* ln_in;
  int ln_width;
  const float* ln_c;   // [Npad] sum_k W'[n][k] (of the packed, rounded W')
  const float* ln_d;   // [Npad] sum_k beta[k] W[n][k] + bias[n]
  // Utterance-aligned rows (EPI_GLU_DW): GEMM row m is frame t = m % 256 of utterance b = m / 256,
  // A / output row b * utt_tp + t (t < utt_tp; utt_M real rows); 0 = rows are plain.
  int utt_tp, utt_M;
  int utt_nt, utt_out, utt_halo;   // tiles per utterance, output frames per tile, context frames either side
  const float* dw_w;   // EPI_GLU_DW: depthwise weight [31][d], bias [d], BatchNorm mean / 1/sqrt(var+eps) / w / b
  const float* dw_b;
  const float *bn_mean, *bn_inv, *bn_w, *bn_b;
  // EPI_SWISH_BWD: pre-activation z (compute type, ld ldz; also the dropout mask's row pitch)
  const void* zin;
  long ldz;
  void* C2;            // EPI_SWISH_Z: second output
};
constexpr int LN_GRANULE = 128;

struct ConvGeom {      // implicit-GEMM A operand for the 2nd subsampling conv (3x3, stride 2, pad 1)
  const void* X1;      // (B, T1, F1, C) channels-last, compute type
  int T1, F1, T2, F2, C;
};

// C = A[M,K] * Wp[N,K]^T with a fused epilogue. `K` = logical K (elements); A rows are `lda` elements.
void gemm(int dtype, const void* A, long lda, int M, int K, const void* Wp, int Kpad, int N,
          const GemmEpi& epi, const void* zero_page, hipStream_t st);
// As gemm() with the packed operand's row stride ldw (elements) decoupled from K (split-K slices).
void gemm_ldw(int dtype, const void* A, long lda, int M, int K, const void* Wp, long ldw, int N, const GemmEpi& epi,
              const void* zero_page, hipStream_t st);
// Split-K: S slices of kchunk K-elements in one launch (grid.y), fp32 partials at epi.X + s*split_x.
void gemm_splitk(int dtype, const void* A, long lda, int M, int K, const void* Wp, long ldw, int N, int S, int kchunk,
                 const GemmEpi& epi, long split_x, const void* zero_page, hipStream_t st);
// -1 = automatic tile choice; otherwise 0:128x128 1:256x128 2:128x256 3:64x128. Returns the previous value.
int set_gemm_tile_override(int tile);
// Microbenchmark probe bits for the dense GEMM (1 no main-loop loads, 2 no epilogue, 4 one K-step); 0 in production.
int set_gemm_probe(int probe);
void gemm_conv(int dtype, const ConvGeom& g, int B, const void* Wp, int Kpad, int N, const GemmEpi& epi,
               const void* zero_page, hipStream_t st);
// conv2's input gradient for one stride phase (pt, pf) of its input pixels (t1, f1) = (2i + pt, 2j + pf),
// as an implicit GEMM over the (1 + pt) * (1 + pf) taps reaching the phase: rows (b, i, j), K = taps x C
// read straight from dY2 (B, T2, F2, C) rows of `ld` elements; epi.mode must be EPI_STORE.
struct TConvGeom {
  const void* dY2;
  long ld;
  int B, T2, F2, C, pt, pf, nI, nJ;
};
bool gemm_tconv_supported(int dtype, int C);
// ConvSubsampling's conv.0 + ReLU + conv.2 + ReLU (bf16, C % 128 == 0, C <= 1024): X1 is recomputed
// inside conv2's implicit GEMM from per-pixel input patches instead of being written and re-read.
// X2 (B, T2, F2, C) bf16; `patch` scratch of conv12_patch_bytes(B, T1, F1) bytes.
bool conv12_supported(int dtype, int C);
size_t conv12_patch_bytes(int B, int T1, int F1, int C);
void conv12_fused(const float* x_bft, int B, int F, int T, int T1, int F1, int T2, int F2, const float* w1,
                  const float* b1, int C, const void* Wp, int Kpad, const float* b2, void* X2, void* patch,
                  const void* zero_page, hipStream_t st);
void gemm_tconv(int dtype, const TConvGeom& g, const void* Wp, int Kpad, int N, const GemmEpi& epi,
                const void* zero_page, hipStream_t st);
// pointwise_conv1 + GLU + depthwise conv + BatchNorm + Swish in one launch (bf16, epi.mode = EPI_GLU_DW,
// epi.utt_tp = T' <= 678, N = d, d % 64 == 0): 256x128 tiles per (utterance, 64 channels), 1-3 per utterance.
bool gemm_glu_dw_supported(int dtype, int Tp, int d, int K);
void gemm_glu_dw(int dtype, const void* A, long lda, int B, int Tp, int K, const void* Wp, int Kpad, int N,
                 const GemmEpi& epi, const void* zero_page, hipStream_t st);

void calc_length(const int32_t* len_in, int32_t* len_out, int B, int T, int repeat, hipStream_t st);
void conv1_subsample(int dtype, const float* x_bft, int B, int F, int T, const float* w9, const float* bias, int C,
                     void* out, hipStream_t st);
// LayerNorm over rows of d fp32 values.  out_x (fp32, may alias x) and/or out_t (compute type).
// If w2/b2 are given, a second LayerNorm is applied to the first's result and written to out_t
// (the fused "norm_out of layer l + norm_feed_forward1 of layer l+1").
void layernorm(int dtype, const float* x, int rows, int d, const float* w, const float* b, float* out_x,
               const float* w2, const float* b2, void* out_t, int swish_out, hipStream_t st);
void dwconv_norm_swish(int dtype, const void* g, int B, int Tp, int d, int K, const float* w, const float* bias,
                       const float* bn_mean, const float* bn_inv, const float* bn_w, const float* bn_b,
                       void* out_t, float* out_prenorm_f32, hipStream_t st);
void transpose_out(const float* X, int B, int Tp, int d, float* y_bdt, hipStream_t st);
// qk: [(q+u)*c | (q+v)*c | k] per row (ldqk = 3*H*dkp, c = log2(e)/sqrt(dk)), written by the EPI_QKV
// GEMM epilogue; the softmax then runs in base 2 on unscaled score sums.
// adrop: training-mode dropout of the attention probabilities (multi_head_attention.py:111).
void rel_pos_attention(int dtype, const void* qk, long ldqk, const void* Vt, int vt_rows, int Tpad, const void* P,
                       long ldp, const int32_t* lens, int B, int Tp, int H,
                       int dk, int dkp, int ctx_left, int ctx_right, void* out, long ldo, hipStream_t st,
                       Drop adrop = Drop{0u, 0u, 1.0f});
// Natural-layout variant (bf16, LDS-resident kernel; attn_natural_layout() says when it applies):
// qkv rows are [q | k | v] exactly as a plain bias GEMM stores them (heads padded to dkp); uv =
// [pos_bias_u | pos_bias_v] (fp32, H*dkp each); the kernel forms (q+u)*qscale, (q+v)*qscale and
// transposes V while staging it into LDS.
bool attn_natural_layout(int dtype, int Tp, int dkp);
void rel_pos_attention_natural(const void* qkv, long ldqkv, const float* uv, float qscale, const void* P, long ldp,
                               const int32_t* lens, int B, int Tp, int H, int dk, int dkp, int ctx_left,
                               int ctx_right, void* out, long ldo, hipStream_t st);
// QKV projection + attention in one launch (bf16 eval forward with the LayerNorm fold, dkp = 64,
// T' <= 256, d in {256, 512}): xb = the normalised-input rows' compute-type copy (M x d), ln_in their
// granule partials, Wqkv the folded q | k | v weight ([3*H*64][Kpad], Kpad = d) with column terms
// lc / ld; uv, qscale, P, out as rel_pos_attention_natural.  Replaces gemm(EPI_STORE) into qkv +
// rel_pos_attention_natural (no qkv buffer).
bool qkv_attention_fused_supported(int dtype, int Tp, int dkp, int d);
void qkv_rel_attention_fused(const void* xb, int d, const float2* ln_in, int ln_parts, const void* Wqkv, int Kpad,
                             const float* lc, const float* ld, const float* uv, float qscale, const void* P, long ldp,
                             const int32_t* lens, int B, int Tp, int H, int dk, int ctx_left, int ctx_right, void* out,
                             long ldo, const void* zero_page, hipStream_t st);
// q, k, v (M, H*dk), p (2T'-1, H*dk) in the compute type -> the qk / Vt / P layouts above, at ws,
// ws + qk_bytes, ws + qk_bytes + vt_bytes (what the QKV and pos GEMM epilogues write in the encoder).
void attn_relayout(int dt, const void* q, const void* k, const void* v, const void* p, const float* pos_u,
                   const float* pos_v, int B, int Tp, int H, int dk, int dkp, int vt_rows, int Tpad, char* ws,
                   long qk_bytes, long vt_bytes, hipStream_t st);
// Backward of rel_pos_attention from the same qk / Vt / P operands (attn_bwd.hip).  dctx (M, H*dk)
// fp32 = gradient of the attention output before linear_out; outputs fp32: dq, dk, dv (M, H*dk, ld
// ld_dqkv), dpos (2T'-1, H*dk, ld ld_dpos), du, dvb (H*dk) = pos_bias_u / pos_bias_v gradients.
size_t rel_pos_attention_backward_ws(int B, int Tp, int H, int dk);
void rel_pos_attention_backward(int dtype, const void* qk, long ldqk, const void* Vt, int vt_rows, int Tpad,
                                const void* P, long ldp, const int32_t* lens, int B, int Tp, int H, int dk, int dkp,
                                int ctx_left, int ctx_right, const float* dctx, long ld_dctx, float* dq, float* dk_,
                                float* dv, long ld_dqkv, float* dpos, long ld_dpos, float* du, float* dvb, char* ws,
                                hipStream_t st, Drop adrop = Drop{0u, 0u, 1.0f});
void convert_f32(int dtype, const float* src, void* dst, long n, hipStream_t st);
// X (B*T', d fp32) += pe[t] (rows of d fp32), d % 4 == 0
void add_rows_f32(float* X, const float* pe, int B, int Tp, int d, hipStream_t st);

// Weight gradient on frame-major operands (wgrad_tn.hip, bf16): out[n][k] (fp32, ld ldo) = sum over
// rows r of A[r][n] * B'[r][k] with B' = B (bfn 0) or dropout(swish(B)) (bfn 1, mask index r*ldb + k),
// the bias sum_r A[r][n] at column K when `ones`; S row splits of `chunk` rows (a multiple of
// 32) write partial tiles at out + s * split_stride.  Columns 0 .. Kout-1 are written.
bool wgrad_tn_supported(int dtype, int N, int K, long lda, long ldb);
// output tiles of one row split (bias in-kernel for bfn 0: no extra column tile) and the block count
// the row splits aim for (two 128x128 blocks or one larger block per CU)
int wgrad_tn_tiles(int N, int K, bool ones, int bfn);
int wgrad_tn_blocks(int bfn);
void wgrad_tn(const void* A, long lda, int N, const void* B, long ldb, int K, bool ones, int bfn, Drop bdr, long rows,
              int S, long chunk, float* out, long ldo, int Kout, long split_stride, hipStream_t st);
// conv.2's weight gradient [dW2 | db2] = dY2^T . [im2col(X1) | 1] with the im2col formed by the loader
// (wgrad_tn.hip): dy frame-major (rows = B*T2*F2 output pixels) x C, x1 = [B][T1][F1][C]; partial
// tiles [s][C][ldo] (columns tap * C + c, the bias at column 9C when `ones`) per `chunk` rows
bool wgrad_tn_conv_supported(int dtype, int C, long lda);
void wgrad_tn_conv(const void* dy, long lda, const void* x1, int B, int T1, int F1, int T2, int F2, int C, bool ones,
                   long rows, int S, long chunk, float* out, long ldo, long split_stride, hipStream_t st);

// ---- backward building blocks (backward.hip) ----
// dst[i][j] = transpose ? src[j][i] : src[i][j] in the compute type for i < rows_pad, j < cols_pad;
// src is fp32 [rows][cols] (ld src_ld), zero outside it.
void pack_matrix(int dtype, const float* src, long src_ld, int rows, int cols, bool transpose, void* dst, long dst_ld,
                 int rows_pad, int cols_pad, hipStream_t st);
// out[n] (+)= sum_m src[m][n], fixed-order (bitwise reproducible); ws >= col_sums_ws(M, N) bytes.
size_t col_sums_ws(int M, int N);
void col_sums(const float* src, long ld, int M, int N, float* out, int accumulate, float* ws, hipStream_t st);
// LayerNorm backward (one wave per row): dx (+)= ..., prod = dy * xhat (for the weight gradient).
void layernorm_backward(const float* x, const float* w, const float* dy, int M, int d, float* dx, int accumulate,
                        float* prod, hipStream_t st);
void swish_backward(const float* z, const float* du, float* dz, long n, hipStream_t st);

}  // namespace cfm
