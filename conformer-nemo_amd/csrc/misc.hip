// Non-GEMM kernels of the encoder forward: lengths, first subsampling conv, LayerNorm,
// depthwise conv + BatchNorm + Swish, output transpose.  All HBM-bound; see DESIGN.md for the
// algorithmic bytes each one moves.
#include "cfm_common.h"
#include "cfm_kernels.h"
#include "cfm_ln.h"

namespace cfm {

namespace {

// calc_length (subsampling.py:272-282): L <- floor((L + 2p - k)/s + 1) in float32, `repeat` times.
__global__ void calc_length_kernel(const int32_t* in, int32_t* out, int B, int T, int repeat) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  float L = in ? (float)in[b] : (float)T;
  for (int i = 0; i < repeat; ++i) L = floorf(__fdiv_rn(L + (2.0f * 1 - 3.0f), 2.0f) + 1.0f);
  out[b] = (int32_t)L;
}

// First Conv2d(1 -> C, 3x3, stride 2, pad 1) + ReLU of ConvSubsampling (subsampling.py:105-116, 173),
// reading the reference's (B, F, T) audio_signal directly (the (B,T,F) transpose of
// conformer_encoder.py:248 is folded into the indexing).  Output channels-last (B, T1, F1, C).
// One block per (b, t1); thread (x = 8-channel group, y = f1 slot); weights held in registers.
constexpr int CONV1_ROWS = 4;   // (b, t1) rows per block: the weight registers are loaded once for all

template <typename T>
__global__ __launch_bounds__(256) void conv1_kernel(const float* __restrict__ x, int F, int Tlen, int T1, int F1,
                                                    const float* __restrict__ w9, const float* __restrict__ bias,
                                                    int C, int BT, T* __restrict__ out) {
  __shared__ float xs[3][264];
  const int c0 = (blockIdx.y * 64 + threadIdx.x) * 8;
  const bool cok = c0 < C;
  // a thread's 8 channels x 9 taps are 72 consecutive floats of the (C, 1, 3, 3) weight: 18 float4
  // loads, kept in registers for the CONV1_ROWS (b, t1) rows of this block
  float w[8][9], bb[8];
  if (cok) {
    float wf[72];
    const float4* wp = (const float4*)(w9 + (long)c0 * 9);
#pragma unroll
    for (int i = 0; i < 18; ++i) {
      const float4 v = wp[i];
      wf[4 * i] = v.x; wf[4 * i + 1] = v.y; wf[4 * i + 2] = v.z; wf[4 * i + 3] = v.w;
    }
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      bb[c] = bias[c0 + c];
#pragma unroll
      for (int k = 0; k < 9; ++k) w[c][k] = wf[c * 9 + k];
    }
  }
  for (int rr = 0; rr < CONV1_ROWS; ++rr) {
    const int bt = blockIdx.x * CONV1_ROWS + rr;
    if (bt >= BT) break;                       // block-uniform
    const int b = bt / T1, t1 = bt - b * T1;
    if (rr > 0) __syncthreads();               // previous row's reads of xs are done
    for (int i = threadIdx.y * 64 + threadIdx.x; i < 3 * F; i += 256) {
      const int kt = i / F, f = i - kt * F;
      const int t = 2 * t1 - 1 + kt;
      xs[kt][f + 1] = (t >= 0 && t < Tlen) ? x[((long)b * F + f) * Tlen + t] : 0.0f;
    }
    if (threadIdx.y == 0 && threadIdx.x < 3) { xs[threadIdx.x][0] = 0.0f; xs[threadIdx.x][F + 1] = 0.0f; }
    __syncthreads();
    if (!cok) continue;
    for (int f1 = threadIdx.y; f1 < F1; f1 += 4) {
      float in[9];
#pragma unroll
      for (int kt = 0; kt < 3; ++kt)
#pragma unroll
        for (int kf = 0; kf < 3; ++kf) in[kt * 3 + kf] = xs[kt][2 * f1 + kf];   // (2f1 - 1 + kf) + 1 pad offset
      float o[8];
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        float a = 0.0f;
#pragma unroll
        for (int k = 0; k < 9; ++k) a = fmaf(w[c][k], in[k], a);
        o[c] = fmaxf(a + bb[c], 0.0f);
      }
      T* dst = out + (((long)b * T1 + t1) * F1 + f1) * C + c0;
      if constexpr (sizeof(T) == 2) {
        *(uint4*)dst = Vec16<bf16_t>::from_f32(o);
      } else {
        *(uint4*)dst = Vec16<float>::from_f32(o);
        *(uint4*)(dst + 4) = Vec16<float>::from_f32(o + 4);
      }
    }
  }
}

// LayerNorm(d, eps=1e-5) over fp32 rows (cfm_ln.h): each wave owns RB consecutive rows and issues
// all their loads before the first reduction, so the HBM latency is paid once per RB rows.
template <typename T, int E4, int RB>
__global__ __launch_bounds__(256) void layernorm_kernel(const float* __restrict__ x, int rows, int d,
                                                        const float* __restrict__ w, const float* __restrict__ b,
                                                        float* out_x, const float* __restrict__ w2,
                                                        const float* __restrict__ b2, T* out_t, int swish_out) {
  const int row0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * RB;
  const int lane = threadIdx.x & 63;
  if (row0 >= rows) return;
  float4 v[RB][E4];
#pragma unroll
  for (int i = 0; i < RB; ++i) ln_load<E4>(x + (long)min(row0 + i, rows - 1) * d, d, lane, v[i]);
#pragma unroll
  for (int i = 0; i < RB; ++i) {
    const int row = row0 + i;
    if (row < rows)
      ln_apply<T, E4>(v[i], d, lane, w, b, out_x ? out_x + (long)row * d : nullptr, w2, b2,
                      out_t ? out_t + (long)row * d : nullptr, swish_out);
  }
}

// Depthwise Conv1d(k, pad (k-1)/2, groups=d) + bias + BatchNorm1d(eval) + Swish
// (conformer_modules.py:139-149, 168-177) on (B, T', d) channels-last data.  The GLU epilogue has
// already zeroed padded frames (the masked_fill of :165-166).  Block = (b, 32 frames, 64 channels);
// the frame tile plus its (k-1)-frame halo is staged in LDS as fp32.
// If out_prenorm_f32 is given (conv_norm_type = layer_norm), writes conv + bias only.
template <typename T>
__global__ __launch_bounds__(256) void dwconv_kernel(const T* __restrict__ g, int Tp, int d, int K,
                                                     const float* __restrict__ w, const float* __restrict__ bias,
                                                     const float* __restrict__ bn_mean, const float* __restrict__ bn_inv,
                                                     const float* __restrict__ bn_w, const float* __restrict__ bn_b,
                                                     T* __restrict__ out, float* __restrict__ prenorm) {
  constexpr int TT = 32;
  __shared__ float xs[TT + 64][65];
  __shared__ float ws[64][65];
  const int b = blockIdx.z, t0 = blockIdx.x * TT, c0 = blockIdx.y * 64;
  const int pad = (K - 1) / 2;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int c = c0 + tx;
  const int nrows = TT + K - 1;
  for (int r = ty; r < nrows; r += 4) {
    const int t = t0 - pad + r;
    float v = 0.0f;
    if (t >= 0 && t < Tp && c < d) v = ld_f<T>(g + ((long)b * Tp + t) * d + c);
    xs[r][tx] = v;
  }
  for (int k = ty; k < K; k += 4) ws[k][tx] = (c < d) ? w[(long)k * d + c] : 0.0f;   // w packed [K][d]
  __syncthreads();
  if (c >= d) return;
  const float bi = bias[c];
  float mu = 0.f, inv = 1.f, gw = 1.f, gb = 0.f;
  if (!prenorm) { mu = bn_mean[c]; inv = bn_inv[c]; gw = bn_w[c]; gb = bn_b[c]; }
  for (int tt = ty; tt < TT; tt += 4) {
    const int t = t0 + tt;
    if (t >= Tp) break;
    float a = 0.0f;
    for (int k = 0; k < K; ++k) a = fmaf(ws[k][tx], xs[tt + k][tx], a);
    a += bi;
    const long o = ((long)b * Tp + t) * d + c;
    if (prenorm) {
      prenorm[o] = a;
    } else {
      const float y = (a - mu) * inv * gw + gb;
      st_f<T>(out + o, swishf(y));
    }
  }
}

// Register-window variant for a compile-time kernel size K (31 in every reference config):
// thread = one channel x DT consecutive frames; its DT + K - 1 input frames are loaded straight from
// global (lanes = consecutive channels -> coalesced rows) into registers, weights ([K][d] packed)
// likewise, and the DT x K products run on fully static register indices.
template <typename T, int K, int DT>
__global__ __launch_bounds__(256) void dwconv_reg_kernel(const T* __restrict__ g, int Tp, int d,
                                                         const float* __restrict__ w, const float* __restrict__ bias,
                                                         const float* __restrict__ bn_mean,
                                                         const float* __restrict__ bn_inv,
                                                         const float* __restrict__ bn_w,
                                                         const float* __restrict__ bn_b, T* __restrict__ out,
                                                         float* __restrict__ prenorm) {
  constexpr int PAD = (K - 1) / 2, NX = DT + K - 1;
  const int c = blockIdx.y * 256 + threadIdx.x;
  const int b = blockIdx.z, t0 = blockIdx.x * DT;
  if (c >= d) return;
  const T* gc = g + (long)b * Tp * d + c;
  float x[NX];
#pragma unroll
  for (int i = 0; i < NX; ++i) {
    const int t = t0 - PAD + i;
    // unconditional load of a clamped frame, zeroed after: a load under a per-element condition
    // would be branched around and serialised behind its own vmcnt(0)
    const float v = ld_f<T>(gc + (long)min(max(t, 0), Tp - 1) * d);
    x[i] = (t >= 0 && t < Tp) ? v : 0.0f;
  }
  float wk[K];
#pragma unroll
  for (int k = 0; k < K; ++k) wk[k] = w[(long)k * d + c];
  const float bi = bias[c];
  float mu = 0.f, inv = 1.f, gw = 1.f, gb = 0.f;
  if (!prenorm) { mu = bn_mean[c]; inv = bn_inv[c]; gw = bn_w[c]; gb = bn_b[c]; }
  T* oc = out + (long)b * Tp * d + c;
#pragma unroll
  for (int j = 0; j < DT; ++j) {
    float a = 0.0f;
#pragma unroll
    for (int k = 0; k < K; ++k) a = fmaf(wk[k], x[j + k], a);
    a += bi;
    const int t = t0 + j;
    if (t < Tp) {
      if (prenorm) prenorm[((long)b * Tp + t) * d + c] = a;
      else st_f<T>(oc + (long)t * d, swishf((a - mu) * inv * gw + gb));
    }
  }
}

// Output layout contract (conformer_encoder.py:280): X (B*T', d) fp32 -> y (B, d, T').
__global__ __launch_bounds__(256) void transpose_kernel(const float* __restrict__ X, int Tp, int d,
                                                        float* __restrict__ y) {
  __shared__ float tile[32][33];
  const int b = blockIdx.z, t0 = blockIdx.x * 32, c0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int i = ty; i < 32; i += 8) {
    const int t = t0 + i, c = c0 + tx;
    tile[i][tx] = (t < Tp && c < d) ? X[((long)b * Tp + t) * d + c] : 0.0f;
  }
  __syncthreads();
  for (int i = ty; i < 32; i += 8) {
    const int c = c0 + i, t = t0 + tx;
    if (c < d && t < Tp) y[((long)b * d + c) * Tp + t] = tile[tx][i];
  }
}

template <typename T>
__global__ void convert_kernel(const float* __restrict__ src, T* __restrict__ dst, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    st_f<T>(dst + i, src[i]);
}

// X (B*T', d) += pe rows 0 .. T'-1 (d % 4 == 0): the absolute positional encoding
__global__ __launch_bounds__(256) void add_rows_kernel(float4* __restrict__ X, const float4* __restrict__ pe, int Tp,
                                                       int d4, long n4) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    const long row = i / d4;
    const int c = (int)(i - row * d4);
    const float4 p = pe[(long)(row % Tp) * d4 + c];
    float4 x = X[i];
    x.x += p.x; x.y += p.y; x.z += p.z; x.w += p.w;
    X[i] = x;
  }
}

}  // namespace

void calc_length(const int32_t* len_in, int32_t* len_out, int B, int T, int repeat, hipStream_t st) {
  if (B <= 0) return;
  cfm_launch(calc_length_kernel, dim3((B + 63) / 64), dim3(64), 0, st, len_in, len_out, B, T, repeat);
}

void conv1_subsample(int dtype, const float* x, int B, int F, int T, const float* w9, const float* bias, int C,
                     void* out, hipStream_t st) {
  const int T1 = (T - 1) / 2 + 1, F1 = (F - 1) / 2 + 1;
  if (B <= 0 || T1 <= 0) return;
  const int BT = B * T1;
  const dim3 grid((BT + CONV1_ROWS - 1) / CONV1_ROWS, (C / 8 + 63) / 64), block(64, 4);
  if (dtype == DT_F32)
    cfm_launch(conv1_kernel<float>, grid, block, 0, st, x, F, T, T1, F1, w9, bias, C, BT, (float*)out);
  else
    cfm_launch(conv1_kernel<bf16_t>, grid, block, 0, st, x, F, T, T1, F1, w9, bias, C, BT, (bf16_t*)out);
}

template <typename T>
static void ln_launch(int E4, const float* x, int rows, int d, const float* w, const float* b, float* ox,
                      const float* w2, const float* b2, T* ot, int sw, hipStream_t st) {
  constexpr int RB = 1;   // RB = 2 measured 8.9 vs 8.4 us per launch (Large-17, B=32)
  const dim3 grid((rows + 4 * RB - 1) / (4 * RB)), block(256);
  switch (E4) {
    case 1: cfm_launch((layernorm_kernel<T, 1, RB>), grid, block, 0, st, x, rows, d, w, b, ox, w2, b2, ot, sw); break;
    case 2: cfm_launch((layernorm_kernel<T, 2, RB>), grid, block, 0, st, x, rows, d, w, b, ox, w2, b2, ot, sw); break;
    case 4: cfm_launch((layernorm_kernel<T, 4, RB>), grid, block, 0, st, x, rows, d, w, b, ox, w2, b2, ot, sw); break;
    default: cfm_launch((layernorm_kernel<T, 8, RB>), grid, block, 0, st, x, rows, d, w, b, ox, w2, b2, ot, sw); break;
  }
}

void layernorm(int dtype, const float* x, int rows, int d, const float* w, const float* b, float* out_x,
               const float* w2, const float* b2, void* out_t, int swish_out, hipStream_t st) {
  if (rows <= 0) return;
  const int d4 = d / 4;
  const int E4 = d4 <= 64 ? 1 : d4 <= 128 ? 2 : d4 <= 256 ? 4 : 8;
  if (dtype == DT_F32) ln_launch<float>(E4, x, rows, d, w, b, out_x, w2, b2, (float*)out_t, swish_out, st);
  else ln_launch<bf16_t>(E4, x, rows, d, w, b, out_x, w2, b2, (bf16_t*)out_t, swish_out, st);
}

void dwconv_norm_swish(int dtype, const void* g, int B, int Tp, int d, int K, const float* w, const float* bias,
                       const float* bn_mean, const float* bn_inv, const float* bn_w, const float* bn_b, void* out_t,
                       float* out_prenorm_f32, hipStream_t st) {
  if (B <= 0 || Tp <= 0) return;
  if (K == 31) {
    constexpr int DT = 32;
    const dim3 grid((Tp + DT - 1) / DT, (d + 255) / 256, B), block(256);
    if (dtype == DT_F32)
      cfm_launch((dwconv_reg_kernel<float, 31, DT>), grid, block, 0, st, (const float*)g, Tp, d, w, bias,
                         bn_mean, bn_inv, bn_w, bn_b, (float*)out_t, out_prenorm_f32);
    else
      cfm_launch((dwconv_reg_kernel<bf16_t, 31, DT>), grid, block, 0, st, (const bf16_t*)g, Tp, d, w, bias,
                         bn_mean, bn_inv, bn_w, bn_b, (bf16_t*)out_t, out_prenorm_f32);
    return;
  }
  const dim3 grid((Tp + 31) / 32, (d + 63) / 64, B), block(256);
  if (dtype == DT_F32)
    cfm_launch(dwconv_kernel<float>, grid, block, 0, st, (const float*)g, Tp, d, K, w, bias, bn_mean, bn_inv,
                       bn_w, bn_b, (float*)out_t, out_prenorm_f32);
  else
    cfm_launch(dwconv_kernel<bf16_t>, grid, block, 0, st, (const bf16_t*)g, Tp, d, K, w, bias, bn_mean, bn_inv,
                       bn_w, bn_b, (bf16_t*)out_t, out_prenorm_f32);
}

void transpose_out(const float* X, int B, int Tp, int d, float* y, hipStream_t st) {
  if (B <= 0 || Tp <= 0) return;
  cfm_launch(transpose_kernel, dim3((Tp + 31) / 32, (d + 31) / 32, B), dim3(256), 0, st, X, Tp, d, y);
}

void add_rows_f32(float* X, const float* pe, int B, int Tp, int d, hipStream_t st) {
  const long n4 = (long)B * Tp * (d / 4);
  if (n4 <= 0) return;
  const int blocks = (int)std::min<long>((n4 + 255) / 256, 4096);
  cfm_launch(add_rows_kernel, dim3(blocks), dim3(256), 0, st, (float4*)X, (const float4*)pe, Tp, d / 4, n4);
}

void convert_f32(int dtype, const float* src, void* dst, long n, hipStream_t st) {
  if (n <= 0) return;
  const int blocks = (int)std::min<long>((n + 255) / 256, 4096);
  if (dtype == DT_F32) cfm_launch(convert_kernel<float>, dim3(blocks), dim3(256), 0, st, src, (float*)dst, n);
  else cfm_launch(convert_kernel<bf16_t>, dim3(blocks), dim3(256), 0, st, src, (bf16_t*)dst, n);
}

}  // namespace cfm
