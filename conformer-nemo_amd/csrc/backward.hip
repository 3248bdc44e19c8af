// Backward building blocks of the Conformer layer (training step of BASELINE
// config 3): operand relayouts for the gradient GEMMs, deterministic column reductions,
// LayerNorm backward and the Swish derivative.  The gradient GEMMs themselves run on the forward
// GEMM kernel (gemm.hip): dX = dY . W on a packed W^T, dW = dY^T . X on transposed operands.
//
// Reference semantics: torch.nn.LayerNorm (conformer_modules.py:66-70 via the layer, eps 1e-5,
// biased variance), nn.Linear (y = x W^T + b), Swish (activations.py:20, x * sigmoid(x)).
#include <algorithm>
#include <cstdio>
#include <cstring>

#include "../../include/cfm_train.h"
#include "cfm_abi.h"
#include "cfm_common.h"
#include "cfm_kernels.h"

namespace cfm {
namespace {

// dst[i][j] = transpose ? src[j][i] : src[i][j] (compute type), zero outside src; 32x32 LDS tiles.
template <typename T>
__global__ __launch_bounds__(256) void pack_kernel(const float* __restrict__ src, long src_ld, int rows, int cols,
                                                   int transpose, T* __restrict__ dst, long dst_ld, int rows_pad,
                                                   int cols_pad) {
  __shared__ float tile[32][33];
  const int i0 = blockIdx.y * 32, j0 = blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int k = ty; k < 32; k += 8) {
    if (transpose) {   // tile[k][tx] = src[j0 + k][i0 + tx]: coalesced along the source rows
      const int si = j0 + k, sj = i0 + tx;
      tile[k][tx] = (si < rows && sj < cols) ? src[(long)si * src_ld + sj] : 0.0f;
    } else {
      const int si = i0 + k, sj = j0 + tx;
      tile[k][tx] = (si < rows && sj < cols) ? src[(long)si * src_ld + sj] : 0.0f;
    }
  }
  __syncthreads();
  for (int k = ty; k < 32; k += 8) {
    const int di = i0 + k, dj = j0 + tx;
    if (di < rows_pad && dj < cols_pad) st_f<T>(dst + (long)di * dst_ld + dj, transpose ? tile[tx][k] : tile[k][tx]);
  }
}

// The non-transposed pack as row runs: a wave converts one row 128 columns at a time (two adjacent columns per
// lane, one 4- or 8-byte store; no LDS), grid-striding over rows.  Same values as pack_kernel (zero outside src,
// the same rounding); needs even dst_ld and cols_pad.
template <typename T>
__global__ __launch_bounds__(256) void pack_rows_kernel(const float* __restrict__ src, long src_ld, int rows, int cols,
                                                        T* __restrict__ dst, long dst_ld, int rows_pad, int cols_pad) {
  const int lane = threadIdx.x & 63;
  for (long r = (long)blockIdx.x * 4 + (threadIdx.x >> 6); r < rows_pad; r += (long)gridDim.x * 4) {
    // loads from a clamped row / column, the value selected afterwards: a load under a per-lane condition
    // is branched around and waited for one at a time (cdna_hip_programming.md §5)
    const float* sr = src + std::min<long>(r, rows - 1) * src_ld;   // rows, cols >= 1 (pack_matrix)
    T* dr = dst + r * dst_ld;
    const bool rok = r < rows;
    for (int c0 = 0; c0 < cols_pad; c0 += 512) {   // 4 x 128 columns: all 8 loads before any store
      float v[4][2];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int c = c0 + 128 * k + 2 * lane;
        v[k][0] = sr[min(c, cols - 1)];
        v[k][1] = sr[min(c + 1, cols - 1)];
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int c = c0 + 128 * k + 2 * lane;
        const float v0 = (rok && c < cols) ? v[k][0] : 0.0f;
        const float v1 = (rok && c + 1 < cols) ? v[k][1] : 0.0f;
        if (c < cols_pad) {
          if constexpr (sizeof(T) == 4) {
            *(float2*)(dr + c) = make_float2(v0, v1);
          } else {
            const bf16_t b0 = f2bf(v0), b1 = f2bf(v1);
            *(uint32_t*)(dr + c) = (uint32_t)__builtin_bit_cast(uint16_t, b0) | ((uint32_t)__builtin_bit_cast(uint16_t, b1) << 16);
          }
        }
      }
    }
  }
}

// Column sums, stage 1: partial[chunk][n] = sum of a 256-row chunk (block = 64 columns x 4 row lanes,
// every row read a coalesced 256-byte segment); stage 2 folds the chunks (16 columns x 16 lanes).
// Fixed order: bitwise reproducible.
constexpr int kColRows = 256;
__global__ __launch_bounds__(256) void colsum_partial_kernel(const float* __restrict__ src, long ld, int M, int N,
                                                             float* __restrict__ partial) {
  __shared__ float red[4][64];
  const int c = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int n = blockIdx.x * 64 + c, nc = min(n, N - 1);
  const int r0 = blockIdx.y * kColRows, r1 = min(M, r0 + kColRows);
  float s = 0.0f;
#pragma unroll 8
  for (int r = r0 + rl; r < r1; r += 4) s += src[(long)r * ld + nc];
  red[rl][c] = s;
  __syncthreads();
  if (rl == 0 && n < N) partial[(long)blockIdx.y * N + n] = (red[0][c] + red[1][c]) + (red[2][c] + red[3][c]);
}
__global__ __launch_bounds__(256) void colsum_final_kernel(const float* __restrict__ partial, int nchunks, int N,
                                                           float* __restrict__ out, int accumulate) {
  __shared__ float red[16][17];
  const int c = threadIdx.x & 15, rl = threadIdx.x >> 4;
  const int n = blockIdx.x * 16 + c, nc = min(n, N - 1);
  float s = 0.0f;
#pragma unroll 8
  for (int k = rl; k < nchunks; k += 16) s += partial[(long)k * N + nc];
  red[rl][c] = s;
  __syncthreads();
  if (rl == 0 && n < N) {
    float v = 0.0f;
#pragma unroll
    for (int k = 0; k < 16; ++k) v += red[k][c];
    out[n] = accumulate ? out[n] + v : v;
  }
}

// LayerNorm backward, one wave per row (E4 float4 chunks per lane, d % 4 == 0):
//   xhat = (x - mean) * rstd, g = dy * w
//   dx   = rstd * (g - mean(g) - xhat * mean(g * xhat))       (+= dx_acc if accumulate)
//   prod = dy * xhat  (rows, for dw = column sums)
template <int E4>
__global__ __launch_bounds__(256) void layernorm_bwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                            const float* __restrict__ dy, int M, int d,
                                                            float* __restrict__ dx, int accumulate,
                                                            float* __restrict__ prod) {
#pragma clang fp contract(off)
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= M) return;
  const int d4 = d >> 2;
  const float4* xr = (const float4*)(x + (long)row * d);
  const float4* dr = (const float4*)(dy + (long)row * d);
  const float4* wr = (const float4*)w;
  float4 xv[E4], dv[E4], wv[E4];
  float s = 0.0f;
#pragma unroll
  for (int e = 0; e < E4; ++e) {
    const int g = min(lane + 64 * e, d4 - 1);
    const bool ok = lane + 64 * e < d4;
    xv[e] = ok ? xr[g] : make_float4(0, 0, 0, 0);
    dv[e] = ok ? dr[g] : make_float4(0, 0, 0, 0);
    wv[e] = wr[g];
    s += xv[e].x + xv[e].y + xv[e].z + xv[e].w;
  }
  const float inv_d = 1.0f / (float)d;
  const float mean = wave_sum(s) * inv_d;
  float q = 0.0f;
#pragma unroll
  for (int e = 0; e < E4; ++e) {
    if (lane + 64 * e < d4) {
      const float a0 = xv[e].x - mean, a1 = xv[e].y - mean, a2 = xv[e].z - mean, a3 = xv[e].w - mean;
      q += a0 * a0 + a1 * a1 + a2 * a2 + a3 * a3;
    }
  }
  const float rstd = 1.0f / sqrtf(wave_sum(q) * inv_d + 1e-5f);
  float sg = 0.0f, sgx = 0.0f;
  float4 xh[E4], gv[E4];
#pragma unroll
  for (int e = 0; e < E4; ++e) {
    xh[e] = make_float4((xv[e].x - mean) * rstd, (xv[e].y - mean) * rstd, (xv[e].z - mean) * rstd,
                        (xv[e].w - mean) * rstd);
    gv[e] = make_float4(dv[e].x * wv[e].x, dv[e].y * wv[e].y, dv[e].z * wv[e].z, dv[e].w * wv[e].w);
    if (lane + 64 * e < d4) {
      sg += gv[e].x + gv[e].y + gv[e].z + gv[e].w;
      sgx += gv[e].x * xh[e].x + gv[e].y * xh[e].y + gv[e].z * xh[e].z + gv[e].w * xh[e].w;
    }
  }
  const float mg = wave_sum(sg) * inv_d, mgx = wave_sum(sgx) * inv_d;
  float4* dxr = (float4*)(dx + (long)row * d);
  float4* pr = (float4*)(prod + (long)row * d);
#pragma unroll
  for (int e = 0; e < E4; ++e) {
    const int g = lane + 64 * e;
    if (g < d4) {
      float4 o = make_float4(rstd * (gv[e].x - mg - xh[e].x * mgx), rstd * (gv[e].y - mg - xh[e].y * mgx),
                             rstd * (gv[e].z - mg - xh[e].z * mgx), rstd * (gv[e].w - mg - xh[e].w * mgx));
      if (accumulate) {
        const float4 a = dxr[g];
        o.x += a.x; o.y += a.y; o.z += a.z; o.w += a.w;
      }
      dxr[g] = o;
      pr[g] = make_float4(dv[e].x * xh[e].x, dv[e].y * xh[e].y, dv[e].z * xh[e].z, dv[e].w * xh[e].w);
    }
  }
}

// dz = du * swish'(z),  swish'(z) = s + z * s * (1 - s), s = sigmoid(z)   (exact sigmoid)
__global__ __launch_bounds__(256) void swish_bwd_kernel(const float* __restrict__ z, const float* __restrict__ du,
                                                        float* __restrict__ dz, long n) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const float zz = z[i];
    const float s = 1.0f / (1.0f + expf(-zz));
    dz[i] = du[i] * (s + zz * s * (1.0f - s));
  }
}

// ---- convolution module (conformer_modules.py:160-180) ---------------------------------------

// GLU(dim=1) + pad mask backward: pre (rows, 2d) = [a | g] (pointwise_conv1 output, channels-last),
// dy (rows, d) = d(masked GLU output).  Padded frames (t >= len[b]) were zeroed after the GLU, so
// their gradient is 0.  dpre = [dy * sigmoid(g) | dy * a * sigmoid(g) * (1 - sigmoid(g))].
__global__ __launch_bounds__(256) void glu_bwd_kernel(const float* __restrict__ pre, const float* __restrict__ dy,
                                                      const int32_t* __restrict__ lens, int Tp, int d, long rows,
                                                      float* __restrict__ dpre) {
  const long n = rows * d;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const long m = i / d;
    const int c = (int)(i - m * d);
    const int b = (int)(m / Tp), t = (int)(m - (long)b * Tp);
    const float g = pre[m * 2 * d + d + c], a = pre[m * 2 * d + c];
    const float s = 1.0f / (1.0f + expf(-g));
    const float dv = (lens && t >= lens[b]) ? 0.0f : dy[i];
    dpre[m * 2 * d + c] = dv * s;
    dpre[m * 2 * d + d + c] = dv * a * s * (1.0f - s);
  }
}

// Depthwise Conv1d(k, pad (k-1)/2, groups=d) input gradient (the forward's cross-correlation with
// the kernel flipped): dx[b,t,c] = sum_k w[c][k] * dy[b, t - k + pad, c].  w is the reference
// (d, 1, k) weight.  Thread = channel, 32 frames per block, register window.
template <int K, int DT>
__global__ __launch_bounds__(256) void dwconv_bwd_x_kernel(const float* __restrict__ dy, const float* __restrict__ w,
                                                           int Tp, int d, float* __restrict__ dx) {
  constexpr int PAD = (K - 1) / 2, NX = DT + K - 1;
  const int c = blockIdx.y * 256 + threadIdx.x, b = blockIdx.z, t0 = blockIdx.x * DT;
  if (c >= d) return;
  const float* yc = dy + (long)b * Tp * d + c;
  float y[NX];
#pragma unroll
  for (int i = 0; i < NX; ++i) {   // y[i] = dy[t0 - PAD + i]
    const int t = t0 - PAD + i;
    const float v = yc[(long)min(max(t, 0), Tp - 1) * d];
    y[i] = (t >= 0 && t < Tp) ? v : 0.0f;
  }
  float wk[K];
#pragma unroll
  for (int k = 0; k < K; ++k) wk[k] = w[(long)c * K + k];
#pragma unroll
  for (int j = 0; j < DT; ++j) {
    float a = 0.0f;
#pragma unroll
    for (int k = 0; k < K; ++k) a = fmaf(wk[k], y[j + 2 * PAD - k], a);   // dy[t0 + j - k + PAD]
    const int t = t0 + j;
    if (t < Tp) dx[((long)b * Tp + t) * d + c] = a;
  }
}

// Depthwise weight gradient, stage 1: partial[b * nt + tile][k][c] = sum over the tile's frames t of
// x[b, t + k - pad, c] * dy[b, t, c]  (x = the conv input, zero outside [0, T')).
template <int K, int DT>
__global__ __launch_bounds__(256) void dwconv_bwd_w_kernel(const float* __restrict__ x, const float* __restrict__ dy,
                                                           int Tp, int d, float* __restrict__ partial) {
  constexpr int PAD = (K - 1) / 2, NX = DT + K - 1;
  const int c = blockIdx.y * 256 + threadIdx.x, b = blockIdx.z, t0 = blockIdx.x * DT;
  if (c >= d) return;
  const float* xc = x + (long)b * Tp * d + c;
  const float* yc = dy + (long)b * Tp * d + c;
  float xv[NX];
#pragma unroll
  for (int i = 0; i < NX; ++i) {   // xv[i] = x[t0 - PAD + i]
    const int t = t0 - PAD + i;
    const float v = xc[(long)min(max(t, 0), Tp - 1) * d];
    xv[i] = (t >= 0 && t < Tp) ? v : 0.0f;
  }
  float acc[K];
#pragma unroll
  for (int k = 0; k < K; ++k) acc[k] = 0.0f;
#pragma unroll
  for (int j = 0; j < DT; ++j) {
    const int t = t0 + j;
    const float g = yc[(long)min(t, Tp - 1) * d];
    const float gv = t < Tp ? g : 0.0f;
#pragma unroll
    for (int k = 0; k < K; ++k) acc[k] = fmaf(xv[j + k], gv, acc[k]);
  }
  float* pc = partial + ((long)(b * gridDim.x + blockIdx.x) * K) * d + c;
#pragma unroll
  for (int k = 0; k < K; ++k) pc[(long)k * d] = acc[k];
}

// BatchNorm1d (train mode, statistics over every (b, t) incl. padded frames, as nn.BatchNorm1d on
// (B, C, T)): y = (x - mean) * rstd * gamma + beta and xhat for the backward.
__global__ __launch_bounds__(256) void bn_apply_kernel(const float* __restrict__ x, const float* __restrict__ mean,
                                                       const float* __restrict__ rstd, const float* __restrict__ gam,
                                                       const float* __restrict__ bet, long rows, int d,
                                                       float* __restrict__ y, float* __restrict__ xhat) {
  const long n = rows * d;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const int c = (int)(i % d);
    const float h = (x[i] - mean[c]) * rstd[c];
    if (xhat) xhat[i] = h;
    y[i] = h * gam[c] + bet[c];
  }
}
// per channel: mean = s1 / n, var = s2 / n (s2 = sum (x - mean)^2), rstd, running stats update
__global__ void bn_stats_kernel(const float* __restrict__ s1, const float* __restrict__ s2, long n, int d,
                                float momentum, float* __restrict__ mean, float* __restrict__ rstd,
                                float* __restrict__ run_mean, float* __restrict__ run_var, int pass) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= d) return;
  if (pass == 0) {
    mean[c] = s1[c] / (float)n;
  } else {
    const float var = s2[c] / (float)n;
    rstd[c] = 1.0f / sqrtf(var + 1e-5f);
    if (run_mean) {
      run_mean[c] = (1.0f - momentum) * run_mean[c] + momentum * mean[c];
      run_var[c] = (1.0f - momentum) * run_var[c] + momentum * (n > 1 ? var * (float)n / (float)(n - 1) : var);
    }
  }
}
__global__ __launch_bounds__(256) void sq_dev_kernel(const float* __restrict__ x, const float* __restrict__ mean, long rows,
                                                     int d, float* __restrict__ out) {
  const long n = rows * d;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const float v = x[i] - mean[i % d];
    out[i] = v * v;
  }
}
// BatchNorm backward given the column sums sdy = sum dy, sdyx = sum dy * xhat over the n rows:
//   dx = gamma * rstd * (dy - sdy / n - xhat * sdyx / n)
__global__ __launch_bounds__(256) void bn_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ xhat,
                                                     const float* __restrict__ gam, const float* __restrict__ rstd,
                                                     const float* __restrict__ sdy, const float* __restrict__ sdyx,
                                                     long rows, int d, float* __restrict__ dx) {
  const long n = rows * d;
  const float inv = 1.0f / (float)rows;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const int c = (int)(i % d);
    dx[i] = gam[c] * rstd[c] * (dy[i] - sdy[c] * inv - xhat[i] * sdyx[c] * inv);
  }
}
__global__ __launch_bounds__(256) void mul_kernel(const float* __restrict__ a, const float* __restrict__ b, long n,
                                                  float* __restrict__ out) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) out[i] = a[i] * b[i];
}

unsigned ew_grid(long n) { return (unsigned)std::min<long>((n + 255) / 256, 8192); }

}  // namespace

void pack_matrix(int dtype, const float* src, long src_ld, int rows, int cols, bool transpose, void* dst, long dst_ld,
                 int rows_pad, int cols_pad, hipStream_t st) {
  if (rows_pad <= 0 || cols_pad <= 0) return;
  static const int rows_path = [] { const char* e = getenv("CFM_PACK_ROWS"); return e ? atoi(e) : 1; }();
  if (rows_path && !transpose && dst_ld % 2 == 0 && cols_pad % 2 == 0 && rows > 0 && cols > 0) {
    const dim3 g((unsigned)std::min<long>(((long)rows_pad + 3) / 4, 32768)), b(256);
    if (dtype == DT_F32)
      cfm_launch(pack_rows_kernel<float>, g, b, 0, st, src, src_ld, rows, cols, (float*)dst, dst_ld, rows_pad, cols_pad);
    else
      cfm_launch(pack_rows_kernel<bf16_t>, g, b, 0, st, src, src_ld, rows, cols, (bf16_t*)dst, dst_ld, rows_pad, cols_pad);
    return;
  }
  const dim3 grid((cols_pad + 31) / 32, (rows_pad + 31) / 32), block(256);
  if (dtype == DT_F32)
    cfm_launch(pack_kernel<float>, grid, block, 0, st, src, src_ld, rows, cols, (int)transpose, (float*)dst, dst_ld,
               rows_pad, cols_pad);
  else
    cfm_launch(pack_kernel<bf16_t>, grid, block, 0, st, src, src_ld, rows, cols, (int)transpose, (bf16_t*)dst, dst_ld,
               rows_pad, cols_pad);
}

size_t col_sums_ws(int M, int N) {
  const int nchunks = (M + kColRows - 1) / kColRows;
  return (size_t)nchunks * N * 4;
}

void col_sums(const float* src, long ld, int M, int N, float* out, int accumulate, float* ws, hipStream_t st) {
  if (M <= 0 || N <= 0) return;
  const int nchunks = (M + kColRows - 1) / kColRows;
  cfm_launch(colsum_partial_kernel, dim3((N + 63) / 64, nchunks), dim3(256), 0, st, src, ld, M, N, ws);
  cfm_launch(colsum_final_kernel, dim3((N + 15) / 16), dim3(256), 0, st, (const float*)ws, nchunks, N, out, accumulate);
}

void layernorm_backward(const float* x, const float* w, const float* dy, int M, int d, float* dx, int accumulate,
                        float* prod, hipStream_t st) {
  if (M <= 0) return;
  const dim3 grid((M + 3) / 4), block(256);
  const int d4 = d / 4;
  if (d4 <= 64) cfm_launch(layernorm_bwd_kernel<1>, grid, block, 0, st, x, w, dy, M, d, dx, accumulate, prod);
  else if (d4 <= 128) cfm_launch(layernorm_bwd_kernel<2>, grid, block, 0, st, x, w, dy, M, d, dx, accumulate, prod);
  else if (d4 <= 256) cfm_launch(layernorm_bwd_kernel<4>, grid, block, 0, st, x, w, dy, M, d, dx, accumulate, prod);
  else cfm_launch(layernorm_bwd_kernel<8>, grid, block, 0, st, x, w, dy, M, d, dx, accumulate, prod);
}

void swish_backward(const float* z, const float* du, float* dz, long n, hipStream_t st) {
  if (n <= 0) return;
  cfm_launch(swish_bwd_kernel, dim3((unsigned)std::min<long>((n + 255) / 256, 4096)), dim3(256), 0, st, z, du, dz, n);
}

}  // namespace cfm

using namespace cfm;

namespace {
// CFM_DW_DT / CFM_DW_DTW (A/B measurements): frames per block of the depthwise-conv backward kernels,
// 16 (default), 32 or 64; anything else is refused rather than silently replaced
int dw_frames_env(const char* name) {
  const char* e = getenv(name);
  if (!e) return 16;
  const int v = atoi(e);
  if (v != 16 && v != 32 && v != 64) {
    fprintf(stderr, "libcfm: %s=%s is not 16, 32 or 64\n", name, e);
    fail(CFM_ERR_INVALID_ARG, "CFM_DW_DT / CFM_DW_DTW must be 16, 32 or 64");
  }
  return v;
}
}  // namespace

namespace {

struct LinBwdWs {
  long a1, wt, a2, b2, cs, total;
  long Np64, Kp256, Mp, Kp;
};

LinBwdWs lin_bwd_ws(int dt, int M, int K, int N) {
  LinBwdWs w;
  const int es = dtype_size(dt);
  const long kg = GEMM_BK_BYTES / es;
  w.Np64 = round_up(N, kg);
  w.Kp256 = round_up(K, GEMM_BN);
  w.Kp = round_up(K, kg);
  w.Mp = round_up(M, kg);
  const long Np256 = round_up(N, GEMM_BN);
  long off = 0;
  auto take = [&](long bytes) { const long o = off; off = round_up(off + bytes, 256); return o; };
  w.a1 = take((long)M * w.Np64 * es);        // dy rows            [M][Np64]
  w.wt = take(w.Kp256 * w.Np64 * es);        // W^T                [Kp256][Np64]
  w.a2 = take(Np256 * w.Mp * es);            // dy^T               [N][Mp]
  w.b2 = take(w.Kp256 * w.Mp * es);          // x^T                [Kp256][Mp]
  w.cs = take((long)col_sums_ws(M, N));
  w.total = off + 4096;                      // + zero page
  return w;
}

GemmEpi epi_out_f32(float* X, long ldx) {
  GemmEpi e;
  std::memset(&e, 0, sizeof(e));
  e.mode = EPI_SCALE_F32;
  e.alpha = 1.0f;
  e.X = X;
  e.ldx = ldx;
  return e;
}

}  // namespace

extern "C" {

cfm_status cfm_op_glu_backward(const float* pre, const float* dy, const int32_t* lens, int B, int Tp, int d, float* dpre,
                               void* stream) {
  return guarded([&] {
    if (!pre || !dy || !dpre) fail(CFM_ERR_INVALID_ARG, "null argument");
    const long rows = (long)B * Tp;
    cfm_launch(glu_bwd_kernel, dim3(ew_grid(rows * d)), dim3(256), 0, (hipStream_t)stream, pre, dy, lens, Tp, d, rows,
               dpre);
    HIP_OK(hipGetLastError());
  });
}

size_t cfm_op_dwconv_backward_ws_size(int B, int Tp, int d, int K) {
  const long nt = (Tp + 15) / 16;   // weight-gradient partials of 16-frame blocks (the finest split)
  return (size_t)round_up((long)B * nt * K * d * 4, 256) +
         std::max(col_sums_ws((int)(B * nt), K * d), col_sums_ws(B * Tp, d)) + 256;
}

cfm_status cfm_op_dwconv_backward(const float* x, const float* w, const float* dy, int B, int Tp, int d, int K,
                                  float* dx, float* dw, float* db, void* ws, size_t ws_bytes, void* stream) {
  return guarded([&] {
    if (!x || !w || !dy) fail(CFM_ERR_INVALID_ARG, "null argument");
    if (K != 31) fail(CFM_ERR_UNSUPPORTED, "depthwise backward is built for kernel size 31");
    if (!ws || ws_bytes < cfm_op_dwconv_backward_ws_size(B, Tp, d, K)) fail(CFM_ERR_WORKSPACE, "workspace too small");
    hipStream_t st = (hipStream_t)stream;
    // frames per block of the input-gradient (CFM_DW_DT) and weight-gradient (CFM_DW_DTW) kernels:
    // 16 (more blocks in flight for these latency-bound kernels: train 32.46-32.53 against 32.60-32.66
    // ms/step for 32, 33.06-33.13 against 32.57-32.67 for 64); 32 / 64 selectable for A/B runs
    static const int dtx = dw_frames_env("CFM_DW_DT");
    static const int dtw = dw_frames_env("CFM_DW_DTW");
    const int nt16 = (Tp + 15) / 16;
    auto grid_of = [&](int dt_) { return dim3((Tp + dt_ - 1) / dt_, (d + 255) / 256, B); };
    const dim3 block(256);
    if (dx) {
      if (dtx == 64) cfm_launch(dwconv_bwd_x_kernel<31, 64>, grid_of(64), block, 0, st, dy, w, Tp, d, dx);
      else if (dtx == 16) cfm_launch(dwconv_bwd_x_kernel<31, 16>, grid_of(16), block, 0, st, dy, w, Tp, d, dx);
      else cfm_launch(dwconv_bwd_x_kernel<31, 32>, grid_of(32), block, 0, st, dy, w, Tp, d, dx);
    }
    const int DTW = (dtw == 16 || dtw == 64) ? dtw : 32;
    const int nt = (Tp + DTW - 1) / DTW;
    float* part = (float*)ws;
    float* cs = (float*)((char*)ws + round_up((long)B * nt16 * K * d * 4, 256));
    if (dw) {
      if (DTW == 64) cfm_launch(dwconv_bwd_w_kernel<31, 64>, grid_of(64), block, 0, st, x, dy, Tp, d, part);
      else if (DTW == 16) cfm_launch(dwconv_bwd_w_kernel<31, 16>, grid_of(16), block, 0, st, x, dy, Tp, d, part);
      else cfm_launch(dwconv_bwd_w_kernel<31, 32>, grid_of(32), block, 0, st, x, dy, Tp, d, part);
      // dw[c][k] = sum over the B * nt partial blocks of partial[blk][k][c]: column sums of a
      // (B*nt) x (K*d) matrix, then the [k][c] result transposed to the reference (d, 1, K) layout
      col_sums(part, (long)K * d, B * nt, K * d, part + (long)B * nt * K * d - (long)K * d, 0, cs, st);
      pack_matrix(DT_F32, part + (long)B * nt * K * d - (long)K * d, d, K, d, true, dw, K, d, K, st);
    }
    if (db) col_sums(dy, d, B * Tp, d, db, 0, cs, st);
    HIP_OK(hipGetLastError());
  });
}

size_t cfm_op_batchnorm_train_ws_size(int rows, int d) {
  return (size_t)round_up((long)rows * d * 4, 256) + 4 * round_up((long)d * 4, 256) + col_sums_ws(rows, d) + 256;
}

cfm_status cfm_op_batchnorm_train_forward(const float* x, int rows, int d, const float* gamma, const float* beta,
                                          float momentum, float* run_mean, float* run_var, float* y, float* xhat,
                                          float* mean, float* rstd, void* ws, size_t ws_bytes, void* stream) {
  return guarded([&] {
    if (!x || !gamma || !beta || !y || !mean || !rstd) fail(CFM_ERR_INVALID_ARG, "null argument");
    if (!ws || ws_bytes < cfm_op_batchnorm_train_ws_size(rows, d)) fail(CFM_ERR_WORKSPACE, "workspace too small");
    hipStream_t st = (hipStream_t)stream;
    char* b = (char*)ws;
    float* tmp = (float*)b;
    float* s1 = (float*)(b + round_up((long)rows * d * 4, 256));
    float* s2 = (float*)((char*)s1 + round_up((long)d * 4, 256));
    float* cs = (float*)((char*)s2 + round_up((long)d * 4, 256));
    const long n = (long)rows * d;
    col_sums(x, d, rows, d, s1, 0, cs, st);
    cfm_launch(bn_stats_kernel, dim3((d + 255) / 256), dim3(256), 0, st, (const float*)s1, (const float*)s2,
               (long)rows, d, momentum, mean, rstd, run_mean, run_var, 0);
    cfm_launch(sq_dev_kernel, dim3(ew_grid(n)), dim3(256), 0, st, x, (const float*)mean, (long)rows, d, tmp);
    col_sums(tmp, d, rows, d, s2, 0, cs, st);
    cfm_launch(bn_stats_kernel, dim3((d + 255) / 256), dim3(256), 0, st, (const float*)s1, (const float*)s2,
               (long)rows, d, momentum, mean, rstd, run_mean, run_var, 1);
    cfm_launch(bn_apply_kernel, dim3(ew_grid(n)), dim3(256), 0, st, x, (const float*)mean, (const float*)rstd, gamma,
               beta, (long)rows, d, y, xhat);
    HIP_OK(hipGetLastError());
  });
}

cfm_status cfm_op_batchnorm_train_backward(const float* dy, const float* xhat, int rows, int d, const float* gamma,
                                           const float* rstd, float* dx, float* dgamma, float* dbeta, void* ws,
                                           size_t ws_bytes, void* stream) {
  return guarded([&] {
    if (!dy || !xhat || !gamma || !rstd || !dx) fail(CFM_ERR_INVALID_ARG, "null argument");
    if (!ws || ws_bytes < cfm_op_batchnorm_train_ws_size(rows, d)) fail(CFM_ERR_WORKSPACE, "workspace too small");
    hipStream_t st = (hipStream_t)stream;
    char* b = (char*)ws;
    float* tmp = (float*)b;
    float* sdy = (float*)(b + round_up((long)rows * d * 4, 256));
    float* sdyx = (float*)((char*)sdy + round_up((long)d * 4, 256));
    float* cs = (float*)((char*)sdyx + 3 * round_up((long)d * 4, 256));
    const long n = (long)rows * d;
    col_sums(dy, d, rows, d, sdy, 0, cs, st);
    cfm_launch(mul_kernel, dim3(ew_grid(n)), dim3(256), 0, st, dy, xhat, n, tmp);
    col_sums(tmp, d, rows, d, sdyx, 0, cs, st);
    if (dgamma) HIP_OK(hipMemcpyAsync(dgamma, sdyx, (size_t)d * 4, hipMemcpyDeviceToDevice, st));
    if (dbeta) HIP_OK(hipMemcpyAsync(dbeta, sdy, (size_t)d * 4, hipMemcpyDeviceToDevice, st));
    cfm_launch(bn_bwd_kernel, dim3(ew_grid(n)), dim3(256), 0, st, dy, xhat, gamma, rstd, (const float*)sdy,
               (const float*)sdyx, (long)rows, d, dx);
    HIP_OK(hipGetLastError());
  });
}

size_t cfm_op_layernorm_backward_ws_size(int rows, int d) {
  return (size_t)round_up((long)rows * d * 4, 256) + col_sums_ws(rows, d) + 256;
}

cfm_status cfm_op_layernorm_backward(const float* x, int rows, int d, const float* w, const float* dy, float* dx,
                                     int accumulate, float* dw, float* db, void* ws, size_t ws_bytes, void* stream) {
  return guarded([&] {
    if (!x || !w || !dy || !dx) fail(CFM_ERR_INVALID_ARG, "null argument");
    if (d % 4 || d > 2048) fail(CFM_ERR_UNSUPPORTED, "d must be a multiple of 4 and <= 2048");
    if (!ws || ws_bytes < cfm_op_layernorm_backward_ws_size(rows, d)) fail(CFM_ERR_WORKSPACE, "workspace too small");
    hipStream_t st = (hipStream_t)stream;
    float* prod = (float*)ws;
    float* cs = (float*)((char*)ws + round_up((long)rows * d * 4, 256));
    layernorm_backward(x, w, dy, rows, d, dx, accumulate, prod, st);
    if (dw) col_sums(prod, d, rows, d, dw, 0, cs, st);
    if (db) col_sums(dy, d, rows, d, db, 0, cs, st);
    HIP_OK(hipGetLastError());
  });
}

size_t cfm_op_linear_backward_ws_size(int dtype, int M, int K, int N) {
  return (size_t)lin_bwd_ws(dtype == CFM_COMPUTE_FP32 ? DT_F32 : DT_BF16, M, K, N).total;
}

cfm_status cfm_op_linear_backward(int dtype, const float* x, int M, int K, const float* w, int N, const float* dy,
                                  float* dx, float* dw, float* db, void* ws, size_t ws_bytes, void* stream) {
  return guarded([&] {
    if (!x || !w || !dy) fail(CFM_ERR_INVALID_ARG, "null argument");
    if (M <= 0 || K <= 0 || N <= 0 || K % 4) fail(CFM_ERR_INVALID_ARG, "bad sizes (K % 4 == 0 required)");
    refuse_half_training(dtype == CFM_COMPUTE_FP32, "cfm_op_linear_backward");
    const int dt = dtype == CFM_COMPUTE_FP32 ? DT_F32 : DT_BF16;
    const LinBwdWs l = lin_bwd_ws(dt, M, K, N);
    if (!ws || ws_bytes < (size_t)l.total) fail(CFM_ERR_WORKSPACE, "workspace too small");
    hipStream_t st = (hipStream_t)stream;
    char* b = (char*)ws;
    char* zero = b + l.total - 4096;
    HIP_OK(hipMemsetAsync(zero, 0, 4096, st));
    if (dx) {   // dx (M, K) = dy (M, N) . W (N, K): A = dy rows, packed operand W^T [K][N]
      pack_matrix(dt, dy, N, M, N, false, b + l.a1, l.Np64, M, (int)l.Np64, st);
      pack_matrix(dt, w, K, N, K, true, b + l.wt, l.Np64, (int)l.Kp256, (int)l.Np64, st);
      gemm(dt, b + l.a1, l.Np64, M, N, b + l.wt, (int)l.Np64, K, epi_out_f32(dx, K), zero, st);
    }
    if (dw) {   // dw (N, K) = dy^T (N, M) . x (M, K): A = dy^T [N][Mp], packed operand x^T [K][Mp]
      pack_matrix(dt, dy, N, M, N, true, b + l.a2, l.Mp, N, (int)l.Mp, st);
      pack_matrix(dt, x, K, M, K, true, b + l.b2, l.Mp, (int)l.Kp256, (int)l.Mp, st);
      gemm(dt, b + l.a2, l.Mp, N, M, b + l.b2, (int)l.Mp, K, epi_out_f32(dw, K), zero, st);
    }
    if (db) col_sums(dy, N, M, N, db, 0, (float*)(b + l.cs), st);
    HIP_OK(hipGetLastError());
  });
}

cfm_status cfm_op_swish_backward(const float* z, const float* du, float* dz, int64_t n, void* stream) {
  return guarded([&] {
    if (!z || !du || !dz) fail(CFM_ERR_INVALID_ARG, "null argument");
    swish_backward(z, du, dz, n, (hipStream_t)stream);
    HIP_OK(hipGetLastError());
  });
}

}  // extern "C"
