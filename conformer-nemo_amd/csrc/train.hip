// Whole-encoder training step (SURVEY §8 rows a16 + e; BASELINE config 3): a stream-ordered
// train-mode forward that records an activation tape, and the backward that replays it in reverse
// and writes every parameter gradient in the reference's state_dict layout.
//
// Reference semantics followed (conformer_modules.py:88-200, multi_head_attention.py:69-316,
// subsampling.py:99-176, conformer_encoder.py:236-281) in training mode:
//   * dropout p = `dropout` on the embedding (RelPositionalEncoding.forward :316), inside both
//     feed-forwards (ConformerFeedForward :198) and on the four residual branches (:101-118);
//     masks come from a counter-based hash of (seed, site, element) so the backward regenerates
//     them instead of storing them;
//   * BatchNorm1d with batch statistics over all B*T' frames (padding included) and the momentum
//     update of running_mean / running_var (unbiased variance); optionally synchronised across
//     ranks (SyncBatchNorm, conformer_ctc_bpe.yaml:175) through a host-called sum-allreduce;
//   * everything else exactly as the eval forward (encoder.hip), from the same kernels.
// Weights are read from the caller's fp32 parameter tensors each step (packed into the workspace
// per layer), so an optimizer can update them in place between steps with no re-registration.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/cfm_train.h"
#include "cfm_abi.h"
#include "cfm_common.h"
#include "cfm_encoder_impl.h"
#include "cfm_kernels.h"

using namespace cfm;

namespace {

// ---------------------------------------------------------------------------------------------
// dropout masks: keep(e) iff hash(seed, site, e) >= thr, thr = p * 2^32; kept values * 1/(1-p)
// ---------------------------------------------------------------------------------------------
unsigned ew_grid(long n) { return (unsigned)std::max<long>(1, std::min<long>((n + 255) / 256, 8192)); }

// ---------------------------------------------------------------------------------------------
// operand packing
// ---------------------------------------------------------------------------------------------
// dst[i][j] = scale * fn(src)[transpose ? (j, i) : (i, j)] in the compute type, zero outside src.
// fn 0 = identity, 1 = dropout(swish(.)) (the FFN hidden recomputed from its pre-activation; the
// mask index is the source element (row * cols + col)).  Destination row `ones_row` (transposed
// packs) is set to 1 over the source rows: appended to the x^T operand of a weight-gradient GEMM it
// makes the GEMM also produce the bias gradient (sum of dy over rows).
// 64x64 LDS tiles; 16-byte (fp32) / 8-byte (bf16) source loads along source rows and 16-byte stores
// along destination rows when the strides and base pointers allow (src_vec / dst_vec).
template <typename Tin, typename Tout>
CFM_DEV void tpack_tile(float (*tile)[65], int bx, int by, const Tin* __restrict__ src, long src_ld, int rows,
                        int cols, int transpose, float scale, int fn, Drop drop, Tout* __restrict__ dst, long dst_ld,
                        int rows_pad, int cols_pad, int ones_row, int src_vec, int dst_vec) {
  const int i0 = by * 64, j0 = bx * 64;
  const int sr0 = transpose ? j0 : i0, sc0 = transpose ? i0 : j0;
  // 16-byte source loads: 4 fp32 or 8 bf16 values per thread and pass
  constexpr int VI = sizeof(Tin) == 2 ? 8 : 4, TPR = 64 / VI, LPP = 256 / TPR;
  const int cv = threadIdx.x % TPR, r = threadIdx.x / TPR;
#pragma unroll
  for (int pass = 0; pass < 64 / LPP; ++pass) {
    const int rr = r + LPP * pass, cc = VI * cv;
    const int si = sr0 + rr, sj = sc0 + cc;
    float v[VI];
#pragma unroll
    for (int e = 0; e < VI; ++e) v[e] = 0.0f;
    if (si < rows) {
      const Tin* sp = src + (long)si * src_ld + sj;
      if (src_vec == 2 && sj + VI - 1 < cols) {
        Vec16<Tin>::to_f32(*(const uint4*)sp, v);
      } else if (sizeof(Tin) == 2 && src_vec == 1 && sj + VI - 1 < cols) {   // 8-byte aligned bf16 rows
#pragma unroll
        for (int h = 0; h < VI / 4; ++h) {
          const uint2 t = *(const uint2*)(sp + 4 * h);
          v[4 * h] = bf2f((bf16_t)(t.x & 0xffffu)); v[4 * h + 1] = bf2f((bf16_t)(t.x >> 16));
          v[4 * h + 2] = bf2f((bf16_t)(t.y & 0xffffu)); v[4 * h + 3] = bf2f((bf16_t)(t.y >> 16));
        }
      } else {
#pragma unroll
        for (int e = 0; e < VI; ++e)
          if (sj + e < cols) v[e] = ld_f<Tin>(sp + e);
      }
#pragma unroll
      for (int e = 0; e < VI; ++e) {
        if (fn == 1 && sj + e < cols) v[e] = swishf(v[e]) * drop_mul(drop, (uint64_t)si * cols + sj + e);
        v[e] *= scale;
      }
    }
#pragma unroll
    for (int e = 0; e < VI; ++e) {
      if (transpose) tile[cc + e][rr] = v[e];
      else tile[rr][cc + e] = v[e];
    }
  }
  __syncthreads();
  constexpr int VE = 16 / (int)sizeof(Tout);
  constexpr int CPR = 64 / VE, RPP = 256 / CPR;
  const int q = threadIdx.x % CPR, k0 = threadIdx.x / CPR;
  for (int k = k0; k < 64; k += RPP) {
    const int di = i0 + k;
    if (di >= rows_pad) break;
    const int dj = j0 + q * VE;
    float o[VE];
#pragma unroll
    for (int e = 0; e < VE; ++e) {
      o[e] = tile[k][q * VE + e];
      if (di == ones_row) o[e] = (dj + e < rows) ? 1.0f : 0.0f;   // bias column of a weight-gradient GEMM
    }
    Tout* dp = dst + (long)di * dst_ld + dj;
    if (dst_vec && dj + VE <= cols_pad) {
      *(uint4*)dp = Vec16<Tout>::from_f32(o);
    } else {
#pragma unroll
      for (int e = 0; e < VE; ++e)
        if (dj + e < cols_pad) st_f<Tout>(dp + e, o[e]);
    }
  }
}

template <typename Tin, typename Tout>
__global__ __launch_bounds__(256) void tpack_kernel(const Tin* __restrict__ src, long src_ld, int rows, int cols,
                                                      int transpose, float scale, int fn, Drop drop,
                                                      Tout* __restrict__ dst, long dst_ld, int rows_pad,
                                                      int cols_pad, int ones_row, int src_vec, int dst_vec) {
  __shared__ float tile[64][65];                      // [dst row][dst col] of this block
  tpack_tile<Tin, Tout>(tile, blockIdx.x, blockIdx.y, src, src_ld, rows, cols, transpose, scale, fn, drop, dst, dst_ld,
                        rows_pad, cols_pad, ones_row, src_vec, dst_vec);
}

// Non-transposed fp32 -> bf16 pack (no LDS tile): dst[i][8q .. 8q+7] = scale * src[i][...],
// zero outside src; rows of cp elements (cp % 8 == 0), 16-byte aligned rows on both sides.
__global__ __launch_bounds__(256) void pack_rows_kernel(const float* __restrict__ src, long src_ld, int rows, int cols,
                                                        float scale, bf16_t* __restrict__ dst, long dst_ld, int rp,
                                                        int cp) {
  const int q8 = cp >> 3;
  const long n = (long)rp * q8;
  for (long t = blockIdx.x * 256L + threadIdx.x; t < n; t += (long)gridDim.x * 256) {
    const int i = (int)(t / q8), j = 8 * (int)(t - (long)i * q8);
    float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (i < rows) {
      const float* sp = src + (long)i * src_ld + j;
      if (j + 8 <= cols) {
        const float4 a = *(const float4*)sp, b = *(const float4*)(sp + 4);
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (j + e < cols) v[e] = sp[e];
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] *= scale;
    }
    *(uint4*)(dst + (long)i * dst_ld + j) = Vec16<bf16_t>::from_f32(v);
  }
}

// Both packs of a dense fp32 output gradient dy (rows x cols) from one read: dA = dy in the compute
// type ([rpA][ldA], the dgrad GEMM's A operand) and dT = dy^T ([rpT][ldT], the wgrad GEMM's A
// operand), zero outside dy.  The grid covers the larger of the two extents per dimension.
template <typename Tout>
__global__ __launch_bounds__(256) void tpack2_kernel(const float* __restrict__ src, long src_ld, int rows, int cols,
                                                       Tout* __restrict__ dA, long ldA, int rpA, int cpA,
                                                       Tout* __restrict__ dT, long ldT, int rpT, int cpT,
                                                       int src_vec, int vecA, int vecT, float scale, Drop dr) {
  __shared__ float tile[64][65];   // [src row][src col]
  const int i0 = blockIdx.y * 64, j0 = blockIdx.x * 64;
  const int c4 = threadIdx.x & 15, r = threadIdx.x >> 4;
#pragma unroll
  for (int pass = 0; pass < 4; ++pass) {
    const int rr = r + 16 * pass, cc = 4 * c4;
    const int si = i0 + rr, sj = j0 + cc;
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    if (si < rows) {
      const float* sp = src + (long)si * src_ld + sj;
      if (src_vec && sj + 3 < cols) {
        const float4 t = *(const float4*)sp;
        v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (sj + e < cols) v[e] = sp[e];
      }
    }
    if (scale != 1.0f || dr.thr) {   // dy = scale * dropout'(g): the residual branch's dropout backward
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] *= scale * drop_mul(dr, (uint64_t)si * (uint64_t)src_ld + (uint64_t)(sj + e));
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) tile[rr][cc + e] = v[e];
  }
  __syncthreads();
  constexpr int VE = 16 / (int)sizeof(Tout);
  constexpr int CPR = 64 / VE, RPP = 256 / CPR;
  const int q = threadIdx.x % CPR, k0 = threadIdx.x / CPR;
  for (int k = k0; k < 64; k += RPP) {
    float o[VE];
    const int ai = i0 + k, aj = j0 + q * VE;   // dA[ai][aj ..]
    if (ai < rpA && aj < cpA) {
#pragma unroll
      for (int e = 0; e < VE; ++e) o[e] = tile[k][q * VE + e];
      Tout* dp = dA + (long)ai * ldA + aj;
      if (vecA && aj + VE <= cpA) {
        *(uint4*)dp = Vec16<Tout>::from_f32(o);
      } else {
#pragma unroll
        for (int e = 0; e < VE; ++e)
          if (aj + e < cpA) st_f<Tout>(dp + e, o[e]);
      }
    }
    const int ti = j0 + k, tj = i0 + q * VE;   // dT[ti][tj ..] = dy[tj ..][ti]
    if (ti < rpT && tj < cpT) {
#pragma unroll
      for (int e = 0; e < VE; ++e) o[e] = tile[q * VE + e][k];
      Tout* dp = dT + (long)ti * ldT + tj;
      if (vecT && tj + VE <= cpT) {
        *(uint4*)dp = Vec16<Tout>::from_f32(o);
      } else {
#pragma unroll
        for (int e = 0; e < VE; ++e)
          if (tj + e < cpT) st_f<Tout>(dp + e, o[e]);
      }
    }
  }
}

// Up to 16 fp32 -> compute-type (or fp32) packs of parameters in one launch: a layer's weight
// matrices and zero-padded bias rows, each job a tpack over its own range of grid blocks.
struct PackJob {
  const float* src;
  void* dst;
  int ld_src, rows, cols, tr, ld_dst, rows_pad, cols_pad, out_f32, src_vec, dst_vec, tiles_x, tile0;
};
struct PackList {
  PackJob j[16];
  int count;
};
template <typename T>
__global__ __launch_bounds__(256) void tpack_multi_kernel(PackList l) {
  __shared__ float tile[64][65];
  int k = 0;
  while (k + 1 < l.count && (int)blockIdx.x >= l.j[k + 1].tile0) ++k;
  const PackJob& J = l.j[k];
  const int t = (int)blockIdx.x - J.tile0, by = t / J.tiles_x, bx = t - by * J.tiles_x;
  const Drop none{0, 0, 1.0f};
  if (J.out_f32)
    tpack_tile<float, float>(tile, bx, by, J.src, J.ld_src, J.rows, J.cols, J.tr, 1.0f, 0, none, (float*)J.dst,
                             J.ld_dst, J.rows_pad, J.cols_pad, -1, J.src_vec, J.dst_vec);
  else
    tpack_tile<float, T>(tile, bx, by, J.src, J.ld_src, J.rows, J.cols, J.tr, 1.0f, 0, none, (T*)J.dst, J.ld_dst,
                         J.rows_pad, J.cols_pad, -1, J.src_vec, J.dst_vec);
}

// dst[i] = i < N && src ? src[i] : 0 for i < npad (GEMM bias arrays, zero-padded to the N granule)
__global__ __launch_bounds__(256) void bias_pad_kernel(const float* __restrict__ src, int N, float* __restrict__ dst,
                                                       int npad) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < npad) dst[i] = (src && i < N) ? src[i] : 0.0f;
}

// Up to 8 independent device copies in one launch (grid.y = copy index): the per-layer gradient
// scatters that would otherwise each cost a runtime copy kernel.
struct CopyList {
  const float* src[8];
  float* dst[8];
  long n[8];
  int count;
};
__global__ __launch_bounds__(256) void copy_multi_kernel(CopyList l) {
  const int c = blockIdx.y;
  if (c >= l.count || l.dst[c] == nullptr) return;
  const float* s = l.src[c];
  float* d = l.dst[c];
  const long n = l.n[c];
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) d[i] = s[i];
}

// Head-padded row gather: dst row n = (part, head, dd) of `parts` stacked (H*dk, K) fp32 sources,
// head dims padded dk -> dkp (the layout the QKV epilogue and attention kernels consume); K = 1
// packs bias vectors (fp32 out).
template <typename T>
__global__ __launch_bounds__(256) void pack_heads_kernel(const float* __restrict__ s0, const float* __restrict__ s1,
                                                         const float* __restrict__ s2, int parts, int H, int dk,
                                                         int dkp, int K, T* __restrict__ dst, long Kp, int rows_pad) {
  const long n = (long)rows_pad * Kp;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const int r = (int)(i / Kp), k = (int)(i - (long)r * Kp);
    float v = 0.0f;
    if (r < parts * H * dkp && k < K) {
      const int part = r / (H * dkp), rr = r % (H * dkp), hh = rr / dkp, dd = rr % dkp;
      const float* s = part == 0 ? s0 : (part == 1 ? s1 : s2);
      if (dd < dk && s) v = s[(long)(hh * dk + dd) * K + k];
    }
    st_f<T>(dst + i, v);
  }
}

// Index-permuting packs of the subsampling weights (rows_pad x cols_pad destination):
//   0  Linear W (d, C*F2) [n][c*F2+f]  -> [n][f*C+c]          (channels-last flatten of conv2's output)
//   1  its transpose                   -> [f*C+c][n]
//   2  conv2 W (C, C, 3, 3)            -> [co][tap*C+ci]       (implicit-GEMM K order)
//   3  its transpose                   -> [tap*C+ci][co]
//   4  gradient un-permute, fp32: dst (d, C*F2) [n][c*F2+f] <- src [n][f*C+c]
//   5  gradient un-permute, fp32: dst (C, C, 3, 3)         <- src [co][tap*C+ci]
template <typename T>
__global__ __launch_bounds__(256) void perm_pack_kernel(const float* __restrict__ src, int mode, int C, int F2, int d,
                                                        T* __restrict__ dst, long ld, int rows_pad, int cols_pad) {
  const long n = (long)rows_pad * cols_pad;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const int r = (int)(i / cols_pad), q = (int)(i - (long)r * cols_pad);
    float v = 0.0f;
    switch (mode) {
      case 0: if (r < d && q < C * F2) { const int f = q / C, c = q % C; v = src[(long)r * C * F2 + (long)c * F2 + f]; } break;
      case 1: if (q < d && r < C * F2) { const int f = r / C, c = r % C; v = src[(long)q * C * F2 + (long)c * F2 + f]; } break;
      case 2: if (r < C && q < 9 * C) { const int tap = q / C, ci = q % C; v = src[((long)r * C + ci) * 9 + tap]; } break;
      case 3: if (q < C && r < 9 * C) { const int tap = r / C, ci = r % C; v = src[((long)q * C + ci) * 9 + tap]; } break;
      case 4: { const int c = q / F2, f = q % F2; v = src[(long)r * C * F2 + (long)f * C + c]; } break;
      case 5: { const int ci = q / 9, tap = q % 9; v = src[(long)r * 9 * C + (long)tap * C + ci]; } break;
    }
    st_f<T>(dst + (long)r * ld + q, v);
  }
}

// ---------------------------------------------------------------------------------------------
// elementwise forward pieces
// ---------------------------------------------------------------------------------------------
// xout = xin + alpha * dropout(br) (residual update, conformer_modules.py:101-118); xout may alias xin
__global__ __launch_bounds__(256) void resid_drop_kernel(const float* xin, const float* __restrict__ br, float alpha,
                                                         long n, Drop drop, float* xout) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    xout[i] = xin[i] + alpha * br[i] * drop_mul(drop, (uint64_t)i);
}
__global__ void fill_kernel(float* __restrict__ p, long n, float v) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) p[i] = v;
}
// y = alpha * dropout(x) (in place allowed)
__global__ __launch_bounds__(256) void scale_drop_kernel(const float* x, float alpha, long n, Drop drop, float* y) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    y[i] = alpha * x[i] * drop_mul(drop, (uint64_t)i);
}
// dropout_emb on the positional-embedding window (multi_head_attention.py:316, RelPositionalEncoding
// returns dropout_emb(pos_emb)): one mask for every layer, in the compute type (linear_pos's A operand)
template <typename T>
__global__ __launch_bounds__(256) void pe_drop_kernel(const T* __restrict__ pe, long n, Drop drop, T* __restrict__ out) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    st_f<T>(out + i, ld_f<T>(pe + i) * drop_mul(drop, (uint64_t)i));
}
// GLU(dim=1) + pad mask (conformer_modules.py:162-167): g = a * sigmoid(gate), 0 on padded frames;
// fp32 for the tape and the compute type for the depthwise conv.
template <typename T>
__global__ __launch_bounds__(256) void glu_fwd_kernel(const float* __restrict__ pre, const int32_t* __restrict__ lens,
                                                      int Tp, int d, long rows, float* __restrict__ g,
                                                      T* __restrict__ gt) {
  const long n = rows * d;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const long m = i / d;
    const int c = (int)(i - m * d);
    const int b = (int)(m / Tp), t = (int)(m - (long)b * Tp);
    const float a = pre[m * 2 * d + c], gg = pre[m * 2 * d + d + c];
    const float v = (!lens || t < lens[b]) ? a * (1.0f / (1.0f + expf(-gg))) : 0.0f;   // lens null: no pad mask
    g[i] = v;
    st_f<T>(gt + i, v);
  }
}

// ---------------------------------------------------------------------------------------------
// reductions (fixed order: bitwise reproducible)
// ---------------------------------------------------------------------------------------------
// Column reduction out[n] (+)= alpha * sum_r f(src[r][n]) with f 0: x, 1: x*y, 2: (x - mean[n])^2.
// Stage 1: block = 64 columns x 4 row lanes over a 256-row chunk (every row read is a coalesced
// 256-byte segment); stage 2 folds the chunks the same way.  Fixed order: bitwise reproducible.
constexpr int kRedRows = 256;
template <int F>
__global__ __launch_bounds__(256) void colred_partial_kernel(const float* __restrict__ src, const float* __restrict__ y,
                                                             const float* __restrict__ mean, long ld, int M, int N,
                                                             float* __restrict__ partial) {
  __shared__ float red[4][64];
  const int c = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int n = blockIdx.x * 64 + c;
  const int r0 = blockIdx.y * kRedRows, r1 = min(M, r0 + kRedRows);
  const int nc = min(n, N - 1);
  const float mu = F == 2 ? mean[nc] : 0.0f;
  float s = 0.0f;
#pragma unroll 8
  for (int r = r0 + rl; r < r1; r += 4) {
    const float v = src[(long)r * ld + nc];
    s += F == 0 ? v : (F == 1 ? v * y[(long)r * ld + nc] : (v - mu) * (v - mu));
  }
  red[rl][c] = s;
  __syncthreads();
  if (rl == 0 && n < N) partial[(long)blockIdx.y * N + n] = (red[0][c] + red[1][c]) + (red[2][c] + red[3][c]);
}
// stage 2: block = 16 columns x 16 chunk lanes (more blocks in flight for narrow N)
__global__ __launch_bounds__(256) void colred_final_kernel(const float* __restrict__ partial, int nchunks, int N,
                                                           float alpha, float* __restrict__ out, int accumulate) {
  __shared__ float red[16][17];
  const int c = threadIdx.x & 15, rl = threadIdx.x >> 4;
  const int n = blockIdx.x * 16 + c;
  const int nc = min(n, N - 1);
  float s = 0.0f;
#pragma unroll 8
  for (int k = rl; k < nchunks; k += 16) s += partial[(long)k * N + nc];
  red[rl][c] = s;
  __syncthreads();
  if (rl == 0 && n < N) {
    float v = 0.0f;
#pragma unroll
    for (int k = 0; k < 16; ++k) v += red[k][c];
    v *= alpha;
    out[n] = accumulate ? out[n] + v : v;
  }
}
// out[i] = sum_s part[s * n + i] (split-K partial slabs, fixed order), float4 when n % 4 == 0
__global__ __launch_bounds__(256) void slab_sum_kernel(const float* __restrict__ part, int S, long n,
                                                       float* __restrict__ out) {
  if ((n & 3) == 0) {
    const long n4 = n >> 2;
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
      float4 a = ((const float4*)part)[i];
      for (int s = 1; s < S; ++s) {
        const float4 b = ((const float4*)(part + (long)s * n))[i];
        a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
      }
      ((float4*)out)[i] = a;
    }
  } else {
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
      float a = part[i];
      for (int s = 1; s < S; ++s) a += part[(long)s * n + i];
      out[i] = a;
    }
  }
}
// Weight-gradient slabs with an appended bias column: part[s][n][0..K+4) ->
//   w[n][k] = sum_s part[s][n][k] (k < K), b[n] = sum_s part[s][n][K]
__global__ __launch_bounds__(256) void slab_sum_wb_kernel(const float* __restrict__ part, int S, int N, int K,
                                                          float* __restrict__ w, float* __restrict__ b) {
  const int ldk = K + 4;
  const long n = (long)N * ldk;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const int r = (int)(i / ldk), k = (int)(i - (long)r * ldk);
    if (k > K) continue;
    float a = part[i];
    for (int s2 = 1; s2 < S; ++s2) a += part[(long)s2 * n + i];
    if (k < K) { if (w) w[(long)r * K + k] = a; }
    else if (b) b[r] = a;
  }
}

// slab_sum_wb_kernel for K % 4 == 0 and a 16-byte aligned w: one float4 of a row per thread step
// (32-bit index math; the bias column K opens the row's last float4)
__global__ __launch_bounds__(256) void slab_sum_wb4_kernel(const float* __restrict__ part, int S, int N, int K,
                                                           float* __restrict__ w, float* __restrict__ b) {
  const int q4 = (K + 4) >> 2;
  const int n4 = N * q4;
  const long n = (long)N * (K + 4);
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n4; i += gridDim.x * 256) {
    const int r = i / q4, k = 4 * (i - r * q4);
    float4 a = ((const float4*)part)[i];
    for (int s2 = 1; s2 < S; ++s2) {
      const float4 c = ((const float4*)(part + (long)s2 * n))[i];
      a.x += c.x; a.y += c.y; a.z += c.z; a.w += c.w;
    }
    if (k < K) {
      if (w) *(float4*)(w + (long)r * K + k) = a;
    } else if (b) {
      b[r] = a.x;
    }
  }
}
void slab_sum_wb(const float* part, int S, int N, int K, float* w, float* b, hipStream_t st) {
  if (K % 4 == 0 && ((uintptr_t)w & 15) == 0 && (long)N * (K + 4) / 4 < (1L << 30)) {
    const long n4 = (long)N * (K + 4) / 4;
    cfm_launch(slab_sum_wb4_kernel, dim3(ew_grid(n4)), dim3(256), 0, st, part, S, N, K, w, b);
  } else {
    cfm_launch(slab_sum_wb_kernel, dim3(ew_grid((long)N * (K + 4))), dim3(256), 0, st, part, S, N, K, w, b);
  }
}

size_t colred_ws(long M, long N) { return (size_t)((M + kRedRows - 1) / kRedRows) * N * 4; }
void colred(const float* src, const float* y, const float* mean, long ld, int M, int N, int f, float alpha, float* out,
            int accumulate, float* ws, hipStream_t st) {
  if (N <= 0) return;
  if (M <= 0) {
    if (!accumulate) HIP_OK(hipMemsetAsync(out, 0, (size_t)N * 4, st));
    return;
  }
  const int nch = (M + kRedRows - 1) / kRedRows;
  const dim3 g1((N + 63) / 64, nch), b(256);
  if (f == 0) cfm_launch(colred_partial_kernel<0>, g1, b, 0, st, src, y, mean, ld, M, N, ws);
  else if (f == 1) cfm_launch(colred_partial_kernel<1>, g1, b, 0, st, src, y, mean, ld, M, N, ws);
  else cfm_launch(colred_partial_kernel<2>, g1, b, 0, st, src, y, mean, ld, M, N, ws);
  cfm_launch(colred_final_kernel, dim3((N + 15) / 16), b, 0, st, (const float*)ws, nch, N, alpha, out, accumulate);
}

// Up to 10 independent column reductions of [nchunks][N] partials in one launch (grid.y = entry; a null
// output is skipped): the weight and bias gradients of a layer's five LayerNorms.
struct ColredList {
  const float* p[10];
  float* o[10];
  int count;
};
__global__ __launch_bounds__(256) void colred_multi_kernel(ColredList l, int nchunks, int N) {
  __shared__ float red[16][17];
  const int y = blockIdx.y;
  if (y >= l.count || l.o[y] == nullptr) return;
  const float* partial = l.p[y];
  float* out = l.o[y];
  const int c = threadIdx.x & 15, rl = threadIdx.x >> 4;
  const int n = blockIdx.x * 16 + c;
  const int nc = min(n, N - 1);
  float s = 0.0f;
#pragma unroll 8
  for (int k = rl; k < nchunks; k += 16) s += partial[(long)k * N + nc];
  red[rl][c] = s;
  __syncthreads();
  if (rl == 0 && n < N) {
    float v = 0.0f;
#pragma unroll
    for (int k = 0; k < 16; ++k) v += red[k][c];
    out[n] = v;
  }
}

// Two independent column reductions of [nchunks][N] partials in one launch (grid.y = 0, 1; a null
// output is skipped): the LayerNorm weight and bias gradients.
__global__ __launch_bounds__(256) void colred_final2_kernel(const float* __restrict__ p0, float* __restrict__ o0,
                                                            const float* __restrict__ p1, float* __restrict__ o1,
                                                            int nchunks, int N) {
  __shared__ float red[16][17];
  const float* partial = blockIdx.y ? p1 : p0;
  float* out = blockIdx.y ? o1 : o0;
  if (out == nullptr) return;
  const int c = threadIdx.x & 15, rl = threadIdx.x >> 4;
  const int n = blockIdx.x * 16 + c;
  const int nc = min(n, N - 1);
  float s = 0.0f;
#pragma unroll 8
  for (int k = rl; k < nchunks; k += 16) s += partial[(long)k * N + nc];
  red[rl][c] = s;
  __syncthreads();
  if (rl == 0 && n < N) {
    float v = 0.0f;
#pragma unroll
    for (int k = 0; k < 16; ++k) v += red[k][c];
    out[n] = v;
  }
}

// LayerNorm backward (eps 1e-5, biased variance; torch.nn.LayerNorm) for 4 rows per wave, 16 rows per
// block, with the weight/bias gradient column partials reduced in-block (fixed order):
//   dx (+)= rstd * (g - mean(g) - xhat * mean(g * xhat)),  g = dy * w
//   pw[blk][c] = sum over the block's rows of dy * xhat,  pb[blk][c] = sum of dy
// pk (bf16, optional): the next consumer's GEMM operand, pk[row][c] = bf16(dx * pscale * dropout'(row*d + c))
// - what tpack2 would make of dx for that consumer, written here instead of re-read in another pass
// rows per wave (one in flight): 2 measured best (same-box training A/B: 30.66-30.84 ms/step against
// 30.94-31.08 at 4 and 30.57-30.73 against 30.44-30.56 at 1) - more blocks keep more rows in flight
#ifndef CFM_LN_ROWS
#define CFM_LN_ROWS 2
#endif
constexpr int kLnRowsPerWave = CFM_LN_ROWS;
template <int E4>
__global__ __launch_bounds__(256) void ln_bwd_fused_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                           const float* __restrict__ dy, int M, int d,
                                                           float* __restrict__ dx, int accumulate,
                                                           float* __restrict__ pw, float* __restrict__ pb,
                                                           bf16_t* __restrict__ pk, float pscale, Drop pdr) {
#pragma clang fp contract(off)
  __shared__ float4 red[2][4][64 * E4];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int d4 = d >> 2;
  const float4* wr = (const float4*)w;
  float4 wv4[E4], aw[E4], ab[E4];
#pragma unroll
  for (int e = 0; e < E4; ++e) {
    wv4[e] = wr[min(lane + 64 * e, d4 - 1)];
    aw[e] = make_float4(0, 0, 0, 0);
    ab[e] = make_float4(0, 0, 0, 0);
  }
  const float inv_d = 1.0f / (float)d;
  // the next row's x / dy loads are issued before this row's reductions (one row in flight per wave)
  const int row0 = (blockIdx.x * 4 + wv) * kLnRowsPerWave;
  float4 xn[E4], dn[E4];
  auto load_row = [&](int row) {
    const float4* xr = (const float4*)(x + (long)min(row, M - 1) * d);
    const float4* dr = (const float4*)(dy + (long)min(row, M - 1) * d);
#pragma unroll
    for (int e = 0; e < E4; ++e) {
      const int g = min(lane + 64 * e, d4 - 1);
      xn[e] = xr[g];
      dn[e] = dr[g];
    }
  };
  load_row(row0);
  for (int i = 0; i < kLnRowsPerWave; ++i) {
    const int row = row0 + i;
    if (row >= M) break;
    float4 xv[E4], dv[E4];
    float sx = 0.0f;
#pragma unroll
    for (int e = 0; e < E4; ++e) {
      const bool ok = lane + 64 * e < d4;
      xv[e] = ok ? xn[e] : make_float4(0, 0, 0, 0);
      dv[e] = ok ? dn[e] : make_float4(0, 0, 0, 0);
    }
    if (i + 1 < kLnRowsPerWave) load_row(row + 1);
#pragma unroll
    for (int e = 0; e < E4; ++e) sx += xv[e].x + xv[e].y + xv[e].z + xv[e].w;
    const float mean = wave_sum(sx) * inv_d;
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
      gv[e] = make_float4(dv[e].x * wv4[e].x, dv[e].y * wv4[e].y, dv[e].z * wv4[e].z, dv[e].w * wv4[e].w);
      if (lane + 64 * e < d4) {
        sg += gv[e].x + gv[e].y + gv[e].z + gv[e].w;
        sgx += gv[e].x * xh[e].x + gv[e].y * xh[e].y + gv[e].z * xh[e].z + gv[e].w * xh[e].w;
      }
    }
    const float mg = wave_sum(sg) * inv_d, mgx = wave_sum(sgx) * inv_d;
    float4* dxr = (float4*)(dx + (long)row * d);
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
        if (pk) {
          float f[4] = {o.x, o.y, o.z, o.w};
          if (pscale != 1.0f || pdr.thr) {
#pragma unroll
            for (int k = 0; k < 4; ++k)
              f[k] *= pscale * drop_mul(pdr, (uint64_t)row * (uint64_t)d + (uint64_t)(4 * g + k));
          }
          uint2 u;
          u.x = (uint32_t)f2bf(f[0]) | ((uint32_t)f2bf(f[1]) << 16);
          u.y = (uint32_t)f2bf(f[2]) | ((uint32_t)f2bf(f[3]) << 16);
          *(uint2*)(pk + (long)row * d + 4 * g) = u;
        }
        aw[e].x += dv[e].x * xh[e].x; aw[e].y += dv[e].y * xh[e].y;
        aw[e].z += dv[e].z * xh[e].z; aw[e].w += dv[e].w * xh[e].w;
        ab[e].x += dv[e].x; ab[e].y += dv[e].y; ab[e].z += dv[e].z; ab[e].w += dv[e].w;
      }
    }
  }
#pragma unroll
  for (int e = 0; e < E4; ++e) { red[0][wv][lane + 64 * e] = aw[e]; red[1][wv][lane + 64 * e] = ab[e]; }
  __syncthreads();
  for (int c4 = threadIdx.x; c4 < d4; c4 += 256) {
    float4 a = red[0][0][c4], b = red[1][0][c4];
    for (int k = 1; k < 4; ++k) {
      const float4 u = red[0][k][c4], v = red[1][k][c4];
      a.x += u.x; a.y += u.y; a.z += u.z; a.w += u.w;
      b.x += v.x; b.y += v.y; b.z += v.z; b.w += v.w;
    }
    ((float4*)(pw + (long)blockIdx.x * d))[c4] = a;
    ((float4*)(pb + (long)blockIdx.x * d))[c4] = b;
  }
}

// ---------------------------------------------------------------------------------------------
// BatchNorm (train) + Swish, and their backward
// ---------------------------------------------------------------------------------------------
// pass 0: mean = s1 / n; pass 1: rstd from s2 / n and the running-stat update (momentum, unbiased)
// n = cnt[0]: the frame count behind the sums -- summed over the ranks with them under SyncBatchNorm
// (ranks may hold different B x T'), so mean / var / the backward's 1/n use the global count
// (torch.nn.SyncBatchNorm all-gathers the per-rank counts the same way).  Pass 0 also keeps it at
// mean[d] (the tape) for the backward.
__global__ void bn_finalize_kernel(const float* __restrict__ s1, const float* __restrict__ s2,
                                   const float* __restrict__ cnt, int d,
                                   float momentum, float* __restrict__ mean, float* __restrict__ rstd,
                                   float* __restrict__ run_mean, float* __restrict__ run_var, int pass) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  const double n = (double)cnt[0];
  if (pass == 0 && c == 0) mean[d] = cnt[0];
  if (c >= d) return;
  if (pass == 0) {
    mean[c] = (float)((double)s1[c] / n);
  } else {
    const float var = (float)((double)s2[c] / n);
    rstd[c] = 1.0f / sqrtf(var + 1e-5f);
    if (run_mean) {
      const float unb = n > 1.0 ? (float)((double)s2[c] / (n - 1.0)) : var;
      run_mean[c] = (1.0f - momentum) * run_mean[c] + momentum * mean[c];
      run_var[c] = (1.0f - momentum) * run_var[c] + momentum * unb;
    }
  }
}
// xhat = (x - mean) * rstd (fp32 tape); s = swish(xhat * gamma + beta) in the compute type
template <typename T>
__global__ __launch_bounds__(256) void bn_swish_kernel(const float* __restrict__ x, const float* __restrict__ mean,
                                                       const float* __restrict__ rstd, const float* __restrict__ gam,
                                                       const float* __restrict__ bet, long rows, int d,
                                                       float* __restrict__ xhat, T* __restrict__ s) {
  const long n = rows * d;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const int c = (int)(i % d);
    const float h = (x[i] - mean[c]) * rstd[c];
    xhat[i] = h;
    st_f<T>(s + i, swishf(h * gam[c] + bet[c]));
  }
}
// dz = ds * swish'(xhat * gamma + beta)
__global__ __launch_bounds__(256) void bn_swish_bwd_kernel(const float* __restrict__ ds, const float* __restrict__ xhat,
                                                           const float* __restrict__ gam, const float* __restrict__ bet,
                                                           long rows, int d, float* __restrict__ dz) {
  const long n = rows * d;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const int c = (int)(i % d);
    const float z = xhat[i] * gam[c] + bet[c];
    const float s = 1.0f / (1.0f + expf(-z));
    dz[i] = ds[i] * (s + z * s * (1.0f - s));
  }
}
// dx = gamma * rstd * (dy - sdy / n - xhat * sdyx / n)   (sdy, sdyx: global sums over n frames)
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const float* __restrict__ dy, const float* __restrict__ xhat,
                                                           const float* __restrict__ gam, const float* __restrict__ rstd,
                                                           const float* __restrict__ sdy, const float* __restrict__ sdyx,
                                                           const float* __restrict__ cnt, long rows, int d,
                                                           float* __restrict__ dx) {
  const long n = rows * d;
  const float inv_n = (float)(1.0 / (double)cnt[0]);   // the forward's (global) frame count
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const int c = (int)(i % d);
    dx[i] = gam[c] * rstd[c] * (dy[i] - sdy[c] * inv_n - xhat[i] * sdyx[c] * inv_n);
  }
}
// dz = dropout'(du) * swish'(z), z in the compute type (FFN hidden pre-activation)
template <typename T>
__global__ __launch_bounds__(256) void swish_drop_bwd_kernel(const T* __restrict__ z, const float* __restrict__ du,
                                                             long n, Drop drop, float* __restrict__ dz) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const float zz = ld_f<T>(z + i);
    const float s = 1.0f / (1.0f + expf(-zz));
    dz[i] = du[i] * drop_mul(drop, (uint64_t)i) * (s + zz * s * (1.0f - s));
  }
}

// ---------------------------------------------------------------------------------------------
// subsampling backward
// ---------------------------------------------------------------------------------------------
// g *= (y > 0) (ReLU backward from the saved output)
template <typename T>
__global__ __launch_bounds__(256) void relu_mask_kernel(float* g, const T* __restrict__ y, long n) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    if (!(ld_f<T>(y + i) > 0.0f)) g[i] = 0.0f;
}
// col2im of conv2's input gradient, masked by conv1's ReLU:
//   dY1[b,t1,f1,c] = [X1 > 0] * sum over taps (kt, kf) with t1 = 2*t2 - 1 + kt, f1 = 2*f2 - 1 + kf of
//                    dCol[(b, t2, f2)][(3*kt + kf) * C + c]
template <typename T>
__global__ __launch_bounds__(256) void col2im_relu_kernel(const T* __restrict__ dcol, const T* __restrict__ x1, int B,
                                                          int T1, int F1, int T2, int F2, int C,
                                                          float* __restrict__ dy1) {
  const long n = (long)B * T1 * F1 * C;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const int c = (int)(i % C);
    const long p = i / C;
    const int f1 = (int)(p % F1);
    const long bt = p / F1;
    const int t1 = (int)(bt % T1), b = (int)(bt / T1);
    float s = 0.0f;
    if (ld_f<T>(x1 + i) > 0.0f) {
      for (int kt = 0; kt < 3; ++kt) {
        const int tt = t1 + 1 - kt;
        if (tt < 0 || (tt & 1) || (tt >> 1) >= T2) continue;
        for (int kf = 0; kf < 3; ++kf) {
          const int ff = f1 + 1 - kf;
          if (ff < 0 || (ff & 1) || (ff >> 1) >= F2) continue;
          const long m = ((long)b * T2 + (tt >> 1)) * F2 + (ff >> 1);
          s += ld_f<T>(dcol + m * 9 * C + (long)(3 * kt + kf) * C + c);
        }
      }
    }
    dy1[i] = s;
  }
}
// im2col of conv2's input, transposed (the weight-gradient GEMM operand):
//   dst[tap*C + ci][m] = X1[b, 2*t2 - 1 + kt, 2*f2 - 1 + kf, ci] (zero outside), m = (b, t2, f2)
template <typename T>
__global__ __launch_bounds__(256) void im2col_t_kernel(const T* __restrict__ x1, int T1, int F1, int T2, int F2, int C,
                                                       int M2, T* __restrict__ dst, long ld, int rows_pad) {
  __shared__ float tile[32][33];
  const int r0 = blockIdx.y * 32, m0 = blockIdx.x * 32;   // r = tap*C + ci (rows of dst), m (columns)
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int k = ty; k < 32; k += 8) {      // tile[k][tx] = src(m0 + k, r0 + tx): coalesced along ci
    const int m = m0 + k, r = r0 + tx;
    float v = 0.0f;
    if (m < M2 && r < 9 * C) {
      const int tap = r / C, ci = r - tap * C, kt = tap / 3, kf = tap - kt * 3;
      const int f2 = m % F2, bt = m / F2, t2 = bt % T2, b = bt / T2;
      const int ti = 2 * t2 - 1 + kt, fi = 2 * f2 - 1 + kf;
      if (ti >= 0 && ti < T1 && fi >= 0 && fi < F1) v = ld_f<T>(x1 + (((long)b * T1 + ti) * F1 + fi) * C + ci);
    }
    tile[k][tx] = v;
  }
  __syncthreads();
  for (int k = ty; k < 32; k += 8) {
    const int r = r0 + k, m = m0 + tx;
    float v = tile[tx][k];
    if (r == 9 * C) v = m < M2 ? 1.0f : 0.0f;   // ones row: the GEMM's column 9C is conv2's bias gradient
    if (r < rows_pad && m < ld) st_f<T>(dst + (long)r * ld + m, v);
  }
}
// 8 consecutive compute-type values <-> fp32 (16-byte bf16 / 2 x 16-byte fp32 accesses)
template <typename T> CFM_DEV void ld8(const T* p, float* v);
template <> CFM_DEV void ld8<float>(const float* p, float* v) {
  const float4 a = *(const float4*)p, b = *(const float4*)(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
template <> CFM_DEV void ld8<bf16_t>(const bf16_t* p, float* v) { Vec16<bf16_t>::to_f32(*(const uint4*)p, v); }
template <typename T> CFM_DEV void st8(T* p, const float* v);
template <> CFM_DEV void st8<float>(float* p, const float* v) {
  *(float4*)p = make_float4(v[0], v[1], v[2], v[3]);
  *(float4*)(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
}
template <> CFM_DEV void st8<bf16_t>(bf16_t* p, const float* v) { *(uint4*)p = Vec16<bf16_t>::from_f32(v); }

// col2im_relu_kernel for C % 8 == 0: one thread per 8 channels of an input pixel (index math once
// per pixel, 16-byte loads of X1 and of each contributing dCol tap, 2 x 16-byte fp32 stores).
template <typename T>
__global__ __launch_bounds__(256) void col2im_relu_vec_kernel(const T* __restrict__ dcol, const T* __restrict__ x1,
                                                              int B, int T1, int F1, int T2, int F2, int C,
                                                              float* __restrict__ dy1) {
  const int C8 = C >> 3;
  const long n = (long)B * T1 * F1 * C8;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const long p = i / C8;
    const int c = (int)(i - p * C8) * 8;
    const int f1 = (int)(p % F1);
    const int bt = (int)(p / F1);
    const int t1 = bt % T1, b = bt / T1;
    float xv[8], s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    ld8<T>(x1 + p * C + c, xv);
    bool any = false;
#pragma unroll
    for (int e = 0; e < 8; ++e) any |= xv[e] > 0.0f;
    if (any) {
      for (int kt = 0; kt < 3; ++kt) {
        const int tt = t1 + 1 - kt;
        if (tt < 0 || (tt & 1) || (tt >> 1) >= T2) continue;
        for (int kf = 0; kf < 3; ++kf) {
          const int ff = f1 + 1 - kf;
          if (ff < 0 || (ff & 1) || (ff >> 1) >= F2) continue;
          const long m = ((long)b * T2 + (tt >> 1)) * F2 + (ff >> 1);
          float v[8];
          ld8<T>(dcol + m * 9 * C + (long)(3 * kt + kf) * C + c, v);
#pragma unroll
          for (int e = 0; e < 8; ++e) s[e] += v[e];
        }
      }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) s[e] = xv[e] > 0.0f ? s[e] : 0.0f;
    st8<float>(dy1 + p * C + c, s);
  }
}

// im2col_t_kernel for C % 8 == 0 and ld % 8 == 0: 64 (tap, ci) rows x 64 pixels per block; 16-byte
// loads of 8 channels of an X1 pixel, 16-byte stores of 8 pixels of a destination row.
template <typename T>
__global__ __launch_bounds__(256) void im2col_t_vec_kernel(const T* __restrict__ x1, int T1, int F1, int T2, int F2,
                                                           int C, int M2, T* __restrict__ dst, long ld, int rows_pad) {
  // one block: 64 pixels x kRT consecutive 64-row tiles; the next row tile's loads are in flight
  // while the current one is stored
  constexpr int kRT = 4;
  __shared__ float tile[64][65];   // [row r - r0][pixel m - m0]
  const int m0 = blockIdx.x * 64;
  float v[2][8];
  auto load = [&](int r0) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {   // pixel m = m0 + (idx >> 3), rows r0 + 8 (idx & 7) .. +7
      const int idx = q * 256 + threadIdx.x;
      const int ml = idx >> 3, rl = 8 * (idx & 7);
      const int m = m0 + ml, r = r0 + rl;
#pragma unroll
      for (int e = 0; e < 8; ++e) v[q][e] = 0.0f;
      if (m < M2 && r < 9 * C) {
        const int tap = r / C, ci = r - tap * C, kt = tap / 3, kf = tap - kt * 3;
        const int f2 = m % F2, bt = m / F2, t2 = bt % T2, b = bt / T2;
        const int ti = 2 * t2 - 1 + kt, fi = 2 * f2 - 1 + kf;
        if (ti >= 0 && ti < T1 && fi >= 0 && fi < F1) ld8<T>(x1 + (((long)b * T1 + ti) * F1 + fi) * C + ci, v[q]);
      }
    }
  };
  const int rt0 = blockIdx.y * kRT;
  load(rt0 * 64);
  for (int rt = rt0; rt < rt0 + kRT; ++rt) {
    const int r0 = rt * 64;
    if (r0 >= rows_pad) break;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int idx = q * 256 + threadIdx.x;
      const int ml = idx >> 3, rl = 8 * (idx & 7);
#pragma unroll
      for (int e = 0; e < 8; ++e) tile[rl + e][ml] = v[q][e];
    }
    __syncthreads();
    if (rt + 1 < rt0 + kRT && (rt + 1) * 64 < rows_pad) load(r0 + 64);
#pragma unroll
    for (int q = 0; q < 2; ++q) {   // store: row r0 + (idx >> 3), pixels m0 + 8 (idx & 7) .. +7
      const int idx = q * 256 + threadIdx.x;
      const int rl = idx >> 3, ml = 8 * (idx & 7);
      const int r = r0 + rl, m = m0 + ml;
      if (r >= rows_pad || m >= ld) continue;
      float o[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = r == 9 * C ? (m + e < M2 ? 1.0f : 0.0f) : tile[rl][ml + e];
      st8<T>(dst + (long)r * ld + m, o);
    }
    __syncthreads();
  }
}

// Packed operand of one stride phase (pt, pf) of conv2's input gradient (gemm_tconv):
//   dst[ci][tap * C + co] = W2[co][ci][kt][kf], tap = a * (1 + pf) + c over the phase's taps, with
//   kt = pt ? (a == 0 ? 0 : 2) : 1 and kf = pf ? (c == 0 ? 0 : 2) : 1 (zero past the taps / rows).
template <typename T>
__global__ __launch_bounds__(256) void tconv_wpack_kernel(const float* __restrict__ w2, int C, int pt, int pf,
                                                          T* __restrict__ dst, int Kp, int rows_pad) {
  const long n = (long)rows_pad * Kp;
  const int nf = 1 + pf, ntap = (1 + pt) * nf;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const int r = (int)(i / Kp), q = (int)(i - (long)r * Kp);
    float v = 0.0f;
    if (r < C && q < ntap * C) {
      const int tap = q / C, co = q - tap * C, a = tap / nf, c = tap - a * nf;
      const int kt = pt ? (a == 0 ? 0 : 2) : 1, kf = pf ? (c == 0 ? 0 : 2) : 1;
      v = w2[((long)co * C + r) * 9 + kt * 3 + kf];
    }
    st_f<T>(dst + i, v);
  }
}

// Phase-major dY1 image written by the four gemm_tconv launches: phase ph = 2*pt + pf holds the
// pixels (2i + pt, 2j + pf) as rows ((b * nI[pt] + i) * nJ[pf] + j), phases stacked in ph order.
struct PhaseRows {
  long base[4];
  int nI[2], nJ[2];
  __host__ __device__ PhaseRows(int B, int T1, int F1) {
    nI[0] = (T1 + 1) / 2; nI[1] = T1 / 2;
    nJ[0] = (F1 + 1) / 2; nJ[1] = F1 / 2;
    long o = 0;
    for (int ph = 0; ph < 4; ++ph) {
      base[ph] = o;
      o += (long)B * nI[ph >> 1] * nJ[ph & 1];
    }
  }
};

// conv1 weight gradient, stage 1: partial[chunk][c][tap] = sum over the chunk's (b, t1) rows and all
// f1 of dY1[b,t1,f1,c] * xpad[b, f = 2*f1 - 1 + kf, t = 2*t1 - 1 + kt]  (x is (B, F, T)).
// PH: dY1 is the unmasked phase-major image (PhaseRows, compute type) and conv1's ReLU mask
// [X1 > 0] is applied here; otherwise dY1 is (B, T1, F1, C) fp32, already masked.
template <typename TX, bool PH>
__global__ __launch_bounds__(256) void conv1_wgrad_kernel(const float* __restrict__ x, int F, int T, int T1, int F1,
                                                          int C, const TX* __restrict__ dy1,
                                                          const TX* __restrict__ x1, int B, int R,
                                                          float* __restrict__ partial, float* __restrict__ partial_b) {
  __shared__ float xs[3][264];
  const int chunk = blockIdx.x;
  const int c = blockIdx.y * 256 + threadIdx.x;
  float acc[9], accb = 0.0f;
#pragma unroll
  for (int k = 0; k < 9; ++k) acc[k] = 0.0f;
  const int r0 = chunk * R, r1 = min(B * T1, r0 + R);
  for (int bt = r0; bt < r1; ++bt) {
    const int b = bt / T1, t1 = bt - b * T1;
    __syncthreads();
    for (int i = threadIdx.x; i < 3 * (F + 2); i += 256) {
      const int kt = i / (F + 2), fp = i - kt * (F + 2), f = fp - 1, t = 2 * t1 - 1 + kt;
      xs[kt][fp] = (f >= 0 && f < F && t >= 0 && t < T) ? x[((long)b * F + f) * T + t] : 0.0f;
    }
    __syncthreads();
    if (c < C) {
      const TX* g = dy1 + ((long)bt * F1) * C + c;
      long prow[2] = {0, 0};
      if constexpr (PH) {
        const PhaseRows pr(B, T1, F1);
        const int pt = t1 & 1;
#pragma unroll
        for (int pf = 0; pf < 2; ++pf)
          prow[pf] = pr.base[2 * pt + pf] + ((long)b * pr.nI[pt] + (t1 >> 1)) * pr.nJ[pf];
      }
      for (int f1 = 0; f1 < F1; ++f1) {
        float gv;
        if constexpr (PH) {
          gv = ld_f<TX>(dy1 + (prow[f1 & 1] + (f1 >> 1)) * C + c);
          if (!(ld_f<TX>(x1 + ((long)bt * F1 + f1) * C + c) > 0.0f)) gv = 0.0f;
        } else {
          gv = ld_f<TX>(g + (long)f1 * C);
        }
        accb += gv;
#pragma unroll
        for (int kt = 0; kt < 3; ++kt)
#pragma unroll
          for (int kf = 0; kf < 3; ++kf) acc[kt * 3 + kf] = fmaf(gv, xs[kt][2 * f1 + kf], acc[kt * 3 + kf]);
      }
    }
  }
  if (c < C) {
#pragma unroll
    for (int k = 0; k < 9; ++k) partial[((long)chunk * C + c) * 9 + k] = acc[k];
    partial_b[(long)chunk * C + c] = accb;
  }
}

// conv1_wgrad_kernel<TX, true> for C % 8 == 0: a thread owns 8 consecutive channels (16-byte loads of
// the phase-major dY1 and of the X1 mask, 9 x 8 accumulators), a 64-thread block 512 channels of R
// (b, t1) rows.  Same per-channel summation order as the scalar kernel (bitwise equal partials).
template <typename TX>
__global__ __launch_bounds__(64) void conv1_wgrad_ph8_kernel(const float* __restrict__ x, int F, int T, int T1,
                                                             int F1, int C, const TX* __restrict__ dy1,
                                                             const TX* __restrict__ x1, int B, int R,
                                                             float* __restrict__ partial, float* __restrict__ partial_b) {
  __shared__ float xs[3][264];
  const int chunk = blockIdx.x;
  const int c0 = (blockIdx.y * 64 + threadIdx.x) * 8;
  float acc[9][8], accb[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    accb[e] = 0.0f;
#pragma unroll
    for (int k = 0; k < 9; ++k) acc[k][e] = 0.0f;
  }
  const PhaseRows pr(B, T1, F1);
  const int r0 = chunk * R, r1 = min(B * T1, r0 + R);
  for (int bt = r0; bt < r1; ++bt) {
    const int b = bt / T1, t1 = bt - b * T1;
    __syncthreads();
    for (int i = threadIdx.x; i < 3 * (F + 2); i += 64) {
      const int kt = i / (F + 2), fp = i - kt * (F + 2), f = fp - 1, t = 2 * t1 - 1 + kt;
      xs[kt][fp] = (f >= 0 && f < F && t >= 0 && t < T) ? x[((long)b * F + f) * T + t] : 0.0f;
    }
    __syncthreads();
    if (c0 < C) {
      const int pt = t1 & 1;
      long prow[2];
#pragma unroll
      for (int pf = 0; pf < 2; ++pf)
        prow[pf] = pr.base[2 * pt + pf] + ((long)b * pr.nI[pt] + (t1 >> 1)) * pr.nJ[pf];
      for (int f1 = 0; f1 < F1; ++f1) {
        float gv[8], mv[8];
        ld8<TX>(dy1 + (prow[f1 & 1] + (f1 >> 1)) * C + c0, gv);
        ld8<TX>(x1 + ((long)bt * F1 + f1) * C + c0, mv);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          if (!(mv[e] > 0.0f)) gv[e] = 0.0f;
          accb[e] += gv[e];
        }
#pragma unroll
        for (int kt = 0; kt < 3; ++kt)
#pragma unroll
          for (int kf = 0; kf < 3; ++kf) {
            const float xv = xs[kt][2 * f1 + kf];
#pragma unroll
            for (int e = 0; e < 8; ++e) acc[kt * 3 + kf][e] = fmaf(gv[e], xv, acc[kt * 3 + kf][e]);
          }
      }
    }
  }
  if (c0 < C) {
    float* pp = partial + ((long)chunk * C + c0) * 9;
#pragma unroll
    for (int e = 0; e < 8; ++e)
#pragma unroll
      for (int k = 0; k < 9; ++k) pp[e * 9 + k] = acc[k][e];
#pragma unroll
    for (int e = 0; e < 8; ++e) partial_b[(long)chunk * C + c0 + e] = accb[e];
  }
}

// (B, T', d) fp32 rows <-> (B, d, T') fp32
__global__ __launch_bounds__(256) void btd_transpose_kernel(const float* __restrict__ src, int Tp, int d, int to_bdt,
                                                            float* __restrict__ dst) {
  __shared__ float tile[32][33];
  const int b = blockIdx.z, t0 = blockIdx.x * 32, c0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const float* s = src + (long)b * Tp * d;
  float* o = dst + (long)b * Tp * d;
  for (int k = ty; k < 32; k += 8) {
    if (to_bdt) {   // src (T', d): tile[t][c]
      const int t = t0 + k, c = c0 + tx;
      tile[k][tx] = (t < Tp && c < d) ? s[(long)t * d + c] : 0.0f;
    } else {        // src (d, T'): tile[c][t]
      const int c = c0 + k, t = t0 + tx;
      tile[k][tx] = (t < Tp && c < d) ? s[(long)c * Tp + t] : 0.0f;
    }
  }
  __syncthreads();
  for (int k = ty; k < 32; k += 8) {
    if (to_bdt) {
      const int c = c0 + k, t = t0 + tx;
      if (t < Tp && c < d) o[(long)c * Tp + t] = tile[tx][k];
    } else {
      const int t = t0 + k, c = c0 + tx;
      if (t < Tp && c < d) o[(long)t * d + c] = tile[tx][k];
    }
  }
}

// ---------------------------------------------------------------------------------------------
// geometry, tape and workspace layouts
// ---------------------------------------------------------------------------------------------
int calc_len_host(int len, int repeat) {
  float L = (float)len;
  for (int i = 0; i < repeat; ++i) L = std::floor((L + (2.0f * 1 - 3.0f)) / 2.0f + 1.0f);
  return (int)L;
}

struct Geo {
  int B, T, T1, T2, Tp, M, Tpad, NP;   // NP = 2T' - 1 position rows
  int d, dff, H, dk, dkp, C, F, F1, F2, K, L, es, dt, kg;
  long Mp, M2, M2p, Mq;                 // Mq: padded row count covering M and NP (wgrad K extent)
};
Geo make_geo(const cfm_encoder* h, int B, int T) {
  Geo g;
  g.B = B; g.T = T;
  g.T1 = calc_len_host(T, 1);
  g.T2 = calc_len_host(T, 2);
  g.Tp = g.T2;
  g.M = B * g.Tp;
  g.Tpad = (int)round_up(std::max(g.Tp, 1), 32);
  g.NP = 2 * g.Tp - 1;
  g.d = h->d; g.dff = h->dff; g.H = h->H; g.dk = h->dk; g.dkp = h->dkp; g.C = h->C; g.F = h->F; g.F1 = h->F1;
  g.F2 = h->F2; g.K = h->K; g.L = h->L; g.es = h->es; g.dt = h->dtype; g.kg = GEMM_BK_BYTES / h->es;
  g.Mp = round_up(std::max(g.M, 1), g.kg);
  // + 16 granules of zero columns: split-K slices (<= 16, each a multiple of kg) never read past a row
  g.Mq = round_up(std::max(g.M, g.NP), g.kg) + 16L * g.kg;
  g.M2 = (long)B * g.T2 * g.F2;
  g.M2p = round_up(std::max<long>(g.M2, 1), g.kg) + 16L * g.kg;
  return g;
}

struct Alloc {
  long off = 0;
  long take(long bytes) { const long o = round_up(off, 256); off = o + round_up(std::max(bytes, 1L), 256); return o; }
};

struct TapeLayer { long x[5], hn[4], z1, z2, u1, u2, qk, vt, P, ctx, pre, g, xhat, mean, rstd, s; };
struct Tape { long xin, lens, X1, X2; std::vector<TapeLayer> lay; long xfin, total; };

Tape tape_layout(const cfm_encoder* h, const Geo& g) {
  Tape t;
  Alloc a;
  const long es = g.es, M = g.M, d = g.d;
  t.xin = a.take((long)g.B * g.F * g.T * 4);
  t.lens = a.take((long)g.B * 4);
  t.X1 = a.take((long)g.B * g.T1 * g.F1 * g.C * es);
  t.X2 = a.take((long)g.M2 * g.C * es);
  t.lay.resize(g.L);
  for (auto& l : t.lay) {
    for (long& v : l.x) v = a.take(M * d * 4);
    for (long& v : l.hn) v = a.take(M * d * es);
    l.z1 = a.take(M * g.dff * es);
    l.z2 = a.take(M * g.dff * es);
    // the FFN hiddens u = dropout(swish(z)) too: the weight gradient of linear2 reads them as they
    // are instead of recomputing the activation and its mask per output tile
    l.u1 = a.take(M * g.dff * es);
    l.u2 = a.take(M * g.dff * es);
    l.qk = a.take(M * 3 * g.H * g.dkp * es);
    l.vt = a.take((long)g.B * g.H * h->vt_rows * g.Tpad * es);
    l.P = a.take((long)g.NP * g.H * g.dkp * es + 64);
    l.ctx = a.take(M * d * es);
    l.pre = a.take(M * 2 * d * 4);
    l.g = a.take(M * d * 4);
    l.xhat = a.take(M * d * 4);
    l.mean = a.take((d + 1) * 4);   // + the BatchNorm frame count (global under SyncBatchNorm)
    l.rstd = a.take(d * 4);
    l.s = a.take(M * d * es);
  }
  t.xfin = a.take(M * d * 4);
  t.total = round_up(a.off, 256);
  return t;
}

// split-K factor of a weight-gradient GEMM (N x K outputs, reduction over `rows`)
// Tile of a weight-gradient GEMM: 256x256 (tile 11, 3x the arithmetic intensity of 64x128) for the
// very long contractions (the conv2 weight gradient over 160 000 im2col rows), 64x128 (the shape
// picker's choice) otherwise.  The split count targets a few tiles per CU for either.
// Weight-gradient GEMM tile: 256x256 for the 160k-row conv2 gradient; CFM_WGRAD_TILE picks another
// gemm.hip tile id for the M-row layer gradients (A/B measurements; default: pick_tile's 64x128).
int g_wgrad_tile = [] { const char* e = getenv("CFM_WGRAD_TILE"); return e ? atoi(e) : -1; }();
int wgrad_tile(int N, int K, long rows) {
  if (N < 256 || K < 256) return -1;
  if (rows >= 32768) return 11;
  return g_wgrad_tile;
}
void tile_dims(int t, int& bm, int& bn) {
  switch (t) {
    case 0: case 8: bm = 128; bn = 128; return;
    case 1: case 9: bm = 256; bn = 128; return;
    case 7: case 11: bm = 256; bn = 256; return;
    case 10: bm = 128; bn = 256; return;
    default: bm = 64; bn = 128; return;
  }
}
int wgrad_splits(int N, int K, long rows) {
  const int t = wgrad_tile(N, K, rows);
  int bm, bn;
  tile_dims(t, bm, bn);
  const bool big = t >= 7;   // one block per CU
  const long tiles = (long)((N + bm - 1) / bm) * ((K + bn - 1) / bn);
  long s = ((big ? 512 : 768) + tiles - 1) / tiles;
  s = std::min<long>(s, std::max<long>(1, rows / 256));
  return (int)std::max<long>(1, std::min<long>(s, 16));
}

// Row splits of a frame-major weight gradient (wgrad_tn): enough (tile, split) blocks for the target
// block count (CFM_TN_BLOCKS overrides it for A/B runs), at least 64 frame rows per split, at most 16
long tn_splits(int N, int K, bool bias, int bfn, long rows) {
  static const long env_target = [] { const char* e = getenv("CFM_TN_BLOCKS"); return e ? atol(e) : 0L; }();
  const long tiles = wgrad_tn_tiles(N, K, bias, bfn);
  const long target = env_target > 0 ? env_target : wgrad_tn_blocks(bfn);
  long S = (target + tiles - 1) / tiles;
  S = std::max<long>(1, std::min<long>({S, rows / 64, 16L}));
  const long chunk = round_up((rows + S - 1) / S, 32);
  return (rows + chunk - 1) / chunk;
}

enum { WT_FF1_W2 = 0, WT_FF1_W1, WT_FF2_W2, WT_FF2_W1, WT_PW2, WT_PW1, WT_OUT };
struct Ws {
  // forward
  long w1, b1, w2, b2, w1b, b1b, w2b, b2b, wqkv, bqkv, uv, wout, bout, wpos, wpw1, bpw1, dww, wpw2, bpw2, wc2, bc2, wsub, bsub;
  long u, br, dwo, gt, s1, s2, sync;
  // backward
  long gA, gB, dbr, lnp, dU, pa, pat, pbt, wt, wtl[7], part, dqkv, dctx, dP, dpre, dG, dD, red;
  long dX2, dcol, i2c, dy1, c1part, gtmp, attws;
  long ped;   // dropout_emb: the dropped positional window (2T'-1, d) in the compute type
  long total;
};

Ws ws_layout(const cfm_encoder* h, const Geo& g) {
  Ws w;
  Alloc a;
  const long es = g.es, M = g.M, d = g.d, dff = g.dff, kg = g.kg;
  auto kp = [&](long k) { return round_up(k, kg); };
  auto np = [&](long n) { return round_up(n, GEMM_BN); };
  const long HP = (long)g.H * g.dkp;
  w.w1 = a.take(np(dff) * kp(d) * es);
  w.b1 = a.take(np(dff) * 4);
  w.w2 = a.take(np(d) * kp(dff) * es);
  w.b2 = a.take(np(d) * 4);
  w.w1b = a.take(np(dff) * kp(d) * es);
  w.b1b = a.take(np(dff) * 4);
  w.w2b = a.take(np(d) * kp(dff) * es);
  w.b2b = a.take(np(d) * 4);
  w.wqkv = a.take(np(3 * HP) * kp(d) * es);
  w.bqkv = a.take(np(3 * HP) * 4);
  w.uv = a.take(2 * HP * 4);
  w.wout = a.take(np(d) * kp(d) * es);
  w.bout = a.take(np(d) * 4);
  w.wpos = a.take(np(HP) * kp(d) * es);
  w.wpw1 = a.take(np(2 * d) * kp(d) * es);
  w.bpw1 = a.take(np(2 * d) * 4);
  w.dww = a.take((long)g.K * d * 4);
  w.wpw2 = a.take(np(d) * kp(d) * es);
  w.bpw2 = a.take(np(d) * 4);
  w.wc2 = a.take(np(g.C) * kp(9L * g.C) * es);
  w.bc2 = a.take(np(g.C) * 4);
  w.wsub = a.take(np(d) * kp((long)g.F2 * g.C) * es);
  w.bsub = a.take(np(d) * 4);
  w.u = a.take(M * dff * es);
  w.br = a.take(M * d * 4);
  w.dwo = a.take(M * d * 4);
  w.gt = a.take(M * d * es);
  w.s1 = a.take(d * 4);
  w.s2 = a.take(d * 4);
  w.sync = a.take((2 * d + 2) * 4);   // [sum x | count] then [sum (x - mean)^2]
  // backward
  const long Kmax = std::max({dff, 3 * d, 2 * d, (long)g.F2 * g.C});
  w.gA = a.take(M * d * 4);
  w.gB = a.take(M * d * 4);
  w.dbr = a.take(M * d * 4);
  w.lnp = a.take(5L * 2 * ((M + 4 * kLnRowsPerWave - 1) / (4 * kLnRowsPerWave)) * d * 4);   // the layer's five LayerNorm backward column partials
  w.dU = a.take(M * std::max(dff, 3 * d) * 4);
  w.pa = a.take(M * kp(Kmax) * es);                                   // dgrad A operand [M][N]
  const long NT = std::max({dff, 3 * d, 2 * d, (long)g.C});
  w.pat = a.take(std::max(NT * g.Mq, (long)g.C * g.M2p) * es);       // dy^T [N][Mp]
  const long KT = np(std::max({dff, d, (long)g.F2 * g.C}) + 4);
  w.pbt = a.take(KT * g.Mq * es);                                      // x^T [Kpad][Mp]
  w.wt = a.take(std::max({np(dff) * kp(d), np(d) * kp(dff), np(d) * kp(3 * d), np(d) * kp(2 * d),
                          np((long)g.F2 * g.C) * kp(d), np(9L * g.C) * kp(g.C),
                          np(g.C) * (kp(g.C) + 2 * kp(2L * g.C) + kp(4L * g.C))}) * es);   // + tconv phases
  // a layer's transposed weights for its dgrad GEMMs, packed in one launch (WT_* order)
  const long wtl_sz[7] = {np(dff) * kp(d), np(d) * kp(dff), np(dff) * kp(d), np(d) * kp(dff), np(d) * kp(d),
                          np(d) * kp(2 * d), np(d) * kp(d)};
  for (int i = 0; i < 7; ++i) w.wtl[i] = a.take(wtl_sz[i] * es);
  long part = 0;
  auto upd = [&](long N, long K, long rows) { part = std::max(part, (long)wgrad_splits((int)N, (int)K, rows) * N * K); };
  upd(dff, d + 4, M); upd(d, dff + 4, M); upd(3 * d, d + 4, M); upd(d, d + 4, M); upd(2 * d, d + 4, M);
  upd(d, d, g.NP); upd(d, (long)g.F2 * g.C + 4, M); upd(g.C, 9L * g.C + 4, g.M2);
  auto upd_tn = [&](long N, long K, bool bias, long rows) {   // Ws::wgrad_rm (both staging forms)
    for (int bfn = 0; bfn < 2; ++bfn) part = std::max(part, tn_splits((int)N, (int)K, bias, bfn, rows) * N * (bias ? K + 4 : K));
  };
  upd_tn(dff, d, true, M); upd_tn(d, dff, true, M); upd_tn(3 * d, d, true, M); upd_tn(d, d, true, M);
  upd_tn(2 * d, d, true, M); upd_tn(d, d, false, g.NP); upd_tn(d, (long)g.F2 * g.C, true, M);
  w.part = a.take(part * 4);
  w.dqkv = a.take(M * 3 * d * 4);
  w.dctx = a.take(M * d * 4);
  w.dP = a.take((long)g.NP * d * 4);
  w.dpre = a.take(M * 2 * d * 4);
  w.dG = a.take(M * d * 4);
  w.dD = a.take(M * d * 4);
  const long red_rows = std::max({(long)M, g.M2, (long)g.B * g.T1 * g.F1, 64L});
  w.red = a.take(std::max({(long)colred_ws(red_rows, std::max(dff, 3 * d)), (long)colred_ws(16, 9L * g.C * g.C),
                           (long)cfm_op_dwconv_backward_ws_size(g.B, g.Tp, (int)d, g.K),
                           (long)colred_ws(g.B * g.T1, 9L * g.C)}) + 1024);
  w.dX2 = a.take(M * (long)g.F2 * g.C * 4);
  w.dcol = a.take(g.M2 * 9L * g.C * es);
  w.i2c = a.take(np(9L * g.C + 4) * g.M2p * es);
  w.dy1 = a.take((long)g.B * g.T1 * g.F1 * g.C * 4);
  const long c1ch = ((long)g.B * g.T1 + 7) / 8;
  w.c1part = a.take(c1ch * 10L * g.C * 4 + 4096);
  w.gtmp = a.take(std::max({d * (long)g.F2 * g.C, 9L * g.C * g.C, 3 * d * d + 3 * d}) * 4);
  w.attws = a.take((long)rel_pos_attention_backward_ws(g.B, g.Tp, g.H, g.dk) + 256);
  w.ped = a.take((long)g.NP * d * es + 64);
  w.total = round_up(a.off, 256);
  return w;
}

// ---------------------------------------------------------------------------------------------
// step context
// ---------------------------------------------------------------------------------------------
enum LnIdx { LN_FF1 = 0, LN_ATT = 1, LN_CONV = 2, LN_FF2 = 3, LN_OUT = 4 };

struct LayerP {   // indices into the parameter table
  int ln_w[5], ln_b[5];
  int ff_w1[2], ff_b1[2], ff_w2[2], ff_b2[2];
  int pw1_w, pw1_b, dw_w, dw_b, bn_w, bn_b, bn_rm, bn_rv, pw2_w, pw2_b;
  int q_w, q_b, k_w, k_b, v_w, v_b, o_w, o_b, pos_w, pu, pv;
};

struct Step {
  cfm_encoder* h;
  Geo g;
  Tape tp;
  Ws wl;
  char* tape;
  char* ws;
  hipStream_t st;
  const float* const* P;
  const cfm_train_opts* o;
  int i_c1w, i_c1b, i_c2w, i_c2b, i_sw, i_sb;
  std::vector<LayerP> lp;

  const float* prm(int i) const { return P[i]; }
  template <typename T = char> T* T_(long off) const { return (T*)(tape + off); }
  template <typename T = char> T* W_(long off) const { return (T*)(ws + off); }
  int kpad(long k) const { return (int)round_up(k, g.kg); }
  int npad(long n) const { return (int)round_up(n, GEMM_BN); }
  Drop drop(int site) const { return make_drop(o->dropout, o->seed, site); }
  // attention-probability dropout of layer l (site j = 6) and the positional-embedding dropout
  // (its own site past the layers'); both regenerated bit for bit by the backward
  Drop drop_att(int l) const { return make_drop(o->dropout_att, o->seed, 1 + 8 * l + 6); }
  Drop drop_emb() const { return make_drop(o->dropout_emb, o->seed, 1 + 8 * g.L); }
  // the positional window linear_pos reads: h->pe's slice, or its dropout_emb copy in the workspace
  const char* pos_window() const {
    const char* pe_slice = h->pe + (long)(h->max_len - g.Tp) * g.d * g.es;
    const Drop de = drop_emb();
    if (!de.thr) return pe_slice;
    const long n = (long)g.NP * g.d;
    if (g.dt == DT_F32)
      cfm_launch(pe_drop_kernel<float>, dim3(ew_grid(n)), dim3(256), 0, st, (const float*)pe_slice, n, de,
                 W_<float>(wl.ped));
    else
      cfm_launch(pe_drop_kernel<bf16_t>, dim3(ew_grid(n)), dim3(256), 0, st, (const bf16_t*)pe_slice, n, de,
                 W_<bf16_t>(wl.ped));
    return W_(wl.ped);
  }

  void pack(const void* src, bool src_ct, long ld, int rows, int cols, bool tr, float scale, void* dst, long dld,
            int rp, int cp, int fn = 0, Drop dr = Drop{0, 0, 1.0f}, int ones_row = -1) const {
    if (rp <= 0 || cp <= 0) return;
    const dim3 grid((cp + 63) / 64, (rp + 63) / 64), block(256);
    const int ses = (g.dt != DT_F32 && src_ct) ? 2 : 4;           // source element bytes
    const int des = g.dt == DT_F32 ? 4 : 2;
    // 2: 16-byte source runs; 1: 8-byte (bf16) runs; 0: element loads
    const int sv = (ld % (16 / ses) == 0 && ((uintptr_t)src % 16) == 0) ? 2
                   : (ld % 4 == 0 && ((uintptr_t)src % (4 * ses)) == 0) ? 1 : 0;
    const int dv = (dld % (16 / des) == 0 && ((uintptr_t)dst % 16) == 0) ? 1 : 0;
    if (g.dt == DT_F32) {
      cfm_launch(tpack_kernel<float, float>, grid, block, 0, st, (const float*)src, ld, rows, cols, (int)tr, scale,
                 fn, dr, (float*)dst, dld, rp, cp, ones_row, sv, dv);
    } else if (src_ct) {
      cfm_launch(tpack_kernel<bf16_t, bf16_t>, grid, block, 0, st, (const bf16_t*)src, ld, rows, cols, (int)tr,
                 scale, fn, dr, (bf16_t*)dst, dld, rp, cp, ones_row, sv, dv);
    } else if (!tr && fn == 0 && ones_row < 0 && sv == 2 && dv == 1 && cp % 8 == 0) {
      cfm_launch(pack_rows_kernel, dim3(ew_grid((long)rp * cp / 8)), block, 0, st, (const float*)src, ld, rows,
                 cols, scale, (bf16_t*)dst, dld, rp, cp);
    } else {
      cfm_launch(tpack_kernel<float, bf16_t>, grid, block, 0, st, (const float*)src, ld, rows, cols, (int)tr, scale,
                 fn, dr, (bf16_t*)dst, dld, rp, cp, ones_row, sv, dv);
    }
  }
  // one-launch parameter packs (tpack_multi_kernel)
  struct Batch {
    PackList l;
    int tiles = 0;
    Batch() { std::memset(&l, 0, sizeof(l)); }
  };
  void job(Batch& b, const float* src, int ld_src, int rows, int cols, bool tr, void* dst, long ld_dst, int rp, int cp,
           bool f32) const {
    if (b.l.count == 16) flush(b);
    PackJob& j = b.l.j[b.l.count++];
    const int des = (f32 || g.dt == DT_F32) ? 4 : 2;
    j.src = src; j.dst = dst; j.ld_src = ld_src; j.rows = rows; j.cols = cols; j.tr = tr ? 1 : 0;
    j.ld_dst = (int)ld_dst; j.rows_pad = rp; j.cols_pad = cp; j.out_f32 = f32 ? 1 : 0;
    j.src_vec = (ld_src % 4 == 0 && ((uintptr_t)src % 16) == 0) ? 2 : 0;
    j.dst_vec = (ld_dst % (16 / des) == 0 && ((uintptr_t)dst % 16) == 0) ? 1 : 0;
    j.tiles_x = (cp + 63) / 64;
    j.tile0 = b.tiles;
    b.tiles += j.tiles_x * ((rp + 63) / 64);
  }
  void jobW(Batch& b, const float* w, int N, int K, void* dst) const { job(b, w, K, N, K, false, dst, kpad(K), npad(N), kpad(K), false); }
  void jobWt(Batch& b, const float* w, int N, int K, void* dst) const { job(b, w, K, N, K, true, dst, kpad(N), npad(K), kpad(N), false); }
  void jobBias(Batch& b, const float* bias, int N, float* dst) const { job(b, bias, N, 1, N, false, dst, npad(N), 1, npad(N), true); }
  void flush(Batch& b) const {
    if (b.l.count == 0) return;
    if (g.dt == DT_F32) cfm_launch(tpack_multi_kernel<float>, dim3(b.tiles), dim3(256), 0, st, b.l);
    else cfm_launch(tpack_multi_kernel<bf16_t>, dim3(b.tiles), dim3(256), 0, st, b.l);
    std::memset(&b.l, 0, sizeof(b.l));
    b.tiles = 0;
  }
  // pack(dy, .., dA, lA, rA, cA) and pack(dy, transposed, .., dT, lT, rT, cT) in one launch
  void pack2(const float* src, long ld, int rows, int cols, void* dA, long lA, int rA, int cA, void* dT, long lT, int rT,
             int cT, float scale = 1.0f, Drop dr = Drop{0, 0, 1.0f}) const {
    const int des = g.dt == DT_F32 ? 4 : 2;
    const int gx = (std::max(cA, rT) + 63) / 64, gy = (std::max(rA, cT) + 63) / 64;
    if (gx <= 0 || gy <= 0) return;
    const int sv = (ld % 4 == 0 && ((uintptr_t)src % 16) == 0) ? 1 : 0;
    const int va = (lA % (16 / des) == 0 && ((uintptr_t)dA % 16) == 0) ? 1 : 0;
    const int vt = (lT % (16 / des) == 0 && ((uintptr_t)dT % 16) == 0) ? 1 : 0;
    if (g.dt == DT_F32)
      cfm_launch(tpack2_kernel<float>, dim3(gx, gy), dim3(256), 0, st, src, ld, rows, cols, (float*)dA, lA, rA, cA,
                 (float*)dT, lT, rT, cT, sv, va, vt, scale, dr);
    else
      cfm_launch(tpack2_kernel<bf16_t>, dim3(gx, gy), dim3(256), 0, st, src, ld, rows, cols, (bf16_t*)dA, lA, rA, cA,
                 (bf16_t*)dT, lT, rT, cT, sv, va, vt, scale, dr);
  }
  // packed forward weight W (N, K) fp32 -> [Npad][Kpad]; transposed Wt -> [Kpad256][Npad_kg]
  void packW(const float* w, int N, int K, void* dst) const {
    pack(w, false, K, N, K, false, 1.0f, dst, kpad(K), npad(N), kpad(K));
  }
  void packWt(const float* w, int N, int K, void* dst) const {
    pack(w, false, K, N, K, true, 1.0f, dst, kpad(N), npad(K), kpad(N));
  }
  // GEMM bias: N floats zero-padded to the N granule, one small launch (a memset + copy pair costs
  // two runtime copy kernels)
  void bias(const float* b, int N, float* dst) const {
    const int np = npad(N);
    cfm_launch(bias_pad_kernel, dim3((np + 255) / 256), dim3(256), 0, st, b, N, dst, np);
  }
  void heads(const float* s0, const float* s1, const float* s2, int parts, int K, void* dst, bool f32, long Kp,
             int rows_pad) const {
    const long n = (long)rows_pad * Kp;
    if (f32 || g.dt == DT_F32)
      cfm_launch(pack_heads_kernel<float>, dim3(ew_grid(n)), dim3(256), 0, st, s0, s1, s2, parts, g.H, g.dk, g.dkp, K,
                 (float*)dst, Kp, rows_pad);
    else
      cfm_launch(pack_heads_kernel<bf16_t>, dim3(ew_grid(n)), dim3(256), 0, st, s0, s1, s2, parts, g.H, g.dk, g.dkp,
                 K, (bf16_t*)dst, Kp, rows_pad);
  }
  void perm(const float* src, int mode, void* dst, bool f32, long ld, int rp, int cp) const {
    const long n = (long)rp * cp;
    if (f32 || g.dt == DT_F32)
      cfm_launch(perm_pack_kernel<float>, dim3(ew_grid(n)), dim3(256), 0, st, src, mode, g.C, g.F2, g.d, (float*)dst,
                 ld, rp, cp);
    else
      cfm_launch(perm_pack_kernel<bf16_t>, dim3(ew_grid(n)), dim3(256), 0, st, src, mode, g.C, g.F2, g.d,
                 (bf16_t*)dst, ld, rp, cp);
  }
  GemmEpi epi(int mode, const float* b, float alpha = 1.0f) const {
    GemmEpi e;
    std::memset(&e, 0, sizeof(e));
    e.mode = mode;
    e.bias = b;
    e.alpha = alpha;
    return e;
  }
  // xout = xin + alpha * dropout(A . W^T + b), the dropout and residual in the GEMM epilogue
  void gemm_resid_drop(const void* A, long lda, int M, int K, const void* Wp, int N, const float* b, float alpha,
                       const float* xin, float* xout, long ld, Drop dr) const {
    GemmEpi e = epi(EPI_RESID, b, alpha);
    e.X = xout;
    e.ldx = ld;
    e.Xin = xin;
    e.drop = dr;
    gemm(g.dt, A, lda, M, K, Wp, kpad(K), N, e, h->zero_page, st);
  }
  void gemm_f32out(const void* A, long lda, int M, int K, const void* Wp, int N, const float* b, float alpha,
                   float* X, long ldx, bool accumulate) const {
    GemmEpi e = epi(accumulate ? EPI_RESID : EPI_SCALE_F32, b, alpha);
    e.X = X;
    e.ldx = ldx;
    gemm(g.dt, A, lda, M, K, Wp, kpad(K), N, e, h->zero_page, st);
  }
  // out (N, K) fp32 = At[N][ldm] . Bt[K][ldm]^T over `rows` (one split-K launch + a fixed-order slab
  // sum; the operand rows carry >= 16 zero granules past `rows`).  With `bias`, Bt has K + 4 rows whose
  // row K is all ones (tpack ones_row), so column K of the product is the bias gradient sum_m dy[m][n].
  void wgrad(const void* At, const void* Bt, long ldm, int N, int K, long rows, float* out, float* bias) const {
    const int Kb = bias ? K + 4 : K;
    const int S = wgrad_splits(N, Kb, rows);
    struct TileScope {   // the wgrad tile for this call only
      int prev = -2;
      explicit TileScope(int t) { if (t >= 0) prev = set_gemm_tile_override(t); }
      ~TileScope() { if (prev != -2) set_gemm_tile_override(prev); }
    } tile_scope(wgrad_tile(N, Kb, rows));
    const int chunk = (int)round_up((rows + S - 1) / S, g.kg);
    GemmEpi e = epi(EPI_SCALE_F32, nullptr);
    e.ldx = Kb;
    if (S == 1 && !bias) {
      e.X = out;
      gemm_ldw(g.dt, At, ldm, N, (int)rows, Bt, ldm, K, e, h->zero_page, st);
      return;
    }
    float* part = W_<float>(wl.part);
    e.X = part;
    if (S == 1) gemm_ldw(g.dt, At, ldm, N, (int)rows, Bt, ldm, Kb, e, h->zero_page, st);
    else gemm_splitk(g.dt, At, ldm, N, (int)rows, Bt, ldm, Kb, S, chunk, e, (long)N * Kb, h->zero_page, st);
    const long n = (long)N * Kb;
    if (bias)
      slab_sum_wb(part, S, N, K, out, bias, st);
    else
      cfm_launch(slab_sum_kernel, dim3(ew_grid(n / 4 + 1)), dim3(256), 0, st, (const float*)part, S, n, out);
  }
  // [dW | db] = A^T . [B' | 1] straight from frame-major compute-type operands (wgrad_tn.hip): A
  // (rows x N, lda) is the packed dy, B (rows x K, ldb) the saved input, B' = dropout(swish(B)) when
  // bfn = 1.  Split-K over the rows into the same [S][N][K+4] partials as wgrad(), at most as many
  // splits as wgrad() would use (the partial buffer is sized for those).
  bool wgrad_rm_ok(int N, int K, long lda, long ldb) const { return wgrad_tn_supported(g.dt, N, K, lda, ldb); }
  void wgrad_rm(const void* A, long lda, int N, const void* B, long ldb, int K, int bfn, Drop bdr, long rows,
                float* out, float* bias) const {
    const int Kb = bias ? K + 4 : K;
    long S = tn_splits(N, K, bias != nullptr, bfn, rows);
    const long chunk = round_up((rows + S - 1) / S, 32);
    S = (rows + chunk - 1) / chunk;
    if (S == 1 && !bias) {
      wgrad_tn(A, lda, N, B, ldb, K, false, bfn, bdr, rows, 1, chunk, out, K, K, 0, st);
      return;
    }
    float* part = W_<float>(wl.part);
    wgrad_tn(A, lda, N, B, ldb, K, bias != nullptr, bfn, bdr, rows, (int)S, chunk, part, Kb, Kb, (long)N * Kb, st);
    const long n = (long)N * Kb;
    if (bias)
      slab_sum_wb(part, (int)S, N, K, out, bias, st);
    else
      cfm_launch(slab_sum_kernel, dim3(ew_grid(n / 4 + 1)), dim3(256), 0, st, (const float*)part, (int)S, n, out);
  }
  void sync(float* buf, long n) const {
    if (o->world > 1 && o->allreduce) {
      if (o->allreduce(o->allreduce_user, buf, (int64_t)n, (void*)st) != 0) fail(CFM_ERR_HIP, "allreduce callback failed");
    }
  }
};

void build_index(Step& S) {
  std::map<std::string, int> idx;
  const auto& pl = S.h->params;
  for (int i = 0; i < (int)pl.size(); ++i) idx[pl[i].first] = i;
  auto I = [&](const std::string& k) {
    auto it = idx.find(k);
    if (it == idx.end()) fail(CFM_ERR_WEIGHTS, "no parameter " + k);
    return it->second;
  };
  S.i_c1w = I("pre_encode.conv.0.weight"); S.i_c1b = I("pre_encode.conv.0.bias");
  S.i_c2w = I("pre_encode.conv.2.weight"); S.i_c2b = I("pre_encode.conv.2.bias");
  S.i_sw = I("pre_encode.out.weight"); S.i_sb = I("pre_encode.out.bias");
  S.lp.resize(S.g.L);
  const char* lnn[5] = {"norm_feed_forward1", "norm_self_att", "norm_conv", "norm_feed_forward2", "norm_out"};
  for (int l = 0; l < S.g.L; ++l) {
    LayerP& q = S.lp[l];
    const std::string p = "layers." + std::to_string(l) + ".";
    for (int i = 0; i < 5; ++i) { q.ln_w[i] = I(p + lnn[i] + ".weight"); q.ln_b[i] = I(p + lnn[i] + ".bias"); }
    for (int f = 0; f < 2; ++f) {
      const std::string ff = p + (f ? "feed_forward2" : "feed_forward1");
      q.ff_w1[f] = I(ff + ".linear1.weight"); q.ff_b1[f] = I(ff + ".linear1.bias");
      q.ff_w2[f] = I(ff + ".linear2.weight"); q.ff_b2[f] = I(ff + ".linear2.bias");
    }
    q.pw1_w = I(p + "conv.pointwise_conv1.weight"); q.pw1_b = I(p + "conv.pointwise_conv1.bias");
    q.dw_w = I(p + "conv.depthwise_conv.weight"); q.dw_b = I(p + "conv.depthwise_conv.bias");
    q.bn_w = I(p + "conv.batch_norm.weight"); q.bn_b = I(p + "conv.batch_norm.bias");
    q.bn_rm = I(p + "conv.batch_norm.running_mean"); q.bn_rv = I(p + "conv.batch_norm.running_var");
    q.pw2_w = I(p + "conv.pointwise_conv2.weight"); q.pw2_b = I(p + "conv.pointwise_conv2.bias");
    q.q_w = I(p + "self_attn.linear_q.weight"); q.q_b = I(p + "self_attn.linear_q.bias");
    q.k_w = I(p + "self_attn.linear_k.weight"); q.k_b = I(p + "self_attn.linear_k.bias");
    q.v_w = I(p + "self_attn.linear_v.weight"); q.v_b = I(p + "self_attn.linear_v.bias");
    q.o_w = I(p + "self_attn.linear_out.weight"); q.o_b = I(p + "self_attn.linear_out.bias");
    q.pos_w = I(p + "self_attn.linear_pos.weight");
    q.pu = I(p + "self_attn.pos_bias_u"); q.pv = I(p + "self_attn.pos_bias_v");
  }
}

// dropout sites: 0 embedding; per layer l: 1 + 8l + {0 ff1 inner, 1 ff1 resid, 2 att resid,
// 3 conv resid, 4 ff2 inner, 5 ff2 resid}
int site(int l, int j) { return 1 + 8 * l + j; }

void check_common(cfm_encoder* h, const float* const* params, int n_params, int B, int T, const cfm_train_opts* o) {
  if (!h || !params || !o) fail(CFM_ERR_INVALID_ARG, "null argument");
  if (n_params != (int)h->params.size()) fail(CFM_ERR_INVALID_ARG, "parameter table size mismatch");
  for (int i = 0; i < n_params; ++i)
    if (!params[i]) fail(CFM_ERR_INVALID_ARG, "null parameter pointer: " + h->params[i].first);
  if (B <= 0 || T <= 0) fail(CFM_ERR_INVALID_ARG, "B and T must be positive");
  if (T > h->max_len) fail(CFM_ERR_INVALID_ARG, "T exceeds max_audio_length");
  if (h->cfg.conv_norm_type != 0) fail(CFM_ERR_UNSUPPORTED, "training supports conv_norm_type='batch_norm' only");
  if (h->has_out_proj) fail(CFM_ERR_UNSUPPORTED, "training with feat_out projection is not built");
  if (h->K != 31) fail(CFM_ERR_UNSUPPORTED, "training is built for conv_kernel_size 31");
  if (o->dropout < 0.0f || o->dropout >= 1.0f) fail(CFM_ERR_INVALID_ARG, "dropout must be in [0, 1)");
  if (o->dropout_att < 0.0f || o->dropout_att >= 1.0f) fail(CFM_ERR_INVALID_ARG, "dropout_att must be in [0, 1)");
  if (o->dropout_emb < 0.0f || o->dropout_emb >= 1.0f) fail(CFM_ERR_INVALID_ARG, "dropout_emb must be in [0, 1)");
  if (o->world < 1) fail(CFM_ERR_INVALID_ARG, "world must be >= 1");
  if (h->d % 8 || h->C % 8) fail(CFM_ERR_UNSUPPORTED, "d_model and conv channels must be multiples of 8");
}

// =============================================================================================
// forward
// =============================================================================================
void train_forward(Step& S, const float* x_bft, const int32_t* len_b, float* y_bdt, int32_t* out_len_b) {
  const Geo& g = S.g;
  cfm_encoder* h = S.h;
  hipStream_t st = S.st;
  const int dt = g.dt, d = g.d, M = g.M, H = g.H, dkp = g.dkp, es = g.es;
  const long HP = (long)H * dkp;
  int32_t* lens = S.T_<int32_t>(S.tp.lens);
  calc_length(len_b, lens, g.B, g.T, 2, st);
  // enable_pad_mask(False) (conformer_encoder.py:269-272): the conv module's GLU output is not zeroed on
  // padded frames (the attention masks stay); the backward reads the same handle flag
  const int32_t* glu_lens = S.h->use_pad_mask ? lens : nullptr;
  HIP_OK(hipMemcpyAsync(S.T_(S.tp.xin), x_bft, (size_t)g.B * g.F * g.T * 4, hipMemcpyDeviceToDevice, st));

  // ---- ConvSubsampling (subsampling.py:163-176) + xscale + embedding dropout ----
  conv1_subsample(dt, x_bft, g.B, g.F, g.T, S.prm(S.i_c1w), S.prm(S.i_c1b), g.C, S.T_(S.tp.X1), st);
  S.perm(S.prm(S.i_c2w), 2, S.W_(S.wl.wc2), false, S.kpad(9L * g.C), S.npad(g.C), S.kpad(9L * g.C));
  S.bias(S.prm(S.i_c2b), g.C, S.W_<float>(S.wl.bc2));
  {
    ConvGeom cg{S.T_(S.tp.X1), g.T1, g.F1, g.T2, g.F2, g.C};
    GemmEpi e = S.epi(EPI_RELU, S.W_<float>(S.wl.bc2));
    e.C = S.T_(S.tp.X2);
    e.ldc = g.C;
    gemm_conv(dt, cg, g.B, S.W_(S.wl.wc2), S.kpad(9L * g.C), g.C, e, h->zero_page, st);
  }
  S.perm(S.prm(S.i_sw), 0, S.W_(S.wl.wsub), false, S.kpad((long)g.F2 * g.C), S.npad(d), S.kpad((long)g.F2 * g.C));
  S.bias(S.prm(S.i_sb), d, S.W_<float>(S.wl.bsub));
  const float xs = h->cfg.xscaling ? (float)std::sqrt((double)d) : 1.0f;
  float* xcur = g.L > 0 ? S.T_<float>(S.tp.lay[0].x[0]) : S.T_<float>(S.tp.xfin);
  S.gemm_f32out(S.T_(S.tp.X2), (long)g.F2 * g.C, M, g.F2 * g.C, S.W_(S.wl.wsub), d, S.W_<float>(S.wl.bsub), xs, xcur,
                d, false);
  // abs_pos: + pe[:, :T'] between the xscale and the embedding dropout (multi_head_attention.py:265-271);
  // a constant, so the backward is unchanged
  if (h->abs_pos) add_rows_f32(xcur, h->pe_abs, g.B, g.Tp, d, st);
  {
    const Drop dr = S.drop(0);
    if (dr.thr) cfm_launch(scale_drop_kernel, dim3(ew_grid((long)M * d)), dim3(256), 0, st, (const float*)xcur, 1.0f,
                           (long)M * d, dr, xcur);
  }
  const char* pe_slice = S.pos_window();
  const long n_md = (long)M * d;

  for (int l = 0; l < g.L; ++l) {
    const LayerP& q = S.lp[l];
    const TapeLayer& t = S.tp.lay[l];
    float* X[5];
    for (int i = 0; i < 5; ++i) X[i] = S.T_<float>(t.x[i]);
    // this layer's linear weights and biases, packed in one launch
    {
      Step::Batch b;
      const long sw1[2] = {S.wl.w1, S.wl.w1b}, sb1[2] = {S.wl.b1, S.wl.b1b}, sw2[2] = {S.wl.w2, S.wl.w2b},
                 sb2[2] = {S.wl.b2, S.wl.b2b};
      for (int f = 0; f < 2; ++f) {
        S.jobW(b, S.prm(q.ff_w1[f]), g.dff, d, S.W_(sw1[f]));
        S.jobBias(b, S.prm(q.ff_b1[f]), g.dff, S.W_<float>(sb1[f]));
        S.jobW(b, S.prm(q.ff_w2[f]), d, g.dff, S.W_(sw2[f]));
        S.jobBias(b, S.prm(q.ff_b2[f]), d, S.W_<float>(sb2[f]));
      }
      S.jobW(b, S.prm(q.o_w), d, d, S.W_(S.wl.wout));
      S.jobBias(b, S.prm(q.o_b), d, S.W_<float>(S.wl.bout));
      S.jobW(b, S.prm(q.pw1_w), 2 * d, d, S.W_(S.wl.wpw1));
      S.jobBias(b, S.prm(q.pw1_b), 2 * d, S.W_<float>(S.wl.bpw1));
      S.jobW(b, S.prm(q.pw2_w), d, d, S.W_(S.wl.wpw2));
      S.jobBias(b, S.prm(q.pw2_b), d, S.W_<float>(S.wl.bpw2));
      S.flush(b);
    }
    // ---- FFN1 / FFN2 (conformer_modules.py:99-101, 116-118, 183-200) ----
    auto ffn = [&](int f, float* xin, void* hn, long z, long u, float* xout) {
      const long w1 = f ? S.wl.w1b : S.wl.w1, b1 = f ? S.wl.b1b : S.wl.b1;
      const long w2 = f ? S.wl.w2b : S.wl.w2, b2 = f ? S.wl.b2b : S.wl.b2;
      const Drop di = S.drop(site(l, f ? 4 : 0));
      // z (the backward's tape) and u = dropout(swish(z)) from one GEMM epilogue
      GemmEpi e = S.epi(EPI_SWISH_Z, S.W_<float>(b1));
      e.C = S.T_(z);
      e.C2 = S.T_(u);
      e.ldc = g.dff;
      e.drop = di;
      gemm(dt, hn, d, M, d, S.W_(w1), S.kpad(d), g.dff, e, h->zero_page, st);
      S.gemm_resid_drop(S.T_(u), g.dff, M, g.dff, S.W_(w2), d, S.W_<float>(b2), 0.5f, xin, xout, d,
                        S.drop(site(l, f ? 5 : 1)));
    };
    layernorm(dt, X[0], M, d, S.prm(q.ln_w[LN_FF1]), S.prm(q.ln_b[LN_FF1]), nullptr, nullptr, nullptr, S.T_(t.hn[0]),
              0, st);
    ffn(0, X[0], S.T_(t.hn[0]), t.z1, t.u1, X[1]);

    // ---- rel-pos MHSA (conformer_modules.py:103-110) ----
    layernorm(dt, X[1], M, d, S.prm(q.ln_w[LN_ATT]), S.prm(q.ln_b[LN_ATT]), nullptr, nullptr, nullptr, S.T_(t.hn[1]),
              0, st);
    {
      S.heads(S.prm(q.pos_w), nullptr, nullptr, 1, d, S.W_(S.wl.wpos), false, S.kpad(d), S.npad(HP));
      GemmEpi ep = S.epi(EPI_STORE, nullptr);
      ep.C = S.T_(t.P);
      ep.ldc = HP;
      gemm(dt, pe_slice, d, g.NP, d, S.W_(S.wl.wpos), S.kpad(d), (int)HP, ep, h->zero_page, st);
      S.heads(S.prm(q.q_w), S.prm(q.k_w), S.prm(q.v_w), 3, d, S.W_(S.wl.wqkv), false, S.kpad(d), S.npad(3 * HP));
      S.heads(S.prm(q.q_b), S.prm(q.k_b), S.prm(q.v_b), 3, 1, S.W_(S.wl.bqkv), true, 1, S.npad(3 * HP));
      S.heads(S.prm(q.pu), S.prm(q.pv), nullptr, 2, 1, S.W_(S.wl.uv), true, 1, (int)(2 * HP));
      GemmEpi e = S.epi(EPI_QKV, S.W_<float>(S.wl.bqkv));
      e.C = S.T_(t.qk); e.ldc = 3 * HP; e.qk_cols = (int)(2 * HP); e.uv = S.W_<float>(S.wl.uv);
      e.qscale = (float)(1.4426950408889634 / std::sqrt((double)g.dk));
      e.Vt = S.T_(t.vt); e.H = H; e.dkp = dkp; e.vt_rows = h->vt_rows; e.Tpad = g.Tpad; e.Tp = g.Tp;
      gemm(dt, S.T_(t.hn[1]), d, M, d, S.W_(S.wl.wqkv), S.kpad(d), (int)(3 * HP), e, h->zero_page, st);
      rel_pos_attention(dt, S.T_(t.qk), 3 * HP, S.T_(t.vt), h->vt_rows, g.Tpad, S.T_(t.P), HP, lens, g.B, g.Tp, H,
                        g.dk, dkp, h->cfg.att_context_left, h->cfg.att_context_right, S.T_(t.ctx), d, st,
                        S.drop_att(l));
      S.gemm_resid_drop(S.T_(t.ctx), d, M, d, S.W_(S.wl.wout), d, S.W_<float>(S.wl.bout), 1.0f, X[1], X[2], d,
                        S.drop(site(l, 2)));
    }

    // ---- convolution module (conformer_modules.py:112-114, 160-180) ----
    layernorm(dt, X[2], M, d, S.prm(q.ln_w[LN_CONV]), S.prm(q.ln_b[LN_CONV]), nullptr, nullptr, nullptr,
              S.T_(t.hn[2]), 0, st);
    {
      float* pre = S.T_<float>(t.pre);
      S.gemm_f32out(S.T_(t.hn[2]), d, M, d, S.W_(S.wl.wpw1), 2 * d, S.W_<float>(S.wl.bpw1), 1.0f, pre, 2 * d, false);
      if (dt == DT_F32)
        cfm_launch(glu_fwd_kernel<float>, dim3(ew_grid(n_md)), dim3(256), 0, st, (const float*)pre,
                   (const int32_t*)glu_lens, g.Tp, d, (long)M, S.T_<float>(t.g), S.W_<float>(S.wl.gt));
      else
        cfm_launch(glu_fwd_kernel<bf16_t>, dim3(ew_grid(n_md)), dim3(256), 0, st, (const float*)pre,
                   (const int32_t*)glu_lens, g.Tp, d, (long)M, S.T_<float>(t.g), S.W_<bf16_t>(S.wl.gt));
      // depthwise conv + bias (fp32 pre-norm output; [K][d] weight layout of the forward kernel)
      pack_matrix(DT_F32, S.prm(q.dw_w), g.K, d, g.K, true, S.W_(S.wl.dww), d, g.K, d, st);
      float* dwo = S.W_<float>(S.wl.dwo);
      dwconv_norm_swish(dt, S.W_(S.wl.gt), g.B, g.Tp, d, g.K, S.W_<float>(S.wl.dww), S.prm(q.dw_b), nullptr, nullptr,
                        nullptr, nullptr, nullptr, dwo, st);
      // BatchNorm1d, training statistics (SyncBatchNorm over `world` ranks when a callback is given)
      float* red = S.W_<float>(S.wl.red);
      float* sy = S.W_<float>(S.wl.sync);
      float* mean = S.T_<float>(t.mean);
      float* rstd = S.T_<float>(t.rstd);
      // [sum x (d) | this rank's frame count] summed over the ranks in one call, then [sum (x-mean)^2]
      float* sy2 = sy + d + 1;
      colred(dwo, nullptr, nullptr, d, M, d, 0, 1.0f, sy, 0, red, st);
      cfm_launch(fill_kernel, dim3(1), dim3(64), 0, st, sy + d, 1L, (float)M);
      S.sync(sy, d + 1);
      cfm_launch(bn_finalize_kernel, dim3((d + 255) / 256), dim3(256), 0, st, (const float*)sy, (const float*)sy,
                 (const float*)(sy + d), d, 0.0f, mean, rstd, (float*)nullptr, (float*)nullptr, 0);
      colred(dwo, nullptr, mean, d, M, d, 2, 1.0f, sy2, 0, red, st);
      S.sync(sy2, d);
      const bool upd = S.o->update_running_stats != 0;
      cfm_launch(bn_finalize_kernel, dim3((d + 255) / 256), dim3(256), 0, st, (const float*)sy, (const float*)sy2,
                 (const float*)(sy + d), d, S.o->bn_momentum, mean, rstd, upd ? (float*)S.prm(q.bn_rm) : (float*)nullptr,
                 upd ? (float*)S.prm(q.bn_rv) : (float*)nullptr, 1);
      if (dt == DT_F32)
        cfm_launch(bn_swish_kernel<float>, dim3(ew_grid(n_md)), dim3(256), 0, st, (const float*)dwo, (const float*)mean,
                   (const float*)rstd, S.prm(q.bn_w), S.prm(q.bn_b), (long)M, d, S.T_<float>(t.xhat),
                   S.T_<float>(t.s));
      else
        cfm_launch(bn_swish_kernel<bf16_t>, dim3(ew_grid(n_md)), dim3(256), 0, st, (const float*)dwo,
                   (const float*)mean, (const float*)rstd, S.prm(q.bn_w), S.prm(q.bn_b), (long)M, d,
                   S.T_<float>(t.xhat), S.T_<bf16_t>(t.s));
      S.gemm_resid_drop(S.T_(t.s), d, M, d, S.W_(S.wl.wpw2), d, S.W_<float>(S.wl.bpw2), 1.0f, X[2], X[3], d,
                        S.drop(site(l, 3)));
    }
    layernorm(dt, X[3], M, d, S.prm(q.ln_w[LN_FF2]), S.prm(q.ln_b[LN_FF2]), nullptr, nullptr, nullptr, S.T_(t.hn[3]),
              0, st);
    ffn(1, X[3], S.T_(t.hn[3]), t.z2, t.u2, X[4]);
    // ---- norm_out (conformer_modules.py:120) -> next layer's input (fp32) ----
    float* nxt = l + 1 < g.L ? S.T_<float>(S.tp.lay[l + 1].x[0]) : S.T_<float>(S.tp.xfin);
    layernorm(dt, X[4], M, d, S.prm(q.ln_w[LN_OUT]), S.prm(q.ln_b[LN_OUT]), nxt, nullptr, nullptr, nullptr, 0, st);
  }
  // (B, T', d) -> (B, d, T') (conformer_encoder.py:280) and the encoded lengths
  {
    const dim3 grid((g.Tp + 31) / 32, (d + 31) / 32, g.B);
    cfm_launch(btd_transpose_kernel, grid, dim3(256), 0, st, (const float*)S.T_<float>(S.tp.xfin), g.Tp, d, 1, y_bdt);
    HIP_OK(hipMemcpyAsync(out_len_b, lens, (size_t)g.B * 4, hipMemcpyDeviceToDevice, st));
  }
}

// =============================================================================================
// backward
// =============================================================================================
// parameter-table rows (build_param_list): pre_encode.* first, then one equal block per layer
constexpr int kPreEncodeRows = 6;

void grad_ready(const Step& S, int first, int n) {
  const cfm_train_opts* o = S.o;
  if (!o->grad_ready || n <= 0) return;
  if (o->grad_ready(o->grad_ready_user, first, n, (void*)S.st) != 0) fail(CFM_ERR_HIP, "grad_ready callback failed");
}

void train_backward(Step& S, const float* dy_bdt, float* const* G) {
  const Geo& g = S.g;
  cfm_encoder* h = S.h;
  hipStream_t st = S.st;
  const int dt = g.dt, d = g.d, M = g.M, H = g.H, dkp = g.dkp, es = g.es;
  const long HP = (long)H * dkp, n_md = (long)M * d;
  const int32_t* lens = S.T_<const int32_t>(S.tp.lens);
  float* gA = S.W_<float>(S.wl.gA);
  float* gB = S.W_<float>(S.wl.gB);
  float* dbr = S.W_<float>(S.wl.dbr);
  float* red = S.W_<float>(S.wl.red);
  const int layer_rows = g.L > 0 ? ((int)h->params.size() - kPreEncodeRows - (h->has_out_proj ? 2 : 0)) / g.L : 0;
  void* pa = S.W_(S.wl.pa);
  void* pat = S.W_(S.wl.pat);
  void* pbt = S.W_(S.wl.pbt);
  void* wt = S.W_(S.wl.wt);
  const long Mq = g.Mq;
  auto Gp = [&](int i) -> float* { return G ? G[i] : nullptr; };
  const char* pos_win = S.pos_window();   // the forward's (dropout_emb) positional window
  // Linear y = x W^T + b backward for a dense fp32 output gradient dy (M, N):
  //   dx (M, K) fp32 (ldx; accumulate or overwrite), dW (N, K) -> G[gw], db -> G[gb]
  //   x is the saved compute-type input (M, K) (ld ldxin), or xfn = 1: dropout(swish(z)) recomputed
  //   dy may carry a scale and a dropout mask (ysc, ydr: the residual branch's dropout backward),
  //   applied while packing (or by one elementwise pass into dbr when no transposed pack is needed)
  auto linear_bwd = [&](const float* dy, int N, const float* w, int K, const void* xin, long ldxin, int xfn, Drop xdr,
                        float* dx, long ldx, bool acc, int gw, int gb, const void* wtp, float ysc = 1.0f,
                        Drop ydr = Drop{0, 0, 1.0f}, bool prepacked = false) {
    const bool want_w = gw >= 0 && Gp(gw), want_b = gb >= 0 && Gp(gb);
    if ((want_w || want_b) && S.wgrad_rm_ok(N, K, S.kpad(N), ldxin)) {
      // dy packed once (row-major, scale + dropout applied), used by the dgrad GEMM and, as it lies,
      // by the weight gradient; the saved input is read in place.  prepacked: the LayerNorm backward
      // that produced dy already wrote that operand into pa (ln_bwd pk)
      if (!prepacked) S.pack2(dy, N, M, N, pa, S.kpad(N), M, S.kpad(N), nullptr, 0, 0, 0, ysc, ydr);
      if (dx) {
        const void* W = wtp;
        if (!W) {
          S.packWt(w, N, K, wt);
          W = wt;
        }
        S.gemm_f32out(pa, S.kpad(N), M, N, W, K, nullptr, 1.0f, dx, ldx, acc);
      }
      S.wgrad_rm(pa, S.kpad(N), N, xin, ldxin, K, xfn, xdr, M, want_w ? Gp(gw) : nullptr, want_b ? Gp(gb) : nullptr);
      return;
    }
    const bool fused_y = dx && (want_w || want_b);
    if (!fused_y && (ysc != 1.0f || ydr.thr)) {
      cfm_launch(scale_drop_kernel, dim3(ew_grid((long)M * N)), dim3(256), 0, st, dy, ysc, (long)M * N, ydr, dbr);
      dy = dbr;
    }
    if (fused_y)
      S.pack2(dy, N, M, N, pa, S.kpad(N), M, S.kpad(N), pat, Mq, N, (int)Mq, ysc, ydr);
    else if (dx)
      S.pack(dy, false, N, M, N, false, 1.0f, pa, S.kpad(N), M, S.kpad(N));
    if (dx) {
      const void* W = wtp;   // prepacked by the layer's batch, or packed here
      if (!W) {
        S.packWt(w, N, K, wt);
        W = wt;
      }
      S.gemm_f32out(pa, S.kpad(N), M, N, W, K, nullptr, 1.0f, dx, ldx, acc);
    }
    if (want_w || want_b) {   // [dW | db] = dy^T . [x | 1]
      if (!dx) S.pack(dy, false, N, M, N, true, 1.0f, pat, Mq, N, (int)Mq);
      S.pack(xin, true, ldxin, M, K, true, 1.0f, pbt, Mq, S.npad(K + 4), (int)Mq, xfn, xdr, want_b ? K : -1);
      S.wgrad(pat, pbt, Mq, N, K, M, want_w ? Gp(gw) : nullptr, want_b ? Gp(gb) : nullptr);
    }
  };
  // pk: also write the next consumer's bf16 GEMM operand (pa) = bf16(dx * pscale * dropout'), see
  // ln_bwd_fused_kernel; only where pa is that operand as it lies (bf16, kpad(d) == d)
  static const bool ln_pack_env = [] {   // CFM_LN_PACK=0: separate pack passes (A/B, equality tests)
    const char* e = getenv("CFM_LN_PACK");
    return !(e && e[0] == '0');
  }();
  const bool ln_pack = ln_pack_env && dt == DT_BF16 && S.kpad(d) == d;
  ColredList ln_slots{};   // this layer's LayerNorm partials awaiting ln_flush (five per layer)
  auto ln_bwd = [&](const float* x, int wi, int bi, const float* dy, float* dx, bool acc, bool pk = false,
                    float pscale = 1.0f, Drop pdr = Drop{0, 0, 1.0f}) {
    bf16_t* pkp = (pk && ln_pack) ? (bf16_t*)pa : nullptr;
    const int slot = ln_slots.count / 2;
    // dx (+)= LN backward; per-block column partials of dy*xhat and dy (in dbr), then folded
    const int nblk = (M + 4 * kLnRowsPerWave - 1) / (4 * kLnRowsPerWave);
    // column partials into the layer's slot; one colred_multi launch per layer folds all five
    float* pw = S.W_<float>(S.wl.lnp) + (long)slot * 2 * nblk * d;
    float* pb = pw + (long)nblk * d;
    const int E4 = (d / 4 + 63) / 64;
    const dim3 grid(nblk), blk(256);
    if (E4 <= 1) cfm_launch(ln_bwd_fused_kernel<1>, grid, blk, 0, st, x, S.prm(wi), dy, M, d, dx, acc ? 1 : 0, pw, pb, pkp, pscale, pdr);
    else if (E4 <= 2) cfm_launch(ln_bwd_fused_kernel<2>, grid, blk, 0, st, x, S.prm(wi), dy, M, d, dx, acc ? 1 : 0, pw, pb, pkp, pscale, pdr);
    else if (E4 <= 4) cfm_launch(ln_bwd_fused_kernel<4>, grid, blk, 0, st, x, S.prm(wi), dy, M, d, dx, acc ? 1 : 0, pw, pb, pkp, pscale, pdr);
    else cfm_launch(ln_bwd_fused_kernel<8>, grid, blk, 0, st, x, S.prm(wi), dy, M, d, dx, acc ? 1 : 0, pw, pb, pkp, pscale, pdr);
    ln_slots.p[ln_slots.count] = pw; ln_slots.o[ln_slots.count++] = Gp(wi);
    ln_slots.p[ln_slots.count] = pb; ln_slots.o[ln_slots.count++] = Gp(bi);
  };
  auto ln_flush = [&]() {
    const int nblk = (M + 4 * kLnRowsPerWave - 1) / (4 * kLnRowsPerWave);
    bool any = false;
    for (int i = 0; i < ln_slots.count; ++i) any = any || ln_slots.o[i] != nullptr;
    if (any)
      cfm_launch(colred_multi_kernel, dim3((d + 15) / 16, ln_slots.count), dim3(256), 0, st, ln_slots, nblk, d);
    ln_slots = ColredList{};
  };

  // dy (B, d, T') -> gA (B*T', d)
  {
    const dim3 grid((g.Tp + 31) / 32, (d + 31) / 32, g.B);
    cfm_launch(btd_transpose_kernel, grid, dim3(256), 0, st, dy_bdt, g.Tp, d, 0, gA);
  }
  for (int l = g.L - 1; l >= 0; --l) {
    const LayerP& q = S.lp[l];
    const TapeLayer& t = S.tp.lay[l];
    const float* X[5];
    for (int i = 0; i < 5; ++i) X[i] = S.T_<const float>(t.x[i]);
    // the layer's transposed weights for every dgrad GEMM (W_q/W_k/W_v stacked into wt), one launch
    void* WT[7];
    for (int i = 0; i < 7; ++i) WT[i] = S.W_(S.wl.wtl[i]);
    {
      Step::Batch b;
      S.jobWt(b, S.prm(q.ff_w2[0]), d, g.dff, WT[WT_FF1_W2]);
      S.jobWt(b, S.prm(q.ff_w1[0]), g.dff, d, WT[WT_FF1_W1]);
      S.jobWt(b, S.prm(q.ff_w2[1]), d, g.dff, WT[WT_FF2_W2]);
      S.jobWt(b, S.prm(q.ff_w1[1]), g.dff, d, WT[WT_FF2_W1]);
      S.jobWt(b, S.prm(q.pw2_w), d, d, WT[WT_PW2]);
      S.jobWt(b, S.prm(q.pw1_w), 2 * d, d, WT[WT_PW1]);
      S.jobWt(b, S.prm(q.o_w), d, d, WT[WT_OUT]);
      const long ldw = S.kpad(3L * d);
      const int wi[3] = {q.q_w, q.k_w, q.v_w};
      for (int p = 0; p < 3; ++p)   // Wt[i][p*d + o] = W_p[o][i]
        S.job(b, S.prm(wi[p]), d, d, d, true, (char*)wt + (long)p * d * es, ldw, S.npad(d),
              p == 2 ? (int)(ldw - 2L * d) : d, false);
      S.flush(b);
    }
    // norm_out: gB = d x4
    ln_bwd(X[4], q.ln_w[LN_OUT], q.ln_b[LN_OUT], gA, gB, false, true, 0.5f, S.drop(site(l, 5)));   // + FFN2's operand

    // FFN block backward: residual grad g (d xout) -> += d xin through the branch
    // packed: pa already holds bf16(0.5 * dropout'(gres)) (the preceding ln_bwd); the block's own
    // closing ln_bwd writes the next consumer's operand (nscale, ndrop) when npack
    auto ffn_bwd = [&](int f, const float* xin, const void* hn, long z, long u, float* gres, bool packed, bool npack,
                       float nscale, Drop ndrop) {
      float* dU = S.W_<float>(S.wl.dU);
      const Drop dres = S.drop(site(l, f ? 5 : 1));
      const Drop di = S.drop(site(l, f ? 4 : 0));
      float* dhn = S.W_<float>(S.wl.dctx);
      if (S.kpad(g.dff) == g.dff) {
        // linear2's dgrad carries the Swish + dropout backward in its epilogue and writes the FFN
        // hidden's gradient dz in the compute type (no fp32 round trip, no elementwise pass); dz then
        // feeds linear1's dgrad as its A operand directly and its wgrad through one transpose pack
        void* dz = S.W_(S.wl.dU);
        {
          const int N = d, K = g.dff;
          const bool want_w = Gp(q.ff_w2[f]) != nullptr, want_b = Gp(q.ff_b2[f]) != nullptr;
          const bool rm = S.wgrad_rm_ok(N, K, S.kpad(N), K) && S.wgrad_rm_ok(K, N, K, d);
          if (rm) {
            if (!(packed && ln_pack)) S.pack2(gres, N, M, N, pa, S.kpad(N), M, S.kpad(N), nullptr, 0, 0, 0, 0.5f, dres);
          } else if (want_w || want_b) {
            S.pack2(gres, N, M, N, pa, S.kpad(N), M, S.kpad(N), pat, Mq, N, (int)Mq, 0.5f, dres);
          } else {
            cfm_launch(scale_drop_kernel, dim3(ew_grid(n_md)), dim3(256), 0, st, (const float*)gres, 0.5f, n_md, dres,
                       dbr);
            S.pack(dbr, false, N, M, N, false, 1.0f, pa, S.kpad(N), M, S.kpad(N));
          }
          GemmEpi e = S.epi(EPI_SWISH_BWD, nullptr);
          e.C = dz; e.ldc = K; e.zin = S.T_(z); e.ldz = K; e.drop = di;
          gemm(dt, pa, S.kpad(N), M, N, WT[f ? WT_FF2_W2 : WT_FF1_W2], S.kpad(N), K, e, h->zero_page, st);
          if (rm && (want_w || want_b)) {   // [dW2 | db2] = dy^T . [u | 1], u = dropout(swish(z)) recomputed
            S.wgrad_rm(pa, S.kpad(N), N, S.T_(u), K, K, 0, Drop{0, 0, 1.0f}, M, want_w ? Gp(q.ff_w2[f]) : nullptr,
                       want_b ? Gp(q.ff_b2[f]) : nullptr);
          } else if (want_w || want_b) {
            S.pack(S.T_(z), true, K, M, K, true, 1.0f, pbt, Mq, S.npad(K + 4), (int)Mq, 1, di, want_b ? K : -1);
            S.wgrad(pat, pbt, Mq, N, K, M, want_w ? Gp(q.ff_w2[f]) : nullptr, want_b ? Gp(q.ff_b2[f]) : nullptr);
          }
        }
        {
          const int N = g.dff, K = d;
          S.gemm_f32out(dz, N, M, N, WT[f ? WT_FF2_W1 : WT_FF1_W1], K, nullptr, 1.0f, dhn, d, false);
          const bool want_w = Gp(q.ff_w1[f]) != nullptr, want_b = Gp(q.ff_b1[f]) != nullptr;
          if ((want_w || want_b) && S.wgrad_rm_ok(N, K, N, d)) {   // [dW1 | db1] = dz^T . [hn | 1]
            S.wgrad_rm(dz, N, N, hn, d, K, 0, Drop{0, 0, 1.0f}, M, want_w ? Gp(q.ff_w1[f]) : nullptr,
                       want_b ? Gp(q.ff_b1[f]) : nullptr);
          } else if (want_w || want_b) {
            S.pack(dz, true, N, M, N, true, 1.0f, pat, Mq, N, (int)Mq);
            S.pack(hn, true, d, M, K, true, 1.0f, pbt, Mq, S.npad(K + 4), (int)Mq, 0, Drop{0, 0, 1.0f},
                   want_b ? K : -1);
            S.wgrad(pat, pbt, Mq, N, K, M, want_w ? Gp(q.ff_w1[f]) : nullptr, want_b ? Gp(q.ff_b1[f]) : nullptr);
          }
        }
      } else {
        // linear2 (input u = dropout(swish(z)) recomputed from z)
        linear_bwd(gres, d, S.prm(q.ff_w2[f]), g.dff, S.T_(z), g.dff, 1, di, dU, g.dff, false, q.ff_w2[f], q.ff_b2[f],
                   WT[f ? WT_FF2_W2 : WT_FF1_W2], 0.5f, dres);
        const long n = (long)M * g.dff;
        if (dt == DT_F32)
          cfm_launch(swish_drop_bwd_kernel<float>, dim3(ew_grid(n)), dim3(256), 0, st, S.T_<const float>(z),
                     (const float*)dU, n, di, dU);
        else
          cfm_launch(swish_drop_bwd_kernel<bf16_t>, dim3(ew_grid(n)), dim3(256), 0, st, S.T_<const bf16_t>(z),
                     (const float*)dU, n, di, dU);
        linear_bwd(dU, g.dff, S.prm(q.ff_w1[f]), d, hn, d, 0, Drop{0, 0, 1.0f}, dhn, d, false, q.ff_w1[f],
                   q.ff_b1[f], WT[f ? WT_FF2_W1 : WT_FF1_W1]);
      }
      ln_bwd(xin, q.ln_w[f ? LN_FF2 : LN_FF1], q.ln_b[f ? LN_FF2 : LN_FF1], dhn, gres, true, npack, nscale, ndrop);
    };
    ffn_bwd(1, X[3], S.T_(t.hn[3]), t.z2, t.u2, gB, true, true, 1.0f, S.drop(site(l, 3)));   // gB = d x3 (+ pw2's operand)

    // ---- convolution module ----
    {
      float* dS = S.W_<float>(S.wl.dD);
      linear_bwd(gB, d, S.prm(q.pw2_w), d, S.T_(t.s), d, 0, Drop{0, 0, 1.0f}, dS, d, false, q.pw2_w, q.pw2_b,
                 WT[WT_PW2], 1.0f, S.drop(site(l, 3)), ln_pack);
      float* dZ = S.W_<float>(S.wl.dG);
      const float* xhat = S.T_<const float>(t.xhat);
      cfm_launch(bn_swish_bwd_kernel, dim3(ew_grid(n_md)), dim3(256), 0, st, (const float*)dS, xhat, S.prm(q.bn_w),
                 S.prm(q.bn_b), (long)M, d, dZ);
      // BatchNorm backward: local sums -> dgamma/dbeta, global sums (SyncBN) -> dx
      float* sy = S.W_<float>(S.wl.sync);
      colred(dZ, nullptr, nullptr, d, M, d, 0, 1.0f, sy, 0, red, st);
      colred(dZ, xhat, nullptr, d, M, d, 1, 1.0f, sy + d, 0, red, st);
      {
        CopyList cl{};
        cl.src[0] = sy; cl.dst[0] = Gp(q.bn_b); cl.n[0] = d;
        cl.src[1] = sy + d; cl.dst[1] = Gp(q.bn_w); cl.n[1] = d;
        cl.count = 2;
        cfm_launch(copy_multi_kernel, dim3(ew_grid(d), 2), dim3(256), 0, st, cl);
      }
      S.sync(sy, 2L * d);
      float* dD = dS;   // dS is dead after dZ
      cfm_launch(bn_bwd_apply_kernel, dim3(ew_grid(n_md)), dim3(256), 0, st, (const float*)dZ, xhat, S.prm(q.bn_w),
                 S.T_<const float>(t.rstd), (const float*)sy, (const float*)(sy + d),
                 S.T_<const float>(t.mean) + d, (long)M, d, dD);
      // depthwise conv backward (dx, dw, db) from the fp32 GLU output
      float* dG = dZ;   // dZ is dead after dD
      const size_t dwws = cfm_op_dwconv_backward_ws_size(g.B, g.Tp, d, g.K);
      const cfm_status s = cfm_op_dwconv_backward(S.T_<const float>(t.g), S.prm(q.dw_w), dD, g.B, g.Tp, d, g.K, dG,
                                                  Gp(q.dw_w), Gp(q.dw_b), red, dwws, st);
      if (s != CFM_OK) fail(s, std::string("dwconv backward: ") + g_last_error);
      float* dpre = S.W_<float>(S.wl.dpre);
      const cfm_status s2 = cfm_op_glu_backward(S.T_<const float>(t.pre), dG, h->use_pad_mask ? lens : nullptr, g.B,
                                                g.Tp, d, dpre, st);
      if (s2 != CFM_OK) fail(s2, std::string("glu backward: ") + g_last_error);
      float* dhn = S.W_<float>(S.wl.dctx);
      linear_bwd(dpre, 2 * d, S.prm(q.pw1_w), d, S.T_(t.hn[2]), d, 0, Drop{0, 0, 1.0f}, dhn, d, false, q.pw1_w,
                 q.pw1_b, WT[WT_PW1]);
      ln_bwd(X[2], q.ln_w[LN_CONV], q.ln_b[LN_CONV], dhn, gB, true, true, 1.0f, S.drop(site(l, 2)));   // gB = d x2 (+ out's operand)
    }

    // ---- attention ----
    {
      float* dctx = S.W_<float>(S.wl.dctx);
      linear_bwd(gB, d, S.prm(q.o_w), d, S.T_(t.ctx), d, 0, Drop{0, 0, 1.0f}, dctx, d, false, q.o_w, q.o_b,
                 WT[WT_OUT], 1.0f, S.drop(site(l, 2)), ln_pack);
      float* dqkv = S.W_<float>(S.wl.dqkv);
      float* dP = S.W_<float>(S.wl.dP);
      const int dk = g.dk;
      rel_pos_attention_backward(dt, S.T_(t.qk), 3 * HP, S.T_(t.vt), h->vt_rows, g.Tpad, S.T_(t.P), HP, lens, g.B,
                                 g.Tp, H, dk, dkp, h->cfg.att_context_left, h->cfg.att_context_right, dctx, d, dqkv,
                                 dqkv + d, dqkv + 2 * d, 3L * d, dP, d, Gp(q.pu), Gp(q.pv), S.W_(S.wl.attws), st,
                                 S.drop_att(l));
      // linear_pos (no bias): dWpos = dP^T . pos_emb   (pos_emb rows = the PE window after
      // dropout_emb, regenerated from the step's seed; compute type)
      if (Gp(q.pos_w)) {
        const char* pe_slice = pos_win;
        if (S.wgrad_rm_ok(d, d, S.kpad(d), d)) {
          S.pack(dP, false, d, g.NP, d, false, 1.0f, pa, S.kpad(d), g.NP, S.kpad(d));
          S.wgrad_rm(pa, S.kpad(d), d, pe_slice, d, d, 0, Drop{0, 0, 1.0f}, g.NP, Gp(q.pos_w), nullptr);
        } else {
          S.pack(dP, false, d, g.NP, d, true, 1.0f, pat, Mq, d, (int)Mq);
          S.pack(pe_slice, true, d, g.NP, d, true, 1.0f, pbt, Mq, S.npad(d), (int)Mq);
          S.wgrad(pat, pbt, Mq, d, d, g.NP, Gp(q.pos_w), nullptr);
        }
      }
      // q/k/v: biases, input gradient through [Wq; Wk; Wv], stacked weight gradient
      S.pack(dqkv, false, 3L * d, M, 3 * d, false, 1.0f, pa, S.kpad(3L * d), M, S.kpad(3L * d));
      {
        const int wi[3] = {q.q_w, q.k_w, q.v_w};   // their W^T is in wt (the layer's batch)
        float* dhn = dctx;   // dctx consumed
        S.gemm_f32out(pa, S.kpad(3L * d), M, 3 * d, wt, d, nullptr, 1.0f, dhn, d, false);
        const int bi3[3] = {q.q_b, q.k_b, q.v_b};
        if (Gp(q.q_w) || Gp(q.k_w) || Gp(q.v_w) || Gp(q.q_b) || Gp(q.k_b) || Gp(q.v_b)) {
          float* tmp = S.W_<float>(S.wl.gtmp);   // (3d, d) stacked weight gradient, then the (3d) biases
          if (S.wgrad_rm_ok(3 * d, d, S.kpad(3L * d), d)) {
            S.wgrad_rm(pa, S.kpad(3L * d), 3 * d, S.T_(t.hn[1]), d, d, 0, Drop{0, 0, 1.0f}, M, tmp, tmp + 3L * d * d);
          } else {
            S.pack(dqkv, false, 3L * d, M, 3 * d, true, 1.0f, pat, Mq, 3 * d, (int)Mq);
            S.pack(S.T_(t.hn[1]), true, d, M, d, true, 1.0f, pbt, Mq, S.npad(d + 4), (int)Mq, 0, Drop{0, 0, 1.0f}, d);
            S.wgrad(pat, pbt, Mq, 3 * d, d, M, tmp, tmp + 3L * d * d);
          }
          CopyList cl{};
          for (int p = 0; p < 3; ++p) {
            cl.src[2 * p] = tmp + (long)p * d * d;
            cl.dst[2 * p] = Gp(wi[p]);
            cl.n[2 * p] = (long)d * d;
            cl.src[2 * p + 1] = tmp + 3L * d * d + (long)p * d;
            cl.dst[2 * p + 1] = Gp(bi3[p]);
            cl.n[2 * p + 1] = d;
          }
          cl.count = 6;
          cfm_launch(copy_multi_kernel, dim3(ew_grid((long)d * d), 6), dim3(256), 0, st, cl);
        }
        ln_bwd(X[1], q.ln_w[LN_ATT], q.ln_b[LN_ATT], dhn, gB, true, true, 0.5f, S.drop(site(l, 1)));   // gB = d x1 (+ FFN1's operand)
      }
    }
    ffn_bwd(0, X[0], S.T_(t.hn[0]), t.z1, t.u1, gB, true, false, 1.0f, Drop{0, 0, 1.0f});   // gB = d x0
    ln_flush();
    std::swap(gA, gB);
    grad_ready(S, kPreEncodeRows + l * layer_rows, layer_rows);   // every gradient of layer l is enqueued
  }

  // ---- subsampling backward: gA = d(layer-0 input) ----
  const float xs = h->cfg.xscaling ? (float)std::sqrt((double)d) : 1.0f;
  cfm_launch(scale_drop_kernel, dim3(ew_grid(n_md)), dim3(256), 0, st, (const float*)gA, xs, n_md, S.drop(0), dbr);
  const int KS = g.F2 * g.C;
  float* dX2 = S.W_<float>(S.wl.dX2);
  S.pack(dbr, false, d, M, d, false, 1.0f, pa, S.kpad(d), M, S.kpad(d));
  S.perm(S.prm(S.i_sw), 1, wt, false, S.kpad(d), S.npad(KS), S.kpad(d));
  S.gemm_f32out(pa, S.kpad(d), M, d, wt, KS, nullptr, 1.0f, dX2, KS, false);
  if (Gp(S.i_sw) || Gp(S.i_sb)) {
    float* tmp = S.W_<float>(S.wl.gtmp);   // (d, KS) permuted gradient
    if (S.wgrad_rm_ok(d, KS, S.kpad(d), KS)) {
      S.wgrad_rm(pa, S.kpad(d), d, S.T_(S.tp.X2), KS, KS, 0, Drop{0, 0, 1.0f}, M, tmp, Gp(S.i_sb));
    } else {
      S.pack(dbr, false, d, M, d, true, 1.0f, pat, Mq, d, (int)Mq);
      S.pack(S.T_(S.tp.X2), true, KS, M, KS, true, 1.0f, pbt, Mq, S.npad(KS + 4), (int)Mq, 0, Drop{0, 0, 1.0f},
             KS);
      S.wgrad(pat, pbt, Mq, d, KS, M, tmp, Gp(S.i_sb));
    }
    if (Gp(S.i_sw)) S.perm(tmp, 4, Gp(S.i_sw), true, KS, d, KS);
  }
  // conv2 + ReLU: dY2 = dX2 * [X2 > 0], rows (b, t2, f2) x C
  const long n2 = g.M2 * g.C;
  if (dt == DT_F32)
    cfm_launch(relu_mask_kernel<float>, dim3(ew_grid(n2)), dim3(256), 0, st, dX2, S.T_<const float>(S.tp.X2), n2);
  else
    cfm_launch(relu_mask_kernel<bf16_t>, dim3(ew_grid(n2)), dim3(256), 0, st, dX2, S.T_<const bf16_t>(S.tp.X2), n2);
  const bool need_c1 = Gp(S.i_c1w) || Gp(S.i_c1b);
  // the frame-major compute-type dY2 (the TN weight gradient's A operand and the transposed conv's input)
  bool pa_dy2 = false;
  // CFM_TN_CONV=0: the im2col image + packed GEMM (A/B).  The bias as column sums of the fp32 dY2 instead of
  // the kernel's bf16 row sums measured slower (29.79-29.85 against 29.70-29.78 ms per step,
  // profiles/r05m_tn_conv_bias_ab.txt).
  static const bool tn_conv_on = [] { const char* e = getenv("CFM_TN_CONV"); return e ? atoi(e) != 0 : true; }();
  if ((Gp(S.i_c2w) || Gp(S.i_c2b)) && tn_conv_on && wgrad_tn_conv_supported(dt, g.C, S.kpad(g.C))) {
    // [dW2 | db2] = dY2^T . [im2col(X1) | 1] on the frame-major TN kernel with the im2col formed by its
    // loader: no transposed dY2, no 1.47 GB im2col image.  One row split per CU over the 256x256 tiles.
    S.pack(dX2, false, g.C, (int)g.M2, g.C, false, 1.0f, pa, S.kpad(g.C), (int)g.M2, S.kpad(g.C));
    pa_dy2 = true;
    const long K9 = 9L * g.C, Kb = K9 + 4;
    const long tiles = (long)((g.C + 255) / 256) * ((K9 + 255) / 256);
    long nsp = std::max<long>(1, std::min<long>(256 / tiles, wgrad_splits(g.C, (int)Kb, g.M2)));
    const long chunk = round_up((g.M2 + nsp - 1) / nsp, 32);
    nsp = (g.M2 + chunk - 1) / chunk;
    float* part = S.W_<float>(S.wl.part);
    float* tmp = S.W_<float>(S.wl.gtmp);   // (C, 9C) permuted gradient
    wgrad_tn_conv(pa, S.kpad(g.C), S.T_(S.tp.X1), g.B, g.T1, g.F1, g.T2, g.F2, g.C, Gp(S.i_c2b) != nullptr, g.M2,
                  (int)nsp, chunk, part, Kb, (long)g.C * Kb, st);
    slab_sum_wb(part, (int)nsp, g.C, (int)K9, tmp, Gp(S.i_c2b), st);
    if (Gp(S.i_c2w)) S.perm(tmp, 5, Gp(S.i_c2w), true, K9, g.C, (int)K9);
  } else if (Gp(S.i_c2w) || Gp(S.i_c2b)) {   // [dW2 | db2] = dY2^T . [im2col(X1) | 1]
    S.pack(dX2, false, g.C, (int)g.M2, g.C, true, 1.0f, pat, g.M2p, g.C, (int)g.M2p);
    const dim3 grid((unsigned)((g.M2p + 31) / 32), (unsigned)((S.npad(9L * g.C + 4) + 31) / 32));
    const dim3 grid64((unsigned)((g.M2p + 63) / 64), (unsigned)((S.npad(9L * g.C + 4) + 255) / 256));   // 4 row tiles / block
    const bool vec = g.C % 8 == 0 && g.M2p % 8 == 0;
    if (vec && dt == DT_F32)
      cfm_launch(im2col_t_vec_kernel<float>, grid64, dim3(256), 0, st, S.T_<const float>(S.tp.X1), g.T1, g.F1, g.T2,
                 g.F2, g.C, (int)g.M2, S.W_<float>(S.wl.i2c), g.M2p, S.npad(9L * g.C + 4));
    else if (vec)
      cfm_launch(im2col_t_vec_kernel<bf16_t>, grid64, dim3(256), 0, st, S.T_<const bf16_t>(S.tp.X1), g.T1, g.F1,
                 g.T2, g.F2, g.C, (int)g.M2, S.W_<bf16_t>(S.wl.i2c), g.M2p, S.npad(9L * g.C + 4));
    else if (dt == DT_F32)
      cfm_launch(im2col_t_kernel<float>, grid, dim3(256), 0, st, S.T_<const float>(S.tp.X1), g.T1, g.F1, g.T2, g.F2,
                 g.C, (int)g.M2, S.W_<float>(S.wl.i2c), g.M2p, S.npad(9L * g.C + 4));
    else
      cfm_launch(im2col_t_kernel<bf16_t>, grid, dim3(256), 0, st, S.T_<const bf16_t>(S.tp.X1), g.T1, g.F1, g.T2, g.F2,
                 g.C, (int)g.M2, S.W_<bf16_t>(S.wl.i2c), g.M2p, S.npad(9L * g.C + 4));
    float* tmp = S.W_<float>(S.wl.gtmp);   // (C, 9C) permuted gradient
    S.wgrad(pat, S.W_(S.wl.i2c), g.M2p, g.C, 9 * g.C, g.M2, tmp, Gp(S.i_c2b));
    if (Gp(S.i_c2w)) S.perm(tmp, 5, Gp(S.i_c2w), true, 9L * g.C, g.C, 9 * g.C);
  }
  static const bool tconv_on = [] { const char* e = getenv("CFM_TCONV"); return e ? atoi(e) != 0 : true; }();
  if (need_c1 && tconv_on && gemm_tconv_supported(dt, g.C)) {
    // dY1 = conv2's transposed conv as four stride-phase implicit GEMMs straight from dY2 (no dCol
    // image, no col2im): phase (pt, pf) of the input pixels gathers the (1+pt)(1+pf) taps reaching it.
    // The phase-major result (compute type) is masked by conv1's ReLU inside conv1's weight-gradient kernel.
    if (!pa_dy2) S.pack(dX2, false, g.C, (int)g.M2, g.C, false, 1.0f, pa, S.kpad(g.C), (int)g.M2, S.kpad(g.C));
    char* dy1 = (char*)S.W_<float>(S.wl.dy1);
    const PhaseRows pr(g.B, g.T1, g.F1);
    char* wp = (char*)wt;
    for (int ph = 0; ph < 4; ++ph) {
      const int pt = ph >> 1, pf = ph & 1, ntap = (1 + pt) * (1 + pf);
      const int Kp = S.kpad((long)ntap * g.C), rp = S.npad(g.C);
      const long n = (long)rp * Kp;
      if (dt == DT_F32)
        cfm_launch(tconv_wpack_kernel<float>, dim3(ew_grid(n)), dim3(256), 0, st, S.prm(S.i_c2w), g.C, pt, pf,
                   (float*)wp, Kp, rp);
      else
        cfm_launch(tconv_wpack_kernel<bf16_t>, dim3(ew_grid(n)), dim3(256), 0, st, S.prm(S.i_c2w), g.C, pt, pf,
                   (bf16_t*)wp, Kp, rp);
      GemmEpi e = S.epi(EPI_STORE, nullptr);
      e.C = dy1 + pr.base[ph] * g.C * es;
      e.ldc = g.C;
      const TConvGeom tg{pa, S.kpad(g.C), g.B, g.T2, g.F2, g.C, pt, pf, pr.nI[pt], pr.nJ[pf]};
      gemm_tconv(dt, tg, wp, Kp, g.C, e, h->zero_page, st);
      wp += n * es;
    }
    const int rows = g.B * g.T1, R = 8, nch = (rows + R - 1) / R;
    float* part = S.W_<float>(S.wl.c1part);
    float* part_b = part + (long)nch * 9 * g.C;
    const dim3 grid8(nch, (g.C / 8 + 63) / 64);
    if (g.C % 8 == 0 && dt == DT_F32)
      cfm_launch(conv1_wgrad_ph8_kernel<float>, grid8, dim3(64), 0, st, S.T_<const float>(S.tp.xin), g.F, g.T, g.T1,
                 g.F1, g.C, (const float*)dy1, S.T_<const float>(S.tp.X1), g.B, R, part, part_b);
    else if (g.C % 8 == 0)
      cfm_launch(conv1_wgrad_ph8_kernel<bf16_t>, grid8, dim3(64), 0, st, S.T_<const float>(S.tp.xin), g.F, g.T, g.T1,
                 g.F1, g.C, (const bf16_t*)dy1, S.T_<const bf16_t>(S.tp.X1), g.B, R, part, part_b);
    else if (dt == DT_F32)
      cfm_launch((conv1_wgrad_kernel<float, true>), dim3(nch, (g.C + 255) / 256), dim3(256), 0, st,
                 S.T_<const float>(S.tp.xin), g.F, g.T, g.T1, g.F1, g.C, (const float*)dy1,
                 S.T_<const float>(S.tp.X1), g.B, R, part, part_b);
    else
      cfm_launch((conv1_wgrad_kernel<bf16_t, true>), dim3(nch, (g.C + 255) / 256), dim3(256), 0, st,
                 S.T_<const float>(S.tp.xin), g.F, g.T, g.T1, g.F1, g.C, (const bf16_t*)dy1,
                 S.T_<const bf16_t>(S.tp.X1), g.B, R, part, part_b);
    if (Gp(S.i_c1w)) colred(part, nullptr, nullptr, 9L * g.C, nch, 9 * g.C, 0, 1.0f, Gp(S.i_c1w), 0, red, st);
    if (Gp(S.i_c1b)) colred(part_b, nullptr, nullptr, g.C, nch, g.C, 0, 1.0f, Gp(S.i_c1b), 0, red, st);
  } else if (need_c1) {   // dCol = dY2 . W2mat, col2im + conv1 ReLU mask, then conv1's weight/bias gradient
    S.pack(dX2, false, g.C, (int)g.M2, g.C, false, 1.0f, pa, S.kpad(g.C), (int)g.M2, S.kpad(g.C));
    S.perm(S.prm(S.i_c2w), 3, wt, false, S.kpad(g.C), S.npad(9L * g.C), S.kpad(g.C));
    GemmEpi e = S.epi(EPI_STORE, nullptr);
    e.C = S.W_(S.wl.dcol);
    e.ldc = 9L * g.C;
    gemm(dt, pa, S.kpad(g.C), (int)g.M2, g.C, wt, S.kpad(g.C), 9 * g.C, e, h->zero_page, st);
    const long n1 = (long)g.B * g.T1 * g.F1 * g.C;
    float* dy1 = S.W_<float>(S.wl.dy1);
    if (g.C % 8 == 0 && dt == DT_F32)
      cfm_launch(col2im_relu_vec_kernel<float>, dim3(ew_grid(n1 / 8)), dim3(256), 0, st, S.W_<const float>(S.wl.dcol),
                 S.T_<const float>(S.tp.X1), g.B, g.T1, g.F1, g.T2, g.F2, g.C, dy1);
    else if (g.C % 8 == 0)
      cfm_launch(col2im_relu_vec_kernel<bf16_t>, dim3(ew_grid(n1 / 8)), dim3(256), 0, st,
                 S.W_<const bf16_t>(S.wl.dcol), S.T_<const bf16_t>(S.tp.X1), g.B, g.T1, g.F1, g.T2, g.F2, g.C, dy1);
    else if (dt == DT_F32)
      cfm_launch(col2im_relu_kernel<float>, dim3(ew_grid(n1)), dim3(256), 0, st, S.W_<const float>(S.wl.dcol),
                 S.T_<const float>(S.tp.X1), g.B, g.T1, g.F1, g.T2, g.F2, g.C, dy1);
    else
      cfm_launch(col2im_relu_kernel<bf16_t>, dim3(ew_grid(n1)), dim3(256), 0, st, S.W_<const bf16_t>(S.wl.dcol),
                 S.T_<const bf16_t>(S.tp.X1), g.B, g.T1, g.F1, g.T2, g.F2, g.C, dy1);
    {
      const int rows = g.B * g.T1, R = 8, nch = (rows + R - 1) / R;
      float* part = S.W_<float>(S.wl.c1part);
      float* part_b = part + (long)nch * 9 * g.C;
      cfm_launch((conv1_wgrad_kernel<float, false>), dim3(nch, (g.C + 255) / 256), dim3(256), 0, st,
                 S.T_<const float>(S.tp.xin), g.F, g.T, g.T1, g.F1, g.C, (const float*)dy1, (const float*)nullptr,
                 g.B, R, part, part_b);
      if (Gp(S.i_c1w)) colred(part, nullptr, nullptr, 9L * g.C, nch, 9 * g.C, 0, 1.0f, Gp(S.i_c1w), 0, red, st);
      if (Gp(S.i_c1b)) colred(part_b, nullptr, nullptr, g.C, nch, g.C, 0, 1.0f, Gp(S.i_c1b), 0, red, st);
    }
  }
  grad_ready(S, 0, kPreEncodeRows);
}

}  // namespace

// =============================================================================================
// C-ABI
// =============================================================================================
extern "C" {

size_t cfm_train_tape_size(const cfm_encoder* h, int B, int T) {
  if (!h || B <= 0 || T <= 0) return 0;
  return (size_t)tape_layout(h, make_geo(h, B, T)).total;
}

size_t cfm_train_workspace_size(const cfm_encoder* h, int B, int T) {
  if (!h || B <= 0 || T <= 0) return 0;
  return (size_t)ws_layout(h, make_geo(h, B, T)).total;
}

static void make_step(Step& S, cfm_encoder* h, const float* const* params, int n_params, int B, int T,
                      const cfm_train_opts* opts, void* tape, size_t tape_bytes, void* ws, size_t ws_bytes,
                      void* stream) {
  check_common(h, params, n_params, B, T, opts);
  refuse_half_training(h->dtype == DT_F32, "cfm_train_forward / cfm_train_backward");
  S.h = h;
  S.g = make_geo(h, B, T);
  S.tp = tape_layout(h, S.g);
  S.wl = ws_layout(h, S.g);
  if (!tape || tape_bytes < (size_t)S.tp.total) fail(CFM_ERR_WORKSPACE, "tape too small");
  if (!ws || ws_bytes < (size_t)S.wl.total) fail(CFM_ERR_WORKSPACE, "workspace too small");
  S.tape = (char*)tape;
  S.ws = (char*)ws;
  S.st = (hipStream_t)stream;
  S.P = params;
  S.o = opts;
  build_index(S);
}

cfm_status cfm_train_forward(cfm_encoder* h, const float* const* params, int n_params, const float* x_bft,
                             const int32_t* len_b, int B, int T, const cfm_train_opts* opts, float* y_bdt,
                             int32_t* out_len_b, void* tape, size_t tape_bytes, void* ws, size_t ws_bytes,
                             void* stream) {
  return guarded([&] {
    if (!x_bft || !y_bdt || !out_len_b) fail(CFM_ERR_INVALID_ARG, "null argument");
    Step S;
    make_step(S, h, params, n_params, B, T, opts, tape, tape_bytes, ws, ws_bytes, stream);
    train_forward(S, x_bft, len_b, y_bdt, out_len_b);
    HIP_OK(hipGetLastError());
  });
}

cfm_status cfm_train_backward(cfm_encoder* h, const float* const* params, int n_params, const float* dy_bdt, int B,
                              int T, const cfm_train_opts* opts, float* const* grads, const void* tape,
                              size_t tape_bytes, void* ws, size_t ws_bytes, void* stream) {
  return guarded([&] {
    if (!dy_bdt) fail(CFM_ERR_INVALID_ARG, "null argument");
    Step S;
    make_step(S, h, params, n_params, B, T, opts, (void*)tape, tape_bytes, ws, ws_bytes, stream);
    train_backward(S, dy_bdt, grads);
    HIP_OK(hipGetLastError());
  });
}

}  // extern "C"
