// Backward of the relative-position multi-head attention (RelPositionMultiHeadAttention.forward,
// multi_head_attention.py:172-210 with forward_attention :94-115), SURVEY §8 row a16.
//
// Operands are the forward's own layouts (cfm_kernels.h): qk = [(q+u)c | (q+v)c | k] per row with
// c = log2(e)/sqrt(dk), V transposed per (b, h) in Vt, and p = linear_pos(pos_emb) per head.
// bf16 compute (T' <= 512, dk % 16 == 0): one fused launch (`attn_bwd_scores_kernel`) recomputes S,
// BD, the softmax and dP per 32 query rows in registers and writes only the bf16 images the
// remaining contractions read (P, dS and the skewed G: 128 MB at BASELINE config 3).  fp32 parity
// mode (and any other shape) materialises the fp32 score matrices per (b, h) and runs every
// contraction on one batched MFMA GEMM (`bgemm`, LDS-staged, any operand orientation):
//   S  = (q+u)c . k^T            BD = (q+v)c . p^T          (log2 units, as the forward)
//   P  = softmax_j(S[i][j] + BD[i][T'-1-i+j]) with the pad / context mask      (rel_shift :159-170)
//   dP = dctx . V^T,   dS = P * (dP - rowsum(P * dP))                          (natural-log units)
//   G[i][r] = dS[i][r - (T'-1-i)]   (rel_shift undone: the gradient on the raw BD matrix)
//   d(q+u) = dS . k / sqrt(dk)      dk = dS^T . (q+u)c * ln2      dv = P^T . dctx
//   d(q+v) = G . p / sqrt(dk)       dp = sum_b G^T . (q+v)c * ln2
//   dq = d(q+u) + d(q+v);  d pos_bias_u = sum_rows d(q+u);  d pos_bias_v = sum_rows d(q+v)
// Masked scores get zero gradient: the reference fills them with -10000 before the softmax and
// zeroes their probabilities after it (:106-107), so both paths into them carry no gradient.
#include <cmath>
#include <cstdlib>
#include <initializer_list>
#include <type_traits>

#include "../../include/cfm_train.h"
#include "cfm_abi.h"
#include "cfm_common.h"
#include "cfm_kernels.h"

namespace cfm {
namespace {

struct BgArgs {
  const void* A; long am, ak, az1, az2;   // A(m, k) at A + z1*az1 + z2*az2 + m*am + k*ak
  const void* B; long bk, bn, bz1, bz2;   // B(k, n)
  float* C; long cm, cn, cz1, cz2;        // C(m, n) fp32
  int M, N, K, Z2;                        // batch z = blockIdx.z = z1 * Z2 + z2
  float alpha; int accumulate;
  int Ktot;                               // split-K over z2: slice z2 covers K rows [z2*K, min((z2+1)*K, Ktot)) (0 = off)
};

// C = alpha * A.B (+ C).  64x64 output tile per 4-wave block (2x2 waves of 32x32 MFMA tiles), K in
// steps of 32 staged through LDS as [row][k] images in the compute type T, so either operand
// orientation is read coalesced from HBM (consecutive threads walk whichever stride is 1).  The
// next K-step's global loads are in flight while the current step's MFMAs run.
template <typename TA, typename TB, typename T>
__global__ __launch_bounds__(256) void bgemm_kernel(BgArgs a) {
  constexpr int RB = 32 * (int)sizeof(T) + 16;   // LDS row: 32 k values + 16 B pad
  __shared__ __attribute__((aligned(16))) char As[64 * RB];
  __shared__ __attribute__((aligned(16))) char Bs[64 * RB];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int z = blockIdx.z, z1 = z / a.Z2, z2 = z - z1 * a.Z2;
  const TA* A = (const TA*)a.A + z1 * a.az1 + z2 * a.az2;
  const TB* Bm = (const TB*)a.B + z1 * a.bz1 + z2 * a.bz2;
  const int m0 = blockIdx.y * 64, n0 = blockIdx.x * 64;
  const bool a_kc = a.ak == 1, b_kc = a.bk == 1;
  const int KZ = a.Ktot ? min(a.K, a.Ktot - z2 * a.K) : a.K;
  float ra[8], rb[8];
  auto coord = [&](bool kc, int e, int& r, int& k) {
    const int idx = e * 256 + tid;
    if (kc) { k = idx & 31; r = idx >> 5; } else { r = idx & 63; k = idx >> 6; }
  };
  auto load = [&](int k0) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      int r, k;
      coord(a_kc, e, r, k);
      const int gm = m0 + r, gk = k0 + k;
      ra[e] = (gm < a.M && gk < KZ) ? ld_f<TA>(A + gm * a.am + gk * a.ak) : 0.0f;
      coord(b_kc, e, r, k);
      const int gn = n0 + r, gk2 = k0 + k;
      rb[e] = (gn < a.N && gk2 < KZ) ? ld_f<TB>(Bm + gk2 * a.bk + gn * a.bn) : 0.0f;
    }
  };
  f32x16 acc = {};
  const int wm = w & 1, wn = w >> 1;
  const char* ap = As + (wm * 32 + (lane & 31)) * RB + 16 * (lane >> 5);
  const char* bp = Bs + (wn * 32 + (lane & 31)) * RB + 16 * (lane >> 5);
  load(0);
  for (int k0 = 0; k0 < KZ; k0 += 32) {
    __syncthreads();
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      int r, k;
      coord(a_kc, e, r, k);
      st_f<T>((T*)(As + r * RB) + k, ra[e]);
      coord(b_kc, e, r, k);
      st_f<T>((T*)(Bs + r * RB) + k, rb[e]);
    }
    __syncthreads();
    if (k0 + 32 < KZ) load(k0 + 32);
#pragma unroll
    for (int s = 0; s < (int)sizeof(T); ++s)
      mfma_slab<T>(acc, *(const uint4*)(ap + 32 * s), *(const uint4*)(bp + 32 * s));
  }
  float* C = a.C + z1 * a.cz1 + z2 * a.cz2;
  const int n = n0 + wn * 32 + (lane & 31);
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int m = m0 + wm * 32 + acc_row(r, lane);
    if (m < a.M && n < a.N) {
      float* c = C + m * a.cm + n * a.cn;
      const float v = a.alpha * acc[r];
      *c = a.accumulate ? *c + v : v;
    }
  }
}

// v2: same contract, K-steps of 64 through a double-buffered LDS image (one barrier per step) and
// 4-element vector global loads along whichever operand stride is 1.  Requires every stride and
// base offset to be a multiple of 4 elements (checked on the host; v1 otherwise).
template <typename TS> struct Quad;
template <> struct Quad<float> {
  static CFM_DEV void ld(const float* p, float* v) { const float4 q = *(const float4*)p; v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w; }
};
template <> struct Quad<bf16_t> {
  static CFM_DEV void ld(const bf16_t* p, float* v) {
    const uint2 q = *(const uint2*)p;
    v[0] = bf2f((bf16_t)(q.x & 0xffffu)); v[1] = bf2f((bf16_t)(q.x >> 16));
    v[2] = bf2f((bf16_t)(q.y & 0xffffu)); v[3] = bf2f((bf16_t)(q.y >> 16));
  }
};

template <typename TA, typename TB, typename T>
__global__ __launch_bounds__(256) void bgemm2_kernel(BgArgs a) {
  constexpr int KS = 64;
  constexpr int RB = KS * (int)sizeof(T) + 16;
  __shared__ __attribute__((aligned(16))) char As[2][64 * RB];
  __shared__ __attribute__((aligned(16))) char Bs[2][64 * RB];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int z = blockIdx.z, z1 = z / a.Z2, z2 = z - z1 * a.Z2;
  const TA* A = (const TA*)a.A + z1 * a.az1 + z2 * a.az2;
  const TB* Bm = (const TB*)a.B + z1 * a.bz1 + z2 * a.bz2;
  const int m0 = blockIdx.y * 64, n0 = blockIdx.x * 64;
  const bool a_kc = a.ak == 1, b_kc = a.bk == 1;
  const int KZ = a.Ktot ? min(a.K, a.Ktot - z2 * a.K) : a.K;
  float ra[16], rb[16];
  // Each thread moves four runs of 4 consecutive k values per operand and K-step, and writes each
  // run to LDS as one 4-element vector.  k-contiguous operand: run q is row idx >> 4, k = 4 (idx & 15)
  // (idx = 256 q + tid).  Otherwise the thread loads a 4x4 micro-block -- 4 k rows of 4 consecutive
  // operand rows r = 4 (tid & 15) .. +3 at k = 4 (tid >> 4) .. +3 -- and transposes it in registers:
  // v[4 kk + e] holds (r + e, k + kk).
  // Interior threads (every run in range) issue their four vector loads in one branch-free block;
  // only threads on a tile edge take the element-wise path (a per-load condition would make hipcc
  // wait for each load before the next, cdna_hip_programming.md §5).
  auto loadop = [&](auto* P, long sr, long sk, bool kc, int r0, int R, int k0, float* v) {
    using TS = typename std::remove_cv<typename std::remove_pointer<decltype(P)>::type>::type;
    const bool full = kc ? (r0 + ((3 * 256 + tid) >> 4) < R && k0 + 4 * (tid & 15) + 3 < KZ)
                         : (k0 + 4 * (tid >> 4) + 3 < KZ && r0 + 4 * (tid & 15) + 3 < R);
    if (full) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (kc) {
          const int idx = q * 256 + tid;
          Quad<TS>::ld(P + (r0 + (idx >> 4)) * sr + k0 + 4 * (idx & 15), v + 4 * q);
        } else {
          Quad<TS>::ld(P + r0 + 4 * (tid & 15) + (k0 + 4 * (tid >> 4) + q) * sk, v + 4 * q);
        }
      }
      return;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float* o = v + 4 * q;
      if (kc) {
        const int idx = q * 256 + tid;
        const int r = r0 + (idx >> 4), k = k0 + 4 * (idx & 15);
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = (r < R && k + e < KZ) ? ld_f(P + r * sr + (k + e)) : 0.0f;
      } else {
        const int r = r0 + 4 * (tid & 15), k = k0 + 4 * (tid >> 4) + q;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = (r + e < R && k < KZ) ? ld_f(P + (r + e) + k * sk) : 0.0f;
      }
    }
  };
  auto put4 = [&](char* p, float x0, float x1, float x2, float x3) {
    if constexpr (sizeof(T) == 2) {
      *(uint2*)p = make_uint2((uint32_t)f2bf(x0) | ((uint32_t)f2bf(x1) << 16), (uint32_t)f2bf(x2) | ((uint32_t)f2bf(x3) << 16));
    } else {
      *(float4*)p = make_float4(x0, x1, x2, x3);
    }
  };
  auto store = [&](char* S, bool kc, const float* v) {
    if (kc) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int idx = q * 256 + tid;
        put4(S + (idx >> 4) * RB + 4 * (idx & 15) * (int)sizeof(T), v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
      }
    } else {
      const int r = 4 * (tid & 15), k = 4 * (tid >> 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) put4(S + (r + e) * RB + k * (int)sizeof(T), v[e], v[4 + e], v[8 + e], v[12 + e]);
    }
  };
  f32x16 acc = {};
  const int wm = w & 1, wn = w >> 1;
  const int aoff = (wm * 32 + (lane & 31)) * RB + 16 * (lane >> 5);
  const int boff = (wn * 32 + (lane & 31)) * RB + 16 * (lane >> 5);
  // both operands already in the 16-bit compute type: they move as raw 16-bit values (no fp32 round
  // trip); a row-major (non k-contiguous) operand's 4x4 micro-block is transposed with v_perm_b32
  constexpr bool RAW = sizeof(T) == 2 && std::is_same<TA, T>::value && std::is_same<TB, T>::value;
  if constexpr (RAW) {
    auto loadraw = [&](const bf16_t* P, long sr, long sk, bool kc, int r0, int R, int k0, uint2* v) {
      const bool full = kc ? (r0 + ((3 * 256 + tid) >> 4) < R && k0 + 4 * (tid & 15) + 3 < KZ)
                           : (k0 + 4 * (tid >> 4) + 3 < KZ && r0 + 4 * (tid & 15) + 3 < R);
      if (full) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if (kc) {
            const int idx = q * 256 + tid;
            v[q] = *(const uint2*)(P + (r0 + (idx >> 4)) * sr + k0 + 4 * (idx & 15));
          } else {
            v[q] = *(const uint2*)(P + r0 + 4 * (tid & 15) + (k0 + 4 * (tid >> 4) + q) * sk);
          }
        }
        return;
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        uint32_t e16[4];
        if (kc) {
          const int idx = q * 256 + tid;
          const int r = r0 + (idx >> 4), k = k0 + 4 * (idx & 15);
#pragma unroll
          for (int e = 0; e < 4; ++e) e16[e] = (r < R && k + e < KZ) ? (uint32_t)P[r * sr + (k + e)] : 0u;
        } else {
          const int r = r0 + 4 * (tid & 15), k = k0 + 4 * (tid >> 4) + q;
#pragma unroll
          for (int e = 0; e < 4; ++e) e16[e] = (r + e < R && k < KZ) ? (uint32_t)P[(r + e) + k * sk] : 0u;
        }
        v[q] = make_uint2(e16[0] | (e16[1] << 16), e16[2] | (e16[3] << 16));
      }
    };
    auto storeraw = [&](char* S, bool kc, const uint2* v) {
      if (kc) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int idx = q * 256 + tid;
          *(uint2*)(S + (idx >> 4) * RB + 8 * (idx & 15)) = v[q];
        }
      } else {
        // v[q] = rows r .. r+3 at k + q; row r + e wants (k, k+1 | k+2, k+3) = element e of v[0..3]
        const int r = 4 * (tid & 15), k = 4 * (tid >> 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const uint32_t sel = (e & 1) ? 0x07060302u : 0x05040100u;
          const uint32_t lo0 = (e < 2) ? v[0].x : v[0].y, lo1 = (e < 2) ? v[1].x : v[1].y;
          const uint32_t hi0 = (e < 2) ? v[2].x : v[2].y, hi1 = (e < 2) ? v[3].x : v[3].y;
          *(uint2*)(S + (r + e) * RB + 2 * k) =
              make_uint2(__builtin_amdgcn_perm(lo1, lo0, sel), __builtin_amdgcn_perm(hi1, hi0, sel));
        }
      }
    };
    uint2 qa[4], qb[4];
    loadraw((const bf16_t*)A, a.am, a.ak, a_kc, m0, a.M, 0, qa);
    loadraw((const bf16_t*)Bm, a.bn, a.bk, b_kc, n0, a.N, 0, qb);
    storeraw(As[0], a_kc, qa);
    storeraw(Bs[0], b_kc, qb);
    __syncthreads();
    int buf = 0;
    for (int k0 = 0; k0 < KZ; k0 += KS) {
      const bool more = k0 + KS < KZ;
      if (more) {
        loadraw((const bf16_t*)A, a.am, a.ak, a_kc, m0, a.M, k0 + KS, qa);
        loadraw((const bf16_t*)Bm, a.bn, a.bk, b_kc, n0, a.N, k0 + KS, qb);
      }
#pragma unroll
      for (int s = 0; s < KS * 2 / 32; ++s)
        mfma_slab<T>(acc, *(const uint4*)(As[buf] + aoff + 32 * s), *(const uint4*)(Bs[buf] + boff + 32 * s));
      if (more) {
        storeraw(As[buf ^ 1], a_kc, qa);
        storeraw(Bs[buf ^ 1], b_kc, qb);
      }
      __syncthreads();
      buf ^= 1;
    }
  } else {
  loadop(A, a.am, a.ak, a_kc, m0, a.M, 0, ra);
  loadop(Bm, a.bn, a.bk, b_kc, n0, a.N, 0, rb);
  store(As[0], a_kc, ra);
  store(Bs[0], b_kc, rb);
  __syncthreads();
  int buf = 0;
  for (int k0 = 0; k0 < KZ; k0 += KS) {
    const bool more = k0 + KS < KZ;
    if (more) {
      loadop(A, a.am, a.ak, a_kc, m0, a.M, k0 + KS, ra);
      loadop(Bm, a.bn, a.bk, b_kc, n0, a.N, k0 + KS, rb);
    }
#pragma unroll
    for (int s = 0; s < KS * (int)sizeof(T) / 32; ++s)
      mfma_slab<T>(acc, *(const uint4*)(As[buf] + aoff + 32 * s), *(const uint4*)(Bs[buf] + boff + 32 * s));
    if (more) {
      store(As[buf ^ 1], a_kc, ra);
      store(Bs[buf ^ 1], b_kc, rb);
    }
    __syncthreads();
    buf ^= 1;
  }
  }
  float* C = a.C + z1 * a.cz1 + z2 * a.cz2;
  const int n = n0 + wn * 32 + (lane & 31);
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int m = m0 + wm * 32 + acc_row(r, lane);
    if (m < a.M && n < a.N) {
      float* c = C + m * a.cm + n * a.cn;
      const float v = a.alpha * acc[r];
      *c = a.accumulate ? *c + v : v;
    }
  }
}

enum { OP_F32 = 0, OP_CT = 1 };   // operand storage: fp32, or the compute type

bool quad_ok(const void* p, int es, std::initializer_list<long> strides) {
  if (((uintptr_t)p) % (4 * es)) return false;
  for (long s : strides)
    if (s != 1 && s % 4) return false;
  return true;
}

template <typename T>
void bgemm_t(const BgArgs& a, int ta, int tb, int Z, hipStream_t st) {
  const dim3 grid((a.N + 63) / 64, (a.M + 63) / 64, Z), block(256);
  const int esa = ta == OP_F32 ? 4 : (int)sizeof(T), esb = tb == OP_F32 ? 4 : (int)sizeof(T);
  const bool v2 = (a.ak == 1 || a.am == 1) && (a.bk == 1 || a.bn == 1) &&
                  quad_ok(a.A, esa, {a.am, a.ak, a.az1, a.az2}) && quad_ok(a.B, esb, {a.bk, a.bn, a.bz1, a.bz2});
  if (v2) {
    if (ta == OP_F32 && tb == OP_F32) cfm_launch((bgemm2_kernel<float, float, T>), grid, block, 0, st, a);
    else if (ta == OP_F32) cfm_launch((bgemm2_kernel<float, T, T>), grid, block, 0, st, a);
    else if (tb == OP_F32) cfm_launch((bgemm2_kernel<T, float, T>), grid, block, 0, st, a);
    else cfm_launch((bgemm2_kernel<T, T, T>), grid, block, 0, st, a);
    return;
  }
  if (ta == OP_F32 && tb == OP_F32) cfm_launch((bgemm_kernel<float, float, T>), grid, block, 0, st, a);
  else if (ta == OP_F32) cfm_launch((bgemm_kernel<float, T, T>), grid, block, 0, st, a);
  else if (tb == OP_F32) cfm_launch((bgemm_kernel<T, float, T>), grid, block, 0, st, a);
  else cfm_launch((bgemm_kernel<T, T, T>), grid, block, 0, st, a);
}

void bgemm(int dt, const BgArgs& a, int ta, int tb, int Z, hipStream_t st) {
  if (a.M <= 0 || a.N <= 0 || Z <= 0) return;
  if (dt == DT_F32) bgemm_t<float>(a, ta, tb, Z, st);
  else bgemm_t<bf16_t>(a, ta, tb, Z, st);
}

CFM_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

CFM_DEV bool key_valid(int i, int j, int len, int cl, int cr) {
  return i < len && j < len && (cl < 0 || j >= i - cl) && (cr < 0 || j <= i + cr);
}

// One wave per score row (b, h, i): S[i][j] + BD[i][T'-1-i+j] (log2 units) -> P in place.
__global__ __launch_bounds__(256) void attn_probs_kernel(float* __restrict__ S, long sld, const float* __restrict__ BD,
                                                         long bdld, const int32_t* __restrict__ lens, int B, int H,
                                                         int Tp, int cl, int cr) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= (long)B * H * Tp) return;
  const int i = (int)(row % Tp);
  const int b = (int)(row / ((long)H * Tp));
  const int len = lens ? min(lens[b], Tp) : Tp;
  float* s = S + row * sld;
  const float* bd = BD + row * bdld + (Tp - 1 - i);
  float m = -INFINITY;
  for (int j = lane; j < Tp; j += 64) {
    if (!key_valid(i, j, len, cl, cr)) continue;
    const float v = s[j] + bd[j];
    s[j] = v;
    m = fmaxf(m, v);
  }
  m = wave_max(m);
  float sum = 0.0f;
  for (int j = lane; j < Tp; j += 64) {
    if (!key_valid(i, j, len, cl, cr)) continue;
    const float e = exp2f(s[j] - m);
    s[j] = e;
    sum += e;
  }
  sum = wave_sum(sum);
  const float inv = sum > 0.0f ? 1.0f / sum : 0.0f;
  for (int j = lane; j < Tp; j += 64) s[j] = key_valid(i, j, len, cl, cr) ? s[j] * inv : 0.0f;
}

// One wave per row: dS = P * (dP - sum_j P dP) into dP; the skewed copy G (layout [h][b][i][r],
// all r < gld written) gets dS at r = T'-1-i+j and zero elsewhere.
// With attention dropout (adrop.thr != 0) dP here is the gradient of the DROPPED probabilities:
// dP <- dP * mask / (1 - p) first, and P <- P * mask / (1 - p) at the end (the dv GEMM's operand).
__global__ __launch_bounds__(256) void attn_dscore_kernel(float* __restrict__ P, float* __restrict__ dP,
                                                          long sld, float* __restrict__ G, long gld, int B, int H,
                                                          int Tp, Drop adrop) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= (long)B * H * Tp) return;
  const int i = (int)(row % Tp);
  const long bh = row / Tp;
  const int h = (int)(bh % H), b = (int)(bh / H);
  float* p = P + row * sld;
  float* dp = dP + row * sld;
  if (adrop.thr)
    for (int j = lane; j < Tp; j += 64) dp[j] *= drop_mul(adrop, (uint64_t)row * Tp + j);
  float D = 0.0f;
  for (int j = lane; j < Tp; j += 64) D += p[j] * dp[j];
  D = wave_sum(D);
  float* g = G + (((long)h * B + b) * Tp + i) * gld;
  const int sh = Tp - 1 - i;
  for (int r = lane; r < gld; r += 64) {
    const int j = r - sh;
    g[r] = (j >= 0 && j < Tp) ? p[j] * (dp[j] - D) : 0.0f;
  }
  for (int j = lane; j < Tp; j += 64) dp[j] = p[j] * (dp[j] - D);
  if (adrop.thr)
    for (int j = lane; j < Tp; j += 64) p[j] *= drop_mul(adrop, (uint64_t)row * Tp + j);
}

// Row reduction over one block's 32 query rows for values held in 32x32 accumulator layout
// (v[e] belongs to row acc_row(e, lane)): the 32 lanes of a half-wave, then the waves through LDS
// in a fixed order.  Every lane returns the block-wide value of its 16 rows.
template <int CTRL> CFM_DEV float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
// reduction over the 32 lanes of a half-wave, the same value in every lane: DPP quad permutes and row
// mirrors (VALU, in-row sources only) for 16 lanes, one xor-16 shuffle (pairwise commutative steps, so every
// lane computes the same bits)
template <bool MAX>
CFM_DEV float halfwave_red(float v) {
  auto op = [](float a, float b) { return MAX ? fmaxf(a, b) : a + b; };
  v = op(v, dpp_f<0xB1>(v));    // quad_perm [1,0,3,2]
  v = op(v, dpp_f<0x4E>(v));    // quad_perm [2,3,0,1]
  v = op(v, dpp_f<0x141>(v));   // row_half_mirror
  v = op(v, dpp_f<0x140>(v));   // row_mirror
  return op(v, __shfl_xor(v, 16, 32));
}
template <bool MAX>
CFM_DEV void block_rows(float (&v)[16], float* red, float* fin, int w, int nw, int lane) {
#pragma unroll
  for (int e = 0; e < 16; ++e) v[e] = halfwave_red<MAX>(v[e]);
  if ((lane & 31) == 0) {
#pragma unroll
    for (int e = 0; e < 16; ++e) red[w * 32 + acc_row(e, lane)] = v[e];
  }
  __syncthreads();
  if (threadIdx.x < 32) {
    float a = red[threadIdx.x];
    for (int ww = 1; ww < nw; ++ww) a = MAX ? fmaxf(a, red[ww * 32 + threadIdx.x]) : a + red[ww * 32 + threadIdx.x];
    fin[threadIdx.x] = a;
  }
  __syncthreads();
#pragma unroll
  for (int e = 0; e < 16; ++e) v[e] = fin[acc_row(e, lane)];
}

// Fused producer of the bf16 attention backward (T' <= 512, dk % 16 == 0): the S and BD GEMMs,
// rel_shift + mask + softmax, the dP GEMM and dS = P (dP - rowsum(P dP)) for 32 query rows of one
// (b, h) per block, never materialising the fp32 score images.  Wave w owns keys [64w, 64w + 64)
// as two 32x32 MFMA tiles held in registers; its BD window (32 rows x 96 positions) goes through a
// wave-private LDS image that is read skewed (bd[i][j] = BD[i][T'-1-i+j], as the forward kernel).
// MFMA operands are 16-byte fragment loads straight from the (L2-resident) qk / pos rows; V
// fragments are gathered from the V^T image.  Writes P and dS ([b][h][i][j], row pitch sld) and the
// skewed G ([h][b][i][r], all r < gld written) in bf16, the operand type of the consumer GEMMs.
template <int NS>
__global__ __launch_bounds__(512) void attn_bwd_scores_kernel(
    const bf16_t* __restrict__ qk, long ldqk, const bf16_t* __restrict__ Vt, int vt_rows, int Tpad,
    const bf16_t* __restrict__ pos, long ldp, const float* __restrict__ dctx, long ld_dctx,
    const int32_t* __restrict__ lens, int B, int Tp, int H, int dkp, int cl, int cr, bf16_t* __restrict__ Pg,
    bf16_t* __restrict__ dSg, long sld, bf16_t* __restrict__ G, long gld, Drop adrop) {
  constexpr int BDP = 97;                       // row pitch (floats) of a wave's BD image
  extern __shared__ float bd_all[];             // [nw][32][BDP]
  __shared__ float red[8 * 32], fin[32];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int nq = (Tp + 31) / 32;
  int blk = blockIdx.x;
  const int nb = gridDim.x;
  if ((nb & 7) == 0) blk = (blk & 7) * (nb >> 3) + (blk >> 3);   // the query tiles of one (b, h) share an XCD
  const int bh = blk / nq, i0 = (blk - bh * nq) * 32, b = bh / H, h = bh - b * H;
  const int len = lens ? min(lens[b], Tp) : Tp;
  const int l32 = lane & 31, kh = 8 * (lane >> 5);
  const long rowq = (long)b * Tp + min(i0 + l32, Tp - 1);
  uint4 aqu[NS], aqv[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    aqu[s] = *(const uint4*)(qk + rowq * ldqk + h * dkp + 16 * s + kh);
    aqv[s] = *(const uint4*)(qk + rowq * ldqk + (long)H * dkp + h * dkp + 16 * s + kh);
  }
  f32x16 sc[2];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int j = min(64 * w + 32 * c + l32, Tp - 1);
    const bf16_t* kp = qk + ((long)b * Tp + j) * ldqk + 2L * H * dkp + h * dkp + kh;
    sc[c] = f32x16{};
#pragma unroll
    for (int s = 0; s < NS; ++s) mfma_slab<bf16_t>(sc[c], aqu[s], *(const uint4*)(kp + 16 * s));
  }
  // dctx fragments (fp32 -> bf16) and the dP tiles are independent of the softmax: issue them first
  uint4 adc[NS];
  {
    const float* dr = dctx + rowq * ld_dctx + h * dkp + kh;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const float4 x0 = *(const float4*)(dr + 16 * s), x1 = *(const float4*)(dr + 16 * s + 4);
      const float f[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
      adc[s] = Vec16<bf16_t>::from_f32(f);
    }
  }
  // V rows of the block's keys [0, 64 nw) into LDS (row pitch dkp + 8 elements; zeros past Tpad),
  // transposed from the V^T image: a job reads 8 keys of channels 2q and 2q + 1 (two 16-byte loads)
  // and writes 8 dwords (one channel pair of one key each); consecutive lanes take consecutive
  // channel pairs, so each ds_write_b32 covers consecutive dwords of one key row.  The dP fragments
  // are then one 16-byte LDS read per slab instead of eight 2-byte global gathers.  The image lives
  // in the (not yet written) BD space.
  const int vpitch = dkp + 8;
  bf16_t* Vs = (bf16_t*)bd_all;
  {
    const int npair = dkp / 2, nkc = 8 * nw;   // channel pairs, 8-key chunks of the 64 nw keys
    const bf16_t* vt = Vt + (long)bh * vt_rows * Tpad;
    for (int job = threadIdx.x; job < npair * nkc; job += blockDim.x) {
      const int q = job % npair, k0 = 8 * (job / npair);
      uint4 a = make_uint4(0, 0, 0, 0), c = make_uint4(0, 0, 0, 0);
      if (k0 + 8 <= Tpad) {
        a = *(const uint4*)(vt + (long)(2 * q) * Tpad + k0);
        c = *(const uint4*)(vt + (long)(2 * q + 1) * Tpad + k0);
      }
      const uint32_t wa[4] = {a.x, a.y, a.z, a.w}, wc[4] = {c.x, c.y, c.z, c.w};
      uint32_t* dst = (uint32_t*)(Vs + (long)k0 * vpitch) + q;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        dst[(2 * e) * (vpitch / 2)] = (wa[e] & 0xffffu) | (wc[e] << 16);
        dst[(2 * e + 1) * (vpitch / 2)] = (wa[e] >> 16) | (wc[e] & 0xffff0000u);
      }
    }
  }
  __syncthreads();
  f32x16 dp[2];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const bf16_t* vr = Vs + (long)(64 * w + 32 * c + l32) * vpitch + kh;
    dp[c] = f32x16{};
#pragma unroll
    for (int s = 0; s < NS; ++s) mfma_slab<bf16_t>(dp[c], adc[s], *(const uint4*)(vr + 16 * s));
  }
  __syncthreads();   // every wave has read its V fragments: the BD images may overwrite them
  // BD for positions rbase .. rbase + 95 (every position a row of this wave's keys can touch)
  float* bw = bd_all + w * 32 * BDP;
  const int rbase = Tp - 1 - (i0 + 31) + 64 * w;
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    const int r = min(max(rbase + 32 * t + l32, 0), 2 * Tp - 2);
    const bf16_t* pp = pos + (long)r * ldp + h * dkp + kh;
    f32x16 a = {};
#pragma unroll
    for (int s = 0; s < NS; ++s) mfma_slab<bf16_t>(a, aqv[s], *(const uint4*)(pp + 16 * s));
#pragma unroll
    for (int e = 0; e < 16; ++e) bw[acc_row(e, lane) * BDP + 32 * t + l32] = a[e];
  }
  __syncthreads();
  // logits (log2 units) with the rel_shift, pad and context-window mask
  float m[16];
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int row = acc_row(e, lane), i = i0 + row;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int j = 64 * w + 32 * c + l32;
      const float v = sc[c][e] + bw[row * BDP + 31 - row + 32 * c + l32];
      const bool ok = key_valid(i, j, len, cl, cr);
      sc[c][e] = ok ? v : -INFINITY;
      if (!ok) dp[c][e] = 0.0f;   // V^T columns past T' may hold anything: keep them out of rowsum(P dP)
    }
    m[e] = fmaxf(sc[0][e], sc[1][e]);
  }
  block_rows<true>(m, red, fin, w, nw, lane);
  float sum[16];
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    sum[e] = 0.0f;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const float p = sc[c][e] == -INFINITY ? 0.0f : exp2f(sc[c][e] - m[e]);
      sc[c][e] = p;
      sum[e] += p;
    }
  }
  block_rows<false>(sum, red, fin, w, nw, lane);
  // attention dropout: dp is the gradient of the dropped probabilities -> chain through the mask (kept
  // as one bit per element for the P staging below: one hash per element)
  uint32_t keep = 0;
  if (adrop.thr) {
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const uint64_t rb = ((uint64_t)bh * Tp + (uint64_t)min(i0 + acc_row(e, lane), Tp - 1)) * (uint64_t)Tp;
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const float m = drop_mul(adrop, rb + (uint64_t)(64 * w + 32 * c + l32));
        dp[c][e] *= m;
        keep |= (m != 0.0f ? 1u : 0u) << (16 * c + e);
      }
    }
  }
  float D[16];
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const float inv = sum[e] > 0.0f ? 1.0f / sum[e] : 0.0f;
    D[e] = 0.0f;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      sc[c][e] *= inv;
      D[e] += sc[c][e] * dp[c][e];
    }
  }
  block_rows<false>(D, red, fin, w, nw, lane);
  // Stage the block's P and dS rows (bf16) in LDS -- the BD images are dead: every wave read its own
  // before the first row reduction's barrier -- then write whole rows as 8-byte runs: P and dS rows
  // (the [T', sld) tail as zeros) and the skewed G rows, zeros included.
  const int SP = 64 * nw;
  bf16_t* Ps = (bf16_t*)bd_all;
  bf16_t* dSs = Ps + 32 * SP;
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int row = acc_row(e, lane);
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int j = 64 * w + 32 * c + l32;
      // P goes to the dv GEMM: the dropped probabilities (the forward's P.V operand)
      const float pm = ((keep >> (16 * c + e)) & 1u) ? sc[c][e] * adrop.scale : 0.0f;
      Ps[row * SP + j] = f2bf(adrop.thr ? pm : sc[c][e]);
      dSs[row * SP + j] = f2bf(sc[c][e] * (dp[c][e] - D[e]));
    }
  }
  __syncthreads();
  const long img = (long)bh * Tp * sld;
  bf16_t* Gb = G + ((long)h * B + b) * Tp * gld;
  // 16-byte runs (sld, gld and the LDS row pitch are multiples of 8 elements)
  const int cps = (int)(sld / 8), cpg = (int)(gld / 8);
  for (int il = w; il < 32 && i0 + il < Tp; il += nw) {
    const int i = i0 + il, sh = Tp - 1 - i;
    const bf16_t* pr = Ps + il * SP;
    const bf16_t* dr = dSs + il * SP;
    for (int c = lane; c < cps; c += 64) {
      *(uint4*)(Pg + img + (long)i * sld + 8 * c) = *(const uint4*)(pr + 8 * c);
      *(uint4*)(dSg + img + (long)i * sld + 8 * c) = *(const uint4*)(dr + 8 * c);
    }
    for (int c = lane; c < cpg; c += 64) {
      uint32_t v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int j = 8 * c + e - sh;
        v[e] = (j >= 0 && j < Tp) ? (uint32_t)dr[j] : 0u;
      }
      *(uint4*)(Gb + (long)i * gld + 8 * c) =
          make_uint4(v[0] | (v[1] << 16), v[2] | (v[3] << 16), v[4] | (v[5] << 16), v[6] | (v[7] << 16));
    }
  }
}

bool attn_bwd_fused_enabled() {
  static const int on = [] { const char* e = getenv("CFM_ATTN_BWD_FUSED"); return e ? atoi(e) : 1; }();
  return on != 0;
}

// dst[r][c] = sum_s part[s][r][c] (fixed order), part rows of `cols` floats
__global__ void slab_rows_kernel(const float* __restrict__ part, int S, long rows, int cols, float* __restrict__ dst,
                                 long ldd) {
  const long n = rows * cols;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    float a = part[e];
    for (int s = 1; s < S; ++s) a += part[(long)s * n + e];
    const long r = e / cols;
    dst[r * ldd + (e - r * cols)] = a;
  }
}

__global__ void add_rows_kernel(float* __restrict__ dst, long ldd, const float* __restrict__ src, long lds, long rows,
                                int cols) {
  const long n = rows * cols;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    const long r = e / cols;
    const int c = (int)(e - r * cols);
    dst[r * ldd + c] += src[r * lds + c];
  }
}

struct BwdGeom {
  long sld, gld, s_bytes, g_bytes, t_bytes, cs_bytes, p_bytes;
  static constexpr int kPosSplit = 16;    // split-K of the position-gradient GEMM (K = B*T')
  BwdGeom(int B, int Tp, int H, int dk) {
    sld = round_up(Tp, 8);            // multiples of 8 elements: 16-byte rows for the TN products
    gld = round_up(2L * Tp - 1, 8);
    const long BH = (long)B * H;
    s_bytes = round_up(BH * Tp * sld * 4, 256);
    g_bytes = round_up(BH * Tp * gld * 4, 256);
    t_bytes = round_up((long)B * Tp * H * dk * 4, 256);
    cs_bytes = round_up((long)col_sums_ws(B * Tp, H * dk), 256);
    p_bytes = round_up((long)kPosSplit * (2L * Tp - 1) * H * dk * 4, 256);
  }
  size_t total() const { return (size_t)(2 * s_bytes + g_bytes + t_bytes + cs_bytes + p_bytes); }
};

}  // namespace

// wgrad_tn.hip: batched C = alpha * A^T . B on row-major bf16 operands (false: operands unsuitable)
bool bgemm_tn(const void* A, long lda, long az1, long az2, const void* B, long ldb, long bz1, long bz2, float* C,
              long ldc, long cz1, long cz2, int M, int N, int K, int Z, int Z2, int Ktot, float alpha, hipStream_t st);

size_t rel_pos_attention_backward_ws(int B, int Tp, int H, int dk) { return BwdGeom(B, Tp, H, dk).total(); }

void rel_pos_attention_backward(int dt, const void* qk, long ldqk, const void* Vt, int vt_rows, int Tpad,
                                const void* P, long ldp, const int32_t* lens, int B, int Tp, int H, int dk, int dkp,
                                int ctx_left, int ctx_right, const float* dctx, long ld_dctx, float* dq, float* dk_,
                                float* dv, long ld_dqkv, float* dpos, long ld_dpos, float* du, float* dvb, char* ws,
                                hipStream_t st, Drop adrop) {
  if (B <= 0 || Tp <= 0) return;
  const BwdGeom g(B, Tp, H, dk);
  float* S = (float*)ws;                          // scores -> P
  float* dP = (float*)(ws + g.s_bytes);           // dP -> dS
  float* BD = (float*)(ws + 2 * g.s_bytes);       // raw BD -> G
  float* tmp = (float*)(ws + 2 * g.s_bytes + g.g_bytes);
  float* cs = (float*)(ws + 2 * g.s_bytes + g.g_bytes + g.t_bytes);
  const int es = dtype_size(dt);
  const char* qkc = (const char*)qk;
  const long BT = (long)B * Tp;
  const float rs = (float)(1.0 / std::sqrt((double)dk));
  const float ln2 = 0.69314718055994531f;
  const long szs = (long)Tp * g.sld, szg = (long)Tp * g.gld;   // one (b, h) score / G image
  auto A0 = [](const void* p, long am, long ak, long az1, long az2) { BgArgs a{}; a.A = p; a.am = am; a.ak = ak; a.az1 = az1; a.az2 = az2; return a; };
  auto setB = [](BgArgs& a, const void* p, long bk, long bn, long bz1, long bz2) { a.B = p; a.bk = bk; a.bn = bn; a.bz1 = bz1; a.bz2 = bz2; };
  auto setC = [](BgArgs& a, float* p, long cm, long cn, long cz1, long cz2) { a.C = p; a.cm = cm; a.cn = cn; a.cz1 = cz1; a.cz2 = cz2; };
  const int Z = B * H;
  (void)es;
  // bf16: one fused launch produces P, dS and G (bf16) for the consumer GEMMs below
  const bool fused = dt == DT_BF16 && Tp <= 512 && dk % 16 == 0 && dk <= 128 && dkp == dk && ld_dctx % 4 == 0 &&
                     Tpad % 8 == 0 && ((uintptr_t)Vt % 16) == 0 &&
                     ((uintptr_t)dctx % 16) == 0 && attn_bwd_fused_enabled();
  const int opS = fused ? OP_CT : OP_F32;    // storage of the P / dS / G images
  if (fused) {
    const int nw = (Tp + 63) / 64, nq = (Tp + 31) / 32;
    const size_t lds = std::max((size_t)nw * 32 * 97 * sizeof(float), (size_t)nw * 64 * (dkp + 8) * sizeof(bf16_t));
    const dim3 grid((unsigned)(nq * Z)), block(64 * nw);
    const bf16_t* q16 = (const bf16_t*)qk;
    bf16_t *P16 = (bf16_t*)S, *dS16 = (bf16_t*)dP, *G16 = (bf16_t*)BD;
    auto go = [&](auto kern) {
      if (lds > 64 * 1024) (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      cfm_launch(kern, grid, block, lds, st, q16, ldqk, (const bf16_t*)Vt, vt_rows, Tpad, (const bf16_t*)P, ldp, dctx,
                 ld_dctx, lens, B, Tp, H, dkp, ctx_left, ctx_right, P16, dS16, g.sld, G16, g.gld, adrop);
    };
    switch (dkp / 16) {
      case 1: go(attn_bwd_scores_kernel<1>); break;
      case 2: go(attn_bwd_scores_kernel<2>); break;
      case 3: go(attn_bwd_scores_kernel<3>); break;
      case 4: go(attn_bwd_scores_kernel<4>); break;
      case 5: go(attn_bwd_scores_kernel<5>); break;
      case 6: go(attn_bwd_scores_kernel<6>); break;
      case 7: go(attn_bwd_scores_kernel<7>); break;
      default: go(attn_bwd_scores_kernel<8>); break;
    }
  }
  // S[b,h] = (q+u)c . k^T
  if (!fused) {
    BgArgs a = A0(qkc, ldqk, 1, (long)Tp * ldqk, dkp);
    setB(a, (const void*)nullptr, 1, ldqk, (long)Tp * ldqk, dkp);
    a.B = (const void*)(qkc + 2L * H * dkp * es);
    setC(a, S, g.sld, 1, (long)H * szs, szs);
    a.M = Tp; a.N = Tp; a.K = dk; a.Z2 = H; a.alpha = 1.0f; a.accumulate = 0;
    bgemm(dt, a, OP_CT, OP_CT, Z, st);
  }
  // BD[b,h] = (q+v)c . p^T   (2T'-1 positions)
  if (!fused) {
    BgArgs a = A0(qkc + (long)H * dkp * es, ldqk, 1, (long)Tp * ldqk, dkp);
    setB(a, P, 1, ldp, 0, dkp);
    setC(a, BD, g.gld, 1, (long)H * szg, szg);
    a.M = Tp; a.N = 2 * Tp - 1; a.K = dk; a.Z2 = H; a.alpha = 1.0f; a.accumulate = 0;
    bgemm(dt, a, OP_CT, OP_CT, Z, st);
  }
  const unsigned rows_blocks = (unsigned)((BT * H + 3) / 4);
  if (!fused) cfm_launch(attn_probs_kernel, dim3(rows_blocks), dim3(256), 0, st, S, g.sld, (const float*)BD, g.gld, lens, B, H, Tp,
             ctx_left, ctx_right);
  // dP[b,h] = dctx . V^T
  if (!fused) {
    BgArgs a = A0(dctx, ld_dctx, 1, (long)Tp * ld_dctx, dk);
    setB(a, Vt, (long)Tpad, 1, (long)H * vt_rows * Tpad, (long)vt_rows * Tpad);
    setC(a, dP, g.sld, 1, (long)H * szs, szs);
    a.M = Tp; a.N = Tp; a.K = dk; a.Z2 = H; a.alpha = 1.0f; a.accumulate = 0;
    bgemm(dt, a, OP_F32, OP_CT, Z, st);
  }
  if (!fused) cfm_launch(attn_dscore_kernel, dim3(rows_blocks), dim3(256), 0, st, S, dP, g.sld, BD, g.gld, B, H, Tp, adrop);
  float* G = BD;
  // d(q+u) = dS . k / sqrt(dk) -> dq
  {
    BgArgs a = A0(dP, g.sld, 1, (long)H * szs, szs);
    setB(a, qkc + 2L * H * dkp * es, ldqk, 1, (long)Tp * ldqk, dkp);
    setC(a, dq, ld_dqkv, 1, (long)Tp * ld_dqkv, dk);
    a.M = Tp; a.N = dk; a.K = Tp; a.Z2 = H; a.alpha = rs; a.accumulate = 0;
    bgemm(dt, a, opS, OP_CT, Z, st);
  }
  if (du) col_sums(dq, ld_dqkv, (int)BT, H * dk, du, 0, cs, st);
  // d(q+v) = G . p / sqrt(dk) -> tmp;  dq += tmp
  {
    BgArgs a = A0(G, g.gld, 1, (long)Tp * g.gld, (long)B * szg);   // G is [h][b][i][r]
    setB(a, P, ldp, 1, 0, dkp);
    setC(a, tmp, (long)H * dk, 1, (long)Tp * H * dk, dk);
    a.M = Tp; a.N = dk; a.K = 2 * Tp - 1; a.Z2 = H; a.alpha = rs; a.accumulate = 0;
    bgemm(dt, a, opS, OP_CT, Z, st);
  }
  if (dvb) col_sums(tmp, (long)H * dk, (int)BT, H * dk, dvb, 0, cs, st);
  cfm_launch(add_rows_kernel, dim3(1024), dim3(256), 0, st, dq, ld_dqkv, (const float*)tmp, (long)H * dk, BT, H * dk);
  // dk = dS^T . (q+u)c * ln2  (bf16: both operands are frame-major -> the TN kernel)
  if (!(fused && bgemm_tn(dP, g.sld, (long)H * szs, szs, qkc, ldqk, (long)Tp * ldqk, dkp, dk_, ld_dqkv,
                          (long)Tp * ld_dqkv, dk, Tp, dk, Tp, Z, H, 0, ln2, st))) {
    BgArgs a = A0(dP, 1, g.sld, (long)H * szs, szs);
    setB(a, qkc, ldqk, 1, (long)Tp * ldqk, dkp);
    setC(a, dk_, ld_dqkv, 1, (long)Tp * ld_dqkv, dk);
    a.M = Tp; a.N = dk; a.K = Tp; a.Z2 = H; a.alpha = ln2; a.accumulate = 0;
    bgemm(dt, a, opS, OP_CT, Z, st);
  }
  // dv = P^T . dctx (bf16: dctx rounded to bf16 in the tmp region, then the TN kernel)
  bool dv_done = false;
  if (fused && ld_dctx == (long)H * dk && dk % 8 == 0) {
    bf16_t* dctx16 = (bf16_t*)tmp;   // tmp (d(q+v)) was consumed by add_rows above
    convert_f32(DT_BF16, dctx, dctx16, BT * H * dk, st);
    dv_done = bgemm_tn(S, g.sld, (long)H * szs, szs, dctx16, (long)H * dk, (long)Tp * H * dk, dk, dv, ld_dqkv,
                       (long)Tp * ld_dqkv, dk, Tp, dk, Tp, Z, H, 0, 1.0f, st);
  }
  if (!dv_done) {
    BgArgs a = A0(S, 1, g.sld, (long)H * szs, szs);
    setB(a, dctx, ld_dctx, 1, (long)Tp * ld_dctx, dk);
    setC(a, dv, ld_dqkv, 1, (long)Tp * ld_dqkv, dk);
    a.M = Tp; a.N = dk; a.K = Tp; a.Z2 = H; a.alpha = 1.0f; a.accumulate = 0;
    bgemm(dt, a, opS, OP_F32, Z, st);
  }
  // dp[h] = sum_(b,i) G^T . (q+v)c * ln2: per head a GEMM with K = B*T' ((b, i) rows are uniform in
  // G and qk), split S ways along K (z = h * S + s) into fp32 slabs, then summed in a fixed order
  if (dpos) {
    const int S = BwdGeom::kPosSplit;
    const int kc = (int)((BT + S - 1) / S);
    const long NP = 2L * Tp - 1;
    float* part = (float*)(ws + 2 * g.s_bytes + g.g_bytes + g.t_bytes + g.cs_bytes);   // [s][NP][H*dk]
    BgArgs a = A0(G, 1, g.gld, (long)B * szg, (long)kc * g.gld);
    setB(a, qkc + (long)H * dkp * es, ldqk, 1, dkp, (long)kc * ldqk);
    setC(a, part, (long)H * dk, 1, dk, NP * H * dk);
    a.M = (int)NP; a.N = dk; a.K = kc; a.Z2 = S; a.alpha = ln2; a.accumulate = 0; a.Ktot = (int)BT;
    if (!(fused && bgemm_tn(G, g.gld, (long)B * szg, (long)kc * g.gld, qkc + (long)H * dkp * es, ldqk, dkp,
                            (long)kc * ldqk, part, (long)H * dk, dk, NP * H * dk, (int)NP, dk, kc, H * S, S,
                            (int)BT, ln2, st)))
      bgemm(dt, a, opS, OP_CT, H * S, st);
    cfm_launch(slab_rows_kernel, dim3(1024), dim3(256), 0, st, (const float*)part, S, NP, H * dk, dpos, ld_dpos);
  }
}

}  // namespace cfm

using namespace cfm;

extern "C" {

size_t cfm_op_rel_attention_backward_ws_size(int dtype, int B, int Tp, int H, int dk) {
  return cfm_op_rel_attention_ws_size(dtype, B, Tp, H, dk) + rel_pos_attention_backward_ws(B, Tp, H, dk) + 256;
}

cfm_status cfm_op_rel_attention_backward(int dtype, const void* q, const void* k, const void* v, const void* p,
                                         const float* pos_u, const float* pos_v, const int32_t* lens, int B, int Tp,
                                         int H, int dk, int ctx_left, int ctx_right, const float* dctx, float* dq,
                                         float* dk_, float* dv, float* dp, float* du, float* dvb, void* ws,
                                         size_t ws_bytes, void* stream) {
  return guarded([&] {
    if (B <= 0 || Tp <= 0 || H <= 0 || dk <= 0) fail(CFM_ERR_INVALID_ARG, "bad shape");
    if (dk > 128) fail(CFM_ERR_UNSUPPORTED, "head dim > 128");
    refuse_half_training(dtype == CFM_COMPUTE_FP32, "cfm_op_rel_attention_backward");
    if (!q || !k || !v || !p || !pos_u || !pos_v || !dctx || !dq || !dk_ || !dv || !ws)
      fail(CFM_ERR_INVALID_ARG, "null pointer");
    if (ws_bytes < cfm_op_rel_attention_backward_ws_size(dtype, B, Tp, H, dk))
      fail(CFM_ERR_INVALID_ARG, "workspace too small");
    const int dt = dtype == CFM_COMPUTE_FP32 ? DT_F32 : DT_BF16, es = dtype_size(dt);
    const int dkp = (int)round_up(dk, 16), vt_rows = (int)round_up(dkp, 32), Tpad = (int)round_up(Tp, 32);
    const long M = (long)B * Tp;
    const long qk_bytes = round_up(M * 3 * H * dkp * es, 256);
    const long vt_bytes = round_up((long)B * H * vt_rows * Tpad * es, 256);
    hipStream_t st = (hipStream_t)stream;
    char* w = (char*)ws;
    attn_relayout(dt, q, k, v, p, pos_u, pos_v, B, Tp, H, dk, dkp, vt_rows, Tpad, w, qk_bytes, vt_bytes, st);
    char* bw = w + round_up((long)cfm_op_rel_attention_ws_size(dtype, B, Tp, H, dk), 256);
    rel_pos_attention_backward(dt, w, 3L * H * dkp, w + qk_bytes, vt_rows, Tpad, w + qk_bytes + vt_bytes,
                               (long)H * dkp, lens, B, Tp, H, dk, dkp, ctx_left, ctx_right, dctx, (long)H * dk, dq,
                               dk_, dv, (long)H * dk, dp, (long)H * dk, du, dvb, bw, st);
    HIP_OK(hipGetLastError());
  });
}

}  // extern "C"
