// RNN-T joint network forward (RNNTJoint.joint, rnnt.py:951-1008), SURVEY §8 row a-ext4.
//
//   f' = enc(f) (B*T, H),  g' = pred(g) (B*U, H)            two small GEMMs, fp32 out
//   Hj[(b,t,u)] = act(f'[b,t] + g'[b,u])                   broadcast-add + activation, compute type
//   out[(b,t,u)] = Hj . W_out^T + b_out                     the big GEMM (B*T*U x C x H), fp32 out
//   optional log_softmax over C, one wave per row, in place
// bf16 (round 5, `joint_logits_kernel`): the hidden is never materialised - one kernel keeps a block's
// f' / g' rows in LDS and forms act(f' + g') as MFMA A-fragments in registers, rounded as the
// hidden kernel would store them; fp32 rows C = V + 1 wide (odd) go out from the accumulators (eval;
// training keeps the path below, whose hidden kernel draws joint_net's dropout mask once per element).
// Otherwise (fp32 compute, or shapes the fused kernel does not cover, or CFM_JOINT_FUSED=0) the hidden
// tensor is materialised in the compute type and the contraction runs on the LDS-DMA MFMA GEMM, its
// fp32 output rows written with the epilogue's element stores.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>

#include "../../include/cfm_joint.h"
#include "../../include/cfm_train.h"
#include <string>
#include "cfm_abi.h"
#include "cfm_common.h"
#include "cfm_kernels.h"

using namespace cfm;

struct cfm_rnnt_joint {
  int H1, H2, H, C, act, device, dtype, es, kg;
  char* wbuf = nullptr;
  long w_enc, b_enc, w_pred, b_pred, w_out, b_out, total;
  void* zero = nullptr;
  bool weights_set = false;
  long kp(long k) const { return round_up(k, kg); }
  long np(long n) const { return round_up(n, GEMM_BN); }
};

namespace {

// (B, D, L) fp32 -> rows (b, l) of D values in the compute type, ld = Dp (zero-padded)
template <typename T>
__global__ __launch_bounds__(256) void bdl_to_rows_kernel(const float* __restrict__ src, int D, int L,
                                                          T* __restrict__ dst, int Dp) {
  __shared__ float tile[32][33];
  const int b = blockIdx.z, l0 = blockIdx.x * 32, d0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int k = ty; k < 32; k += 8) {
    const int d = d0 + k, l = l0 + tx;
    tile[k][tx] = (d < D && l < L) ? src[((long)b * D + d) * L + l] : 0.0f;
  }
  __syncthreads();
  for (int k = ty; k < 32; k += 8) {
    const int l = l0 + k, d = d0 + tx;
    if (l < L && d < Dp) st_f<T>(dst + ((long)b * L + l) * Dp + d, tile[tx][k]);
  }
}

// Hj[(b,t,u)][h] = act(f[b*T+t][h] + g[b*U+u][h]); 8 h per thread (16-byte bf16 / 2x16-byte fp32 stores).
// Block (b*T + t, chunk of kHidU u's): 32-bit index math only, f's row loaded once per thread item,
// 16-byte f / g loads when H % 8 == 0.
// Tail columns (ntail > 0, compute-type hidden): the last ntail logits of every row, out[row][col0 + c] =
// Hj[row] . W[col0 + c] + b[col0 + c], from the hidden values as stored (rounded to the compute type) and
// the packed W rows - so the logits GEMM covers a whole number of 128-column tiles (V + 1 = 1025 -> 1024:
// its last 256-wide tile would otherwise compute 1 column of 256).  Per-row sums in a fixed order.
constexpr int kHidU = 16;
constexpr int kTailMax = 4;
template <typename TO>
__global__ __launch_bounds__(256) void joint_hidden_kernel(const float* __restrict__ f, const float* __restrict__ g,
                                                           int B, int T, int U, int H, int Hp, int act,
                                                           TO* __restrict__ out, Drop drop, int ntail,
                                                           const TO* __restrict__ wt, long ldw, const float* __restrict__ bt,
                                                           float* __restrict__ lo, long ldo) {
  __shared__ float tred[kTailMax * kHidU * 128];   // [c][uu][hg] partial dot products (Hp <= 1024)
  const int HG = Hp / 8;
  const int bt_ = blockIdx.x;
  const int b = bt_ / T;
  const int u0 = blockIdx.y * kHidU;
  const int nu = min(kHidU, U - u0);
  const bool vec = (H & 7) == 0;
  const float* fr = f + (long)bt_ * H;
  for (int j = threadIdx.x; j < nu * HG; j += 256) {
    const int uu = j / HG, hg = j - uu * HG;
    const int u = u0 + uu;
    const long row = (long)bt_ * U + u;
    const float* gr = g + ((long)b * U + u) * H;
    float v[8];
    if (vec && hg * 8 < H) {
      const float4 f0 = *(const float4*)(fr + hg * 8), f1 = *(const float4*)(fr + hg * 8 + 4);
      const float4 g0 = *(const float4*)(gr + hg * 8), g1 = *(const float4*)(gr + hg * 8 + 4);
      v[0] = f0.x + g0.x; v[1] = f0.y + g0.y; v[2] = f0.z + g0.z; v[3] = f0.w + g0.w;
      v[4] = f1.x + g1.x; v[5] = f1.y + g1.y; v[6] = f1.z + g1.z; v[7] = f1.w + g1.w;
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int h = hg * 8 + e;
        v[e] = h < H ? fr[h] + gr[h] : 0.0f;
      }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int h = hg * 8 + e;
      float x = v[e];
      if (act == CFM_JOINT_RELU) x = fmaxf(x, 0.0f);
      else if (act == CFM_JOINT_SIGMOID) x = 1.0f / (1.0f + expf(-x));
      else x = tanhf(x);
      v[e] = h < H ? x * drop_mul(drop, (uint64_t)row * H + h) : 0.0f;   // joint_net's Dropout (training)
    }
    TO* o = out + row * Hp + hg * 8;
    if constexpr (sizeof(TO) == 2) {
      const uint4 packed = Vec16<bf16_t>::from_f32(v);
      *(uint4*)o = packed;
      if (ntail > 0) {
        float vr[8], w8[8];
        Vec16<bf16_t>::to_f32(packed, vr);   // the hidden as the logits GEMM reads it
        for (int c = 0; c < ntail; ++c) {
          Vec16<bf16_t>::to_f32(*(const uint4*)(wt + (long)c * ldw + hg * 8), w8);
          float a = 0.0f;
#pragma unroll
          for (int e = 0; e < 8; ++e) a = fmaf(vr[e], w8[e], a);
          tred[(c * kHidU + uu) * 128 + hg] = a;
        }
      }
    } else {
      *(uint4*)o = Vec16<float>::from_f32(v);
      *(uint4*)(o + 4) = Vec16<float>::from_f32(v + 4);
    }
  }
  if (ntail > 0) {
    __syncthreads();
    for (int t = threadIdx.x; t < nu * ntail; t += 256) {
      const int uu = t / ntail, c = t - uu * ntail;
      float a = 0.0f;
      for (int hg = 0; hg < HG; ++hg) a += tred[(c * kHidU + uu) * 128 + hg];
      lo[((long)bt_ * U + u0 + uu) * ldo + c] = a + bt[c];
    }
  }
}
// As joint_hidden_kernel for H % 8 == 0 and Hp <= 1024, with the loads batched: thread (hg, group) keeps
// f's 8-column chunk hg (and the tail W chunk) in registers and issues the g chunks of all its u's
// (u = group + k * groups) before any arithmetic, so a block's memory traffic is in flight at once.
// The same values and the same tail partials as joint_hidden_kernel (bitwise).
template <typename TO>
__global__ __launch_bounds__(256) void joint_hidden_batched_kernel(const float* __restrict__ f,
                                                                   const float* __restrict__ g, int B, int T, int U,
                                                                   int H, int Hp, int act, TO* __restrict__ out,
                                                                   Drop drop, int ntail, const TO* __restrict__ wt,
                                                                   long ldw, const float* __restrict__ bt,
                                                                   float* __restrict__ lo, long ldo) {
  __shared__ float tred[kTailMax * kHidU * 128];
  constexpr int UPG = kHidU / 2;                    // u's per group (>= 2 groups since Hp <= 1024)
  const int HG = Hp / 8;
  const int ngrp = 256 / HG;
  const int bt_ = blockIdx.x;
  const int b = bt_ / T;
  const int u0 = blockIdx.y * kHidU;
  const int nu = min(kHidU, U - u0);
  const int hg = threadIdx.x % HG, grp = threadIdx.x / HG;
  const int h0 = hg * 8;
  const bool hok = h0 < H;                          // columns H..Hp-1: zero padding
  const int hc = hok ? h0 : 0;
  if (grp < ngrp) {
    const float* fr = f + (long)bt_ * H + hc;
    const float4 f0 = *(const float4*)fr, f1 = *(const float4*)(fr + 4);
    float4 ga[UPG], gb[UPG];
#pragma unroll
    for (int k = 0; k < UPG; ++k) {
      const int uu = min(grp + k * ngrp, nu - 1);
      const float* gr = g + ((long)b * U + u0 + uu) * H + hc;
      ga[k] = *(const float4*)gr;
      gb[k] = *(const float4*)(gr + 4);
    }
    float wtail[kTailMax][8] = {};
    if constexpr (sizeof(TO) == 2) {
      if (ntail > 0) {   // block-uniform
#pragma unroll
        for (int c = 0; c < kTailMax; ++c)
          Vec16<bf16_t>::to_f32(*(const uint4*)(wt + (long)min(c, ntail - 1) * ldw + h0), wtail[c]);
      }
    }
#pragma unroll
    for (int k = 0; k < UPG; ++k) {
      const int uu = grp + k * ngrp;
      if (uu >= nu) continue;
      const long row = (long)bt_ * U + u0 + uu;
      float v[8] = {f0.x + ga[k].x, f0.y + ga[k].y, f0.z + ga[k].z, f0.w + ga[k].w,
                    f1.x + gb[k].x, f1.y + gb[k].y, f1.z + gb[k].z, f1.w + gb[k].w};
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float x = v[e];
        if (act == CFM_JOINT_RELU) x = fmaxf(x, 0.0f);
        else if (act == CFM_JOINT_SIGMOID) x = 1.0f / (1.0f + expf(-x));
        else x = tanhf(x);
        v[e] = hok ? x * drop_mul(drop, (uint64_t)row * H + h0 + e) : 0.0f;
      }
      TO* o = out + row * Hp + h0;
      if constexpr (sizeof(TO) == 2) {
        const uint4 packed = Vec16<bf16_t>::from_f32(v);
        *(uint4*)o = packed;
        if (ntail > 0) {
          float vr[8];
          Vec16<bf16_t>::to_f32(packed, vr);
          for (int c = 0; c < ntail; ++c) {
            float a = 0.0f;
#pragma unroll
            for (int e = 0; e < 8; ++e) a = fmaf(vr[e], wtail[c][e], a);
            tred[(c * kHidU + uu) * 128 + hg] = a;
          }
        }
      } else {
        *(uint4*)o = Vec16<float>::from_f32(v);
        *(uint4*)(o + 4) = Vec16<float>::from_f32(v + 4);
      }
    }
  }
  if (ntail > 0) {
    __syncthreads();
    for (int t = threadIdx.x; t < nu * ntail; t += 256) {
      const int uu = t / ntail, c = t - uu * ntail;
      float a = 0.0f;
      for (int q = 0; q < HG; ++q) a += tred[(c * kHidU + uu) * 128 + q];
      lo[((long)bt_ * U + u0 + uu) * ldo + c] = a + bt[c];
    }
  }
}

template <typename TO>
void joint_hidden(const float* f, const float* g, int B, int T, int U, int H, int Hp, int act, TO* out, Drop drop,
                  hipStream_t st, int ntail = 0, const TO* wt = nullptr, long ldw = 0, const float* bt = nullptr,
                  float* lo = nullptr, long ldo = 0) {
  static const bool batched = [] { const char* e = getenv("CFM_JOINT_HID_BATCHED"); return !(e && !atoi(e)); }();
  const dim3 grid((unsigned)(B * T), (unsigned)((U + kHidU - 1) / kHidU));
  if (batched && H % 8 == 0 && Hp <= 1024 && Hp % 8 == 0)
    cfm_launch(joint_hidden_batched_kernel<TO>, grid, dim3(256), 0, st, f, g, B, T, U, H, Hp, act, out, drop, ntail,
               wt, ldw, bt, lo, ldo);
  else
    cfm_launch(joint_hidden_kernel<TO>, grid, dim3(256), 0, st, f, g, B, T, U, H, Hp, act, out, drop, ntail, wt, ldw,
               bt, lo, ldo);
}

// ---- the logits with the hidden formed in registers (bf16, round 5) ----------------------------------
// One block = one utterance's 16 frames x 16 labels = 256 lattice rows, all Cm logit columns in chunks of
// 256. The block's f' and g' rows (fp32) sit in LDS for its whole life; each wave builds the MFMA
// A-fragments of act(f' + g'), rounded to the compute type exactly as joint_hidden_kernel
// stores them, straight from those rows: a 16 x 32 fragment of v_mfma_f32_16x16x32 is one frame t and
// the 16 labels, so a lane reads its label's 8 g' values and the frame's 8 f' values (a broadcast). The
// hidden lattice never goes to memory. W_out streams from L2 through a two-stage LDS ring (64 K per
// stage, 128-byte rows XOR-swizzled by row pair), moved by waves 0-3 only; the <= 16 tail columns past
// the last whole chunk (V + 1 = 1025 -> 1024 + 1) are one more pass over K after the last chunk.
// Waves: 4 (frames: 4 each) x 2 (columns: 128 each); accumulators go straight from registers to the
// fp32 rows (stride C, any alignment): per store, 16 consecutive columns of 4 label rows.
namespace jl {
constexpr int TT = 16, UT = 16, NC = 256, KS = 64, HMAX = 640;
constexpr int STAGE = NC * KS * 2;                      // 32 KB: 256 W rows x 128 B
constexpr int FG_BYTES = 2 * 16 * (HMAX + 4) * 4;       // f' and g' rows, stride H + 4 floats
constexpr int LDS = FG_BYTES + 2 * STAGE;               // 147968 B
}  // namespace jl

struct JointLogits {
  const float* f; const float* g; const bf16_t* w; const float* bias; float* out;
  long ldw, ldo;
  int B, T, U, H, Cm, ntail;
  int split;   // W loads by waves 0-3 only (CFM_JOINT_SPLIT, default 1)
  int probe;   // timing probes only (CFM_JOINT_PROBE): 1 no logits stores, 2 no MFMAs, 4 no hidden formation
};

typedef float jf2 __attribute__((ext_vector_type(2)));
typedef short js2 __attribute__((ext_vector_type(2)));
#ifndef CFM_HALF_F16
typedef __bf16 jbf2 __attribute__((ext_vector_type(2)));
CFM_DEV uint32_t jpk(jf2 v) { return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, jbf2)); }   // RNE, as f2bf
CFM_DEV uint32_t relu_pk(uint32_t v, js2 z) { return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(js2, v), z)); }
#endif
template <int ACT> CFM_DEV float joint_act(float x) {
  if constexpr (ACT == CFM_JOINT_RELU) return fmaxf(x, 0.0f);
  else if constexpr (ACT == CFM_JOINT_SIGMOID) return 1.0f / (1.0f + expf(-x));
  else return tanhf(x);
}

template <int ACT, bool PROBE = false>
__global__ __launch_bounds__(512) void joint_logits_kernel(JointLogits p) {
  __shared__ __attribute__((aligned(16))) char smem[jl::LDS];
  const int hs = p.H + 4;
  float* Fs = (float*)smem;   // rows 0..15: f' of frames t0.., rows 16..31: g' of labels u0..
  const float* Gs = Fs + 16 * hs;
  char* Bs = smem + jl::FG_BYTES;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  const int nut = (p.U + jl::UT - 1) / jl::UT, ntt = (p.T + jl::TT - 1) / jl::TT;
  const int ut = blockIdx.x % nut, rest = blockIdx.x / nut;
  const int tt = rest % ntt, b = rest / ntt;
  const int t0 = tt * jl::TT, u0 = ut * jl::UT;
  {
    const int h4 = p.H / 4;
    for (int i = tid; i < 32 * h4; i += 512) {
      const int r = i / h4, c = i - r * h4;
      const bool isf = r < 16;
      const int x = isf ? t0 + r : u0 + r - 16, X = isf ? p.T : p.U;
      const float* src = isf ? p.f + ((long)b * p.T + min(x, X - 1)) * p.H : p.g + ((long)b * p.U + min(x, X - 1)) * p.H;
      float4 v = *(const float4*)(src + c * 4);   // clamped row, zeroed past the end
      if (x >= X) v = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
      *(float4*)(Fs + r * hs + c * 4) = v;
    }
  }
  const int kst = p.H / jl::KS, nstage = kst * (p.Cm / jl::NC);
  const bool tail = p.ntail > 0;
  // stage s -> ring slot s & 1 by LDS-DMA: wave-chunk cw = 8 W rows x 128 B; lane l fills slot (row
  // 8 cw + l / 8, position l % 8), i.e. the row's 16-byte K piece (l % 8) ^ ((row / 2) % 8)
  const uint32_t bs0 = lds_addr(Bs);
  // lane l's K piece is the same for every wave-chunk of a wave: rows 8 cw + l / 8 with cw = wave + 4 i
  // (or + 8 i) have (row / 2) % 8 = (4 (wave % 2) + l / 16) % 8; 32-bit element offsets from the stage's
  // wave-uniform W base
  const int lq = (lane & 7) ^ ((((wave & 1) << 2) + (lane >> 4)) & 7);
  const int lo = (wave * 8 + (lane >> 3)) * (int)p.ldw + lq * 8;
  const int ldw = (int)p.ldw;
  auto issue = [&](int s) {
    const int c = s / kst, ks = s - c * kst;
    const bf16_t* wb = p.w + (long)c * jl::NC * p.ldw + ks * jl::KS;
    const uint32_t dst = bs0 + (s & 1) * jl::STAGE;
    if (!p.split) {
#pragma unroll
      for (int i = 0; i < 4; ++i) glds16_asm(wb + lo + i * 64 * ldw, dst + (wave + 8 * i) * 1024);
    } else if (wave < 4) {
#pragma unroll
      for (int i = 0; i < 8; ++i) glds16_asm(wb + lo + i * 32 * ldw, dst + (wave + 4 * i) * 1024);
    }
  };
  // split: waves 0-3 move W and wait for it; waves 4-7 issue no loads, so their logits stores drain while
  // they compute (vmcnt counts stores and loads in one in-order counter per wave)
  const bool waiter = !p.split || wave < 4;
  f32x4 acc[4][8];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
  const int ul = lane & 15, kq = lane >> 4;
  // A-fragment of frame row tr (0..15) at K offset kk: act(f' + g') in the compute type
  auto afrag = [&](int tr, int kk, const float4& g0, const float4& g1) {
    const float* fr = Fs + tr * hs + kk;
    const float4 f0 = *(const float4*)fr, f1 = *(const float4*)(fr + 4);
#ifndef CFM_HALF_F16
    if constexpr (ACT == CFM_JOINT_RELU) {
      // packed: 4 v_pk_add_f32, 4 v_cvt_pk_bf16_f32, then ReLU on the bf16 pairs as 16-bit integers
      // (v_pk_max_i16: a sign-magnitude value is negative iff its sign bit is set; rounding keeps signs)
      const jf2 s0 = jf2{f0.x, f0.y} + jf2{g0.x, g0.y}, s1 = jf2{f0.z, f0.w} + jf2{g0.z, g0.w};
      const jf2 s2 = jf2{f1.x, f1.y} + jf2{g1.x, g1.y}, s3 = jf2{f1.z, f1.w} + jf2{g1.z, g1.w};
      const js2 z = js2{0, 0};
      return make_uint4(relu_pk(jpk(s0), z), relu_pk(jpk(s1), z), relu_pk(jpk(s2), z), relu_pk(jpk(s3), z));
    }
#endif
    float v[8] = {f0.x + g0.x, f0.y + g0.y, f0.z + g0.z, f0.w + g0.w, f1.x + g1.x, f1.y + g1.y, f1.z + g1.z, f1.w + g1.w};
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = joint_act<ACT>(v[e]);
#ifndef CFM_HALF_F16
    return make_uint4(jpk(jf2{v[0], v[1]}), jpk(jf2{v[2], v[3]}), jpk(jf2{v[4], v[5]}), jpk(jf2{v[6], v[7]}));
#else
    return Vec16<bf16_t>::from_f32(v);
#endif
  };
  // the four A-fragments (frame rows wr * 4 + i, the 16 labels) of K offset kk
  auto build4 = [&](int kk, uint4* a) {
    const float4 g0 = *(const float4*)(Gs + ul * hs + kk), g1 = *(const float4*)(Gs + ul * hs + kk + 4);
    if (PROBE && (p.probe & 4)) {
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = make_uint4(__float_as_uint(g0.x), __float_as_uint(g0.y), __float_as_uint(g1.x), __float_as_uint(g1.y));
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = afrag(wr * 4 + i, kk, g0, g1);
    }
  };
  __syncthreads();   // f', g' rows in LDS (compiler-visible loads: drained here)
  constexpr bool PIPE = ACT == CFM_JOINT_RELU;
  uint4 af[4];
  if constexpr (PIPE) build4(8 * kq, af);
  issue(0);
  wait_vmcnt<0>();
  __syncthreads();
  for (int s = 0; s < nstage; ++s) {
    const int c = s / kst, ks = s - c * kst;
    if (s + 1 < nstage) issue(s + 1);
    const char* bs = Bs + (s & 1) * jl::STAGE;
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      // the next K sub-step's fragments (K restarts with every column chunk) are formed while this
      // sub-step's MFMAs run: they depend on the resident f' / g' rows only, not on the W ring
      // (ReLU: the cheap formation; the others keep it in place, for their registers)
      uint4 an[4];
      if constexpr (PIPE) {
        int kn = ks * 2 + sub + 1;
        if (kn == 2 * kst) kn = 0;
        build4(kn * 32 + 8 * kq, an);
      } else {
        build4((ks * 2 + sub) * 32 + 8 * kq, af);
      }
      const int q = sub * 4 + kq;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int n = wc * 128 + j * 16 + ul;
        const uint4 bf = *(const uint4*)(bs + n * 128 + ((q ^ ((n >> 1) & 7)) << 4));
        if (!(PROBE && (p.probe & 2))) {
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[i][j] = mfma16_16x16x32(af[i], bf, acc[i][j]);
        }
      }
      if constexpr (PIPE) {
#pragma unroll
        for (int i = 0; i < 4; ++i) af[i] = an[i];
      }
    }
    if (ks == kst - 1 && !(PROBE && (p.probe & 1))) {
      // accumulator element r of lane l: label row 4 * (l >> 4) + r, column l & 15. Whole tiles (every
      // block but the last label tile's) store without per-element conditions.
      const int n0 = c * jl::NC + wc * 128 + ul;
      float bn[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) bn[j] = p.bias[n0 + j * 16];
      const bool full = t0 + jl::TT <= p.T && u0 + jl::UT <= p.U;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int t = t0 + wr * 4 + i;
        float* o = p.out + (((long)b * p.T + t) * p.U + u0 + 4 * kq) * p.ldo + n0;
        if (full) {
#pragma unroll
          for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int j = 0; j < 8; ++j) o[r * p.ldo + j * 16] = acc[i][j][r] + bn[j];
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (t < p.T && u0 + 4 * kq + r < p.U) {
#pragma unroll
              for (int j = 0; j < 8; ++j) o[r * p.ldo + j * 16] = acc[i][j][r] + bn[j];
            }
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
      }
    }
    if (waiter) wait_vmcnt<0>();   // stage s + 1 landed (and this wave's logits stores left)
    __syncthreads();
  }
  if (!tail) return;
  // the <= 16 tail columns Cm..: their whole W rows (16 x H, zero past C) in the ring, then per wave two
  // frame rows x one 16-column fragment over all of K
  {
    const int kb = p.H / 8;   // 16-byte pieces per row
    for (int i = tid; i < 16 * kb; i += 512) {
      const int r = i / kb, q = i - r * kb;
      *(uint4*)(Bs + r * p.H * 2 + q * 16) = *(const uint4*)(p.w + (long)(p.Cm + r) * p.ldw + q * 8);
    }
  }
  __syncthreads();
  f32x4 at[2] = {f32x4{0.0f, 0.0f, 0.0f, 0.0f}, f32x4{0.0f, 0.0f, 0.0f, 0.0f}};
  for (int k0 = 0; k0 < p.H; k0 += 32) {
    const int kk = k0 + 8 * kq;
    const float4 g0 = *(const float4*)(Gs + ul * hs + kk), g1 = *(const float4*)(Gs + ul * hs + kk + 4);
    const uint4 bt = *(const uint4*)(Bs + ul * p.H * 2 + kk * 2);
#pragma unroll
    for (int i = 0; i < 2; ++i) at[i] = mfma16_16x16x32(afrag(wave * 2 + i, kk, g0, g1), bt, at[i]);
  }
  if (ul < p.ntail) {
    const int n = p.Cm + ul;
    const float bn = p.bias[n];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int t = t0 + wave * 2 + i;
      const long rowb = ((long)b * p.T + t) * p.U + u0 + 4 * kq;
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (t < p.T && u0 + 4 * kq + r < p.U) p.out[(rowb + r) * p.ldo + n] = at[i][r] + bn;
    }
  }
}

// the fused form applies: bf16, H a multiple of 64 up to 640, whole 256-column chunks + <= 16 tail columns
bool joint_logits_fusable(int dt, int H, int C) {
  const char* e = getenv("CFM_JOINT_FUSED");   // read per call: 0 = the hidden kernel + logits GEMM (A/B)
  const bool on = !(e && !atoi(e));
  return on && dt == DT_BF16 && H % jl::KS == 0 && H <= jl::HMAX && C >= jl::NC && C % jl::NC <= 16;
}

void joint_logits(const float* f, const float* g, int B, int T, int U, int H, int act, const bf16_t* w, long ldw,
                  const float* bias, int C, float* out, hipStream_t st) {
  JointLogits p;
  p.f = f; p.g = g; p.w = w; p.bias = bias; p.out = out; p.ldw = ldw; p.ldo = C;
  p.B = B; p.T = T; p.U = U; p.H = H; p.ntail = C % jl::NC; p.Cm = C - p.ntail;
  const char* se = getenv("CFM_JOINT_SPLIT");
  p.split = se ? atoi(se) : 1;
  const char* pe = getenv("CFM_JOINT_PROBE");
  p.probe = pe ? atoi(pe) : 0;
  const long blocks = (long)B * ((T + jl::TT - 1) / jl::TT) * ((U + jl::UT - 1) / jl::UT);
  if (blocks > 0x7fffffffL) fail(CFM_ERR_UNSUPPORTED, "joint: too many lattice tiles");
  const dim3 grid((unsigned)blocks), block(512);
  if (p.probe && act == CFM_JOINT_RELU)
    cfm_launch(joint_logits_kernel<CFM_JOINT_RELU, true>, grid, block, 0, st, p);
  else if (act == CFM_JOINT_RELU)
    cfm_launch(joint_logits_kernel<CFM_JOINT_RELU>, grid, block, 0, st, p);
  else if (act == CFM_JOINT_SIGMOID)
    cfm_launch(joint_logits_kernel<CFM_JOINT_SIGMOID>, grid, block, 0, st, p);
  else
    cfm_launch(joint_logits_kernel<CFM_JOINT_TANH>, grid, block, 0, st, p);
}

// in-place log_softmax over rows of C fp32 values, one wave per row
__global__ __launch_bounds__(256) void row_log_softmax_kernel(float* __restrict__ x, long rows, int C) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  float* r = x + row * C;
  float m = -INFINITY;
  for (int c = lane; c < C; c += 64) m = fmaxf(m, r[c]);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  float s = 0.0f;
  for (int c = lane; c < C; c += 64) s += expf(r[c] - m);
  s = wave_sum(s);
  const float lse = m + logf(s);
  for (int c = lane; c < C; c += 64) r[c] -= lse;
}

unsigned ew_grid(long n) { return (unsigned)std::max<long>(1, std::min<long>((n + 255) / 256, 16384)); }

struct JWs { long af, ag, fp, gp, hid, total; };
JWs jws(const cfm_rnnt_joint* h, int B, int T, int U) {
  JWs w;
  long off = 0;
  auto take = [&](long bytes) { const long o = round_up(off, 256); off = o + round_up(std::max(bytes, 1L), 256); return o; };
  const long Hp = round_up(h->H, std::max(8, h->kg));
  w.af = take((long)B * T * h->kp(h->H1) * h->es);
  w.ag = take((long)B * U * h->kp(h->H2) * h->es);
  w.fp = take((long)B * T * h->H * 4);
  w.gp = take((long)B * U * h->H * 4);
  // the hidden lattice (training, and the unfused path; the fused eval kernel forms it in registers)
  w.hid = take((long)B * T * U * Hp * h->es);
  w.total = round_up(off, 256);
  return w;
}

GemmEpi epi_f32(const float* bias, float* X, long ldx, int scalar) {
  GemmEpi e;
  std::memset(&e, 0, sizeof(e));
  e.mode = EPI_SCALE_F32;
  e.bias = bias;
  e.alpha = 1.0f;
  e.X = X;
  e.ldx = ldx;
  // unaligned rows: out_scalar 1 = heads / tails one element per lane; CFM_LOGITS_STORE=1 keeps the
  // round-3 single-thread form (A/B)
  static const int legacy = [] { const char* v = getenv("CFM_LOGITS_STORE"); return v ? atoi(v) : 0; }();
  e.out_scalar = scalar ? (legacy == 1 ? 2 : 1) : 0;
  return e;
}

// dz[(b,t,u)][j] = dh * dropout'(row, j) * act'(z), z = f[b,t][j] + g[b,u][j]; reduced over u (per (b, t))
__device__ __forceinline__ float act_grad(int act, float z) {
  if (act == CFM_JOINT_RELU) return z > 0.0f ? 1.0f : 0.0f;
  if (act == CFM_JOINT_SIGMOID) { const float s = 1.0f / (1.0f + expf(-z)); return s * (1.0f - s); }
  const float t = tanhf(z);
  return 1.0f - t * t;
}
__global__ __launch_bounds__(256) void joint_act_bwd_t_kernel(const float* __restrict__ f, const float* __restrict__ g,
                                                              const float* __restrict__ dh, int B, int T, int U, int H,
                                                              int act, Drop drop, float* __restrict__ df) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  const long bt = blockIdx.y;
  if (j >= H) return;
  const int b = (int)(bt / T);
  const float fv = f[bt * H + j];
  float s = 0.0f;
  for (int u = 0; u < U; ++u) {
    const long row = bt * U + u;
    const float z = fv + g[((long)b * U + u) * H + j];
    s += dh[row * H + j] * drop_mul(drop, (uint64_t)row * H + j) * act_grad(act, z);
  }
  df[bt * H + j] = s;
}
// ... reduced over t (per (b, u))
__global__ __launch_bounds__(256) void joint_act_bwd_u_kernel(const float* __restrict__ f, const float* __restrict__ g,
                                                              const float* __restrict__ dh, int B, int T, int U, int H,
                                                              int act, Drop drop, float* __restrict__ dp) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  const long bu = blockIdx.y;
  if (j >= H) return;
  const int b = (int)(bu / U), u = (int)(bu % U);
  const float gv = g[bu * H + j];
  float s = 0.0f;
  for (int t = 0; t < T; ++t) {
    const long row = ((long)b * T + t) * U + u;
    const float z = f[((long)b * T + t) * H + j] + gv;
    s += dh[row * H + j] * drop_mul(drop, (uint64_t)row * H + j) * act_grad(act, z);
  }
  dp[bu * H + j] = s;
}

// Both reductions in one pass over dh (round 5): block (128 columns, 16 frames, b). Each dz is formed once
// (one dropout hash); df over u in ascending order (the same sums as joint_act_bwd_t_kernel, bitwise), dp
// as per-tile partials over the tile's frames (ascending) summed over the tiles by joint_act_bwd_dp_kernel.
constexpr int kActTT = 16;
__global__ __launch_bounds__(128) void joint_act_bwd_tu_kernel(const float* __restrict__ f, const float* __restrict__ g,
                                                               const float* __restrict__ dh, int B, int T, int U, int H,
                                                               int act, Drop drop, float* __restrict__ df,
                                                               float* __restrict__ part) {
  const int j = blockIdx.x * 128 + threadIdx.x;
  const int tt = blockIdx.y, b = blockIdx.z;
  const int ntt = gridDim.y;
  if (j >= H) return;
  const int t0 = tt * kActTT;
  const int nt = min(kActTT, T - t0);
  float fv[kActTT], dfa[kActTT];
#pragma unroll
  for (int i = 0; i < kActTT; ++i) {
    fv[i] = f[((long)b * T + t0 + min(i, nt - 1)) * H + j];
    dfa[i] = 0.0f;
  }
  for (int u = 0; u < U; ++u) {
    const float gv = g[((long)b * U + u) * H + j];
    float dpa = 0.0f;
#pragma unroll
    for (int i = 0; i < kActTT; ++i) {
      const long row = ((long)b * T + t0 + min(i, nt - 1)) * U + u;
      const float dz = dh[row * H + j] * drop_mul(drop, (uint64_t)row * H + j) * act_grad(act, fv[i] + gv);
      if (i < nt) { dfa[i] += dz; dpa += dz; }
    }
    part[(((long)b * ntt + tt) * U + u) * H + j] = dpa;
  }
#pragma unroll
  for (int i = 0; i < kActTT; ++i)
    if (i < nt) df[((long)b * T + t0 + i) * H + j] = dfa[i];
}
__global__ __launch_bounds__(256) void joint_act_bwd_dp_kernel(const float* __restrict__ part, int B, int ntt, int U,
                                                               int H, float* __restrict__ dp) {
  const long n = (long)B * U * H;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const long bu = i / H;
    const int j = (int)(i - bu * H);
    const long b = bu / U, u = bu - b * U;
    float a = 0.0f;
    for (int q = 0; q < ntt; ++q) a += part[((b * ntt + q) * U + u) * H + j];
    dp[i] = a;
  }
}

// joint_net[-1] weight/bias gradient partials (bf16 path): [S][C][H + 4] -> dW (C, H) and db at column H
__global__ __launch_bounds__(256) void joint_slab_kernel(const float* __restrict__ part, int S, int N, int K,
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

// bf16 output-layer backward (joint_net[-1]): dlogits packed once to bf16 rows, the dgrad GEMM on them and
// the weight gradient on the frame-major TN kernel (row splits, bias in-kernel) - no transposed copies of
// the (B*T*U, C) gradient or of the hidden
bool joint_fast_bwd(const cfm_rnnt_joint* h) { return h->dtype == DT_BF16 && h->H % 8 == 0 && h->H <= 4096; }
struct JFast { long S, chunk; };
JFast joint_fast_splits(const cfm_rnnt_joint* h, long rows) {
  const long tiles = ((h->C + 127) / 128) * ((h->H + 127) / 128);
  long S = std::max<long>(1, std::min<long>({(512 + tiles - 1) / tiles, rows / 64, 16L}));
  const long chunk = round_up((rows + S - 1) / S, 32);
  return JFast{(rows + chunk - 1) / chunk, chunk};
}

struct JBWs { long er, dr, fp, gp, hid, dh, df, dp, dx, lin, a1, wtp, part, actp, total; };
JBWs jbws(const cfm_rnnt_joint* h, int B, int T, int U) {
  JBWs w;
  long off = 0;
  auto take = [&](long bytes) { const long o = round_up(off, 256); off = o + round_up(std::max(bytes, 1L), 256); return o; };
  const long rows = (long)B * T * U;
  const int mode = h->dtype == DT_F32 ? CFM_COMPUTE_FP32 : CFM_COMPUTE_BF16;
  const bool fast = joint_fast_bwd(h);
  const long Cp = round_up(h->C, 64);
  w.er = take((long)B * T * h->H1 * 4);
  w.dr = take((long)B * U * h->H2 * 4);
  w.fp = take((long)B * T * h->H * 4);
  w.gp = take((long)B * U * h->H * 4);
  w.hid = take(rows * h->H * (fast ? 2 : 4));   // the output Linear's input (bf16 on the fast path)
  w.a1 = fast ? take(rows * Cp * 2) : 0;
  w.wtp = fast ? take(round_up(h->H, 256) * Cp * 2) : 0;
  w.part = fast ? take(joint_fast_splits(h, rows).S * h->C * (h->H + 4) * 4) : 0;
  // dh also holds the compute-type projection inputs before it is written
  w.dh = take(std::max(rows * h->H * 4, (long)B * T * h->kp(h->H1) * h->es + (long)B * U * h->kp(h->H2) * h->es + 512));
  w.df = take((long)B * T * h->H * 4);
  w.dp = take((long)B * U * h->H * 4);
  w.actp = take((long)B * ((T + kActTT - 1) / kActTT) * U * h->H * 4);   // dp partials per 16-frame tile
  w.dx = take((long)std::max(B * T * h->H1, B * U * h->H2) * 4);
  const size_t l1 = fast ? 0 : cfm_op_linear_backward_ws_size(mode, (int)rows, h->H, h->C);
  const size_t l2 = cfm_op_linear_backward_ws_size(mode, B * T, h->H1, h->H);
  const size_t l3 = cfm_op_linear_backward_ws_size(mode, B * U, h->H2, h->H);
  w.lin = take((long)std::max(l1, std::max(l2, l3)));
  w.total = round_up(off, 256);
  return w;
}

}  // namespace

extern "C" {

cfm_status cfm_rnnt_joint_create(int encoder_hidden, int pred_hidden, int joint_hidden, int num_classes,
                                 int activation, int device, int compute_mode, cfm_rnnt_joint** out) {
  return guarded([&] {
    if (!out) fail(CFM_ERR_INVALID_ARG, "null output");
    *out = nullptr;
    if (encoder_hidden <= 0 || pred_hidden <= 0 || joint_hidden <= 0 || num_classes <= 0)
      fail(CFM_ERR_INVALID_ARG, "sizes must be positive");
    if (activation < 0 || activation > 2) fail(CFM_ERR_INVALID_ARG, "activation must be relu, sigmoid or tanh");
    if (compute_mode != CFM_COMPUTE_FP32 && compute_mode != CFM_COMPUTE_BF16) fail(CFM_ERR_INVALID_ARG, "compute mode");
    if (encoder_hidden % 4 || pred_hidden % 4) fail(CFM_ERR_UNSUPPORTED, "encoder/pred hidden must be multiples of 4");
    int ndev = 0;
    HIP_OK(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) fail(CFM_ERR_INVALID_ARG, "bad device");
    HIP_OK(hipSetDevice(device));
    auto* h = new cfm_rnnt_joint();
    h->H1 = encoder_hidden; h->H2 = pred_hidden; h->H = joint_hidden; h->C = num_classes; h->act = activation;
    h->device = device;
    h->dtype = compute_mode == CFM_COMPUTE_FP32 ? DT_F32 : DT_BF16;
    h->es = dtype_size(h->dtype);
    h->kg = GEMM_BK_BYTES / h->es;
    long off = 0;
    auto take = [&](long bytes) { const long o = round_up(off, 256); off = o + round_up(bytes, 256); return o; };
    const long Hk = h->kp(h->H);
    h->w_enc = take(h->np(h->H) * h->kp(h->H1) * h->es);
    h->b_enc = take(h->np(h->H) * 4);
    h->w_pred = take(h->np(h->H) * h->kp(h->H2) * h->es);
    h->b_pred = take(h->np(h->H) * 4);
    h->w_out = take(h->np(h->C) * Hk * h->es);
    h->b_out = take(h->np(h->C) * 4);
    h->total = off;
    if (hipMalloc(&h->wbuf, (size_t)off) != hipSuccess || hipMalloc(&h->zero, 4096) != hipSuccess) {
      if (h->wbuf) (void)hipFree(h->wbuf);
      delete h;
      fail(CFM_ERR_NOMEM, "joint weight allocation failed");
    }
    HIP_OK(hipMemset(h->zero, 0, 4096));
    HIP_OK(hipMemset(h->wbuf, 0, (size_t)off));
    *out = h;
  });
}

void cfm_rnnt_joint_destroy(cfm_rnnt_joint* h) {
  if (!h) return;
  (void)hipSetDevice(h->device);
  if (h->wbuf) (void)hipFree(h->wbuf);
  if (h->zero) (void)hipFree(h->zero);
  delete h;
}

cfm_status cfm_rnnt_joint_set_weights(cfm_rnnt_joint* h, const float* w_enc, const float* b_enc, const float* w_pred,
                                      const float* b_pred, const float* w_out, const float* b_out, void* stream) {
  return guarded([&] {
    if (!h || !w_enc || !w_pred || !w_out) fail(CFM_ERR_INVALID_ARG, "null argument");
    HIP_OK(hipSetDevice(h->device));
    hipStream_t st = (hipStream_t)stream;
    auto packw = [&](const float* w, int N, int K, long off) {
      pack_matrix(h->dtype, w, K, N, K, false, h->wbuf + off, h->kp(K), (int)h->np(N), (int)h->kp(K), st);
    };
    auto packb = [&](const float* b, int N, long off) {
      HIP_OK(hipMemsetAsync(h->wbuf + off, 0, (size_t)h->np(N) * 4, st));
      if (b) HIP_OK(hipMemcpyAsync(h->wbuf + off, b, (size_t)N * 4, hipMemcpyDeviceToDevice, st));
    };
    packw(w_enc, h->H, h->H1, h->w_enc);
    packb(b_enc, h->H, h->b_enc);
    packw(w_pred, h->H, h->H2, h->w_pred);
    packb(b_pred, h->H, h->b_pred);
    packw(w_out, h->C, h->H, h->w_out);
    packb(b_out, h->C, h->b_out);
    HIP_OK(hipGetLastError());
    h->weights_set = true;
  });
}

size_t cfm_rnnt_joint_workspace_size(const cfm_rnnt_joint* h, int B, int T, int U) {
  if (!h || B <= 0 || T <= 0 || U <= 0) return 0;
  return (size_t)jws(h, B, T, U).total;
}

}  // extern "C"

namespace {
// RNNTJoint.joint (rnnt.py:951-1008) with joint_net's Dropout as `drop` (training; none in eval)
void joint_forward(cfm_rnnt_joint* h, const float* enc_bdt, const float* dec_bdu, int B, int T, int U, int log_softmax,
                   float* out, void* workspace, size_t workspace_bytes, hipStream_t stream, Drop drop) {
    if (!h || !enc_bdt || !dec_bdu || !out) fail(CFM_ERR_INVALID_ARG, "null argument");
    if (!h->weights_set) fail(CFM_ERR_WEIGHTS, "weights not set");
    if (B <= 0 || T <= 0 || U <= 0) fail(CFM_ERR_INVALID_ARG, "B, T and U must be positive");
    const long rows = (long)B * T * U;
    if (rows > 0x7fffffffL) fail(CFM_ERR_UNSUPPORTED, "B*T*U exceeds 2^31 rows");
    const JWs w = jws(h, B, T, U);
    if (!workspace || workspace_bytes < (size_t)w.total) fail(CFM_ERR_WORKSPACE, "workspace too small");
    hipStream_t st = stream;
    char* ws = (char*)workspace;
    const int dt = h->dtype;
    const int H1p = (int)h->kp(h->H1), H2p = (int)h->kp(h->H2);
    const int Hp = (int)round_up(h->H, std::max(8, h->kg));
    // (B, D, L) -> rows
    if (dt == DT_F32) {
      cfm_launch(bdl_to_rows_kernel<float>, dim3((T + 31) / 32, (H1p + 31) / 32, B), dim3(256), 0, st, enc_bdt, h->H1,
                 T, (float*)(ws + w.af), H1p);
      cfm_launch(bdl_to_rows_kernel<float>, dim3((U + 31) / 32, (H2p + 31) / 32, B), dim3(256), 0, st, dec_bdu, h->H2,
                 U, (float*)(ws + w.ag), H2p);
    } else {
      cfm_launch(bdl_to_rows_kernel<bf16_t>, dim3((T + 31) / 32, (H1p + 31) / 32, B), dim3(256), 0, st, enc_bdt,
                 h->H1, T, (bf16_t*)(ws + w.af), H1p);
      cfm_launch(bdl_to_rows_kernel<bf16_t>, dim3((U + 31) / 32, (H2p + 31) / 32, B), dim3(256), 0, st, dec_bdu,
                 h->H2, U, (bf16_t*)(ws + w.ag), H2p);
    }
    float* fp = (float*)(ws + w.fp);
    float* gp = (float*)(ws + w.gp);
    const int sc = h->H % 4 ? 1 : 0;
    gemm(dt, ws + w.af, H1p, B * T, h->H1, h->wbuf + h->w_enc, H1p, h->H,
         epi_f32((const float*)(h->wbuf + h->b_enc), fp, h->H, sc), h->zero, st);
    gemm(dt, ws + w.ag, H2p, B * U, h->H2, h->wbuf + h->w_pred, H2p, h->H,
         epi_f32((const float*)(h->wbuf + h->b_pred), gp, h->H, sc), h->zero, st);
    // the last (C % 128) <= kTailMax logits of each row come from the hidden kernel, the GEMM covers
    // whole 128-column tiles (bf16 mode; V + 1 = 1025 -> 1024 + 1)
    const int ntail = (dt == DT_BF16 && h->C > 128 && h->C % 128 <= kTailMax && Hp <= 1024) ? h->C % 128 : 0;
    const int Cm = h->C - ntail;
    // inference: the lattice in chunks of `chunk` utterances (hidden kernel, then logits GEMM, per chunk), so
    // each chunk's hidden is read back while it is still in the Infinity Cache (CFM_JOINT_CHUNK, 0 = whole)
    static const int chunk_env = [] { const char* e = getenv("CFM_JOINT_CHUNK"); return e ? atoi(e) : 0; }();
    const int chunk = (drop.thr == 0 && chunk_env > 0) ? std::min(chunk_env, B) : B;
    // eval: the fused logits kernel. Training keeps the hidden kernel + GEMM: with joint_net's dropout
    // the fused kernel would hash every hidden element once per 256-column chunk (RNN-T training step
    // 43.8-44.2 -> 44.9-45.0 ms, profiles/r05jd_joint_fused_ab.txt)
    const bool fused = drop.thr == 0 && joint_logits_fusable(dt, h->H, h->C);
    if (fused)
      joint_logits(fp, gp, B, T, U, h->H, h->act, (const bf16_t*)(h->wbuf + h->w_out), h->kp(h->H),
                   (const float*)(h->wbuf + h->b_out), h->C, out, st);
    for (int b0 = 0; b0 < (fused ? 0 : B); b0 += chunk) {
      const int nb = std::min(chunk, B - b0);
      const long r0 = (long)b0 * T * U, nrows = (long)nb * T * U;
      const float* fpc = fp + (long)b0 * T * h->H;
      const float* gpc = gp + (long)b0 * U * h->H;
      float* outc = out + r0 * h->C;
      if (dt == DT_F32)
        joint_hidden<float>(fpc, gpc, nb, T, U, h->H, Hp, h->act, (float*)(ws + w.hid), drop, st);
      else
        joint_hidden<bf16_t>(fpc, gpc, nb, T, U, h->H, Hp, h->act, (bf16_t*)(ws + w.hid), drop, st, ntail,
                             (const bf16_t*)(h->wbuf + h->w_out) + (long)Cm * h->kp(h->H), h->kp(h->H),
                             (const float*)(h->wbuf + h->b_out) + Cm, outc + Cm, h->C);
      GemmEpi le = epi_f32((const float*)(h->wbuf + h->b_out), outc, h->C, h->C % 4 ? 1 : 0);
      static const int nt_env = [] { const char* e = getenv("CFM_LOGITS_NT"); return e ? atoi(e) : 0; }();
      le.nt_store = le.out_scalar ? nt_env : 0;
      gemm(dt, ws + w.hid, Hp, (int)nrows, h->H, h->wbuf + h->w_out, (int)h->kp(h->H), Cm, le, h->zero, st);
    }
    if (log_softmax)
      cfm_launch(row_log_softmax_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, st, out, rows, h->C);
    HIP_OK(hipGetLastError());
}
}  // namespace

extern "C" {

cfm_status cfm_rnnt_joint_forward(cfm_rnnt_joint* h, const float* enc_bdt, const float* dec_bdu, int B, int T, int U,
                                  int log_softmax, float* out, void* workspace, size_t workspace_bytes, void* stream) {
  return guarded([&] {
    joint_forward(h, enc_bdt, dec_bdu, B, T, U, log_softmax, out, workspace, workspace_bytes, (hipStream_t)stream,
                  Drop{0u, 0u, 1.0f});
  });
}

cfm_status cfm_rnnt_joint_forward_train(cfm_rnnt_joint* h, const float* enc_bdt, const float* dec_bdu, int B, int T,
                                        int U, float dropout, uint64_t seed, float* out, void* workspace,
                                        size_t workspace_bytes, void* stream) {
  return guarded([&] {
    if (h) refuse_half_training(h->dtype == DT_F32, "cfm_rnnt_joint_forward_train");
    joint_forward(h, enc_bdt, dec_bdu, B, T, U, 0, out, workspace, workspace_bytes, (hipStream_t)stream,
                  make_drop(dropout, seed, 1));
  });
}

size_t cfm_rnnt_joint_backward_workspace_size(const cfm_rnnt_joint* h, int B, int T, int U) {
  if (!h || B <= 0 || T <= 0 || U <= 0) return 0;
  return (size_t)jbws(h, B, T, U).total;
}

cfm_status cfm_rnnt_joint_backward(cfm_rnnt_joint* h, const float* enc_bdt, const float* dec_bdu, int B, int T, int U,
                                   float dropout, uint64_t seed, const float* dlogits, const float* w_enc,
                                   const float* w_pred, const float* w_out, float* d_enc_bdt, float* d_dec_bdu,
                                   float* dw_enc, float* db_enc, float* dw_pred, float* db_pred, float* dw_out,
                                   float* db_out, void* workspace, size_t workspace_bytes, void* stream) {
  return guarded([&] {
    if (!h || !enc_bdt || !dec_bdu || !dlogits || !w_enc || !w_pred || !w_out) fail(CFM_ERR_INVALID_ARG, "null argument");
    refuse_half_training(h->dtype == DT_F32, "cfm_rnnt_joint_backward");
    if (!h->weights_set) fail(CFM_ERR_WEIGHTS, "weights not set");
    if (B <= 0 || T <= 0 || U <= 0) fail(CFM_ERR_INVALID_ARG, "B, T and U must be positive");
    const long rows = (long)B * T * U;
    if (rows > 0x7fffffffL) fail(CFM_ERR_UNSUPPORTED, "B*T*U exceeds 2^31 rows");
    if (h->H % 4 || h->H1 % 4 || h->H2 % 4) fail(CFM_ERR_UNSUPPORTED, "joint backward: hidden sizes must be multiples of 4");
    const JBWs w = jbws(h, B, T, U);
    if (!workspace || workspace_bytes < (size_t)w.total) fail(CFM_ERR_WORKSPACE, "workspace too small");
    HIP_OK(hipSetDevice(h->device));
    hipStream_t st = (hipStream_t)stream;
    char* ws = (char*)workspace;
    const int dt = h->dtype, mode = dt == DT_F32 ? CFM_COMPUTE_FP32 : CFM_COMPUTE_BF16;
    const int H = h->H, H1 = h->H1, H2 = h->H2, C = h->C;
    const Drop drop = make_drop(dropout, seed, 1);
    float* er = (float*)(ws + w.er);   // encoder rows (B*T, H1) fp32
    float* dr = (float*)(ws + w.dr);   // decoder rows (B*U, H2) fp32
    float* fp = (float*)(ws + w.fp);
    float* gp = (float*)(ws + w.gp);
    float* hid = (float*)(ws + w.hid);
    float* dh = (float*)(ws + w.dh);
    float* df = (float*)(ws + w.df);
    float* dp = (float*)(ws + w.dp);
    float* dxr = (float*)(ws + w.dx);
    char* lws = ws + w.lin;
    const size_t lws_bytes = (size_t)(w.total - w.lin);
    cfm_launch(bdl_to_rows_kernel<float>, dim3((T + 31) / 32, (H1 + 31) / 32, B), dim3(256), 0, st, enc_bdt, H1, T, er, H1);
    cfm_launch(bdl_to_rows_kernel<float>, dim3((U + 31) / 32, (H2 + 31) / 32, B), dim3(256), 0, st, dec_bdu, H2, U, dr, H2);
    // the forward's projections and hidden, recomputed (fp32 hidden = the output Linear's input)
    {
      const int H1p = (int)h->kp(H1), H2p = (int)h->kp(H2);
      char* af = (char*)dh;   // scratch: the compute-type rows live in dh until it is written
      char* ag = af + round_up((long)B * T * H1p * h->es, 256);
      if (dt == DT_F32) {
        cfm_launch(bdl_to_rows_kernel<float>, dim3((T + 31) / 32, (H1p + 31) / 32, B), dim3(256), 0, st, enc_bdt, H1, T,
                   (float*)af, H1p);
        cfm_launch(bdl_to_rows_kernel<float>, dim3((U + 31) / 32, (H2p + 31) / 32, B), dim3(256), 0, st, dec_bdu, H2, U,
                   (float*)ag, H2p);
      } else {
        cfm_launch(bdl_to_rows_kernel<bf16_t>, dim3((T + 31) / 32, (H1p + 31) / 32, B), dim3(256), 0, st, enc_bdt, H1,
                   T, (bf16_t*)af, H1p);
        cfm_launch(bdl_to_rows_kernel<bf16_t>, dim3((U + 31) / 32, (H2p + 31) / 32, B), dim3(256), 0, st, dec_bdu, H2,
                   U, (bf16_t*)ag, H2p);
      }
      gemm(dt, af, H1p, B * T, H1, h->wbuf + h->w_enc, H1p, H, epi_f32((const float*)(h->wbuf + h->b_enc), fp, H, H % 4 ? 1 : 0),
           h->zero, st);
      gemm(dt, ag, H2p, B * U, H2, h->wbuf + h->w_pred, H2p, H,
           epi_f32((const float*)(h->wbuf + h->b_pred), gp, H, H % 4 ? 1 : 0), h->zero, st);
      if (H % 8)
        fail(CFM_ERR_UNSUPPORTED, "joint backward: joint_hidden must be a multiple of 8");
      else if (joint_fast_bwd(h))
        joint_hidden<bf16_t>((const float*)fp, (const float*)gp, B, T, U, H, H, h->act, (bf16_t*)hid, drop, st);
      else
        joint_hidden<float>((const float*)fp, (const float*)gp, B, T, U, H, H, h->act, hid, drop, st);
    }
    auto lin_bwd = [&](const float* x, long M, int K, const float* wt, int N, const float* dy, float* dx, float* dw,
                       float* db) {
      const size_t need = cfm_op_linear_backward_ws_size(mode, (int)M, K, N);
      if (need > lws_bytes) fail(CFM_ERR_WORKSPACE, "joint backward: linear workspace");
      const cfm_status r = cfm_op_linear_backward(mode, x, (int)M, K, wt, N, dy, dx, dw, db, lws, lws_bytes, st);
      if (r != CFM_OK) fail(r, std::string("joint backward: ") + cfm_last_error());
    };
    // joint_net[-1]: logits = hid . W_out^T + b_out
    if (joint_fast_bwd(h)) {
      const long Cp = round_up(C, 64);
      bf16_t* a1 = (bf16_t*)(ws + w.a1);
      pack_matrix(DT_BF16, dlogits, C, (int)rows, C, false, a1, Cp, (int)rows, (int)Cp, st);
      if (dw_out || db_out) {
        const JFast js = joint_fast_splits(h, rows);
        float* part = (float*)(ws + w.part);
        wgrad_tn(a1, Cp, C, hid, H, H, true, 0, Drop{0u, 0u, 1.0f}, rows, (int)js.S, js.chunk, part, H + 4, H + 4,
                 (long)C * (H + 4), st);
        cfm_launch(joint_slab_kernel, dim3(ew_grid((long)C * (H + 4))), dim3(256), 0, st, (const float*)part, (int)js.S,
                   C, H, dw_out, db_out);
      }
      pack_matrix(DT_BF16, w_out, H, C, H, true, ws + w.wtp, Cp, (int)round_up(H, 256), (int)Cp, st);
      gemm(DT_BF16, a1, Cp, (int)rows, C, ws + w.wtp, (int)Cp, H, epi_f32(nullptr, dh, H, 0), h->zero, st);
    } else {
      lin_bwd(hid, rows, H, w_out, C, dlogits, dh, dw_out, db_out);
    }
    // dz = dh * dropout mask * act'(z); df = sum over u, dp = sum over t
    const char* tu_env = getenv("CFM_JOINT_ACT_FUSED");   // read per call: 0 = the two-pass form (A/B)
    if (!tu_env || atoi(tu_env) != 0) {
      const int ntt = (T + kActTT - 1) / kActTT;
      float* actp = (float*)(ws + w.actp);
      cfm_launch(joint_act_bwd_tu_kernel, dim3((H + 127) / 128, ntt, B), dim3(128), 0, st, fp, gp, dh, B, T, U, H, h->act,
                 drop, df, actp);
      cfm_launch(joint_act_bwd_dp_kernel, dim3(ew_grid((long)B * U * H)), dim3(256), 0, st, (const float*)actp, B, ntt, U, H,
                 dp);
    } else {
      cfm_launch(joint_act_bwd_t_kernel, dim3((H + 255) / 256, B * T), dim3(256), 0, st, fp, gp, dh, B, T, U, H, h->act,
                 drop, df);
      cfm_launch(joint_act_bwd_u_kernel, dim3((H + 255) / 256, B * U), dim3(256), 0, st, fp, gp, dh, B, T, U, H, h->act,
                 drop, dp);
    }
    // enc / pred Linears
    lin_bwd(er, (long)B * T, H1, w_enc, H, df, d_enc_bdt ? dxr : nullptr, dw_enc, db_enc);
    if (d_enc_bdt) transpose_out(dxr, B, T, H1, d_enc_bdt, st);
    lin_bwd(dr, (long)B * U, H2, w_pred, H, dp, d_dec_bdu ? dxr : nullptr, dw_pred, db_pred);
    if (d_dec_bdu) transpose_out(dxr, B, U, H2, d_dec_bdu, st);
    HIP_OK(hipGetLastError());
  });
}

}  // extern "C"
