// Cache-aware chunked streaming of the Conformer encoder (include/cfm_cache_stream.h).
//
// The definition (causal subsampling pads, attention context [left, 0], causal depthwise conv) is
// in the header; oracle/cache_aware_oracle.py restates it as a full-sequence forward.  Per chunk of
// c encoder frames (4c input frames) for B streams:
//   subsampling : the forward's conv1 kernel (symmetric pad) over [7 cached input frames | 4c new]
//                 writes the conv2 input image of 2c + 4 frames, image row a = causal conv1 frame
//                 a - 3 (rows 1, 2 = the previous chunk's last two frames, zeroed on the first
//                 chunk: conv2's causal padding); conv2 on the implicit GEMM with its symmetric pad
//                 over that image (output o = t + 1 is the causal frame t), the Linear on all c + 2
//                 rows, then rows 1 .. c kept (one 2-D copy);
//   each layer  : the eval forward's GEMMs / LayerNorms on M = B*c rows; q|k|v from a plain bias
//                 GEMM, the new k|v rows scattered into a per-layer ring of left + c frames, one wave
//                 per (stream, frame, head) attends to frames t-left .. t of that ring with the
//                 position projections of distances left .. 0 (built once per reset);
//                 GLU outputs scattered into a ring of kernel_size - 1 + c frames, the causal
//                 depthwise conv + BatchNorm + Swish reads frames t-K+1 .. t from it.
// Ring slot of frame f is f mod R, so no cache is ever shifted; frames < 0 are skipped (zero pad).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <cstdlib>
#include <memory>

#include "../../include/cfm_cache_stream.h"
#include "cfm_abi.h"
#include "cfm_common.h"
#include "cfm_encoder_impl.h"
#include "cfm_kernels.h"

namespace cfm {
namespace {

template <typename T>
__device__ __forceinline__ void load8(const T* p, float* f);
template <>
__device__ __forceinline__ void load8<bf16_t>(const bf16_t* p, float* f) {
  Vec16<bf16_t>::to_f32(*(const uint4*)p, f);
}
template <>
__device__ __forceinline__ void load8<float>(const float* p, float* f) {
  Vec16<float>::to_f32(*(const uint4*)p, f);
  Vec16<float>::to_f32(*(const uint4*)(p + 4), f + 4);
}

// ring[(b, (t0 + i) mod R)][0 .. w) <- src[(b * c + i) * lds + off + (0 .. w)], in units of E
// (16-byte vectors when every width / stride / offset allows it)
template <typename E>
__global__ __launch_bounds__(256) void cs_ring_put_kernel(const E* __restrict__ src, long lds, long off, int B, int c,
                                                          int w, E* __restrict__ ring, long ldr, int R, long t0) {
  const long n = (long)B * c * w;
  for (long e = blockIdx.x * 256L + threadIdx.x; e < n; e += (long)gridDim.x * 256) {
    const int col = (int)(e % w);
    const long row = e / w;
    const int i = (int)(row % c), b = (int)(row / c);
    ring[((long)b * R + (t0 + i) % R) * ldr + col] = src[row * lds + off + col];
  }
}

// One wave per (stream b, head h, chunk frame i), the 4 waves of a block on consecutive frames of
// one (b, h) so they share key / value / position rows in L1: frame t = t0 + i attends to frames
// max(0, t - Lc) .. t.  q|k|v rows of the chunk: qkv (B*c, 3*H*dkp); keys | values of frame j in
// ring row (b, j mod R) = [k (H*dkp) | v (H*dkp)]; P row r = linear_pos(pe(position Lc - r)).
// score = ((q + u) . k_j + (q + v) . p(t - j)) / sqrt(dk)  (multi_head_attention.py:196-201 with
// the rel_shift reduced to the distance t - j), softmax over the window, then P . V.
// DKP = dkp (compile time, multiple of 16): lanes own keys for the scores (rows read as 16-byte
// vectors, fully unrolled), then head dims lane and lane + 64 for P . V (8 keys in flight).
template <typename T, int DKP>
__global__ __launch_bounds__(256) void cs_attn_kernel(const T* __restrict__ qkv, long ldq, const T* __restrict__ kv,
                                                      long ldkv, int R, const T* __restrict__ P, long ldp,
                                                      const float* __restrict__ uv, int B, int c, int H, int dk,
                                                      int Lc, long t0, float scale, T* __restrict__ out, long ldo) {
  extern __shared__ float sm[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int per = 2 * DKP + ((Lc + 4) & ~3);
  float* qu = sm + w * per;
  float* qv = qu + DKP;
  float* pr = qv + DKP;
  const long nq = (long)B * H * c;
  const long qid = blockIdx.x * 4L + w;
  const bool active = qid < nq;
  const long q = active ? qid : nq - 1;
  const int i = (int)(q % c);
  const long bh = q / c;
  const int h = (int)(bh % H), b = (int)(bh / H);
  const T* qrow = qkv + ((long)b * c + i) * ldq + (long)h * DKP;
  for (int k = lane; k < DKP; k += 64) {
    const float v = ld_f(qrow + k);
    qu[k] = v + uv[h * DKP + k];
    qv[k] = v + uv[(H + h) * DKP + k];
  }
  __syncthreads();
  const long t = t0 + i;
  const long jlo = t - Lc > 0 ? t - Lc : 0;
  const int nk = (int)(t - jlo + 1);
  const int slot0 = (int)(jlo % R);
  const T* kb = kv + (long)b * R * ldkv + (long)h * DKP;
  float mx = -INFINITY;
  for (int s = lane; s < nk; s += 64) {
    int slot = slot0 + s;
    if (slot >= R) slot -= R;
    const T* kr = kb + (long)slot * ldkv;
    const T* pp = P + (long)(Lc - nk + 1 + s) * ldp + (long)h * DKP;   // distance t - j = nk - 1 - s
    float acc = 0.0f;
#pragma unroll
    for (int k = 0; k < DKP; k += 8) {
      float kf[8], pf[8];
      load8<T>(kr + k, kf);
      load8<T>(pp + k, pf);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc += qu[k + e] * kf[e] + qv[k + e] * pf[e];
    }
    acc *= scale;
    pr[s] = acc;
    mx = fmaxf(mx, acc);
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
  float sum = 0.0f;
  for (int s = lane; s < nk; s += 64) {
    const float e = __expf(pr[s] - mx);
    pr[s] = e;
    sum += e;
  }
  sum = wave_sum(sum);
  __syncthreads();
  const float inv = 1.0f / sum;
  const T* vb = kb + (long)H * DKP;
  const int k0 = lane, k1 = lane + 64;
  const bool ok0 = k0 < dk, ok1 = DKP > 64 && k1 < dk;
  float o0 = 0.0f, o1 = 0.0f;
  for (int s0 = 0; s0 < nk; s0 += 8) {
    float pv[8], a0[8], a1[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int s = min(s0 + u, nk - 1);
      int slot = slot0 + s;
      if (slot >= R) slot -= R;
      const T* vr = vb + (long)slot * ldkv;
      pv[u] = s0 + u < nk ? pr[s] : 0.0f;
      a0[u] = ok0 ? ld_f(vr + k0) : 0.0f;
      a1[u] = ok1 ? ld_f(vr + k1) : 0.0f;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      o0 += pv[u] * a0[u];
      o1 += pv[u] * a1[u];
    }
  }
  T* orow = out + ((long)b * c + i) * ldo + (long)h * dk;
  if (active && ok0) st_f(orow + k0, o0 * inv);
  if (active && ok1) st_f(orow + k1, o1 * inv);
}

// One block per (stream b, head h) when the window fits LDS: the keys / values of frames
// max(0, t0 - Lc) .. t0 + c - 1 and the Lc + 1 position rows are staged once in LDS (compute type,
// rows padded by 16 bytes against bank conflicts); wave w then serves chunk frames w, w + 4, ...:
// lanes over keys for the scores, softmax by wave reductions, lanes over head dims for P . V.
// Same arithmetic and summation order per query as cs_attn_kernel.
template <typename T, int DKP>
__global__ __launch_bounds__(256) void cs_attn_block_kernel(const T* __restrict__ qkv, long ldq,
                                                            const T* __restrict__ kv, long ldkv, int R,
                                                            const T* __restrict__ P, long ldp,
                                                            const float* __restrict__ uv, int B, int c, int H, int dk,
                                                            int Lc, long t0, float scale, T* __restrict__ out,
                                                            long ldo) {
  constexpr int RS = DKP + 16 / (int)sizeof(T);       // LDS row stride (elements)
  constexpr int VPR = DKP * (int)sizeof(T) / 16;      // 16-byte vectors per row
  extern __shared__ __align__(16) unsigned char smem[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int b = blockIdx.x / H, h = blockIdx.x - (blockIdx.x / H) * H;
  const long jmin = t0 - Lc > 0 ? t0 - Lc : 0;
  const int nw = (int)(t0 + c - jmin);                // window frames
  T* Ks = (T*)smem;
  T* Vs = Ks + (long)nw * RS;
  T* Ps = Vs + (long)nw * RS;
  float* wsm = (float*)(Ps + (long)(Lc + 1) * RS);
  const int per = 2 * DKP + ((Lc + 4) & ~3);
  float* qu = wsm + w * per;
  float* qv = qu + DKP;
  float* pr = qv + DKP;
  // stage K, V (ring) and P
  const int slot_min = (int)(jmin % R);
  for (int e = threadIdx.x; e < nw * VPR * 2; e += 256) {
    const int half = e / (nw * VPR), r = (e - half * nw * VPR) / VPR, v = e % VPR;
    int slot = slot_min + r;
    if (slot >= R) slot -= R;
    const T* src = kv + ((long)b * R + slot) * ldkv + (long)half * ldkv / 2 + (long)h * DKP;
    *(uint4*)((half ? Vs : Ks) + (long)r * RS + v * (16 / sizeof(T))) = ((const uint4*)src)[v];
  }
  for (int e = threadIdx.x; e < (Lc + 1) * VPR; e += 256) {
    const int r = e / VPR, v = e - r * VPR;
    *(uint4*)(Ps + (long)r * RS + v * (16 / sizeof(T))) = ((const uint4*)(P + (long)r * ldp + (long)h * DKP))[v];
  }
  __syncthreads();
  for (int i = w; i < c; i += 4) {
    const T* qrow = qkv + ((long)b * c + i) * ldq + (long)h * DKP;
    for (int k = lane; k < DKP; k += 64) {
      const float v = ld_f(qrow + k);
      qu[k] = v + uv[h * DKP + k];
      qv[k] = v + uv[(H + h) * DKP + k];
    }
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    const long t = t0 + i;
    const long jlo = t - Lc > 0 ? t - Lc : 0;
    const int nk = (int)(t - jlo + 1);
    const int r0 = (int)(jlo - jmin);                   // window row of key s = 0
    float mx = -INFINITY;
    for (int s = lane; s < nk; s += 64) {
      const T* kr = Ks + (long)(r0 + s) * RS;
      const T* pp = Ps + (long)(Lc - nk + 1 + s) * RS;
      float acc = 0.0f;
#pragma unroll
      for (int k = 0; k < DKP; k += 8) {
        float kf[8], pf[8];
        load8<T>(kr + k, kf);
        load8<T>(pp + k, pf);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc += qu[k + e] * kf[e] + qv[k + e] * pf[e];
      }
      acc *= scale;
      pr[s] = acc;
      mx = fmaxf(mx, acc);
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    float sum = 0.0f;
    for (int s = lane; s < nk; s += 64) {
      const float e = __expf(pr[s] - mx);
      pr[s] = e;
      sum += e;
    }
    sum = wave_sum(sum);
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    const float inv = 1.0f / sum;
    const int k0 = lane, k1 = lane + 64;
    const bool ok0 = k0 < dk, ok1 = DKP > 64 && k1 < dk;
    float o0 = 0.0f, o1 = 0.0f;
    for (int s = 0; s < nk; ++s) {
      const T* vr = Vs + (long)(r0 + s) * RS;
      const float p = pr[s];
      if (ok0) o0 += p * ld_f(vr + k0);
      if (ok1) o1 += p * ld_f(vr + k1);
    }
    T* orow = out + ((long)b * c + i) * ldo + (long)h * dk;
    if (ok0) st_f(orow + k0, o0 * inv);
    if (ok1) st_f(orow + k1, o1 * inv);
    __builtin_amdgcn_wave_barrier();                    // qu / qv / pr reused by the next frame
  }
}

// Causal depthwise conv, K = KK taps, TT consecutive frames per thread from a register window of
// KK - 1 + TT ring frames (weights in registers); BatchNorm (running statistics) + Swish -> out, or
// the pre-norm value (fp32) for the LayerNorm variant.  Threads: (b, frame group, channel), channel
// fastest so every ring / weight read is coalesced.
template <typename T, int KK, int TT>
__global__ __launch_bounds__(256) void cs_dwconv_win_kernel(const T* __restrict__ ring, int R, int B, int c, int d,
                                                            long t0, const float* __restrict__ w,
                                                            const float* __restrict__ bias,
                                                            const float* __restrict__ bn_mean,
                                                            const float* __restrict__ bn_inv,
                                                            const float* __restrict__ bn_w,
                                                            const float* __restrict__ bn_b, T* __restrict__ out,
                                                            float* __restrict__ pre) {
  const int ng = (c + TT - 1) / TT;
  const long n = (long)B * ng * d;
  const long e = blockIdx.x * 256L + threadIdx.x;
  if (e >= n) return;
  const int ch = (int)(e % d);
  const long r = e / d;
  const int g = (int)(r % ng), b = (int)(r / ng);
  const int i0 = g * TT;
  float wr[KK];
#pragma unroll
  for (int k = 0; k < KK; ++k) wr[k] = w[(long)k * d + ch];
  float win[KK - 1 + TT];
  const long f0 = t0 + i0 - (KK - 1);                 // frame of win[0]
  const long base = (long)b * R;
#pragma unroll
  for (int u = 0; u < KK - 1 + TT; ++u) {
    const long f = f0 + u;
    const bool ok = f >= 0 && i0 - (KK - 1) + u < c;   // frames < 0 are the zero padding
    const float v = ld_f(ring + (base + (ok ? f : 0) % R) * d + ch);
    win[u] = ok ? v : 0.0f;
  }
  const float bb = bias[ch];
  float mu = 0.0f, iv = 1.0f, gw = 1.0f, gb = 0.0f;
  if (!pre) { mu = bn_mean[ch]; iv = bn_inv[ch]; gw = bn_w[ch]; gb = bn_b[ch]; }
#pragma unroll
  for (int tt = 0; tt < TT; ++tt) {
    const int i = i0 + tt;
    if (i >= c) break;
    float acc = bb;
#pragma unroll
    for (int k = 0; k < KK; ++k) acc += wr[k] * win[tt + k];
    const long row = (long)b * c + i;
    if (pre) pre[row * d + ch] = acc;
    else st_f(out + row * d + ch, swishf((acc - mu) * iv * gw + gb));
  }
}

// Causal depthwise conv (kernel K, time pad (K-1, 0)) over the GLU ring + BatchNorm (running
// statistics) + Swish -> out (compute type), or the pre-norm value (fp32) for the LayerNorm variant.
template <typename T>
__global__ __launch_bounds__(256) void cs_dwconv_kernel(const T* __restrict__ ring, int R, int B, int c, int d, int K,
                                                        long t0, const float* __restrict__ w,
                                                        const float* __restrict__ bias, const float* __restrict__ bn_mean,
                                                        const float* __restrict__ bn_inv, const float* __restrict__ bn_w,
                                                        const float* __restrict__ bn_b, T* __restrict__ out,
                                                        float* __restrict__ pre) {
  const long n = (long)B * c * d;
  for (long e = blockIdx.x * 256L + threadIdx.x; e < n; e += (long)gridDim.x * 256) {
    const int ch = (int)(e % d);
    const long row = e / d;
    const int i = (int)(row % c), b = (int)(row / c);
    const long t = t0 + i;
    float acc = bias[ch];
    for (int k = 0; k < K; ++k) {
      const long f = t - (K - 1) + k;
      if (f >= 0) acc += w[(long)k * d + ch] * ld_f(ring + ((long)b * R + f % R) * d + ch);
    }
    if (pre) {
      pre[row * d + ch] = acc;
    } else {
      const float y = (acc - bn_mean[ch]) * bn_inv[ch] * bn_w[ch] + bn_b[ch];
      st_f(out + row * d + ch, swishf(y));
    }
  }
}

unsigned ew_blocks(long n) { return (unsigned)std::max<long>(1, std::min<long>((n + 255) / 256, 8192)); }

GemmEpi mk_epi(int mode, const float* bias, float alpha = 1.0f) {
  GemmEpi e;
  std::memset(&e, 0, sizeof(e));
  e.mode = mode;
  e.bias = bias;
  e.alpha = alpha;
  return e;
}

}  // namespace
}  // namespace cfm

using namespace cfm;

struct cfm_cache_stream {
  cfm_encoder* h = nullptr;
  int B = 0, c = 0, Lc = 0;
  int R = 0, R2 = 0;            // ring frames: keys/values (Lc + c), GLU outputs (K - 1 + c)
  long t0 = 0;                  // encoder frames emitted
  char* state = nullptr;        // one device allocation
  size_t state_bytes = 0;
  long melc = 0, P = 0;            // offsets into state: last 7 input frames (B, F, 7) fp32, positions
  std::vector<long> kv, gr;        // per layer
  // workspace layout (offsets)
  long wMel, wX1, wX2, wXs, wX, wHn, wU, wQ, wO, wG, wS, wPN, wY, wtotal;
};

namespace {

void ws_plan(cfm_cache_stream* s) {
  const cfm_encoder* h = s->h;
  const int B = s->B, c = s->c, es = h->es, d = h->d;
  const long M = (long)B * c;
  long off = 0;
  auto take = [&](long bytes) { const long o = off; off += round_up(bytes, 256); return o; };
  s->wMel = take((long)B * h->F * (4 * c + 7) * 4);
  s->wX1 = take((long)B * (2 * c + 4) * h->F1 * h->C * es);
  s->wX2 = take((long)B * (c + 2) * h->F2 * h->C * es);
  s->wXs = take((long)B * (c + 2) * d * 4);
  s->wX = take(M * d * 4);
  s->wHn = take(M * d * es);
  s->wU = take(M * h->dff * es);
  s->wQ = take(M * 3L * h->H * h->dkp * es);
  s->wO = take(M * d * es);
  s->wG = take(M * d * es);
  s->wS = take(M * d * es);
  s->wPN = h->cfg.conv_norm_type == 1 ? take(M * d * 4) : -1;
  s->wY = h->has_out_proj ? take(M * h->dout * 4) : -1;
  s->wtotal = round_up(off, 256);
}

void build_pos(cfm_cache_stream* s, hipStream_t st) {
  // P = linear_pos(pe) of every layer at once for positions Lc .. 0 (pe row max_len - 1 - p)
  cfm_encoder* h = s->h;
  if (h->L == 0) return;
  GemmEpi e = mk_epi(EPI_STORE, nullptr);
  e.C = s->state + s->P;
  e.ldc = (long)h->L * h->H * h->dkp;
  const char* pe = h->pe + (long)(h->max_len - 1 - s->Lc) * h->d * h->es;
  gemm(h->dtype, pe, h->d, s->Lc + 1, h->d, h->wbuf + h->pos_w, (int)h->kpad(h->d), (int)e.ldc, e, h->zero_page, st);
}

void step(cfm_cache_stream* s, const float* x, float* y, char* ws, hipStream_t st) {
  cfm_encoder* h = s->h;
  const int dt = h->dtype, es = h->es, d = h->d, H = h->H, dkp = h->dkp, B = s->B, c = s->c, L = h->L;
  const int M = B * c;
  const long t0 = s->t0;
  auto W = [&](long off) { return (const void*)(h->wbuf + off); };
  auto Wf = [&](long off) { return (const float*)(h->wbuf + off); };
  char* S = s->state;
  const bool f32 = dt == DT_F32;
  // ---- subsampling ----
  {
    // [7 cached input frames | 4c new] -> conv1 (T = 4c + 7, symmetric pad) -> image rows 0 .. 2c+3
    float* mel = (float*)(ws + s->wMel);
    const size_t TM = (size_t)4 * c + 7;
    HIP_OK(hipMemcpy2DAsync(mel, TM * 4, S + s->melc, 7 * 4, 7 * 4, (size_t)B * h->F, hipMemcpyDeviceToDevice, st));
    HIP_OK(hipMemcpy2DAsync(mel + 7, TM * 4, x, (size_t)4 * c * 4, (size_t)4 * c * 4, (size_t)B * h->F,
                            hipMemcpyDeviceToDevice, st));
    HIP_OK(hipMemcpy2DAsync(S + s->melc, 7 * 4, mel + 4 * c, TM * 4, 7 * 4, (size_t)B * h->F, hipMemcpyDeviceToDevice,
                            st));
    conv1_subsample(dt, mel, B, h->F, (int)TM, Wf(h->conv1_w), Wf(h->conv1_b), h->C, ws + s->wX1, st);
    const size_t fr = (size_t)h->F1 * h->C * es;
    if (t0 == 0)   // conv1 frames -2, -1 are conv2's causal zero padding, not conv1(zero input)
      HIP_OK(hipMemset2DAsync(ws + s->wX1 + fr, (2 * c + 4) * fr, 0, 2 * fr, B, st));
  }
  {
    ConvGeom g{ws + s->wX1, 2 * c + 4, h->F1, c + 2, h->F2, h->C};
    GemmEpi e = mk_epi(EPI_RELU, Wf(h->conv2_b));
    e.C = ws + s->wX2;
    e.ldc = h->C;
    gemm_conv(dt, g, B, W(h->conv2_w), (int)h->kpad(9 * h->C), h->C, e, h->zero_page, st);
  }
  float* X = (float*)(ws + s->wX);
  {
    const float xs = h->cfg.xscaling ? (float)std::sqrt((double)d) : 1.0f;
    GemmEpi e = mk_epi(EPI_SCALE_F32, Wf(h->sub_b), xs);
    e.X = (float*)(ws + s->wXs);
    e.ldx = d;
    gemm(dt, ws + s->wX2, (long)h->F2 * h->C, B * (c + 2), h->F2 * h->C, W(h->sub_w), (int)h->kpad(h->F2 * h->C), d,
         e, h->zero_page, st);
    HIP_OK(hipMemcpy2DAsync(X, (size_t)c * d * 4, ws + s->wXs + (size_t)d * 4, (size_t)(c + 2) * d * 4,
                            (size_t)c * d * 4, B, hipMemcpyDeviceToDevice, st));
  }
  void* Hn = ws + s->wHn;
  const long ldq = 3L * H * dkp, ldkv = 2L * H * dkp, ldp = (long)L * H * dkp;
  const float scale = (float)(1.0 / std::sqrt((double)h->dk));
  // ring rows (b, (t0 + i) mod R) <- w elements of chunk row b * c + i at column off
  auto ring_put = [&](const char* src, long lds, long off, int w, char* ring, long ldr, int R) {
    const bool vec = (lds * es) % 16 == 0 && (off * es) % 16 == 0 && (w * es) % 16 == 0 && (ldr * es) % 16 == 0;
    if (vec) {
      const int k = 16 / es;
      const long n = (long)M * (w / k);
      cfm_launch(cs_ring_put_kernel<uint4>, dim3(ew_blocks(n)), dim3(256), 0, st, (const uint4*)src, lds / k, off / k,
                 B, c, w / k, (uint4*)ring, ldr / k, R, t0);
    } else if (f32) {
      cfm_launch(cs_ring_put_kernel<float>, dim3(ew_blocks((long)M * w)), dim3(256), 0, st, (const float*)src, lds,
                 off, B, c, w, (float*)ring, ldr, R, t0);
    } else {
      cfm_launch(cs_ring_put_kernel<bf16_t>, dim3(ew_blocks((long)M * w)), dim3(256), 0, st, (const bf16_t*)src, lds,
                 off, B, c, w, (bf16_t*)ring, ldr, R, t0);
    }
  };
  auto attention = [&](const char* q, long ldq_, const char* kv, long ldkv_, const char* Pl, long ldp_,
                       const float* uv, float sc, char* o) {
    const int nw = 4;
    const size_t lds = (size_t)nw * (2 * dkp + ((s->Lc + 4) & ~3)) * sizeof(float);
    const unsigned blocks = (unsigned)(((long)M * H + nw - 1) / nw);
    // block kernel when K, V and P of one (b, h) fit LDS next to the per-wave scratch
    const long jmin = t0 - s->Lc > 0 ? t0 - s->Lc : 0;
    const long nwin = t0 + c - jmin;
    const size_t rs = (size_t)(dkp + 16 / es) * es;
    const size_t blds = (size_t)(2 * nwin + s->Lc + 1) * rs + lds;
    static const bool force_wave = [] { const char* e = getenv("CFM_CS_ATTN_WAVE"); return e && atoi(e) != 0; }();
    const bool block = blds <= 160 * 1024 && !force_wave;   // CFM_CS_ATTN_WAVE=1: per-wave kernel (tests)
    auto go = [&](auto kern, auto bkern, auto tag) {
      using T = decltype(tag);
      if (block) {
        if (blds > 64 * 1024) (void)hipFuncSetAttribute((const void*)bkern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)blds);
        cfm_launch(bkern, dim3((unsigned)(B * H)), dim3(256), (uint32_t)blds, st, (const T*)q, ldq_, (const T*)kv,
                   ldkv_, s->R, (const T*)Pl, ldp_, uv, B, c, H, h->dk, s->Lc, t0, sc, (T*)o, (long)d);
      } else {
        cfm_launch(kern, dim3(blocks), dim3(256), (uint32_t)lds, st, (const T*)q, ldq_, (const T*)kv, ldkv_, s->R,
                   (const T*)Pl, ldp_, uv, B, c, H, h->dk, s->Lc, t0, sc, (T*)o, (long)d);
      }
    };
#define CS_ATTN(DK)                                                                                   \
  case DK / 16:                                                                                       \
    if (f32) go(cs_attn_kernel<float, DK>, cs_attn_block_kernel<float, DK>, 0.0f);                    \
    else go(cs_attn_kernel<bf16_t, DK>, cs_attn_block_kernel<bf16_t, DK>, (bf16_t)0);                 \
    break;
    switch (dkp / 16) {
      CS_ATTN(16) CS_ATTN(32) CS_ATTN(48) CS_ATTN(64) CS_ATTN(80) CS_ATTN(96) CS_ATTN(112) CS_ATTN(128)
      default: fail(CFM_ERR_INVALID_ARG, "cache-aware streaming supports head widths up to 128");
    }
#undef CS_ATTN
  };
  auto dwconv = [&](const char* ring, const LayerW& Lw, bool bn, char* out, float* pre) {
    const float* mean = bn ? Wf(Lw.bn_mean) : nullptr;
    const float* inv = bn ? Wf(Lw.bn_inv) : nullptr;
    if (h->K == 31) {
      constexpr int TT = 8;
      const long n = (long)B * ((c + TT - 1) / TT) * d;
      const unsigned blocks = (unsigned)((n + 255) / 256);
      if (f32)
        cfm_launch(cs_dwconv_win_kernel<float, 31, TT>, dim3(blocks), dim3(256), 0, st, (const float*)ring, s->R2, B,
                   c, d, t0, Wf(Lw.dw_w), Wf(Lw.dw_b), mean, inv, Wf(Lw.bn_w), Wf(Lw.bn_b), (float*)out, pre);
      else
        cfm_launch(cs_dwconv_win_kernel<bf16_t, 31, TT>, dim3(blocks), dim3(256), 0, st, (const bf16_t*)ring, s->R2,
                   B, c, d, t0, Wf(Lw.dw_w), Wf(Lw.dw_b), mean, inv, Wf(Lw.bn_w), Wf(Lw.bn_b), (bf16_t*)out, pre);
      return;
    }
    const long n = (long)M * d;
    if (f32)
      cfm_launch(cs_dwconv_kernel<float>, dim3(ew_blocks(n)), dim3(256), 0, st, (const float*)ring, s->R2, B, c, d,
                 h->K, t0, Wf(Lw.dw_w), Wf(Lw.dw_b), mean, inv, Wf(Lw.bn_w), Wf(Lw.bn_b), (float*)out, pre);
    else
      cfm_launch(cs_dwconv_kernel<bf16_t>, dim3(ew_blocks(n)), dim3(256), 0, st, (const bf16_t*)ring, s->R2, B, c,
                 d, h->K, t0, Wf(Lw.dw_w), Wf(Lw.dw_b), mean, inv, Wf(Lw.bn_w), Wf(Lw.bn_b), (bf16_t*)out, pre);
  };
  if (L > 0)
    layernorm(dt, X, M, d, Wf(h->layers[0].ln_w[0]), Wf(h->layers[0].ln_b[0]), nullptr, nullptr, nullptr, Hn, 0, st);
  for (int l = 0; l < L; ++l) {
    const LayerW& Lw = h->layers[l];
    // FFN1
    {
      GemmEpi e = mk_epi(EPI_SWISH, Wf(Lw.ff1_b1));
      e.C = ws + s->wU; e.ldc = h->dff;
      gemm(dt, Hn, d, M, d, W(Lw.ff1_w1), (int)h->kpad(d), h->dff, e, h->zero_page, st);
      GemmEpi r = mk_epi(EPI_RESID, Wf(Lw.ff1_b2), 0.5f);
      r.X = X; r.ldx = d;
      gemm(dt, ws + s->wU, h->dff, M, h->dff, W(Lw.ff1_w2), (int)h->kpad(h->dff), d, r, h->zero_page, st);
    }
    // MHSA with the key / value ring
    layernorm(dt, X, M, d, Wf(Lw.ln_w[1]), Wf(Lw.ln_b[1]), nullptr, nullptr, nullptr, Hn, 0, st);
    {
      GemmEpi e = mk_epi(EPI_STORE, Wf(Lw.qkv_b));
      e.C = ws + s->wQ; e.ldc = ldq;
      gemm(dt, Hn, d, M, d, W(Lw.qkv_w), (int)h->kpad(d), 3 * H * dkp, e, h->zero_page, st);
      ring_put(ws + s->wQ, ldq, H * dkp, (int)ldkv, S + s->kv[l], ldkv, s->R);
      attention(ws + s->wQ, ldq, S + s->kv[l], ldkv, S + s->P + (long)l * H * dkp * es, ldp, Wf(Lw.uv), scale,
                ws + s->wO);
      GemmEpi r = mk_epi(EPI_RESID, Wf(Lw.out_b), 1.0f);
      r.X = X; r.ldx = d;
      gemm(dt, ws + s->wO, d, M, d, W(Lw.out_w), (int)h->kpad(d), d, r, h->zero_page, st);
    }
    // convolution module with the GLU ring
    layernorm(dt, X, M, d, Wf(Lw.ln_w[2]), Wf(Lw.ln_b[2]), nullptr, nullptr, nullptr, Hn, 0, st);
    {
      GemmEpi e = mk_epi(EPI_GLU_MASK, Wf(Lw.pw1_b));
      e.C = ws + s->wG; e.ldc = d; e.lens = nullptr; e.Tp = c;
      gemm(dt, Hn, d, M, d, W(Lw.pw1_w), (int)h->kpad(d), d, e, h->zero_page, st);
      const bool bn = h->cfg.conv_norm_type == 0;
      float* pre = bn ? nullptr : (float*)(ws + s->wPN);
      ring_put(ws + s->wG, d, 0, d, S + s->gr[l], d, s->R2);
      dwconv(S + s->gr[l], Lw, bn, ws + s->wS, pre);
      if (!bn) layernorm(dt, pre, M, d, Wf(Lw.bn_w), Wf(Lw.bn_b), nullptr, nullptr, nullptr, ws + s->wS, 1, st);
      GemmEpi r = mk_epi(EPI_RESID, Wf(Lw.pw2_b), 1.0f);
      r.X = X; r.ldx = d;
      gemm(dt, ws + s->wS, d, M, d, W(Lw.pw2_w), (int)h->kpad(d), d, r, h->zero_page, st);
    }
    // FFN2
    layernorm(dt, X, M, d, Wf(Lw.ln_w[3]), Wf(Lw.ln_b[3]), nullptr, nullptr, nullptr, Hn, 0, st);
    {
      GemmEpi e = mk_epi(EPI_SWISH, Wf(Lw.ff2_b1));
      e.C = ws + s->wU; e.ldc = h->dff;
      gemm(dt, Hn, d, M, d, W(Lw.ff2_w1), (int)h->kpad(d), h->dff, e, h->zero_page, st);
      GemmEpi r = mk_epi(EPI_RESID, Wf(Lw.ff2_b2), 0.5f);
      r.X = X; r.ldx = d;
      gemm(dt, ws + s->wU, h->dff, M, h->dff, W(Lw.ff2_w2), (int)h->kpad(h->dff), d, r, h->zero_page, st);
    }
    // norm_out, fused with the next layer's first LayerNorm
    const bool next = l + 1 < L;
    layernorm(dt, X, M, d, Wf(Lw.ln_w[4]), Wf(Lw.ln_b[4]), X, next ? Wf(h->layers[l + 1].ln_w[0]) : nullptr,
              next ? Wf(h->layers[l + 1].ln_b[0]) : nullptr, (next || h->has_out_proj) ? Hn : nullptr, 0, st);
  }
  const float* fin = X;
  if (h->has_out_proj) {
    if (L == 0) convert_f32(dt, X, Hn, (long)M * d, st);
    GemmEpi e = mk_epi(EPI_SCALE_F32, Wf(h->outp_b), 1.0f);
    float* Y = (float*)(ws + s->wY);
    e.X = Y; e.ldx = h->dout;
    gemm(dt, Hn, d, M, d, W(h->outp_w), (int)h->kpad(d), h->dout, e, h->zero_page, st);
    fin = Y;
  }
  transpose_out(fin, B, c, h->dout, y, st);
  HIP_OK(hipGetLastError());
  s->t0 += c;
}

}  // namespace

extern "C" {

cfm_status cfm_cache_stream_create(cfm_encoder* enc, int batch, int chunk, int left_context, cfm_cache_stream** out) {
  return guarded([&] {
    if (!enc || !out) fail(CFM_ERR_INVALID_ARG, "null argument");
    *out = nullptr;
    if (batch < 1 || chunk < 1) fail(CFM_ERR_INVALID_ARG, "batch and chunk must be >= 1");
    if (left_context < 1 || left_context >= enc->max_len || left_context > 2048)
      fail(CFM_ERR_INVALID_ARG, "left_context must be in [1, min(pos_emb_max_len - 1, 2048)]");
    if (enc->abs_pos) fail(CFM_ERR_UNSUPPORTED, "cache-aware streaming is implemented for rel_pos encoders");
    if (enc->C % 8 != 0) fail(CFM_ERR_INVALID_ARG, "subsampling channels must be a multiple of 8");
    if (enc->dkp % 16 != 0 || enc->dkp > 128) fail(CFM_ERR_INVALID_ARG, "head width must be at most 128");
    std::unique_ptr<cfm_cache_stream> s(new cfm_cache_stream);
    s->h = enc;
    s->B = batch;
    s->c = chunk;
    s->Lc = left_context;
    s->R = left_context + chunk;
    s->R2 = std::max(enc->K - 1, 0) + chunk;
    const int es = enc->es, L = enc->L;
    long off = 0;
    auto take = [&](long bytes) { const long o = off; off += round_up(bytes, 256); return o; };
    s->melc = take((long)batch * enc->F * 7 * 4);
    s->P = take((long)(left_context + 1) * L * enc->H * enc->dkp * es + 64);
    for (int l = 0; l < L; ++l) {
      s->kv.push_back(take((long)batch * s->R * 2 * enc->H * enc->dkp * es));
      s->gr.push_back(take((long)batch * s->R2 * enc->d * es));
    }
    s->state_bytes = (size_t)round_up(off, 256);
    int prev = 0;
    HIP_OK(hipGetDevice(&prev));
    HIP_OK(hipSetDevice(enc->device));
    const hipError_t e = hipMalloc(&s->state, s->state_bytes);
    (void)hipSetDevice(prev);
    if (e != hipSuccess) fail(CFM_ERR_HIP, std::string("hipMalloc: ") + hipGetErrorString(e));
    ws_plan(s.get());
    *out = s.release();
  });
}

cfm_status cfm_cache_stream_destroy(cfm_cache_stream* s) {
  return guarded([&] {
    if (!s) return;
    if (s->state) (void)hipFree(s->state);
    delete s;
  });
}

cfm_status cfm_cache_stream_reset(cfm_cache_stream* s, void* stream) {
  return guarded([&] {
    if (!s) fail(CFM_ERR_INVALID_ARG, "null argument");
    if (!s->h->weights_set) fail(CFM_ERR_WEIGHTS, "weights not set");
    hipStream_t st = (hipStream_t)stream;
    HIP_OK(hipMemsetAsync(s->state, 0, s->state_bytes, st));
    build_pos(s, st);
    HIP_OK(hipGetLastError());
    s->t0 = 0;
  });
}

size_t cfm_cache_stream_workspace_size(const cfm_cache_stream* s) { return s ? (size_t)s->wtotal : 0; }

cfm_status cfm_cache_stream_step(cfm_cache_stream* s, const float* x_bft, float* y_bdt, void* workspace,
                                 size_t workspace_bytes, void* stream) {
  return guarded([&] {
    if (!s || !x_bft || !y_bdt) fail(CFM_ERR_INVALID_ARG, "null argument");
    if (!s->h->weights_set) fail(CFM_ERR_WEIGHTS, "weights not set");
    if (!workspace || workspace_bytes < (size_t)s->wtotal) fail(CFM_ERR_WORKSPACE, "workspace too small");
    step(s, x_bft, y_bdt, (char*)workspace, (hipStream_t)stream);
  });
}

int64_t cfm_cache_stream_position(const cfm_cache_stream* s) { return s ? (int64_t)s->t0 : -1; }

}  // extern "C"
