// RNN-T loss: warp-transducer semantics of the reference's numba GPU loss
// (gpu_rnnt.py:122-238, gpu_rnnt_kernel.py:66-399), contract in include/cfm_rnnt_loss.h.
//
//   rnnt_denom_kernel  one wave per lattice node (b, t, u): max + sum of exp over the V logits ->
//                      denom = -logsumexp, plus the two log-probabilities the lattice needs
//                      (blank, and the next label) in compact (B, T, U) arrays.  Reads acts once.
//   rnnt_lattice_kernel one block per (utterance, direction): the alpha (forward) or beta
//                      (backward) recursion swept by anti-diagonals, one thread per label position
//                      u; the recursion's own neighbour comes from the previous diagonal through LDS,
//                      its own previous value stays in a register.  Writes the lattices (for the
//                      gradient) and the log-likelihood / costs.
//   rnnt_grad_kernel   one wave per (b, t, u): the gradient w.r.t. the raw logits with FastEmit and
//                      clamp (gpu_rnnt_kernel.py:262-399).  Reads acts once more, writes grads once.
// All arithmetic is fp32 like the reference kernels.  HBM-bound: ~3 passes over the (B,T,U,V) tensor.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <string>

#include "../../include/cfm_rnnt_loss.h"
#include "cfm_abi.h"

using namespace cfm;

namespace {

constexpr float kNegInf = -INFINITY;

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float wave_sumf(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
// rnnt_helper.log_sum_exp (rnnt_helper.py:42-52)
__device__ __forceinline__ float log_sum_exp(float a, float b) {
  if (a == kNegInf) return b;
  if (b == kNegInf) return a;
  return a > b ? log1pf(expf(b - a)) + a : log1pf(expf(a - b)) + b;
}

struct Dims {
  int B, T, U, V, blank, ld;
};

__device__ __forceinline__ void lens(const Dims& d, const int32_t* act_lens, const int32_t* label_lens, int b, int& Tb,
                                     int& Ub) {
  Tb = min(max(act_lens[b], 0), d.T);
  Ub = min(max(label_lens[b], 0) + 1, d.U);
}
__device__ __forceinline__ int label_at(const Dims& d, const int32_t* labels, int b, int u) {
  return min(max(labels[(long)b * d.ld + u], 0), d.V - 1);
}

constexpr int kDenomRegs = 32;   // V <= 2048: single read of the logits row
// KR: registers per lane for the row (V <= 64 KR; 0 = two passes for V > 2048). The loads are unconditional
// (clamped column, the value selected afterwards): a load under a per-lane condition is branched around and
// waited for alone. Summing KR < 32 terms drops only trailing zero terms, so the values are unchanged.
template <int KR>
__global__ __launch_bounds__(256) void rnnt_denom_kernel(const float* __restrict__ acts, const int32_t* __restrict__ labels,
                                                         const int32_t* __restrict__ act_lens,
                                                         const int32_t* __restrict__ label_lens, Dims d,
                                                         float* __restrict__ denom, float* __restrict__ lpb,
                                                         float* __restrict__ lpl) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= (long)d.B * d.T * d.U) return;
  const int u = (int)(row % d.U);
  const long bt = row / d.U;
  const int t = (int)(bt % d.T), b = (int)(bt / d.T);
  int Tb, Ub;
  lens(d, act_lens, label_lens, b, Tb, Ub);
  if (t >= Tb || u >= Ub) return;
  const float* a = acts + row * d.V;
  float m = kNegInf, s = 0.0f;
  if constexpr (KR > 0) {
    // one pass over HBM: the row's logits stay in registers for the max and the exp-sum
    float r[KR];
#pragma unroll
    for (int k = 0; k < KR; ++k) r[k] = a[min(lane + 64 * k, d.V - 1)];
#pragma unroll
    for (int k = 0; k < KR; ++k) {
      r[k] = lane + 64 * k < d.V ? r[k] : kNegInf;
      m = fmaxf(m, r[k]);
    }
    m = wave_max(m);
#pragma unroll
    for (int k = 0; k < KR; ++k) s += lane + 64 * k < d.V ? expf(r[k] - m) : 0.0f;
  } else {
    for (int v = lane; v < d.V; v += 64) m = fmaxf(m, a[v]);
    m = wave_max(m);
    for (int v = lane; v < d.V; v += 64) s += expf(a[v] - m);
  }
  s = wave_sumf(s);
  if (lane == 0) {
    const float dn = -(m + logf(s));
    denom[row] = dn;
    lpb[row] = dn + a[d.blank];
    lpl[row] = u < Ub - 1 ? dn + a[label_at(d, labels, b, u)] : kNegInf;
  }
}

// blockIdx.y == 0: alphas (gpu_rnnt_kernel.py:66-166); == 1: betas (168-260).
template <int PT>   // per-thread label positions (u = tid + k * blockDim): 1 up to U = 1024, else 8
__global__ __launch_bounds__(1024) void rnnt_lattice_kernel(const float* __restrict__ lpb, const float* __restrict__ lpl,
                                                            const int32_t* __restrict__ act_lens,
                                                            const int32_t* __restrict__ label_lens, Dims d,
                                                            float* __restrict__ alphas, float* __restrict__ betas,
                                                            float* __restrict__ llf, float* __restrict__ llb,
                                                            float* __restrict__ costs, float fastemit_lambda,
                                                            int per_thread, int dir0) {
  extern __shared__ float prev[];  // the previous diagonal, indexed by u
  const int b = blockIdx.x;
  const bool fwd = blockIdx.y + dir0 == 0;
  int Tb, Ub;
  lens(d, act_lens, label_lens, b, Tb, Ub);
  if (Tb < 1) {
    if (threadIdx.x == 0) {
      if (fwd) { llf[b] = kNegInf; costs[b] = INFINITY; } else { llb[b] = kNegInf; }
    }
    return;
  }
  const long off = (long)b * d.T * d.U;
  float* lat = fwd ? alphas : betas;
  float mine[PT];  // this thread's value on the previous diagonal, per owned u (u = tid + k * blockDim)
#pragma unroll
  for (int k = 0; k < PT; ++k) mine[k] = kNegInf;
  const int ndiag = Tb + Ub - 1;
  // The log-probabilities a thread needs on diagonal n (vb: lpb, vl: lpl; 0 where unused) are fetched two
  // diagonals ahead, so their global-load latency overlaps two diagonals' LDS exchange and barriers instead of
  // stalling every diagonal.  The arithmetic is unchanged.
  auto fetch = [&](int n, int k, float& vb, float& vl) {
    vb = 0.0f;
    vl = 0.0f;
    const int u = threadIdx.x + k * blockDim.x;
    if (k >= per_thread || u >= Ub || n >= ndiag) return;
    if (fwd) {
      const int t = n - u;
      if (t < 0 || t >= Tb) return;
      if (t > 0) vb = lpb[off + (long)(t - 1) * d.U + u];
      if (u > 0) vl = lpl[off + (long)t * d.U + u - 1];
    } else {
      const int t = Tb - 1 - (n - (Ub - 1 - u));
      if (t < 0 || t >= Tb || n < Ub - 1 - u) return;
      const long idx = off + (long)t * d.U + u;
      vb = lpb[idx];
      if (u < Ub - 1) vl = lpl[idx];
    }
  };
  float pb0[PT], pl0[PT], pb1[PT], pl1[PT];   // diagonals n and n + 1
#pragma unroll
  for (int k = 0; k < PT; ++k) {
    fetch(0, k, pb0[k], pl0[k]);
    fetch(1, k, pb1[k], pl1[k]);
  }
  for (int n = 0; n < ndiag; ++n) {
    float pb2[PT], pl2[PT];
#pragma unroll
    for (int k = 0; k < PT; ++k) fetch(n + 2, k, pb2[k], pl2[k]);
    float cur[PT];
#pragma unroll
    for (int k = 0; k < PT; ++k) {
      cur[k] = kNegInf;
      if (k >= per_thread) continue;
      const int u = threadIdx.x + k * blockDim.x;
      if (u >= Ub) continue;
      if (fwd) {
        const int t = n - u;
        if (t < 0 || t >= Tb) continue;
        float v;
        if (t == 0 && u == 0) v = 0.0f;
        else if (u == 0) v = mine[k] + pb0[k];
        else if (t == 0) v = prev[u - 1] + pl0[k];
        else v = log_sum_exp(prev[u - 1] + pl0[k], mine[k] + pb0[k]);
        cur[k] = v;
        lat[off + (long)t * d.U + u] = v;
      } else {
        // anti-diagonal n counted from the end: t = Tb - 1 - (n - (Ub - 1 - u))
        const int t = Tb - 1 - (n - (Ub - 1 - u));
        if (t < 0 || t >= Tb || n < Ub - 1 - u) continue;
        float v;
        const long idx = off + (long)t * d.U + u;
        if (t == Tb - 1 && u == Ub - 1) v = pb0[k];
        else if (u == Ub - 1) v = mine[k] + pb0[k];
        else if (t == Tb - 1) v = prev[u + 1] + pl0[k];
        else v = log_sum_exp(prev[u + 1] + pl0[k], mine[k] + pb0[k]);
        cur[k] = v;
        lat[idx] = v;
      }
    }
#pragma unroll
    for (int k = 0; k < PT; ++k) {
      pb0[k] = pb1[k]; pl0[k] = pl1[k];
      pb1[k] = pb2[k]; pl1[k] = pl2[k];
    }
    __syncthreads();  // everyone has read the previous diagonal
#pragma unroll
    for (int k = 0; k < PT; ++k) {
      if (k >= per_thread) continue;
      const int u = threadIdx.x + k * blockDim.x;
      if (u < Ub) {  // this diagonal's value (or -inf): read by u itself and by its neighbour next diagonal
        mine[k] = cur[k];
        prev[u] = cur[k];
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    if (fwd) {
      const float ll = alphas[off + (long)(Tb - 1) * d.U + Ub - 1] + lpb[off + (long)(Tb - 1) * d.U + Ub - 1];
      llf[b] = ll;
      costs[b] = (-ll) * (1.0f + fastemit_lambda);  // compute_costs_data
    } else {
      llb[b] = betas[off];
    }
  }
}

__global__ __launch_bounds__(256) void rnnt_grad_kernel(const float* __restrict__ acts, const int32_t* __restrict__ labels,
                                                        const int32_t* __restrict__ act_lens,
                                                        const int32_t* __restrict__ label_lens, Dims d,
                                                        const float* __restrict__ denom, const float* __restrict__ alphas,
                                                        const float* __restrict__ betas, const float* __restrict__ llf,
                                                        float fastemit_lambda, float clamp, float pre,
                                                        const float* __restrict__ scale, float* __restrict__ grads) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= (long)d.B * d.T * d.U) return;
  const int u = (int)(row % d.U);
  const long bt = row / d.U;
  const int t = (int)(bt % d.T), b = (int)(bt / d.T);
  int Tb, Ub;
  lens(d, act_lens, label_lens, b, Tb, Ub);
  float* g = grads + row * d.V;
  if (t >= Tb || u >= Ub) {
    for (int v = lane; v < d.V; v += 64) g[v] = 0.0f;
    return;
  }
  const float* a = acts + row * d.V;
  const float dn = denom[row], al = alphas[row], be = betas[row], ll = llf[b];
  const int lab = u < Ub - 1 ? label_at(d, labels, b, u) : -1;
  const float be_t1 = t < Tb - 1 ? betas[row + d.U] : 0.0f;
  const float be_u1 = u < Ub - 1 ? betas[row + 1] : 0.0f;
  const float lp_lab = lab >= 0 ? dn + a[lab] : 0.0f;
  const float l1p = log1pf(fastemit_lambda);
  const float sc = scale ? scale[b] : 1.0f;
  auto gval = [&](int v, float av) {
    const float logpk = dn + av;
    float gr = expf(al + be + logpk - ll);
    if (fastemit_lambda > 0.0f && u < Ub - 1) gr = gr + fastemit_lambda * expf(al + lp_lab + be_u1 + logpk - ll);
    if (v == d.blank && t == Tb - 1 && u == Ub - 1) gr -= expf(al + logpk - ll);
    if (v == d.blank && t < Tb - 1) gr -= expf(al + logpk - ll + be_t1);
    if (u < Ub - 1 && v == lab) gr -= expf(l1p + al + logpk - ll + be_u1);
    if (clamp > 0.0f) gr = fmaxf(fminf(gr, clamp), -clamp);
    if (pre != 1.0f) gr *= pre;   // as the host's in-place multiplies after the kernel, same order
    if (scale) gr *= sc;
    return gr;
  };
  if (d.V <= 64 * kDenomRegs) {
    // the whole row in flight per lane (up to 32 independent loads), then the math and the stores: the wave's
    // bytes in flight, not HBM bandwidth, bounded the four-at-a-time loop below
    float av[kDenomRegs];
#pragma unroll
    for (int k = 0; k < kDenomRegs; ++k) {
      const int v = lane + 64 * k;
      av[k] = v < d.V ? a[v] : 0.0f;
    }
#pragma unroll
    for (int k = 0; k < kDenomRegs; ++k) {
      const int v = lane + 64 * k;
      if (v < d.V) g[v] = gval(v, av[k]);
    }
    return;
  }
  // four logits in flight per lane (independent loads, then the math)
  int v0 = lane;
  for (; v0 + 192 < d.V; v0 += 256) {
    float av[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) av[k] = a[v0 + 64 * k];
#pragma unroll
    for (int k = 0; k < 4; ++k) g[v0 + 64 * k] = gval(v0 + 64 * k, av[k]);
  }
  for (int v = v0; v < d.V; v += 64) g[v] = gval(v, a[v]);
}

// The same gradient over a flat, 16-byte aligned span: a block owns kGradRows consecutive lattice rows, i.e.
// kGradRows * V contiguous floats, which start 16-byte aligned whatever V (kGradRows * 4 bytes is a multiple
// of 16).  The rows' scalars (denominator, lattice values, label terms, flags) go to LDS first; then float4
// loads and stores stream the span, each element finding its row by a running (row, v) walk.  The unaligned
// 1025-float rows made every wave-per-row store straddle cache lines.  Element values are rnnt_grad_kernel's
// (same expression, same order).
constexpr int kGradRows = 64;
struct GradRow {
  float dn, al, be, ll, be_t1, be_u1, lp_lab, sc;
  int lab, flags;   // flags: 1 inside the lattice, 2 u < Ub - 1, 4 last node (t, u) = (Tb - 1, Ub - 1), 8 t < Tb - 1
};
__global__ __launch_bounds__(256) void rnnt_grad_flat_kernel(const float* __restrict__ acts,
                                                             const int32_t* __restrict__ labels,
                                                             const int32_t* __restrict__ act_lens,
                                                             const int32_t* __restrict__ label_lens, Dims d,
                                                             const float* __restrict__ denom,
                                                             const float* __restrict__ alphas,
                                                             const float* __restrict__ betas,
                                                             const float* __restrict__ llf, float fastemit_lambda,
                                                             float clamp, float pre, const float* __restrict__ scale,
                                                             float* __restrict__ grads) {
  __shared__ GradRow rows[kGradRows];
  const long nrow = (long)d.B * d.T * d.U;
  const long r0 = (long)blockIdx.x * kGradRows;
  const int nr = (int)min((long)kGradRows, nrow - r0);
  if (threadIdx.x < nr) {
    const long row = r0 + threadIdx.x;
    const int u = (int)(row % d.U);
    const long bt = row / d.U;
    const int t = (int)(bt % d.T), b = (int)(bt / d.T);
    int Tb, Ub;
    lens(d, act_lens, label_lens, b, Tb, Ub);
    GradRow g{};
    if (t < Tb && u < Ub) {
      g.dn = denom[row]; g.al = alphas[row]; g.be = betas[row]; g.ll = llf[b];
      g.lab = u < Ub - 1 ? label_at(d, labels, b, u) : -1;
      g.be_t1 = t < Tb - 1 ? betas[row + d.U] : 0.0f;
      g.be_u1 = u < Ub - 1 ? betas[row + 1] : 0.0f;
      g.lp_lab = g.lab >= 0 ? g.dn + acts[row * d.V + g.lab] : 0.0f;
      g.sc = scale ? scale[b] : 1.0f;
      g.flags = 1 | (u < Ub - 1 ? 2 : 0) | (t == Tb - 1 && u == Ub - 1 ? 4 : 0) | (t < Tb - 1 ? 8 : 0);
    }
    rows[threadIdx.x] = g;
  }
  __syncthreads();
  const float l1p = log1pf(fastemit_lambda);
  auto gval = [&](const GradRow& r, int v, float av) {
    if (!(r.flags & 1)) return 0.0f;
    const float logpk = r.dn + av;
    float gr = expf(r.al + r.be + logpk - r.ll);
    if (fastemit_lambda > 0.0f && (r.flags & 2)) gr = gr + fastemit_lambda * expf(r.al + r.lp_lab + r.be_u1 + logpk - r.ll);
    if (v == d.blank && (r.flags & 4)) gr -= expf(r.al + logpk - r.ll);
    if (v == d.blank && (r.flags & 8)) gr -= expf(r.al + logpk - r.ll + r.be_t1);
    if ((r.flags & 2) && v == r.lab) gr -= expf(l1p + r.al + logpk - r.ll + r.be_u1);
    if (clamp > 0.0f) gr = fmaxf(fminf(gr, clamp), -clamp);
    if (pre != 1.0f) gr *= pre;
    if (scale) gr *= r.sc;
    return gr;
  };
  const float* a = acts + r0 * d.V;
  float* g = grads + r0 * d.V;
  const int len = nr * d.V, nvec = len / 4;
  constexpr int UNR = 4;
  for (int q0 = threadIdx.x; q0 < nvec; q0 += 256 * UNR) {
    float4 av[UNR];
#pragma unroll
    for (int j = 0; j < UNR; ++j) {
      const int q = q0 + 256 * j;
      av[j] = q < nvec ? *(const float4*)(a + 4 * q) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int j = 0; j < UNR; ++j) {
      const int q = q0 + 256 * j;
      if (q >= nvec) break;
      const int e = 4 * q;
      int rl = e / d.V, v = e - rl * d.V;
      float o[4];
      const float in[4] = {av[j].x, av[j].y, av[j].z, av[j].w};
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        if (v >= d.V) { v -= d.V; ++rl; }
        o[c] = gval(rows[rl], v, in[c]);
        ++v;
      }
      *(float4*)(g + e) = make_float4(o[0], o[1], o[2], o[3]);
    }
  }
  for (int e = 4 * nvec + threadIdx.x; e < len; e += 256) {   // < 4 trailing floats
    const int rl = e / d.V;
    g[e] = gval(rows[rl], e - rl * d.V, a[e]);
  }
}

size_t ws_floats(int B, int T, int U) { return (size_t)5 * B * T * U + 2 * (size_t)B + 64; }

// the flat kernel when both tensors are 16-byte aligned (CFM_RNNT_GRAD_FLAT=0: the wave-per-row kernel)
void launch_grad(const float* acts, const int32_t* labels, const int32_t* act_lens, const int32_t* label_lens,
                 const Dims& d, const float* denom, const float* alphas, const float* betas, const float* llf,
                 float fastemit_lambda, float clamp, float pre, const float* scale, float* grads, hipStream_t st) {
  static const int flat = [] { const char* e = getenv("CFM_RNNT_GRAD_FLAT"); return e ? atoi(e) : 1; }();
  const long n = (long)d.B * d.T * d.U;
  if (flat && !(((uintptr_t)acts | (uintptr_t)grads) & 15) && (long)kGradRows * d.V < (1L << 30))
    hipLaunchKernelGGL(rnnt_grad_flat_kernel, dim3((unsigned)((n + kGradRows - 1) / kGradRows)), dim3(256), 0, st,
                       acts, labels, act_lens, label_lens, d, denom, alphas, betas, llf, fastemit_lambda, clamp, pre,
                       scale, grads);
  else
    hipLaunchKernelGGL(rnnt_grad_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, st, acts, labels, act_lens,
                       label_lens, d, denom, alphas, betas, llf, fastemit_lambda, clamp, pre, scale, grads);
  HIP_OK(hipGetLastError());
}

void check_loss_args(const char* who, int B, int T, int U, int V, int blank, int labels_ld, size_t workspace_bytes,
                      const void* workspace, size_t need) {
  if (B < 0 || T < 1 || U < 1 || V < 1 || blank < 0 || blank >= V || labels_ld < U - 1)
    fail(CFM_ERR_INVALID_ARG, std::string(who) + ": need T, U, V >= 1, 0 <= blank < V, labels_ld >= U - 1");
  if (U > 8 * 1024) fail(CFM_ERR_UNSUPPORTED, std::string(who) + ": more than 8191 labels per utterance");
  if (B > 0 && (workspace_bytes < need || !workspace)) fail(CFM_ERR_WORKSPACE, std::string(who) + ": workspace too small");
}

// denominators, the alpha lattice and the costs; the beta lattice when `betas`; the gradient when grads
void loss_impl(const float* acts, const int32_t* labels, int labels_ld, const int32_t* act_lens,
               const int32_t* label_lens, int B, int T, int U, int V, int blank, float fastemit_lambda, float clamp,
               float* costs, float* grads, bool betas_too, void* workspace, size_t workspace_bytes, void* stream) {
  check_loss_args("cfm_rnnt_loss", B, T, U, V, blank, labels_ld, workspace_bytes, workspace,
                  ws_floats(B, T, U) * sizeof(float));
  if (B == 0) return;
  if (!acts || !act_lens || !label_lens || !costs || (U > 1 && !labels))
    fail(CFM_ERR_INVALID_ARG, "cfm_rnnt_loss: null input");
  hipStream_t st = (hipStream_t)stream;
  const long n = (long)B * T * U;
  float* w = (float*)workspace;
  float *denom = w, *lpb = w + n, *lpl = w + 2 * n, *alphas = w + 3 * n, *betas = w + 4 * n;
  float *llf = w + 5 * n, *llb = llf + B;
  Dims d{B, T, U, V, blank, labels_ld};
  const unsigned rows_blocks = (unsigned)((n + 3) / 4);
  {
    auto kern = rnnt_denom_kernel<0>;
    if (V <= 64 * 8) kern = rnnt_denom_kernel<8>;
    else if (V <= 64 * 17) kern = rnnt_denom_kernel<17>;   // V + 1 = 1025
    else if (V <= 64 * kDenomRegs) kern = rnnt_denom_kernel<kDenomRegs>;
    hipLaunchKernelGGL(kern, dim3(rows_blocks), dim3(256), 0, st, acts, labels, act_lens, label_lens, d, denom, lpb, lpl);
  }
  HIP_OK(hipGetLastError());
  const int threads = std::min(1024, (U + 63) / 64 * 64);
  const int per_thread = (U + threads - 1) / threads;
  hipLaunchKernelGGL(per_thread == 1 ? rnnt_lattice_kernel<1> : rnnt_lattice_kernel<8>, dim3(B, betas_too ? 2 : 1), dim3(threads), (size_t)U * sizeof(float), st,
                     lpb, lpl, act_lens, label_lens, d, alphas, betas, llf, llb, costs, fastemit_lambda, per_thread, 0);
  HIP_OK(hipGetLastError());
  if (grads) {
    launch_grad(acts, labels, act_lens, label_lens, d, denom, alphas, betas, llf, fastemit_lambda, clamp, 1.0f, nullptr,
                grads, st);
  }
}

}  // namespace

extern "C" {

size_t cfm_rnnt_loss_workspace_size(int B, int T, int U) {
  if (B < 0 || T < 0 || U < 0) return 0;
  return ws_floats(B, T, U) * sizeof(float);
}

cfm_status cfm_rnnt_loss(const float* acts, const int32_t* labels, int labels_ld, const int32_t* act_lens,
                         const int32_t* label_lens, int B, int T, int U, int V, int blank, float fastemit_lambda,
                         float clamp, float* costs, float* grads, void* workspace, size_t workspace_bytes,
                         void* stream) {
  return guarded([&] {
    loss_impl(acts, labels, labels_ld, act_lens, label_lens, B, T, U, V, blank, fastemit_lambda, clamp, costs, grads,
              grads != nullptr, workspace, workspace_bytes, stream);
  });
}

cfm_status cfm_rnnt_loss_costs(const float* acts, const int32_t* labels, int labels_ld, const int32_t* act_lens,
                               const int32_t* label_lens, int B, int T, int U, int V, int blank, float fastemit_lambda,
                               float* costs, void* workspace, size_t workspace_bytes, void* stream) {
  return guarded([&] {
    loss_impl(acts, labels, labels_ld, act_lens, label_lens, B, T, U, V, blank, fastemit_lambda, 0.0f, costs, nullptr,
              true, workspace, workspace_bytes, stream);
  });
}

cfm_status cfm_rnnt_loss_grad(const float* acts, const int32_t* labels, int labels_ld, const int32_t* act_lens,
                              const int32_t* label_lens, int B, int T, int U, int V, int blank, float fastemit_lambda,
                              float clamp, float pre_scale, const float* scale, float* grads, const void* workspace,
                              size_t workspace_bytes, void* stream) {
  return guarded([&] {
    check_loss_args("cfm_rnnt_loss_grad", B, T, U, V, blank, labels_ld, workspace_bytes, workspace,
                    ws_floats(B, T, U) * sizeof(float));
    if (B == 0) return;
    if (!acts || !act_lens || !label_lens || !grads || (U > 1 && !labels))
      fail(CFM_ERR_INVALID_ARG, "cfm_rnnt_loss_grad: null input");
    const long n = (long)B * T * U;
    const float* w = (const float*)workspace;
    const float *denom = w, *alphas = w + 3 * n, *betas = w + 4 * n, *llf = w + 5 * n;
    Dims d{B, T, U, V, blank, labels_ld};
    launch_grad(acts, labels, act_lens, label_lens, d, denom, alphas, betas, llf, fastemit_lambda, clamp, pre_scale, scale,
                grads, (hipStream_t)stream);
  });
}

}  // extern "C"
