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
  if (d.V <= 64 * kDenomRegs) {
    // one pass over HBM: the row's logits stay in registers for the max and the exp-sum
    float r[kDenomRegs];
#pragma unroll
    for (int k = 0; k < kDenomRegs; ++k) {
      const int v = lane + 64 * k;
      r[k] = v < d.V ? a[v] : kNegInf;
      m = fmaxf(m, r[k]);
    }
    m = wave_max(m);
#pragma unroll
    for (int k = 0; k < kDenomRegs; ++k) s += lane + 64 * k < d.V ? expf(r[k] - m) : 0.0f;
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
__global__ __launch_bounds__(1024) void rnnt_lattice_kernel(const float* __restrict__ lpb, const float* __restrict__ lpl,
                                                            const int32_t* __restrict__ act_lens,
                                                            const int32_t* __restrict__ label_lens, Dims d,
                                                            float* __restrict__ alphas, float* __restrict__ betas,
                                                            float* __restrict__ llf, float* __restrict__ llb,
                                                            float* __restrict__ costs, float fastemit_lambda,
                                                            int per_thread) {
  extern __shared__ float prev[];  // the previous diagonal, indexed by u
  const int b = blockIdx.x;
  const bool fwd = blockIdx.y == 0;
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
  float mine[8];  // this thread's value on the previous diagonal, per owned u (u = tid + k * blockDim)
#pragma unroll
  for (int k = 0; k < 8; ++k) mine[k] = kNegInf;
  const int ndiag = Tb + Ub - 1;
  for (int n = 0; n < ndiag; ++n) {
    float cur[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      cur[k] = kNegInf;
      if (k >= per_thread) continue;
      const int u = threadIdx.x + k * blockDim.x;
      if (u >= Ub) continue;
      if (fwd) {
        const int t = n - u;
        if (t < 0 || t >= Tb) continue;
        float v;
        if (t == 0 && u == 0) v = 0.0f;
        else if (u == 0) v = mine[k] + lpb[off + (long)(t - 1) * d.U];
        else if (t == 0) v = prev[u - 1] + lpl[off + u - 1];
        else v = log_sum_exp(prev[u - 1] + lpl[off + (long)t * d.U + u - 1], mine[k] + lpb[off + (long)(t - 1) * d.U + u]);
        cur[k] = v;
        lat[off + (long)t * d.U + u] = v;
      } else {
        // anti-diagonal n counted from the end: t = Tb - 1 - (n - (Ub - 1 - u))
        const int t = Tb - 1 - (n - (Ub - 1 - u));
        if (t < 0 || t >= Tb || n < Ub - 1 - u) continue;
        float v;
        const long idx = off + (long)t * d.U + u;
        if (t == Tb - 1 && u == Ub - 1) v = lpb[idx];
        else if (u == Ub - 1) v = mine[k] + lpb[idx];
        else if (t == Tb - 1) v = prev[u + 1] + lpl[idx];
        else v = log_sum_exp(prev[u + 1] + lpl[idx], mine[k] + lpb[idx]);
        cur[k] = v;
        lat[idx] = v;
      }
    }
    __syncthreads();  // everyone has read the previous diagonal
#pragma unroll
    for (int k = 0; k < 8; ++k) {
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
                                                        float fastemit_lambda, float clamp, float* __restrict__ grads) {
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
  auto gval = [&](int v, float av) {
    const float logpk = dn + av;
    float gr = expf(al + be + logpk - ll);
    if (fastemit_lambda > 0.0f && u < Ub - 1) gr = gr + fastemit_lambda * expf(al + lp_lab + be_u1 + logpk - ll);
    if (v == d.blank && t == Tb - 1 && u == Ub - 1) gr -= expf(al + logpk - ll);
    if (v == d.blank && t < Tb - 1) gr -= expf(al + logpk - ll + be_t1);
    if (u < Ub - 1 && v == lab) gr -= expf(l1p + al + logpk - ll + be_u1);
    if (clamp > 0.0f) gr = fmaxf(fminf(gr, clamp), -clamp);
    return gr;
  };
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

size_t ws_floats(int B, int T, int U) { return (size_t)5 * B * T * U + 2 * (size_t)B + 64; }

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
    if (B < 0 || T < 1 || U < 1 || V < 1 || blank < 0 || blank >= V || labels_ld < U - 1)
      fail(CFM_ERR_INVALID_ARG, "cfm_rnnt_loss: need T, U, V >= 1, 0 <= blank < V, labels_ld >= U - 1");
    if (U > 8 * 1024) fail(CFM_ERR_UNSUPPORTED, "cfm_rnnt_loss: more than 8191 labels per utterance");
    if (B == 0) return;
    if (!acts || !act_lens || !label_lens || !costs || (U > 1 && !labels))
      fail(CFM_ERR_INVALID_ARG, "cfm_rnnt_loss: null input");
    if (workspace_bytes < cfm_rnnt_loss_workspace_size(B, T, U) || !workspace)
      fail(CFM_ERR_WORKSPACE, "cfm_rnnt_loss: workspace too small");
    hipStream_t st = (hipStream_t)stream;
    const long n = (long)B * T * U;
    float* w = (float*)workspace;
    float *denom = w, *lpb = w + n, *lpl = w + 2 * n, *alphas = w + 3 * n, *betas = w + 4 * n;
    float *llf = w + 5 * n, *llb = llf + B;
    Dims d{B, T, U, V, blank, labels_ld};
    const unsigned rows_blocks = (unsigned)((n + 3) / 4);
    hipLaunchKernelGGL(rnnt_denom_kernel, dim3(rows_blocks), dim3(256), 0, st, acts, labels, act_lens, label_lens, d,
                       denom, lpb, lpl);
    HIP_OK(hipGetLastError());
    const int threads = std::min(1024, (U + 63) / 64 * 64);
    const int per_thread = (U + threads - 1) / threads;
    hipLaunchKernelGGL(rnnt_lattice_kernel, dim3(B, grads ? 2 : 1), dim3(threads), (size_t)U * sizeof(float), st, lpb,
                       lpl, act_lens, label_lens, d, alphas, betas, llf, llb, costs, fastemit_lambda, per_thread);
    HIP_OK(hipGetLastError());
    if (grads) {
      hipLaunchKernelGGL(rnnt_grad_kernel, dim3(rows_blocks), dim3(256), 0, st, acts, labels, act_lens, label_lens, d,
                         denom, alphas, betas, llf, fastemit_lambda, clamp, grads);
      HIP_OK(hipGetLastError());
    }
  });
}

}  // extern "C"
