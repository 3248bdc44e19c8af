// RNN-T prediction network (LSTM) and greedy batch decoding (SURVEY §8 a-ext4 / f2); contract in
// include/cfm_rnnt_decode.h.
//
// Everything here is a skinny fp32 contraction: a handful of utterances (rows) against weight
// matrices of a few MB, so the kernels are weight-bandwidth bound (L2 / MALL resident after the first
// iteration).  Shape of every kernel: a block stages RB utterance rows of its input in LDS once; each
// wave owns 4 output columns, its lanes stride the contraction axis with coalesced weight loads and
// keep 4 x RB partial sums, which one LDS transpose turns into per-(column, row) totals; the epilogue
// is fused (LSTM cell update, joint activation, or the per-block max / argmax / sum-exp of the logits).
//   lstm_step_kernel   one layer step: the 4 gate rows (i, f, g, o) of a hidden unit live in one wave,
//                      so the cell update needs no second pass
//   joint_hidden_kernel  act(f[b, t_b] + W_pred h + b_pred) for each utterance's current frame
//   joint_logits_kernel  W_out hid + b_out -> block partials (max, first argmax, sum exp(z - max))
//   greedy_commit_kernel one block: argmax/log-sum-exp fold, emit-or-advance decision per utterance,
//                        state commit for emitting utterances, the any-active flag
//   enc_proj_kernel      f = enc W_enc^T + b_enc for all (b, t) up front (64x64 LDS-tiled fp32 GEMM
//                        reading the (B, D1, T) encoder output along time)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <string>
#include <vector>

#include "../../include/cfm_rnnt_decode.h"
#include "../../include/cfm_train.h"
#include "cfm_abi.h"
#include "cfm_common.h"
#include "cfm_kernels.h"

using namespace cfm;

struct cfm_rnnt_decoder {
  int V = 0, H = 0, L = 0, device = 0;
  float* wbuf = nullptr;        // emb (V+1, H) | per layer [W_ih | W_hh] (4H, 2H) | per layer bias (4H)
  long emb_off = 0, w_off = 0, b_off = 0;
  bool x_want = false;          // the matrix-core step can use the layer-0 input table below
  bool x_ready = false;         // the table matches the current weights (set_weights clears it)
  float* xbuf = nullptr;        // that table: allocated by the first inference call (ensure_xtab), never by
                                // training-only handles ((V+1) x 4H fp32: 10.5 MB at V 1024 / H 640, 134 MB at V 8192)
  int* host_flag = nullptr;     // pinned, 2 slots (greedy done-flag polling)
  hipEvent_t ev[2] = {nullptr, nullptr};
  const float* emb() const { return wbuf + emb_off; }
  const float* W(int l) const { return wbuf + w_off + (long)l * 4 * H * 2 * H; }
  const float* bias(int l) const { return wbuf + b_off + (long)l * 4 * H; }
  // layer 0's input projection for every embedding row: xtab[e][r] = sum_k emb[e][k] W_ih[r][k], (V+1, 4H),
  // built on first use after set_weights; inference steps gather a row instead of contracting over the input
  float* xtab() const { return xbuf; }
};

namespace {

constexpr int RB = 8;                 // utterance rows per block
constexpr int RED = 4 * 64 * 33;      // per-block transpose-reduce scratch (floats)

__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }

__device__ __forceinline__ float act_fn(int act, float x) {
  return act == CFM_JOINT_RELU ? fmaxf(x, 0.0f) : act == CFM_JOINT_SIGMOID ? sigm(x) : tanhf(x);
}

// Stage rows [b0, b0 + nb) of concat(x, h) (I + Hh floats per row, both multiples of 4) into As as
// float4s.  x comes from xsrc, or from the embedding row xlab[b] (xlab < 0: the zero
// start-of-sequence vector).  All of a thread's loads are issued before the LDS stores (latency).
__device__ __forceinline__ void stage_rows(float* As, int K, int I, int Hh, int b0, int nb, const float* xsrc,
                                           const int32_t* xlab, const float* emb, int nemb, const float* h) {
  const int K4 = K >> 2, I4 = I >> 2;
#pragma unroll
  for (int r = 0; r < RB; ++r) {
    const long b = b0 + r;
    const float4* xs = nullptr;
    if (r < nb) {
      if (xsrc) xs = (const float4*)(xsrc + b * I);
      else if (xlab[b] >= 0) xs = (const float4*)(emb + (long)min(xlab[b], nemb - 1) * I);
    }
    const float4* hs = (r < nb && Hh > 0) ? (const float4*)(h + b * Hh) : nullptr;
    for (int k4 = threadIdx.x; k4 < K4; k4 += blockDim.x) {
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (k4 < I4) { if (xs) v = xs[k4]; }
      else if (hs) v = hs[k4 - I4];
      ((float4*)As)[r * K4 + k4] = v;
    }
  }
}

// acc[c][r] = sum_k As[r][k] * Wrow_c[k] over this lane's float4 slots; then the per-wave transpose:
// lane l < 4*RB returns the total for (c = l / RB, r = l % RB).  K % 4 == 0.
__device__ __forceinline__ float wave_dot4(const float* As, int K, const float* const (&wr)[4], bool valid,
                                           float* red_wave) {
  const int lane = threadIdx.x & 63;
  const int K4 = K >> 2;
  float acc[4][RB];
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int r = 0; r < RB; ++r) acc[c][r] = 0.0f;
  if (valid) {
    // UK float4 steps of weight loads are issued before any is consumed: the loop is latency-bound,
    // so this keeps 4 * UK 16-byte loads in flight per lane.
    constexpr int UK = 2;
    for (int k4 = lane; k4 < K4; k4 += 64 * UK) {
      float4 w[UK][4];
#pragma unroll
      for (int u = 0; u < UK; ++u)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int kk = k4 + 64 * u;
          w[u][c] = (wr[c] && kk < K4) ? ((const float4*)wr[c])[kk] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
      for (int u = 0; u < UK; ++u) {
        const int kk = min(k4 + 64 * u, K4 - 1);   // out-of-range steps multiply zero weights
#pragma unroll
        for (int r = 0; r < RB; ++r) {
          const float4 a = ((const float4*)(As + r * K))[kk];
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            float t = acc[c][r];
            t = fmaf(w[u][c].x, a.x, t);
            t = fmaf(w[u][c].y, a.y, t);
            t = fmaf(w[u][c].z, a.z, t);
            acc[c][r] = fmaf(w[u][c].w, a.w, t);
          }
        }
      }
    }
  }
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int r = 0; r < RB; ++r) red_wave[lane * 33 + c * RB + r] = acc[c][r];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  float s = 0.0f;
  if (lane < 4 * RB)
    for (int l = 0; l < 64; ++l) s += red_wave[l * 33 + lane];
  return s;
}

// One LSTM layer step for rows [b0, b0 + RB): wave w owns hidden unit j = 4 * blockIdx.x + w.
__global__ __launch_bounds__(256) void lstm_step_kernel(const float* __restrict__ W, const float* __restrict__ bias,
                                                        const float* __restrict__ emb, int nemb,
                                                        const int32_t* __restrict__ xlab, const float* __restrict__ xsrc,
                                                        const float* __restrict__ h, const float* __restrict__ c,
                                                        float* __restrict__ h2, float* __restrict__ c2,
                                                        float* __restrict__ gout, long gstride, int B, int I, int H,
                                                        const int* __restrict__ run_flag,
                                                        float* __restrict__ gates_out = nullptr, Drop gdrop = Drop{0u, 0u, 1.0f},
                                                        int gstep = 0) {
  extern __shared__ float lds[];
  const int K = I + H;
  const int b0 = blockIdx.y * RB, nb = min(RB, B - b0);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int j = blockIdx.x * 4 + wave;
  const bool valid = j < H;
  // loads the epilogue needs, issued before the staging so their latency overlaps it
  const int run = run_flag ? *run_flag : 1;
  const int jc = min(j, H - 1), bl = b0 + min(lane, nb - 1);
  const float cprev = c[(long)bl * H + jc];
  const float bs0 = bias[jc], bs1 = bias[H + jc], bs2 = bias[2 * H + jc], bs3 = bias[3 * H + jc];
  float* As = lds;
  float* red = lds + RB * K;
  float* gsum = red + RED;               // [4 waves][4 * RB] gate totals
  stage_rows(As, K, I, H, b0, nb, xsrc, xlab, emb, nemb, h);
  __syncthreads();
  if (run == 0) return;                  // uniform: every utterance finished, nothing written yet
  const float* wr[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) wr[g] = valid ? W + (long)(g * H + j) * K : nullptr;
  float* rw = red + wave * 64 * 33;
  const float s = wave_dot4(As, K, wr, valid, rw);
  // gather the 4 gates of row r into lane r
  float* gs = gsum + wave * 4 * RB;
  if (lane < 4 * RB) gs[lane] = s;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  if (!valid || lane >= nb) return;
  const long b = b0 + lane;
  const float gi = sigm(gs[0 * RB + lane] + bs0);
  const float gf = sigm(gs[1 * RB + lane] + bs1);
  const float gg = tanhf(gs[2 * RB + lane] + bs2);
  const float go = sigm(gs[3 * RB + lane] + bs3);
  const float cn = gf * cprev + gi * gg;
  const float hn = go * tanhf(cn);
  c2[b * H + j] = cn;
  h2[b * H + j] = hn;
  // LSTMDropout's output Dropout (rnn.py:151-237; training), mask index (b, step, j) of g (B, S, H)
  if (gout) gout[b * gstride + j] = hn * drop_mul(gdrop, ((uint64_t)b * (gstride / H) + gstep) * H + j);
  if (gates_out) {   // training tape: post-activation gates [i | f | g | o] of this step
    float* gr = gates_out + b * 4L * H;
    gr[j] = gi; gr[H + j] = gf; gr[2 * H + j] = gg; gr[3 * H + j] = go;
  }
}

// hid[b][n] = act(F[b, t_b][n] + sum_k h[b][k] Wp[n][k] + bp[n]),  n < J
__global__ __launch_bounds__(256) void joint_hidden_kernel(const float* __restrict__ Wp, const float* __restrict__ bp,
                                                           const float* __restrict__ h, const float* __restrict__ F,
                                                           const int32_t* __restrict__ tptr, int T, int B, int H,
                                                           int J, int act, float* __restrict__ hid,
                                                           const int* __restrict__ run_flag) {
  extern __shared__ float lds[];
  const int b0 = blockIdx.y * RB, nb = min(RB, B - b0);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int n0 = blockIdx.x * 16 + wave * 4;
  // the epilogue's operands (this lane's (row, column) after the transpose), fetched up front
  const int run = run_flag ? *run_flag : 1;
  const int ec = (lane % (4 * RB)) / RB, er = lane % RB;
  const int en = min(n0 + ec, J - 1);
  const long eb = b0 + min(er, nb - 1);
  const int et = min(max(tptr[eb], 0), T - 1);
  const float fe = F[(eb * T + et) * J + en] + bp[en];
  float* As = lds;
  float* red = lds + RB * H;
  stage_rows(As, H, H, 0, b0, nb, h, nullptr, nullptr, 1, nullptr);
  __syncthreads();
  if (run == 0) return;
  const float* wr[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) wr[c] = (n0 + c < J) ? Wp + (long)(n0 + c) * H : nullptr;
  const float s = wave_dot4(As, H, wr, n0 < J, red + wave * 64 * 33);
  if (lane >= 4 * RB) return;
  const int c = lane / RB, r = lane % RB, n = n0 + c;
  if (r >= nb || n >= J) return;
  hid[(b0 + r) * (long)J + n] = act_fn(act, s + fe);
}

struct Part {
  float m;
  int idx;
  float se;
};

// z[b][n] = sum_k hid[b][k] Wo[n][k] + bo[n] for the block's 16 columns -> part[blockIdx.x * B + b]
__global__ __launch_bounds__(256) void joint_logits_kernel(const float* __restrict__ Wo, const float* __restrict__ bo,
                                                           const float* __restrict__ hid, int B, int J, int N,
                                                           Part* __restrict__ part, const int* __restrict__ run_flag) {
  extern __shared__ float lds[];
  const int b0 = blockIdx.y * RB, nb = min(RB, B - b0);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int n0 = blockIdx.x * 16 + wave * 4;
  const int run = run_flag ? *run_flag : 1;
  const float be = bo[min(n0 + (lane % (4 * RB)) / RB, N - 1)];
  float* As = lds;
  float* red = lds + RB * J;
  float* zs = red + RED;                 // [16][RB]
  stage_rows(As, J, J, 0, b0, nb, hid, nullptr, nullptr, 1, nullptr);
  __syncthreads();
  if (run == 0) return;
  const float* wr[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) wr[c] = (n0 + c < N) ? Wo + (long)(n0 + c) * J : nullptr;
  const float s = wave_dot4(As, J, wr, n0 < N, red + wave * 64 * 33);
  if (lane < 4 * RB) {
    const int c = lane / RB, r = lane % RB;
    const int n = n0 + c;
    zs[(wave * 4 + c) * RB + r] = (n < N) ? s + be : -INFINITY;
  }
  __syncthreads();
  if (threadIdx.x >= nb) return;
  const int r = threadIdx.x;
  const int nend = min(16, N - blockIdx.x * 16);
  float m = -INFINITY;
  int idx = -1;
  for (int c = 0; c < nend; ++c) {
    const float z = zs[c * RB + r];
    if (idx < 0 || z > m) { m = z; idx = blockIdx.x * 16 + c; }
  }
  float se = 0.0f;
  for (int c = 0; c < nend; ++c) se += expf(zs[c * RB + r] - m);
  part[(long)blockIdx.x * B + b0 + r] = Part{m, idx, se};
}

struct Ctrl {
  int32_t* t;        // current frame
  int32_t* s;        // labels emitted at this frame
  int32_t* xlab;     // next LSTM input label (-1: zero SOS vector)
  int32_t* active;
  int32_t* copy;     // 1: commit the new state this iteration
  int* flag;         // any utterance still active
};

__global__ __launch_bounds__(256) void greedy_init_kernel(const int64_t* __restrict__ len, int B, int T, Ctrl ct,
                                                          int32_t* __restrict__ ntok, double* __restrict__ scores,
                                                          float* __restrict__ hc, long nhc) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < B) {
    ct.t[i] = 0;
    ct.s[i] = 0;
    ct.xlab[i] = -1;
    const long L = len[i];
    ct.active[i] = (min(L, (long)T) > 0) ? 1 : 0;
    ct.copy[i] = 0;
    ntok[i] = 0;
    scores[i] = 0.0;
  }
  if (i == 0) *ct.flag = 1;
  for (long k = i; k < nhc; k += (long)gridDim.x * blockDim.x) hc[k] = 0.0f;
}

// One wave per utterance (grid B): fold the logits partials (lanes stride the column blocks), decide
// emit-or-advance, record the label, commit the new LSTM state if a label was emitted.
__global__ __launch_bounds__(64) void greedy_commit_kernel(const Part* __restrict__ part, int nblk, int B, int T,
                                                           const int64_t* __restrict__ len, int blank,
                                                           int max_symbols, int log_normalize, int sos_until_label,
                                                           Ctrl ct, int32_t* __restrict__ tokens,
                                                           int32_t* __restrict__ tsteps, long cap,
                                                           int32_t* __restrict__ ntok, double* __restrict__ scores,
                                                           float* __restrict__ h, float* __restrict__ c,
                                                           const float* __restrict__ h2, const float* __restrict__ c2,
                                                           int L, int H) {
  if (*ct.flag == 0) return;
  const int b = blockIdx.x, lane = threadIdx.x;
  if (!ct.active[b]) return;                    // block-uniform
  float m = -INFINITY;
  int k = -1;
  for (int q = lane; q < nblk; q += 64) {
    const Part p = part[(long)q * B + b];
    if (k < 0 || p.m > m) { m = p.m; k = p.idx; }
  }
  // wave argmax (ties -> lowest column: the partials' own first-max rule, folded in index order)
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const float m2 = __shfl_xor(m, o, 64);
    const int k2 = __shfl_xor(k, o, 64);
    if (k2 >= 0 && (k < 0 || m2 > m || (m2 == m && k2 < k))) { m = m2; k = k2; }
  }
  double v = m;
  if (log_normalize) {
    double s = 0.0;
    for (int q = lane; q < nblk; q += 64) {
      const Part p = part[(long)q * B + b];
      s += (double)p.se * exp((double)p.m - (double)m);
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o, 64);
    v = -log(s);                                // z[k] - logsumexp(z) with z[k] = max
  }
  const int tb = ct.t[b];
  const bool emit = k != blank;
  if (lane == 0) {
    if (emit) {
      const int n = ntok[b];
      tokens[b * cap + n] = k;
      tsteps[b * cap + n] = tb;
      ntok[b] = n + 1;
      scores[b] += v;
      ct.xlab[b] = k;
      if (ct.s[b] + 1 >= max_symbols) { ct.t[b] = tb + 1; ct.s[b] = 0; } else { ct.s[b] += 1; }
    } else {
      // batched decoding embeds the blank (padding) row after the first step; the per-utterance
      // decoder keeps feeding the zero SOS vector until a label is emitted (rnnt_greedy_decoding.py:315-318)
      if (ct.xlab[b] < 0 && !sos_until_label) ct.xlab[b] = blank;
      ct.t[b] = tb + 1;
      ct.s[b] = 0;
    }
    const long lb = min(len[b], (long)T);
    if (ct.t[b] >= lb) ct.active[b] = 0;
  }
  if (emit) {
    for (int l = 0; l < L; ++l) {
      const long o = ((long)l * B + b) * H;
      for (int j = lane; j < H; j += 64) { h[o + j] = h2[o + j]; c[o + j] = c2[o + j]; }
    }
  }
}

// flag = any utterance still active (one block; run once per chunk of iterations)
__global__ __launch_bounds__(256) void greedy_flag_kernel(const int32_t* __restrict__ active, int B, int* flag) {
  __shared__ int any;
  if (threadIdx.x == 0) any = 0;
  __syncthreads();
  int a = 0;
  for (int b = threadIdx.x; b < B; b += blockDim.x) a |= active[b];
  if (a) any = 1;                               // benign race: every writer stores 1
  __syncthreads();
  if (threadIdx.x == 0) *flag = any;
}

// F[(b*T + t)*J + n] = sum_d enc[b][d][t] * W[n][d] + bias[n]
__global__ __launch_bounds__(256) void enc_proj_kernel(const float* __restrict__ enc, const float* __restrict__ W,
                                                       const float* __restrict__ bias, int B, int T, int D, int J,
                                                       float* __restrict__ F) {
  __shared__ float As[16][64 + 4];
  __shared__ float Ws[16][64 + 4];
  const long M = (long)B * T;
  const long m0 = (long)blockIdx.x * 64;
  const int n0 = blockIdx.y * 64;
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  float acc[4][4] = {};
  for (int k0 = 0; k0 < D; k0 += 16) {
    for (int i = threadIdx.x; i < 16 * 64; i += 256) {
      const int kk = i >> 6, mm = i & 63;
      const long m = m0 + mm;
      const int k = k0 + kk;
      float v = 0.0f;
      if (m < M && k < D) {
        const long b = m / T, t = m - b * T;
        v = enc[(b * D + k) * T + t];
      }
      As[kk][mm] = v;
      const int nn = i >> 4, kw = i & 15;
      const int n = n0 + nn, k2 = k0 + kw;
      Ws[kw][nn] = (n < J && k2 < D) ? W[(long)n * D + k2] : 0.0f;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) {
      float a[4], w[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = As[kk][ty * 4 + i];
#pragma unroll
      for (int j = 0; j < 4; ++j) w[j] = Ws[kk][tx * 4 + j];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(a[i], w[j], acc[i][j]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const long m = m0 + ty * 4 + i;
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + tx * 4 + j;
      if (n < J) F[m * J + n] = acc[i][j] + bias[n];
    }
  }
}

__global__ void predict_labels_kernel(const int64_t* __restrict__ y, int B, int U, int S, int add_sos, int nemb,
                                      int32_t* __restrict__ xlab) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)S * B) return;
  const int u = (int)(i / B), b = (int)(i % B);
  const int uu = u - add_sos;
  int lab = -1;
  if (y && uu >= 0) lab = (int)min(max(y[(long)b * U + uu], (int64_t)0), (int64_t)(nemb - 1));
  xlab[i] = lab;
}

__global__ void pack_lstm_kernel(const float* __restrict__ wih, const float* __restrict__ whh,
                                 const float* __restrict__ bih, const float* __restrict__ bhh, int H,
                                 float* __restrict__ Wc, float* __restrict__ bc) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long n = 4L * H * 2 * H;
  if (i < n) {
    const long r = i / (2 * H), k = i % (2 * H);
    Wc[i] = k < H ? wih[r * H + k] : whh[r * H + (k - H)];
  }
  if (i < 4L * H) bc[i] = bih[i] + bhh[i];
}

// The same LSTM step on the matrix cores (fp32 in, fp32 sums: v_mfma_f32_16x16x4_f32, exact fp32
// products like the VALU kernel, in another summation order).  Block = 4 hidden units x 16 batch rows;
// its 16 W rows are ordered unit-major (row 4u + g = gate g of unit u0 + u), so the 16x16 output puts
// the four gates (i, f, g, o) of unit u0 + (lane >> 4) for batch row b0 + (lane & 15) in one lane's
// accumulator: the cell update needs no exchange.  K = I + H is split over the 8 waves in 16-wide
// groups (a float4 of A and of B per lane and group: MFMA j takes element j of both, so each group's
// 16 products are summed whatever the k order inside it); the eight partial tiles are summed in a
// fixed order through LDS.  A block reads its 16 W rows (80 KB at H = 640) and the batch's [x | h]
// rows once per step; the XCD that owns a unit block keeps its W rows in L2 across steps.
template <int NT>
__global__ __launch_bounds__(512) void lstm_step_mfma_kernel(const float* __restrict__ W, const float* __restrict__ bias,
                                                             const float* __restrict__ emb, int nemb,
                                                             const int32_t* __restrict__ xlab, const float* __restrict__ xsrc,
                                                             const float* __restrict__ h, const float* __restrict__ c,
                                                             float* __restrict__ h2, float* __restrict__ c2,
                                                             float* __restrict__ gout, long gstride, int B, int I, int H,
                                                             const int* __restrict__ run_flag,
                                                             float* __restrict__ gates_out, Drop gdrop, int gstep,
                                                             const float* __restrict__ xtab) {
  __shared__ f32x4 part[8][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int u0 = blockIdx.x * 4, b0 = blockIdx.y * 16;
  // xtab (layer 0 from embedding rows only): the input part comes from the gathered table row, the
  // contraction covers the h part alone
  const int K = I + H, kb = xtab ? I : 0, G = (K - kb) / 16;   // NT = ceil(G / 8) groups per wave
  if (run_flag && *run_flag == 0) return;   // uniform: every utterance finished
  // operand rows of this lane: W row (unit u0 + rr / 4, gate rr % 4), batch row b0 + rr
  const int rr = lane & 15, kq = lane >> 4;
  const int wu = min(u0 + (rr >> 2), H - 1), wg = rr & 3;
  const float* wrow = W + ((long)wg * H + wu) * K + kb + 4 * kq;
  const int b = b0 + rr;
  const int bc = min(b, B - 1);
  // the row's input part: the previous layer's h, an embedding row, or zero (start of sequence; rows past
  // B) - always loaded from a valid address and zeroed by a select (no per-lane conditional loads)
  const int lab = xsrc ? 0 : xlab[bc];
  const bool xok = b < B && (xsrc != nullptr || lab >= 0);
  const float* xrow = xsrc ? xsrc + (long)bc * I : emb + (long)min(max(lab, 0), nemb - 1) * I;
  const float* hrow = h + (long)bc * H;
  const bool hok = b < B;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  float4 wa[NT], xa[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {   // all loads first (latency), then the MFMAs
    const int gi = min(w + 8 * t, G - 1);
    const int k = kb + gi * 16 + 4 * kq;
    wa[t] = *(const float4*)(wrow + gi * 16);
    const bool inx = k < I;
    const float4 v = *(const float4*)(inx ? xrow + k : hrow + (k - I));
    xa[t] = (inx ? xok : hok) ? v : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  // wave 0's epilogue lanes fetch their table entries now, under the MFMA latency
  f32x4 xg = {0.f, 0.f, 0.f, 0.f};
  if (xtab && w == 0) {
    const int bb = b0 + (lane & 15), j = u0 + (lane >> 4);
    const int lb = (bb < B && j < H) ? xlab[bb] : -1;
    if (lb >= 0) {
      const float* xr = xtab + (long)min(lb, nemb - 1) * 4 * H + j;
      xg[0] = xr[0]; xg[1] = xr[H]; xg[2] = xr[2 * H]; xg[3] = xr[3 * H];
    }
  }
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    if (w + 8 * t < G) {   // wave-uniform
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[t].x, xa[t].x, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[t].y, xa[t].y, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[t].z, xa[t].z, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[t].w, xa[t].w, acc, 0, 0, 0);
    }
  }
  part[w][lane] = acc;
  __syncthreads();
  if (w != 0) return;
  f32x4 s = part[0][lane];
  s[0] += xg[0]; s[1] += xg[1]; s[2] += xg[2]; s[3] += xg[3];
#pragma unroll
  for (int ww = 1; ww < 8; ++ww) {
    const f32x4 t = part[ww][lane];
    s[0] += t[0]; s[1] += t[1]; s[2] += t[2]; s[3] += t[3];
  }
  // lane: batch row b0 + (lane & 15), unit u0 + (lane >> 4); s[e] = gate e's sum
  const int bb = b0 + (lane & 15), j = u0 + (lane >> 4);
  if (bb >= B || j >= H) return;
  const float gi = sigm(s[0] + bias[j]);
  const float gf = sigm(s[1] + bias[H + j]);
  const float gg = tanhf(s[2] + bias[2 * H + j]);
  const float go = sigm(s[3] + bias[3 * H + j]);
  const float cn = gf * c[(long)bb * H + j] + gi * gg;
  const float hn = go * tanhf(cn);
  c2[(long)bb * H + j] = cn;
  h2[(long)bb * H + j] = hn;
  if (gout) gout[(long)bb * gstride + j] = hn * drop_mul(gdrop, ((uint64_t)bb * (gstride / H) + gstep) * H + j);
  if (gates_out) {
    float* gr = gates_out + (long)bb * 4L * H;
    gr[j] = gi; gr[H + j] = gf; gr[2 * H + j] = gg; gr[3 * H + j] = go;
  }
}

// xtab[e][r] = sum_{k < I} emb[e][k] W[r][k] (W rows of stride ldw: layer 0's packed [W_ih | W_hh]);
// 64x64 LDS-tiled fp32, once per set_weights (the table is (V+1) x 4H)
__global__ __launch_bounds__(256) void lstm_xtab_kernel(const float* __restrict__ emb, const float* __restrict__ W,
                                                        int M, int N, int I, int ldw, float* __restrict__ X) {
  __shared__ float As[16][64 + 4];
  __shared__ float Ws[16][64 + 4];
  const int m0 = blockIdx.x * 64, n0 = blockIdx.y * 64;
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  float acc[4][4] = {};
  for (int k0 = 0; k0 < I; k0 += 16) {
    for (int i = threadIdx.x; i < 16 * 64; i += 256) {
      const int rr = i >> 4, kk = i & 15;
      const int m = m0 + rr, n = n0 + rr, k = k0 + kk;
      As[kk][rr] = (m < M && k < I) ? emb[(long)m * I + k] : 0.0f;
      Ws[kk][rr] = (n < N && k < I) ? W[(long)n * ldw + k] : 0.0f;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) {
      float a[4], w[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = As[kk][ty * 4 + i];
#pragma unroll
      for (int j = 0; j < 4; ++j) w[j] = Ws[kk][tx * 4 + j];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(a[i], w[j], acc[i][j]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + ty * 4 + i;
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + tx * 4 + j;
      if (n < N) X[(long)m * N + n] = acc[i][j];
    }
  }
}

size_t lstm_lds(int K) { return (size_t)(RB * K + RED + 4 * 4 * RB) * sizeof(float); }

// > 64 KB of dynamic LDS needs the per-kernel opt-in; done once per process.
void set_lds_limits() {
  static const bool once = [] {
    constexpr int kMax = 160 * 1024;
    (void)hipFuncSetAttribute((const void*)lstm_step_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, kMax);
    (void)hipFuncSetAttribute((const void*)joint_hidden_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, kMax);
    (void)hipFuncSetAttribute((const void*)joint_logits_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, kMax);
    return true;
  }();
  (void)once;
}

void check_device(const cfm_rnnt_decoder* h) {
  int cur = -1;
  HIP_OK(hipGetDevice(&cur));
  if (cur != h->device) HIP_OK(hipSetDevice(h->device));
}

bool lstm_mfma_nt(int NT) { return NT == 1 || NT == 2 || NT == 3 || NT == 4 || NT == 5 || NT == 6 || NT == 8 || NT == 10 || NT == 12 || NT == 16; }

// one LSTM layer step: the matrix-core kernel when the shapes allow it (I, H multiples of 16, H % 4 == 0,
// K <= 3072; CFM_LSTM_MFMA=0 keeps the VALU kernel), else lstm_step_kernel.  Layer 0 fed from embedding rows
// outside training (no gates_out) uses the input table when the handle has one and it is current.
void launch_lstm_step(const cfm_rnnt_decoder* d, int l, const int32_t* xlab, const float* xsrc, const float* hcur,
                      const float* ccur, float* hn, float* cn, float* gout, long gstride, int B, const int* flag,
                      float* gates_out, Drop gdrop, int gstep, hipStream_t st) {
  static const int mfma = [] { const char* e = getenv("CFM_LSTM_MFMA"); return e ? atoi(e) : 1; }();
  const int H = d->H, I = H, K = I + H;
  const float* xt = (l == 0 && !xsrc && !gates_out && d->x_ready) ? d->xtab() : nullptr;
  const int NT = ((xt ? H : K) / 16 + 7) / 8;
  if (mfma && H % 16 == 0 && I % 16 == 0 && lstm_mfma_nt(NT)) {
    auto go = [&](auto kern) {
      hipLaunchKernelGGL(kern, dim3((unsigned)(H / 4), (unsigned)((B + 15) / 16)), dim3(512), 0, st, d->W(l), d->bias(l),
                         d->emb(), d->V + 1, xlab, xsrc, hcur, ccur, hn, cn, gout, gstride, B, I, H, flag, gates_out,
                         gdrop, gstep, xt);
    };
    switch (NT) {
      case 1: go(lstm_step_mfma_kernel<1>); break;
      case 2: go(lstm_step_mfma_kernel<2>); break;
      case 3: go(lstm_step_mfma_kernel<3>); break;
      case 4: go(lstm_step_mfma_kernel<4>); break;
      case 5: go(lstm_step_mfma_kernel<5>); break;
      case 6: go(lstm_step_mfma_kernel<6>); break;
      case 8: go(lstm_step_mfma_kernel<8>); break;
      case 10: go(lstm_step_mfma_kernel<10>); break;
      case 12: go(lstm_step_mfma_kernel<12>); break;
      default: go(lstm_step_mfma_kernel<16>); break;
    }
    return;
  }
  const dim3 grid((H + 3) / 4, (B + RB - 1) / RB);
  hipLaunchKernelGGL(lstm_step_kernel, grid, dim3(256), lstm_lds(K), st, d->W(l), d->bias(l), d->emb(), d->V + 1,
                     xlab, xsrc, hcur, ccur, hn, cn, gout, gstride, B, I, H, flag, gates_out, gdrop, gstep);
}

// (re)build the layer-0 input table after set_weights, on the stream of the call that will read it; only
// when the matrix-core step can take it (shapes above; CFM_LSTM_XTAB=0 disables it)
void ensure_xtab(cfm_rnnt_decoder* d, hipStream_t st) {
  if (d->x_ready || !d->x_want) return;
  const int H = d->H, N = 4 * H, M = d->V + 1;
  if (!d->xbuf && hipMalloc((void**)&d->xbuf, (size_t)M * N * sizeof(float)) != hipSuccess) {
    (void)hipGetLastError();   // no room for the table: the steps contract over [x | h] as training does
    d->xbuf = nullptr;
    d->x_want = false;
    return;
  }
  hipLaunchKernelGGL(lstm_xtab_kernel, dim3((unsigned)((M + 63) / 64), (unsigned)((N + 63) / 64)), dim3(256), 0, st,
                     d->emb(), d->W(0), M, N, H, 2 * H, d->xtab());
  HIP_OK(hipGetLastError());
  d->x_ready = true;
}

void lstm_layer(const cfm_rnnt_decoder* d, int l, const int32_t* xlab, const float* xsrc, const float* hcur,
                const float* ccur, float* hn, float* cn, float* gout, long gstride, int B, const int* flag,
                hipStream_t st) {
  launch_lstm_step(d, l, xlab, xsrc, hcur, ccur, hn, cn, gout, gstride, B, flag, nullptr, Drop{0u, 0u, 1.0f}, 0, st);
}

struct GreedyWs {
  long F, h, c, h2, c2, hid, part, ctrl, total;
};

GreedyWs greedy_layout(const cfm_rnnt_decoder* d, int B, int T, int J) {
  GreedyWs w{};
  long o = 0;
  auto take = [&](long bytes) { const long at = o; o += round_up(std::max(bytes, 1L), 256); return at; };
  const long lbh = (long)d->L * B * d->H * 4;
  w.F = take((long)B * T * J * 4);
  w.h = take(lbh);
  w.c = take(lbh);
  w.h2 = take(lbh);
  w.c2 = take(lbh);
  w.hid = take((long)B * J * 4);
  const long nblk = (d->V + 1 + 15) / 16;
  w.part = take(nblk * B * (long)sizeof(Part));
  w.ctrl = take(5L * B * 4 + 64);
  w.total = o;
  return w;
}

// training tape: per layer l and step u, gates (B, 4H), c (B, H), h (B, H); then the step labels
struct TrainTape {
  float* base;
  long B, H, S;
  int32_t* xlab;
  float* zero;
  float* gates(int l, int u) const { return base + ((long)l * S + u) * B * 6 * H; }
  float* c(int l, int u) const { return gates(l, u) + B * 4 * H; }
  float* h(int l, int u) const { return gates(l, u) + B * 5 * H; }
};
TrainTape train_tape(const cfm_rnnt_decoder* d, char* tape, int B, int S) {
  TrainTape t;
  t.base = (float*)tape;
  t.B = B; t.H = d->H; t.S = S;
  char* after = tape + (long)d->L * S * B * 6 * d->H * 4;
  t.xlab = (int32_t*)after;
  t.zero = (float*)(after + round_up((long)(S + 1) * B * 4, 256));   // (B, H) zeros: the initial state
  return t;
}
struct BwdWs { long dy, dgates, dh, dc, x, hp, wt, lin, total; };
constexpr int kHhSplits = 16;   // row splits of the recurrent W_hh^T . dgates product
BwdWs bwd_ws(const cfm_rnnt_decoder* d, int B, int S) {
  BwdWs w{};
  long o = 0;
  auto take = [&](long bytes) { const long at = round_up(o, 256); o = at + round_up(std::max(bytes, 1L), 256); return at; };
  const long sbh = (long)S * B * d->H * 4;
  w.dy = take(sbh);
  w.dgates = take(4 * sbh);
  w.dh = take((long)kHhSplits * B * d->H * 4);   // recurrent dh partials (lstm_hh_bwd_kernel)
  w.dc = take((long)B * d->H * 4);
  w.x = take(sbh);
  w.hp = take(sbh);
  w.wt = take(4L * d->H * d->H * 4);              // W_hh^T of the layer (the matrix-core recurrent product)
  w.lin = take((long)cfm_op_linear_backward_ws_size(CFM_COMPUTE_FP32, S * B, d->H, 4 * d->H));
  w.total = round_up(o, 256);
  return w;
}

// W_hh (4H, H) -> W_hh^T (H, 4H), 32x32 LDS tiles
__global__ __launch_bounds__(256) void transpose_whh_kernel(const float* __restrict__ w, int R, int Cc, float* __restrict__ wt) {
  __shared__ float tile[32][33];
  const int r0 = blockIdx.y * 32, c0 = blockIdx.x * 32, tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int k = ty; k < 32; k += 8)
    if (r0 + k < R && c0 + tx < Cc) tile[k][tx] = w[(long)(r0 + k) * Cc + c0 + tx];
  __syncthreads();
  for (int k = ty; k < 32; k += 8)
    if (c0 + k < Cc && r0 + tx < R) wt[(long)(c0 + k) * R + r0 + tx] = tile[tx][k];
}

// The recurrent gradient dh[b][k] = sum_r W_hh[r][k] dgates[b][r] of one step on the matrix cores
// (v_mfma_f32_16x16x4_f32, fp32 sums): block = 16 hidden rows k x 16 batch rows, the 4H-long contraction
// split over 8 waves in 16-wide groups (a float4 of W_hh^T and of dgates per lane and group), partial
// tiles summed in a fixed order through LDS; writes the whole dh (the cell backward reads one part).
template <int NT>
__global__ __launch_bounds__(512) void lstm_hh_bwd_mfma_kernel(const float* __restrict__ dgates,
                                                               const float* __restrict__ whhT, int B, int H,
                                                               float* __restrict__ dh) {
  __shared__ f32x4 part[8][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int k0 = blockIdx.x * 16, b0 = blockIdx.y * 16;
  const int R = 4 * H, G = R / 16;
  const int rr = lane & 15, kq = lane >> 4;
  const float* arow = whhT + (long)min(k0 + rr, H - 1) * R + 4 * kq;
  const int b = min(b0 + rr, B - 1);
  const float* brow = dgates + (long)b * R + 4 * kq;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  float4 wa[NT], xa[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int gi = min(w + 8 * t, G - 1);
    wa[t] = *(const float4*)(arow + gi * 16);
    xa[t] = *(const float4*)(brow + gi * 16);
  }
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    if (w + 8 * t < G) {
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[t].x, xa[t].x, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[t].y, xa[t].y, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[t].z, xa[t].z, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[t].w, xa[t].w, acc, 0, 0, 0);
    }
  }
  part[w][lane] = acc;
  __syncthreads();
  if (w != 0) return;
  f32x4 s = part[0][lane];
#pragma unroll
  for (int ww = 1; ww < 8; ++ww) {
    const f32x4 t = part[ww][lane];
    s[0] += t[0]; s[1] += t[1]; s[2] += t[2]; s[3] += t[3];
  }
  // lane: batch column b0 + (lane & 15), hidden rows k0 + 4 (lane >> 4) + e
  const int bb = b0 + (lane & 15);
  if (bb >= B) return;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int k = k0 + 4 * (lane >> 4) + e;
    if (k < H) dh[(long)bb * H + k] = s[e];
  }
}

// dy[u][b][j] = dg[b][u][j] * dropout'(b, u, j)  (LSTMDropout's output dropout)
__global__ void dg_to_dy_kernel(const float* __restrict__ dg, int B, int S, int H, Drop drop, float* __restrict__ dy) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)S * B * H) return;
  const int j = (int)(i % H);
  const long r = i / H;
  const int b = (int)(r % B), u = (int)(r / B);
  const uint64_t e = ((uint64_t)b * S + u) * H + j;
  dy[i] = dg[e] * drop_mul(drop, e);
}

// LSTM cell backward (gate order i, f, g, o; c = f*c' + i*g, h = o*tanh(c)) for one step:
// dh = dy + the recurrent part (the nparts row-split partials lstm_hh_bwd wrote for the step after this
// one, summed in split order), dc (in/out), dgates (B, 4H) pre-activation gradients
__global__ void lstm_cell_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ gates,
                                     const float* __restrict__ c, const float* __restrict__ cprev, int B, int H,
                                     const float* __restrict__ dhp, int nparts, float* __restrict__ dc,
                                     float* __restrict__ dgates) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * H) return;
  const int b = i / H, j = i - b * H;
  const float* gr = gates + (long)b * 4 * H;
  const float gi = gr[j], gf = gr[H + j], gg = gr[2 * H + j], go = gr[3 * H + j];
  const float ct = c[i], tc = tanhf(ct);
  float rec = 0.0f;
  for (int s = 0; s < nparts; ++s) rec += dhp[(long)s * B * H + i];
  const float dht = dy[i] + rec;
  const float dct = dht * go * (1.0f - tc * tc) + dc[i];
  float* dgr = dgates + (long)b * 4 * H;
  dgr[j] = dct * gg * gi * (1.0f - gi);
  dgr[H + j] = dct * cprev[i] * gf * (1.0f - gf);
  dgr[2 * H + j] = dct * gi * (1.0f - gg * gg);
  dgr[3 * H + j] = dht * tc * go * (1.0f - go);
  dc[i] = dct * gf;
}

// part[s][b][k] = sum over the rows r of split s of W_hh[r][k] * dgates[b][r]  (W_hh the reference
// (4H, H) weight).  Block (column group of 64, split s), 4 waves: the split's dgates [r][16 b] staged in
// LDS, lane = column, wave w takes rows r0 + w, r0 + w + 4, ... (one coalesced W row load and four
// broadcast 16-byte LDS reads per row), 16 batch rows per pass; the 4 waves' sums are added through
// LDS in wave order (deterministic).
constexpr int kHhRows = 4 * 1536 / kHhSplits + 1;   // rows of a split (4H / kHhSplits, H <= 1536)
__global__ __launch_bounds__(256) void lstm_hh_bwd_kernel(const float* __restrict__ dgates,
                                                          const float* __restrict__ whh, int B, int H,
                                                          float* __restrict__ part) {
  __shared__ float4 dgl[kHhRows][4];        // [row - r0][b / 4] for the pass's 16 batch rows
  __shared__ float red[4][16][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int k = blockIdx.x * 64 + lane;
  const int s = blockIdx.y;
  const int R = (4 * H + kHhSplits - 1) / kHhSplits;
  const int r0 = s * R, r1 = min(4 * H, r0 + R);
  const int kc = min(k, H - 1);
  for (int b0 = 0; b0 < B; b0 += 16) {
    const int nb = min(16, B - b0);
    for (int i = threadIdx.x; i < (r1 - r0) * 16; i += 256) {
      const int rr = i >> 4, b = i & 15;
      ((float*)dgl[rr])[b] = b < nb ? dgates[(long)(b0 + b) * 4 * H + r0 + rr] : 0.0f;
    }
    __syncthreads();
    float acc[16];
#pragma unroll
    for (int b = 0; b < 16; ++b) acc[b] = 0.0f;
    for (int r = r0 + w; r < r1; r += 4) {
      const float wv = whh[(long)r * H + kc];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 d4 = dgl[r - r0][q];
        acc[4 * q] = fmaf(wv, d4.x, acc[4 * q]);
        acc[4 * q + 1] = fmaf(wv, d4.y, acc[4 * q + 1]);
        acc[4 * q + 2] = fmaf(wv, d4.z, acc[4 * q + 2]);
        acc[4 * q + 3] = fmaf(wv, d4.w, acc[4 * q + 3]);
      }
    }
#pragma unroll
    for (int b = 0; b < 16; ++b) red[w][b][lane] = acc[b];
    __syncthreads();
    for (int b = w; b < nb; b += 4) {
      const float v = ((red[0][b][lane] + red[1][b][lane]) + red[2][b][lane]) + red[3][b][lane];
      if (k < H) part[((long)s * B + b0 + b) * H + k] = v;
    }
    __syncthreads();
  }
}

// layer-0 input rows: the embedding row of each step's label (zero for the SOS step)
__global__ void gather_emb_kernel(const int32_t* __restrict__ xlab, const float* __restrict__ emb, int S, int B, int H,
                                  int nemb, float* __restrict__ x) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)S * B * H) return;
  const long r = i / H;
  const int j = (int)(i % H);
  const int lab = xlab[r];
  x[i] = lab >= 0 ? emb[(long)min(lab, nemb - 1) * H + j] : 0.0f;
}

// d_embed[label] += dx rows; the blank (padding_idx = V) and SOS rows get none (nn.Embedding padding_idx)
// d(embedding) row v = sum of dx over the steps whose label is v, in step order (deterministic: one
// block column per row, no atomics); the padding row (blank = V) and unused rows come out zero
// d_embed[v] = sum over rows r with xlab[r] == v of dx[r] (r ascending: deterministic).  One block per
// embedding row covering all H columns (<= 6 per thread); the labels are staged through LDS in chunks and
// scanned four at a time, so a block costs ~S*B/4 LDS reads instead of S*B dependent global loads.
constexpr int kEmbCols = 6, kEmbChunk = 8192;
__global__ __launch_bounds__(256) void embed_grad_kernel(const int32_t* __restrict__ xlab, const float* __restrict__ dx,
                                                         int SB, int H, int V, float* __restrict__ demb) {
  __shared__ int4 lab[kEmbChunk / 4];
  const int v = blockIdx.x;
  float acc[kEmbCols];
#pragma unroll
  for (int c = 0; c < kEmbCols; ++c) acc[c] = 0.0f;
  if (v < V) {
    for (int r0 = 0; r0 < SB; r0 += kEmbChunk) {
      const int n = min(kEmbChunk, SB - r0);
      __syncthreads();
      for (int i = threadIdx.x; i < kEmbChunk; i += 256) ((int*)lab)[i] = i < n ? xlab[r0 + i] : -1;
      __syncthreads();
      for (int q = 0; q < (n + 3) / 4; ++q) {
        const int4 l4 = lab[q];
        const int ls[4] = {l4.x, l4.y, l4.z, l4.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if (ls[e] != v) continue;   // block-uniform
          const float* row = dx + (long)(r0 + 4 * q + e) * H;
#pragma unroll
          for (int c = 0; c < kEmbCols; ++c) {
            const int j = threadIdx.x + 256 * c;
            if (j < H) acc[c] += row[j];
          }
        }
      }
    }
  }
#pragma unroll
  for (int c = 0; c < kEmbCols; ++c) {
    const int j = threadIdx.x + 256 * c;
    if (j < H) demb[(long)v * H + j] = acc[c];
  }
}

long predict_ws_bytes(const cfm_rnnt_decoder* d, int B, int U) {
  const long lbh = round_up((long)d->L * B * d->H * 4, 256);
  return 4 * lbh + round_up((long)(U + 2) * B * 4, 256);
}

}  // namespace

extern "C" {

cfm_status cfm_rnnt_decoder_create(int vocab_size, int pred_hidden, int layers, int device, cfm_rnnt_decoder** out) {
  return guarded([&] {
    if (!out) fail(CFM_ERR_INVALID_ARG, "null out");
    *out = nullptr;
    if (vocab_size < 1 || pred_hidden < 4 || pred_hidden > 1536 || pred_hidden % 4 || layers < 1 || layers > 16)
      fail(CFM_ERR_INVALID_ARG, "cfm_rnnt_decoder_create: need vocab_size >= 1, pred_hidden % 4 == 0 in [4, 1536], "
                                "1 <= layers <= 16");
    HIP_OK(hipSetDevice(device));
    set_lds_limits();
    auto* d = new cfm_rnnt_decoder();
    d->V = vocab_size;
    d->H = pred_hidden;
    d->L = layers;
    d->device = device;
    const long H = pred_hidden;
    d->emb_off = 0;
    d->w_off = round_up((long)(vocab_size + 1) * H, 64);
    d->b_off = d->w_off + (long)layers * 4 * H * 2 * H;
    long total = d->b_off + (long)layers * 4 * H;
    static const int xtab_on = [] { const char* e = getenv("CFM_LSTM_XTAB"); return e ? atoi(e) : 1; }();
    d->x_want = xtab_on && H % 16 == 0 && lstm_mfma_nt((int)(H / 16 + 7) / 8);
    hipError_t e = hipMalloc((void**)&d->wbuf, total * sizeof(float));
    if (e == hipSuccess) e = hipHostMalloc((void**)&d->host_flag, 2 * sizeof(int), hipHostMallocDefault);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&d->ev[0], hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&d->ev[1], hipEventDisableTiming);
    if (e != hipSuccess) {
      cfm_rnnt_decoder_destroy(d);
      fail(CFM_ERR_NOMEM, std::string("cfm_rnnt_decoder_create: ") + hipGetErrorString(e));
    }
    *out = d;
  });
}

void cfm_rnnt_decoder_destroy(cfm_rnnt_decoder* d) {
  if (!d) return;
  (void)hipSetDevice(d->device);
  if (d->wbuf) (void)hipFree(d->wbuf);
  if (d->xbuf) (void)hipFree(d->xbuf);
  if (d->host_flag) (void)hipHostFree(d->host_flag);
  for (auto& e : d->ev)
    if (e) (void)hipEventDestroy(e);
  delete d;
}

cfm_status cfm_rnnt_decoder_set_weights(cfm_rnnt_decoder* d, const float* embed, const float* const* w_ih,
                                        const float* const* w_hh, const float* const* b_ih,
                                        const float* const* b_hh, void* stream) {
  return guarded([&] {
    if (!d || !embed || !w_ih || !w_hh || !b_ih || !b_hh) fail(CFM_ERR_INVALID_ARG, "null argument");
    check_device(d);
    hipStream_t st = (hipStream_t)stream;
    const long H = d->H;
    d->x_ready = false;
    HIP_OK(hipMemcpyAsync(d->wbuf + d->emb_off, embed, (size_t)(d->V + 1) * H * sizeof(float),
                          hipMemcpyDeviceToDevice, st));
    for (int l = 0; l < d->L; ++l) {
      if (!w_ih[l] || !w_hh[l] || !b_ih[l] || !b_hh[l]) fail(CFM_ERR_INVALID_ARG, "null LSTM parameter");
      const long n = 4 * H * 2 * H;
      hipLaunchKernelGGL(pack_lstm_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, w_ih[l], w_hh[l],
                         b_ih[l], b_hh[l], (int)H, d->wbuf + d->w_off + (long)l * n, d->wbuf + d->b_off + l * 4 * H);
    }
    HIP_OK(hipGetLastError());
  });
}

size_t cfm_rnnt_decoder_predict_workspace_size(const cfm_rnnt_decoder* d, int B, int U) {
  if (!d || B < 0 || U < 0) return 0;
  return (size_t)predict_ws_bytes(d, B, std::max(U, 1));
}

cfm_status cfm_rnnt_decoder_predict(cfm_rnnt_decoder* d, const int64_t* y, int B, int U, int add_sos, const float* h0,
                                    const float* c0, float* g, float* h_out, float* c_out, void* workspace,
                                    size_t workspace_bytes, void* stream) {
  return guarded([&] {
    if (!d || !g || !h_out || !c_out) fail(CFM_ERR_INVALID_ARG, "null argument");
    if (B < 0 || U < 0 || (y && U < 1)) fail(CFM_ERR_INVALID_ARG, "cfm_rnnt_decoder_predict: bad B / U");
    if (B == 0) return;
    check_device(d);
    const int Ue = y ? U : 1;
    const int S = Ue + (add_sos ? 1 : 0);
    if (!workspace || (long)workspace_bytes < predict_ws_bytes(d, B, Ue))
      fail(CFM_ERR_WORKSPACE, "cfm_rnnt_decoder_predict: workspace too small");
    hipStream_t st = (hipStream_t)stream;
    const long lbh = (long)d->L * B * d->H;
    const long lbh_b = round_up(lbh * 4, 256);
    char* ws = (char*)workspace;
    float* hs[2] = {(float*)ws, (float*)(ws + 2 * lbh_b)};
    float* cs[2] = {(float*)(ws + lbh_b), (float*)(ws + 3 * lbh_b)};
    int32_t* xlab = (int32_t*)(ws + 4 * lbh_b);
    if (h0) HIP_OK(hipMemcpyAsync(hs[0], h0, lbh * 4, hipMemcpyDeviceToDevice, st));
    else HIP_OK(hipMemsetAsync(hs[0], 0, lbh * 4, st));
    if (c0) HIP_OK(hipMemcpyAsync(cs[0], c0, lbh * 4, hipMemcpyDeviceToDevice, st));
    else HIP_OK(hipMemsetAsync(cs[0], 0, lbh * 4, st));
    hipLaunchKernelGGL(predict_labels_kernel, dim3((unsigned)(((long)S * B + 255) / 256)), dim3(256), 0, st, y, B,
                       U, S, add_sos ? 1 : 0, d->V + 1, xlab);
    ensure_xtab(d, st);
    const long bh = (long)B * d->H;
    int cur = 0;
    for (int u = 0; u < S; ++u) {
      const int nx = cur ^ 1;
      for (int l = 0; l < d->L; ++l) {
        const bool top = l == d->L - 1;
        lstm_layer(d, l, xlab + (long)u * B, l ? hs[nx] + (l - 1) * bh : nullptr, hs[cur] + l * bh, cs[cur] + l * bh,
                   hs[nx] + l * bh, cs[nx] + l * bh, top ? g + (long)u * d->H : nullptr, (long)S * d->H, B, nullptr,
                   st);
      }
      cur = nx;
    }
    HIP_OK(hipMemcpyAsync(h_out, hs[cur], lbh * 4, hipMemcpyDeviceToDevice, st));
    HIP_OK(hipMemcpyAsync(c_out, cs[cur], lbh * 4, hipMemcpyDeviceToDevice, st));
    HIP_OK(hipGetLastError());
  });
}

// ---- training: BPTT through the prediction network (rnnt.py:190-283 under autograd) -------------
size_t cfm_rnnt_decoder_train_tape_size(const cfm_rnnt_decoder* d, int B, int U, int add_sos) {
  if (!d || B < 1 || U < 1) return 0;
  const long S = U + (add_sos ? 1 : 0);
  return (size_t)(d->L * S * (long)B * 6 * d->H * 4 + round_up((S + 1) * (long)B * 4, 256) + (long)B * d->H * 4 + 256);
}

cfm_status cfm_rnnt_decoder_train_forward(cfm_rnnt_decoder* d, const int64_t* y, int B, int U, int add_sos,
                                          float dropout, uint64_t seed, float* g, void* tape, size_t tape_bytes,
                                          void* stream) {
  return guarded([&] {
    if (!d || !y || !g || !tape) fail(CFM_ERR_INVALID_ARG, "null argument");
    if (B < 1 || U < 1) fail(CFM_ERR_INVALID_ARG, "cfm_rnnt_decoder_train_forward: B, U >= 1");
    if (tape_bytes < cfm_rnnt_decoder_train_tape_size(d, B, U, add_sos)) fail(CFM_ERR_WORKSPACE, "tape too small");
    check_device(d);
    hipStream_t st = (hipStream_t)stream;
    const int H = d->H, L = d->L, S = U + (add_sos ? 1 : 0);
    const long bh = (long)B * H;
    TrainTape tp = train_tape(d, (char*)tape, B, S);
    hipLaunchKernelGGL(predict_labels_kernel, dim3((unsigned)(((long)S * B + 255) / 256)), dim3(256), 0, st, y, B, U, S,
                       add_sos ? 1 : 0, d->V + 1, tp.xlab);
    HIP_OK(hipMemsetAsync(tp.zero, 0, (size_t)bh * 4, st));
    const Drop gdrop = make_drop(dropout, seed, 2);
    for (int u = 0; u < S; ++u)
      for (int l = 0; l < L; ++l) {
        const bool top = l == L - 1;
        const float* hprev = u ? tp.h(l, u - 1) : tp.zero;
        const float* cprev = u ? tp.c(l, u - 1) : tp.zero;
        launch_lstm_step(d, l, tp.xlab + (long)u * B, l ? tp.h(l - 1, u) : nullptr, hprev, cprev, tp.h(l, u), tp.c(l, u),
                         top ? g + (long)u * H : nullptr, (long)S * H, B, (const int*)nullptr, tp.gates(l, u), gdrop, u,
                         st);
      }
    HIP_OK(hipGetLastError());
  });
}

size_t cfm_rnnt_decoder_backward_workspace_size(const cfm_rnnt_decoder* d, int B, int U, int add_sos) {
  if (!d || B < 1 || U < 1) return 0;
  const int S = U + (add_sos ? 1 : 0);
  return (size_t)bwd_ws(d, B, S).total;
}

cfm_status cfm_rnnt_decoder_backward(cfm_rnnt_decoder* d, const int64_t* y, int B, int U, int add_sos, float dropout,
                                     uint64_t seed, const void* tape, const float* dg, const float* const* w_ih,
                                     const float* const* w_hh, float* d_embed, float* const* dw_ih,
                                     float* const* dw_hh, float* const* db_ih, float* const* db_hh, void* workspace,
                                     size_t workspace_bytes, void* stream) {
  return guarded([&] {
    if (!d || !tape || !dg || !w_ih || !w_hh) fail(CFM_ERR_INVALID_ARG, "null argument");
    if (B < 1 || U < 1) fail(CFM_ERR_INVALID_ARG, "cfm_rnnt_decoder_backward: B, U >= 1");
    check_device(d);
    const int H = d->H, L = d->L, S = U + (add_sos ? 1 : 0);
    const BwdWs w = bwd_ws(d, B, S);
    if (!workspace || (long)workspace_bytes < w.total) fail(CFM_ERR_WORKSPACE, "workspace too small");
    hipStream_t st = (hipStream_t)stream;
    char* ws = (char*)workspace;
    TrainTape tp = train_tape(d, (char*)tape, B, S);
    float* dy = (float*)(ws + w.dy);          // (S, B, H): the current layer's output gradient
    float* dgt = (float*)(ws + w.dgates);     // (S, B, 4H)
    float* dh = (float*)(ws + w.dh);          // (kHhSplits, B, H) recurrent dh partials
    float* dc = (float*)(ws + w.dc);          // (B, H) recurrent dc
    float* xin = (float*)(ws + w.x);          // (S, B, H) the layer's input rows
    float* hpv = (float*)(ws + w.hp);         // (S, B, H) h_{u-1}
    char* lws = ws + w.lin;
    const size_t lws_bytes = (size_t)(w.total - w.lin);
    const long n = (long)S * B * H;
    const Drop gdrop = make_drop(dropout, seed, 2);
    hipLaunchKernelGGL(dg_to_dy_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, dg, B, S, H, gdrop, dy);
    auto lin_bwd = [&](const float* x, const float* wt, float* dx, float* dw, float* db) {
      const cfm_status r = cfm_op_linear_backward(CFM_COMPUTE_FP32, x, S * B, H, wt, 4 * H, dgt, dx, dw, db, lws,
                                                  lws_bytes, st);
      if (r != CFM_OK) fail(r, std::string("prediction-net backward: ") + cfm_last_error());
    };
    // the recurrent product on the matrix cores (CFM_LSTM_MFMA=0: 16 VALU row splits)
    static const int mfma = [] { const char* e = getenv("CFM_LSTM_MFMA"); return e ? atoi(e) : 1; }();
    const int NT = (4 * H / 16 + 7) / 8;
    const bool hh_mfma = mfma && H % 16 == 0 && (NT == 10 || NT == 16 || NT == 20);
    float* whhT = (float*)(ws + w.wt);
    for (int l = L - 1; l >= 0; --l) {
      HIP_OK(hipMemsetAsync(dc, 0, (size_t)B * H * 4, st));
      if (hh_mfma)
        hipLaunchKernelGGL(transpose_whh_kernel, dim3((unsigned)((H + 31) / 32), (unsigned)((4 * H + 31) / 32)), dim3(256),
                           0, st, w_hh[l], 4 * H, H, whhT);
      for (int u = S - 1; u >= 0; --u) {
        hipLaunchKernelGGL(lstm_cell_bwd_kernel, dim3((unsigned)((B * H + 255) / 256)), dim3(256), 0, st,
                           dy + (long)u * B * H, tp.gates(l, u), tp.c(l, u), u ? tp.c(l, u - 1) : tp.zero, B, H,
                           (const float*)dh, u == S - 1 ? 0 : (hh_mfma ? 1 : kHhSplits), dc, dgt + (long)u * B * 4 * H);
        if (u > 0 && hh_mfma) {
          const dim3 grid((unsigned)((H + 15) / 16), (unsigned)((B + 15) / 16));
          const float* dgu = dgt + (long)u * B * 4 * H;
          if (NT == 10) hipLaunchKernelGGL(lstm_hh_bwd_mfma_kernel<10>, grid, dim3(512), 0, st, dgu, whhT, B, H, dh);
          else if (NT == 16) hipLaunchKernelGGL(lstm_hh_bwd_mfma_kernel<16>, grid, dim3(512), 0, st, dgu, whhT, B, H, dh);
          else hipLaunchKernelGGL(lstm_hh_bwd_mfma_kernel<20>, grid, dim3(512), 0, st, dgu, whhT, B, H, dh);
        } else if (u > 0) {
          hipLaunchKernelGGL(lstm_hh_bwd_kernel, dim3((unsigned)((H + 63) / 64), kHhSplits), dim3(256), 0, st,
                             dgt + (long)u * B * 4 * H, w_hh[l], B, H, dh);
        }
      }
      // the layer's input rows and h_{u-1} rows (S, B, H)
      if (l == 0)
        hipLaunchKernelGGL(gather_emb_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, tp.xlab, d->emb(), S, B,
                           H, d->V + 1, xin);
      else   // the tape's h rows of layer l-1 (one (B, H) block per step, 6BH apart)
        HIP_OK(hipMemcpy2DAsync(xin, (size_t)B * H * 4, tp.h(l - 1, 0), (size_t)6 * B * H * 4, (size_t)B * H * 4, S,
                                hipMemcpyDeviceToDevice, st));
      HIP_OK(hipMemsetAsync(hpv, 0, (size_t)B * H * 4, st));
      if (S > 1)
        HIP_OK(hipMemcpy2DAsync(hpv + (long)B * H, (size_t)B * H * 4, tp.h(l, 0), (size_t)6 * B * H * 4,
                                (size_t)B * H * 4, S - 1, hipMemcpyDeviceToDevice, st));
      // W_ih (+ both biases) and the input gradient; W_hh
      lin_bwd(xin, w_ih[l], dy, dw_ih ? dw_ih[l] : nullptr, db_ih ? db_ih[l] : nullptr);
      lin_bwd(hpv, w_hh[l], nullptr, dw_hh ? dw_hh[l] : nullptr, nullptr);
      if (db_hh && db_hh[l] && db_ih && db_ih[l])
        HIP_OK(hipMemcpyAsync(db_hh[l], db_ih[l], (size_t)4 * H * 4, hipMemcpyDeviceToDevice, st));
      else if (db_hh && db_hh[l])
        fail(CFM_ERR_INVALID_ARG, "db_hh needs db_ih (the two bias gradients are equal)");
    }
    // dy now holds d(embedding rows) (S, B, H): summed per label row (not blank = padding_idx)
    if (d_embed) {
      hipLaunchKernelGGL(embed_grad_kernel, dim3((unsigned)(d->V + 1)), dim3(256), 0, st,
                         tp.xlab, dy, S * B, H, d->V, d_embed);
    }
    HIP_OK(hipGetLastError());
  });
}

size_t cfm_rnnt_greedy_workspace_size(const cfm_rnnt_decoder* d, int B, int T, int J) {
  if (!d || B < 0 || T < 0 || J < 1) return 0;
  return (size_t)greedy_layout(d, B, T, J).total;
}

cfm_status cfm_rnnt_greedy_decode(cfm_rnnt_decoder* d, const float* enc_bdt, const int64_t* enc_len, int B, int T,
                                  int D1, int J, const float* w_enc, const float* b_enc, const float* w_pred,
                                  const float* b_pred, const float* w_out, const float* b_out, int activation,
                                  int max_symbols, int log_normalize, int sos_until_label, int32_t* tokens,
                                  int32_t* timesteps, int32_t* ntok, double* scores, float* h_out, float* c_out,
                                  void* workspace, size_t workspace_bytes, void* stream) {
  return guarded([&] {
    if (!d || !enc_bdt || !enc_len || !w_enc || !b_enc || !w_pred || !b_pred || !w_out || !b_out || !tokens ||
        !timesteps || !ntok || !scores || !h_out || !c_out)
      fail(CFM_ERR_INVALID_ARG, "null argument");
    if (B < 0 || T < 0 || D1 < 1 || J < 4 || J > 3072 || J % 4 || D1 > (1 << 20) || max_symbols < 1)
      fail(CFM_ERR_INVALID_ARG, "cfm_rnnt_greedy_decode: need D1 >= 1, J % 4 == 0 in [4, 3072], max_symbols >= 1");
    if (((uintptr_t)w_pred | (uintptr_t)w_out) & 15) fail(CFM_ERR_INVALID_ARG, "joint weights must be 16-byte aligned");
    if (activation < CFM_JOINT_RELU || activation > CFM_JOINT_TANH) fail(CFM_ERR_INVALID_ARG, "bad activation");
    check_device(d);
    hipStream_t st = (hipStream_t)stream;
    const long lbh = (long)d->L * B * d->H;
    if (B == 0) return;
    if (T == 0) {
      HIP_OK(hipMemsetAsync(ntok, 0, (size_t)B * 4, st));
      HIP_OK(hipMemsetAsync(scores, 0, (size_t)B * 8, st));
      HIP_OK(hipMemsetAsync(h_out, 0, lbh * 4, st));
      HIP_OK(hipMemsetAsync(c_out, 0, lbh * 4, st));
      HIP_OK(hipStreamSynchronize(st));
      return;
    }
    const GreedyWs w = greedy_layout(d, B, T, J);
    if (!workspace || (long)workspace_bytes < w.total) fail(CFM_ERR_WORKSPACE, "cfm_rnnt_greedy_decode: workspace too small");
    char* ws = (char*)workspace;
    float* F = (float*)(ws + w.F);
    float* hS = (float*)(ws + w.h);
    float* cS = (float*)(ws + w.c);
    float* h2 = (float*)(ws + w.h2);
    float* c2 = (float*)(ws + w.c2);
    float* hid = (float*)(ws + w.hid);
    Part* part = (Part*)(ws + w.part);
    int32_t* ci = (int32_t*)(ws + w.ctrl);
    Ctrl ct{ci, ci + B, ci + 2 * B, ci + 3 * B, ci + 4 * B, (int*)(ci + 5 * B)};
    const int N = d->V + 1, H = d->H;
    const int nblk = (N + 15) / 16;
    const long cap = (long)T * max_symbols;

    // f = enc W_enc^T + b_enc for every frame (rnnt.py:981 joint's enc projection), state and control init
    hipLaunchKernelGGL(enc_proj_kernel, dim3((unsigned)(((long)B * T + 63) / 64), (J + 63) / 64), dim3(256), 0, st,
                       enc_bdt, w_enc, b_enc, B, T, D1, J, F);
    // hS and cS are adjacent in the workspace: zero both in one pass
    ensure_xtab(d, st);
    hipLaunchKernelGGL(greedy_init_kernel, dim3((unsigned)std::max<long>(1, std::min<long>((2 * lbh + 255) / 256, 1024))),
                       dim3(256), 0, st, enc_len, B, T, ct, ntok, scores, hS, (long)((char*)h2 - (char*)hS) / 4);
    HIP_OK(hipGetLastError());
    const long bh = (long)B * H;
    auto iteration = [&]() {
      for (int l = 0; l < d->L; ++l)
        lstm_layer(d, l, ct.xlab, l ? h2 + (l - 1) * bh : nullptr, hS + l * bh, cS + l * bh, h2 + l * bh, c2 + l * bh,
                   nullptr, 0, B, ct.flag, st);
      const dim3 gh((J + 15) / 16, (B + RB - 1) / RB);
      hipLaunchKernelGGL(joint_hidden_kernel, gh, dim3(256), (size_t)(RB * H + RED) * 4, st, w_pred, b_pred,
                         h2 + (long)(d->L - 1) * bh, F, ct.t, T, B, H, J, activation, hid, ct.flag);
      const dim3 gl(nblk, (B + RB - 1) / RB);
      hipLaunchKernelGGL(joint_logits_kernel, gl, dim3(256), (size_t)(RB * J + RED + 16 * RB) * 4, st, w_out, b_out,
                         hid, B, J, N, part, ct.flag);
      hipLaunchKernelGGL(greedy_commit_kernel, dim3(B), dim3(64), 0, st, part, nblk, B, T, enc_len, d->V,
                         max_symbols, log_normalize, sos_until_label, ct, tokens, timesteps, cap, ntok, scores, hS, cS, h2, c2, d->L, H);
    };
    // Every iteration advances each active utterance by one frame or one label, so T * (max_symbols + 1)
    // iterations always suffice.  Chunks of CH iterations are queued ahead; the done-flag copied after
    // chunk i is read while chunk i + 1 runs (finished utterances make the extra kernels no-ops).
    constexpr int CH = 8;
    const long max_iter = (long)T * (max_symbols + 1) + 1;
    long done_iter = 0;
    int pending = -1;
    for (int chunk = 0; done_iter < max_iter; ++chunk) {
      for (int i = 0; i < CH && done_iter < max_iter; ++i, ++done_iter) iteration();
      hipLaunchKernelGGL(greedy_flag_kernel, dim3(1), dim3(256), 0, st, ct.active, B, ct.flag);
      const int slot = chunk & 1;
      HIP_OK(hipMemcpyAsync(d->host_flag + slot, ct.flag, sizeof(int), hipMemcpyDeviceToHost, st));
      HIP_OK(hipEventRecord(d->ev[slot], st));
      if (pending >= 0) {
        HIP_OK(hipEventSynchronize(d->ev[pending]));
        if (d->host_flag[pending] == 0) break;
      }
      pending = slot;
    }
    HIP_OK(hipGetLastError());
    HIP_OK(hipMemcpyAsync(h_out, hS, lbh * 4, hipMemcpyDeviceToDevice, st));
    HIP_OK(hipMemcpyAsync(c_out, cS, lbh * 4, hipMemcpyDeviceToDevice, st));
    HIP_OK(hipStreamSynchronize(st));
  });
}

}  // extern "C"
