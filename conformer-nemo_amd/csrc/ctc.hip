// CTC head (ConvASRDecoder, conv_asr.py:397-444) and CTC loss (CTCLoss, ctc.py:25-70 over
// torch.nn.functional.ctc_loss), forward and backward, for gfx950.  SURVEY §8 row a17.
//
// Head forward:   enc (B, D, T) -> rows (B*T, D) compute type -> MFMA GEMM (+bias, fp32 logits)
//                 -> row log_softmax (+ argmax)                               = conv_asr.py:444
// Head backward:  dlogits = dlp - softmax * sum(dlp)   (log_softmax backward, one wave per row)
//                 denc    = dlogits . W       (GEMM on packed W^T)
//                 dW      = dlogits^T . enc   (GEMM on the transposed operands, K = B*T)
//                 dbias   = column sums of dlogits (fixed-order reduction: deterministic)
// The operand relayouts (pack_matrix) and column sums are shared with backward.hip.
// CTC loss:       one wave per utterance walks the 2U+1 extended states (blank, l1, blank, l2, ...,
//                 blank), states held in registers (SPL per lane, shuffles for the s-1/s-2 links):
//                 alpha recursion forward (alphas kept in the workspace), beta recursion backward
//                 fused with the posterior per class and the gradient in torch's convention
//                 grad[t][c] = exp(lp[t][c]) - exp(log sum_{s: l'_s = c} alpha_t(s) beta_t(s) + nll - lp[t][c])
//                 (aten LossCTC: the gradient it returns w.r.t. log_probs), 0 beyond the input length.
#include <algorithm>
#include <cmath>
#include <memory>
#include <type_traits>

#include "../../include/cfm_ctc.h"
#include "cfm_abi.h"
#include "cfm_common.h"
#include "cfm_kernels.h"

namespace cfm {
namespace {

constexpr float NEG_INF = -INFINITY;

CFM_DEV float lse2(float a, float b) {
  const float m = fmaxf(a, b);
  if (m == NEG_INF) return NEG_INF;
  return m + logf(expf(a - m) + expf(b - m));
}
CFM_DEV float lse3(float a, float b, float c) {
  const float m = fmaxf(fmaxf(a, b), c);
  if (m == NEG_INF) return NEG_INF;
  return m + logf(expf(a - m) + expf(b - m) + expf(c - m));
}
CFM_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// ---- relayouts -------------------------------------------------------------------------------

// (B, D, T) fp32 -> rows[(b*T + t)][d] (ld) compute type (the GEMM A operand of the head).
template <typename T>
__global__ __launch_bounds__(256) void bdt_rows_kernel(const float* __restrict__ x, int D, int Tn, T* __restrict__ dst,
                                                       long ld) {
  __shared__ float tile[32][33];
  const int b = blockIdx.z, d0 = blockIdx.y * 32, t0 = blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int k = ty; k < 32; k += 8) {
    const int d = d0 + k, t = t0 + tx;
    tile[k][tx] = (d < D && t < Tn) ? x[((long)b * D + d) * Tn + t] : 0.0f;
  }
  __syncthreads();
  for (int k = ty; k < 32; k += 8) {
    const int t = t0 + k, d = d0 + tx;
    if (t < Tn && d < D) st_f<T>(dst + ((long)b * Tn + t) * ld + d, tile[tx][k]);
  }
}

// (B, D, T) fp32 -> dst[d][b*T + t] (ld, compute type): the W operand of the weight-gradient GEMM
// (rows = d, K = b*T + t).  Rows up to rows_pad and columns up to ld are zero-filled.
template <typename T>
__global__ __launch_bounds__(256) void bdt_dm_kernel(const float* __restrict__ x, int B, int D, int Tn,
                                                     T* __restrict__ dst, long ld, int rows_pad) {
  const int d = blockIdx.y;
  const long M = (long)B * Tn;
  for (long m = blockIdx.x * 256L + threadIdx.x; m < ld; m += (long)gridDim.x * 256) {
    float v = 0.0f;
    if (d < D && m < M) {
      const long b = m / Tn, t = m - b * Tn;
      v = x[(b * D + d) * Tn + t];
    }
    st_f<T>(dst + (long)d * ld + m, v);
  }
  (void)rows_pad;
}

// ---- log_softmax over classes, one wave per row ------------------------------------------------
template <int CPL>
__global__ __launch_bounds__(256) void log_softmax_kernel(const float* __restrict__ logits, long ldl, int M, int C,
                                                          float* __restrict__ out, int32_t* __restrict__ argmax) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= M) return;
  const float* x = logits + (long)row * ldl;
  float v[CPL];
  float m = NEG_INF;
  int am = 0;
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    const int c = lane + 64 * i;
    const float t = x[min(c, C - 1)];
    v[i] = c < C ? t : NEG_INF;
    if (v[i] > m) { m = v[i]; am = c; }   // first maximum within the lane (c increasing)
  }
  // argmax with torch's tie rule (first index): reduce (value, index)
  float bm = m;
  int bi = am;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const float om = __shfl_xor(bm, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (om > bm || (om == bm && oi < bi)) { bm = om; bi = oi; }
  }
  float s = 0.0f;
#pragma unroll
  for (int i = 0; i < CPL; ++i) s += (lane + 64 * i < C) ? expf(v[i] - bm) : 0.0f;
  const float lz = bm + logf(wave_sum(s));
  float* o = out + (long)row * C;
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    const int c = lane + 64 * i;
    if (c < C) o[c] = v[i] - lz;
  }
  if (argmax && lane == 0) argmax[row] = bi;
}

// log_softmax backward: g[m][c] = dlp[m][c] - exp(lp[m][c]) * sum_c dlp[m][c]   (fp32 rows)
template <int CPL>
__global__ __launch_bounds__(256) void log_softmax_bwd_kernel(const float* __restrict__ lp,
                                                              const float* __restrict__ dlp, int M, int C,
                                                              float* __restrict__ g) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= M) return;
  const float* l = lp + (long)row * C;
  const float* d = dlp + (long)row * C;
  float dv[CPL], lv[CPL];
  float s = 0.0f;
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    const int c = min(lane + 64 * i, C - 1);
    dv[i] = d[c];
    lv[i] = l[c];
    if (lane + 64 * i < C) s += dv[i];
  }
  s = wave_sum(s);
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    const int c = lane + 64 * i;
    if (c < C) g[(long)row * C + c] = dv[i] - expf(lv[i]) * s;
  }
}

// ---- CTC ---------------------------------------------------------------------------------------
struct CtcArgs {
  const float* lp; const int32_t* tgt; const int32_t* ilen; const int32_t* tlen;
  int B, T, C, U, blank, zero_inf;
  float scale;
  float* E;       // [B][T][U+1]: emissions of the extended classes (0 = blank, 1 + k = label k)
  float* A;       // [B][T][S]: log alphas, S = 2U + 1
  float* Bt;      // [B][T][S]: log betas (gradient only)
  int32_t* fl;    // [B][U]: label k is the first occurrence of its class (gradient only)
  int32_t* nx;    // [B][U]: next k' > k with the same class, -1 none
  float* nll; float* grad;
  uint8_t* dead;  // [B]: 1 where zero_infinity zeroed an infinite loss (its gradient is 0 too)
};

// E[b][t][k'] = lp[b][t][class(k')]
__global__ __launch_bounds__(256) void ctc_gather_kernel(CtcArgs a) {
  const int b = blockIdx.y;
  const int K1 = a.U + 1;
  const long n = (long)a.T * K1;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const int t = (int)(i / K1), k = (int)(i - (long)t * K1);
    const int c = k == 0 ? a.blank : a.tgt[(long)b * a.U + min(k - 1, a.U - 1)];
    a.E[((long)b * a.T + t) * K1 + k] = a.lp[((long)b * a.T + t) * a.C + min(max(c, 0), a.C - 1)];
  }
}

// state s of the extended label sequence: emission column and whether the s-2 link exists
CFM_DEV int ctc_ecol(int s) { return (s & 1) ? 1 + (s >> 1) : 0; }

template <int SPL>
CFM_DEV void ctc_alpha_run(const CtcArgs& a) {
  const int b = blockIdx.x, lane = threadIdx.x;
  const int Tb = min(a.ilen[b], a.T), Ub = min(a.tlen[b], a.U), S = 2 * Ub + 1;
  const int K1 = a.U + 1;
  const int32_t* tg = a.tgt + (long)b * a.U;
  const float* Eb = a.E + (long)b * a.T * K1;
  float* Ab = a.A + (long)b * a.T * (2 * a.U + 1);
  int col[SPL];
  bool skip[SPL];
#pragma unroll
  for (int j = 0; j < SPL; ++j) {
    const int s = lane * SPL + j;
    col[j] = s < S ? ctc_ecol(s) : 0;
    skip[j] = (s < S) && (s & 1) && s >= 3 && tg[(s >> 1)] != tg[(s >> 1) - 1];
  }
  float al[SPL];
#pragma unroll
  for (int j = 0; j < SPL; ++j) al[j] = NEG_INF;
  for (int t = 0; t < Tb; ++t) {
    float e[SPL];
#pragma unroll
    for (int j = 0; j < SPL; ++j) e[j] = Eb[(long)t * K1 + col[j]];
    // neighbours s-1, s-2 of this lane's first states live in the previous lane
    const float up1 = __shfl_up(al[SPL - 1], 1, 64);
    const float up2 = __shfl_up(SPL >= 2 ? al[SPL - 2] : NEG_INF, 1, 64);
    const float p1l = lane == 0 ? NEG_INF : up1, p2l = lane == 0 ? NEG_INF : up2;
    float nw[SPL];
#pragma unroll
    for (int j = 0; j < SPL; ++j) {
      const int s = lane * SPL + j;
      float v;
      if (t == 0) {
        v = (s <= 1 && s < S) ? e[j] : NEG_INF;
      } else {
        const float p1 = j >= 1 ? al[j - 1] : p1l;
        const float p2 = j >= 2 ? al[j - 2] : (j == 1 ? p1l : p2l);
        v = s < S ? e[j] + lse3(al[j], p1, skip[j] ? p2 : NEG_INF) : NEG_INF;
      }
      nw[j] = v;
    }
#pragma unroll
    for (int j = 0; j < SPL; ++j) {
      al[j] = nw[j];
      const int s = lane * SPL + j;
      if (s < S) Ab[(long)t * S + s] = al[j];
    }
  }
  // nll = -lse(alpha_{T-1}(S-1), alpha_{T-1}(S-2))
  float fin = NEG_INF;
#pragma unroll
  for (int j = 0; j < SPL; ++j) {
    const int s = lane * SPL + j;
    if (Tb > 0 && (s == S - 1 || (S >= 2 && s == S - 2))) fin = lse2(fin, al[j]);
  }
  const float m = wave_max(fin);
  float sum = m == NEG_INF ? 0.0f : expf(fin - m);
  sum = wave_sum(sum);
  if (lane == 0) {
    float nll = m == NEG_INF ? INFINITY : -(m + logf(sum));
    const bool dead = a.zero_inf && isinf(nll);
    a.nll[b] = dead ? 0.0f : nll;
    a.dead[b] = dead ? 1 : 0;
  }
}

// The beta recursion alone (gradient): log betas into a.Bt, plus the per-utterance label bookkeeping
// the posterior kernel needs (a.fl / a.nx).  Independent of the alphas, so it runs beside them.
template <int SPL>
CFM_DEV void ctc_beta_run(const CtcArgs& a) {
  const int b = blockIdx.x, lane = threadIdx.x;
  const int Tb = min(a.ilen[b], a.T), Ub = min(a.tlen[b], a.U), S = 2 * Ub + 1;
  const int K1 = a.U + 1;
  const int32_t* tg = a.tgt + (long)b * a.U;
  for (int k = lane; k < Ub; k += 64) {
    const int c = tg[k];
    int first = 1, nk = -1;
    for (int k2 = 0; k2 < k; ++k2) first &= tg[k2] != c;
    for (int k2 = Ub - 1; k2 > k; --k2)
      if (tg[k2] == c) nk = k2;
    a.fl[(long)b * a.U + k] = first;
    a.nx[(long)b * a.U + k] = nk;
  }
  if (Tb <= 0) return;
  const float* Eb = a.E + (long)b * a.T * K1;
  float* Bb = a.Bt + (long)b * a.T * (2 * a.U + 1);
  int col[SPL];
  bool skipn[SPL];   // the s -> s+2 link of beta (exists iff state s+2 has its s-2 link)
#pragma unroll
  for (int j = 0; j < SPL; ++j) {
    const int s = lane * SPL + j;
    col[j] = s < S ? ctc_ecol(s) : 0;
    const int s2 = s + 2;
    skipn[j] = (s2 < S) && (s2 & 1) && s2 >= 3 && tg[(s2 >> 1)] != tg[(s2 >> 1) - 1];
  }
  float bt[SPL];
#pragma unroll
  for (int j = 0; j < SPL; ++j) bt[j] = NEG_INF;
  float e[SPL];
#pragma unroll
  for (int j = 0; j < SPL; ++j) e[j] = Eb[(long)(Tb - 1) * K1 + col[j]];
  for (int t = Tb - 1; t >= 0; --t) {
    float e_n[SPL];
    const int tn = max(t - 1, 0);
#pragma unroll
    for (int j = 0; j < SPL; ++j) e_n[j] = Eb[(long)tn * K1 + col[j]];
    const float dn1 = __shfl_down(bt[0], 1, 64);
    const float dn2 = __shfl_down(SPL >= 2 ? bt[1] : NEG_INF, 1, 64);
    const float n1l = lane == 63 ? NEG_INF : dn1, n2l = lane == 63 ? NEG_INF : dn2;
    float nw[SPL];
#pragma unroll
    for (int j = 0; j < SPL; ++j) {
      const int s = lane * SPL + j;
      float v;
      if (t == Tb - 1) {
        v = (s < S && s >= S - 2) ? e[j] : NEG_INF;
      } else {
        const float q1 = j + 1 < SPL ? bt[j + 1] : n1l;
        const float q2 = j + 2 < SPL ? bt[j + 2] : (j + 1 < SPL ? n1l : n2l);
        v = s < S ? e[j] + lse3(bt[j], q1, skipn[j] ? q2 : NEG_INF) : NEG_INF;
      }
      nw[j] = v;
    }
#pragma unroll
    for (int j = 0; j < SPL; ++j) {
      bt[j] = nw[j];
      const int s = lane * SPL + j;
      if (s < S) Bb[(long)t * S + s] = bt[j];
      e[j] = e_n[j];
    }
  }
}

// blockIdx.y == 0: alphas + nll; == 1: betas (gradient launches only)
template <int SPL>
__global__ __launch_bounds__(64) void ctc_lattice_kernel(CtcArgs a) {
  if (blockIdx.y == 0) ctc_alpha_run<SPL>(a);
  else ctc_beta_run<SPL>(a);
}

// grad[b][t][c] = scale * exp(lp) for t < Tb (0 beyond, and 0 for zero_infinity'd utterances);
// the posterior terms of the target classes are subtracted by ctc_post_kernel afterwards.
__global__ __launch_bounds__(256) void ctc_grad_base_kernel(CtcArgs a) {
  const int b = blockIdx.y;
  const int Tb = min(a.ilen[b], a.T);
  const bool dead = a.dead[b] != 0;
  const long n = (long)a.T * a.C;
  const float* lpb = a.lp + (long)b * n;
  float* gb = a.grad + (long)b * n;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const int t = (int)(i / a.C);
    gb[i] = (t < Tb && !dead) ? a.scale * expf(lpb[i]) : 0.0f;
  }
}

// Posterior terms of the target classes, one wave per (b, t) (after ctc_grad_base_kernel): with
// v[s] = alpha_t(s) + beta_t(s), grad[b][t][blank] = scale * (exp(lp) - exp(lse_even(v) + nll - lp)) and
// for each class c of the labels the same with the lse over the odd states of every k with label c
// (the first occurrence of the class writes it, walking the nx chain) - the arithmetic of the fused beta
// kernel this replaces, moved out of the serial recursion.
__global__ __launch_bounds__(256) void ctc_post_kernel(CtcArgs a) {
  extern __shared__ float vsm[];   // [4 waves][S]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int b = blockIdx.y, t = blockIdx.x * 4 + w;
  const int Tb = min(a.ilen[b], a.T), Ub = min(a.tlen[b], a.U), S = 2 * Ub + 1;
  if (a.dead[b] || t >= Tb) return;
  const int Sld = 2 * a.U + 1;
  float* vs = vsm + w * Sld;
  // the lattices' rows have the utterance's own stride S (as the recursions write them)
  const float* Ar = a.A + (long)b * a.T * Sld + (long)t * S;
  const float* Br = a.Bt + (long)b * a.T * Sld + (long)t * S;
  for (int s = lane; s < S; s += 64) vs[s] = Ar[s] + Br[s];
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
  const float nll = a.nll[b];
  const int32_t* tg = a.tgt + (long)b * a.U;
  float lb = NEG_INF;
  for (int s = 2 * lane; s < S; s += 128) lb = lse2(lb, vs[s]);
  const float mb = wave_max(lb);
  float sb = mb == NEG_INF ? 0.0f : expf(lb - mb);
  sb = wave_sum(sb);
  const float lcab_blank = mb == NEG_INF ? NEG_INF : mb + logf(sb);
  const float* lpt = a.lp + ((long)b * a.T + t) * a.C;
  float* gt = a.grad + ((long)b * a.T + t) * a.C;
  if (lane == 0 && lcab_blank != NEG_INF) {
    const float lpv = lpt[a.blank];
    gt[a.blank] = a.scale * (expf(lpv) - expf(lcab_blank + nll - lpv));
  }
  const int32_t* fl = a.fl + (long)b * a.U;
  const int32_t* nx = a.nx + (long)b * a.U;
  for (int k = lane; k < Ub; k += 64) {
    if (!fl[k]) continue;
    float lc = NEG_INF;
    for (int k2 = k; k2 >= 0; k2 = nx[k2]) lc = lse2(lc, vs[2 * k2 + 1]);
    if (lc != NEG_INF) {
      const int c = tg[k];
      const float lpv = lpt[c];
      gt[c] = a.scale * (expf(lpv) - expf(lc + nll - lpv));
    }
  }
}

}  // namespace
}  // namespace cfm

using namespace cfm;

struct cfm_ctc_head {
  int D, C, dtype, es, device;
  long Dp, Cp64, Cp256, Dp256;   // padded dims: K granules and N granules
  char* w = nullptr;             // [Cp256][Dp]   compute type
  char* wt = nullptr;            // [Dp256][Cp64] compute type
  float* bias = nullptr;         // [Cp256]
  char* zero = nullptr;
  bool weights_set = false;
  ~cfm_ctc_head() {
    (void)hipFree(w);
    (void)hipFree(wt);
    (void)hipFree(bias);
    (void)hipFree(zero);
  }
};

namespace {

struct HeadWs {
  long rows, logits, gl, glp, glt, encT, xg, cs, total;
  long M, Mp, ldl;
};

HeadWs head_ws(const cfm_ctc_head* h, int B, int T) {
  HeadWs w;
  w.M = (long)B * T;
  w.Mp = round_up(w.M, GEMM_BK_BYTES / h->es);
  w.ldl = round_up(h->C, 4);
  long off = 0;
  auto take = [&](long bytes) { const long o = off; off = round_up(off + bytes, 256); return o; };
  w.rows = take(w.M * h->Dp * h->es);
  w.logits = take(w.M * w.ldl * 4);
  w.gl = take(w.M * h->C * 4);
  w.glp = take(w.M * h->Cp64 * h->es);
  w.glt = take((long)h->C * w.Mp * h->es);
  w.encT = take(h->Dp256 * w.Mp * h->es);
  w.xg = take(w.M * h->D * 4);
  w.cs = take((long)col_sums_ws((int)w.M, h->C));
  w.total = off;
  return w;
}

template <typename F>
void by_dtype(int dt, F&& f) {
  if (dt == DT_F32) f(float{});
  else f(bf16_t{});
}

// f(std::integral_constant<int, CPL>) with CPL = classes per lane of a one-wave-per-row kernel
template <typename F>
void by_cpl(int C, F&& f) {
  const int cpl = (C + 63) / 64;
  if (cpl <= 2) f(std::integral_constant<int, 2>{});
  else if (cpl <= 4) f(std::integral_constant<int, 4>{});
  else if (cpl <= 8) f(std::integral_constant<int, 8>{});
  else if (cpl <= 16) f(std::integral_constant<int, 16>{});
  else if (cpl <= 32) f(std::integral_constant<int, 32>{});
  else fail(CFM_ERR_UNSUPPORTED, "num_classes > 2048");
}

GemmEpi epi_f32(const float* bias, float* X, long ldx) {
  GemmEpi e;
  std::memset(&e, 0, sizeof(e));
  e.mode = EPI_SCALE_F32;
  e.bias = bias;
  e.alpha = 1.0f;
  e.X = X;
  e.ldx = ldx;
  return e;
}

}  // namespace

extern "C" {

cfm_status cfm_ctc_head_create(int feat_in, int num_classes, int device, int compute_mode, cfm_ctc_head** out) {
  return guarded([&] {
    if (!out) fail(CFM_ERR_INVALID_ARG, "out is null");
    *out = nullptr;
    if (feat_in <= 0 || feat_in % 4 || num_classes < 2 || num_classes > 2048)
      fail(CFM_ERR_UNSUPPORTED, "feat_in must be a positive multiple of 4, 2 <= num_classes <= 2048");
    if (compute_mode != CFM_COMPUTE_FP32 && compute_mode != CFM_COMPUTE_BF16) fail(CFM_ERR_INVALID_ARG, "compute_mode");
    HIP_OK(hipSetDevice(device));
    auto h = std::make_unique<cfm_ctc_head>();
    h->D = feat_in;
    h->C = num_classes;
    h->device = device;
    h->dtype = compute_mode == CFM_COMPUTE_FP32 ? DT_F32 : DT_BF16;
    h->es = dtype_size(h->dtype);
    const long kg = GEMM_BK_BYTES / h->es;
    h->Dp = round_up(h->D, kg);
    h->Cp64 = round_up(h->C, kg);
    h->Cp256 = round_up(h->C, GEMM_BN);
    h->Dp256 = round_up(h->D, GEMM_BN);
    HIP_OK(hipMalloc(&h->w, h->Cp256 * h->Dp * h->es));
    HIP_OK(hipMalloc(&h->wt, h->Dp256 * h->Cp64 * h->es));
    HIP_OK(hipMalloc(&h->bias, h->Cp256 * 4));
    HIP_OK(hipMalloc(&h->zero, 4096));
    HIP_OK(hipMemset(h->zero, 0, 4096));
    HIP_OK(hipMemset(h->bias, 0, h->Cp256 * 4));
    *out = h.release();
  });
}

void cfm_ctc_head_destroy(cfm_ctc_head* h) { delete h; }

cfm_status cfm_ctc_head_set_weights(cfm_ctc_head* h, const float* weight, const float* bias, void* stream) {
  return guarded([&] {
    if (!h || !weight) fail(CFM_ERR_INVALID_ARG, "null argument");
    hipStream_t st = (hipStream_t)stream;
    pack_matrix(h->dtype, weight, h->D, h->C, h->D, false, h->w, h->Dp, (int)h->Cp256, (int)h->Dp, st);
    pack_matrix(h->dtype, weight, h->D, h->C, h->D, true, h->wt, h->Cp64, (int)h->Dp256, (int)h->Cp64, st);
    if (bias) HIP_OK(hipMemcpyAsync(h->bias, bias, (size_t)h->C * 4, hipMemcpyDeviceToDevice, st));
    else HIP_OK(hipMemsetAsync(h->bias, 0, (size_t)h->C * 4, st));
    HIP_OK(hipGetLastError());
    h->weights_set = true;
  });
}

size_t cfm_ctc_head_workspace_size(const cfm_ctc_head* h, int B, int T) {
  if (!h || B <= 0 || T <= 0) return 0;
  return (size_t)head_ws(h, B, T).total;
}

cfm_status cfm_ctc_head_forward(cfm_ctc_head* h, const float* enc_bdt, int B, int T, float* logprobs_btc,
                                int32_t* greedy_bt, void* workspace, size_t workspace_bytes, void* stream) {
  return guarded([&] {
    if (!h || !enc_bdt || !logprobs_btc) fail(CFM_ERR_INVALID_ARG, "null argument");
    if (!h->weights_set) fail(CFM_ERR_WEIGHTS, "weights not set");
    if (B <= 0 || T <= 0) fail(CFM_ERR_INVALID_ARG, "B and T must be positive");
    const HeadWs w = head_ws(h, B, T);
    if (!workspace || workspace_bytes < (size_t)w.total) fail(CFM_ERR_WORKSPACE, "workspace too small");
    hipStream_t st = (hipStream_t)stream;
    char* ws = (char*)workspace;
    by_dtype(h->dtype, [&](auto tag) {
      using Tt = decltype(tag);
      cfm_launch(bdt_rows_kernel<Tt>, dim3((T + 31) / 32, (h->D + 31) / 32, B), dim3(256), 0, st, enc_bdt, h->D, T,
                 (Tt*)(ws + w.rows), h->Dp);
    });
    float* logits = (float*)(ws + w.logits);
    gemm(h->dtype, ws + w.rows, h->Dp, (int)w.M, h->D, h->w, (int)h->Dp, h->C, epi_f32(h->bias, logits, w.ldl), h->zero,
         st);
    by_cpl(h->C, [&](auto cpl) {
      cfm_launch(log_softmax_kernel<decltype(cpl)::value>, dim3((unsigned)((w.M + 3) / 4)), dim3(256), 0, st,
                 (const float*)logits, w.ldl, (int)w.M, h->C, logprobs_btc, greedy_bt);
    });
    HIP_OK(hipGetLastError());
  });
}

cfm_status cfm_ctc_head_backward(cfm_ctc_head* h, const float* enc_bdt, int B, int T, const float* logprobs_btc,
                                 const float* grad_lp_btc, float* grad_enc_bdt, float* grad_weight, float* grad_bias,
                                 void* workspace, size_t workspace_bytes, void* stream) {
  return guarded([&] {
    if (!h || !enc_bdt || !logprobs_btc || !grad_lp_btc) fail(CFM_ERR_INVALID_ARG, "null argument");
    refuse_half_training(h->dtype == DT_F32, "cfm_ctc_head_backward");
    if (!h->weights_set) fail(CFM_ERR_WEIGHTS, "weights not set");
    if (B <= 0 || T <= 0) fail(CFM_ERR_INVALID_ARG, "B and T must be positive");
    const HeadWs w = head_ws(h, B, T);
    if (!workspace || workspace_bytes < (size_t)w.total) fail(CFM_ERR_WORKSPACE, "workspace too small");
    hipStream_t st = (hipStream_t)stream;
    char* ws = (char*)workspace;
    const int M = (int)w.M;
    float* gl = (float*)(ws + w.gl);
    by_cpl(h->C, [&](auto cpl) {
      cfm_launch(log_softmax_bwd_kernel<decltype(cpl)::value>, dim3((unsigned)((M + 3) / 4)), dim3(256), 0, st,
                 logprobs_btc, grad_lp_btc, M, h->C, gl);
    });
    if (grad_bias) col_sums(gl, h->C, M, h->C, grad_bias, 0, (float*)(ws + w.cs), st);
    if (grad_enc_bdt) {
      // denc rows (M, D) = gl (M, C) . W (C, D): A = gl rows, packed operand W^T [D][C]
      pack_matrix(h->dtype, gl, h->C, M, h->C, false, ws + w.glp, h->Cp64, M, (int)h->Cp64, st);
      float* xg = (float*)(ws + w.xg);
      gemm(h->dtype, ws + w.glp, h->Cp64, M, h->C, h->wt, (int)h->Cp64, h->D, epi_f32(nullptr, xg, h->D), h->zero, st);
      transpose_out(xg, B, T, h->D, grad_enc_bdt, st);
    }
    if (grad_weight) {
      // dW (C, D) = gl^T (C, M) . enc (M, D): A = gl^T [C][Mp], packed operand enc^T [D][Mp]
      pack_matrix(h->dtype, gl, h->C, M, h->C, true, ws + w.glt, w.Mp, h->C, (int)w.Mp, st);
      by_dtype(h->dtype, [&](auto tag) {
        using Tt = decltype(tag);
        cfm_launch(bdt_dm_kernel<Tt>, dim3((unsigned)std::min<long>((w.Mp + 255) / 256, 1024), (unsigned)h->Dp256),
                   dim3(256), 0, st, enc_bdt, B, h->D, T, (Tt*)(ws + w.encT), w.Mp, (int)h->Dp256);
      });
      gemm(h->dtype, ws + w.glt, w.Mp, h->C, M, ws + w.encT, (int)w.Mp, h->D, epi_f32(nullptr, grad_weight, h->D),
           h->zero, st);
    }
    HIP_OK(hipGetLastError());
  });
}

size_t cfm_ctc_loss_workspace_size(int B, int T, int C, int U) {
  (void)C;
  if (B <= 0 || T <= 0 || U < 0) return 0;
  const long S = 2L * U + 1;
  return (size_t)(round_up((long)B * T * (U + 1) * 4, 256) + 2 * round_up((long)B * T * S * 4, 256) + round_up(B, 256) +
                  2 * round_up((long)B * std::max(U, 1) * 4, 256) + 256);
}

cfm_status cfm_ctc_loss(const float* logprobs_btc, const int32_t* targets_bu, const int32_t* input_lengths,
                        const int32_t* target_lengths, int B, int T, int C, int U, int blank, int zero_infinity,
                        float grad_scale, float* nll_b, float* grad_btc, void* workspace, size_t workspace_bytes,
                        void* stream) {
  return guarded([&] {
    if (!logprobs_btc || !input_lengths || !target_lengths || !nll_b || (U > 0 && !targets_bu))
      fail(CFM_ERR_INVALID_ARG, "null argument");
    if (B <= 0 || T <= 0 || C < 2 || U < 0 || blank < 0 || blank >= C) fail(CFM_ERR_INVALID_ARG, "bad sizes");
    const long S = 2L * U + 1;
    if (S > 1024) fail(CFM_ERR_UNSUPPORTED, "2*U+1 > 1024 extended states");
    if (!workspace || workspace_bytes < cfm_ctc_loss_workspace_size(B, T, C, U))
      fail(CFM_ERR_WORKSPACE, "workspace too small");
    hipStream_t st = (hipStream_t)stream;
    char* ws = (char*)workspace;
    CtcArgs a;
    a.lp = logprobs_btc; a.tgt = targets_bu; a.ilen = input_lengths; a.tlen = target_lengths;
    a.B = B; a.T = T; a.C = C; a.U = U; a.blank = blank; a.zero_inf = zero_infinity;
    a.scale = grad_scale;
    a.E = (float*)ws;
    a.A = (float*)(ws + round_up((long)B * T * (U + 1) * 4, 256));
    a.dead = (uint8_t*)(ws + round_up((long)B * T * (U + 1) * 4, 256) + round_up((long)B * T * S * 4, 256));
    a.Bt = (float*)((char*)a.dead + round_up(B, 256));
    a.fl = (int32_t*)((char*)a.Bt + round_up((long)B * T * S * 4, 256));
    a.nx = (int32_t*)((char*)a.fl + round_up((long)B * std::max(U, 1) * 4, 256));
    a.nll = nll_b;
    a.grad = grad_btc;
    if (U == 0) a.tgt = input_lengths;   // never dereferenced for a label (no odd states)
    cfm_launch(ctc_gather_kernel, dim3((unsigned)std::min<long>(((long)T * (U + 1) + 255) / 256, 256), B), dim3(256), 0,
               st, a);
    const int spl = (int)((S + 63) / 64);
    // alphas (+ nll) and, for the gradient, betas in one launch (independent recursions, grid.y);
    // then scale * exp(lp) everywhere and the target classes' posterior terms, fully parallel
    auto lattice = [&](auto klat) { cfm_launch(klat, dim3(B, grad_btc ? 2 : 1), dim3(64), 0, st, a); };
    if (spl <= 2) lattice(ctc_lattice_kernel<2>);
    else if (spl <= 4) lattice(ctc_lattice_kernel<4>);
    else if (spl <= 8) lattice(ctc_lattice_kernel<8>);
    else lattice(ctc_lattice_kernel<16>);
    if (grad_btc) {
      cfm_launch(ctc_grad_base_kernel, dim3((unsigned)std::min<long>(((long)T * C + 255) / 256, 512), B), dim3(256), 0, st,
                 a);
      cfm_launch(ctc_post_kernel, dim3((unsigned)((T + 3) / 4), B), dim3(256), (uint32_t)(4 * S * 4), st, a);
    }
    HIP_OK(hipGetLastError());
  });
}

}  // extern "C"
