// Fused Transformer-XL relative-position multi-head attention
// (RelPositionMultiHeadAttention.forward, multi_head_attention.py:172-210, with forward_attention 94-115).
//
// For one (batch b, head h, 32-query tile) per wave:
//   ac[i][j]  = (q_i + u_h) . k_j                               (:191, :199)
//   bd[i][j]  = (q_i + v_h) . p_{T'-1-i+j}                      (:193, :203-206; rel_shift folded:
//                                                                 bd_shifted[i][j] = bd[i][T'-1-i+j])
//   s = (ac + bd) / sqrt(dk); masked keys excluded; softmax; P.V  (:208, :104-112)
// The score matrix is never written to HBM.  Keys are visited in 32-key tiles with an online
// (running max / sum) softmax.  Reference masking uses -10000 then zeroes masked probabilities;
// for a query row with at least one valid key (every valid row: j = i is always valid) the
// masked terms are exactly 0 in fp32, so excluding them is identical.  Rows i >= len are all
// masked in the reference: their probabilities are zeroed (:107), so the output row is exactly 0.
//
// Per key tile and wave: 32x32 ac (NS MFMA slabs), 32x64 bd window (2 x NS slabs), the skewed
// gather bd[i][j - i + 31] through an LDS image, a row-per-lane-pair softmax pass, and P.V with
// V read pre-transposed (Vt, written by the QKV GEMM epilogue) so both MFMA operands are
// contiguous 16-byte loads.  K, P and Vt come straight from L2 (shared by all query tiles).
#include "cfm_common.h"
#include "cfm_kernels.h"

namespace cfm {

namespace {

struct AttnParams {
  const char* qk; long ldqk;      // elements; Q at col h*dkp, K at col H*dkp + h*dkp
  const char* Vt; int vt_rows; int Tpad;
  const char* P; long ldp;        // P for head h at col h*dkp, rows 0 .. 2T'-2
  const float* pos_u; const float* pos_v;
  const int32_t* lens;
  int Tp, H, dk, dkp;
  int ctx_left, ctx_right;
  float s_dk;
  char* out; long ldo;
};

constexpr int ACS = 33;   // fp32 row stride of the ac image (conflict-free row-pair reads)
constexpr int BDS = 66;   // fp32 row stride of the 32x64 bd image

template <typename T, int NS, int ND>
__global__ __launch_bounds__(64) void rel_attn_kernel(AttnParams p) {
  constexpr int es = sizeof(T);
  constexpr int SE = 32 / es;            // elements per 32-byte slab
  constexpr int NSK = es;                // slabs per 32-key row (32 keys * es bytes / 32)
  constexpr int PS = 32 * es + 16;       // byte stride of the P tile rows (padded)
  __shared__ float ac_s[32 * ACS];
  __shared__ float bd_s[32 * BDS];
  __shared__ __attribute__((aligned(16))) char pt_s[32 * PS];
  __shared__ float alpha_s[32];
  __shared__ float l_s[32];

  const int lane = threadIdx.x;
  const int hsel = lane >> 5, col = lane & 31;
  const int i0 = blockIdx.x * 32, h = blockIdx.y, b = blockIdx.z;
  const int Tp = p.Tp;
  const int len = min(p.lens[b], Tp);
  const T* qk = (const T*)p.qk;
  const long rowbase = (long)b * Tp;

  // Q fragments with the two per-head biases (q + u for ac, q + v for bd), in fp32 then back.
  uint4 qu[NS], qv[NS];
  {
    const int i = min(i0 + col, Tp - 1);
    const T* qrow = qk + (rowbase + i) * p.ldqk + (long)h * p.dkp;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int d0 = s * SE + hsel * (SE / 2);
      const uint4 raw = *(const uint4*)(qrow + d0);
      float f[SE / 2], fu[SE / 2], fv[SE / 2];
      Vec16<T>::to_f32(raw, f);
#pragma unroll
      for (int e = 0; e < SE / 2; ++e) {
        const int d = d0 + e;
        const bool ok = d < p.dk;
        fu[e] = ok ? f[e] + p.pos_u[h * p.dk + d] : 0.0f;
        fv[e] = ok ? f[e] + p.pos_v[h * p.dk + d] : 0.0f;
      }
      qu[s] = Vec16<T>::from_f32(fu);
      qv[s] = Vec16<T>::from_f32(fv);
    }
  }

  f32x16 o[ND];
#pragma unroll
  for (int n = 0; n < ND; ++n) o[n] = f32x16{};
  float m_run = -INFINITY, l_run = 0.0f;

  int jbeg = 0, jend = len;
  if (p.ctx_left >= 0) jbeg = max(0, (i0 - p.ctx_left) & ~31);
  if (p.ctx_right >= 0) jend = min(jend, i0 + 31 + p.ctx_right + 1);

  const int ri = lane >> 1, rc = lane & 1;     // softmax pass: row ri, keys 16rc .. 16rc+15
  const int ig_row = i0 + ri;
  const T* vt_head = (const T*)p.Vt + ((long)b * p.H + h) * p.vt_rows * p.Tpad;

  for (int j0 = jbeg; j0 < jend; j0 += 32) {
    // ---- scores ----
    f32x16 sac = f32x16{}, sbd0 = f32x16{}, sbd1 = f32x16{};
    {
      const int j = min(j0 + col, Tp - 1);
      const T* krow = qk + (rowbase + j) * p.ldqk + (long)(p.H + h) * p.dkp;
      const int pr0 = Tp - 1 - (i0 + 31) + j0;
      const int pa = min(max(pr0 + col, 0), 2 * Tp - 2);
      const int pb = min(max(pr0 + 32 + col, 0), 2 * Tp - 2);
      const T* prowa = (const T*)p.P + (long)pa * p.ldp + (long)h * p.dkp;
      const T* prowb = (const T*)p.P + (long)pb * p.ldp + (long)h * p.dkp;
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        const int d0 = s * SE + hsel * (SE / 2);
        const uint4 kf = *(const uint4*)(krow + d0);
        const uint4 pfa = *(const uint4*)(prowa + d0);
        const uint4 pfb = *(const uint4*)(prowb + d0);
        mfma_slab<T>(sac, qu[s], kf);
        mfma_slab<T>(sbd0, qv[s], pfa);
        mfma_slab<T>(sbd1, qv[s], pfb);
      }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int i = acc_row(r, lane);
      ac_s[i * ACS + col] = sac[r];
      bd_s[i * BDS + col] = sbd0[r];
      bd_s[i * BDS + 32 + col] = sbd1[r];
    }
    __syncthreads();

    // ---- online softmax, two lanes per query row ----
    float sv[16];
    float mloc = -INFINITY;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int jj = 16 * rc + e;
      const int jg = j0 + jj;
      float s = (ac_s[ri * ACS + jj] + bd_s[ri * BDS + jj - ri + 31]) / p.s_dk;
      bool masked = jg >= len;
      if (p.ctx_left >= 0) masked |= jg < ig_row - p.ctx_left;
      if (p.ctx_right >= 0) masked |= jg > ig_row + p.ctx_right;
      sv[e] = masked ? -INFINITY : s;
      mloc = fmaxf(mloc, sv[e]);
    }
    mloc = fmaxf(mloc, __shfl_xor(mloc, 1, 64));
    const float m_new = fmaxf(m_run, mloc);
    float alpha = 1.0f, psum = 0.0f;
    float pv[16];
    if (m_new == -INFINITY) {
#pragma unroll
      for (int e = 0; e < 16; ++e) pv[e] = 0.0f;
    } else {
      alpha = __expf(m_run - m_new);
#pragma unroll
      for (int e = 0; e < 16; ++e) { pv[e] = __expf(sv[e] - m_new); psum += pv[e]; }
    }
    psum += __shfl_xor(psum, 1, 64);
    l_run = l_run * alpha + psum;
    m_run = m_new;
    {
      char* dst = pt_s + ri * PS + 16 * rc * es;
#pragma unroll
      for (int q = 0; q < 16 / Vec16<T>::N; ++q)
        *(uint4*)(dst + 16 * q) = Vec16<T>::from_f32(pv + q * Vec16<T>::N);
    }
    if (rc == 0) alpha_s[ri] = alpha;
    __syncthreads();

    // ---- rescale and accumulate P.V ----
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float a = alpha_s[acc_row(r, lane)];
#pragma unroll
      for (int n = 0; n < ND; ++n) o[n][r] *= a;
    }
    const bool tail = j0 + 32 > Tp;
#pragma unroll
    for (int s = 0; s < NSK; ++s) {
      const uint4 pa4 = *(const uint4*)(pt_s + col * PS + s * 32 + hsel * 16);
      const int k0 = j0 + s * SE + hsel * (SE / 2);
#pragma unroll
      for (int n = 0; n < ND; ++n) {
        uint4 vb = *(const uint4*)(vt_head + (long)(n * 32 + col) * p.Tpad + k0);
        if (tail) {   // keys >= T' hold unspecified data in Vt's padding: force them to 0
          float f[SE / 2];
          Vec16<T>::to_f32(vb, f);
#pragma unroll
          for (int e = 0; e < SE / 2; ++e) if (k0 + e >= Tp) f[e] = 0.0f;
          vb = Vec16<T>::from_f32(f);
        }
        mfma_slab<T>(o[n], pa4, vb);
      }
    }
    __syncthreads();
  }

  if (rc == 0) l_s[ri] = l_run;
  __syncthreads();
  T* out = (T*)p.out;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int i = acc_row(r, lane);
    const int ig = i0 + i;
    if (ig >= Tp) continue;
    const float l = l_s[i];
    const bool valid = ig < len && l > 0.0f;
    const float inv = valid ? 1.0f / l : 0.0f;
#pragma unroll
    for (int n = 0; n < ND; ++n) {
      const int d = n * 32 + col;
      if (d < p.dk) st_f<T>(out + (rowbase + ig) * p.ldo + (long)h * p.dk + d, valid ? o[n][r] * inv : 0.0f);
    }
  }
}

template <typename T, int NS>
void launch_nd(const AttnParams& p, dim3 grid, hipStream_t st) {
  constexpr int es = sizeof(T);
  constexpr int DKP = NS * 32 / es;
  constexpr int ND = (DKP + 31) / 32;
  hipLaunchKernelGGL((rel_attn_kernel<T, NS, ND>), grid, dim3(64), 0, st, p);
}

template <typename T>
void launch_t(const AttnParams& p, dim3 grid, hipStream_t st) {
  constexpr int es = sizeof(T);
  const int NS = p.dkp * es / 32;
  switch (NS) {
    case 1: launch_nd<T, 1>(p, grid, st); break;
    case 2: launch_nd<T, 2>(p, grid, st); break;
    case 3: launch_nd<T, 3>(p, grid, st); break;
    case 4: launch_nd<T, 4>(p, grid, st); break;
    case 6: launch_nd<T, 6>(p, grid, st); break;
    case 8: launch_nd<T, 8>(p, grid, st); break;
    case 16: launch_nd<T, 16>(p, grid, st); break;
    default: break;
  }
}

}  // namespace

void rel_pos_attention(int dtype, const void* qk, long ldqk, const void* Vt, int vt_rows, int Tpad, const void* P,
                       long ldp, const float* pos_u, const float* pos_v, const int32_t* lens, int B, int Tp, int H,
                       int dk, int dkp, int ctx_left, int ctx_right, void* out, long ldo, hipStream_t st) {
  if (B <= 0 || Tp <= 0) return;
  AttnParams p;
  p.qk = (const char*)qk; p.ldqk = ldqk;
  p.Vt = (const char*)Vt; p.vt_rows = vt_rows; p.Tpad = Tpad;
  p.P = (const char*)P; p.ldp = ldp;
  p.pos_u = pos_u; p.pos_v = pos_v; p.lens = lens;
  p.Tp = Tp; p.H = H; p.dk = dk; p.dkp = dkp;
  p.ctx_left = ctx_left; p.ctx_right = ctx_right;
  p.s_dk = (float)__builtin_sqrt((double)dk);
  p.out = (char*)out; p.ldo = ldo;
  const dim3 grid((Tp + 31) / 32, H, B);
  if (dtype == DT_F32) launch_t<float>(p, grid, st);
  else launch_t<bf16_t>(p, grid, st);
}

}  // namespace cfm
