// Fused Transformer-XL relative-position multi-head attention
// (RelPositionMultiHeadAttention.forward, multi_head_attention.py:172-210, with forward_attention 94-115).
//
// One wave per (batch b, head h, 32-query tile).  For each 32-key tile:
//   S^T[j][i] = k_j . (q_i + u_h)                       (ac, :191/:199; computed transposed)
//   BD^T[r][i] = p_{r0+r} . (q_i + v_h), r in [0, 64)   (:193/:203 over the 63-row window the tile
//                                                          needs; rel_shift (:159-170) is the skew
//                                                          bd[i][j] = BD[i][j - i + 31], taken
//                                                          through a 64x32 fp32 LDS image)
//   s = (ac + bd) / sqrt(dk), masked keys excluded, online softmax, O += P.V  (:104-112)
// The transposed orientation puts one query per lane (16 keys in lane l, 16 in lane l^32), so the
// row max / row sum are in-register plus one cross-half swap, and the probabilities are already
// the A operand of the P.V MFMA (no LDS round trip; the k-order permutation of a 32x32
// accumulator used as operand is matched by the Vt chunk loads, see cdna_hip_programming.md §3).
// Vt (V transposed, keys contiguous) is written by the QKV GEMM epilogue.  K/P/Vt fragments of the
// next key tile are prefetched into registers while the current tile computes.
//
// Masking (SURVEY §7 hard part 2): a query row with >= 1 valid key gets exactly the reference's
// probabilities (the -10000-filled entries underflow to 0 in fp32); rows i >= len are fully masked
// in the reference, whose probabilities are then zeroed (:107) -> their output is exactly 0.
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

constexpr int BDS = 32;   // fp32 row stride of the 64x32 BD^T image (conflict-free skewed reads)

template <typename T> struct VChunk;                          // 4 keys of one Vt row
template <> struct VChunk<bf16_t> { using type = uint2; };
template <> struct VChunk<float> { using type = uint4; };

template <typename T, int NS, int ND>
struct TileRegs {
  uint4 k[NS];
  uint4 pa[NS], pb[NS];
  typename VChunk<T>::type v[ND][4];
};

template <typename T, int NS, int ND>
CFM_DEV void load_tile(TileRegs<T, NS, ND>& t, const AttnParams& p, const T* qk, long rowbase, const T* vt_head,
                       int j0, int i0, int lane) {
  constexpr int SE = 32 / (int)sizeof(T);
  const int hsel = lane >> 5, col = lane & 31;
  const int Tp = p.Tp;
  const int j = min(j0 + col, Tp - 1);
  const T* krow = qk + (rowbase + j) * p.ldqk + (long)(p.H + (int)blockIdx.y) * p.dkp;
  const int pr0 = Tp - 1 - (i0 + 31) + j0;
  const int ra = min(max(pr0 + col, 0), 2 * Tp - 2);
  const int rb = min(max(pr0 + 32 + col, 0), 2 * Tp - 2);
  const T* prowa = (const T*)p.P + (long)ra * p.ldp + (long)blockIdx.y * p.dkp;
  const T* prowb = (const T*)p.P + (long)rb * p.ldp + (long)blockIdx.y * p.dkp;
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int d0 = s * SE + hsel * (SE / 2);
    t.k[s] = *(const uint4*)(krow + d0);
    t.pa[s] = *(const uint4*)(prowa + d0);
    t.pb[s] = *(const uint4*)(prowb + d0);
  }
#pragma unroll
  for (int n = 0; n < ND; ++n)
#pragma unroll
    for (int q = 0; q < 4; ++q)
      t.v[n][q] = *(const typename VChunk<T>::type*)(vt_head + (long)(n * 32 + col) * p.Tpad + j0 + 8 * q + 4 * hsel);
}

// O[n] += P . V for the 32 keys of the tile; s_acc holds P^T (rows = keys, lane = query).
template <typename T, int ND> struct PV;
template <int ND> struct PV<bf16_t, ND> {
  static CFM_DEV void run(f32x16 (&o)[ND], const f32x16& pt, const uint2 (&v)[ND][4]) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      float f[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] = pt[8 * s + e];
      const uint4 a = Vec16<bf16_t>::from_f32(f);
#pragma unroll
      for (int n = 0; n < ND; ++n) {
        const uint4 b = make_uint4(v[n][2 * s].x, v[n][2 * s].y, v[n][2 * s + 1].x, v[n][2 * s + 1].y);
        mfma_slab<bf16_t>(o[n], a, b);
      }
    }
  }
};
template <int ND> struct PV<float, ND> {
  static CFM_DEV void run(f32x16 (&o)[ND], const f32x16& pt, const uint4 (&v)[ND][4]) {
#pragma unroll
    for (int n = 0; n < ND; ++n)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const uint4 c = v[n][r >> 2];
        const uint32_t bw = (r & 3) == 0 ? c.x : (r & 3) == 1 ? c.y : (r & 3) == 2 ? c.z : c.w;
        o[n] = __builtin_amdgcn_mfma_f32_32x32x2f32(pt[r], __uint_as_float(bw), o[n], 0, 0, 0);
      }
  }
};

template <typename T, int NS, int ND>
__global__ __launch_bounds__(64) void rel_attn_kernel(AttnParams p) {
  constexpr int SE = 32 / (int)sizeof(T);
  __shared__ float bd_s[64 * BDS];
  __shared__ float row_s[32];

  const int lane = threadIdx.x;
  const int hsel = lane >> 5, col = lane & 31;
  const int i0 = blockIdx.x * 32, h = blockIdx.y, b = blockIdx.z;
  const int Tp = p.Tp;
  const int len = min(p.lens[b], Tp);
  const T* qk = (const T*)p.qk;
  const long rowbase = (long)b * Tp;
  const T* vt_head = (const T*)p.Vt + ((long)b * p.H + h) * p.vt_rows * p.Tpad;

  // Q fragments (B operand, lane = query) with the per-head biases: q + u (ac), q + v (bd)
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
        const float bu = p.pos_u[h * p.dk + min(d, p.dk - 1)];   // unconditional loads
        const float bv = p.pos_v[h * p.dk + min(d, p.dk - 1)];
        fu[e] = ok ? f[e] + bu : 0.0f;
        fv[e] = ok ? f[e] + bv : 0.0f;
      }
      qu[s] = Vec16<T>::from_f32(fu);
      qv[s] = Vec16<T>::from_f32(fv);
    }
  }

  f32x16 o[ND];
#pragma unroll
  for (int n = 0; n < ND; ++n) o[n] = f32x16{};
  float m_run = -INFINITY, l_run = 0.0f;
  const int iq = i0 + col;                     // this lane's query

  int jbeg = 0, jend = len;
  if (p.ctx_left >= 0) jbeg = max(0, (i0 - p.ctx_left) & ~31);
  if (p.ctx_right >= 0) jend = min(jend, i0 + 31 + p.ctx_right + 1);

  // register prefetch of the next key tile when it fits the VGPR budget (bf16, dk <= 64)
  constexpr bool PREFETCH = sizeof(T) == 2 && NS <= 4;
  TileRegs<T, NS, ND> cur, nxt;
  if (PREFETCH && jbeg < jend) load_tile(cur, p, qk, rowbase, vt_head, jbeg, i0, lane);

  for (int j0 = jbeg; j0 < jend; j0 += 32) {
    const bool more = j0 + 32 < jend;
    if constexpr (PREFETCH) {
      if (more) load_tile(nxt, p, qk, rowbase, vt_head, j0 + 32, i0, lane);
    } else {
      load_tile(cur, p, qk, rowbase, vt_head, j0, i0, lane);
    }

    f32x16 st = f32x16{}, bd0 = f32x16{}, bd1 = f32x16{};
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      mfma_slab<T>(st, cur.k[s], qu[s]);
      mfma_slab<T>(bd0, cur.pa[s], qv[s]);
      mfma_slab<T>(bd1, cur.pb[s], qv[s]);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int rr = acc_row(r, lane);
      bd_s[rr * BDS + col] = bd0[r];
      bd_s[(rr + 32) * BDS + col] = bd1[r];
    }
    __syncthreads();

    // scores for this lane's query and its 16 keys
    float mloc = -INFINITY;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int jj = acc_row(r, lane);          // key within the tile
      const int jg = j0 + jj;
      float s = (st[r] + bd_s[(jj - col + 31) * BDS + col]) / p.s_dk;
      bool masked = jg >= len;
      if (p.ctx_left >= 0) masked |= jg < iq - p.ctx_left;
      if (p.ctx_right >= 0) masked |= jg > iq + p.ctx_right;
      st[r] = masked ? -INFINITY : s;
      mloc = fmaxf(mloc, st[r]);
    }
    mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
    const float m_new = fmaxf(m_run, mloc);
    float alpha = 1.0f, psum = 0.0f;
    if (m_new == -INFINITY) {
#pragma unroll
      for (int r = 0; r < 16; ++r) st[r] = 0.0f;
    } else {
      alpha = __expf(m_run - m_new);
#pragma unroll
      for (int r = 0; r < 16; ++r) { st[r] = __expf(st[r] - m_new); psum += st[r]; }
    }
    psum += __shfl_xor(psum, 32, 64);
    l_run = l_run * alpha + psum;
    m_run = m_new;
    if (hsel == 0) row_s[col] = alpha;
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float a = row_s[acc_row(r, lane)];
#pragma unroll
      for (int n = 0; n < ND; ++n) o[n][r] *= a;
    }
    if (j0 + 32 > Tp) {   // keys >= T' read Vt padding (unspecified): force those V entries to 0
#pragma unroll
      for (int n = 0; n < ND; ++n)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int kb = j0 + 8 * q + 4 * hsel;
          if constexpr (sizeof(T) == 2) {
            uint2& c = cur.v[n][q];
            if (kb + 0 >= Tp) c.x &= 0xffff0000u;
            if (kb + 1 >= Tp) c.x &= 0x0000ffffu;
            if (kb + 2 >= Tp) c.y &= 0xffff0000u;
            if (kb + 3 >= Tp) c.y &= 0x0000ffffu;
          } else {
            uint4& c = cur.v[n][q];
            if (kb + 0 >= Tp) c.x = 0;
            if (kb + 1 >= Tp) c.y = 0;
            if (kb + 2 >= Tp) c.z = 0;
            if (kb + 3 >= Tp) c.w = 0;
          }
        }
    }
    PV<T, ND>::run(o, st, cur.v);
    __syncthreads();
    if constexpr (PREFETCH) {
      if (more) cur = nxt;
    }
  }

  if (hsel == 0) row_s[col] = l_run;
  __syncthreads();
  T* out = (T*)p.out;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int i = acc_row(r, lane);
    const int ig = i0 + i;
    if (ig >= Tp) continue;
    const float l = row_s[i];
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
  if constexpr (sizeof(T) == 2) {      // dkp in {16, 32, 48, 64, 128}
    switch (NS) {
      case 1: launch_nd<T, 1>(p, grid, st); break;
      case 2: launch_nd<T, 2>(p, grid, st); break;
      case 3: launch_nd<T, 3>(p, grid, st); break;
      case 4: launch_nd<T, 4>(p, grid, st); break;
      case 8: launch_nd<T, 8>(p, grid, st); break;
      default: break;
    }
  } else {
    switch (NS) {
      case 2: launch_nd<T, 2>(p, grid, st); break;
      case 4: launch_nd<T, 4>(p, grid, st); break;
      case 6: launch_nd<T, 6>(p, grid, st); break;
      case 8: launch_nd<T, 8>(p, grid, st); break;
      case 16: launch_nd<T, 16>(p, grid, st); break;
      default: break;
    }
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
