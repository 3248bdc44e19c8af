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
#include <cstdlib>
#include <stdexcept>
#include <type_traits>

#include "cfm_common.h"
#include "cfm_kernels.h"

#define CFM_DEV_HOST_INLINE __host__ __device__ inline

namespace cfm {

namespace {

struct AttnParams {
  const char* qk; long ldqk;      // [q+u | q+v | k], each H*dkp columns (EPI_QKV epilogue)
  const char* Vt; int vt_rows; int Tpad;
  const char* P; long ldp;        // P for head h at col h*dkp, rows 0 .. 2T'-2
  const int32_t* lens;
  int Tp, H, dk, dkp;
  int ctx_left, ctx_right;
  // (q + u), (q + v) arrive pre-scaled by log2(e)/sqrt(dk): scores are in log2 units
  char* out; long ldo;
  // natural layout (bf16 LDS kernel only): qk rows are [q | k | v] as the QKV GEMM stores them
  // (bias added, heads padded to dkp); the kernel forms (q + u)*c, (q + v)*c itself from `uv`
  // ([u | v], fp32, H*dkp each) and transposes V into its LDS image while staging.
  const float* uv; float qscale;
  int vec_out;   // 16-byte output stores through LDS (env CFM_ATTN_VECOUT=0 turns them off: A/B)
  // training: dropout on the attention probabilities (multi_head_attention.py:111, p_attn =
  // dropout(attn)); element (b, h, i, j) is kept iff its counter hash passes (drop_mul), so the
  // backward regenerates the same mask.  thr = 0: no dropout.
  Drop adrop;
};

// P^T tile (rows = keys j0 + acc_row(r), lane = query iq) *= dropout mask of (b*H + h, iq, key):
// the softmax denominator keeps the undropped sum (dropout acts on normalised probabilities).
CFM_DEV void drop_tile(f32x16& st, const Drop& dr, long bh, int Tp, int iq, int j0, int lane) {
  if (dr.thr == 0) return;
  const uint64_t base = ((uint64_t)bh * Tp + (uint64_t)min(iq, Tp - 1)) * (uint64_t)Tp + j0;
#pragma unroll
  for (int r = 0; r < 16; ++r) st[r] *= drop_mul(dr, base + acc_row(r, lane));
}

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
  const T* krow = qk + (rowbase + j) * p.ldqk + (long)(2 * p.H + (int)blockIdx.y) * p.dkp;
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

// ---- shared per-tile pieces ------------------------------------------------------------------
constexpr float RESCALE_THR = 8.0f;   // log2 units: P entries may reach 2^8 before O is rescaled (T13)

// Scores of this lane's query against its 16 keys of the tile: s = ac + bd (already in log2 units,
// Q was pre-scaled by log2(e)/sqrt(dk)); masked keys -> -inf.  Masking runs only on tiles that
// need it (uniform branch).
// `rowx` XORs the BD image row (0 or 32): the LDS kernel keeps the two 32-position halves of the
// window in a 2-slot ring and swaps their roles every key tile.
// value of lane l ^ 32 combined with this lane's by a half exchange (v_permlane32_swap, no LDS trip)
CFM_DEV float halves_max(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
CFM_DEV float halves_sum(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

CFM_DEV float tile_scores(f32x16& st, const float* bd_s, const AttnParams& p, int j0, int len, int iq, int lane,
                          int rowx = 0) {
  const int col = lane & 31;
  const bool need_mask = (j0 + 32 > len) || p.ctx_left >= 0 || p.ctx_right >= 0;
  float mloc = -INFINITY;
  if (!need_mask) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int jj = acc_row(r, lane);
      st[r] += bd_s[((jj - col + 31) ^ rowx) * BDS + col];
      mloc = fmaxf(mloc, st[r]);
    }
  } else {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int jj = acc_row(r, lane);
      const int jg = j0 + jj;
      const float sc = st[r] + bd_s[((jj - col + 31) ^ rowx) * BDS + col];
      bool masked = jg >= len;
      if (p.ctx_left >= 0) masked |= jg < iq - p.ctx_left;
      if (p.ctx_right >= 0) masked |= jg > iq + p.ctx_right;
      st[r] = masked ? -INFINITY : sc;
      mloc = fmaxf(mloc, st[r]);
    }
  }
  return halves_max(mloc);
}

// Online softmax with deferred rescale: the running max of a row is raised only when the tile max
// exceeds it by more than RESCALE_THR (then O and l are rescaled, alpha broadcast through row_s);
// otherwise probabilities are taken against the stale max (<= 2^THR, exact after the final 1/l).
// Rows with no valid key so far (m = -inf) get p = exp2(-inf) = 0.
template <int ND>
CFM_DEV void softmax_tile(f32x16& st, float mloc, float& m_run, float& l_run, f32x16 (&o)[ND], float* row_s,
                          int lane) {
  const int hsel = lane >> 5, col = lane & 31;
  const bool grow = mloc > m_run + RESCALE_THR;
  if (__any(grow)) {
    const float m_new = grow ? mloc : m_run;
    // rows that did not grow keep alpha = 1 (also avoids (-inf) - (-inf)); 0 when m_run was -inf
    const float alpha = grow ? __builtin_amdgcn_exp2f(m_run - m_new) : 1.0f;
    l_run *= alpha;
    m_run = m_new;
    if (hsel == 0) row_s[col] = alpha;
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float a = row_s[acc_row(r, lane)];
#pragma unroll
      for (int n = 0; n < ND; ++n) o[n][r] *= a;
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
  }
  const float m_use = m_run == -INFINITY ? 0.0f : m_run;
  float psum = 0.0f;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    st[r] = __builtin_amdgcn_exp2f(st[r] - m_use);
    psum += st[r];
  }
  l_run += halves_sum(psum);
}

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

  // Q fragments (B operand, lane = query), already biased by the QKV epilogue: q + u (ac), q + v (bd)
  uint4 qu[NS], qv[NS];
  {
    const int i = min(i0 + col, Tp - 1);
    const T* qrow = qk + (rowbase + i) * p.ldqk + (long)h * p.dkp;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int d0 = s * SE + hsel * (SE / 2);
      qu[s] = *(const uint4*)(qrow + d0);
      qv[s] = *(const uint4*)(qrow + (long)p.H * p.dkp + d0);
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

    // scores for this lane's query and its 16 keys, then the online softmax
    const float mloc = tile_scores(st, bd_s, p, j0, len, iq, lane);
    softmax_tile<ND>(st, mloc, m_run, l_run, o, row_s, lane);
    drop_tile(st, p.adrop, (long)b * p.H + h, Tp, iq, j0, lane);
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

// ---------------------------------------------------------------------------------------------
// LDS-resident variant (bf16): one block per (b, h) with NW waves; K and Vt of the utterance-head
// are copied into LDS once (zero-filled beyond T'), every wave walks its 32-query tiles reading K/V
// fragments from LDS (conflict-free strides: K rows padded by 16 B, Vt rows by 8 B) while the
// P window is streamed from L2 one key tile ahead.  Same arithmetic as rel_attn_kernel.
// ---------------------------------------------------------------------------------------------
struct LdsGeom {
  int tp32, ks, vs;           // keys rounded to 32, K row stride (bytes), Vt row stride (bytes)
  int k_off, v_off, bd_off, bytes;
};

CFM_DEV_HOST_INLINE LdsGeom lds_geom(int Tp, int dkp, int vt_rows, int nw) {
  LdsGeom g;
  g.tp32 = (Tp + 31) / 32 * 32;
  g.ks = dkp * 2 + 16;
  g.vs = g.tp32 * 2 + 8;
  g.k_off = 0;
  g.v_off = g.tp32 * g.ks;
  g.bd_off = g.v_off + vt_rows * g.vs;
  g.bd_off = (g.bd_off + 15) / 16 * 16;
  g.bytes = g.bd_off + nw * (64 * BDS * 4 + 32 * 4);
  return g;
}

// One wave's 32-query tile [i0, i0 + 32) against the LDS-resident K (Ks) / Vt (Vs) of its (b, h):
// qu / qv are the (q + u)*c / (q + v)*c B-operand slabs of the wave's queries (lane = query).
// bd_s / row_s: the wave's private BD image and row table.  Writes the tile's output rows.
// PF: prefetch the next key tile's P rows into registers (8*NS VGPRs; with NW = 8, two waves per
// SIMD must fit 256 registers: on for dk <= 64).
template <int NS, int ND, bool PF>
CFM_DEV void attn_query_tile(const AttnParams& p, const LdsGeom& g, const char* Ks, const char* Vs, float* bd_s,
                             float* row_s, const uint4 (&qu)[NS], const uint4 (&qv)[NS], int i0, int len, long rowbase,
                             int h, int bh, int lane) {
  using T = bf16_t;
  constexpr int SE = 16;
  const int hsel = lane >> 5, col = lane & 31;
  const int Tp = p.Tp;
  f32x16 o[ND];
#pragma unroll
  for (int n = 0; n < ND; ++n) o[n] = f32x16{};
  float m_run = -INFINITY, l_run = 0.0f;
  const int iq = i0 + col;
  int jbeg = 0, jend = len;
  if (p.ctx_left >= 0) jbeg = max(0, (i0 - p.ctx_left) & ~31);
  if (p.ctx_right >= 0) jend = min(jend, i0 + 31 + p.ctx_right + 1);

  // BD window of key tile k = positions [j0 - i0 + T' - 32, j0 - i0 + T' + 32): its upper half is
  // the lower half of tile k+1, so each tile computes one new 32-position block (P rows loaded
  // one tile ahead) into the ring slot the block before last used.
  auto load_p = [&](int prow0, uint4 (&pr)[NS]) {
    const int ra = min(max(prow0 + col, 0), 2 * Tp - 2);
    const T* prow = (const T*)p.P + (long)ra * p.ldp + (long)h * p.dkp;
#pragma unroll
    for (int s = 0; s < NS; ++s) pr[s] = *(const uint4*)(prow + s * SE + hsel * (SE / 2));
  };
  auto bd_block = [&](const uint4 (&pr)[NS], int slot) {
    f32x16 bd = f32x16{};
#pragma unroll
    for (int s = 0; s < NS; ++s) mfma_slab<T>(bd, pr[s], qv[s]);
#pragma unroll
    for (int r = 0; r < 16; ++r) bd_s[(acc_row(r, lane) + 32 * slot) * BDS + col] = bd[r];
  };
  // P row of position block start for key tile j0: lower = Tp - 1 - (i0 + 31) + j0, upper = +32
  uint4 pu[NS], pn[PF ? NS : 1];
  if (jbeg < jend) {
    uint4 pl[NS];
    load_p(Tp - 1 - (i0 + 31) + jbeg, pl);
    load_p(Tp - 1 - (i0 + 31) + jbeg + 32, pu);
    bd_block(pl, 0);
  }
  int k = 0;
  for (int j0 = jbeg; j0 < jend; j0 += 32, ++k) {
    const bool more = j0 + 32 < jend;
    if constexpr (PF) {
      if (more) load_p(Tp - 1 - (i0 + 31) + j0 + 64, (uint4(&)[NS])pn);
    }
    f32x16 st = f32x16{};
    const char* krow = Ks + (j0 + col) * g.ks + hsel * 16;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const uint4 kf = *(const uint4*)(krow + s * 32);
      mfma_slab<T>(st, kf, qu[s]);
    }
    bd_block(pu, (k + 1) & 1);
    __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): this wave's LDS writes are done
    __builtin_amdgcn_wave_barrier();
    const float mloc = tile_scores(st, bd_s, p, j0, len, iq, lane, (k & 1) << 5);
    softmax_tile<ND>(st, mloc, m_run, l_run, o, row_s, lane);
    drop_tile(st, p.adrop, bh, Tp, iq, j0, lane);
    uint2 v[ND][4];
#pragma unroll
    for (int n = 0; n < ND; ++n)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        v[n][q] = *(const uint2*)(Vs + (n * 32 + col) * g.vs + (j0 + 8 * q + 4 * hsel) * 2);
    PV<T, ND>::run(o, st, v);
    __builtin_amdgcn_s_waitcnt(0xc07f);   // bd_s / row_s reads done before the next tile rewrites them
    __builtin_amdgcn_wave_barrier();
    if (more) {
      if constexpr (PF) {
#pragma unroll
        for (int s = 0; s < NS; ++s) pu[s] = pn[s];
      } else {
        load_p(Tp - 1 - (i0 + 31) + j0 + 64, pu);
      }
    }
  }
  if (hsel == 0) row_s[col] = l_run;
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
  T* out = (T*)p.out;
  if (ND <= 2 && p.vec_out && p.dk == ND * 32 && p.ldo % 8 == 0) {
    // the wave's 32 x dk output tile goes through its (now free) BD image as fp32, then leaves as
    // 16-byte rows of 8 bf16 (4 stores per lane instead of 16 * ND two-byte stores)
    constexpr int OW = ND * 32;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int i = acc_row(r, lane);
      const float l = row_s[i];
      const bool valid = i0 + i < len && l > 0.0f;
      const float inv = valid ? 1.0f / l : 0.0f;
#pragma unroll
      for (int n = 0; n < ND; ++n) bd_s[i * OW + n * 32 + col] = valid ? o[n][r] * inv : 0.0f;
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    constexpr int CH = OW / 8;   // 16-byte chunks per row
#pragma unroll
    for (int q = 0; q < 32 * CH / 64; ++q) {
      const int j = lane + 64 * q, i = j / CH, c8 = j - i * CH;
      if (i0 + i >= Tp) continue;
      const float4 a = *(const float4*)(bd_s + i * OW + c8 * 8);
      const float4 b2 = *(const float4*)(bd_s + i * OW + c8 * 8 + 4);
      const float f[8] = {a.x, a.y, a.z, a.w, b2.x, b2.y, b2.z, b2.w};
      *(uint4*)(out + (rowbase + i0 + i) * p.ldo + (long)h * p.dk + c8 * 8) = Vec16<bf16_t>::from_f32(f);
    }
  } else {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int i = acc_row(r, lane);
      const int ig = i0 + i;
      const float l = row_s[i];
      const bool valid = ig < len && l > 0.0f;
      const float inv = valid ? 1.0f / l : 0.0f;
      if (ig >= Tp) continue;
#pragma unroll
      for (int n = 0; n < ND; ++n) {
        const int d = n * 32 + col;
        if (d < p.dk) st_f<T>(out + (rowbase + ig) * p.ldo + (long)h * p.dk + d, valid ? o[n][r] * inv : 0.0f);
      }
    }
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
}

template <int NS, int ND, int NW, bool PF, bool QN>
__global__ __launch_bounds__(NW * 64) void rel_attn_lds_kernel(AttnParams p) {
  using T = bf16_t;
  constexpr int SE = 16;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int hsel = lane >> 5, col = lane & 31;
  const int bh = blockIdx.x;
  const int b = bh / p.H, h = bh - b * p.H;
  const int Tp = p.Tp;
  const int len = min(p.lens[b], Tp);
  const LdsGeom g = lds_geom(Tp, p.dkp, p.vt_rows, NW);
  const T* qk = (const T*)p.qk;
  const long rowbase = (long)b * Tp;
  char* Ks = smem + g.k_off;
  char* Vs = smem + g.v_off;
  float* bd_s = (float*)(smem + g.bd_off + wave * (64 * BDS * 4 + 32 * 4));
  float* row_s = bd_s + 64 * BDS;

  // ---- stage K [tp32][dkp] and Vt [vt_rows][tp32] of this (b, h) into LDS (zeros past T') ----
  // Loads are issued in batches of BATCH (all in flight) before their LDS writes: a load->write
  // loop body would otherwise expose one full HBM latency per iteration.
  {
    constexpr int BATCH = 8;
    const int kchunks = p.dkp / 8;                          // 16-byte chunks per K row
    const int kn = g.tp32 * kchunks;
    const T* kbase = qk + rowbase * p.ldqk + (long)((QN ? 1 : 2) * p.H + h) * p.dkp;
    for (int i0 = tid; i0 < kn; i0 += NW * 64 * BATCH) {
      uint4 v[BATCH];
#pragma unroll
      for (int u = 0; u < BATCH; ++u) {
        const int i = min(i0 + u * NW * 64, kn - 1);
        const int r = i / kchunks, c = i - r * kchunks;
        v[u] = *(const uint4*)(kbase + (long)min(r, Tp - 1) * p.ldqk + c * 8);
      }
#pragma unroll
      for (int u = 0; u < BATCH; ++u) {
        const int i = i0 + u * NW * 64;
        const int r = i / kchunks, c = i - r * kchunks;
        if (i < kn) *(uint4*)(Ks + r * g.ks + c * 16) = r < Tp ? v[u] : make_uint4(0, 0, 0, 0);
      }
    }
    if constexpr (QN) {
      // V rows [t][dd] -> LDS Vs[dd][t]: a job = 2 consecutive keys x 8 channels (two 16-byte row
      // loads) -> 8 dwords, one per channel row, holding the key pair.  Consecutive lanes take
      // consecutive key pairs, so each ds_write_b32 wave-instruction covers one channel row's
      // consecutive dwords (conflict-free).  Keys >= T' and channels >= dkp are zero.
      const T* vbase = qk + rowbase * p.ldqk + (long)(2 * p.H + h) * p.dkp;
      const int npair = g.tp32 / 2, nchunk = p.vt_rows / 8;
      const int vn = npair * nchunk;
      for (int i0 = tid; i0 < vn; i0 += NW * 64 * (BATCH / 2)) {
        uint4 va[BATCH / 2], vb[BATCH / 2];
#pragma unroll
        for (int u = 0; u < BATCH / 2; ++u) {
          const int i = min(i0 + u * NW * 64, vn - 1);
          const int c = i / npair, tp = i - c * npair;
          const int t0 = min(2 * tp, Tp - 1), t1 = min(2 * tp + 1, Tp - 1), cc = min(c, p.dkp / 8 - 1);
          va[u] = *(const uint4*)(vbase + (long)t0 * p.ldqk + cc * 8);
          vb[u] = *(const uint4*)(vbase + (long)t1 * p.ldqk + cc * 8);
        }
#pragma unroll
        for (int u = 0; u < BATCH / 2; ++u) {
          const int i = i0 + u * NW * 64;
          if (i >= vn) continue;
          const int c = i / npair, tp = i - c * npair;
          const bool ok_c = c < p.dkp / 8;
          const uint32_t ma = (ok_c && 2 * tp < Tp) ? 0x0000ffffu : 0u;
          const uint32_t mb = (ok_c && 2 * tp + 1 < Tp) ? 0xffff0000u : 0u;
          const uint32_t wa[4] = {va[u].x, va[u].y, va[u].z, va[u].w};
          const uint32_t wb[4] = {vb[u].x, vb[u].y, vb[u].z, vb[u].w};
          char* dst = Vs + (c * 8) * g.vs + tp * 4;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            *(uint32_t*)(dst + (2 * e) * g.vs) = ((wa[e] & 0xffffu) & ma) | ((wb[e] << 16) & mb);
            *(uint32_t*)(dst + (2 * e + 1) * g.vs) = ((wa[e] >> 16) & ma) | ((wb[e] & 0xffff0000u) & mb);
          }
        }
      }
    } else {
    const T* vt_head = (const T*)p.Vt + ((long)b * p.H + h) * p.vt_rows * p.Tpad;
    const int vchunks = g.tp32 / 4;                         // 8-byte chunks (4 keys) per Vt row
    const int vn = p.vt_rows * vchunks;
    for (int i0 = tid; i0 < vn; i0 += NW * 64 * BATCH) {
      uint2 v[BATCH];
#pragma unroll
      for (int u = 0; u < BATCH; ++u) {
        const int i = min(i0 + u * NW * 64, vn - 1);
        const int r = i / vchunks, c = i - r * vchunks;
        v[u] = *(const uint2*)(vt_head + (long)r * p.Tpad + c * 4);
      }
#pragma unroll
      for (int u = 0; u < BATCH; ++u) {
        const int i = i0 + u * NW * 64;
        const int r = i / vchunks, c = i - r * vchunks;
        const int k0 = c * 4;
        uint2 w = v[u];
        if (k0 + 0 >= Tp) w.x &= 0xffff0000u;
        if (k0 + 1 >= Tp) w.x &= 0x0000ffffu;
        if (k0 + 2 >= Tp) w.y &= 0xffff0000u;
        if (k0 + 3 >= Tp) w.y &= 0x0000ffffu;
        if (i < vn) *(uint2*)(Vs + r * g.vs + c * 8) = w;
      }
    }
    }
  }
  __syncthreads();

  // query tiles: blockIdx.y of gridDim.y blocks per (b, h) (each stages the whole K / Vt), NW waves each
  const int nqt = (Tp + 31) / 32;
  for (int qt = blockIdx.y * NW + wave; qt < nqt; qt += NW * gridDim.y) {
    const int i0 = qt * 32;
    uint4 qu[NS], qv[NS];
    {
      const int i = min(i0 + col, Tp - 1);
      const T* qrow = qk + (rowbase + i) * p.ldqk + (long)h * p.dkp;
      if constexpr (QN) {
        const float* ub = p.uv + h * p.dkp;
        const float* vb = p.uv + (long)p.H * p.dkp + h * p.dkp;
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          const int d0 = s * SE + hsel * (SE / 2);
          float q[8], a[8], c[8];
          Vec16<bf16_t>::to_f32(*(const uint4*)(qrow + d0), q);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            a[e] = (q[e] + ub[d0 + e]) * p.qscale;
            c[e] = (q[e] + vb[d0 + e]) * p.qscale;
          }
          qu[s] = Vec16<bf16_t>::from_f32(a);
          qv[s] = Vec16<bf16_t>::from_f32(c);
        }
      } else {
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          const int d0 = s * SE + hsel * (SE / 2);
          qu[s] = *(const uint4*)(qrow + d0);
          qv[s] = *(const uint4*)(qrow + (long)p.H * p.dkp + d0);
        }
      }
    }
    attn_query_tile<NS, ND, PF>(p, g, Ks, Vs, bd_s, row_s, qu, qv, i0, len, rowbase, h, bh, lane);
  }
}

// ---------------------------------------------------------------------------------------------
// QKV projection + rel-pos attention in one launch (bf16 eval forward with the LayerNorm fold,
// dkp = 64, T' <= 256; conformer_modules.py:104-105, multi_head_attention.py:172-210).
// Block = (utterance b, head h), 8 waves; wave w owns frames [32w, 32w + 32).
// Phase 1, this head's slice of the QKV GEMM: the 192 folded weight rows (q | k | v of head h) stream
// through a 3-stage LDS ring (glds, 24 KiB per 64-element K-step, XOR-swizzled as gemm_kernel's
// images); each wave's 32 normalised-input rows (xb, the residual producer's compute-type copy) come
// straight from global memory as MFMA operands.  Q and K are computed transposed (weights as A:
// rows = channels, lane = frame), V as rows = frames, so after the folded-LayerNorm epilogue
// y = rstd (acc - mean c) + d:
//   * Q stays in registers: (y + u)c / (y + v)c become the attention's B-operand slabs after one
//     v_permlane32_swap per 4 values (lane = query, 8 consecutive channels per slab half);
//   * K goes to the LDS K image as 8-byte rows of 4 channels, V to the Vt image as 8-byte runs of
//     4 frames of one channel; frames >= T' are zero in both.
// Phase 2: attn_query_tile on the LDS-resident K / Vt, as rel_attn_lds_kernel.
// Gone against the two-kernel path: the QKV GEMM launch and its M x 3*H*dkp output written to and
// re-read from HBM.  The heads of one utterance are placed on one XCD (its xb rows stay in that L2).
// ---------------------------------------------------------------------------------------------
struct QkvFold {
  const char* xb; long ldx_b;          // normalised-input rows (compute type), bytes per row
  const float2* ln_in; int ln_parts, ln_width;   // producer granule partials (GemmEpi::ln_out)
  const char* W; long ldw_b;           // folded q | k | v weight [3*H*dkp][Kpad] (compute type)
  const float* lc; const float* ld;    // fold column terms [3*H*dkp]
  const char* zero;                    // >= 1 KiB of zeros
  int probe;                           // timing probes only (env CFM_QA_PROBE): 1 no attention phase, 2 no K loop,
                                       // 4 half the weight-fragment LDS reads, 8 no loads in the K loop
                                       // (both give wrong results)
};
constexpr int QA_NS = 4;               // weight ring stages
constexpr int QA_STAGE = 192 * 128;    // 192 weight rows x 128 bytes of K
constexpr int QA_TAB_BYTES = (256 + 192 + 64) * 8;   // rs (per frame), cd (per channel), uv (per q channel)

// the weight ring (phase 1) aliases the K / Vt / BD images (phase 2); the tables follow both
CFM_DEV_HOST_INLINE int qkv_attn_tab_off(int Tp) {
  const int b = lds_geom(Tp, 64, 64, 8).bytes;
  return b > QA_NS * QA_STAGE ? b : QA_NS * QA_STAGE;
}
CFM_DEV_HOST_INLINE int qkv_attn_lds_bytes(int Tp) { return qkv_attn_tab_off(Tp) + QA_TAB_BYTES; }

template <int NK>
__global__ __launch_bounds__(512) void qkv_rel_attn_kernel(AttnParams p, QkvFold f) {
  using T = bf16_t;
  constexpr int NS = 4, ND = 2, DKP = 64;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hsel = lane >> 5, col = lane & 31;
  const int nblocks = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, qq = nblocks >> 3, rr = nblocks & 7;
  const int bh = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
  const int b = bh / p.H, h = bh - b * p.H;
  const int Tp = p.Tp;
  const int len = min(p.lens[b], Tp);
  const LdsGeom g = lds_geom(Tp, DKP, DKP, 8);
  const long rowbase = (long)b * Tp;
  char* Ks = smem + g.k_off;
  char* Vs = smem + g.v_off;
  float2* rs_tab = (float2*)(smem + qkv_attn_tab_off(Tp));
  float2* cd_tab = rs_tab + 256;
  float2* uv_tab = cd_tab + 192;

  // ---- phase 1: the head's QKV GEMM ----
  // ring chunk c (0..23) of a stage = weight rows 8c .. 8c+7 (1 KiB); wave w fills chunks w, w+8, w+16
  const char* wsrc[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int row = (i * 8 + wave) * 8 + lane / 8, part = row / DKP;
    const long n = (long)part * p.H * DKP + h * DKP + (row - part * DKP);
    wsrc[i] = f.W + n * f.ldw_b + (((lane & 7) ^ ((row >> 1) & 7)) * 16);
  }
  const uint32_t sbase = lds_addr(smem);
  auto stage = [&](int kt) {   // past the last K-step: the zero page (uniform vmcnt counts)
    const uint32_t base = sbase + (kt % QA_NS) * QA_STAGE;
#pragma unroll
    for (int i = 0; i < 3; ++i)
      glds16_asm(kt < NK ? (const void*)(wsrc[i] + kt * 128) : (const void*)(f.zero + lane * 16),
                 base + (i * 8 + wave) * 1024);
  };
  const char* xrow = f.xb + (rowbase + min(32 * wave + col, Tp - 1)) * f.ldx_b + hsel * 16;
  // x fragments by inline-asm loads: hipcc does not count them, so its waits cannot over-wait on the
  // weight stages issued in between; each group is retired by the counted wait that names it
  typedef uint32_t v4u __attribute__((ext_vector_type(4)));
  auto load_x = [&](int kt, v4u (&x)[4]) {
#pragma unroll
    for (int kk = 0; kk < 4; ++kk)
      asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(x[kk]) : "v"(xrow + (kt * 4 + kk) * 32) : "memory");
  };
  // vmcnt(N) naming the x group it retires (N = the loads issued after it: x group + stage, or the
  // stage alone past the last x group - no x loads are issued past the end, as an x register the
  // kernel never reads would be handed to other values while its load is in flight)
  auto wait_x = [&](auto n, v4u (&x)[4]) {
    asm volatile("s_waitcnt vmcnt(%4)" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]) : "n"(decltype(n)::value)
                 : "memory");
  };
  const int sw = (col >> 1) & 7;
  auto read_w = [&](int slot, int kk, uint4 (&w)[6]) {
    const char* Sb = smem + slot * QA_STAGE;
    const int so = ((2 * kk + hsel) ^ sw) * 16;
#pragma unroll
    for (int j = 0; j < 6; ++j) w[j] = *(const uint4*)(Sb + (32 * ((f.probe & 4) ? j % 3 : j) + col) * 128 + so);
  };

  f32x16 acc[6];
#pragma unroll
  for (int j = 0; j < 6; ++j) acc[j] = f32x16{};
  // x rows and weight stages three K-steps ahead; the issue order (x(k), stage(k)) per K-step is what
  // the counted waits assume: x(k) and stage k are retired once only the groups of k+1 .. k+2 (x groups
  // stop at the last K-step, stages are issued past it from the zero page) may still be in flight
  v4u x[4][4];
  uint4 wc[6], wn[6];
  // the epilogue's tables: per-frame LayerNorm granule partials, per-channel (c, d), (u, v) - loaded
  // first (in flight with the first stages), reduced and written to LDS after the loop
  float2 part[4] = {};
  float2 tab_a = make_float2(0.f, 0.f), tab_b = make_float2(0.f, 0.f);
  if (tid < 256) {
    const float2* pp = f.ln_in + (rowbase + min(tid, Tp - 1)) * f.ln_parts;
#pragma unroll
    for (int gi = 0; gi < 4; ++gi) part[gi] = pp[min(gi, f.ln_parts - 1)];
  } else if (tid < 448) {
    const int c = tid - 256, part_ = c / DKP;
    const long n = (long)part_ * p.H * DKP + h * DKP + (c - part_ * DKP);
    tab_a = make_float2(f.lc[n], f.ld[n]);
  } else {
    const int c = tid - 448;
    tab_b = make_float2(p.uv[h * DKP + c], p.uv[(long)p.H * DKP + h * DKP + c]);
  }
  auto retire = [&](int k, v4u (&xg)[4]) {   // retire x(k) and stage k
    const int younger = 3 * 2 + (k + 1 < NK ? 4 : 0) + (k + 2 < NK ? 4 : 0);
    if (younger == 14) wait_x(std::integral_constant<int, 14>{}, xg);
    else if (younger == 10) wait_x(std::integral_constant<int, 10>{}, xg);
    else wait_x(std::integral_constant<int, 6>{}, xg);
  };
  static_assert(NK >= 3, "three K-steps in flight");
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    load_x(k, x[k]);
    stage(k);
  }
  retire(0, x[0]);
  raw_barrier();
  read_w(0, 0, wc);
  if (!(f.probe & 2))
#pragma unroll
  for (int kt = 0; kt < NK; ++kt) {
    if (!(f.probe & 8)) {
      if (kt + 3 < NK) load_x(kt + 3, x[(kt + 3) % 4]);
      stage(kt + 3);
    }
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      if (kk < 3) {
        read_w(kt % QA_NS, kk + 1, wn);
      } else if (kt + 1 < NK) {
        retire(kt + 1, x[(kt + 1) % 4]);
        wait_lgkm0();
        raw_barrier();
        read_w((kt + 1) % QA_NS, 0, wn);
      }
      const uint4 xf = __builtin_bit_cast(uint4, x[kt % 4][kk]);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] = mfma16_32x32x16(wc[j], xf, acc[j]);   // Q^T, K^T
#pragma unroll
      for (int j = 4; j < 6; ++j) acc[j] = mfma16_32x32x16(xf, wc[j], acc[j]);   // V
#pragma unroll
      for (int j = 0; j < 6; ++j) wc[j] = wn[j];
    }
  }
  wait_vmcnt<0>();
  // per-frame (mean, rstd) from the granule partials (the GEMM epilogue's fold expressions)
  if (tid < 256) {
    const int W = f.ln_width, np = f.ln_parts;
    float sm = 0.0f;
#pragma unroll
    for (int gi = 0; gi < 4; ++gi) sm += gi < np ? (float)min(LN_GRANULE, W - gi * LN_GRANULE) * part[gi].x : 0.0f;
    const float mean = sm / (float)W;
    float m2 = 0.0f;
#pragma unroll
    for (int gi = 0; gi < 4; ++gi) {
      const float dm = part[gi].x - mean;
      m2 += gi < np ? part[gi].y + (float)min(LN_GRANULE, W - gi * LN_GRANULE) * dm * dm : 0.0f;
    }
    rs_tab[tid] = make_float2(mean, 1.0f / sqrtf(m2 / (float)W + 1e-5f));
  } else if (tid < 448) {
    cd_tab[tid - 256] = tab_a;
  } else {
    uv_tab[tid - 448] = tab_b;
  }
  wait_lgkm0();
  raw_barrier();        // tables written; every wave is done with the ring (the K / Vt images overwrite it)

  // ---- phase 1 epilogue ----
  const int tq = 32 * wave + col;                  // this lane's frame in the Q / K products
  const float2 rsq = rs_tab[tq];
  uint4 qu[NS], qv[NS];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int sm = 0; sm < 2; ++sm) {
      // slab 2j + sm = channels 32j + 16sm + [0, 16): rows m = 2sm (this half's channels +0..3, the other
      // half's +4..7) and m = 2sm + 1 (+8..11 / +12..15) swap across the lane halves
      float au[8], av[8];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int ra = 8 * sm + i, rb = ra + 4;
        const int ca = 32 * j + acc_row(ra, lane), cb = 32 * j + acc_row(rb, lane);
        const float2 fa = cd_tab[ca], fb = cd_tab[cb];
        const float ya = rsq.y * (acc[j][ra] - rsq.x * fa.x) + fa.y;
        const float yb = rsq.y * (acc[j][rb] - rsq.x * fb.x) + fb.y;
        const float2 pa = uv_tab[ca], pb = uv_tab[cb];
        const auto su = __builtin_amdgcn_permlane32_swap(__float_as_uint((ya + pa.x) * p.qscale),
                                                         __float_as_uint((yb + pb.x) * p.qscale), false, false);
        const auto sv = __builtin_amdgcn_permlane32_swap(__float_as_uint((ya + pa.y) * p.qscale),
                                                         __float_as_uint((yb + pb.y) * p.qscale), false, false);
        au[i] = __uint_as_float(su[0]);
        au[4 + i] = __uint_as_float(su[1]);
        av[i] = __uint_as_float(sv[0]);
        av[4 + i] = __uint_as_float(sv[1]);
      }
      qu[2 * j + sm] = Vec16<bf16_t>::from_f32(au);
      qv[2 * j + sm] = Vec16<bf16_t>::from_f32(av);
    }
  // K rows: frame tq, channels 32(j-2) + 8m + 4*hsel + [0, 4)
  if (tq < g.tp32) {
#pragma unroll
    for (int j = 2; j < 4; ++j)
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const int c0 = 32 * (j - 2) + 8 * m + 4 * hsel;
        float y[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float2 fc = cd_tab[64 + c0 + i];
          y[i] = tq < Tp ? rsq.y * (acc[j][4 * m + i] - rsq.x * fc.x) + fc.y : 0.0f;
        }
        *(uint2*)(Ks + tq * g.ks + c0 * 2) =
            make_uint2((uint32_t)f2bf(y[0]) | ((uint32_t)f2bf(y[1]) << 16), (uint32_t)f2bf(y[2]) | ((uint32_t)f2bf(y[3]) << 16));
      }
  }
  // Vt: channel 32(j-4) + col, frames 32w + 8m + 4*hsel + [0, 4)
#pragma unroll
  for (int j = 4; j < 6; ++j) {
    const int c = 32 * (j - 4) + col;
    const float2 fc = cd_tab[128 + c];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int t0 = 32 * wave + 8 * m + 4 * hsel;
      if (t0 >= g.tp32) continue;
      float y[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float2 rs = rs_tab[t0 + i];
        y[i] = t0 + i < Tp ? rs.y * (acc[j][4 * m + i] - rs.x * fc.x) + fc.y : 0.0f;
      }
      *(uint2*)(Vs + c * g.vs + t0 * 2) =
          make_uint2((uint32_t)f2bf(y[0]) | ((uint32_t)f2bf(y[1]) << 16), (uint32_t)f2bf(y[2]) | ((uint32_t)f2bf(y[3]) << 16));
    }
  }
  wait_lgkm0();
  __syncthreads();

  // ---- phase 2: attention of the wave's query tile ----
  const int i0 = 32 * wave;
  if (i0 < Tp && !(f.probe & 1)) {
    float* bd_s = (float*)(smem + g.bd_off + wave * (64 * BDS * 4 + 32 * 4));
    attn_query_tile<NS, ND, true>(p, g, Ks, Vs, bd_s, bd_s + 64 * BDS, qu, qv, i0, len, rowbase, h, bh, lane);
  }
}

// launches the LDS-resident kernel if its image fits; returns false otherwise.  8 waves per block
// (one 32-query tile each at T' <= 256, two waves per SIMD) when the image fits, else 4.
template <int NS, bool QN>
bool launch_lds(const AttnParams& p, int B, hipStream_t st) {
  constexpr int DKP = NS * 16;
  constexpr int ND = (DKP + 31) / 32;
  constexpr int LDS_MAX = 160 * 1024;
  static bool attr_set = [] {
    (void)hipFuncSetAttribute((const void*)rel_attn_lds_kernel<NS, ND, 4, true, QN>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
    (void)hipFuncSetAttribute((const void*)rel_attn_lds_kernel<NS, ND, 8, (NS <= 4), QN>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
    return true;
  }();
  (void)attr_set;
  static const int force_nw = [] { const char* s = getenv("CFM_ATTN_NW"); return s ? atoi(s) : 0; }();
  const LdsGeom g8 = lds_geom(p.Tp, p.dkp, p.vt_rows, 8);
  const LdsGeom g4 = lds_geom(p.Tp, p.dkp, p.vt_rows, 4);
  // fewer (b, h) pairs than CUs: split each pair's query tiles over blocks (every block stages the
  // whole K / Vt; the tiles are computed exactly as by one block)
  const int nqt = (p.Tp + 31) / 32;
  static const bool split_ok = [] { const char* e = getenv("CFM_ATTN_QSPLIT"); return !(e && !atoi(e)); }();
  auto qsplit = [&](int nw) {
    if (!split_ok) return 1;
    const int want = 256 / std::max(B * p.H, 1);
    return std::max(1, std::min(want, (nqt + nw - 1) / nw));
  };
  if (force_nw != 4 && g8.bytes <= LDS_MAX) {
    cfm_launch((rel_attn_lds_kernel<NS, ND, 8, (NS <= 4), QN>), dim3(B * p.H, qsplit(8)), dim3(512), g8.bytes, st, p);
    return true;
  }
  if (g4.bytes <= LDS_MAX) {
    cfm_launch((rel_attn_lds_kernel<NS, ND, 4, true, QN>), dim3(B * p.H, qsplit(4)), dim3(256), g4.bytes, st, p);
    return true;
  }
  return false;
}

bool lds_path_fits(int Tp, int dkp) {
  const int vt_rows = (dkp + 31) / 32 * 32;
  return lds_geom(Tp, dkp, vt_rows, 4).bytes <= 160 * 1024;
}

template <typename T, int NS>
void launch_nd(const AttnParams& p, dim3 grid, hipStream_t st) {
  constexpr int es = sizeof(T);
  constexpr int DKP = NS * 32 / es;
  constexpr int ND = (DKP + 31) / 32;
  cfm_launch((rel_attn_kernel<T, NS, ND>), grid, dim3(64), 0, st, p);
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

bool attn_natural_layout(int dtype, int Tp, int dkp) {
  static const bool lds_ok = [] { const char* s = getenv("CFM_ATTN_STREAM"); return !(s && atoi(s)); }();
  static const bool nat_ok = [] { const char* s = getenv("CFM_ATTN_NATURAL"); return !(s && !atoi(s)); }();
  if (dtype != DT_BF16 || !lds_ok || !nat_ok) return false;
  if (dkp != 16 && dkp != 32 && dkp != 48 && dkp != 64 && dkp != 128) return false;
  return lds_path_fits(Tp, dkp);
}

void rel_pos_attention_natural(const void* qkv, long ldqkv, const float* uv, float qscale, const void* P, long ldp,
                               const int32_t* lens, int B, int Tp, int H, int dk, int dkp, int ctx_left,
                               int ctx_right, void* out, long ldo, hipStream_t st) {
  if (B <= 0 || Tp <= 0) return;
  AttnParams p;
  p.qk = (const char*)qkv; p.ldqk = ldqkv;
  p.Vt = nullptr; p.vt_rows = (dkp + 31) / 32 * 32; p.Tpad = 0;
  p.P = (const char*)P; p.ldp = ldp;
  p.lens = lens;
  p.Tp = Tp; p.H = H; p.dk = dk; p.dkp = dkp;
  p.ctx_left = ctx_left; p.ctx_right = ctx_right;
  p.out = (char*)out; p.ldo = ldo;
  p.uv = uv; p.qscale = qscale;
  p.adrop = Drop{0u, 0u, 1.0f};
  static const int vec_out = [] { const char* e = getenv("CFM_ATTN_VECOUT"); return e ? atoi(e) : 1; }();
  p.vec_out = vec_out;
  bool done = false;
  switch (dkp) {
    case 16: done = launch_lds<1, true>(p, B, st); break;
    case 32: done = launch_lds<2, true>(p, B, st); break;
    case 48: done = launch_lds<3, true>(p, B, st); break;
    case 64: done = launch_lds<4, true>(p, B, st); break;
    case 128: done = launch_lds<8, true>(p, B, st); break;
    default: break;
  }
  if (!done) throw std::runtime_error("rel_pos_attention_natural: shape does not fit the LDS kernel");
}

bool qkv_attention_fused_supported(int dtype, int Tp, int dkp, int d) {
  if (dtype != DT_BF16 || dkp != 64 || Tp < 1 || Tp > 256 || (d != 256 && d != 512)) return false;
  return qkv_attn_lds_bytes(Tp) <= 160 * 1024;
}

void qkv_rel_attention_fused(const void* xb, int d, const float2* ln_in, int ln_parts, const void* Wqkv, int Kpad,
                             const float* lc, const float* ld, const float* uv, float qscale, const void* P, long ldp,
                             const int32_t* lens, int B, int Tp, int H, int dk, int ctx_left, int ctx_right, void* out,
                             long ldo, const void* zero_page, hipStream_t st) {
  if (B <= 0 || Tp <= 0) return;
  if (!qkv_attention_fused_supported(DT_BF16, Tp, 64, d) || Kpad != d || dk > 64 || (dk + 15) / 16 * 16 != 64)
    throw std::runtime_error("qkv_rel_attention_fused: bf16, dkp = 64, d in {256, 512}, T' <= 256 only");
  AttnParams p;
  p.qk = nullptr; p.ldqk = 0;
  p.Vt = nullptr; p.vt_rows = 64; p.Tpad = 0;
  p.P = (const char*)P; p.ldp = ldp;
  p.lens = lens;
  p.Tp = Tp; p.H = H; p.dk = dk; p.dkp = 64;
  p.ctx_left = ctx_left; p.ctx_right = ctx_right;
  p.out = (char*)out; p.ldo = ldo;
  p.uv = uv; p.qscale = qscale;
  p.adrop = Drop{0u, 0u, 1.0f};
  p.vec_out = 1;
  QkvFold f;
  f.xb = (const char*)xb; f.ldx_b = (long)d * 2;
  f.ln_in = ln_in; f.ln_parts = ln_parts; f.ln_width = d;
  f.W = (const char*)Wqkv; f.ldw_b = (long)Kpad * 2;
  f.lc = lc; f.ld = ld;
  f.zero = (const char*)zero_page;
  static const int probe = [] { const char* e = getenv("CFM_QA_PROBE"); return e ? atoi(e) : 0; }();
  f.probe = probe;
  const int bytes = qkv_attn_lds_bytes(Tp);
  static const bool attr = [] {
    (void)hipFuncSetAttribute((const void*)qkv_rel_attn_kernel<8>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)qkv_rel_attn_kernel<4>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    return true;
  }();
  (void)attr;
  if (d == 512) cfm_launch(qkv_rel_attn_kernel<8>, dim3(B * H), dim3(512), bytes, st, p, f);
  else cfm_launch(qkv_rel_attn_kernel<4>, dim3(B * H), dim3(512), bytes, st, p, f);
}

void rel_pos_attention(int dtype, const void* qk, long ldqk, const void* Vt, int vt_rows, int Tpad, const void* P,
                       long ldp, const int32_t* lens, int B, int Tp, int H,
                       int dk, int dkp, int ctx_left, int ctx_right, void* out, long ldo, hipStream_t st,
                       Drop adrop) {
  if (B <= 0 || Tp <= 0) return;
  AttnParams p;
  p.uv = nullptr; p.qscale = 1.0f; p.vec_out = 1;
  p.adrop = adrop;
  p.qk = (const char*)qk; p.ldqk = ldqk;
  p.Vt = (const char*)Vt; p.vt_rows = vt_rows; p.Tpad = Tpad;
  p.P = (const char*)P; p.ldp = ldp;
  p.lens = lens;
  p.Tp = Tp; p.H = H; p.dk = dk; p.dkp = dkp;
  p.ctx_left = ctx_left; p.ctx_right = ctx_right;
  p.out = (char*)out; p.ldo = ldo;
  const dim3 grid((Tp + 31) / 32, H, B);
  if (dtype == DT_F32) {
    launch_t<float>(p, grid, st);
    return;
  }
  static const bool lds_ok = [] { const char* s = getenv("CFM_ATTN_STREAM"); return !(s && atoi(s)); }();
  if (lds_ok) {
    bool done = false;
    switch (dkp) {
      case 16: done = launch_lds<1, false>(p, B, st); break;
      case 32: done = launch_lds<2, false>(p, B, st); break;
      case 48: done = launch_lds<3, false>(p, B, st); break;
      case 64: done = launch_lds<4, false>(p, B, st); break;
      case 128: done = launch_lds<8, false>(p, B, st); break;
      default: break;
    }
    if (done) return;
  }
  launch_t<bf16_t>(p, grid, st);
}

}  // namespace cfm
