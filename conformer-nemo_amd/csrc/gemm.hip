// MFMA GEMM for every dense contraction of the encoder.
//
//   C[M, N] = A[M, K] . Wp[N, K]^T   (+ fused epilogue)
//
// Wp is a weight pre-packed at load time ([Npad][Kpad], compute type, zero padded) in the
// nn.Linear / Conv1d(k=1) layout, so both operands are read along K.
//
// Main loop (per block: BM x BN tile, WM x WN waves, each wave (BM/WM) x (BN/WN) = MR x NR MFMA
// 32x32 tiles):
//   * K is consumed in 128-byte steps (64 bf16 / 32 fp32).  Each step's A and B tiles are copied
//     HBM/L2 -> LDS by global_load_lds_dwordx4 (16 B per lane, 1 KiB = 8 rows per wave-instruction)
//     issued from inline asm, so hipcc's waitcnt pass does not see them (it would otherwise put a
//     vmcnt(0) in front of every ds_read and serialise the prefetch with the MFMAs).
//   * 3-slot LDS ring: tiles k+1 and k+2 are in flight while tile k is multiplied; a counted
//     `s_waitcnt vmcnt(G)` + raw s_barrier retires exactly tile k.
//   * The XOR swizzle `slot ^ ((row >> 1) & 7)` is applied to the per-lane SOURCE address (the LDS
//     image is lane-linear) and to the ds_read_b128 fragment read: every 16-lane read group hits
//     16 distinct (bank-row half, slot) positions -> conflict-free.
//   * Out-of-range A rows / K bytes read a zero page: no tail handling in the loop.
//   * Blocks are remapped so that each XCD owns a contiguous range of tiles (A panels stay in one L2).
// Epilogue: the fp32 accumulators are staged through LDS and written back row-major with 16-byte
// vector accesses (bias, activation, GLU, residual read-modify-write all vectorised).
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <vector>
#include <cstdlib>
#include <type_traits>

#include "cfm_common.h"
#include "cfm_abi.h"
#include "cfm_kernels.h"

namespace cfm {

namespace {

// NS_ = LDS ring depth: NS_ - 1 K-steps are in flight while one is multiplied.
// EP_ = epilogue passes: the fp32 accumulator image is staged through LDS BM/EP_ rows at a time
// (the wave rows wm in [p*WM/EP, (p+1)*WM/EP) write in pass p), so a 256x256 tile fits 128 KiB.
// BK_ = bytes of K per stage and row (128 or 64; the packed K granule GEMM_BK_BYTES is a multiple).
//   One glds wave-instruction fills 1 KiB = RPI rows x BK bytes; the 16-byte slots of a row are
//   XOR-swizzled by (row / (16 / SLOTS)) % SLOTS so each 16-lane ds_read_b128 group hits 16
//   distinct bank positions.
// KG_ = K-groups: the block's waves form KG groups of WM x WN that split every K-step's 32-byte
// substeps between them (2 waves per SIMD on a 4-wave output tiling); the groups' accumulators
// are summed through the LDS image before the epilogue (fixed order: bitwise reproducible).
template <int BM_, int BN_, int WM_, int WN_, int NS_, int EP_ = 1, int BK_ = 128, int KG_ = 1>
struct Tile {
  static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_, NSTAGE = NS_, EP = EP_, BKB = BK_, KG = KG_;
  static constexpr int NW = WM * WN * KG, NT = 64 * NW;
  static constexpr int MR = BM / WM / 32, NR = BN / WN / 32;
  static constexpr int SLOTS = BKB / 16, RPI = 1024 / BKB, SWDIV = 16 / SLOTS;
  static constexpr int GA = BM / RPI / NW, GB = BN / RPI / NW;     // glds per thread per stage
  static constexpr int STAGE_BYTES = (BM + BN) * BKB;
  static constexpr int EPS = BN;     // fp32 stride of the epilogue image (row writes / 16-B row reads are conflict-free)
  static constexpr int EPI_BYTES = BM / EP * EPS * 4;
  // folded LayerNorm (GemmEpi::ln_in) tables behind the ring / image: per row (mean, rstd), per
  // column (c, d)
  static constexpr int RS_OFF = (NSTAGE * STAGE_BYTES > EPI_BYTES) ? NSTAGE * STAGE_BYTES : EPI_BYTES;
  static constexpr int CD_OFF = RS_OFF + BM * 8;
  static constexpr int LDS_BYTES = CD_OFF + BN * 8;
  static_assert(GA >= 1 && GB >= 1 && MR >= 1 && NR >= 1, "tile");
  static_assert(BKB == 64 || BKB == 128 || BKB == 256, "stage depth");
  // 256-byte K-steps run only where the host checked p.kb % 256 == 0 (dispatch)
  static_assert(GEMM_BK_BYTES % BKB == 0 || BKB == 256, "packed K granule");
  static_assert(WM % EP == 0, "epilogue passes split the wave rows");
  static_assert(KG == 1 || (EP == 1 && (BKB / 32) % KG == 0), "K-groups");
  static_assert(LDS_BYTES <= 160 * 1024, "LDS");
  static CFM_DEV int swz(int row) { return (row / SWDIV) % SLOTS; }
};
// The rows of one epilogue pass, seen by the epilogue as a (BM/EP) x BN tile.
template <class TL, bool SWZ_ = false>
struct EpiView {
  static constexpr int BM = TL::BM / TL::EP, BN = TL::BN, NT = TL::NT, EPS = TL::EPS;
  // fp32 image element (r, c).  SWZ: the swapped-operand tiles write 4 consecutive columns of one row per
  // lane (ds_write_b128), so the 16-byte slots of a row are XOR-swizzled by (r & 7): the 8 rows of a
  // write lane group then hit 8 distinct slots (conflict-free), and so do the row-wise float4 reads.
  static CFM_DEV int fidx(int r, int c) {
    if constexpr (SWZ_) return r * EPS + ((((c >> 2) ^ (r & 7)) << 2) | (c & 3));
    else return r * EPS + c;
  }
};

using T128x128 = Tile<128, 128, 2, 2, 2>;   // 2 x 32 KiB ring: 2 blocks / CU
using T256x128 = Tile<256, 128, 4, 2, 3>;   // 3 x 48 KiB
using T64x128s2 = Tile<64, 128, 2, 2, 2>;   // 2 x 24 KiB: 3 blocks / CU
// 1 block / CU tiles
using T256x256 = Tile<256, 256, 2, 4, 4, 2, 64>;    // 8 waves, 4 x 32 KiB, wave tile 128 x 64
using T128x128d = Tile<128, 128, 2, 2, 8, 1, 64>;   // 4 waves, 8 x 16 KiB
using T256x128d = Tile<256, 128, 4, 2, 5, 1, 64>;   // 8 waves, 5 x 24 KiB, wave tile 64 x 64
using T128x256d = Tile<128, 256, 2, 4, 5, 1, 64>;   // 8 waves, 5 x 24 KiB, wave tile 64 x 64
using T256x256w = Tile<256, 256, 2, 4, 2, 2, 128>;  // 8 waves, 2 x 64 KiB
using T128x128k = Tile<128, 128, 2, 2, 3, 1, 128, 2>;  // 8 waves = 2 K-groups x 4, 3 x 32 KiB, wave tile 64 x 64
using T128x128k2 = Tile<128, 128, 2, 2, 2, 1, 128, 2>; // as above, 2 x 32 KiB (2 blocks / CU by LDS)
using T128x128k4 = Tile<128, 128, 2, 2, 4, 1, 128, 2>; // as above, 4 x 32 KiB
using T128x256k = Tile<128, 256, 2, 2, 3, 1, 128, 2>;  // 8 waves = 2 K-groups x 4, 3 x 48 KiB, wave tile 64 x 128
using T64x128k = Tile<64, 128, 2, 2, 3, 1, 128, 2>;    // 8 waves = 2 K-groups x 4, 3 x 24 KiB, wave tile 32 x 64
using T128x128q = Tile<128, 128, 2, 2, 4, 1, 128, 4>;  // 16 waves = 4 K-groups x 4, 4 x 32 KiB, wave tile 64 x 64
using T128x128w = Tile<128, 128, 2, 2, 2, 1, 256, 2>;  // 8 waves = 2 K-groups x 4, 2 x 64 KiB of 256-byte K-steps:
                                                       // 16 MFMAs per wave between barriers (K % 128 == 0 only)

// LDS-DMA (glds16_asm) and counted waits: cfm_common.h
// wait until at most `ahead` stages of G loads each are still in flight (ahead in [0, MAXA])
template <int G, int MAXA> CFM_DEV void wait_stages(int ahead) {
  if constexpr (MAXA <= 0) {
    wait_vmcnt<0>();
  } else {
    if (ahead >= MAXA) wait_vmcnt<G * MAXA>();
    else wait_stages<G, MAXA - 1>(ahead);
  }
}

// ---- A-operand loaders -----------------------------------------------------------------------
template <int G>
struct ALoadDense {
  static constexpr bool kConv = false;
  const char* A; long lda_b; int M; long kbytes; const char* zero;
  // utterance-aligned rows (GemmEpi::utt_tp): tile i = m / utt_rows is tile j = i % utt_nt of utterance
  // b = i / utt_nt, its row r = m % utt_rows frame t = j * utt_out - utt_halo + r (valid in [0, utt_tp))
  int utt_tp, utt_rows, utt_nt, utt_out, utt_halo;
  struct State { const char* row_ptr[G]; };
  CFM_DEV void shift_k(long koff) { A += koff; kbytes -= koff; }
  CFM_DEV void prepare(State& s, int m0, const int* rows) const {
#pragma unroll
    for (int i = 0; i < G; ++i) {
      int m = m0 + rows[i];
      bool ok = m < M;
      if (utt_tp > 0) {
        const int ti = m / utt_rows, r = m - ti * utt_rows;
        const int b = ti / utt_nt, t = (ti - b * utt_nt) * utt_out - utt_halo + r;
        m = b * utt_tp + t;
        ok = t >= 0 && t < utt_tp && m < M;
      }
      s.row_ptr[i] = ok ? A + (long)m * lda_b : nullptr;
    }
  }
  // kb0: the K-step's first byte (wave-uniform); lo: this lane's byte offset within the step
  CFM_DEV const void* src(const State& s, int i, long kb0, int lo) const {
    const long kb = kb0 + lo;
    return (s.row_ptr[i] != nullptr && kb < kbytes) ? (const void*)(s.row_ptr[i] + kb) : (const void*)zero;
  }
};

// Row m = (b, t2, f2) of the implicit im2col matrix; column byte kb = (tap * C + c) * es with
// tap = 3*kt + kf; source = X1[b][2*t2 - 1 + kt][2*f2 - 1 + kf][c] (zero outside the image).
template <int G>
struct ALoadConv {
  static constexpr bool kConv = true;   // conv2 + ReLU only
  const char* X1; int T1, F1, T2, F2; long tapb; int M; const char* zero;
  int tap_steps;   // tapb / 128 when a 3x3 tap spans whole 128-byte K-steps (C*es % 128 == 0), else 0
  struct State { const char* base[G]; uint32_t valid[G]; };
  CFM_DEV void shift_k(long) {}   // never split
  CFM_DEV void prepare(State& s, int m0, const int* rows) const {
#pragma unroll
    for (int i = 0; i < G; ++i) {
      const int m = m0 + rows[i];
      uint32_t v = 0;
      const char* base = nullptr;
      if (m < M) {
        const int f2 = m % F2;
        const int bt = m / F2;
        const int t2 = bt % T2;
        const int b = bt / T2;
        const int ti0 = 2 * t2 - 1, fi0 = 2 * f2 - 1;
        for (int kt = 0; kt < 3; ++kt)
          for (int kf = 0; kf < 3; ++kf) {
            const int ti = ti0 + kt, fi = fi0 + kf;
            if (ti >= 0 && ti < T1 && fi >= 0 && fi < F1) v |= 1u << (kt * 3 + kf);
          }
        base = X1 + (((long)b * T1 + ti0) * F1 + fi0) * tapb;   // only dereferenced for valid taps
      }
      s.base[i] = base;
      s.valid[i] = v;
    }
  }
  CFM_DEV const void* src(const State& s, int i, long kb0, int lo) const {
    int tap;
    long cb;
    if (tap_steps > 0) {
      // the whole K-step lies in one tap: tap and the tap's byte offset are wave-uniform (scalar
      // unit, 32-bit), only the validity bit and the address add are per lane
      const int k0 = __builtin_amdgcn_readfirstlane((int)kb0);
      tap = __builtin_amdgcn_readfirstlane(k0 / (int)tapb);
      cb = (long)(k0 - tap * (int)tapb) + lo;
    } else {
      const long kb = kb0 + lo;
      tap = (int)(kb / tapb);
      cb = kb - (long)tap * tapb;
    }
    if (tap >= 9 || !((s.valid[i] >> tap) & 1u)) return zero;
    const int kt = tap / 3, kf = tap - kt * 3;
    return s.base[i] + ((long)kt * F1 + kf) * tapb + cb;
  }
};

// Transposed-conv A operand (conv2's input gradient, one stride phase (pt, pf)): row m = (b, i, j) is
// conv2 input pixel (t1, f1) = (2i + pt, 2j + pf); its K columns are the taps that reach that pixel,
// tap = a * nf + c over nt = 1 + pt time taps and nf = 1 + pf frequency taps.  Time tap a = 0 is
// kt = 1 (pt = 0, source t2 = i) or kt = 0 (pt = 1, source t2 = i + 1); a = 1 is kt = 2 (t2 = i);
// frequency alike.  Column byte kb = tap * tapb + co * es reads dY2[b][t2][f2][co] (zero off-image).
// tapb % 128 == 0 (host-checked), so a K-step never straddles two taps.
template <int G>
struct ALoadTConv {
  static constexpr bool kConv = false;
  const char* dY; long ldb; int T2, F2, nI, nJ, pt, pf; long tapb; int M; const char* zero;
  struct State { const char* base[G]; uint32_t valid[G]; };
  CFM_DEV void shift_k(long) {}   // never split
  CFM_DEV void prepare(State& s, int m0, const int* rows) const {
#pragma unroll
    for (int i = 0; i < G; ++i) {
      const int m = m0 + rows[i];
      uint32_t v = 0;
      const char* base = nullptr;
      if (m < M) {
        const int j = m % nJ, bi = m / nJ;
        const int ii = bi % nI, b = bi / nI;
        base = dY + ((long)(b * T2 + ii) * F2 + j) * ldb;
        const int nf = 1 + pf;
        for (int a = 0; a <= pt; ++a)
          for (int c = 0; c < nf; ++c) {
            const int dt = (pt && a == 0) ? 1 : 0, df = (pf && c == 0) ? 1 : 0;
            if (ii + dt < T2 && j + df < F2) v |= 1u << (a * nf + c);
          }
      }
      s.base[i] = base;
      s.valid[i] = v;
    }
  }
  CFM_DEV const void* src(const State& s, int i, long kb0, int lo) const {
    const int k0 = __builtin_amdgcn_readfirstlane((int)kb0);
    const int tap = __builtin_amdgcn_readfirstlane(k0 / (int)tapb);
    if (tap >= 4 || !((s.valid[i] >> tap) & 1u)) return zero;
    const int nf = 1 + pf, a = tap / nf, c = tap - a * nf;
    const int dt = (pt && a == 0) ? 1 : 0, df = (pf && c == 0) ? 1 : 0;
    return s.base[i] + ((long)dt * F2 + df) * ldb + (long)(k0 - tap * (int)tapb) + lo;
  }
};

thread_local int g_splits = 1;
// bf16 dense STORE / RELU / SWISH / RESID GEMMs with swapped MFMA operands and register epilogues
// (gemm_kernel's SW); CFM_GEMM_SWAP=0 keeps the unswapped kernels
int g_gemm_swap = [] { const char* s = getenv("CFM_GEMM_SWAP"); return s ? atoi(s) : 0; }();

constexpr int LN_PRE = 4;   // folded-LayerNorm granule partials prefetched per row (d <= 512 fully)   // grid.y of the next split-K launch (gemm_splitk)

struct GemmParams {
  const char* W; long ldw_b; int kb; int Mtiles, Ntiles; int M, N;   // kb = packed K bytes per row
  long split_x;   // split-K (gridDim.y > 1, dense A only): slice y covers K bytes [y*kb, (y+1)*kb) and
                  // writes its fp32 partial at epi.X + y * split_x
  int probe;   // microbenchmark probes only (cfm_bench_gemm): 1 no main-loop loads, 2 no epilogue, 4 one K-step
  int ahead;   // K-group tiles with >= 3 stages: the read-ahead main loop (g_gemm_ahead)
  GemmEpi epi;
};

// ---- epilogue: LDS image -> global, 16-byte vectors -------------------------------------------
// Every global load here is unconditional (clamped address, value selected afterwards): a load
// under a per-thread condition is branched around by hipcc and serialised behind its own
// vmcnt(0) (cdna_hip_programming.md §5, 'Three .s-level traps' (c)).
// The stored row of GEMM row m (clamped into range): itself, or for utterance-aligned rows
// (GemmEpi::utt_tp, tile height BM) frame m % BM of utterance m / BM.
CFM_DEV int real_row(const GemmParams& p, int m, int BM) {
  if (p.epi.utt_tp <= 0) return min(m, p.M - 1);
  const int ti = m / BM, r = m - ti * BM;
  const int b = ti / p.epi.utt_nt, t = (ti - b * p.epi.utt_nt) * p.epi.utt_out - p.epi.utt_halo + r;
  return min(b * p.epi.utt_tp + min(max(t, 0), p.epi.utt_tp - 1), p.epi.utt_M - 1);
}

// Folded LayerNorm (GemmEpi::ln_in): rs[r] = (mean, rstd) of the pass's local row r, cd[j] = (c, d)
// of the tile's local column j.
CFM_DEV float ln_fold(float2 s, float v, float2 cd) { return s.y * (v - s.x * cd.x) + cd.y; }

// Sum over the 32 lanes of a half-wave, the same value in every lane: DPP quad permutes and row
// mirrors (VALU) for 16 lanes, one xor-16 shuffle.
template <int CTRL> CFM_DEV float dpp_mov(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
// two fp32 -> a packed pair of the 16-bit compute type, as f2bf rounds each: bf16 in one v_cvt_pk_bf16_f32
#ifdef CFM_HALF_F16
CFM_DEV uint32_t pk_bf16x2(float a, float b) { return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16); }
#else
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
CFM_DEV uint32_t pk_bf16x2(float a, float b) { return __builtin_bit_cast(uint32_t, bf16x2_t{(__bf16)a, (__bf16)b}); }
#endif
CFM_DEV float halfwave_sum(float v) {
  v += dpp_mov<0xB1>(v);    // quad_perm [1,0,3,2]
  v += dpp_mov<0x4E>(v);    // quad_perm [2,3,0,1]
  v += dpp_mov<0x141>(v);   // row_half_mirror: lane i <- 7 - i (the other quad of the 8)
  v += dpp_mov<0x140>(v);   // row_mirror: lane i <- 15 - i (the other 8 of the row)
  v += __shfl_xor(v, 16, 32);
  return v;
}

// FOLD: the LayerNorm fold is active for this launch (GemmEpi::ln_in set: consumer; ln_out / xb
// set: EPI_RESID producer) - a compile-time flag, so no per-element branches in the unrolled loops.
template <typename T, int EPI, class TL, bool FOLD>
CFM_DEV void epilogue(const GemmParams& p, const float* img, int m0, int n0, long xoff, const float2* rs,
                      const float2* cd) {
  const GemmEpi& e = p.epi;
  const int tid = threadIdx.x;
  constexpr bool fold = FOLD;
  if constexpr (EPI == EPI_RESID || EPI == EPI_SCALE_F32) {
    // fp32 output (N % 4 == 0), 4 columns per thread-chunk
    constexpr int CPR = TL::BN / 4;                 // chunks per row
    constexpr int RPP = TL::NT / CPR;               // rows per pass
    constexpr int NP = TL::BM / RPP;
    const int cc = tid % CPR, r0 = tid / CPR;
    const int n = n0 + cc * 4;
    const int nc = min(n, p.N - 4);
    const bool colok = n < p.N;
    if constexpr (EPI == EPI_SCALE_F32) {
      if (e.out_scalar) {
        // fp32 rows whose stride is not a multiple of 4 (e.g. the RNN-T joint's V + 1 = 1025 logits): each
        // tile row is re-cut at the 16-byte boundaries of ITS global address - float4 stores for the
        // aligned body, scalar stores for the < 4 leading and trailing elements (one thread per row)
        const int ncols = min(TL::BN, p.N - n0);
#pragma unroll
        for (int q = 0; q < NP; ++q) {
          const int r = r0 + q * RPP;
          const int m = m0 + r;
          if (m >= p.M || ncols <= 0) continue;
          const long g0 = xoff + (long)m * e.ldx + n0;
          const int lead = min((int)(((16 - ((uintptr_t)(e.X + g0) & 15)) & 15) >> 2), ncols);   // fp32 base: 4-B aligned
          const int nfull = (ncols - lead) / 4;
          const int ntl = ncols - lead - 4 * nfull;   // < 4 trailing elements
          const float* ir = img + r * TL::EPS;
          if (cc < nfull) {
            const int j = lead + 4 * cc;
            typedef float f4v __attribute__((ext_vector_type(4)));
            const f4v v4 = {ir[j] * e.alpha, ir[j + 1] * e.alpha, ir[j + 2] * e.alpha, ir[j + 3] * e.alpha};
            if (e.nt_store) __builtin_nontemporal_store(v4, (f4v*)(e.X + g0 + j));
            else *(f4v*)(e.X + g0 + j) = v4;
          }
          if (e.out_scalar == 2) {   // A/B: the round-3 form, one thread storing all heads and tails
            if (cc == CPR - 1) {
              for (int j = 0; j < lead; ++j) e.X[g0 + j] = ir[j] * e.alpha;
              for (int j = lead + 4 * nfull; j < ncols; ++j) e.X[g0 + j] = ir[j] * e.alpha;
            }
            continue;
          }
          // the <= 3 leading and <= 3 trailing elements: one element per lane (lanes 0.. and ..CPR-1),
          // one store instruction for all of them
          const int j1 = cc < lead ? cc : (cc >= CPR - ntl ? lead + 4 * nfull + (cc - (CPR - ntl)) : -1);
          if (j1 >= 0 && CPR >= 8) e.X[g0 + j1] = ir[j1] * e.alpha;
        }
        return;
      }
    }
    float4 xv[NP];
    if constexpr (EPI == EPI_RESID) {
      const float* XI = e.Xin ? e.Xin : e.X;
#pragma unroll
      for (int q = 0; q < NP; ++q) {
        const int m = min(m0 + r0 + q * RPP, p.M - 1);
        xv[q] = *(const float4*)(XI + xoff + (long)m * e.ldx + nc);
      }
    }
#pragma unroll
    for (int q = 0; q < NP; ++q) {
      const int r = r0 + q * RPP;
      const int m = m0 + r;
      const float4 a = *(const float4*)(img + TL::fidx(r, cc * 4));
      float4 o;
      if constexpr (EPI == EPI_RESID) {
        if (e.drop.thr) {   // training: x_out = x_in + alpha * dropout(branch)
          const uint64_t i = (uint64_t)m * e.ldx + n;
          o.x = xv[q].x + (e.alpha * a.x) * drop_mul(e.drop, i);
          o.y = xv[q].y + (e.alpha * a.y) * drop_mul(e.drop, i + 1);
          o.z = xv[q].z + (e.alpha * a.z) * drop_mul(e.drop, i + 2);
          o.w = xv[q].w + (e.alpha * a.w) * drop_mul(e.drop, i + 3);
        } else {
          o.x = xv[q].x + a.x * e.alpha; o.y = xv[q].y + a.y * e.alpha;
          o.z = xv[q].z + a.z * e.alpha; o.w = xv[q].w + a.w * e.alpha;
        }
      } else {
        o.x = a.x * e.alpha; o.y = a.y * e.alpha; o.z = a.z * e.alpha; o.w = a.w * e.alpha;
      }
      if (e.out_scalar) {   // unaligned rows (ldx % 4 != 0): element stores, tail-masked
        float* xr = e.X + xoff + (long)m * e.ldx + n;
        if (m < p.M) {
          if (n < p.N) xr[0] = o.x;
          if (n + 1 < p.N) xr[1] = o.y;
          if (n + 2 < p.N) xr[2] = o.z;
          if (n + 3 < p.N) xr[3] = o.w;
        }
      } else if (colok && m < p.M) {
        const long off = xoff + (long)m * e.ldx + n;
        if (e.wt) store16_wt(e.X, off * 4, make_uint4(__float_as_uint(o.x), __float_as_uint(o.y), __float_as_uint(o.z),
                                                      __float_as_uint(o.w)));
        else *(float4*)(e.X + off) = o;
        if constexpr (EPI == EPI_RESID && FOLD) {
          {   // compute-type copy of the new rows: the A operand of the LayerNorm-folded GEMM
            if constexpr (sizeof(T) == 2) {
              *(uint2*)((T*)e.xb + off) = make_uint2((uint32_t)f2bf(o.x) | ((uint32_t)f2bf(o.y) << 16),
                                                     (uint32_t)f2bf(o.z) | ((uint32_t)f2bf(o.w) << 16));
            } else {
              *(float4*)((T*)e.xb + off) = o;
            }
          }
        }
      }
      if constexpr (EPI == EPI_RESID && FOLD) {
        {
          // (mean, M2) of this row's 128-column granule: the 32 consecutive threads holding it reduce
          // by xor shuffles inside their half-wave (CPR % 32 == 0), two passes (mean, then the
          // squared deviations) - no cancellation
          static_assert(CPR % 32 == 0, "LayerNorm granule = 32 threads x 4 columns");
          const bool ok = colok && m < p.M;
          const int g = (n0 + (cc & ~31) * 4) / LN_GRANULE;
          const int cnt = min(LN_GRANULE, p.N - g * LN_GRANULE);
          const float s = halfwave_sum(ok ? (o.x + o.y) + (o.z + o.w) : 0.0f);
          const float mean = s / (float)max(cnt, 1);
          const float a0 = o.x - mean, a1 = o.y - mean, a2 = o.z - mean, a3 = o.w - mean;
          const float q2 = halfwave_sum(ok ? (a0 * a0 + a1 * a1) + (a2 * a2 + a3 * a3) : 0.0f);
          if ((cc & 31) == 0 && m < p.M && cnt > 0) e.ln_out[(long)m * e.ln_parts + g] = make_float2(mean, q2);
        }
      }
    }
  } else if constexpr (EPI == EPI_GLU_DW) {
    // pointwise_conv1 -> GLU -> pad mask -> depthwise conv (k 31, zero padding) -> BatchNorm
    // (running statistics) -> Swish (conformer_modules.py:160-176) for one utterance (the tile's
    // 256 rows are its frames, T' <= 256) and 64 channels (the tile's 128 GLU-packed columns); the
    // GLU output never leaves LDS (the unfused path writes and re-reads it through HBM).
    if constexpr (TL::BM == 256 && TL::BN == 128 && TL::NT == 512) {
      constexpr int VE = 8, CPR = 8, RPP = 64, NP = 4, K = 31, PAD = 15, DT = 16, NX = DT + K - 1;
      const int cc = tid % CPR, r0 = tid / CPR;
      const int oc_local = cc * VE;
      const int ca = (oc_local / 32) * 64 + oc_local % 32, cg = ca + 32;
      // tile j of utterance b: row r is frame f0 + r (T' > 256: tiles of utt_out frames with utt_halo
      // frames of context either side; the conv's zero padding outside [0, len))
      const int ti = m0 / 256, b = ti / e.utt_nt, f0 = (ti - b * e.utt_nt) * e.utt_out - e.utt_halo, Tp = e.utt_tp;
      const int len = e.lens ? min(e.lens[b], Tp) : Tp;   // frames >= T' are zero padding of the conv
      float gv[NP][VE];
#pragma unroll
      for (int q = 0; q < NP; ++q) {
        const int r = r0 + q * RPP;
        float2 st;
        if constexpr (fold) st = rs[r];
#pragma unroll
        for (int i = 0; i < VE; ++i) {
          float a = img[r * TL::EPS + ca + i];
          float g = img[r * TL::EPS + cg + i];
          if constexpr (fold) { a = ln_fold(st, a, cd[ca + i]); g = ln_fold(st, g, cd[cg + i]); }
          gv[q][i] = (f0 + r >= 0 && f0 + r < len) ? a * sigmoidf_(g) : 0.0f;
        }
      }
      __syncthreads();                     // every wave has read the accumulator image
      float* gimg = (float*)img;           // [256 frames][64 channels] fp32
#pragma unroll
      for (int q = 0; q < NP; ++q) {
        float4* d4 = (float4*)(gimg + (r0 + q * RPP) * 64 + oc_local);
        d4[0] = make_float4(gv[q][0], gv[q][1], gv[q][2], gv[q][3]);
        d4[1] = make_float4(gv[q][4], gv[q][5], gv[q][6], gv[q][7]);
      }
      __syncthreads();
      const int c = tid & 63;
      const int ch = n0 / 2 + c;           // output channel
      const int chc = min(ch, p.N - 1);
      float wk[K];
#pragma unroll
      for (int k = 0; k < K; ++k) wk[k] = e.dw_w[(long)k * p.N + chc];
      const float bi = e.dw_b[chc], mu = e.bn_mean[chc], inv = e.bn_inv[chc], gw = e.bn_w[chc], gb = e.bn_b[chc];
      // outputs are staged as bf16 [256 frames][64 channels] behind the GLU image, then stored as
      // 16-byte row runs (2-byte per-lane stores would make the tail store-issue bound)
      T* simg = (T*)((char*)img + 256 * 64 * 4);
      // 8 waves x 2 windows of 16 frames = 256 frames; lanes = consecutive channels (conflict-free)
#pragma unroll 1
      for (int h = 0; h < 2; ++h) {
        const int t0 = ((tid >> 6) * 2 + h) * DT;
        float x[NX];
#pragma unroll
        for (int i = 0; i < NX; ++i) {
          const int t = t0 - PAD + i;
          const float v = gimg[min(max(t, 0), 255) * 64 + c];
          x[i] = (t >= 0 && t < 256) ? v : 0.0f;
        }
#pragma unroll
        for (int j = 0; j < DT; ++j) {
          float a = 0.0f;
#pragma unroll
          for (int k = 0; k < K; ++k) a = fmaf(wk[k], x[j + k], a);
          a += bi;
          st_f<T>(simg + (t0 + j) * 64 + c, swishf((a - mu) * inv * gw + gb));
        }
      }
      __syncthreads();
      constexpr int VO = 16 / (int)sizeof(T);            // channels per 16-byte run
      for (int i = tid; i < 256 * 64 / VO; i += TL::NT) {
        const int t = i / (64 / VO), c8 = (i % (64 / VO)) * VO;
        const int ft = f0 + t;
        if (t >= e.utt_halo && t < e.utt_halo + e.utt_out && ft < Tp && n0 / 2 + c8 < p.N)
          *(uint4*)((T*)e.C + ((long)b * Tp + ft) * e.ldc + n0 / 2 + c8) = *(const uint4*)(simg + t * 64 + c8);
      }
    }
  } else if constexpr (EPI == EPI_GLU_MASK) {
    // packed columns: per 64-column group g, [0,32) = value channels 32g.., [32,64) = gates
    constexpr int VE = 16 / (int)sizeof(T);          // output elements per 16-byte chunk
    constexpr int CPR = (TL::BN / 2) / VE;
    constexpr int RPP = TL::NT / CPR;
    constexpr int NP = TL::BM / RPP;
    const int cc = tid % CPR, r0 = tid / CPR;
    const int oc_local = cc * VE;                    // output channel within the block (BN/2 wide)
    const int grp = oc_local / 32, j = oc_local % 32;
    const int ca = grp * 64 + j, cg = grp * 64 + 32 + j;   // packed columns within the tile
    const int c = n0 / 2 + oc_local;                 // output channel
    int lenq[NP];
#pragma unroll
    for (int q = 0; q < NP; ++q) lenq[q] = e.lens ? e.lens[min(m0 + r0 + q * RPP, p.M - 1) / e.Tp] : e.Tp;
#pragma unroll
    for (int q = 0; q < NP; ++q) {
      const int r = r0 + q * RPP;
      const int m = m0 + r;
      const int t = m % e.Tp;
      const bool masked = t >= lenq[q];
      float2 st;
      if constexpr (fold) st = rs[r];
      float o[VE];
#pragma unroll
      for (int i = 0; i < VE; ++i) {
        float a = img[r * TL::EPS + ca + i];
        float g = img[r * TL::EPS + cg + i];
        if constexpr (fold) { a = ln_fold(st, a, cd[ca + i]); g = ln_fold(st, g, cd[cg + i]); }
        o[i] = masked ? 0.0f : a * sigmoidf_(g);
      }
      if (m >= p.M || c >= p.N) continue;
      T* dst = (T*)e.C + (long)m * e.ldc + c;
      if (c + VE <= p.N) {
        if (e.wt) store16_wt(e.C, ((long)m * e.ldc + c) * (long)sizeof(T), Vec16<T>::from_f32(o));
        else *(uint4*)dst = Vec16<T>::from_f32(o);
      } else {
        for (int i = 0; i < VE && c + i < p.N; ++i) st_f<T>(dst + i, o[i]);
      }
    }
  } else {
    // compute-type output (EPI_STORE / RELU / SWISH / QKV's q,k part); EPI_QKV's v part transposed
    constexpr int VE = 16 / (int)sizeof(T);
    constexpr int CPR = TL::BN / VE;
    constexpr int RPP = TL::NT / CPR;
    constexpr int NP = TL::BM / RPP;
    const int cc = tid % CPR, r0 = tid / CPR;
    const int n = n0 + cc * VE;
    const int nlim = (EPI == EPI_QKV) ? e.qk_cols : p.N;
    // EPI_QKV: q chunk -> (q + u) at n and (q + v) at n + H*dkp; k chunk -> n + H*dkp
    const int hq = (EPI == EPI_QKV) ? e.qk_cols / 2 : 0;
    float ub[VE], vb[VE];
    if constexpr (EPI == EPI_QKV) {
#pragma unroll
      for (int i = 0; i < VE; ++i) {
        const int nq = min(n + i, hq - 1);
        ub[i] = e.uv[nq];
        vb[i] = e.uv[hq + nq];
      }
    }
    const bool vec = n + VE <= nlim && ((e.ldc * (long)sizeof(T)) % 16 == 0);
#pragma unroll
    for (int q = 0; q < NP; ++q) {
      const int r = r0 + q * RPP;
      const int m = m0 + r;
      float2 st;
      if constexpr (fold) st = rs[r];
      float zf[VE];
      if constexpr (EPI == EPI_SWISH_BWD) {
        // z row chunk of this output chunk (host guarantees N % VE == 0); rows past M read row M-1
        const T* zp = (const T*)e.zin + (long)min(m, p.M - 1) * e.ldz + min(n, nlim - VE);
        Vec16<T>::to_f32(*(const uint4*)zp, zf);
      }
      float o[VE];
#pragma unroll
      for (int i = 0; i < VE; ++i) {
        float v = img[r * TL::EPS + cc * VE + i];
        if constexpr (fold) v = ln_fold(st, v, cd[cc * VE + i]);
        if constexpr (EPI == EPI_RELU) v = fmaxf(v, 0.0f);
        if constexpr (EPI == EPI_SWISH) v = swishf(v);
        if constexpr (EPI == EPI_SWISH_BWD) {
          const float zz = zf[i], sg = sigmoidf_(zz);
          v *= drop_mul(e.drop, (uint64_t)m * (uint64_t)e.ldz + (uint64_t)(n + i)) * (sg + zz * sg * (1.0f - sg));
        }
        o[i] = v;
      }
      if (m >= p.M || n >= nlim) continue;
      if constexpr (EPI == EPI_QKV) {
        T* row = (T*)e.C + (long)m * e.ldc;
        if (n < hq) {
          float ou[VE], ov[VE];
#pragma unroll
          for (int i = 0; i < VE; ++i) { ou[i] = (o[i] + ub[i]) * e.qscale; ov[i] = (o[i] + vb[i]) * e.qscale; }
          if (e.wt) {
            store16_wt(e.C, ((long)m * e.ldc + n) * (long)sizeof(T), Vec16<T>::from_f32(ou));
            store16_wt(e.C, ((long)m * e.ldc + hq + n) * (long)sizeof(T), Vec16<T>::from_f32(ov));
          } else {
            *(uint4*)(row + n) = Vec16<T>::from_f32(ou);
            *(uint4*)(row + hq + n) = Vec16<T>::from_f32(ov);
          }
        } else if (e.wt) {
          store16_wt(e.C, ((long)m * e.ldc + hq + n) * (long)sizeof(T), Vec16<T>::from_f32(o));
        } else {
          *(uint4*)(row + hq + n) = Vec16<T>::from_f32(o);
        }
        continue;
      }
      T* dst = (T*)e.C + (long)m * e.ldc + n;
      if (vec) {
        if (e.wt) store16_wt(e.C, ((long)m * e.ldc + n) * (long)sizeof(T), Vec16<T>::from_f32(o));
        else *(uint4*)dst = Vec16<T>::from_f32(o);
      } else {
        for (int i = 0; i < VE && n + i < nlim; ++i) st_f<T>(dst + i, o[i]);
      }
      if constexpr (EPI == EPI_SWISH_Z) {
        // the FFN hidden u = dropout(swish(z)) next to z itself (z is the backward's tape); u is formed
        // from z as stored (compute type), exactly as the backward recomputes it
        T zt[VE];
#pragma unroll
        for (int i = 0; i < VE; ++i) st_f<T>(&zt[i], o[i]);
        float u[VE];
#pragma unroll
        for (int i = 0; i < VE; ++i)
          u[i] = swishf(ld_f<T>((const T*)&zt[i])) * drop_mul(e.drop, (uint64_t)m * (uint64_t)e.ldc + (uint64_t)(n + i));
        T* du = (T*)e.C2 + (long)m * e.ldc + n;
        if (vec) *(uint4*)du = Vec16<T>::from_f32(u);
        else for (int i = 0; i < VE && n + i < nlim; ++i) st_f<T>(du + i, u[i]);
      }
    }
    if constexpr (EPI == EPI_QKV) {
      // V columns -> Vt[(b*H + h)][dd][t] as 16-byte runs of G consecutive frames ("octets" for bf16):
      // a thread takes (octet, column) jobs, consecutive threads consecutive columns (conflict-free
      // image reads).  An octet whose frames (< Tp) all lie in this tile is one vector store (frames
      // >= Tp are Vt padding and get 0); one cut by the tile edge stores only this tile's frames.
      if (n0 + TL::BN > e.qk_cols) {
        constexpr int G = 16 / (int)sizeof(T);
        const int c_lo = (e.qk_cols > n0 ? e.qk_cols - n0 : 0);
        const int ncols = min(TL::BN, p.N - n0) - c_lo;
        const int mlast = min(m0 + TL::BM, p.M) - 1;
        if (ncols > 0 && mlast >= m0) {
          const int Tp = e.Tp;
          const int ba = m0 / Tp, bb = mlast / Tp;
          auto tlo = [&](int b) { return max(m0 - b * Tp, 0); };
          auto thi = [&](int b) { return min(mlast - b * Tp, Tp - 1); };
          int noct = 0;
          for (int b = ba; b <= bb; ++b) noct += thi(b) / G - tlo(b) / G + 1;
          for (int j = tid; j < noct * ncols; j += TL::NT) {
            const int cl = c_lo + j % ncols;
            int oi = j / ncols, b = ba;
            for (;; ++b) {                             // the utterance this octet belongs to
              const int n_b = thi(b) / G - tlo(b) / G + 1;
              if (oi < n_b) break;
              oi -= n_b;
            }
            const int t0 = (tlo(b) / G + oi) * G;
            const int nv = n0 + cl - e.qk_cols;
            const int h = nv / e.dkp, dd = nv - h * e.dkp;
            float v[G];
            bool full = true;
            float2 vcd;
            if constexpr (fold) vcd = cd[cl];
#pragma unroll
            for (int q = 0; q < G; ++q) {
              const int t = t0 + q;
              const int r = b * Tp + t - m0;
              const bool own = t < Tp && r >= 0 && b * Tp + t <= mlast;
              if (t < Tp && !own) full = false;
              const int rc = min(max(r, 0), TL::BM - 1);
              float x = img[rc * TL::EPS + cl];
              if constexpr (fold) x = ln_fold(rs[rc], x, vcd);
              v[q] = own ? x : 0.0f;
            }
            T* dst = (T*)e.Vt + (((long)b * e.H + h) * e.vt_rows + dd) * e.Tpad + t0;
            if (full) {
              *(uint4*)dst = Vec16<T>::from_f32(v);
            } else {
#pragma unroll
              for (int q = 0; q < G; ++q) {
                const int t = t0 + q, r = b * Tp + t - m0;
                if (t < Tp && r >= 0 && b * Tp + t <= mlast) st_f<T>(dst + q, v[q]);
              }
            }
          }
        }
      }
    }
  }
}

// 16 values of a C^T 32x32 MFMA block (lane l: column (l & 31), rows acc_row(r, l) = four runs of 4) ->
// compute-type pairs regrouped by four v_permlane32_swap into two 16-byte chunks of 8 consecutive rows:
// lanes < 32 hold rows 0-7 / 16-23, lanes >= 32 rows 8-15 / 24-31 (conv12_kernel's computed A operand)
CFM_DEV void pack_chunks16(const float* v, uint4& c0, uint4& c1) {
  uint32_t d[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) d[q] = (uint32_t)f2bf(v[2 * q]) | ((uint32_t)f2bf(v[2 * q + 1]) << 16);
  const auto s0 = __builtin_amdgcn_permlane32_swap(d[0], d[2], false, false);
  const auto s1 = __builtin_amdgcn_permlane32_swap(d[1], d[3], false, false);
  const auto s2 = __builtin_amdgcn_permlane32_swap(d[4], d[6], false, false);
  const auto s3 = __builtin_amdgcn_permlane32_swap(d[5], d[7], false, false);
  c0 = make_uint4(s0[0], s1[0], s0[1], s1[1]);
  c1 = make_uint4(s2[0], s3[0], s2[1], s3[1]);
}

// SW (bf16 dense STORE / RELU / SWISH / RESID): the MFMA operands are swapped (weight rows as the A
// operand), so each lane's accumulator groups hold 4 consecutive output COLUMNS of one row.  The epilogue
// then works from registers: RESID writes its fp32 image as float4 runs (swizzled, EpiView SWZ), the
// compute-type outputs apply bias / fold / activation in registers and write a bf16 image of the whole
// tile in one pass (8-byte runs, 16-byte slots swizzled by row % 16) that is copied out as 16-byte rows.
// Same products in the same K order: bitwise the same values as the unswapped kernel.
template <typename T, int EPI, class TL, bool SW>
struct SwapCfg {
  static constexpr bool OUT16 = SW && (EPI == EPI_SWISH || EPI == EPI_STORE || EPI == EPI_RELU);
  static constexpr bool F32 = SW && EPI == EPI_RESID;
  static_assert(!SW || sizeof(T) == 2, "swapped operands: 16-bit compute type only");
  static_assert(!OUT16 || TL::BM * TL::BN * 2 <= TL::RS_OFF, "bf16 tile image fits below the tables");
  static_assert(!OUT16 || TL::BN >= 128, "bf16 image swizzle needs >= 16 slots per row");
  static_assert(!F32 || TL::EP == 1, "swapped RESID: one epilogue pass");
};

template <typename T, int EPI, class TL, class ALoad, bool SW = false>
__global__ __launch_bounds__(TL::NT) void gemm_kernel(GemmParams p, ALoad aload) {
  using SC = SwapCfg<T, EPI, TL, SW>;
  __shared__ __attribute__((aligned(16))) char smem[TL::LDS_BYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kg = wave / (TL::WM * TL::WN);
  const int wm = (wave % (TL::WM * TL::WN)) / TL::WN, wn = wave % TL::WN;

  // XCD-aware bijective remap: blocks sharing an XCD (bid % 8) get a contiguous tile range.
  const int nblocks = p.Mtiles * p.Ntiles;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q = nblocks >> 3, r = nblocks & 7;
  const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  const int mt = wg / p.Ntiles, nt = wg - mt * p.Ntiles;
  const int m0 = mt * TL::BM, n0 = nt * TL::BN;

  // staging geometry: instruction i of this wave covers tile rows (i*NW + wave)*8 .. +7
  int rows[TL::GA];
  int aslot[TL::GA];
#pragma unroll
  for (int i = 0; i < TL::GA; ++i) {
    rows[i] = (i * TL::NW + wave) * TL::RPI + lane / TL::SLOTS;
    aslot[i] = ((lane % TL::SLOTS) ^ TL::swz(rows[i])) * 16;
  }
  const long koff = (long)blockIdx.y * p.kb;   // split-K slice (0 without split)
  aload.shift_k(koff);
  typename ALoad::State ast;
  aload.prepare(ast, m0, rows);
  const char* wrow[TL::GB];
#pragma unroll
  for (int i = 0; i < TL::GB; ++i) {
    const int rr = (i * TL::NW + wave) * TL::RPI + lane / TL::SLOTS;
    wrow[i] = p.W + koff + (long)(n0 + rr) * p.ldw_b + ((lane % TL::SLOTS) ^ TL::swz(rr)) * 16;
  }
  const uint32_t smem_base = lds_addr(smem);
  if (p.probe & 16) {   // debug probe: poison the whole LDS image (NaN) so a read of an unwritten byte shows
    for (int i = tid; i < TL::LDS_BYTES / 4; i += TL::NT) ((uint32_t*)smem)[i] = 0xffffffffu;
    __syncthreads();
  }

  // folded LayerNorm operands, loaded now and consumed by the epilogue (the loads complete during
  // the main loop): row tid's first LN_PRE granule partials, column tid's (c, d)
  float2 ln_pre[LN_PRE];
  float2 cd_pre = make_float2(0.0f, 0.0f);
  const float2* ln_src = p.epi.ln_in;
  if (ln_src) {
    const int np = p.epi.ln_parts;
    const float2* pp = ln_src + (long)real_row(p, m0 + min(tid, TL::BM - 1), TL::BM) * np;
#pragma unroll
    for (int g = 0; g < LN_PRE; ++g) ln_pre[g] = pp[min(g, np - 1)];
    const int nc = n0 + min(tid, TL::BN - 1);
    cd_pre = make_float2(p.epi.ln_c[nc], p.epi.ln_d[nc]);
  }

  auto stage = [&](int kt, int slot) {
    const long kb0 = (long)kt * TL::BKB;
    const uint32_t sb = smem_base + slot * TL::STAGE_BYTES;
#pragma unroll
    for (int i = 0; i < TL::GA; ++i)
      glds16_asm(aload.src(ast, i, kb0, aslot[i]), sb + (i * TL::NW + wave) * 1024);
#pragma unroll
    for (int i = 0; i < TL::GB; ++i)
      glds16_asm(wrow[i] + kb0, sb + TL::BM * TL::BKB + (i * TL::NW + wave) * 1024);
  };

  f32x16 acc[TL::MR][TL::NR];
#pragma unroll
  for (int i = 0; i < TL::MR; ++i)
#pragma unroll
    for (int j = 0; j < TL::NR; ++j) acc[i][j] = f32x16{};

  const int hsel = lane >> 5;
  const int a_row0 = wm * (TL::BM / TL::WM) + (lane & 31);
  const int b_row0 = TL::BM + wn * (TL::BN / TL::WN) + (lane & 31);
  const int sw = TL::swz(lane & 31);       // rows are 32-aligned + (lane & 31)

  const int nk = (p.probe & 4) ? 1 : p.kb / TL::BKB;
  constexpr int NS = TL::NSTAGE, G = TL::GA + TL::GB, KSUB = TL::BKB / 32 / TL::KG;
  const int kk0 = kg * KSUB;   // this K-group's first substep of every K-step
  auto read_frags = [&](const char* Sb, int kk, uint4* af, uint4* bf) {
    const int so = ((2 * (kk0 + kk) + hsel) ^ sw) * 16;
#pragma unroll
    for (int i = 0; i < TL::MR; ++i) af[i] = *(const uint4*)(Sb + (a_row0 + i * 32) * TL::BKB + so);
#pragma unroll
    for (int j = 0; j < TL::NR; ++j) bf[j] = *(const uint4*)(Sb + (b_row0 + j * 32) * TL::BKB + so);
  };
  constexpr bool kAheadTile = TL::KG > 1 && NS >= 3;
  const bool ahead = kAheadTile && p.ahead;
  const int npro = ahead ? NS : NS - 1;   // the read-ahead loop keeps one more stage in flight
#pragma unroll
  for (int s = 0; s < NS; ++s)
    if (s < npro && s < nk) stage(s, s);
  float2* rs_tab = (float2*)(smem + TL::RS_OFF);
  float2* cd_tab = (float2*)(smem + TL::CD_OFF);
  if constexpr (kAheadTile) {
    if (ahead) {
      // Read-ahead loop: K-step kt's fragments (all substeps) are in registers when kt starts, and
      // kt+1's are read from LDS while kt multiplies.  The barrier at the top of kt certifies that
      // K-step kt+1 has landed for every wave and that every wave holds kt's fragments, so kt's slot
      // is refilled at once (stage kt+NS: NS-1 stages in flight).  Two fragment sets alternate (the
      // loop is unrolled by two), so no register copies.
      uint4 fa[KSUB][TL::MR + TL::NR], fb[KSUB][TL::MR + TL::NR];
      wait_stages<G, NS - 1>(min(NS - 1, nk - 1));   // K-step 0 has landed (this wave's part)
      wait_lgkm0();
      raw_barrier();
#pragma unroll
      for (int kk = 0; kk < KSUB; ++kk) read_frags(smem, kk, fa[kk], fa[kk] + TL::MR);
      auto body = [&](int kt, uint4 (&cur)[KSUB][TL::MR + TL::NR], uint4 (&nxt)[KSUB][TL::MR + TL::NR]) {
        if (kt + 1 < nk) {
          wait_stages<G, NS - 2>(min(NS - 2, nk - 2 - kt));   // K-step kt+1 has landed (this wave's part)
          wait_lgkm0();                                      // this wave holds K-step kt's fragments
          raw_barrier();
          if (kt + NS < nk && !(p.probe & 1)) stage(kt + NS, kt % NS);
        }
        // past the last K-step the reads fetch a stale slot that no MFMA uses
        const char* Sn = smem + ((kt + 1) % NS) * TL::STAGE_BYTES;
#pragma unroll
        for (int kk = 0; kk < KSUB; ++kk) {
          read_frags(Sn, kk, nxt[kk], nxt[kk] + TL::MR);
          // keep the reads ahead of this substep's MFMAs (the scheduler would sink them past all of
          // them, and the next barrier's lgkmcnt(0) would then wait on their full latency)
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int i = 0; i < TL::MR; ++i)
#pragma unroll
            for (int j = 0; j < TL::NR; ++j) {
              if constexpr (SW) mfma_slab<T>(acc[i][j], cur[kk][TL::MR + j], cur[kk][i]);
              else mfma_slab<T>(acc[i][j], cur[kk][i], cur[kk][TL::MR + j]);
            }
        }
      };
      for (int kt = 0; kt < nk; kt += 2) {
        body(kt, fa, fb);
        if (kt + 1 < nk) body(kt + 1, fb, fa);
      }
    }
  }
  if (!ahead) {
    // Software pipeline: the fragments of substep g+1 are read from LDS while the MFMAs of substep
    // g run.  The ring wait + barrier for K-step kt+1 sit in front of the LAST substep of kt, so the
    // first fragments of kt+1 are already in registers when kt+1 starts.  Two fragment sets alternate
    // by substep parity (compile-time indices): a copy of the next set into the current one at the
    // end of each substep made hipcc wait for the reads it had just issued (lgkmcnt(0) ahead of the
    // copy), exposing every LDS read latency; with the alternation nothing waits on the reads in flight
    // until the substep that uses them.  An odd substep count runs the K-step loop unrolled by two.
    wait_stages<G, NS - 2>(min(NS - 2, nk - 1));
    wait_lgkm0();
    raw_barrier();
    uint4 fa[2][TL::MR], fb[2][TL::NR];
    read_frags(smem, 0, fa[0], fb[0]);
    int slot = 0;
    auto kstep = [&](int kt, auto par0) {
      constexpr int P0 = decltype(par0)::value;   // the set holding this K-step's first fragments
      // refill the slot K-step kt-1 used: every wave finished reading it before the last barrier
      if (kt + NS - 1 < nk && !(p.probe & 1)) stage(kt + NS - 1, slot == 0 ? NS - 1 : slot - 1);
      const char* Sb = smem + slot * TL::STAGE_BYTES;
      const int nslot = (slot == NS - 1) ? 0 : slot + 1;
#pragma unroll
      for (int kk = 0; kk < KSUB; ++kk) {
        const int cur = (P0 + kk) & 1;
        const bool last = kk + 1 == KSUB, more = kt + 1 < nk;
        if (!last) {
          read_frags(Sb, kk + 1, fa[cur ^ 1], fb[cur ^ 1]);
        } else if (more) {
          wait_stages<G, NS - 2>(min(NS - 2, nk - 2 - kt));   // K-step kt+1 has landed
          // lgkmcnt(0) through the builtin, which hipcc's wait pass sees (this wave's reads of kt are done)
          __builtin_amdgcn_s_waitcnt(0xC07F);
          raw_barrier();
        }
#pragma unroll
        for (int i = 0; i < TL::MR; ++i)
#pragma unroll
          for (int j = 0; j < TL::NR; ++j) {
            if constexpr (SW) mfma_slab<T>(acc[i][j], fb[cur][j], fa[cur][i]);
            else mfma_slab<T>(acc[i][j], fa[cur][i], fb[cur][j]);
          }
        if (last && more) {
          // the next K-step's first fragments are read behind this substep's MFMAs, whose operands are
          // already in registers (read ahead of them, hipcc waited for these reads before the MFMAs)
          __builtin_amdgcn_sched_barrier(0);
          read_frags(smem + nslot * TL::STAGE_BYTES, 0, fa[cur ^ 1], fb[cur ^ 1]);
        }
      }
      slot = nslot;
    };
    if constexpr (KSUB % 2 == 0) {
      for (int kt = 0; kt < nk; ++kt) kstep(kt, std::integral_constant<int, 0>{});
    } else {
      for (int kt = 0; kt < nk; kt += 2) {
        kstep(kt, std::integral_constant<int, 0>{});
        if (kt + 1 < nk) kstep(kt + 1, std::integral_constant<int, 1>{});
      }
    }
  }

  if (p.probe & 2) {   // probe: no epilogue (keep the accumulators alive)
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < TL::MR; ++i)
#pragma unroll
      for (int j = 0; j < TL::NR; ++j) t += acc[i][j][0];
    if (t == 1234.5f) ((float*)p.epi.C)[threadIdx.x] = t;
    return;
  }
  // ---- epilogue through LDS, BM/EP rows per pass ----
  wait_lgkm0();
  raw_barrier();                         // every wave is done reading the ring
  float* img = (float*)smem;
  const int col = lane & 31;
  if constexpr (TL::KG > 1 && SW) {
    // as below, with float4 runs of the swapped layout (4 consecutive columns per accumulator group)
    using EV = EpiView<TL, true>;
    auto at4 = [&](int i, int j, int g) -> float4* {
      const int r = wm * (TL::BM / TL::WM) + i * 32 + col;
      const int c = wn * (TL::BN / TL::WN) + j * 32 + 8 * g + 4 * (lane >> 5);
      return (float4*)(img + EV::fidx(r, c));
    };
#pragma unroll
    for (int g = 1; g < TL::KG; ++g) {
      if (kg == g) {
#pragma unroll
        for (int i = 0; i < TL::MR; ++i)
#pragma unroll
          for (int j = 0; j < TL::NR; ++j)
#pragma unroll
            for (int q4 = 0; q4 < 4; ++q4) {
              float4* d = at4(i, j, q4);
              const float4 v = make_float4(acc[i][j][4 * q4], acc[i][j][4 * q4 + 1], acc[i][j][4 * q4 + 2],
                                           acc[i][j][4 * q4 + 3]);
              if (g == 1) {
                *d = v;
              } else {
                const float4 o = *d;
                *d = make_float4(o.x + v.x, o.y + v.y, o.z + v.z, o.w + v.w);
              }
            }
      }
      __syncthreads();
    }
    if (kg == 0) {
#pragma unroll
      for (int i = 0; i < TL::MR; ++i)
#pragma unroll
        for (int j = 0; j < TL::NR; ++j)
#pragma unroll
          for (int q4 = 0; q4 < 4; ++q4) {
            const float4 o = *at4(i, j, q4);
            acc[i][j][4 * q4] += o.x; acc[i][j][4 * q4 + 1] += o.y;
            acc[i][j][4 * q4 + 2] += o.z; acc[i][j][4 * q4 + 3] += o.w;
          }
    }
    __syncthreads();
  } else if constexpr (TL::KG > 1) {
    // the other K-groups hand their partial sums to K-group 0 through the image, in a fixed order
    // (img = p1; img += p2; ...; acc0 += img): bitwise reproducible, the same for every tile with
    // the same K-grouping
    auto img_at = [&](int i, int j, int rr) -> float& {
      return img[(wm * (TL::BM / TL::WM) + i * 32 + acc_row(rr, lane)) * TL::EPS + wn * (TL::BN / TL::WN) + j * 32 +
                 col];
    };
#pragma unroll
    for (int g = 1; g < TL::KG; ++g) {
      if (kg == g) {
#pragma unroll
        for (int i = 0; i < TL::MR; ++i)
#pragma unroll
          for (int j = 0; j < TL::NR; ++j)
#pragma unroll
            for (int rr = 0; rr < 16; ++rr) {
              if (g == 1) img_at(i, j, rr) = acc[i][j][rr];
              else img_at(i, j, rr) += acc[i][j][rr];
            }
      }
      __syncthreads();
    }
    if (kg == 0) {
#pragma unroll
      for (int i = 0; i < TL::MR; ++i)
#pragma unroll
        for (int j = 0; j < TL::NR; ++j)
#pragma unroll
          for (int rr = 0; rr < 16; ++rr) acc[i][j][rr] += img_at(i, j, rr);
    }
    __syncthreads();
  }
  float bcol[TL::NR];                    // bias arrays are zero-padded to the N granule (GEMM_BN)
#pragma unroll
  for (int j = 0; j < TL::NR; ++j) bcol[j] = 0.0f;
  if (p.epi.bias && !SW) {
#pragma unroll
    for (int j = 0; j < TL::NR; ++j) bcol[j] = p.epi.bias[n0 + wn * (TL::BN / TL::WN) + j * 32 + col];
  }
  // folded LayerNorm: (mean, rstd) of row tid from its granule partials (Chan et al.'s pairwise
  // combination of (count, mean, M2)) and (c, d) of column tid, from the values prefetched at the
  // kernel start; visible after the first pass's barrier
  if (ln_src) {
    const int W = p.epi.ln_width, np = p.epi.ln_parts;
    const float2* pp = ln_src + (long)real_row(p, m0 + min(tid, TL::BM - 1), TL::BM) * np;
    float sm = 0.0f;
#pragma unroll
    for (int g = 0; g < LN_PRE; ++g)
      sm += g < np ? (float)min(LN_GRANULE, W - g * LN_GRANULE) * ln_pre[g].x : 0.0f;
    for (int g = LN_PRE; g < np; ++g) sm += (float)min(LN_GRANULE, W - g * LN_GRANULE) * pp[g].x;
    const float mean = sm / (float)W;
    float m2 = 0.0f;
#pragma unroll
    for (int g = 0; g < LN_PRE; ++g) {
      const float dm = ln_pre[g].x - mean;
      m2 += g < np ? ln_pre[g].y + (float)min(LN_GRANULE, W - g * LN_GRANULE) * dm * dm : 0.0f;
    }
    for (int g = LN_PRE; g < np; ++g) {
      const float2 pg = pp[g];
      const float dm = pg.x - mean;
      m2 += pg.y + (float)min(LN_GRANULE, W - g * LN_GRANULE) * dm * dm;
    }
    if (tid < TL::BM) rs_tab[tid] = make_float2(mean, 1.0f / sqrtf(m2 / (float)W + 1e-5f));
    if (tid < TL::BN) cd_tab[tid] = cd_pre;
  }
  if constexpr (SW) {
    // this lane's 4-column bias runs (zero-padded arrays: every read in range)
    float4 b4[TL::NR][4];
#pragma unroll
    for (int j = 0; j < TL::NR; ++j)
#pragma unroll
      for (int q4 = 0; q4 < 4; ++q4)
        b4[j][q4] = p.epi.bias ? *(const float4*)(p.epi.bias + n0 + wn * (TL::BN / TL::WN) + j * 32 + 8 * q4 + 4 * (lane >> 5))
                               : make_float4(0.f, 0.f, 0.f, 0.f);
    if constexpr (SC::F32) {
      using EV = EpiView<TL, true>;
      if (kg == 0) {
#pragma unroll
        for (int i = 0; i < TL::MR; ++i)
#pragma unroll
          for (int j = 0; j < TL::NR; ++j)
#pragma unroll
            for (int q4 = 0; q4 < 4; ++q4) {
              const int r = wm * (TL::BM / TL::WM) + i * 32 + col;
              const int c = wn * (TL::BN / TL::WN) + j * 32 + 8 * q4 + 4 * (lane >> 5);
              *(float4*)(img + EV::fidx(r, c)) =
                  make_float4(acc[i][j][4 * q4] + b4[j][q4].x, acc[i][j][4 * q4 + 1] + b4[j][q4].y,
                              acc[i][j][4 * q4 + 2] + b4[j][q4].z, acc[i][j][4 * q4 + 3] + b4[j][q4].w);
            }
      }
      __syncthreads();
      if (p.epi.ln_in || p.epi.ln_out)
        epilogue<T, EPI, EV, true>(p, img, m0, n0, (long)blockIdx.y * p.split_x, rs_tab, cd_tab);
      else
        epilogue<T, EPI, EV, false>(p, img, m0, n0, (long)blockIdx.y * p.split_x, rs_tab, cd_tab);
      return;
    } else {
      // compute-type output from registers into a bf16 image [BM][BN] (16-byte slots ^ row % 16)
      constexpr int RB = TL::BN * 2, SL = TL::BN / 8;
      char* im = smem;
      __syncthreads();                   // the tables are visible; every wave is done with the image above
      if (kg == 0) {
        const bool fold = p.epi.ln_in != nullptr;
#pragma unroll
        for (int i = 0; i < TL::MR; ++i) {
          const int r = wm * (TL::BM / TL::WM) + i * 32 + col;
          float2 st = make_float2(0.f, 0.f);
          if (fold) st = rs_tab[r];
#pragma unroll
          for (int j = 0; j < TL::NR; ++j)
#pragma unroll
            for (int q4 = 0; q4 < 4; ++q4) {
              const int c = wn * (TL::BN / TL::WN) + j * 32 + 8 * q4 + 4 * (lane >> 5);
              const float bb[4] = {b4[j][q4].x, b4[j][q4].y, b4[j][q4].z, b4[j][q4].w};
              float v[4];
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                float a = acc[i][j][4 * q4 + e];
                if (fold) a = ln_fold(st, a, cd_tab[c + e]);
                else a += bb[e];
                if constexpr (EPI == EPI_RELU) a = fmaxf(a, 0.0f);
                if constexpr (EPI == EPI_SWISH) a = swishf(a);
                v[e] = a;
              }
              const uint2 pk = make_uint2((uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16),
                                          (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16));
              *(uint2*)(im + r * RB + ((((c >> 3) ^ (r & 15)) << 4) | ((c & 4) * 2))) = pk;
            }
        }
      }
      __syncthreads();
      const bool vec = (p.epi.ldc * (long)sizeof(T)) % 16 == 0;
#pragma unroll 4
      for (int idx = tid; idx < TL::BM * SL; idx += TL::NT) {
        const int r = idx / SL, c = idx - r * SL;
        const int m = m0 + r, n = n0 + 8 * c;
        if (m >= p.M || n >= p.N) continue;
        const uint4 v = *(const uint4*)(im + r * RB + ((c ^ (r & 15)) << 4));
        if (vec && n + 8 <= p.N) {
          if (p.epi.wt) store16_wt(p.epi.C, ((long)m * p.epi.ldc + n) * (long)sizeof(T), v);
          else *(uint4*)((T*)p.epi.C + (long)m * p.epi.ldc + n) = v;
        } else {
          const uint32_t w[4] = {v.x, v.y, v.z, v.w};
          for (int e = 0; e < 8 && n + e < p.N; ++e)
            ((T*)p.epi.C)[(long)m * p.epi.ldc + n + e] = (T)((w[e >> 1] >> (16 * (e & 1))) & 0xffffu);
        }
      }
      return;
    }
  }
  constexpr int WPP = TL::WM / TL::EP;   // wave rows per pass
#pragma unroll
  for (int pass = 0; pass < TL::EP; ++pass) {
    if (pass > 0) __syncthreads();       // the previous pass has read the image
    if (wm / WPP == pass && kg == 0) {
#pragma unroll
      for (int i = 0; i < TL::MR; ++i)
#pragma unroll
        for (int j = 0; j < TL::NR; ++j) {
          const int cl = wn * (TL::BN / TL::WN) + j * 32 + col;
#pragma unroll
          for (int rr = 0; rr < 16; ++rr) {
            const int rl = (wm % WPP) * (TL::BM / TL::WM) + i * 32 + acc_row(rr, lane);
            img[rl * TL::EPS + cl] = acc[i][j][rr] + bcol[j];
          }
        }
    }
    __syncthreads();
    if (p.epi.ln_in || p.epi.ln_out)
      epilogue<T, EPI, EpiView<TL>, true>(p, img, m0 + pass * EpiView<TL>::BM, n0, (long)blockIdx.y * p.split_x,
                                          rs_tab + pass * EpiView<TL>::BM, cd_tab);
    else
      epilogue<T, EPI, EpiView<TL>, false>(p, img, m0 + pass * EpiView<TL>::BM, n0, (long)blockIdx.y * p.split_x,
                                           rs_tab + pass * EpiView<TL>::BM, cd_tab);
  }
}

// ---------------------------------------------------------------------------------------------
// 8-phase 256x256 GEMM for long-K contractions (bf16; the conv2 implicit GEMM, K = 9*C):
// cdna_hip_programming.md §5 "The 256² 8-phase template" re-derived for this library's loaders.
//   * 8 waves = 2 (M) x 4 (N), wave tile 128 x 64 = 8 x 4 v_mfma_f32_16x16x32_bf16 tiles.
//   * A K-tile is 64 elements (128 B per row) in two K-halves X0 | X1 (64 B per row each); LDS holds
//     two K-tiles (parity kt & 1), each [A0 | B0 | A1 | B1] of 256 rows x 64 B (16 KB): 128 KB.
//   * 4 phases per K-tile; phase q multiplies K-half q >> 1 for the wave's row half q & 1 (16 MFMAs).
//     Each phase is [R: ds_read the phase's fragments, issue one item of global->LDS loads] barrier
//     [M: lgkmcnt(0), 16 MFMAs] barrier.  The two wave rows run one barrier apart (group 1 starts
//     with an extra barrier), so on every SIMD one wave multiplies while the other reads and loads.
//   * Loads (4 glds per thread = one K-half of A and B): R_1 of K-tile kt loads X1 of kt+1, R_3
//     loads X0 of kt+2 - each into a region whose last reader finished >= 2 barriers earlier.  Every
//     wave waits vmcnt(8) (two items younger than the one needed) before the barrier that precedes
//     wave row 0's R_0 / R_2, so the data is complete for both rows' reads.  Past the last K-tile
//     the items load the zero page (the counts stay uniform).
//   * LDS rows are 64 B: the 16-byte slot of a row is XOR-swizzled by f((row >> 2) & 3),
//     f = {0, 2, 3, 1}: every 16-lane group of a fragment ds_read_b128 hits 16 distinct bank slots.
//   * Epilogue: the same LDS image + epilogue<> as gemm_kernel, two 128-row passes.
// ---------------------------------------------------------------------------------------------
struct T8 {
  static constexpr int BM = 256, BN = 256, NT = 512, EP = 2, EPS = 256, WM = 2;
};
constexpr int G8_HALF = 256 * 64;       // one K-half image of one operand
constexpr int G8_BUF = 4 * G8_HALF;     // one K-tile: A0 | B0 | A1 | B1
static_assert(2 * G8_BUF >= T8::BM / T8::EP * T8::EPS * 4, "epilogue image fits the ring");
CFM_DEV int g8_swz(int row) { return (0x78 >> (2 * ((row >> 2) & 3))) & 3; }

template <int EPI, class ALoad, bool SPREAD = false>
__global__ __launch_bounds__(512) void gemm8_kernel(GemmParams p, ALoad aload) {
  __shared__ __attribute__((aligned(16))) char smem[2 * G8_BUF];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;   // wave row = stagger group (waves w and w+4 share a SIMD)

  const int nblocks = p.Mtiles * p.Ntiles;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, qq = nblocks >> 3, rr = nblocks & 7;
  const int wg = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
  const int mt = wg / p.Ntiles, ntl = wg - mt * p.Ntiles;
  const int m0 = mt * 256, n0 = ntl * 256;

  // staging: instruction i (0, 1) of this wave fills rows (i*8 + wave)*16 .. +15 of a K-half image
  int rows[2], lo[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    rows[i] = (i * 8 + wave) * 16 + (lane >> 2);
    lo[i] = ((lane & 3) ^ g8_swz(rows[i])) * 16;
  }
  typename ALoad::State ast;
  aload.prepare(ast, m0, rows);
  const char* wrow[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) wrow[i] = p.W + (long)(n0 + rows[i]) * p.ldw_b + lo[i];
  const char* zsrc = aload.zero + lane * 16;
  const uint32_t sbase = lds_addr(smem);
  const int nk = p.kb / 128;

  auto issue = [&](int kt, int h, int parts = 3) {   // K-half h of K-tile kt, A (parts & 1) then B (parts & 2)
    const uint32_t base = sbase + (kt & 1) * G8_BUF + h * 2 * G8_HALF;
    const bool live = kt < nk;        // past the end: the zero page (uniform vmcnt counts)
    const int kb0 = kt * 128 + h * 64;
    if (!(parts & 1)) {
    } else if constexpr (ALoad::kConv) {
      const int tapb = (int)aload.tapb;   // bytes of one 3x3 tap (C * 2); a K-half never straddles two
      int tap = 0;                        // wave-uniform: count the tap boundaries below kb0 (no division)
#pragma unroll
      for (int t = 1; t < 9; ++t) tap += kb0 >= t * tapb ? 1 : 0;
      const int tr = (tap >= 3 ? 1 : 0) + (tap >= 6 ? 1 : 0), tf = tap - 3 * tr;
      const long toff = ((long)tr * aload.F1 + tf) * tapb + (kb0 - tap * tapb);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const bool v = live && ((ast.valid[i] >> tap) & 1u);
        const char* src = v ? ast.base[i] + toff + lo[i] : zsrc;
        glds16_asm(src, base + (i * 8 + wave) * 1024);
      }
    } else {   // dense rows (GEMM A operand): rows past M and bytes past K read the zero page
#pragma unroll
      for (int i = 0; i < 2; ++i)
        glds16_asm(live ? aload.src(ast, i, kb0, lo[i]) : (const void*)zsrc, base + (i * 8 + wave) * 1024);
    }
    if (parts & 2) {
#pragma unroll
      for (int i = 0; i < 2; ++i) glds16_asm(live ? wrow[i] + kb0 : zsrc, base + G8_HALF + (i * 8 + wave) * 1024);
    }
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{};

  const int fr = lane & 15, fc = lane >> 4;
  const int fslot = (fc ^ g8_swz(fr)) * 16;   // rows are 16-aligned + fr
  uint4 af[4], bfr[4];
  auto read_frags = [&](int kt, int q) {
    const char* hb = smem + (kt & 1) * G8_BUF + (q >> 1) * 2 * G8_HALF;
    const int r0 = wm * 128 + (q & 1) * 64 + fr;
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = *(const uint4*)(hb + (r0 + i * 16) * 64 + fslot);
    if ((q & 1) == 0) {
      const int c0 = wn * 64 + fr;
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = *(const uint4*)(hb + G8_HALF + (c0 + j * 16) * 64 + fslot);
    }
  };

  // prologue: X0(0), X1(0), X0(1); X0(0) complete for every wave, then wave row 1 falls one barrier behind
  issue(0, 0);
  issue(0, 1);
  issue(1, 0);
  wait_vmcnt<8>();
  wait_lgkm0();
  raw_barrier();
  if (wm == 1) raw_barrier();
  for (int kt = 0; kt < nk; ++kt) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      // R_q
      read_frags(kt, q);
      if constexpr (SPREAD) {
        // one operand's half per phase (2 glds), each as early as its region's last read allows: B1 was
        // last read in R_2 of kt-1, A1 in R_3 of kt-1, B0 in R_0 of kt, A0 in R_1 of kt (the counts seen
        // by the vmcnt(8) waits are unchanged: the same 8 glds are younger at each wait)
        if (q == 0) issue(kt + 1, 1, 2);
        if (q == 1) issue(kt + 1, 1, 1);
        if (q == 2) issue(kt + 2, 0, 2);
        if (q == 3) issue(kt + 2, 0, 1);
      } else {
        if (q == 1) issue(kt + 1, 1);
        if (q == 3) issue(kt + 2, 0);
      }
      if (wm == 1 && (q & 1)) wait_vmcnt<8>();   // before the barrier preceding row 0's R_{q+1}
      raw_barrier();
      // M_q
      wait_lgkm0();
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[(q & 1) * 4 + i][j] = mfma16_16x16x32(af[i], bfr[j], acc[(q & 1) * 4 + i][j]);
      __builtin_amdgcn_s_setprio(0);
      if (wm == 0 && (q & 1)) wait_vmcnt<8>();
      raw_barrier();
    }
  }
  if (wm == 0) raw_barrier();   // re-align the barrier counts of the two wave rows
  wait_vmcnt<0>();
  wait_lgkm0();
  raw_barrier();

  if (p.probe & 2) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) t += acc[i][j][0];
    if (t == 1234.5f) ((float*)p.epi.C)[threadIdx.x] = t;
    return;
  }
  // ---- epilogue: two passes of 128 rows (pass p = wave row p), image [128][256] fp32 ----
  float* img = (float*)smem;
  float bcol[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) bcol[j] = p.epi.bias ? p.epi.bias[n0 + wn * 64 + j * 16 + fr] : 0.0f;
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    if (pass > 0) __syncthreads();
    if (wm == pass) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            img[(i * 16 + fc * 4 + e) * T8::EPS + wn * 64 + j * 16 + fr] = acc[i][j][e] + bcol[j];
    }
    __syncthreads();
    epilogue<bf16_t, EPI, EpiView<T8>, false>(p, img, m0 + pass * 128, n0, 0, nullptr, nullptr);
  }
}

// ---------------------------------------------------------------------------------------------
// conv1 -> conv2 fused (ConvSubsampling conv.0 + ReLU + conv.2 + ReLU, subsampling.py:105-116, 173):
// the 8-phase implicit GEMM above (gemm8_kernel) with its A operand COMPUTED on the matrix cores instead
// of loaded.  A[m][tap*C + c] = X1[b][t1][f1][c] = ReLU(b1[c] + sum_k W1[c][k] * x[b][2f1-1+e][2t1-1+a]),
// k = 3a + e, at the conv2 input pixel (t1, f1) = (2t2-1+kt, 2f2-1+kf) of output row m = (b, t2, f2)
// (zero outside the X1 image), so the 655 MB X1 image of the two-kernel path (and conv.2's 2.5x
// over-fetch of it) is never written nor read.
//   * conv.0 is itself a K = 16 contraction: [9 taps | in-image flag | 0 x 6] . [W1[c][0..8] | b1[c] | 0].
//     A pre-pass (conv12_patch_kernel) writes every conv2-input pixel's 16-element fp16 patch (taps
//     zero-padded as conv.0 pads; all zero on conv.2's padding ring, so X1 = ReLU(0) = 0 there) and W1 as
//     [c][16] fp16.  The products run on v_mfma_f32_32x32x16_f16 (fp16 operands, fp32 sums; the patch and
//     W1 in fp16 round to 11 bits, finer than the 8-bit bf16 rounding of X1 that follows).
//   * Per K-half (32 channels of one tap) wave w computes X1 for tile rows 32w .. 32w+31: ONE MFMA
//     (W1 rows = channels as the A operand, the patch as B: lane l holds row 32w + (l & 31) and four runs of
//     4 consecutive channels), ReLU, bf16 pairs regrouped into 16-byte chunks of 8 channels by four
//     v_permlane32_swap, two ds_write_b128 into the XOR-swizzled A half-image - in the R-phase slots where
//     gemm8_kernel issues the A half's LDS-DMA, so every write lands >= 2 barriers after the region's last
//     read and before its first.
//   * LDS: the 8-phase ring (128 KiB: A images computed, B = W2 by LDS-DMA as before), W1 as [C][16] fp16
//     (C * 32 B, loaded once per block) and the patch fragments [tap & 1][wave][lane] (2 x 8 KiB).
//     Wave w's patch rows for tap(kt + 4) are fetched by ONE 1-KiB LDS-DMA per K-tile (R_3, next to the
//     B half), four K-tiles ahead of their first use; a tap's rows are re-fetched into the same buffer
//     until the next tap's begin (identical bytes), which keeps the vmcnt counts uniform:
//     R_1 issues 2 DMAs (B), R_3 issues 3 (B + patch), so "two items younger" is vmcnt(5).
// ---------------------------------------------------------------------------------------------
struct Conv12Args {
  const uint4* patch;   // conv12_patch_kernel: (B, T1+2, F1+2) x 32 B fp16 patches (conv.2's padding ring included)
  const uint4* w1h;     // conv.0 weight + bias as [c][16] fp16
  const char* zero;     // zero page
  int T1, F1, T2, F2, C;
};
constexpr int C12_MAXC = 512;

__global__ __launch_bounds__(256) void conv12_patch_kernel(const float* __restrict__ x, int B, int F, int T, int T1,
                                                           int F1, uint4* __restrict__ patch, const float* __restrict__ w1,
                                                           const float* __restrict__ b1, int C, uint4* __restrict__ w1h) {
  typedef __attribute__((ext_vector_type(2))) _Float16 h2;
  // saturated to the fp16 range (v_med3_f32) before the conversion: an input or weight beyond +-65504
  // gives a clamped product instead of inf / NaN in X1 (the two-kernel path stays in fp32 there)
  auto sat = [](float v) { return (_Float16)__builtin_amdgcn_fmed3f(v, -65504.0f, 65504.0f); };
  auto pk = [&](float a, float b) { return __builtin_bit_cast(uint32_t, h2{sat(a), sat(b)}); };
  const int W = F1 + 2, Hh = T1 + 2;
  const long n = (long)B * Hh * W;
  if (blockIdx.x == 0)   // conv.0 weights as [c][16] fp16 rows: W1[c][0..8], b1[c], zeros
    for (int c = threadIdx.x; c < C; c += 256) {
      float v[16] = {};
      for (int k = 0; k < 9; ++k) v[k] = w1[(long)c * 9 + k];
      v[9] = b1[c];
      w1h[2 * c] = make_uint4(pk(v[0], v[1]), pk(v[2], v[3]), pk(v[4], v[5]), pk(v[6], v[7]));
      w1h[2 * c + 1] = make_uint4(pk(v[8], v[9]), 0u, 0u, 0u);
    }
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const int fi = (int)(i % W);
    const long r = i / W;
    const int ti = (int)(r % Hh), b = (int)(r / Hh);
    const int t1 = ti - 1, f1 = fi - 1;
    const bool ok = t1 >= 0 && t1 < T1 && f1 >= 0 && f1 < F1;
    float v[10];
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
      for (int e = 0; e < 3; ++e) {
        const int t = 2 * t1 - 1 + a, f = 2 * f1 - 1 + e;
        v[3 * a + e] = (ok && t >= 0 && t < T && f >= 0 && f < F) ? x[((long)b * F + f) * T + t] : 0.0f;
      }
    v[9] = ok ? 1.0f : 0.0f;
    patch[2 * i] = make_uint4(pk(v[0], v[1]), pk(v[2], v[3]), pk(v[4], v[5]), pk(v[6], v[7]));
    patch[2 * i + 1] = make_uint4(pk(v[8], v[9]), 0u, 0u, 0u);
  }
}

constexpr int C12_PATCH = 2 * 8 * 1024;               // [tap & 1][wave][64 lanes x 16 B]
constexpr int C12_LDS = 2 * G8_BUF + C12_PATCH + C12_MAXC * 32;
static_assert(C12_LDS <= 160 * 1024, "conv12 LDS");

__global__ __launch_bounds__(512) void conv12_kernel(GemmParams p, Conv12Args ca) {
  __shared__ __attribute__((aligned(16))) char smem[C12_LDS];
  typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int C = ca.C;

  // block -> tile as gemm8_kernel (giving each XCD parity one of the two column tiles, so that an XCD's L2
  // holds half of W2, measured neutral: profiles/r04g_conv12_xcd_cols_ab.txt)
  const int nblocks = p.Mtiles * p.Ntiles;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, qq = nblocks >> 3, rr = nblocks & 7;
  const int wg = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
  const int mt = wg / p.Ntiles, ntl = wg - mt * p.Ntiles;
  const int m0 = mt * 256, n0 = ntl * 256;

  // B staging (W2 rows): as gemm8_kernel
  int rows[2], lo[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    rows[i] = (i * 8 + wave) * 16 + (lane >> 2);
    lo[i] = ((lane & 3) ^ g8_swz(rows[i])) * 16;
  }
  const char* wrow[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) wrow[i] = p.W + (long)(n0 + rows[i]) * p.ldw_b + lo[i];
  const char* zsrc = ca.zero + lane * 16;
  const uint32_t sbase = lds_addr(smem);
  const int nk = p.kb / 128;
  const int ktap = C / 64;                       // K-tiles per conv.2 tap

  // this lane's X1 row (tile row 32 * wave + (lane & 31)) and its conv2-input pixel base (ring grid)
  const int xrow = 32 * wave + (lane & 31);
  const int am = m0 + xrow;
  const bool arow_ok = am < p.M;
  const int amc = min(am, p.M - 1);
  const int af2 = amc % ca.F2, bt = amc / ca.F2;
  const int at2 = bt % ca.T2, ab = bt / ca.T2;
  const uint4* prow = ca.patch + 2 * (((long)ab * (ca.T1 + 2) + 2 * at2) * (ca.F1 + 2) + 2 * af2) + (lane >> 5);
  const uint32_t pbase = sbase + 2 * G8_BUF;     // patch fragments
  const char* w1img = smem + 2 * G8_BUF + C12_PATCH;

  // LDS-DMA of this wave's patch rows for conv.2 tap `tap` (clamped) into buffer tap & 1
  auto issue_patch = [&](int tap) {
    tap = min(tap, 8);
    const int kt2 = tap / 3, kf2 = tap - 3 * kt2;
    const void* src = arow_ok ? (const void*)(prow + 2 * (kt2 * (ca.F1 + 2) + kf2)) : (const void*)zsrc;
    glds16_asm(src, pbase + (tap & 1) * 8192 + wave * 1024);
  };
  auto issue_b = [&](int kt, int h) {   // K-half h of K-tile kt of W2: 2 LDS-DMA
    const uint32_t base = sbase + (kt & 1) * G8_BUF + h * 2 * G8_HALF;
    const bool live = kt < nk;
    const int kb0 = kt * 128 + h * 64;
#pragma unroll
    for (int i = 0; i < 2; ++i) glds16_asm(live ? wrow[i] + kb0 : zsrc, base + G8_HALF + (i * 8 + wave) * 1024);
  };
  // X1 for K-half (kt, h): 32 channels of tap kt / ktap, rows 32 * wave + (lane & 31).  Two halves so
  // that the MFMA's latency is not waited for inside one R phase: x1_mfma issues the contraction, one
  // phase later x1_store converts (bf16 pairs, ReLU as a packed int16 max on the bf16 bits: negative
  // values have the sign bit set, so max(x, 0) as int16 is max(x, +0) as bf16), regroups and writes.
  // its operands (W1 rows, this wave's patch rows) read before the phase's fragment reads, so the
  // contraction waits only for them; past the last K-tile the clamped K-tile's operands (the result is
  // not stored), so the result is not consumed in the phase it is issued in
  auto x1_ops = [&](int kt, int h, uint4& wf, uint4& pf) {
    const int ktc = min(kt, nk - 1);
    const int tap = ktc / ktap;
    const int c0 = (ktc - tap * ktap) * 64 + 32 * h;
    wf = *(const uint4*)(w1img + (c0 + (lane & 31)) * 32 + (lane >> 5) * 16);
    pf = *(const uint4*)(smem + 2 * G8_BUF + (tap & 1) * 8192 + wave * 1024 + lane * 16);
  };
  auto x1_mma = [&](const uint4& wf, const uint4& pf) -> f32x16 {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, wf), __builtin_bit_cast(f16x8, pf),
                                                 f32x16{}, 0, 0, 0);
  };
  auto x1_mfma = [&](int kt, int h) -> f32x16 {
    uint4 wf, pf;
    x1_ops(kt, h, wf, pf);
    return x1_mma(wf, pf);
  };
  auto x1_store = [&](int kt, int h, const f32x16& d) {
    if (kt >= nk) return;
    typedef __attribute__((ext_vector_type(2))) short s16x2;
    uint32_t q[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const uint32_t u = pk_bf16x2(d[2 * i], d[2 * i + 1]);
      q[i] = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(s16x2, u), (s16x2){0, 0}));
    }
    const auto s0 = __builtin_amdgcn_permlane32_swap(q[0], q[2], false, false);
    const auto s1 = __builtin_amdgcn_permlane32_swap(q[1], q[3], false, false);
    const auto s2 = __builtin_amdgcn_permlane32_swap(q[4], q[6], false, false);
    const auto s3 = __builtin_amdgcn_permlane32_swap(q[5], q[7], false, false);
    char* img = smem + (kt & 1) * G8_BUF + h * 2 * G8_HALF;
    const int hi = lane >> 5, sw = g8_swz(xrow);
    // lanes < 32: channels 0-7 / 16-23 of the K-half, lanes >= 32: 8-15 / 24-31
    *(uint4*)(img + xrow * 64 + ((hi) ^ sw) * 16) = make_uint4(s0[0], s1[0], s0[1], s1[1]);
    *(uint4*)(img + xrow * 64 + ((2 + hi) ^ sw) * 16) = make_uint4(s2[0], s3[0], s2[1], s3[1]);
  };
  auto compute_x1 = [&](int kt, int h) { x1_store(kt, h, x1_mfma(kt, h)); };

  // conv.0's weights into LDS (C x 32 B), once per block, before any LDS-DMA is in flight (plain loads:
  // hipcc waits for them here); visible to every wave after the raw barrier
  for (int i = tid; i < 2 * C; i += 512) ((uint4*)w1img)[i] = ca.w1h[i];
  wait_lgkm0();
  raw_barrier();

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{};

  const int fr = lane & 15, fc = lane >> 4;
  const int fslot = (fc ^ g8_swz(fr)) * 16;
  uint4 af[4], bfr[4];
  auto read_frags = [&](int kt, int q) {
    const char* hb = smem + (kt & 1) * G8_BUF + (q >> 1) * 2 * G8_HALF;
    const int r0 = wm * 128 + (q & 1) * 64 + fr;
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = *(const uint4*)(hb + (r0 + i * 16) * 64 + fslot);
    if ((q & 1) == 0) {
      const int c0 = wn * 64 + fr;
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = *(const uint4*)(hb + G8_HALF + (c0 + j * 16) * 64 + fslot);
    }
  };

  // prologue: tap 0's patch, B halves (0,0), (0,1), (1,0) (+ the patch of tap(4), as R_3 does), then the
  // A halves (0,0), (0,1), (1,0) computed
  issue_patch(0);
  issue_b(0, 0);
  issue_b(0, 1);
  issue_b(1, 0);
  issue_patch(4 / ktap);
  wait_vmcnt<7>();            // tap 0's patch has landed (this wave's own rows: no barrier needed)
  compute_x1(0, 0);
  compute_x1(0, 1);
  compute_x1(1, 0);
  wait_vmcnt<5>();            // B (0,0) complete; (0,1) and (1,0) + patch in flight
  wait_lgkm0();
  raw_barrier();
  if (wm == 1) raw_barrier();
  f32x16 xd;
  // timing probes (CFM_GEMM_PROBE, wrong results): 8 no X1 computation in the loop, 16 no W2 / patch
  // LDS-DMA in the loop, 32 no MFMAs in the M phases, 64 no fragment reads
  const int probe = p.probe;
  const int nkl = (probe & 128) ? 0 : nk;   // 128: no main loop (prologue + epilogue only)
  for (int kt = 0; kt < nkl; ++kt) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      // R_q
      uint4 xw, xp;
      if (!(probe & 8)) {
        if (q == 0) x1_ops(kt + 1, 1, xw, xp);
        if (q == 2) x1_ops(kt + 2, 0, xw, xp);
      }
      if (!(probe & 64)) read_frags(kt, q);
      // the A halves the DMA version loads at R_1 / R_3: contraction issued one phase earlier
      if (!(probe & 8)) {
        if (q == 0 || q == 2) xd = x1_mma(xw, xp);
        if (q == 1) x1_store(kt + 1, 1, xd);
        if (q == 3) x1_store(kt + 2, 0, xd);
      }
      if (!(probe & 16)) {
        if (q == 1) issue_b(kt + 1, 1);
        if (q == 3) { issue_b(kt + 2, 0); issue_patch((kt + 4) / ktap); }
      }
      if (wm == 1 && (q & 1)) wait_vmcnt<5>();   // before the barrier preceding row 0's R_{q+1}
      raw_barrier();
      // M_q
      wait_lgkm0();
      __builtin_amdgcn_s_setprio(1);
      if (!(probe & 32)) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[(q & 1) * 4 + i][j] = mfma16_16x16x32(af[i], bfr[j], acc[(q & 1) * 4 + i][j]);
      }
      __builtin_amdgcn_s_setprio(0);
      if (wm == 0 && (q & 1)) wait_vmcnt<5>();
      raw_barrier();
    }
  }
  if (wm == 0) raw_barrier();   // re-align the barrier counts of the two wave rows
  wait_vmcnt<0>();
  wait_lgkm0();
  raw_barrier();

  if (probe & 256) {   // 256: no epilogue (keep the accumulators live)
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) t += acc[i][j][0];
    if (t == 1234.5f) ((float*)p.epi.C)[threadIdx.x] = t;
    return;
  }
  float* img = (float*)smem;
  float bcol[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) bcol[j] = p.epi.bias ? p.epi.bias[n0 + wn * 64 + j * 16 + fr] : 0.0f;
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    if (pass > 0) __syncthreads();
    if (wm == pass) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            img[(i * 16 + fc * 4 + e) * T8::EPS + wn * 64 + j * 16 + fr] = acc[i][j][e] + bcol[j];
    }
    __syncthreads();
    epilogue<bf16_t, EPI_RELU, EpiView<T8>, false>(p, img, m0 + pass * 128, n0, 0, nullptr, nullptr);
  }
}

// PROBE: timing studies only (CFM_GEMM_PROBE bits as conv12_kernel's: 8 no X1, 16 no LDS-DMA, 32 no main MFMAs,
// 64 no fragment reads, 256 no epilogue; wrong results)
template <bool PROBE>
__global__ __launch_bounds__(512) void conv12b_kernel(GemmParams p, Conv12Args ca) {
  __shared__ __attribute__((aligned(16))) char smem[C12_LDS];
  typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int C = ca.C;

  // block -> tile as gemm8_kernel (giving each XCD parity one of the two column tiles, so that an XCD's L2
  // holds half of W2, measured neutral: profiles/r04g_conv12_xcd_cols_ab.txt)
  const int nblocks = p.Mtiles * p.Ntiles;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, qq = nblocks >> 3, rr = nblocks & 7;
  const int wg = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
  const int mt = wg / p.Ntiles, ntl = wg - mt * p.Ntiles;
  const int m0 = mt * 256, n0 = ntl * 256;

  // B staging (W2 rows): as gemm8_kernel
  int rows[2], lo[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    rows[i] = (i * 8 + wave) * 16 + (lane >> 2);
    lo[i] = ((lane & 3) ^ g8_swz(rows[i])) * 16;
  }
  const char* wrow[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) wrow[i] = p.W + (long)(n0 + rows[i]) * p.ldw_b + lo[i];
  const char* zsrc = ca.zero + lane * 16;
  const uint32_t sbase = lds_addr(smem);
  const int nk = p.kb / 128;
  const int ktap = C / 64;                       // K-tiles per conv.2 tap

  // this lane's X1 row (tile row 32 * wave + (lane & 31)) and its conv2-input pixel base (ring grid)
  const int xrow = 32 * wave + (lane & 31);
  const int am = m0 + xrow;
  const bool arow_ok = am < p.M;
  const int amc = min(am, p.M - 1);
  const int af2 = amc % ca.F2, bt = amc / ca.F2;
  const int at2 = bt % ca.T2, ab = bt / ca.T2;
  const uint4* prow = ca.patch + 2 * (((long)ab * (ca.T1 + 2) + 2 * at2) * (ca.F1 + 2) + 2 * af2) + (lane >> 5);
  const uint32_t pbase = sbase + 2 * G8_BUF;     // patch fragments
  const char* w1img = smem + 2 * G8_BUF + C12_PATCH;

  // LDS-DMA of this wave's patch rows for conv.2 tap `tap` (clamped) into buffer tap & 1
  auto issue_patch = [&](int tap) {
    tap = min(tap, 8);
    const int kt2 = tap / 3, kf2 = tap - 3 * kt2;
    const void* src = arow_ok ? (const void*)(prow + 2 * (kt2 * (ca.F1 + 2) + kf2)) : (const void*)zsrc;
    glds16_asm(src, pbase + (tap & 1) * 8192 + wave * 1024);
  };
  auto issue_b = [&](int kt, int h) {   // K-half h of K-tile kt of W2: 2 LDS-DMA
    const uint32_t base = sbase + (kt & 1) * G8_BUF + h * 2 * G8_HALF;
    const bool live = kt < nk;
    const int kb0 = kt * 128 + h * 64;
#pragma unroll
    for (int i = 0; i < 2; ++i) glds16_asm(live ? wrow[i] + kb0 : zsrc, base + G8_HALF + (i * 8 + wave) * 1024);
  };
  // X1 for K-half (kt, h): 32 channels of tap kt / ktap, rows 32 * wave + (lane & 31).  Two halves so
  // that the MFMA's latency is not waited for inside one R phase: x1_mfma issues the contraction, one
  // phase later x1_store converts (bf16 pairs, ReLU as a packed int16 max on the bf16 bits: negative
  // values have the sign bit set, so max(x, 0) as int16 is max(x, +0) as bf16), regroups and writes.
  // its operands (W1 rows, this wave's patch rows) read before the phase's fragment reads, so the
  // contraction waits only for them; past the last K-tile the clamped K-tile's operands (the result is
  // not stored), so the result is not consumed in the phase it is issued in
  auto x1_ops = [&](int kt, int h, uint4& wf, uint4& pf) {
    const int ktc = min(kt, nk - 1);
    const int tap = ktc / ktap;
    const int c0 = (ktc - tap * ktap) * 64 + 32 * h;
    wf = *(const uint4*)(w1img + (c0 + (lane & 31)) * 32 + (lane >> 5) * 16);
    pf = *(const uint4*)(smem + 2 * G8_BUF + (tap & 1) * 8192 + wave * 1024 + lane * 16);
  };
  auto x1_mma = [&](const uint4& wf, const uint4& pf) -> f32x16 {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, wf), __builtin_bit_cast(f16x8, pf),
                                                 f32x16{}, 0, 0, 0);
  };
  auto x1_mfma = [&](int kt, int h) -> f32x16 {
    uint4 wf, pf;
    x1_ops(kt, h, wf, pf);
    return x1_mma(wf, pf);
  };
  auto x1_store = [&](int kt, int h, const f32x16& d) {
    if (kt >= nk) return;
    typedef __attribute__((ext_vector_type(2))) short s16x2;
    uint32_t q[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const uint32_t u = pk_bf16x2(d[2 * i], d[2 * i + 1]);
      q[i] = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(s16x2, u), (s16x2){0, 0}));
    }
    const auto s0 = __builtin_amdgcn_permlane32_swap(q[0], q[2], false, false);
    const auto s1 = __builtin_amdgcn_permlane32_swap(q[1], q[3], false, false);
    const auto s2 = __builtin_amdgcn_permlane32_swap(q[4], q[6], false, false);
    const auto s3 = __builtin_amdgcn_permlane32_swap(q[5], q[7], false, false);
    char* img = smem + (kt & 1) * G8_BUF + h * 2 * G8_HALF;
    const int hi = lane >> 5, sw = g8_swz(xrow);
    // lanes < 32: channels 0-7 / 16-23 of the K-half, lanes >= 32: 8-15 / 24-31
    *(uint4*)(img + xrow * 64 + ((hi) ^ sw) * 16) = make_uint4(s0[0], s1[0], s0[1], s1[1]);
    *(uint4*)(img + xrow * 64 + ((2 + hi) ^ sw) * 16) = make_uint4(s2[0], s3[0], s2[1], s3[1]);
  };
  auto compute_x1 = [&](int kt, int h) { x1_store(kt, h, x1_mfma(kt, h)); };

  // conv.0's weights into LDS (C x 32 B), once per block, before any LDS-DMA is in flight (plain loads:
  // hipcc waits for them here); visible to every wave after the raw barrier
  for (int i = tid; i < 2 * C; i += 512) ((uint4*)w1img)[i] = ca.w1h[i];
  wait_lgkm0();
  raw_barrier();

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{};

  const int fr = lane & 15, fc = lane >> 4;
  const int fslot = (fc ^ g8_swz(fr)) * 16;
  uint4 af[8], bfr[4];
  auto read_frags = [&](int kt, int h) {   // K-half h of K-tile kt: the wave's 128 rows and 64 columns
    const char* hb = smem + (kt & 1) * G8_BUF + h * 2 * G8_HALF;
    const int r0 = wm * 128 + fr;
#pragma unroll
    for (int i = 0; i < 8; ++i) af[i] = *(const uint4*)(hb + (r0 + i * 16) * 64 + fslot);
    const int c0 = wn * 64 + fr;
#pragma unroll
    for (int j = 0; j < 4; ++j) bfr[j] = *(const uint4*)(hb + G8_HALF + (c0 + j * 16) * 64 + fslot);
  };

  // prologue: tap 0's patch and the B halves (0,0), (0,1); the A halves (0,0), (0,1) computed, (1,0)'s
  // contraction issued (stored in R_0 of K-tile 0)
  issue_patch(0);
  issue_b(0, 0);
  issue_b(0, 1);
  wait_vmcnt<4>();            // tap 0's patch has landed (this wave's own rows: no barrier needed)
  compute_x1(0, 0);
  compute_x1(0, 1);
  f32x16 xd0 = x1_mfma(1, 0), xd1;
  wait_vmcnt<2>();            // B (0,0) complete; (0,1) in flight
  wait_lgkm0();
  raw_barrier();
  if (wm == 1) raw_barrier();
  for (int kt = 0; kt < nk; ++kt) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      // R_h: K-half h's fragments; K-half h of K-tile kt + 1 into the other buffer (its last readers
      // finished R_h of K-tile kt - 1, two phases ago): W2 by LDS-DMA, X1 computed (contraction one
      // phase earlier)
      const int pb = PROBE ? p.probe : 0;
      uint4 xw, xp;
      if (!(pb & 8)) x1_ops(h == 0 ? kt + 1 : kt + 2, h ^ 1, xw, xp);
      if (!(pb & 64)) read_frags(kt, h);
      if (h == 0) {
        if (!(pb & 8)) { x1_store(kt + 1, 0, xd0); xd1 = x1_mma(xw, xp); }
        if (!(pb & 16)) { issue_b(kt + 1, 0); issue_patch((kt + 4) / ktap); }
      } else {
        if (!(pb & 8)) { x1_store(kt + 1, 1, xd1); xd0 = x1_mma(xw, xp); }
        if (!(pb & 16)) issue_b(kt + 1, 1);
      }
      // before the barrier preceding row 0's next R phase: that phase's W2 half has landed (three
      // younger LDS-DMA per wave: the next half's two and a patch)
      if (wm == 1) wait_vmcnt<3>();
      raw_barrier();
      // M_h: 32 MFMAs
      wait_lgkm0();
      __builtin_amdgcn_s_setprio(1);
      if (!(pb & 32)) {
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = mfma16_16x16x32(af[i], bfr[j], acc[i][j]);
      }
      __builtin_amdgcn_s_setprio(0);
      if (wm == 0) wait_vmcnt<3>();
      raw_barrier();
    }
  }
  if (wm == 0) raw_barrier();   // re-align the barrier counts of the two wave rows
  wait_vmcnt<0>();
  wait_lgkm0();
  raw_barrier();

  if (PROBE && (p.probe & 256)) {   // keep the accumulators live
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) t += acc[i][j][0];
    if (t == 1234.5f) ((float*)p.epi.C)[threadIdx.x] = t;
    return;
  }
  float* img = (float*)smem;
  float bcol[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) bcol[j] = p.epi.bias ? p.epi.bias[n0 + wn * 64 + j * 16 + fr] : 0.0f;
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    if (pass > 0) __syncthreads();
    if (wm == pass) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            img[(i * 16 + fc * 4 + e) * T8::EPS + wn * 64 + j * 16 + fr] = acc[i][j][e] + bcol[j];
    }
    __syncthreads();
    epilogue<bf16_t, EPI_RELU, EpiView<T8>, false>(p, img, m0 + pass * 128, n0, 0, nullptr, nullptr);
  }
}

template <typename T, class TL, template <int> class AL, class ALArgs>
void launch_epi(const GemmParams& p, const ALArgs& args, hipStream_t st) {
  using ALoad = AL<TL::GA>;
  ALoad al;
  args.fill(al);
  const dim3 grid(p.Mtiles * p.Ntiles, p.split_x > 0 ? g_splits : 1), block(TL::NT);
  if constexpr (ALoad::kConv) {
    cfm_launch((gemm_kernel<T, EPI_RELU, TL, ALoad>), grid, block, 0, st, p, al);
    return;
  }
  if constexpr (sizeof(T) == 2) {
    // the swapped-operand epilogues (SwapCfg); CFM_GEMM_SWAP=0 keeps the unswapped kernels (A/B)
    const bool resid_ok = TL::EP == 1 && !p.epi.out_scalar;
    if (g_gemm_swap && p.epi.utt_tp <= 0) {
      switch (p.epi.mode) {
        case EPI_STORE: cfm_launch((gemm_kernel<T, EPI_STORE, TL, ALoad, true>), grid, block, 0, st, p, al); return;
        case EPI_RELU: cfm_launch((gemm_kernel<T, EPI_RELU, TL, ALoad, true>), grid, block, 0, st, p, al); return;
        case EPI_SWISH: cfm_launch((gemm_kernel<T, EPI_SWISH, TL, ALoad, true>), grid, block, 0, st, p, al); return;
        case EPI_RESID:
          if constexpr (TL::EP == 1) {
            if (resid_ok) {
              cfm_launch((gemm_kernel<T, EPI_RESID, TL, ALoad, true>), grid, block, 0, st, p, al);
              return;
            }
          }
          break;
        default: break;
      }
    }
  }
  switch (p.epi.mode) {
    case EPI_STORE: cfm_launch((gemm_kernel<T, EPI_STORE, TL, ALoad>), grid, block, 0, st, p, al); break;
    case EPI_RELU: cfm_launch((gemm_kernel<T, EPI_RELU, TL, ALoad>), grid, block, 0, st, p, al); break;
    case EPI_SWISH: cfm_launch((gemm_kernel<T, EPI_SWISH, TL, ALoad>), grid, block, 0, st, p, al); break;
    case EPI_RESID: cfm_launch((gemm_kernel<T, EPI_RESID, TL, ALoad>), grid, block, 0, st, p, al); break;
    case EPI_SCALE_F32: cfm_launch((gemm_kernel<T, EPI_SCALE_F32, TL, ALoad>), grid, block, 0, st, p, al); break;
    case EPI_GLU_MASK: cfm_launch((gemm_kernel<T, EPI_GLU_MASK, TL, ALoad>), grid, block, 0, st, p, al); break;
    case EPI_QKV: cfm_launch((gemm_kernel<T, EPI_QKV, TL, ALoad>), grid, block, 0, st, p, al); break;
    case EPI_SWISH_BWD: cfm_launch((gemm_kernel<T, EPI_SWISH_BWD, TL, ALoad>), grid, block, 0, st, p, al); break;
    case EPI_SWISH_Z: cfm_launch((gemm_kernel<T, EPI_SWISH_Z, TL, ALoad>), grid, block, 0, st, p, al); break;
    default: break;
  }
}

struct DenseArgs {
  const char* A; long lda_b; int M; long kbytes; const char* zero;
  int utt_tp = 0, utt_rows = 0, utt_nt = 1, utt_out = 0, utt_halo = 0;
  template <class AL> void fill(AL& al) const {
    al.A = A; al.lda_b = lda_b; al.M = M; al.kbytes = kbytes; al.zero = zero; al.utt_tp = utt_tp; al.utt_rows = utt_rows;
    al.utt_nt = utt_nt; al.utt_out = utt_out; al.utt_halo = utt_halo;
  }
};
struct ConvArgs {
  const char* X1; int T1, F1, T2, F2; long tapb; int M; const char* zero;
  template <class AL> void fill(AL& al) const {
    al.X1 = X1; al.T1 = T1; al.F1 = F1; al.T2 = T2; al.F2 = F2; al.tapb = tapb; al.M = M; al.zero = zero;
    al.tap_steps = (tapb % 128 == 0 && tapb * 9 < (1L << 31)) ? (int)(tapb / 128) : 0;
  }
};

int packed_width(const GemmEpi& epi, int N) {
  return (epi.mode == EPI_GLU_MASK || epi.mode == EPI_GLU_DW) ? 64 * ((N + 31) / 32) : N;
}

int g_tile_override = [] { const char* s = getenv("CFM_GEMM_TILE"); return s ? atoi(s) : -1; }();
// the 8-phase kernel for the conv2 implicit GEMM (CFM_GEMM8=0: the tiled kernel, A/B)
int g_gemm8 = [] { const char* s = getenv("CFM_GEMM8"); return s ? atoi(s) : 1; }();
// ... and for the dense Swish GEMMs (CFM_GEMM8_DENSE=1; off by default: at K = 512 the 8-phase loop
// measured no faster than the tiled 256x256 kernel in the forward (4.957-4.966 against 4.963-4.968 ms)
// and 0.07 ms slower per training step - these GEMMs lose their time in the fill and the epilogue)
int g_gemm8_dense = [] { const char* s = getenv("CFM_GEMM8_DENSE"); return s ? atoi(s) : 0; }();
// 8-phase loop: one operand half (2 glds) per phase instead of both halves every other phase (A/B)
int g_g8_spread = [] { const char* s = getenv("CFM_G8_SPREAD"); return s ? atoi(s) : 0; }();
// write-through (sc1) output stores: CFM_GEMM_WT=0 turns them off (A/B measurements)
int g_gemm_wt = [] { const char* s = getenv("CFM_GEMM_WT"); return s ? atoi(s) : 1; }();
// K-group tiles (KG > 1, >= 3 ring stages): the whole next K-step's fragments are read while the
// current one multiplies (gemm_kernel's read-ahead loop); CFM_GEMM_AHEAD=0 keeps the substep pipeline
int g_gemm_ahead = [] { const char* s = getenv("CFM_GEMM_AHEAD"); return s ? atoi(s) : 0; }();

// Tile ids (CFM_GEMM_TILE / set_gemm_tile_override; other ids run tile 0):
//   0 128x128 NS2 | 1 256x128 NS3 | 5 64x128 NS2          (128-byte K-steps, several blocks / CU)
//   11 256x256 NS2 (128-byte K-steps) | 12 128x128 2 K-groups NS3 | 14 128x128 2 K-groups NS4 |
//   16 64x128 2 K-groups NS3
// Measured and no longer instantiated (DESIGN §4 dead ends; their Tile aliases stay as the record):
//   7 / 8 / 9 / 10 (64-byte K-step 1-block tiles), 13 / 15 / 17 (K-group variants), 18 (256-byte K-steps,
//   2-deep ring: loop 17.0 -> 14.2 us without loads but 29.8 -> 36.4 us per ffn_down in the forward,
//   profiles/r04e_tile18_ab.txt: one 64 KiB stage in flight does not cover the forward's load latency).
// The fp32 parity mode instantiates 0, 1 and 5 only (other ids fall back to 0).
// Automatic choice (tools/gemm_bench.py, MI355X, bf16): the implicit conv and the wide FFN-up
// GEMM run best on 256x256 (tile 11); the N = 512 layer GEMMs on 64x128 at 3 blocks / CU (tile 5);
// the GLU GEMM on 256x128.
// CFM_TILES="epi:tile[@minM[k minK]],..." overrides the bf16 choice per epilogue id (A/B
// measurements; epilogue ids as in cfm_kernels.h, 9 = the implicit conv); the first entry whose
// minM <= M and minK <= K wins.
struct TileRule { int epi, tile, min_m, min_k; };
const std::vector<TileRule>& tile_rules() {
  static const std::vector<TileRule> rules = [] {
    std::vector<TileRule> r;
    const char* s = getenv("CFM_TILES");
    while (s && *s) {
      TileRule t{-1, -1, 0, 0};
      if (sscanf(s, "%d:%d@%dk%d", &t.epi, &t.tile, &t.min_m, &t.min_k) >= 2) r.push_back(t);
      s = strchr(s, ',');
      if (s) ++s;
    }
    return r;
  }();
  return rules;
}

int pick_tile(int dtype, int M, int Nw, int epi, bool conv, int K = 0) {
  if (g_tile_override >= 0) return g_tile_override;
  if (dtype == DT_BF16) {
    for (const TileRule& t : tile_rules())
      if (t.epi == (conv ? 9 : epi) && M >= t.min_m && K >= t.min_k) return t.tile;
  }
  if (dtype == DT_BF16) {
    // forward A/B on MI355X (tools/fwd_ab.sh, single stream, B=32 T=1000): the N = 512 residual
    // GEMMs (FFN linear2, linear_out, pointwise_conv2) run best on 128x128 tiles (one per CU, the
    // fewest L2 -> LDS bytes per CU) with two K-groups of 4 waves (two waves per SIMD) and a
    // 4-deep ring: 5.48 -> 5.20 ms per forward against 256x128 / 128x128 one-group tiles (the 4-deep
    // ring another 1.4 % over 3-deep)
    if (conv) return 11;
    if (Nw >= 2048 && M >= 4096) return 11;
    if (epi == EPI_GLU_MASK) return 1;
    // K-grouped tiles split each 128-byte K-step's substeps {0,1} | {2,3} between the groups, so
    // the small-M residual tile must be K-grouped the same way: an utterance's output is then
    // bitwise independent of the batch it runs in (tests/test_gpu_encoder.py)
    // K = 512 (linear_out, pointwise_conv2): the 64x128 K-group tile, two blocks per CU, so one block's
    // store-bound epilogue overlaps the other's main loop (forward 4.716-4.751 -> 4.677-4.719 ms,
    // profiles/r04r_resid_tile_ab.txt); K = 2048 (FFN linear2) keeps 128x128 (fewer bytes per CU)
    if (epi == EPI_RESID) return (M >= 4096 && (K == 0 || K >= 1024)) ? 14 : 16;
    // the subsampling Linear (K = C * F2 = 10240, N = d): 64 tiles of 256x256 fill a quarter of the
    // chip; 128x128 in two K-groups (same K order as the small-M 64x128 K-group tile): 154 -> ~100 us
    if (epi == EPI_SCALE_F32 && K >= 4096) return M >= 4096 ? 12 : 16;
    // very tall fp32-output GEMMs (the RNN-T joint's B*T'*(U+1) x (V+1) logits, 646k rows at config 4):
    // 256x256 tiles, bench.py --mode joint 9.68 against 10.21 ms for 128x128 K-group tiles
    // (profiles/r04e_joint_tile_ab.txt)
    if (epi == EPI_SCALE_F32 && M >= 65536 && Nw >= 512) return 11;
    // the training step's fp32-output dgrads (M = B*T' rows, N = d): 128x128 K-group tiles
    // (tools/train_ab.sh: 38.5-38.8 against 38.9-39.2 ms per step for the 64x128 tile)
    if (epi == EPI_SCALE_F32 && M >= 4096) return 14;
    return 5;
  }
  if (conv || (long)M * Nw >= (long)32 << 20) return 1;
  if (epi == EPI_GLU_MASK) return 0;
  return 5;
}

template <typename T, template <int> class AL, class ALArgs>
void dispatch(int tile, GemmParams p, const ALArgs& args, hipStream_t st) {
  const int Nw = packed_width(p.epi, p.N);
  auto setup = [&](int bm, int bn) {
    p.Mtiles = (p.M + bm - 1) / bm;
    p.Ntiles = (Nw + bn - 1) / bn;
  };
  constexpr bool kDeep = std::is_same<T, bf16_t>::value;
  switch (tile) {
    case 1: setup(256, 128); launch_epi<T, T256x128, AL>(p, args, st); return;
    case 5: setup(64, 128); launch_epi<T, T64x128s2, AL>(p, args, st); return;
    default: break;
  }
  if constexpr (kDeep) {
    switch (tile) {
      case 11: setup(256, 256); launch_epi<T, T256x256w, AL>(p, args, st); return;
      case 12: setup(128, 128); launch_epi<T, T128x128k, AL>(p, args, st); return;
      case 14: setup(128, 128); launch_epi<T, T128x128k4, AL>(p, args, st); return;
      case 16: setup(64, 128); launch_epi<T, T64x128k, AL>(p, args, st); return;
      default: break;
    }
  }
  setup(128, 128);
  launch_epi<T, T128x128, AL>(p, args, st);
}

GemmParams make_params(int es, int M, const void* Wp, int Kpad, int N, const GemmEpi& epi) {
  GemmParams p;
  p.W = (const char*)Wp;
  p.ldw_b = (long)Kpad * es;
  p.kb = (int)((long)Kpad * es);
  p.probe = 0;
  p.ahead = g_gemm_ahead;
  p.split_x = 0;
  p.Mtiles = p.Ntiles = 0;
  p.M = M;
  p.N = N;
  p.epi = epi;
  // buffer-descriptor offsets are 31-bit: write-through only for outputs below 2 GiB
  const long out_bytes = std::max((long)M * epi.ldc * es, (long)M * epi.ldx * 4);
  p.epi.wt = (g_gemm_wt && out_bytes < 0x7fffffffL) ? 1 : 0;
  return p;
}

}  // namespace

// CFM_GEMM_PROBE: the cfm_bench_gemm probe bits on every dense / GLU GEMM of a run (timing studies only:
// the outputs are garbage)
int g_gemm_probe = [] { const char* s = getenv("CFM_GEMM_PROBE"); return s ? atoi(s) : 0; }();
int set_gemm_probe(int probe) {
  const int prev = g_gemm_probe;
  g_gemm_probe = probe;
  return prev;
}

int set_gemm_tile_override(int tile) {
  const int prev = g_tile_override;
  g_tile_override = tile;
  return prev;
}

void gemm(int dtype, const void* A, long lda, int M, int K, const void* Wp, int Kpad, int N, const GemmEpi& epi,
          const void* zero_page, hipStream_t st) {
  if (M <= 0) return;
  const int es = dtype_size(dtype);
  GemmParams p = make_params(es, M, Wp, Kpad, N, epi);
  DenseArgs a{(const char*)A, lda * es, M, (long)K * es, (const char*)zero_page};
  p.probe = g_gemm_probe;
  // the 8-phase 256x256 kernel for the un-folded Swish GEMMs (FFN linear1 + Swish; training's z / u
  // pair): bf16, 128-byte K-tiles, N on the 256 granule of the packed weight, no LayerNorm fold
  if (dtype == DT_BF16 && g_gemm8_dense && g_tile_override < 0 && !epi.ln_in && epi.utt_tp <= 0 &&
      (epi.mode == EPI_SWISH || epi.mode == EPI_SWISH_Z) && p.kb % 128 == 0 && M >= 4096 && N >= 1024 &&
      (lda * es) % 16 == 0) {
    ALoadDense<2> al;
    a.fill(al);
    p.Mtiles = (M + 255) / 256;
    p.Ntiles = (N + 255) / 256;
    if (epi.mode == EPI_SWISH && g_g8_spread)
      cfm_launch((gemm8_kernel<EPI_SWISH, ALoadDense<2>, true>), dim3(p.Mtiles * p.Ntiles), dim3(512), 0, st, p, al);
    else if (epi.mode == EPI_SWISH)
      cfm_launch((gemm8_kernel<EPI_SWISH, ALoadDense<2>>), dim3(p.Mtiles * p.Ntiles), dim3(512), 0, st, p, al);
    else if (g_g8_spread)
      cfm_launch((gemm8_kernel<EPI_SWISH_Z, ALoadDense<2>, true>), dim3(p.Mtiles * p.Ntiles), dim3(512), 0, st, p, al);
    else
      cfm_launch((gemm8_kernel<EPI_SWISH_Z, ALoadDense<2>>), dim3(p.Mtiles * p.Ntiles), dim3(512), 0, st, p, al);
    return;
  }
  int tile = pick_tile(dtype, M, packed_width(epi, N), epi.mode, false, K);
  if (dtype == DT_F32) dispatch<float, ALoadDense>(tile, p, a, st);
  else dispatch<bf16_t, ALoadDense>(tile, p, a, st);
}

// As gemm(), with the packed operand's row stride `ldw` (elements) decoupled from its K extent:
// the main loop covers round_up(K, 128 bytes) only.  Used for split-K slices of wide operands.
void gemm_ldw(int dtype, const void* A, long lda, int M, int K, const void* Wp, long ldw, int N, const GemmEpi& epi,
              const void* zero_page, hipStream_t st) {
  if (M <= 0 || K <= 0) return;
  const int es = dtype_size(dtype);
  GemmParams p = make_params(es, M, Wp, (int)ldw, N, epi);
  p.kb = round_up_int(K * es, GEMM_BK_BYTES);
  DenseArgs a{(const char*)A, lda * es, M, (long)K * es, (const char*)zero_page};
  int tile = pick_tile(dtype, M, packed_width(epi, N), epi.mode, false);
  if (dtype == DT_F32) dispatch<float, ALoadDense>(tile, p, a, st);
  else dispatch<bf16_t, ALoadDense>(tile, p, a, st);
}

// Split-K GEMM: slice s (of S) contracts K elements [s*kchunk, min((s+1)*kchunk, K)) and writes its
// fp32 partial to epi.X + s * split_x (EPI_SCALE_F32 only).  kchunk % (128 bytes / es) == 0; the
// packed operand rows (ldw) must hold S * kchunk elements (zero beyond K).  One launch, grid.y = S.
void gemm_splitk(int dtype, const void* A, long lda, int M, int K, const void* Wp, long ldw, int N, int S, int kchunk,
                 const GemmEpi& epi, long split_x, const void* zero_page, hipStream_t st) {
  if (M <= 0 || K <= 0) return;
  const int es = dtype_size(dtype);
  GemmParams p = make_params(es, M, Wp, (int)ldw, N, epi);
  p.kb = kchunk * es;
  p.split_x = split_x;
  if ((long)S * split_x * 4 + (long)M * epi.ldx * 4 >= 0x7fffffffL) p.epi.wt = 0;
  g_splits = S;
  DenseArgs a{(const char*)A, lda * es, M, (long)K * es, (const char*)zero_page};
  int tile = pick_tile(dtype, M, packed_width(epi, N), epi.mode, false);
  if (dtype == DT_F32) dispatch<float, ALoadDense>(tile, p, a, st);
  else dispatch<bf16_t, ALoadDense>(tile, p, a, st);
  g_splits = 1;
}

// T' <= 256: one 256-row tile per utterance; up to 3 tiles of 226 output frames with 15 frames of
// context either side (the depthwise conv's reach) up to T' = 678
constexpr int kGluTileOut = 256 - 2 * 15;
bool gemm_glu_dw_supported(int dtype, int Tp, int d, int K) {
  return dtype == DT_BF16 && Tp >= 1 && Tp <= 3 * kGluTileOut && d % 64 == 0 && K == 31;
}

void gemm_glu_dw(int dtype, const void* A, long lda, int B, int Tp, int K, const void* Wp, int Kpad, int N,
                 const GemmEpi& epi, const void* zero_page, hipStream_t st) {
  if (B <= 0) return;
  if (!gemm_glu_dw_supported(dtype, Tp, N, 31) || epi.mode != EPI_GLU_DW || epi.utt_tp != Tp)
    fail(CFM_ERR_UNSUPPORTED, "gemm_glu_dw: bf16, T' <= 678, d % 64 == 0 only");
  using TL = T256x128;
  const int nt = Tp <= TL::BM ? 1 : (Tp + kGluTileOut - 1) / kGluTileOut;
  GemmParams p = make_params(2, B * nt * TL::BM, Wp, Kpad, N, epi);
  p.probe = g_gemm_probe;
  p.epi.utt_M = B * Tp;
  p.epi.utt_nt = nt;
  p.epi.utt_out = nt == 1 ? TL::BM : kGluTileOut;
  p.epi.utt_halo = nt == 1 ? 0 : 15;
  DenseArgs a{(const char*)A, lda * 2, B * Tp, (long)K * 2, (const char*)zero_page};
  a.utt_tp = Tp;
  a.utt_rows = TL::BM;
  a.utt_nt = p.epi.utt_nt;
  a.utt_out = p.epi.utt_out;
  a.utt_halo = p.epi.utt_halo;
  p.Mtiles = B * nt;
  p.Ntiles = packed_width(epi, N) / TL::BN;
  ALoadDense<TL::GA> al;
  a.fill(al);
  cfm_launch((gemm_kernel<bf16_t, EPI_GLU_DW, TL, ALoadDense<TL::GA>>), dim3(p.Mtiles * p.Ntiles), dim3(TL::NT), 0, st,
             p, al);
}

void gemm_conv(int dtype, const ConvGeom& g, int B, const void* Wp, int Kpad, int N, const GemmEpi& epi,
               const void* zero_page, hipStream_t st) {
  const int M = B * g.T2 * g.F2;
  if (M <= 0) return;
  const int es = dtype_size(dtype);
  GemmParams p = make_params(es, M, Wp, Kpad, N, epi);
  ConvArgs a{(const char*)g.X1, g.T1, g.F1, g.T2, g.F2, (long)g.C * es, M, (const char*)zero_page};
  if (dtype == DT_BF16 && g_gemm8 && g_tile_override < 0 && p.kb % 128 == 0 && ((long)g.C * es) % 64 == 0) {
    // the 8-phase 256x256 kernel (long K): N granule 256 (packed weights are zero-padded to it)
    ALoadConv<2> al;
    a.fill(al);
    p.Mtiles = (M + 255) / 256;
    p.Ntiles = (N + 255) / 256;
    if (g_g8_spread)
      cfm_launch((gemm8_kernel<EPI_RELU, ALoadConv<2>, true>), dim3(p.Mtiles * p.Ntiles), dim3(512), 0, st, p, al);
    else
      cfm_launch((gemm8_kernel<EPI_RELU, ALoadConv<2>>), dim3(p.Mtiles * p.Ntiles), dim3(512), 0, st, p, al);
    return;
  }
  int tile = pick_tile(dtype, M, N, epi.mode, true);
  if (dtype == DT_F32) dispatch<float, ALoadConv>(tile, p, a, st);
  else dispatch<bf16_t, ALoadConv>(tile, p, a, st);
}

bool conv12_supported(int dtype, int C) {
  return dtype == DT_BF16 && C >= 256 && C <= C12_MAXC && C % 64 == 0 && g_tile_override < 0;
}

size_t conv12_patch_bytes(int B, int T1, int F1, int C) {
  return (size_t)B * (T1 + 2) * (F1 + 2) * 32 + 256 + (size_t)C * 32;
}

// conv.0 + ReLU + conv.2 + ReLU: x (B, F, T) fp32 -> X2 (B, T2, F2, C) bf16; `patch` is scratch of
// conv12_patch_bytes(B, T1, F1, C) bytes
void conv12_fused(const float* x_bft, int B, int F, int T, int T1, int F1, int T2, int F2, const float* w1,
                  const float* b1, int C, const void* Wp, int Kpad, const float* b2, void* X2, void* patch,
                  const void* zero_page, hipStream_t st) {
  const int M = B * T2 * F2;
  if (M <= 0) return;
  if (!conv12_supported(DT_BF16, C)) fail(CFM_ERR_UNSUPPORTED, "conv12_fused: 16-bit, C % 64 == 0, 256 <= C <= 512");
  if ((long)Kpad != 9L * C) fail(CFM_ERR_UNSUPPORTED, "conv12_fused: conv.2 weight K must be 9 * C");
  const long npix = (long)B * (T1 + 2) * (F1 + 2);
  uint4* w1h = (uint4*)((char*)patch + ((npix * 32 + 255) / 256) * 256);
  cfm_launch(conv12_patch_kernel, dim3((unsigned)std::min<long>((npix + 255) / 256, 4096)), dim3(256), 0, st, x_bft, B,
             F, T, T1, F1, (uint4*)patch, w1, b1, C, w1h);
  GemmEpi e;
  std::memset(&e, 0, sizeof(e));
  e.mode = EPI_RELU;
  e.bias = b2;
  e.alpha = 1.0f;
  e.C = X2;
  e.ldc = C;
  GemmParams p = make_params(2, M, Wp, Kpad, C, e);
  p.probe = g_gemm_probe & (8 | 16 | 32 | 64 | 128 | 256);   // timing studies only (wrong results), see conv12_kernel
  p.Mtiles = (M + 255) / 256;
  p.Ntiles = (C + 255) / 256;
  Conv12Args a{(const uint4*)patch, w1h, (const char*)zero_page, T1, F1, T2, F2, C};
  // two phases of 32 MFMAs per K-tile (conv12b_kernel, default) or four of 16 (conv12_kernel, CFM_CONV12B=0):
  // the same products in the same K order (bitwise equal), 886 -> 738 us per forward (profiles/r05u_conv12b_ab.txt)
  const char* tp_env = getenv("CFM_CONV12B");   // read per call (tests switch it between forwards)
  const bool two_phase = !tp_env || atoi(tp_env) != 0;
  if (two_phase && p.probe) cfm_launch(conv12b_kernel<true>, dim3(p.Mtiles * p.Ntiles), dim3(512), 0, st, p, a);
  else if (two_phase) cfm_launch(conv12b_kernel<false>, dim3(p.Mtiles * p.Ntiles), dim3(512), 0, st, p, a);
  else cfm_launch(conv12_kernel, dim3(p.Mtiles * p.Ntiles), dim3(512), 0, st, p, a);
}

bool gemm_tconv_supported(int dtype, int C) { return C > 0 && ((long)C * dtype_size(dtype)) % 128 == 0; }

// One stride phase of conv2's input gradient (the transposed conv, cfm_kernels.h TConvGeom): rows
// of the phase-major dY1 image in the compute type (EPI_STORE).  bf16 runs on the 256x256 tile (CFM_TCONV_TILE=14: 128x128 K-group).
void gemm_tconv(int dtype, const TConvGeom& g, const void* Wp, int Kpad, int N, const GemmEpi& epi,
                const void* zero_page, hipStream_t st) {
  const int M = g.B * g.nI * g.nJ;
  if (M <= 0) return;
  if (!gemm_tconv_supported(dtype, g.C) || epi.mode != EPI_STORE)
    fail(CFM_ERR_UNSUPPORTED, "gemm_tconv: C * element size % 128 == 0 and a plain store only");
  const int es = dtype_size(dtype);
  GemmParams p = make_params(es, M, Wp, Kpad, N, epi);
  auto fill = [&](auto& al) {
    al.dY = (const char*)g.dY2; al.ldb = g.ld * es; al.T2 = g.T2; al.F2 = g.F2; al.nI = g.nI; al.nJ = g.nJ;
    al.pt = g.pt; al.pf = g.pf; al.tapb = (long)g.C * es; al.M = M; al.zero = (const char*)zero_page;
  };
  auto go = [&](auto kern, auto& al, int bm, int bn, int nt) {
    fill(al);
    p.Mtiles = (M + bm - 1) / bm;
    p.Ntiles = (N + bn - 1) / bn;
    cfm_launch(kern, dim3(p.Mtiles * p.Ntiles), dim3(nt), 0, st, p, al);
  };
  static const int tile = [] { const char* e = getenv("CFM_TCONV_TILE"); return e ? atoi(e) : 11; }();
  if (dtype == DT_BF16 && tile == 14) {
    using TL = T128x128k4;
    ALoadTConv<TL::GA> al;
    go(gemm_kernel<bf16_t, EPI_STORE, TL, ALoadTConv<TL::GA>>, al, TL::BM, TL::BN, TL::NT);
  } else if (dtype == DT_BF16) {
    using TL = T256x256w;
    ALoadTConv<TL::GA> al;
    go(gemm_kernel<bf16_t, EPI_STORE, TL, ALoadTConv<TL::GA>>, al, TL::BM, TL::BN, TL::NT);
  } else {
    using TL = T128x128;
    ALoadTConv<TL::GA> al;
    go(gemm_kernel<float, EPI_STORE, TL, ALoadTConv<TL::GA>>, al, TL::BM, TL::BN, TL::NT);
  }
}

}  // namespace cfm
