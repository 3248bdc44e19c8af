// MFMA GEMM for every dense contraction of the encoder.
//
//   C[M, N] = A[M, K] . Wp[N, K]^T   (+ fused epilogue)
//
// Wp is a weight pre-packed at load time ([Npad][Kpad], compute type, zero padded) — the
// nn.Linear / Conv1d(k=1) layout, so both operands are read along K.  Tile 128x128, 4 waves (2x2),
// each wave 64x64 = 2x2 MFMA 32x32 tiles.  K is consumed in 128-byte steps staged into a
// double-buffered LDS image by global_load_lds_dwordx4 (16 B per lane); the XOR swizzle
// `slot ^ ((row >> 1) & 7)` is applied on the SOURCE address (the LDS image is lane-linear) and
// on the ds_read_b128 fragment read, which makes every 16-lane read group conflict-free.
// Out-of-range A rows / K bytes read a zero page, so no tail handling is needed in the main loop.
// Blocks are remapped so that each XCD owns a contiguous range of tiles (A panels stay in one L2).
#include "cfm_common.h"
#include "cfm_kernels.h"

namespace cfm {

namespace {

constexpr int BM = GEMM_BM, BN = GEMM_BN, BKB = GEMM_BK_BYTES;
constexpr int NTHREADS = 256;
constexpr int A_ROWS_PER_THREAD = BM / 32;   // glds instructions per thread for the A tile
constexpr int B_ROWS_PER_THREAD = BN / 32;
constexpr int MR = BM / 64, NR = BN / 64;    // 32x32 tiles per wave

struct ALoadDense {
  const char* A; long lda_b; int M; long kbytes; const char* zero;
  struct State { const char* row_ptr[A_ROWS_PER_THREAD]; };
  CFM_DEV void prepare(State& s, int m0, const int* rows) const {
#pragma unroll
    for (int i = 0; i < A_ROWS_PER_THREAD; ++i) {
      const int m = m0 + rows[i];
      s.row_ptr[i] = (m < M) ? A + (long)m * lda_b : nullptr;
    }
  }
  CFM_DEV const void* src(const State& s, int i, long kb) const {
    return (s.row_ptr[i] != nullptr && kb < kbytes) ? (const void*)(s.row_ptr[i] + kb) : (const void*)zero;
  }
};

// Row m = (b, t2, f2) of the implicit im2col matrix; column byte kb = (tap * C + c) * es with
// tap = 3*kt + kf; source = X1[b][2*t2 - 1 + kt][2*f2 - 1 + kf][c] (zero outside the image).
struct ALoadConv {
  const char* X1; int T1, F1, T2, F2; long tapb; int M; const char* zero;
  struct State { const char* base[A_ROWS_PER_THREAD]; uint32_t valid[A_ROWS_PER_THREAD]; };
  CFM_DEV void prepare(State& s, int m0, const int* rows) const {
#pragma unroll
    for (int i = 0; i < A_ROWS_PER_THREAD; ++i) {
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
        // pointer to (ti0, fi0) may be out of range; only dereferenced for valid taps
        base = X1 + (((long)b * T1 + ti0) * F1 + fi0) * tapb;
      }
      s.base[i] = base;
      s.valid[i] = v;
    }
  }
  CFM_DEV const void* src(const State& s, int i, long kb) const {
    int tap = (int)(kb / tapb);
    const long cb = kb - (long)tap * tapb;
    if (tap >= 9 || !((s.valid[i] >> tap) & 1u)) return zero;
    const int kt = tap / 3, kf = tap - kt * 3;
    return s.base[i] + ((long)kt * F1 + kf) * tapb + cb;
  }
};

struct GemmParams {
  const char* W; long ldw_b; int nk; int Mtiles, Ntiles; int M, N;
  GemmEpi epi;
};

template <typename T, int EPI>
CFM_DEV void epi_store(const GemmParams& p, int m, int n, float v) {
  const GemmEpi& e = p.epi;
  if (m >= p.M || n >= p.N) return;
  const float bias = e.bias ? e.bias[n] : 0.0f;
  if constexpr (EPI == EPI_STORE) {
    st_f<T>((T*)e.C + (long)m * e.ldc + n, v + bias);
  } else if constexpr (EPI == EPI_RELU) {
    st_f<T>((T*)e.C + (long)m * e.ldc + n, fmaxf(v + bias, 0.0f));
  } else if constexpr (EPI == EPI_SWISH) {
    st_f<T>((T*)e.C + (long)m * e.ldc + n, swishf(v + bias));
  } else if constexpr (EPI == EPI_RESID) {
    float* x = e.X + (long)m * e.ldx + n;
    *x = *x + (v + bias) * e.alpha;
  } else if constexpr (EPI == EPI_SCALE_F32) {
    e.X[(long)m * e.ldx + n] = (v + bias) * e.alpha;
  } else if constexpr (EPI == EPI_QKV) {
    if (n < e.qk_cols) {
      st_f<T>((T*)e.C + (long)m * e.ldc + n, v + bias);
    } else {
      const int nv = n - e.qk_cols;
      const int h = nv / e.dkp, dd = nv - h * e.dkp;
      const int b = m / e.Tp, t = m - b * e.Tp;
      st_f<T>((T*)e.Vt + (((long)b * e.H + h) * e.vt_rows + dd) * e.Tpad + t, v + bias);
    }
  }
}

template <typename T, int EPI, class ALoad>
__global__ __launch_bounds__(NTHREADS) void gemm_kernel(GemmParams p, ALoad aload) {
  __shared__ __attribute__((aligned(16))) char smem[2 * (BM + BN) * BKB];
  auto As = [&](int buf) { return smem + buf * (BM + BN) * BKB; };
  auto Bs = [&](int buf) { return smem + buf * (BM + BN) * BKB + BM * BKB; };

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  // XCD-aware bijective remap: blocks sharing an XCD (bid % 8) get a contiguous tile range.
  const int nblocks = p.Mtiles * p.Ntiles;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q = nblocks >> 3, r = nblocks & 7;
  const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  const int mt = wg / p.Ntiles, nt = wg - mt * p.Ntiles;
  const int m0 = mt * BM, n0 = nt * BN;

  // staging geometry: instruction i of this wave covers tile rows (i*4 + wave)*8 .. +7
  int rows[A_ROWS_PER_THREAD];
  int slot_off[A_ROWS_PER_THREAD];
#pragma unroll
  for (int i = 0; i < A_ROWS_PER_THREAD; ++i) {
    rows[i] = (i * 4 + wave) * 8 + (lane >> 3);
    slot_off[i] = ((lane & 7) ^ ((rows[i] >> 1) & 7)) * 16;   // logical 16-B slot for this lane
  }
  typename ALoad::State ast;
  aload.prepare(ast, m0, rows);
  const char* wrow[B_ROWS_PER_THREAD];
  int wslot[B_ROWS_PER_THREAD];
#pragma unroll
  for (int i = 0; i < B_ROWS_PER_THREAD; ++i) {
    const int rr = (i * 4 + wave) * 8 + (lane >> 3);
    wrow[i] = p.W + (long)(n0 + rr) * p.ldw_b;
    wslot[i] = ((lane & 7) ^ ((rr >> 1) & 7)) * 16;
  }

  auto stage = [&](int kt, int buf) {
    const long kb0 = (long)kt * BKB;
#pragma unroll
    for (int i = 0; i < A_ROWS_PER_THREAD; ++i)
      glds16(aload.src(ast, i, kb0 + slot_off[i]), As(buf) + (i * 4 + wave) * 1024);
#pragma unroll
    for (int i = 0; i < B_ROWS_PER_THREAD; ++i)
      glds16(wrow[i] + kb0 + wslot[i], Bs(buf) + (i * 4 + wave) * 1024);
  };

  f32x16 acc[MR][NR];
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int j = 0; j < NR; ++j) acc[i][j] = f32x16{};

  // fragment read offsets (row-dependent swizzle), per 32x32 sub-tile
  int a_off[MR], b_off[NR];
  const int hsel = lane >> 5;
#pragma unroll
  for (int i = 0; i < MR; ++i) {
    const int rr = wm * (BM / 2) + i * 32 + (lane & 31);
    a_off[i] = rr * BKB;
  }
#pragma unroll
  for (int j = 0; j < NR; ++j) {
    const int rr = wn * (BN / 2) + j * 32 + (lane & 31);
    b_off[j] = rr * BKB;
  }
  const int a_sw = ((lane & 31) >> 1) & 7;   // (row >> 1) & 7 : rows are 32-aligned + (lane & 31)

  stage(0, 0);
  __syncthreads();
  for (int kt = 0; kt < p.nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < p.nk) stage(kt + 1, buf ^ 1);
    const char* Ab = As(buf);
    const char* Bb = Bs(buf);
#pragma unroll
    for (int kk = 0; kk < BKB / 32; ++kk) {
      const int slot = ((2 * kk + hsel) ^ a_sw) * 16;
      uint4 af[MR], bfv[NR];
#pragma unroll
      for (int i = 0; i < MR; ++i) af[i] = *(const uint4*)(Ab + a_off[i] + slot);
#pragma unroll
      for (int j = 0; j < NR; ++j) bfv[j] = *(const uint4*)(Bb + b_off[j] + slot);
#pragma unroll
      for (int i = 0; i < MR; ++i)
#pragma unroll
        for (int j = 0; j < NR; ++j) mfma_slab<T>(acc[i][j], af[i], bfv[j]);
    }
    __syncthreads();
  }

  // epilogue
  const int col = lane & 31;
  if constexpr (EPI == EPI_GLU_MASK) {
    // packed columns: per 64-column group g, [0,32) = value channels 32g.., [32,64) = gates
    const GemmEpi& e = p.epi;
#pragma unroll
    for (int i = 0; i < MR; ++i) {
      const int ngrp = (n0 + wn * (BN / 2)) / 64;     // wave covers exactly one 64-col group (NR == 2)
      const int c = ngrp * 32 + col;
      const float ba = e.bias[ngrp * 64 + col], bg = e.bias[ngrp * 64 + 32 + col];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * (BM / 2) + i * 32 + acc_row(r, lane);
        if (m >= p.M || c >= p.N) continue;
        const int b = m / e.Tp, t = m - b * e.Tp;
        float v = (acc[i][0][r] + ba) * sigmoidf_(acc[i][1][r] + bg);
        if (t >= e.lens[b]) v = 0.0f;
        st_f<T>((T*)e.C + (long)m * e.ldc + c, v);
      }
    }
  } else {
#pragma unroll
    for (int i = 0; i < MR; ++i)
#pragma unroll
      for (int j = 0; j < NR; ++j) {
        const int n = n0 + wn * (BN / 2) + j * 32 + col;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + wm * (BM / 2) + i * 32 + acc_row(r, lane);
          epi_store<T, EPI>(p, m, n, acc[i][j][r]);
        }
      }
  }
}

template <typename T, class ALoad>
void launch(const GemmParams& p, const ALoad& al, hipStream_t st) {
  const dim3 grid(p.Mtiles * p.Ntiles), block(NTHREADS);
  switch (p.epi.mode) {
    case EPI_STORE: hipLaunchKernelGGL((gemm_kernel<T, EPI_STORE, ALoad>), grid, block, 0, st, p, al); break;
    case EPI_RELU: hipLaunchKernelGGL((gemm_kernel<T, EPI_RELU, ALoad>), grid, block, 0, st, p, al); break;
    case EPI_SWISH: hipLaunchKernelGGL((gemm_kernel<T, EPI_SWISH, ALoad>), grid, block, 0, st, p, al); break;
    case EPI_RESID: hipLaunchKernelGGL((gemm_kernel<T, EPI_RESID, ALoad>), grid, block, 0, st, p, al); break;
    case EPI_SCALE_F32: hipLaunchKernelGGL((gemm_kernel<T, EPI_SCALE_F32, ALoad>), grid, block, 0, st, p, al); break;
    case EPI_GLU_MASK: hipLaunchKernelGGL((gemm_kernel<T, EPI_GLU_MASK, ALoad>), grid, block, 0, st, p, al); break;
    case EPI_QKV: hipLaunchKernelGGL((gemm_kernel<T, EPI_QKV, ALoad>), grid, block, 0, st, p, al); break;
    default: break;
  }
}

GemmParams make_params(int es, int M, const void* Wp, int Kpad, int N, const GemmEpi& epi) {
  GemmParams p;
  p.W = (const char*)Wp;
  p.ldw_b = (long)Kpad * es;
  p.nk = (int)((long)Kpad * es / BKB);
  p.Mtiles = (M + BM - 1) / BM;
  p.Ntiles = (N + BN - 1) / BN;
  if (epi.mode == EPI_GLU_MASK) p.Ntiles = (2 * ((N + 31) / 32) * 32 + BN - 1) / BN;  // packed width 64*ceil(N/32)
  p.M = M;
  p.N = N;
  p.epi = epi;
  return p;
}

}  // namespace

void gemm(int dtype, const void* A, long lda, int M, int K, const void* Wp, int Kpad, int N, const GemmEpi& epi,
          const void* zero_page, hipStream_t st) {
  if (M <= 0) return;
  const int es = dtype_size(dtype);
  GemmParams p = make_params(es, M, Wp, Kpad, N, epi);
  ALoadDense al{(const char*)A, lda * es, M, (long)K * es, (const char*)zero_page};
  if (dtype == DT_F32) launch<float>(p, al, st);
  else launch<bf16_t>(p, al, st);
}

void gemm_conv(int dtype, const ConvGeom& g, int B, const void* Wp, int Kpad, int N, const GemmEpi& epi,
               const void* zero_page, hipStream_t st) {
  const int M = B * g.T2 * g.F2;
  if (M <= 0) return;
  const int es = dtype_size(dtype);
  GemmParams p = make_params(es, M, Wp, Kpad, N, epi);
  ALoadConv al{(const char*)g.X1, g.T1, g.F1, g.T2, g.F2, (long)g.C * es, M, (const char*)zero_page};
  if (dtype == DT_F32) launch<float>(p, al, st);
  else launch<bf16_t>(p, al, st);
}

}  // namespace cfm
