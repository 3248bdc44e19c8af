// Weight-gradient GEMM on row-major operands (training, bf16): out[n][k] = sum_r A[r][n] * B'[r][k].
//
// The layer gradients dW = dy^T . x reduce over the B*T' frame rows, and both dy and x are stored
// frame-major ([rows][features], features contiguous).  The MFMA operands want 8 consecutive
// reduction rows per lane, i.e. a column of those images: each K-step stages 32 frame rows of A and
// of B into LDS exactly as they lie in HBM (16-byte chunks, XOR-swizzled 256-byte rows) and the
// fragments are read with ds_read_b64_tr_b16, gfx950's transposing LDS read (4 rows x 16 columns
// per 16-lane group, delivered column-major).  No transposed copy of any activation is made.
//
// B' extends B: column K is all ones when `ones` (the bias gradient sum_r A[r][n] comes out as
// column K), columns beyond are zero; bfn = 1 recomputes B' = dropout(swish(B)) while staging (the
// FFN hidden from its pre-activation tape, mask index r * ldb + k as the forward epilogue).
// Split-K over frame rows: split s writes its partial tile at out + s * split_stride.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "cfm_common.h"
#include "cfm_kernels.h"

namespace cfm {
namespace {

typedef short v4s __attribute__((ext_vector_type(4)));

constexpr int TB = 128;   // output tile (n rows x k columns)
constexpr int TK = 32;    // frame rows per K-step

// byte offset of 16-byte chunk `ch` (0..15) of image row `row` (256-byte rows)
__device__ __forceinline__ int img_off(int row, int ch) {
  return 256 * row + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}

// 32x32x16 operand fragment of columns cb .. cb+31, frame rows kb .. kb+15 of an image
__device__ __forceinline__ uint4 tr_frag(const char* img, int cb, int kb, int lane) {
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  const int c0 = (cb + 16 * (g & 1)) >> 3;
  const int r0 = kb + 8 * (g >> 1);
  const v4s a = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) v4s*)(img + img_off(r0 + q, c0 + (p >> 1)) + 8 * (p & 1)));
  const v4s b = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) v4s*)(img + img_off(r0 + 4 + q, c0 + (p >> 1)) + 8 * (p & 1)));
  const uint2 ua = __builtin_bit_cast(uint2, a), ub = __builtin_bit_cast(uint2, b);
  return make_uint4(ua.x, ua.y, ub.x, ub.y);
}

// 1.0 in the 16-bit compute type (bf16, or IEEE fp16 in the CFM_HALF_F16 build)
#ifdef CFM_HALF_F16
constexpr uint32_t kOne16 = 0x3c00u;
#else
constexpr uint32_t kOne16 = 0x3f80u;
#endif
template <int BFN>
__global__ __launch_bounds__(256) void wgrad_tn_kernel(const bf16_t* __restrict__ A, long lda, int N,
                                                       const bf16_t* __restrict__ B, long ldb, int K, int ones,
                                                       Drop bdr, long rows, long chunk, float* __restrict__ out,
                                                       long ldo, int Kout, long split_stride) {
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * TK * 256];   // [buf][A|B][32 rows][256 B]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int n0 = blockIdx.y * TB, k0 = blockIdx.x * TB;
  const long r_beg = (long)blockIdx.z * chunk;
  const long r_end = min(rows, r_beg + chunk);
  const int nsteps = (int)((r_end - r_beg + TK - 1) / TK);

  // staging: thread tid moves chunks tid and tid + 256 of each 32 x 16-chunk operand tile
  uint4 ra[2], rb[2];
  auto load = [&](long r0) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int c = tid + 256 * j, r = c >> 4, ch = c & 15;
      const long rr = r0 + r;
      const bool rok = rr < r_end;
      const int na = n0 + ch * 8;
      ra[j] = (rok && na < N) ? *(const uint4*)(A + rr * lda + na) : make_uint4(0, 0, 0, 0);
      const int kb = k0 + ch * 8;
      if (rok && kb < K) {
        uint4 v = *(const uint4*)(B + rr * ldb + kb);
        if (BFN == 1) {
          float f[8];
          Vec16<bf16_t>::to_f32(v, f);
#pragma unroll
          for (int e = 0; e < 8; ++e) f[e] = swishf(f[e]) * drop_mul(bdr, (uint64_t)rr * (uint64_t)ldb + (uint64_t)(kb + e));
          v = Vec16<bf16_t>::from_f32(f);
        }
        rb[j] = v;
      } else {
        rb[j] = make_uint4((rok && ones && kb == K) ? kOne16 : 0u, 0, 0, 0);   // 16-bit 1.0 in column K
      }
    }
  };
  auto store = [&](int buf) {
    char* ia = smem + buf * (2 * TK * 256);
    char* ib = ia + TK * 256;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int c = tid + 256 * j, r = c >> 4, ch = c & 15;
      *(uint4*)(ia + img_off(r, ch)) = ra[j];
      *(uint4*)(ib + img_off(r, ch)) = rb[j];
    }
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};

  if (nsteps > 0) {
    load(r_beg);
    store(0);
  }
  __syncthreads();
  for (int s = 0; s < nsteps; ++s) {
    const bool more = s + 1 < nsteps;
    if (more) load(r_beg + (long)(s + 1) * TK);
    const char* ia = smem + (s & 1) * (2 * TK * 256);
    const char* ib = ia + TK * 256;
#pragma unroll
    for (int ks = 0; ks < TK; ks += 16) {
      uint4 fa[2], fb[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) fa[i] = tr_frag(ia, wm * 64 + i * 32, ks, lane);
#pragma unroll
      for (int j = 0; j < 2; ++j) fb[j] = tr_frag(ib, wn * 64 + j * 32, ks, lane);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) mfma_slab<bf16_t>(acc[i][j], fa[i], fb[j]);
    }
    if (more) store((s + 1) & 1);
    __syncthreads();
  }
  float* o = out + (long)blockIdx.z * split_stride;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = k0 + wn * 64 + j * 32 + (lane & 31);
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = n0 + wm * 64 + i * 32 + acc_row(e, lane);
        if (row < N && col < Kout) o[(long)row * ldo + col] = acc[i][j][e];
      }
    }
}

// ---- LDS-DMA variant (bfn = 0): NST-stage ring filled by global_load_lds_dwordx4, counted waits ----
__device__ uint4 g_zero16 = {0u, 0u, 0u, 0u};
__device__ uint4 g_one16 = {kOne16, 0u, 0u, 0u};   // 16-bit 1.0 then zeros: the bias column's chunk

__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_dst) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(lds_dst) : "memory");
}
template <int N> __device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// at most `ahead` stages of G loads each still in flight
template <int G, int MAXA> __device__ __forceinline__ void wait_ahead(int ahead) {
  if constexpr (MAXA <= 0) {
    wait_vm<0>();
  } else {
    if (ahead >= MAXA) wait_vm<G * MAXA>();
    else wait_ahead<G, MAXA - 1>(ahead);
  }
}
__device__ __forceinline__ void bar() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

#ifndef CFM_TN_NST
#define CFM_TN_NST 4
#endif
// ring stages (prefetch distance NST - 1): 3 x 16 KB, so three blocks (12 waves) share a CU's LDS; same-box
// training A/B (tools/train_lib_ab.sh): 31.49-31.61 ms/step at 3 stages against 31.70-31.77 at 4, 2 and 5
// stages slower than 4
constexpr int NST = CFM_TN_NST;
constexpr int STAGE = 2 * TK * 256;       // A and B images of one K-step (16 KB)

// General form (both weight gradients and the attention backward's batched products):
//   C[z][m][n] (fp32, ld ldc) = alpha * sum_{r < rows_z} A[z][r][m] * B'[z][r][n]
// with z = blockIdx.z = z1 * Z2 + z2 placing A at A + z1*az1 + z2*az2 (likewise B, C) and rows_z = K,
// or min(K, Ktot - z2*K) when Ktot > 0 (split-K slices of one reduction).  Columns m < M of A and
// n < N of B are real (reads past them only feed discarded outputs); B' column N is all ones when
// `ones`.  Output columns < Nout are written.
struct TnArgs {
  const bf16_t* A; long lda, az1, az2;
  const bf16_t* B; long ldb, bz1, bz2;
  float* C; long ldc, cz1, cz2;
  int M, N, Nout, K, Z2, Ktot, ones;
  float alpha;
  // CONV (conv.2's weight gradient): B is the implicit im2col of the conv.2 input X1 [b][T1][F1][C]
  // (= p.B): frame row r = (b, t2, f2) of the T2 x F2 output grid, column tap * C + c reads
  // X1[b][2 t2 - 1 + tap / 3][2 f2 - 1 + tap % 3][c] (zero outside the image); C % 128 == 0
  int cT1, cF1, cT2, cF2, cC;
};

// Output tile (128*MI) x (128*NI) on 4*MI*NI waves of 64 x 64; a stage holds MI A and NI B column
// images of 32 frame rows x 128 columns (8 KB each, the 128x128 image layout), so every wave reads
// its fragments exactly as in the 128x128 kernel.  Larger tiles move fewer L2 -> LDS bytes per MFMA.
// Bias (p.ones): the block whose column tile is (row tile % column tiles) also sums its A fragments
// (frame rows of dy for its columns) in VALU beside the MFMAs (waves of the first wave column) and
// writes sum_r A[r][m] at output column p.N - no appended ones column, so no extra column tile.
template <int MI, int NI, bool CONV = false>
__global__ __launch_bounds__(256 * MI * NI) void tn_glds_kernel(TnArgs p) {
  constexpr int TM = TB * MI, TN = TB * NI, NW = 4 * MI * NI, WN = 2 * NI;
  constexpr int STG = (MI + NI) * TK * 256;          // one stage: MI A images, NI B images
  constexpr int G = (MI + NI) * 8 / NW;              // 1 KB glds per wave per stage
  static_assert(G * NW == (MI + NI) * 8, "stage split");
  __shared__ __attribute__((aligned(16))) char smem[NST * STG];
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w / WN, wn = w % WN;
  const int m0 = blockIdx.y * TM, c0 = blockIdx.x * TN;
  const int z = blockIdx.z, z1 = z / p.Z2, z2 = z - z1 * p.Z2;
  const bf16_t* A = p.A + z1 * p.az1 + z2 * p.az2;
  const bf16_t* B = p.B + z1 * p.bz1 + z2 * p.bz2;
  const long rows = p.Ktot > 0 ? min((long)p.K, (long)p.Ktot - (long)z2 * p.K) : (long)p.K;
  const int nsteps = rows > 0 ? (int)((rows + TK - 1) / TK) : 0;
  const uint32_t sb = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)smem;
  const bool bias = p.ones && (int)blockIdx.x == (int)(blockIdx.y % gridDim.x) && wn == 0;
  // stage s -> slot s % NST: glds j of wave w moves 1 KB row group (w*G + j) % 8 (4 rows) of image
  // (w*G + j) / 8; lane l fills physical chunk l % 16 of row 4*rg + l / 16, i.e. loads the logical
  // chunk that the XOR swizzle puts there (LDS-DMA writes are lane-linear).  The per-lane source of
  // each glds is set up once and advanced by 32 rows per stage (stages are issued in order), so a
  // stage costs an add, a row check and the DMA per glds.
  const char* gp[G];
  long gstep[G];
  int grow[G];
  bool gok[G];
  // CONV: this lane's output pixel (b, t2, f2) for its row of the next stage, advanced by TK rows per
  // stage (F2 >= 16: at most two wraps of f2), and its tap's pixel offset (kt, kf) and channel base
  int cb[G], ct2[G], cf2[G], ckt[G], ckf[G], ccc[G];
  const void* zp = (const void*)&g_zero16;
#pragma unroll
  for (int j = 0; j < G; ++j) {
    const int gi = w * G + j, im = gi >> 3, rg = gi & 7;
    const int row = rg * 4 + (lane >> 4), pc = lane & 15;
    const int ch = pc ^ (((row & 3) << 2) | ((row >> 2) & 3));
    grow[j] = row;
    cb[j] = ct2[j] = cf2[j] = ckt[j] = ckf[j] = ccc[j] = 0;
    if (im < MI) {
      const int na = m0 + im * TB + ch * 8;
      gok[j] = na < p.M;
      gp[j] = (const char*)(A + (long)row * p.lda + na);
      gstep[j] = (long)TK * p.lda * 2;
    } else {
      const int kb = c0 + (im - MI) * TB + ch * 8;
      gok[j] = kb < p.N;
      gp[j] = (const char*)(B + (long)row * p.ldb + kb);
      gstep[j] = (long)TK * p.ldb * 2;
      if constexpr (CONV) {
        const int tap = kb / p.cC;
        ckt[j] = tap / 3;
        ckf[j] = tap - 3 * ckt[j];
        ccc[j] = kb - tap * p.cC;
        const int r = z2 * p.K + row, grid2 = p.cT2 * p.cF2;   // global frame row of stage 0
        cb[j] = r / grid2;
        const int rem = r - cb[j] * grid2;
        ct2[j] = rem / p.cF2;
        cf2[j] = rem - ct2[j] * p.cF2;
      }
    }
  }
  auto issue = [&](int s) {
    const uint32_t base = sb + (uint32_t)((s % NST) * STG);
    const long r0 = (long)s * TK;
#pragma unroll
    for (int j = 0; j < G; ++j) {
      const int gi = w * G + j, im = gi >> 3, rg = gi & 7;
      const void* src = (gok[j] && r0 + grow[j] < rows) ? (const void*)gp[j] : zp;
      if constexpr (CONV) {
        if (im >= MI) {
          const int t1 = 2 * ct2[j] - 1 + ckt[j], f1 = 2 * cf2[j] - 1 + ckf[j];
          const bool in = t1 >= 0 && t1 < p.cT1 && f1 >= 0 && f1 < p.cF1;
          src = (gok[j] && in && r0 + grow[j] < rows)
                    ? (const void*)(p.B + (((long)cb[j] * p.cT1 + t1) * p.cF1 + f1) * p.cC + ccc[j])
                    : zp;
          cf2[j] += TK;
          while (cf2[j] >= p.cF2) { cf2[j] -= p.cF2; ++ct2[j]; }
          while (ct2[j] >= p.cT2) { ct2[j] -= p.cT2; ++cb[j]; }
        }
      }
      glds16(src, base + im * (TK * 256) + rg * 1024);
      gp[j] += gstep[j];
    }
  };
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};
  float bsum[2] = {0.0f, 0.0f};
  const int ai = wm >> 1, acol = (wm & 1) * 64, bi = wn >> 1, bcol = (wn & 1) * 64;
  constexpr int D = NST - 1;
  for (int s = 0; s < D && s < nsteps; ++s) issue(s);
  for (int s = 0; s < nsteps; ++s) {
    wait_ahead<G, D - 1>(min(D, nsteps - s) - 1);   // this wave's loads of stage s have landed
    bar();                                           // everyone's have; slot (s-1) % NST is free
    if (s + D < nsteps) issue(s + D);
    const char* ia = smem + (s % NST) * STG + ai * (TK * 256);
    const char* ib = smem + (s % NST) * STG + (MI + bi) * (TK * 256);
    // every substep's fragments are read up front (two register sets; the barrier above orders them),
    // so the second substep's reads land while the first substep's MFMAs run: read, wait, multiply per
    // substep left each wave's MFMAs waiting on its own transposing reads
    constexpr int NKS = TK / 16;
    uint4 fa[NKS][2], fb[NKS][2];
#pragma unroll
    for (int q = 0; q < NKS; ++q) {
#pragma unroll
      for (int i = 0; i < 2; ++i) fa[q][i] = tr_frag(ia, acol + i * 32, 16 * q, lane);
#pragma unroll
      for (int j = 0; j < 2; ++j) fb[q][j] = tr_frag(ib, bcol + j * 32, 16 * q, lane);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int q = 0; q < NKS; ++q) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) mfma_slab<bf16_t>(acc[i][j], fa[q][i], fb[q][j]);
      if (bias) {   // lane l holds 8 frame rows of column (l & 31) of fragment i
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const uint32_t u[4] = {fa[q][i].x, fa[q][i].y, fa[q][i].z, fa[q][i].w};
#pragma unroll
          for (int e = 0; e < 4; ++e)
            bsum[i] += bf2f((bf16_t)(u[e] & 0xffffu)) + bf2f((bf16_t)(u[e] >> 16));
        }
      }
    }
  }
  float* o = p.C + z1 * p.cz1 + z2 * p.cz2;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = c0 + bi * TB + bcol + j * 32 + (lane & 31);
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = m0 + ai * TB + acol + i * 32 + acc_row(e, lane);
        if (row < p.M && col < p.Nout) o[(long)row * p.ldc + col] = p.alpha * acc[i][j][e];
      }
    }
  if (bias) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const float t = bsum[i] + __shfl_xor(bsum[i], 32);
      const int row = m0 + ai * TB + acol + i * 32 + lane;
      if (lane < 32 && row < p.M) o[(long)row * p.ldc + p.N] = p.alpha * t;
    }
  }
}

// weight-gradient tile (CFM_TN_TILE = MI*10 + NI: 11, 21, 12, 22); the batched attention products
// stay on 128x128
int tn_tile() {
  static const int t = [] {
    const char* e = getenv("CFM_TN_TILE");
    const int v = e ? atoi(e) : 11;
    return (v == 11 || v == 21 || v == 12 || v == 22) ? v : 11;
  }();
  return t;
}

}  // namespace

// Batched TN product for attn_bwd.hip (see TnArgs); false when the operands do not qualify
// (bf16, 16-byte aligned bases, strides multiples of 8 elements).
bool bgemm_tn(const void* A, long lda, long az1, long az2, const void* B, long ldb, long bz1, long bz2, float* C,
              long ldc, long cz1, long cz2, int M, int N, int K, int Z, int Z2, int Ktot, float alpha, hipStream_t st) {
  auto al = [](const void* q) { return ((uintptr_t)q & 15) == 0; };
  if (!al(A) || !al(B) || lda % 8 || ldb % 8 || az1 % 8 || az2 % 8 || bz1 % 8 || bz2 % 8 || N % 8) return false;
  TnArgs p{};
  p.A = (const bf16_t*)A; p.lda = lda; p.az1 = az1; p.az2 = az2;
  p.B = (const bf16_t*)B; p.ldb = ldb; p.bz1 = bz1; p.bz2 = bz2;
  p.C = C; p.ldc = ldc; p.cz1 = cz1; p.cz2 = cz2;
  p.M = M; p.N = N; p.Nout = N; p.K = K; p.Z2 = Z2; p.Ktot = Ktot; p.ones = 0; p.alpha = alpha;
  const dim3 grid((unsigned)((N + TB - 1) / TB), (unsigned)((M + TB - 1) / TB), (unsigned)Z), block(256);
  cfm_launch((tn_glds_kernel<1, 1>), grid, block, 0, st, p);
  return true;
}

bool wgrad_tn_supported(int dtype, int N, int K, long lda, long ldb) {
  return dtype == DT_BF16 && N % 8 == 0 && K % 8 == 0 && lda % 8 == 0 && ldb % 8 == 0;
}

int wgrad_tn_tiles(int N, int K, bool ones, int bfn) {
  if (bfn == 0) {
    const int t = tn_tile(), tm = TB * (t / 10), tn = TB * (t % 10);
    return ((N + tm - 1) / tm) * ((K + tn - 1) / tn);
  }
  const int Kb = ones ? K + 4 : K;
  return ((N + TB - 1) / TB) * ((Kb + TB - 1) / TB);
}

int wgrad_tn_blocks(int bfn) { return (bfn == 0 && tn_tile() != 11) ? 256 : 512; }

void wgrad_tn(const void* A, long lda, int N, const void* B, long ldb, int K, bool ones, int bfn, Drop bdr, long rows,
              int S, long chunk, float* out, long ldo, int Kout, long split_stride, hipStream_t st) {
  if (N <= 0 || Kout <= 0) return;
  const dim3 grid((unsigned)((Kout + TB - 1) / TB), (unsigned)((N + TB - 1) / TB), (unsigned)S), block(256);
  if (bfn == 0) {
    // bias (ones): written by the kernel at column K of the ldo-wide output, not as a ones column
    TnArgs p{};
    p.A = (const bf16_t*)A; p.lda = lda; p.az2 = chunk * lda;
    p.B = (const bf16_t*)B; p.ldb = ldb; p.bz2 = chunk * ldb;
    p.C = out; p.ldc = ldo; p.cz2 = split_stride;
    p.M = N; p.N = K; p.Nout = std::min(K, Kout); p.K = (int)chunk; p.Z2 = S; p.Ktot = (int)rows; p.ones = ones ? 1 : 0;
    p.alpha = 1.0f;
    const int t = tn_tile(), mi = t / 10, ni = t % 10;
    const dim3 g2((unsigned)((K + TB * ni - 1) / (TB * ni)), (unsigned)((N + TB * mi - 1) / (TB * mi)), (unsigned)S);
    switch (t) {
      case 21: cfm_launch((tn_glds_kernel<2, 1>), g2, dim3(512), 0, st, p); break;
      case 12: cfm_launch((tn_glds_kernel<1, 2>), g2, dim3(512), 0, st, p); break;
      case 22: cfm_launch((tn_glds_kernel<2, 2>), g2, dim3(1024), 0, st, p); break;
      default: cfm_launch((tn_glds_kernel<1, 1>), g2, dim3(256), 0, st, p); break;
    }
    return;
  }
  if (bfn == 1)
    cfm_launch(wgrad_tn_kernel<1>, grid, block, 0, st, (const bf16_t*)A, lda, N, (const bf16_t*)B, ldb, K,
               ones ? 1 : 0, bdr, rows, chunk, out, ldo, Kout, split_stride);
  else
    cfm_launch(wgrad_tn_kernel<0>, grid, block, 0, st, (const bf16_t*)A, lda, N, (const bf16_t*)B, ldb, K,
               ones ? 1 : 0, bdr, rows, chunk, out, ldo, Kout, split_stride);
}

// conv.2's weight gradient straight from the frame-major dY2 (rows x C, lda) and the conv.2 input X1
// ([B][T1][F1][C], compute type): out[s][n][tap * C + c] (ld ldo, split stride split_stride) partial sums
// over frame-row chunks of `chunk` rows (S = ceil(rows / chunk) splits), the bias sums at column 9C when
// `ones`.  256x256 tiles (one block per CU, 16 waves): the per-CU L2 -> LDS stream is the bound of this
// long-K product, and the larger tile halves its bytes per MFMA.  No im2col image is written.
bool wgrad_tn_conv_supported(int dtype, int C, long lda) { return dtype == DT_BF16 && C % 256 == 0 && lda % 8 == 0; }
void wgrad_tn_conv(const void* dy, long lda, const void* x1, int B, int T1, int F1, int T2, int F2, int C, bool ones,
                   long rows, int S, long chunk, float* out, long ldo, long split_stride, hipStream_t st) {
  (void)B;
  TnArgs p{};
  p.A = (const bf16_t*)dy; p.lda = lda; p.az2 = chunk * lda;
  p.B = (const bf16_t*)x1; p.ldb = 9L * C; p.bz2 = 0;
  p.C = out; p.ldc = ldo; p.cz2 = split_stride;
  p.M = C; p.N = 9 * C; p.Nout = 9 * C; p.K = (int)chunk; p.Z2 = S; p.Ktot = (int)rows; p.ones = ones ? 1 : 0;
  p.alpha = 1.0f;
  p.cT1 = T1; p.cF1 = F1; p.cT2 = T2; p.cF2 = F2; p.cC = C;
  const dim3 grid((unsigned)((9 * C + 255) / 256), (unsigned)((C + 255) / 256), (unsigned)S);
  cfm_launch((tn_glds_kernel<2, 2, true>), grid, dim3(1024), 0, st, p);
}

}  // namespace cfm
