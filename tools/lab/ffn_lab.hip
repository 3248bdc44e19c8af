// Round-5 GEMM lab for the FFN pair (M = 8000: ffn_up N 2048 K 512 + Swish, ffn_down N 512 K 2048 + residual).
// Standalone: hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/lab/ffn_lab.hip -o tools/lab/ffn_lab -ldl
// Times lab kernel variants against the library's own GEMM (cfm_bench_gemm through dlopen), interleaved in
// one process, and checks every variant against a naive fp32 reference kernel.
#include <dlfcn.h>
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../conformer-nemo_amd/csrc/cfm_common.h"

using namespace cfm;

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));    \
      exit(2);                                                                             \
    }                                                                                      \
  } while (0)

struct LP {
  const char* A; long lda_b;     // bf16 rows (bytes per row)
  const char* W; long ldw_b;     // packed weight [Npad][K] bf16
  int M, N, kb;                  // kb = K bytes (multiple of BK)
  const float* bias;
  bf16_t* C; long ldc;           // bf16 output (EPI 0 / 2)
  float* X; long ldx;            // fp32 residual (EPI 3)
  float alpha;
  const char* zero;
  int Mtiles, Ntiles;
  unsigned long long* stamps;   // per block: 8 x (memtime), 2 x memrealtime (null: off)
  int probe;                    // 1: no main-loop loads, 2: no epilogue
};
CFM_DEV void stamp(const LP& p, int i) {
  if (p.stamps && threadIdx.x == 0) {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    p.stamps[blockIdx.x * 10 + i] = __builtin_amdgcn_s_memtime();
  }
}
CFM_DEV void rstamp(const LP& p, int i) {
  if (p.stamps && threadIdx.x == 0) p.stamps[blockIdx.x * 10 + 8 + i] = __builtin_amdgcn_s_memrealtime();
}

enum { L_STORE = 0, L_SWISH = 2, L_RESID = 3 };

template <int N> CFM_DEV void waitv() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
// s_waitcnt vmcnt(n) for a runtime n in [0, 15] (larger values clamp to 15: stricter, still correct)
CFM_DEV void waitv_rt(int n) {
  switch (n) {
    case 0: waitv<0>(); break;   case 1: waitv<1>(); break;   case 2: waitv<2>(); break;
    case 3: waitv<3>(); break;   case 4: waitv<4>(); break;   case 5: waitv<5>(); break;
    case 6: waitv<6>(); break;   case 7: waitv<7>(); break;   case 8: waitv<8>(); break;
    case 9: waitv<9>(); break;   case 10: waitv<10>(); break; case 11: waitv<11>(); break;
    case 12: waitv<12>(); break; case 13: waitv<13>(); break; case 14: waitv<14>(); break;
    case 15: waitv<15>(); break; case 16: waitv<16>(); break; case 17: waitv<17>(); break;
    case 18: waitv<18>(); break; case 19: waitv<19>(); break; case 20: waitv<20>(); break;
    case 21: waitv<21>(); break; case 22: waitv<22>(); break; case 23: waitv<23>(); break;
    default: waitv<24>(); break;
  }
}

// ---------------------------------------------------------------------------------------------
// G4: 4 waves (one per SIMD), 2 x 2 wave grid, wave tile (BM/2) x (BN/2) of 32x32x16 MFMAs with the
// operands swapped (weight rows as the MFMA A operand), so each lane's accumulator groups hold 4
// consecutive output COLUMNS of one row: the epilogue converts in registers and writes 8-byte runs
// into a swizzled bf16 LDS image, then stores 16-byte row chunks.
// ---------------------------------------------------------------------------------------------
template <int BM, int BN, int BK, int NS, int EPI, bool OVL = false>
struct G4 {
  static constexpr int WM = 2, WN = 2, TWM = BM / WM, TWN = BN / WN, MR = TWM / 32, NR = TWN / 32;
  static constexpr int SLOTS = BK / 16, RPI = 1024 / BK, SWDIV = 16 / SLOTS;
  static constexpr int STAGE = (BM + BN) * BK;
  static constexpr int GA = BM / RPI / 4, GB = BN / RPI / 4, G = GA + GB;
  static constexpr int KSUB = BK / 32;
  static constexpr int RING = NS * STAGE;
  static constexpr int IMG_BYTES = (EPI == L_RESID) ? BM * BN * 4 : BM * BN * 2;
  // the epilogue image sits behind the ring, or over it (after a barrier) when both do not fit
  static constexpr bool OVERLAY = OVL || RING + IMG_BYTES > 160 * 1024;
  static constexpr int IMG_OFF = OVERLAY ? 0 : RING;
  static constexpr int LDS = OVERLAY ? (RING > IMG_BYTES ? RING : IMG_BYTES) : RING + IMG_BYTES;
  static_assert(LDS <= 160 * 1024, "LDS");
  static_assert(GA >= 1 && GB >= 1 && MR >= 1 && NR >= 1, "tile");
  static CFM_DEV int swz(int row) { return (row / SWDIV) % SLOTS; }
};

template <int BM, int BN, int BK, int NS, int EPI, int OCC = 1>
__global__ __launch_bounds__(256, OCC) void g4_kernel(LP p) {
  using C = G4<BM, BN, BK, NS, EPI, (OCC > 1)>;
  __shared__ __attribute__((aligned(16))) char smem[C::LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / C::WN, wn = wave % C::WN;

  const int nblocks = p.Mtiles * p.Ntiles;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q = nblocks >> 3, r = nblocks & 7;
  const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  const int mt = wg / p.Ntiles, nt = wg - mt * p.Ntiles;
  const int m0 = mt * BM, n0 = nt * BN;
  rstamp(p, 0);
  stamp(p, 0);

  const char* asrc[C::GA];
  const char* wsrc[C::GB];
#pragma unroll
  for (int i = 0; i < C::GA; ++i) {
    const int row = (i * 4 + wave) * C::RPI + lane / C::SLOTS;
    const int m = m0 + row;
    const int so = ((lane % C::SLOTS) ^ C::swz(row)) * 16;
    asrc[i] = m < p.M ? p.A + (long)m * p.lda_b + so : nullptr;
  }
#pragma unroll
  for (int i = 0; i < C::GB; ++i) {
    const int row = (i * 4 + wave) * C::RPI + lane / C::SLOTS;
    wsrc[i] = p.W + (long)(n0 + row) * p.ldw_b + ((lane % C::SLOTS) ^ C::swz(row)) * 16;
  }
  const uint32_t sbase = lds_addr(smem);
  auto stage = [&](int kt, int slot) {
    const int kb0 = kt * BK;
    const uint32_t sb = sbase + slot * C::STAGE;
#pragma unroll
    for (int i = 0; i < C::GA; ++i)
      glds16_asm(asrc[i] ? (const void*)(asrc[i] + kb0) : (const void*)p.zero, sb + (i * 4 + wave) * 1024);
#pragma unroll
    for (int i = 0; i < C::GB; ++i) glds16_asm(wsrc[i] + kb0, sb + BM * BK + (i * 4 + wave) * 1024);
  };

  // epilogue operands, loaded before the loop
  const int h = lane >> 5, l32 = lane & 31;

  f32x16 acc[C::MR][C::NR];
#pragma unroll
  for (int i = 0; i < C::MR; ++i)
#pragma unroll
    for (int j = 0; j < C::NR; ++j) acc[i][j] = f32x16{};

  const int nk = p.kb / BK;
  const int sw = C::swz(l32);
  const int a_row0 = wm * C::TWM + l32, b_row0 = BM + wn * C::TWN + l32;
  auto read_frags = [&](int slot, int kk, uint4* af, uint4* bf) {
    const char* S = smem + slot * C::STAGE;
    const int so = ((2 * kk + h) ^ sw) * 16;
#pragma unroll
    for (int i = 0; i < C::MR; ++i) af[i] = *(const uint4*)(S + (a_row0 + i * 32) * BK + so);
#pragma unroll
    for (int j = 0; j < C::NR; ++j) bf[j] = *(const uint4*)(S + (b_row0 + j * 32) * BK + so);
  };

#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < nk) stage(s, s);
  waitv_rt(C::G * min(NS - 2, nk - 1));
  wait_lgkm0();
  raw_barrier();
  stamp(p, 1);
  uint4 fa[2][C::MR], fb[2][C::NR];
  read_frags(0, 0, fa[0], fb[0]);
  int slot = 0;
  auto kstep = [&](int kt, auto par0) {
    constexpr int P0 = decltype(par0)::value;
    if (kt + NS - 1 < nk && !(p.probe & 1)) stage(kt + NS - 1, slot == 0 ? NS - 1 : slot - 1);
    const int nslot = slot == NS - 1 ? 0 : slot + 1;
#pragma unroll
    for (int kk = 0; kk < C::KSUB; ++kk) {
      const int cur = (P0 + kk) & 1;
      const bool last = kk + 1 == C::KSUB, more = kt + 1 < nk;
      if (!last) {
        read_frags(slot, kk + 1, fa[cur ^ 1], fb[cur ^ 1]);
      } else if (more) {
        waitv_rt(C::G * min(NS - 2, nk - 2 - kt));
        __builtin_amdgcn_s_waitcnt(0xC07F);
        raw_barrier();
      }
#pragma unroll
      for (int i = 0; i < C::MR; ++i)
#pragma unroll
        for (int j = 0; j < C::NR; ++j) acc[i][j] = mfma16_32x32x16(fb[cur][j], fa[cur][i], acc[i][j]);
      if (last && more) {
        __builtin_amdgcn_sched_barrier(0);
        read_frags(nslot, 0, fa[cur ^ 1], fb[cur ^ 1]);
      }
    }
    slot = nslot;
  };
  if constexpr (C::KSUB % 2 == 0) {
    for (int kt = 0; kt < nk; ++kt) kstep(kt, std::integral_constant<int, 0>{});
  } else {
    for (int kt = 0; kt < nk; kt += 2) {
      kstep(kt, std::integral_constant<int, 0>{});
      if (kt + 1 < nk) kstep(kt + 1, std::integral_constant<int, 1>{});
    }
  }

  stamp(p, 2);
  if (p.probe & 2) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < C::MR; ++i)
#pragma unroll
      for (int j = 0; j < C::NR; ++j) t += acc[i][j][0];
    if (t == 1234.5f) p.X[threadIdx.x] = t;
    stamp(p, 4);
    rstamp(p, 1);
    return;
  }
  // ---- epilogue ----
  char* img = smem + C::IMG_OFF;
  if constexpr (C::OVERLAY) {
    wait_lgkm0();
    raw_barrier();
  }
  if constexpr (EPI == L_RESID) {
    // fp32 image [BM][BN], 16-byte slots XOR-swizzled by (row % 8)
    constexpr int RB = BN * 4, SL = BN / 4;
#pragma unroll
    for (int i = 0; i < C::MR; ++i)
#pragma unroll
      for (int j = 0; j < C::NR; ++j)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int ml = wm * C::TWM + i * 32 + l32;
          const int nl = wn * C::TWN + j * 32 + 8 * g + 4 * h;
          const float4 b = p.bias ? *(const float4*)(p.bias + n0 + nl) : make_float4(0.f, 0.f, 0.f, 0.f);
          float4 v = make_float4(acc[i][j][4 * g] + b.x, acc[i][j][4 * g + 1] + b.y, acc[i][j][4 * g + 2] + b.z,
                                 acc[i][j][4 * g + 3] + b.w);
          *(float4*)(img + ml * RB + (((nl >> 2) ^ (ml & 7)) << 4)) = v;
        }
    __syncthreads();
    stamp(p, 3);
    for (int idx = tid; idx < BM * SL; idx += 256) {
      const int rr = idx / SL, c = idx % SL;
      const int m = m0 + rr;
      const float4 a = *(const float4*)(img + rr * RB + ((c ^ (rr & 7)) << 4));
      if (m < p.M) {
        float* xp = p.X + (long)m * p.ldx + n0 + 4 * c;
        const float4 x = *(const float4*)xp;
        const float4 o = make_float4(x.x + p.alpha * a.x, x.y + p.alpha * a.y, x.z + p.alpha * a.z, x.w + p.alpha * a.w);
        store16_wt(p.X, ((long)m * p.ldx + n0 + 4 * c) * 4,
                   make_uint4(__float_as_uint(o.x), __float_as_uint(o.y), __float_as_uint(o.z), __float_as_uint(o.w)));
      }
    }
    stamp(p, 4);
    rstamp(p, 1);
    return;
  } else {
    // bf16 image [BM][BN], 16-byte slots XOR-swizzled by (row % 16)
    constexpr int RB = BN * 2, SL = BN / 8;
#pragma unroll
    for (int i = 0; i < C::MR; ++i)
#pragma unroll
      for (int j = 0; j < C::NR; ++j)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int ml = wm * C::TWM + i * 32 + l32;
          const int nl = wn * C::TWN + j * 32 + 8 * g + 4 * h;
          const float4 b = p.bias ? *(const float4*)(p.bias + n0 + nl) : make_float4(0.f, 0.f, 0.f, 0.f);
          float v0 = acc[i][j][4 * g] + b.x, v1 = acc[i][j][4 * g + 1] + b.y;
          float v2 = acc[i][j][4 * g + 2] + b.z, v3 = acc[i][j][4 * g + 3] + b.w;
          if constexpr (EPI == L_SWISH) { v0 = swishf(v0); v1 = swishf(v1); v2 = swishf(v2); v3 = swishf(v3); }
          const uint2 pk = make_uint2((uint32_t)f2bf(v0) | ((uint32_t)f2bf(v1) << 16),
                                      (uint32_t)f2bf(v2) | ((uint32_t)f2bf(v3) << 16));
          *(uint2*)(img + ml * RB + ((((nl >> 3) ^ (ml & 15)) << 4) | (8 * h))) = pk;
        }
    __syncthreads();
    stamp(p, 3);
#pragma unroll 4
    for (int idx = tid; idx < BM * SL; idx += 256) {
      const int rr = idx / SL, c = idx % SL;
      const int m = m0 + rr;
      const uint4 v = *(const uint4*)(img + rr * RB + ((c ^ (rr & 15)) << 4));
      if (m < p.M) store16_wt(p.C, ((long)m * p.ldc + n0 + 8 * c) * 2, v);
    }
  }
  stamp(p, 4);
  rstamp(p, 1);
}

// ---------------------------------------------------------------------------------------------
// Reference: one thread per output, fp32 accumulation
// ---------------------------------------------------------------------------------------------
__global__ void ref_kernel(LP p, int epi, float* out) {
  const long idx = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (idx >= (long)p.M * p.N) return;
  const int m = idx / p.N, n = idx % p.N;
  const bf16_t* a = (const bf16_t*)(p.A + (long)m * p.lda_b);
  const bf16_t* w = (const bf16_t*)(p.W + (long)n * p.ldw_b);
  float s = 0.f;
  for (int k = 0; k < p.kb / 2; ++k) s += bf2f(a[k]) * bf2f(w[k]);
  s += p.bias ? p.bias[n] : 0.f;
  if (epi == L_SWISH) s = swishf(s);
  out[idx] = s;
}

__global__ void fill_kernel(uint16_t* p, long n, uint32_t seed) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    uint32_t x = (uint32_t)i * 2654435761u ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    p[i] = f2bf(((x & 0xffffff) / 16777216.0f) * 2.0f - 1.0f);
  }
}
__global__ void fillf_kernel(float* p, long n, uint32_t seed, float scale) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    uint32_t x = (uint32_t)i * 2654435761u ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    p[i] = (((x & 0xffffff) / 16777216.0f) * 2.0f - 1.0f) * scale;
  }
}

// ---------------------------------------------------------------------------------------------
struct Variant {
  std::string name;
  void (*launch)(const LP&, hipStream_t);
  int bm, bn;
};

template <int BM, int BN, int BK, int NS, int EPI, int OCC = 1>
void launch_g4(const LP& p0, hipStream_t st) {
  LP p = p0;
  p.Mtiles = (p.M + BM - 1) / BM;
  p.Ntiles = (p.N + BN - 1) / BN;
  hipLaunchKernelGGL((g4_kernel<BM, BN, BK, NS, EPI, OCC>), dim3(p.Mtiles * p.Ntiles), dim3(256), 0, st, p);
}

typedef int (*bench_fn)(int, int, int, int, int, int, int, float*);

int main(int argc, char** argv) {
  const char* shape = argc > 1 ? argv[1] : "ffn_up";
  const int iters = argc > 2 ? atoi(argv[2]) : 20;
  const int rounds = argc > 3 ? atoi(argv[3]) : 5;
  int M = 8000, N, K, epi, libtile;
  std::vector<Variant> vs;
  if (!strcmp(shape, "ffn_up")) {
    N = 2048; K = 512; epi = L_SWISH; libtile = 11;
    vs.push_back({"g4 256x128 bk64 ns3 occ2", launch_g4<256, 128, 64, 3, L_SWISH, 2>, 256, 128});
    vs.push_back({"g4 256x128 bk64 ns2 occ2", launch_g4<256, 128, 64, 2, L_SWISH, 2>, 256, 128});
    vs.push_back({"g4 128x256 bk64 ns3 occ2", launch_g4<128, 256, 64, 3, L_SWISH, 2>, 128, 256});
    vs.push_back({"g4 128x128 bk128 ns2 occ2", launch_g4<128, 128, 128, 2, L_SWISH, 2>, 128, 128});
    vs.push_back({"g4 256x128 bk64 ns4 occ1", launch_g4<256, 128, 64, 4, L_SWISH, 1>, 256, 128});
  } else if (!strcmp(shape, "ffn_up_store")) {
    N = 2048; K = 512; epi = L_STORE; libtile = 11;
    vs.push_back({"g4 256x128 bk64 ns4", launch_g4<256, 128, 64, 4, L_STORE>, 256, 128});

  } else if (!strcmp(shape, "ffn_down")) {
    N = 512; K = 2048; epi = L_RESID; libtile = 14;
    vs.push_back({"g4 128x128 bk128 ns3 occ1", launch_g4<128, 128, 128, 3, L_RESID, 1>, 128, 128});
    vs.push_back({"g4 64x128 bk128 ns2 occ2", launch_g4<64, 128, 128, 2, L_RESID, 2>, 64, 128});
  } else {
    fprintf(stderr, "unknown shape\n");
    return 1;
  }
  const long Np = ((N + 255) / 256) * 256;
  char *A, *W, *zero;
  float *bias, *X, *X0, *ref, *Cf;
  bf16_t* Cb;
  CK(hipMalloc(&A, (size_t)M * K * 2));
  CK(hipMalloc(&W, (size_t)Np * K * 2));
  CK(hipMalloc(&zero, 4096));
  CK(hipMalloc(&bias, Np * 4));
  CK(hipMalloc(&X, (size_t)M * N * 4));
  CK(hipMalloc(&X0, (size_t)M * N * 4));
  CK(hipMalloc(&ref, (size_t)M * N * 4));
  CK(hipMalloc(&Cb, (size_t)M * N * 2));
  CK(hipMemset(zero, 0, 4096));
  hipLaunchKernelGGL(fill_kernel, dim3(1024), dim3(256), 0, 0, (uint16_t*)A, (long)M * K, 1u);
  hipLaunchKernelGGL(fill_kernel, dim3(1024), dim3(256), 0, 0, (uint16_t*)W, (long)Np * K, 2u);
  hipLaunchKernelGGL(fillf_kernel, dim3(64), dim3(256), 0, 0, bias, Np, 3u, 0.5f);
  hipLaunchKernelGGL(fillf_kernel, dim3(1024), dim3(256), 0, 0, X0, (long)M * N, 4u, 1.0f);
  LP p{};
  p.A = A; p.lda_b = (long)K * 2; p.W = W; p.ldw_b = (long)K * 2; p.M = M; p.N = N; p.kb = K * 2; p.bias = bias;
  p.C = Cb; p.ldc = N; p.X = X; p.ldx = N; p.alpha = 0.5f; p.zero = zero;
  hipLaunchKernelGGL(ref_kernel, dim3((M * (long)N + 255) / 256), dim3(256), 0, 0, p, epi, ref);
  CK(hipDeviceSynchronize());
  std::vector<float> href((size_t)M * N), hx0((size_t)M * N), hout((size_t)M * N);
  CK(hipMemcpy(href.data(), ref, href.size() * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hx0.data(), X0, hx0.size() * 4, hipMemcpyDeviceToHost));
  // correctness
  for (auto& v : vs) {
    CK(hipMemcpy(X, X0, (size_t)M * N * 4, hipMemcpyDeviceToDevice));
    CK(hipMemset(Cb, 0xff, (size_t)M * N * 2));
    v.launch(p, 0);
    CK(hipDeviceSynchronize());
    double num = 0, den = 0;
    if (epi == L_RESID) {
      CK(hipMemcpy(hout.data(), X, hout.size() * 4, hipMemcpyDeviceToHost));
      for (size_t i = 0; i < hout.size(); ++i) {
        const double e = hx0[i] + 0.5 * href[i];
        num += (hout[i] - e) * (hout[i] - e);
        den += e * e;
      }
    } else {
      std::vector<uint16_t> hb((size_t)M * N);
      CK(hipMemcpy(hb.data(), Cb, hb.size() * 2, hipMemcpyDeviceToHost));
      for (size_t i = 0; i < hb.size(); ++i) {
        const uint32_t u = (uint32_t)hb[i] << 16;
        float o;
        memcpy(&o, &u, 4);
        num += (o - href[i]) * (double)(o - href[i]);
        den += (double)href[i] * href[i];
      }
    }
    printf("check %-24s relL2 %.3e %s\n", v.name.c_str(), sqrt(num / den), sqrt(num / den) < 1e-2 ? "ok" : "FAIL");
  }
  // timing, interleaved rounds
  void* lib = dlopen("conformer-nemo_amd/conformer_amd/libcfm.so", RTLD_NOW);
  bench_fn bench = lib ? (bench_fn)dlsym(lib, "cfm_bench_gemm") : nullptr;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<std::vector<float>> t(vs.size() + 1);
  for (int r = 0; r < rounds; ++r) {
    if (bench) {
      float ms = 0;
      bench(1, libtile, epi, M, N, K, iters, &ms);
      t[vs.size()].push_back(ms * 1000);
    }
    for (size_t i = 0; i < vs.size(); ++i) {
      for (int w = 0; w < 3; ++w) vs[i].launch(p, 0);
      CK(hipEventRecord(e0, 0));
      for (int it = 0; it < iters; ++it) vs[i].launch(p, 0);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      t[i].push_back(ms * 1000 / iters);
    }
  }
  // probes and in-kernel stamps (one launch each, after a warm-up)
  unsigned long long* dst;
  CK(hipMalloc(&dst, 8192 * 10 * 8));
  for (size_t i = 0; i < vs.size(); ++i) {
    for (int probe : {0, 1, 2, 3}) {
      LP q = p;
      q.probe = probe;
      for (int w = 0; w < 3; ++w) vs[i].launch(q, 0);
      CK(hipEventRecord(e0, 0));
      for (int it = 0; it < iters; ++it) vs[i].launch(q, 0);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      q.stamps = dst;
      CK(hipMemset(dst, 0, 8192 * 10 * 8));
      vs[i].launch(q, 0);
      CK(hipDeviceSynchronize());
      const int nb = ((M + vs[i].bm - 1) / vs[i].bm) * ((N + vs[i].bn - 1) / vs[i].bn);
      std::vector<unsigned long long> hs((size_t)nb * 10);
      CK(hipMemcpy(hs.data(), dst, hs.size() * 8, hipMemcpyDeviceToHost));
      // clock: cycles / realtime ticks (100 MHz)
      unsigned long long rmin = ~0ull, rmax = 0;
      std::vector<double> d[4], clk;
      for (int b = 0; b < nb; ++b) {
        const unsigned long long* x = &hs[(size_t)b * 10];
        rmin = std::min(rmin, x[8]);
        rmax = std::max(rmax, x[9]);
        if (x[9] > x[8]) clk.push_back((double)(x[4] - x[0]) / (double)(x[9] - x[8]) * 0.1);   // GHz
        d[0].push_back(x[1] - x[0]);
        d[1].push_back(x[2] - x[1]);
        if (x[3]) { d[2].push_back(x[3] - x[2]); d[3].push_back(x[4] - x[3]); }
        else d[3].push_back(x[4] - x[2]);
      }
      auto med = [](std::vector<double> v) { if (v.empty()) return 0.0; std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
      const double ghz = med(clk);
      printf("%-24s probe %d: %7.2f us/launch | span %6.2f us, clk %.2f GHz | us: prologue %5.2f loop %5.2f epi-img %5.2f "
             "epi-store %5.2f\n", vs[i].name.c_str(), probe, ms * 1000 / iters, (rmax - rmin) * 0.01, ghz,
             med(d[0]) / ghz * 1e-3, med(d[1]) / ghz * 1e-3, med(d[2]) / ghz * 1e-3, med(d[3]) / ghz * 1e-3);
    }
  }
  const double flop = 2.0 * M * N * K;
  for (size_t i = 0; i <= vs.size(); ++i) {
    if (t[i].empty()) continue;
    std::vector<float> s = t[i];
    std::sort(s.begin(), s.end());
    const float med = s[s.size() / 2];
    printf("%-24s %s: median %7.2f us  min %7.2f us  %6.1f TF/s\n", i < vs.size() ? vs[i].name.c_str() : "library",
           shape, med, s[0], flop / med * 1e-6);
  }
  return 0;
}
