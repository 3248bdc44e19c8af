// Round-5 lab for the weight-gradient TN product (training): C[m][n] = sum_r A[r][m] * B[r][n], frame-major
// bf16 operands, split-K over frame rows as train.hip's wgrad_rm does.  Times the library kernel
// (tn_glds_kernel<1,1>, included from wgrad_tn.hip) against lab variants in one process, interleaved, and
// checks every variant bitwise against the library kernel (same MFMA order per output element).
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I conformer-nemo_amd/csrc tools/lab/tn_lab.hip -o tools/lab/tn_lab
#include "../../conformer-nemo_amd/csrc/wgrad_tn.hip"

#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

using namespace cfm;
namespace cfm { thread_local KernelClock* g_kclock = nullptr; }

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));    \
      exit(2);                                                                             \
    }                                                                                      \
  } while (0)

namespace lab {

// V: the library loop with TKS frame rows per stage (32 or 64: 8 or 16 MFMAs per wave per barrier),
// NS stages, full K-steps without the per-glds row check (a tail step is zero-filled by the row check
// only when the split's row count is not a multiple of TKS), PROBE 1 = no loads in the main loop.
template <int TKS, int NS, int PROBE>
__global__ __launch_bounds__(256) void tn_v(TnArgs p) {
  constexpr int IMG = TKS * 256;                 // one operand image: TKS rows x 128 columns
  constexpr int STG = 2 * IMG;                   // A and B images
  constexpr int G = 2 * (TKS / 4) / 4;           // 1 KB glds per wave per stage (4 rows each)
  __shared__ __attribute__((aligned(16))) char smem[NS * STG];
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w >> 1, wn = w & 1;
  const int m0 = blockIdx.y * 128, c0 = blockIdx.x * 128;
  const int z = blockIdx.z, z1 = z / p.Z2, z2 = z - z1 * p.Z2;
  const bf16_t* A = p.A + z1 * p.az1 + z2 * p.az2;
  const bf16_t* B = p.B + z1 * p.bz1 + z2 * p.bz2;
  const long rows = p.Ktot > 0 ? min((long)p.K, (long)p.Ktot - (long)z2 * p.K) : (long)p.K;
  const int nsteps = rows > 0 ? (int)((rows + TKS - 1) / TKS) : 0;
  const uint32_t sb = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)smem;
  const char* gp[G];
  long gstep[G];
  int grow[G];
  bool gok[G];
  const void* zp = (const void*)&g_zero16;
#pragma unroll
  for (int j = 0; j < G; ++j) {
    const int gi = w * G + j, im = gi / (TKS / 4), rg = gi % (TKS / 4);
    const int row = rg * 4 + (lane >> 4), pc = lane & 15;
    const int ch = pc ^ (((row & 3) << 2) | ((row >> 2) & 3));
    grow[j] = row;
    if (im == 0) {
      const int na = m0 + ch * 8;
      gok[j] = na < p.M;
      gp[j] = (const char*)(A + (long)row * p.lda + na);
      gstep[j] = (long)TKS * p.lda * 2;
    } else {
      const int kb = c0 + ch * 8;
      gok[j] = kb < p.N;
      gp[j] = (const char*)(B + (long)row * p.ldb + kb);
      gstep[j] = (long)TKS * p.ldb * 2;
    }
  }
  auto issue = [&](int s) {
    const uint32_t base = sb + (uint32_t)((s % NS) * STG);
    const long r0 = (long)s * TKS;
    const bool full = r0 + TKS <= rows;
#pragma unroll
    for (int j = 0; j < G; ++j) {
      const int gi = w * G + j, im = gi / (TKS / 4), rg = gi % (TKS / 4);
      const void* src = (gok[j] && (full || r0 + grow[j] < rows)) ? (const void*)gp[j] : zp;
      if (PROBE != 1 || s < NS - 1) glds16(src, base + im * IMG + rg * 1024);
      gp[j] += gstep[j];
    }
  };
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};
  const int acol = wm * 64, bcol = wn * 64;
  constexpr int D = NS - 1;
  for (int s = 0; s < D && s < nsteps; ++s) issue(s);
  for (int s = 0; s < nsteps; ++s) {
    if (PROBE == 1) wait_vm<0>();
    else wait_ahead<G, D - 1>(min(D, nsteps - s) - 1);
    bar();
    if (s + D < nsteps) issue(s + D);
    const char* ia = smem + (s % NS) * STG;
    const char* ib = ia + IMG;
    constexpr int NKS = TKS / 16;
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
    for (int q = 0; q < NKS; ++q)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) mfma_slab<bf16_t>(acc[i][j], fa[q][i], fb[q][j]);
  }
  float* o = p.C + z1 * p.cz1 + z2 * p.cz2;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = c0 + bcol + j * 32 + (lane & 31);
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = m0 + acol + i * 32 + acc_row(e, lane);
        if (row < p.M && col < p.Nout) o[(long)row * p.ldc + col] = p.alpha * acc[i][j][e];
      }
    }
}

}  // namespace lab

__global__ void fill_bf16(uint16_t* p, long n, uint32_t seed) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    uint32_t x = (uint32_t)i * 2654435761u ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    const float f = ((x & 0xffffff) / 16777216.0f) * 2.0f - 1.0f;
    p[i] = (uint16_t)(__float_as_uint(f) >> 16);
  }
}

struct Var { std::string name; void (*k)(TnArgs); int tks; dim3 block; };

// the training step's split reduction (train.hip slab_sum_kernel form): out = sum_s part[s] in order
__global__ void slab_lab(const float* __restrict__ part, int S, long n, float* __restrict__ out) {
  for (long i = (blockIdx.x * 256L + threadIdx.x) * 4; i < n; i += (long)gridDim.x * 256 * 4) {
    float4 a = *(const float4*)(part + i);
    for (int s = 1; s < S; ++s) {
      const float4 b = *(const float4*)(part + (long)s * n + i);
      a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    }
    *(float4*)(out + i) = a;
  }
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 20, rounds = argc > 2 ? atoi(argv[2]) : 5;
  struct Shape { const char* name; int N, K; } shapes[] = {{"ffn_w1 2048x512", 2048, 512}, {"ffn_w2 512x2048", 512, 2048},
                                                            {"qkv 1536x512", 1536, 512}, {"out 512x512", 512, 512}};
  const long R = 8000;
  std::vector<Var> vs = {
      {"lib tn_glds<1,1>", tn_glds_kernel<1, 1>, 32, dim3(256)},
      {"v tk32 ns3", lab::tn_v<32, 3, 0>, 32, dim3(256)},
      {"v tk64 ns2", lab::tn_v<64, 2, 0>, 64, dim3(256)},
      {"v tk64 ns3", lab::tn_v<64, 3, 0>, 64, dim3(256)},
      {"v tk32 ns3 noload", lab::tn_v<32, 3, 1>, 32, dim3(256)},
      {"v tk64 ns2 noload", lab::tn_v<64, 2, 1>, 64, dim3(256)},
  };
  uint16_t *A, *B;
  float *C0, *C1;
  CK(hipMalloc(&A, R * 2048 * 2));
  CK(hipMalloc(&B, R * 2048 * 2));
  CK(hipMalloc(&C0, 16L * 2048 * 2048 * 4));
  CK(hipMalloc(&C1, 16L * 2048 * 2048 * 4));
  hipLaunchKernelGGL(fill_bf16, dim3(1024), dim3(256), 0, 0, A, R * 2048, 1u);
  hipLaunchKernelGGL(fill_bf16, dim3(1024), dim3(256), 0, 0, B, R * 2048, 2u);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  if (argc > 3 && !strcmp(argv[3], "conv")) {   // conv2 weight-gradient proxy: N 512, K 4608, 160000 frame rows
    const long RC = 160000;
    const int N = 512, K = 4608;
    uint16_t *Ac, *Bc;
    float* Cc;
    CK(hipMalloc(&Ac, RC * N * 2));
    CK(hipMalloc(&Bc, RC * K * 2));
    CK(hipMalloc(&Cc, 16L * N * K * 4));
    hipLaunchKernelGGL(fill_bf16, dim3(1024), dim3(256), 0, 0, Ac, RC * N, 5u);
    hipLaunchKernelGGL(fill_bf16, dim3(1024), dim3(256), 0, 0, Bc, RC * K, 6u);
    struct Cv { const char* name; void (*k)(TnArgs); int mi, ni, thr; } cvs[] = {
        {"tn 128x128", tn_glds_kernel<1, 1>, 1, 1, 256}, {"tn 256x128", tn_glds_kernel<2, 1>, 2, 1, 512},
        {"tn 128x256", tn_glds_kernel<1, 2>, 1, 2, 512}, {"tn 256x256", tn_glds_kernel<2, 2>, 2, 2, 1024}};
    for (const Cv& cv : cvs) {
      for (int Sreq : {1, 2, 4, 7, 8, 14}) {
        const long tiles = (long)(N / (128 * cv.mi)) * ((K + 128 * cv.ni - 1) / (128 * cv.ni));
        long chunk = ((RC + Sreq - 1) / Sreq + 31) / 32 * 32;
        const long S = (RC + chunk - 1) / chunk;
        TnArgs p{};
        p.A = (const bf16_t*)Ac; p.lda = N; p.az2 = chunk * N;
        p.B = (const bf16_t*)Bc; p.ldb = K; p.bz2 = chunk * K;
        p.ldc = K; p.cz2 = (long)N * K; p.C = Cc;
        p.M = N; p.N = K; p.Nout = K; p.K = (int)chunk; p.Z2 = (int)S; p.Ktot = (int)RC; p.alpha = 1.0f;
        const dim3 grid((unsigned)((K + 128 * cv.ni - 1) / (128 * cv.ni)), (unsigned)(N / (128 * cv.mi)), (unsigned)S);
        std::vector<float> tk;
        for (int r = 0; r < 3; ++r) {
          hipLaunchKernelGGL(cv.k, grid, dim3(cv.thr), 0, 0, p);
          CK(hipEventRecord(e0, 0));
          for (int it = 0; it < 3; ++it) hipLaunchKernelGGL(cv.k, grid, dim3(cv.thr), 0, 0, p);
          CK(hipEventRecord(e1, 0));
          CK(hipEventSynchronize(e1));
          float ms = 0;
          CK(hipEventElapsedTime(&ms, e0, e1));
          tk.push_back(ms * 1000 / 3);
        }
        std::sort(tk.begin(), tk.end());
        printf("conv2 wgrad proxy %-11s S=%2ld tiles %3ld blocks %4ld  %8.1f us  %6.1f TF/s\n", cv.name, S, tiles, tiles * S,
               tk[1], 2.0 * RC * N * K / tk[1] * 1e-6);
      }
    }
    return 0;
  }
  if (argc > 3) {   // split sweep: library kernel + the split reduction, per S
    float* out;
    CK(hipMalloc(&out, 2048L * 2048 * 4));
    for (const Shape& sh : shapes) {
      const int N = sh.N, K = sh.K;
      for (int Sreq : {1, 2, 3, 4, 6, 8, 12, 16}) {
        long chunk = ((R + Sreq - 1) / Sreq + 31) / 32 * 32;
        const long S = (R + chunk - 1) / chunk;
        TnArgs p{};
        p.A = (const bf16_t*)A; p.lda = N; p.az2 = chunk * N;
        p.B = (const bf16_t*)B; p.ldb = K; p.bz2 = chunk * K;
        p.ldc = K; p.cz2 = (long)N * K; p.C = C1;
        p.M = N; p.N = K; p.Nout = K; p.K = (int)chunk; p.Z2 = (int)S; p.Ktot = (int)R; p.alpha = 1.0f;
        const dim3 grid((unsigned)((K + 127) / 128), (unsigned)((N + 127) / 128), (unsigned)S);
        const long n = (long)N * K;
        std::vector<float> tk, ts;
        for (int r = 0; r < rounds; ++r) {
          for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((tn_glds_kernel<1, 1>), grid, dim3(256), 0, 0, p);
          CK(hipEventRecord(e0, 0));
          for (int it = 0; it < iters; ++it) hipLaunchKernelGGL((tn_glds_kernel<1, 1>), grid, dim3(256), 0, 0, p);
          CK(hipEventRecord(e1, 0));
          CK(hipEventSynchronize(e1));
          float ms = 0;
          CK(hipEventElapsedTime(&ms, e0, e1));
          tk.push_back(ms * 1000 / iters);
          if (S > 1) {
            CK(hipEventRecord(e0, 0));
            for (int it = 0; it < iters; ++it)
              hipLaunchKernelGGL(slab_lab, dim3((unsigned)std::min<long>((n / 4 + 255) / 256, 4096)), dim3(256), 0, 0, C1, (int)S, n, out);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&ms, e0, e1));
            ts.push_back(ms * 1000 / iters);
          } else {
            ts.push_back(0.f);
          }
        }
        std::sort(tk.begin(), tk.end());
        std::sort(ts.begin(), ts.end());
        printf("%-18s S=%2ld blocks %5u  tn %7.2f us  slab %6.2f us  sum %7.2f us\n", sh.name, S, grid.x * grid.y * grid.z,
               tk[tk.size() / 2], ts[ts.size() / 2], tk[tk.size() / 2] + ts[ts.size() / 2]);
      }
    }
    return 0;
  }
  for (const Shape& sh : shapes) {
    const int N = sh.N, K = sh.K;
    const long tiles = (long)((N + 127) / 128) * ((K + 127) / 128);
    long S = (512 + tiles - 1) / tiles;
    S = std::max<long>(1, std::min<long>({S, R / 64, 16L}));
    long chunk = ((R + S - 1) / S + 63) / 64 * 64;   // multiple of 64: the tk64 variants see whole steps
    S = (R + chunk - 1) / chunk;
    TnArgs p{};
    p.A = (const bf16_t*)A; p.lda = N; p.az2 = chunk * N;
    p.B = (const bf16_t*)B; p.ldb = K; p.bz2 = chunk * K;
    p.ldc = K; p.cz2 = (long)N * K;
    p.M = N; p.N = K; p.Nout = K; p.K = (int)chunk; p.Z2 = (int)S; p.Ktot = (int)R; p.ones = 0; p.alpha = 1.0f;
    const dim3 grid((unsigned)((K + 127) / 128), (unsigned)((N + 127) / 128), (unsigned)S);
    const size_t cbytes = (size_t)S * N * K * 4;
    // reference: the library kernel
    p.C = C0;
    hipLaunchKernelGGL((tn_glds_kernel<1, 1>), grid, dim3(256), 0, 0, p);
    CK(hipDeviceSynchronize());
    std::vector<float> ref(cbytes / 4), got(cbytes / 4);
    CK(hipMemcpy(ref.data(), C0, cbytes, hipMemcpyDeviceToHost));
    for (auto& v : vs) {
      if (strstr(v.name.c_str(), "noload")) continue;
      p.C = C1;
      CK(hipMemset(C1, 0xff, cbytes));
      hipLaunchKernelGGL(v.k, grid, v.block, 0, 0, p);
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(got.data(), C1, cbytes, hipMemcpyDeviceToHost));
      const bool same = memcmp(ref.data(), got.data(), cbytes) == 0;
      double num = 0, den = 0;
      for (size_t i = 0; i < ref.size(); ++i) { num += (got[i] - ref[i]) * (double)(got[i] - ref[i]); den += (double)ref[i] * ref[i]; }
      printf("check %-8s %-22s %s relL2 %.2e\n", sh.name, v.name.c_str(), same ? "bitwise" : "DIFF", sqrt(num / den));
    }
    std::vector<std::vector<float>> t(vs.size());
    for (int r = 0; r < rounds; ++r)
      for (size_t i = 0; i < vs.size(); ++i) {
        p.C = C1;
        for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(vs[i].k, grid, vs[i].block, 0, 0, p);
        CK(hipEventRecord(e0, 0));
        for (int it = 0; it < iters; ++it) hipLaunchKernelGGL(vs[i].k, grid, vs[i].block, 0, 0, p);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        t[i].push_back(ms * 1000 / iters);
      }
    const double flop = 2.0 * R * N * K;
    for (size_t i = 0; i < vs.size(); ++i) {
      std::sort(t[i].begin(), t[i].end());
      printf("%-18s S=%2ld %-22s median %7.2f us  min %7.2f  %6.1f TF/s\n", sh.name, S, vs[i].name.c_str(), t[i][t[i].size() / 2],
             t[i][0], flop / t[i][t[i].size() / 2] * 1e-6);
    }
  }
  return 0;
}
