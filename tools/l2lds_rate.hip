// L2 -> LDS delivered rate per CU against the bytes a CU keeps in flight.
//
// One workgroup per CU streams `per_block` bytes of a source buffer into an LDS ring of D stages of S bytes
// with global_load_lds_dwordx4 (the GEMM kernels' staging path), keeping D-1 stages in flight: a counted
// s_waitcnt vmcnt retires the oldest stage, an s_barrier (like the GEMM main loops) before its slot is
// refilled.  No compute: the rate is the staging path's own ceiling at that depth.
//   source "l2":   every workgroup of an XCD re-reads the same 2 MiB window (L2-resident after first touch)
//   source "hbm":  every workgroup streams its own region of a 2 GiB buffer (HBM / Infinity Cache)
// Prints one line per (S, D): KiB in flight, us per launch, GB/s per CU, TB/s chip-wide.
//   hipcc --offload-arch=gfx950 -O3 -o tools/l2lds_rate tools/l2lds_rate.hip && tools/l2lds_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__device__ __forceinline__ void glds16(const void* src, uint32_t lds) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(src), "s"(lds) : "memory");
}
template <int N> __device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

// G = glds per thread per stage, D = ring depth; the wait keeps (D-1)*G loads of this wave in flight
template <int NT, int G, int D>
__global__ __launch_bounds__(NT) void stream_kernel(const char* __restrict__ src, long window, long per_block,
                                                    int barrier, float* sink) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int SB = G * NT * 16;   // stage bytes
  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const uint32_t base = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)smem;
  const char* b = src + (window > 0 ? ((long)(blockIdx.x & 7) * window) : (long)blockIdx.x * per_block);
  const long wrap = window > 0 ? window : per_block;
  const int nst = (int)(per_block / SB);
  auto issue = [&](int s) {
    const long off = ((long)s * SB) % wrap;
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const int chunk = g * (NT / 64) + wave;   // 1 KiB wave-instruction pieces
      glds16(b + off + chunk * 1024 + lane * 16, __builtin_amdgcn_readfirstlane(base + (s % D) * SB + chunk * 1024));
    }
  };
  for (int s = 0; s < D - 1 && s < nst; ++s) issue(s);
  for (int s = 0; s < nst; ++s) {
    wait_vm<(D - 2) * G>();   // stage s landed (the D-2 younger stages may still fly)
    if (barrier) __builtin_amdgcn_s_barrier();
    if (s + D - 1 < nst) issue(s + D - 1);   // refill the slot stage s-1 used
  }
  wait_vm<0>();
  if (tid == 0 && sink) sink[blockIdx.x] = (float)smem[lane];
}

template <int NT, int G, int D>
void run(const char* src, long window, long per_block, int blocks, int barrier, const char* label) {
  constexpr int SB = G * NT * 16;
  const size_t lds = (size_t)SB * D;
  if (lds > 160 * 1024) return;
  auto k = stream_kernel<NT, G, D>;
  CK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(k, dim3(blocks), dim3(NT), lds, 0, src, window, per_block, barrier, nullptr);
  const int it = 20;
  CK(hipEventRecord(e0, 0));
  for (int i = 0; i < it; ++i) hipLaunchKernelGGL(k, dim3(blocks), dim3(NT), lds, 0, src, window, per_block, barrier, nullptr);
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double us = 1e3 * ms / it;
  const double gbs = per_block / (us * 1e-6) / 1e9;
  printf("%-4s waves %2d stage %3d KiB depth %d in-flight %4d KiB barrier %d: %8.2f us  %6.1f GB/s per CU  %6.2f TB/s chip\n",
         label, NT / 64, SB / 1024, D, SB * (D - 1) / 1024, barrier, us, gbs, gbs * blocks / 1e3);
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
}

template <int NT, int G>
void sweep(const char* src, long window, long per_block, int blocks, int barrier, const char* label) {
  run<NT, G, 2>(src, window, per_block, blocks, barrier, label);
  run<NT, G, 3>(src, window, per_block, blocks, barrier, label);
  run<NT, G, 4>(src, window, per_block, blocks, barrier, label);
  run<NT, G, 5>(src, window, per_block, blocks, barrier, label);
  run<NT, G, 6>(src, window, per_block, blocks, barrier, label);
  run<NT, G, 8>(src, window, per_block, blocks, barrier, label);
  run<NT, G, 10>(src, window, per_block, blocks, barrier, label);
}

int main() {
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  const long per_block = 1L << 20;              // 1 MiB per CU: ffn_down's 128x128 tile at K = 2048
  const long big = (long)ncu * per_block * 2;   // HBM source: distinct regions
  char* src = nullptr;
  CK(hipMalloc(&src, big));
  CK(hipMemset(src, 1, big));
  const long window = 2L << 20;                 // L2 source: a 2 MiB window per XCD
  printf("CUs %d, %ld KiB per workgroup\n", ncu, per_block >> 10);
  for (int barrier = 1; barrier >= 0; --barrier) {
    sweep<256, 2>(src, window, per_block, ncu, barrier, "l2");    // 8 KiB stages, 4 waves
    sweep<256, 4>(src, window, per_block, ncu, barrier, "l2");    // 16 KiB stages
    sweep<512, 2>(src, window, per_block, ncu, barrier, "l2");    // 16 KiB stages, 8 waves
    sweep<512, 4>(src, window, per_block, ncu, barrier, "l2");    // 32 KiB stages, 8 waves
  }
  sweep<512, 2>(src, 0, per_block, ncu, 1, "hbm");
  sweep<512, 4>(src, 0, per_block, ncu, 1, "hbm");
  CK(hipFree(src));
  return 0;
}
