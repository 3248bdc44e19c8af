// On-device spectrogram augmentation, contract in include/cfm_augment.h.
//
// Masking is pure HBM work on the (B, F, T) fp32 spectrogram, so the kernels touch only what the
// reference overwrites: one workgroup per (utterance, rectangle) writes that rectangle with
// time-contiguous (coalesced) stores; SpecShot is one streaming pass with 16-byte vectors.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>

#include "../../include/cfm_augment.h"
#include "cfm_abi.h"

using namespace cfm;

namespace {

// Python slice bounds for a non-negative start and stop on an axis of length n.
__device__ __forceinline__ int clamp_axis(int v, int n) { return v < 0 ? 0 : (v > n ? n : v); }

__global__ __launch_bounds__(256) void mask_rects_kernel(float* __restrict__ spec, int F, int T,
                                                         const int32_t* __restrict__ rects, int n, float value) {
  const int b = blockIdx.x / n, r = blockIdx.x % n;
  const int4 q = ((const int4*)rects)[(long)b * n + r];
  const int f0 = clamp_axis(q.x, F), f1 = clamp_axis(q.y, F), t0 = clamp_axis(q.z, T), t1 = clamp_axis(q.w, T);
  const int w = t1 - t0;
  if (f1 <= f0 || w <= 0) return;
  const long cells = (long)(f1 - f0) * w;
  float* base = spec + (long)b * F * T;
  for (long i = threadIdx.x; i < cells; i += blockDim.x) {
    const int f = f0 + (int)(i / w), t = t0 + (int)(i % w);
    base[(long)f * T + t] = value;
  }
}

// splitmix64 finaliser: a counter-based generator, so any element's uniform is independent of
// the launch geometry.
__device__ __forceinline__ float hash_uniform(uint64_t seed, uint64_t i) {
  uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (float)(z >> 40) * (1.0f / 16777216.0f);   // 24 random bits -> [0, 1)
}

__global__ __launch_bounds__(256) void spec_shot_kernel(const float* __restrict__ in, float* __restrict__ out,
                                                        int64_t n, float ratio, uint64_t seed) {
  const int64_t n4 = n >> 2;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < n4; v += stride) {
    float4 x = ((const float4*)in)[v];
    const uint64_t i = (uint64_t)v * 4;
    x.x *= (1.0f - hash_uniform(seed, i + 0) > ratio) ? 1.0f : 0.0f;
    x.y *= (1.0f - hash_uniform(seed, i + 1) > ratio) ? 1.0f : 0.0f;
    x.z *= (1.0f - hash_uniform(seed, i + 2) > ratio) ? 1.0f : 0.0f;
    x.w *= (1.0f - hash_uniform(seed, i + 3) > ratio) ? 1.0f : 0.0f;
    ((float4*)out)[v] = x;
  }
  // tail (n % 4 elements), handled by the first threads of block 0
  const int64_t tail = n4 * 4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (blockIdx.x == 0 && tail < n) out[tail] = in[tail] * ((1.0f - hash_uniform(seed, (uint64_t)tail) > ratio) ? 1.0f : 0.0f);
}

}  // namespace

extern "C" cfm_status cfm_spec_mask_rects(float* spec, int B, int F, int T, const int32_t* rects, int n, float value,
                                          void* stream) {
  return guarded([&] {
    if (B < 0 || F < 0 || T < 0 || n < 0) fail(CFM_ERR_INVALID_ARG, "cfm_spec_mask_rects: negative size");
    if ((long)B * n == 0 || (long)F * T == 0) return;
    if (!spec || !rects) fail(CFM_ERR_INVALID_ARG, "cfm_spec_mask_rects: null spec / rects");
    if ((long)B * n > 0x7fffffffL) fail(CFM_ERR_UNSUPPORTED, "cfm_spec_mask_rects: too many rectangles");
    if (((uintptr_t)rects & 15) != 0) fail(CFM_ERR_INVALID_ARG, "cfm_spec_mask_rects: rects must be 16-byte aligned");
    hipLaunchKernelGGL(mask_rects_kernel, dim3((unsigned)(B * n)), dim3(256), 0, (hipStream_t)stream, spec, F, T,
                       rects, n, value);
    HIP_OK(hipGetLastError());
  });
}

extern "C" cfm_status cfm_spec_shot(const float* in, float* out, int64_t n, float mask_ratio, uint64_t seed,
                                    void* stream) {
  return guarded([&] {
    if (n < 0) fail(CFM_ERR_INVALID_ARG, "cfm_spec_shot: negative size");
    if (n == 0) return;
    if (!in || !out) fail(CFM_ERR_INVALID_ARG, "cfm_spec_shot: null in / out");
    if ((((uintptr_t)in | (uintptr_t)out) & 15) != 0) fail(CFM_ERR_INVALID_ARG, "cfm_spec_shot: 16-byte alignment");
    const int64_t n4 = std::max<int64_t>(1, n >> 2);
    const unsigned blocks = (unsigned)std::min<int64_t>((n4 + 255) / 256, 8192);
    hipLaunchKernelGGL(spec_shot_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, in, out, n, mask_ratio,
                       seed);
    HIP_OK(hipGetLastError());
  });
}
