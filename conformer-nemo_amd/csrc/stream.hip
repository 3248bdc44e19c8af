// Buffered-streaming front end (SURVEY §8 row a-ext5): shift-and-append of the per-stream feature
// buffer plus its per-feature normalisation, the numpy work FeatureFrameBufferer /
// BatchedFeatureFrameBufferer do on the host before each encoder call (streaming_utils.py:516-549,
// 757-806).  Contract in include/cfm_stream.h.
//
// One wave per (stream, feature) row: the row's previous buffer and its k new chunks are staged
// once in LDS (time-contiguous, coalesced loads), each of the k windows is reduced with fp64
// accumulation and wave shuffles (mean, then the centred second moment, as np.mean / np.std with
// ddof=0 define them), and the normalised windows are written time-contiguous, i.e. straight into
// the encoder's (B, F, T) input layout.  HBM-bound: F*Tbuf*4 B read + (k+1)*F*Tbuf*4 B written
// per stream.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <string>

#include "../../include/cfm_stream.h"
#include "cfm_abi.h"

using namespace cfm;

namespace {

constexpr int kMaxSrc = 8192;  // Tbuf + k * n_frame, floats per row staged in LDS

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__global__ __launch_bounds__(256) void frame_buffer_kernel(float* __restrict__ buffer, const float* __restrict__ frames,
                                                           const uint8_t* __restrict__ active, int S, int F, int Tbuf,
                                                           int n, int k, float eps, float* __restrict__ out) {
  extern __shared__ float lds[];
  const int waves = blockDim.x >> 6;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int L = Tbuf + k * n;
  const long row = (long)blockIdx.x * waves + wave;  // s * F + f
  if (row >= (long)S * F) return;                   // wave-uniform; no block barrier below
  const int s = (int)(row / F), f = (int)(row % F);
  float* src = lds + (long)wave * L;
  float* prev = buffer + row * Tbuf;
  if (active != nullptr && active[s] == 0) {
    // reference: buffer[idx] *= 0 and feature_buffer[idx] *= 0 -> mean 0, std 0 -> (0 - 0) / eps = 0
    float* o = out + ((long)s * k * F + f) * Tbuf;
    for (int t = lane; t < Tbuf; t += 64) { prev[t] = 0.0f; o[t] = 0.0f; }
    return;
  }
  const float* fr = frames + row * ((long)k * n);
  for (int t = lane; t < Tbuf; t += 64) src[t] = prev[t];
  for (int t = lane; t < k * n; t += 64) src[Tbuf + t] = fr[t];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  const double inv_n = 1.0 / (double)Tbuf;
  for (int i = 0; i < k; ++i) {
    const float* w = src + (i + 1) * n;
    double sum = 0.0;
    for (int t = lane; t < Tbuf; t += 64) sum += (double)w[t];
    const double mean = wave_sum_d(sum) * inv_n;
    double sq = 0.0;
    for (int t = lane; t < Tbuf; t += 64) {
      const double d = (double)w[t] - mean;
      sq += d * d;
    }
    const float mean_f = (float)mean;
    const float den = (float)sqrt(wave_sum_d(sq) * inv_n) + eps;  // float32 (std + CONSTANT), as numpy
    float* o = out + (((long)s * k + i) * F + f) * Tbuf;
    for (int t = lane; t < Tbuf; t += 64) o[t] = (w[t] - mean_f) / den;
  }
  for (int t = lane; t < Tbuf; t += 64) prev[t] = src[k * n + t];
}

}  // namespace

extern "C" cfm_status cfm_frame_buffer_step(float* buffer, const float* frames, const uint8_t* active, int S, int F,
                                            int Tbuf, int n_frame, int k, float eps, float* out, void* stream) {
  return guarded([&] {
    if (S < 0 || F < 1 || Tbuf < 1 || n_frame < 1 || n_frame > Tbuf || k < 1)
      fail(CFM_ERR_INVALID_ARG, "cfm_frame_buffer_step: need F >= 1, 1 <= n_frame <= Tbuf, k >= 1");
    if ((long)Tbuf + (long)k * n_frame > kMaxSrc)
      fail(CFM_ERR_UNSUPPORTED, "cfm_frame_buffer_step: Tbuf + k*n_frame exceeds " + std::to_string(kMaxSrc));
    if (active != nullptr && k != 1)
      fail(CFM_ERR_INVALID_ARG, "cfm_frame_buffer_step: per-stream `active` flags need k == 1 (batched bufferer)");
    if (S == 0) return;
    if (buffer == nullptr || out == nullptr || frames == nullptr)
      fail(CFM_ERR_INVALID_ARG, "cfm_frame_buffer_step: null buffer / frames / out");
    const int L = Tbuf + k * n_frame;
    const int waves = std::max(1, std::min(4, 16384 / L));  // <= 64 KB of LDS per block
    const long rows = (long)S * F;
    const unsigned blocks = (unsigned)((rows + waves - 1) / waves);
    hipLaunchKernelGGL(frame_buffer_kernel, dim3(blocks), dim3(64 * waves), (size_t)waves * L * sizeof(float),
                       (hipStream_t)stream, buffer, frames, active, S, F, Tbuf, n_frame, k, eps, out);
    HIP_OK(hipGetLastError());
  });
}
