// Log-mel front end: FilterbankFeatures.forward (features.py:382-453) for gfx950.
// Contract in include/cfm_mel.h.
//
// mel_frames_kernel — one block = 64 STFT frames of one utterance, one wave = 16 of them:
//   * the frame's n_fft samples are gathered straight from the raw batch with the reference's
//     index algebra folded in (exact-pad reflection, optional dither, pre-emphasis as a separate
//     fp32 multiply and subtract, the center reflect pad) and multiplied by the zero-padded window;
//   * the real n_fft-point DFT is a complex n_fft/2-point radix-2 Stockham FFT in the wave's LDS
//     (even samples real, odd samples imaginary) followed by the split step to n_fft/2+1 bins;
//   * |X| (sqrt of re^2 + im^2, as torch), |X|^mag_power, the mel filterbank as a compacted
//     per-filter band of nonzero weights, log(. + guard) / log(clamp(., guard));
//   * the block's (nfilt x 64) tile is staged in LDS and written time-contiguous into the
//     (B, nfilt, T) output, 256-byte rows.
// HBM traffic: the samples once (frames overlap by n_fft - hop, served from L1/L2) and the
// features once.  FLOPs are tiny (n_fft/2 log n_fft butterflies per frame): HBM / latency bound.
//
// mel_norm_kernel — per (utterance, feature) row, one wave: normalize_batch's per-feature mean and
// unbiased std over t < seq_len (fp64 accumulation), then the t >= seq_len mask and pad_to tail.
// all_features runs one 256-thread block per utterance.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <string>
#include <vector>

#include "../../include/cfm_mel.h"
#include "cfm_abi.h"

using namespace cfm;

struct cfm_mel {
  cfm_mel_cfg c{};
  int device = 0;
  int nbins = 0, woff = 0;
  float* d_win = nullptr;   // n_fft: window zero-padded as torch.stft does (left = (n_fft - win) / 2)
  float2* d_tw = nullptr;   // n_fft/2 + 1 twiddles exp(-2 pi i k / n_fft)
  int* d_band = nullptr;    // per filter: first bin, count, offset into d_wts
  float* d_wts = nullptr;
  int nnz = 0;
  bool tables_set = false;
  size_t lds_bytes = 0;
};

namespace {

constexpr int kFramesPerBlock = 64;
constexpr int kWaves = 4;

struct MelGeom {
  long N;           // samples per utterance in the padded batch
  long Ns;          // length of the pre-STFT signal (N, or N + 2P with exact_pad)
  int P;            // exact_pad reflect amount
  int cpad;         // stft center pad (n_fft / 2) or 0
  int hop, n_fft, nfilt, nbins;
  int use_pre;
  float pre;
  int mag_mode;     // 0: |X|, 1: |X|^2, 2: powf
  float mag_power;
  int log, guard_type;
  float guard;
  float dither;
  unsigned long long seed;
};

__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
// Standard normal from a counter (seed, utterance, sample): Box-Muller on two 24-bit uniforms.
__device__ __forceinline__ float gauss(unsigned long long seed, int b, long i) {
  const unsigned long long h = mix64(seed ^ mix64(((unsigned long long)b << 40) ^ (unsigned long long)i));
  const float u1 = ((float)(h >> 40) + 0.5f) * (1.0f / 16777216.0f);
  const float u2 = (float)((h >> 16) & 0xffffff) * (1.0f / 16777216.0f);
  return sqrtf(-2.0f * logf(u1)) * cospif(2.0f * u2);
}

__device__ __forceinline__ long reflect(long i, long n) {
  if (i < 0) i = -i;
  if (i >= n) i = 2 * (n - 1) - i;
  return i;
}

// u[i]: the (exact-pad reflected, dithered) signal, i in [0, Ns)
__device__ __forceinline__ float u_at(const float* __restrict__ xb, const MelGeom& g, int b, long i) {
  float v = xb[reflect(i - g.P, g.N)];
  if (g.dither > 0.0f) v = __fadd_rn(v, __fmul_rn(g.dither, gauss(g.seed, b, i)));
  return v;
}
// s[i] = pre-emphasis of u (features.py:395-396): u[0], u[i] - preemph * u[i-1] (no FMA contraction)
__device__ __forceinline__ float s_at(const float* __restrict__ xb, const MelGeom& g, int b, long i) {
  const float v = u_at(xb, g, b, i);
  if (!g.use_pre || i == 0) return v;
  return __fsub_rn(v, __fmul_rn(g.pre, u_at(xb, g, b, i - 1)));
}

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

__global__ __launch_bounds__(256) void mel_frames_kernel(const float* __restrict__ x, int T, long Tout, MelGeom g,
                                                         const float* __restrict__ win, const float2* __restrict__ tw_g,
                                                         const int* __restrict__ band_g, const float* __restrict__ wts_g,
                                                         int nnz, const uint8_t* __restrict__ nb_mask, int nb_max_bin,
                                                         float* __restrict__ out) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int N2 = g.n_fft >> 1;
  float2* tw = (float2*)smem;                                  // N2 + 1
  int* band = (int*)(tw + N2 + 1);                             // 3 * nfilt
  float* wts = (float*)(band + 3 * g.nfilt);                   // nnz
  float* tile = wts + ((nnz + 3) & ~3);                        // nfilt * 64
  float2* wbuf = (float2*)(tile + g.nfilt * kFramesPerBlock);  // per wave: 2 * N2
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int i = threadIdx.x; i <= N2; i += blockDim.x) tw[i] = tw_g[i];
  for (int i = threadIdx.x; i < 3 * g.nfilt; i += blockDim.x) band[i] = band_g[i];
  for (int i = threadIdx.x; i < nnz; i += blockDim.x) wts[i] = wts_g[i];
  __syncthreads();

  const int b = blockIdx.y;
  const float* xb = x + (long)b * g.N;
  const bool nb = nb_mask != nullptr && nb_mask[b] != 0;
  float2* A = wbuf + (long)wave * 2 * N2;
  float2* Bf = A + N2;
  const int t_base = blockIdx.x * kFramesPerBlock;
  for (int f = 0; f < kFramesPerBlock / kWaves; ++f) {
    const int fl = wave * (kFramesPerBlock / kWaves) + f;
    const int t = t_base + fl;
    if (t >= T) break;  // wave-uniform
    // gather + window: z[n] = (s_w[2n], s_w[2n+1])
    const long base = (long)t * g.hop - g.cpad;
    for (int n = lane; n < N2; n += 64) {
      float v[2];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int j = 2 * n + e;
        const float w = win[j];
        v[e] = (w == 0.0f) ? 0.0f : __fmul_rn(s_at(xb, g, b, reflect(base + j, g.Ns)), w);
      }
      A[n] = make_float2(v[0], v[1]);
    }
    wave_lds_sync();
    // Stockham radix-2 FFT of size N2 (natural order out)
    float2* src = A;
    float2* dst = Bf;
    const int tw_scale = g.n_fft;  // exp(-2 pi i k / (2 Ns)) = tw[k * n_fft / (2 Ns)]
    for (int Ns = 1; Ns < N2; Ns <<= 1) {
      for (int jj = lane; jj < (N2 >> 1); jj += 64) {
        const int k = jj & (Ns - 1);
        const float2 w = tw[k * (tw_scale / (2 * Ns))];
        const float2 v0 = src[jj];
        const float2 a1 = src[jj + (N2 >> 1)];
        const float2 v1 = make_float2(a1.x * w.x - a1.y * w.y, a1.x * w.y + a1.y * w.x);
        const int d = ((jj - k) << 1) + k;
        dst[d] = make_float2(v0.x + v1.x, v0.y + v1.y);
        dst[d + Ns] = make_float2(v0.x - v1.x, v0.y - v1.y);
      }
      wave_lds_sync();
      float2* tmp = src;
      src = dst;
      dst = tmp;
    }
    // split step -> bins k = 0..N2 ; power into dst (free buffer) as floats
    float* P = (float*)dst;
    for (int k = lane; k <= N2; k += 64) {
      const float2 zk = src[k & (N2 - 1)];
      const float2 zc = src[(N2 - k) & (N2 - 1)];
      const float er = 0.5f * (zk.x + zc.x), ei = 0.5f * (zk.y - zc.y);     // (Z[k] + conj Z[N2-k]) / 2
      const float dr = zk.x - zc.x, di = zk.y + zc.y;                       // Z[k] - conj Z[N2-k]
      const float or_ = 0.5f * di, oi = -0.5f * dr;                          // / (2i)
      const float2 w = tw[k];
      const float re = er + (w.x * or_ - w.y * oi);
      const float im = ei + (w.x * oi + w.y * or_);
      float m = sqrtf(__fadd_rn(__fmul_rn(re, re), __fmul_rn(im, im)));     // features.py:406
      if (nb && k >= nb_max_bin) m = 0.0f;                                  // 408-411
      if (g.mag_mode == 1) m = __fmul_rn(m, m);                             // 414-415
      else if (g.mag_mode == 2) m = powf(m, g.mag_power);
      P[k] = m;
    }
    wave_lds_sync();
    for (int mf = lane; mf < g.nfilt; mf += 64) {  // features.py:418 fb @ x, then 421-427
      const int lo = band[3 * mf], cnt = band[3 * mf + 1], off = band[3 * mf + 2];
      float acc = 0.0f;
      for (int q = 0; q < cnt; ++q) acc = fmaf(wts[off + q], P[lo + q], acc);
      if (g.log) acc = g.guard_type == CFM_LOG_GUARD_ADD ? logf(__fadd_rn(acc, g.guard)) : logf(fmaxf(acc, g.guard));
      tile[mf * kFramesPerBlock + fl] = acc;
    }
    wave_lds_sync();
  }
  __syncthreads();
  const int nvalid = min(kFramesPerBlock, T - t_base);
  for (int i = threadIdx.x; i < g.nfilt * kFramesPerBlock; i += blockDim.x) {
    const int mf = i / kFramesPerBlock, tl = i % kFramesPerBlock;
    if (tl < nvalid) out[((long)b * g.nfilt + mf) * Tout + t_base + tl] = tile[i];
  }
}

struct LenRule {
  int pad_amount, n_fft, hop;
};
// get_seq_len (features.py:368-376), float32 op by op: floor((len + pad - n_fft) / hop) + 1
__device__ __forceinline__ long seq_len_of(int64_t len, const LenRule& r) {
  float v = __fadd_rn((float)len, (float)r.pad_amount);
  v = __fsub_rn(v, (float)r.n_fft);
  v = __fdiv_rn(v, (float)r.hop);
  return (long)(floorf(v) + 1.0f);
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// one wave per (b, f) row.  norm: 0 none / 1 per_feature.  lens_are_samples: lengths are raw
// sample counts (mel forward: seq_len derived here and written to out_len) or frame counts.
__global__ __launch_bounds__(256) void mel_norm_rows_kernel(const float* __restrict__ in, float* __restrict__ out,
                                                            const int64_t* __restrict__ len, int lens_are_samples,
                                                            LenRule rule, int B, int F, int T, long ld, long Tout,
                                                            int norm, int do_mask, float pad_value,
                                                            int64_t* __restrict__ out_len) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + wave;
  if (row >= (long)B * F) return;
  const int b = (int)(row / F), f = (int)(row % F);
  const long n = lens_are_samples ? seq_len_of(len[b], rule) : (long)len[b];
  if (lens_are_samples && f == 0 && lane == 0) out_len[b] = n;
  const float* xi = in + row * ld;
  float* xo = out + row * ld;
  const long nv = std::min<long>(std::max<long>(n, 0), T);
  float mean_f = 0.0f, den = 1.0f;
  if (norm == CFM_NORM_PER_FEATURE) {
    double s = 0.0;
    for (long t = lane; t < nv; t += 64) s += (double)xi[t];
    const double mean = wave_sum_d(s) / (double)n;  // n <= 0: NaN as torch's mean of an empty slice
    double q = 0.0;
    for (long t = lane; t < nv; t += 64) {
      const double d = (double)xi[t] - mean;
      q += d * d;
    }
    const double var = wave_sum_d(q) / (double)(n - 1);  // unbiased (torch.std); n == 1 -> NaN
    mean_f = (float)mean;
    den = __fadd_rn((float)sqrt(var), 1e-5f);             // x_std += CONSTANT (features.py:67)
  }
  const long tend = do_mask ? Tout : T;
  for (long t = lane; t < tend; t += 64) {
    float v;
    if (do_mask && t >= n) v = pad_value;
    else v = norm == CFM_NORM_PER_FEATURE ? __fdiv_rn(__fsub_rn(xi[t], mean_f), den) : xi[t];
    xo[t] = v;
  }
}

// all_features: one block per utterance; statistics over F x [0, seq_len)
__global__ __launch_bounds__(256) void mel_norm_all_kernel(const float* __restrict__ in, float* __restrict__ out,
                                                           const int64_t* __restrict__ len, int lens_are_samples,
                                                           LenRule rule, int F, int T, long ld, long Tout, int do_mask,
                                                           float pad_value, int64_t* __restrict__ out_len) {
  __shared__ double red[4];
  const int b = blockIdx.x, wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long n = lens_are_samples ? seq_len_of(len[b], rule) : (long)len[b];
  if (lens_are_samples && threadIdx.x == 0) out_len[b] = n;
  const long nv = std::min<long>(std::max<long>(n, 0), T);
  const float* xb = in + (long)b * F * ld;
  float* ob = out + (long)b * F * ld;
  const long cnt = (long)F * nv;
  double s = 0.0;
  for (long i = threadIdx.x; i < cnt; i += 256) s += (double)xb[(i / nv) * ld + i % nv];
  s = wave_sum_d(s);
  if (lane == 0) red[wave] = s;
  __syncthreads();
  const double mean = (red[0] + red[1] + red[2] + red[3]) / (double)(F * n);
  __syncthreads();
  double q = 0.0;
  for (long i = threadIdx.x; i < cnt; i += 256) {
    const double d = (double)xb[(i / nv) * ld + i % nv] - mean;
    q += d * d;
  }
  q = wave_sum_d(q);
  if (lane == 0) red[wave] = q;
  __syncthreads();
  const double var = (red[0] + red[1] + red[2] + red[3]) / (double)(F * n - 1);
  const float mean_f = (float)mean;
  const float den = __fadd_rn((float)sqrt(var), 1e-5f);
  const long tend = do_mask ? Tout : T;
  for (int f = wave; f < F; f += 4)
    for (long t = lane; t < tend; t += 64)
      ob[f * ld + t] = (do_mask && t >= n) ? pad_value : __fdiv_rn(__fsub_rn(xb[f * ld + t], mean_f), den);
}

// ---- host: librosa.filters.mel restated (Slaney / HTK mel scale, Slaney area normalisation) ----
double hz_to_mel(double f, bool htk) {
  if (htk) return 2595.0 * std::log10(1.0 + f / 700.0);
  const double f_sp = 200.0 / 3.0, min_log_hz = 1000.0, min_log_mel = min_log_hz / f_sp;
  const double logstep = std::log(6.4) / 27.0;
  return f >= min_log_hz ? min_log_mel + std::log(f / min_log_hz) / logstep : f / f_sp;
}
double mel_to_hz(double m, bool htk) {
  if (htk) return 700.0 * (std::pow(10.0, m / 2595.0) - 1.0);
  const double f_sp = 200.0 / 3.0, min_log_hz = 1000.0, min_log_mel = min_log_hz / f_sp;
  const double logstep = std::log(6.4) / 27.0;
  return m >= min_log_mel ? min_log_hz * std::exp(logstep * (m - min_log_mel)) : f_sp * m;
}

long num_frames(const cfm_mel_cfg& c, long N) {
  if (c.exact_pad) {
    const long Ns = N + 2L * ((c.n_fft - c.n_window_stride) / 2);
    return Ns < c.n_fft ? 0 : 1 + (Ns - c.n_fft) / c.n_window_stride;
  }
  return 1 + N / c.n_window_stride;
}

long output_frames(const cfm_mel_cfg& c, long N) {
  const long T = num_frames(c, N);
  if (c.pad_to == -1) return std::max<long>(T, c.max_length);
  if (c.pad_to > 0 && T % c.pad_to) return T + c.pad_to - T % c.pad_to;
  return T;
}

LenRule len_rule(const cfm_mel_cfg& c) {
  const int pad = c.exact_pad ? 2 * ((c.n_fft - c.n_window_stride) / 2) : c.n_fft / 2 * 2;
  return LenRule{pad, c.n_fft, c.n_window_stride};
}

}  // namespace

extern "C" {

cfm_status cfm_mel_filterbank_slaney(int sr, int n_fft, int n_mels, double fmin, double fmax, int htk, int slaney_norm,
                                     float* out) {
  return guarded([&] {
    if (sr <= 0 || n_fft <= 0 || n_mels <= 0 || out == nullptr || !(fmax > fmin))
      fail(CFM_ERR_INVALID_ARG, "cfm_mel_filterbank_slaney: bad arguments");
    const int nb = 1 + n_fft / 2;
    std::vector<double> fft(nb), mel_f(n_mels + 2);
    for (int k = 0; k < nb; ++k) fft[k] = (double)k * ((double)sr / (double)n_fft);  // fft_frequencies
    const double m0 = hz_to_mel(fmin, htk), m1 = hz_to_mel(fmax, htk);
    const double step = (m1 - m0) / (double)(n_mels + 1);                            // np.linspace
    for (int i = 0; i < n_mels + 2; ++i) mel_f[i] = mel_to_hz(i == n_mels + 1 ? m1 : m0 + i * step, htk);
    for (int i = 0; i < n_mels; ++i) {
      const double fd0 = mel_f[i + 1] - mel_f[i], fd1 = mel_f[i + 2] - mel_f[i + 1];
      const double enorm = 2.0 / (mel_f[i + 2] - mel_f[i]);
      for (int k = 0; k < nb; ++k) {
        const double lower = -(mel_f[i] - fft[k]) / fd0, upper = (mel_f[i + 2] - fft[k]) / fd1;
        const float w = (float)std::max(0.0, std::min(lower, upper));  // stored into a float32 array
        out[(long)i * nb + k] = slaney_norm ? (float)((double)w * enorm) : w;
      }
    }
  });
}

cfm_status cfm_mel_create(const cfm_mel_cfg* cfg, int device, cfm_mel** out) {
  return guarded([&] {
    if (!cfg || !out) fail(CFM_ERR_INVALID_ARG, "cfm_mel_create: null argument");
    const cfm_mel_cfg& c = *cfg;
    if (c.n_fft < 64 || c.n_fft > 2048 || (c.n_fft & (c.n_fft - 1)))
      fail(CFM_ERR_UNSUPPORTED, "cfm_mel_create: n_fft must be a power of two in [64, 2048]");
    if (c.n_window_size < 1 || c.n_window_size > c.n_fft || c.n_window_stride < 1 || c.nfilt < 1)
      fail(CFM_ERR_INVALID_ARG, "cfm_mel_create: need 1 <= n_window_size <= n_fft, hop >= 1, nfilt >= 1");
    if (c.exact_pad && (c.n_window_stride & 1))
      fail(CFM_ERR_UNSUPPORTED, "exact_pad == True needs an even hop size (features.py:242-246)");
    if (c.normalize < 0 || c.normalize > 2 || c.pad_to < -1)
      fail(CFM_ERR_INVALID_ARG, "cfm_mel_create: bad normalize / pad_to");
    HIP_OK(hipSetDevice(device));
    auto* h = new cfm_mel();
    h->c = c;
    h->device = device;
    h->nbins = c.n_fft / 2 + 1;
    h->woff = (c.n_fft - c.n_window_size) / 2;
    const int N2 = c.n_fft / 2;
    std::vector<float2> tw(N2 + 1);
    for (int k = 0; k <= N2; ++k) {
      const double a = -2.0 * M_PI * (double)k / (double)c.n_fft;
      tw[k] = make_float2((float)std::cos(a), (float)std::sin(a));
    }
    tw[0] = make_float2(1.0f, 0.0f);
    tw[N2] = make_float2(-1.0f, 0.0f);
    if (N2 % 2 == 0) tw[N2 / 2] = make_float2(0.0f, -1.0f);
    if (hipMalloc(&h->d_tw, tw.size() * sizeof(float2)) != hipSuccess ||
        hipMalloc(&h->d_win, (size_t)c.n_fft * sizeof(float)) != hipSuccess ||
        hipMalloc(&h->d_band, (size_t)3 * c.nfilt * sizeof(int)) != hipSuccess) {
      cfm_mel_destroy(h);
      fail(CFM_ERR_NOMEM, "cfm_mel_create: hipMalloc failed");
    }
    HIP_OK(hipMemcpy(h->d_tw, tw.data(), tw.size() * sizeof(float2), hipMemcpyHostToDevice));
    *out = h;
  });
}

void cfm_mel_destroy(cfm_mel* h) {
  if (!h) return;
  (void)hipFree(h->d_tw);
  (void)hipFree(h->d_win);
  (void)hipFree(h->d_band);
  (void)hipFree(h->d_wts);
  delete h;
}

cfm_status cfm_mel_set_tables(cfm_mel* h, const float* window, const float* fb, void* stream) {
  return guarded([&] {
    if (!h || !fb) fail(CFM_ERR_INVALID_ARG, "cfm_mel_set_tables: null handle / filterbank");
    HIP_OK(hipSetDevice(h->device));
    const cfm_mel_cfg& c = h->c;
    hipStream_t st = (hipStream_t)stream;
    std::vector<float> w(c.n_window_size, 1.0f), fbh((size_t)c.nfilt * h->nbins);
    if (window) HIP_OK(hipMemcpyAsync(w.data(), window, w.size() * sizeof(float), hipMemcpyDeviceToHost, st));
    HIP_OK(hipMemcpyAsync(fbh.data(), fb, fbh.size() * sizeof(float), hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    std::vector<float> wfull(c.n_fft, 0.0f);
    for (int j = 0; j < c.n_window_size; ++j) wfull[h->woff + j] = w[j];
    // compact each filter to [first nonzero, last nonzero]
    std::vector<int> band(3 * c.nfilt);
    std::vector<float> wts;
    for (int m = 0; m < c.nfilt; ++m) {
      const float* row = &fbh[(size_t)m * h->nbins];
      int lo = 0, hi = -1;
      for (int k = 0; k < h->nbins; ++k)
        if (row[k] != 0.0f) { if (hi < 0) lo = k; hi = k; }
      band[3 * m] = lo;
      band[3 * m + 1] = hi < 0 ? 0 : hi - lo + 1;
      band[3 * m + 2] = (int)wts.size();
      for (int k = lo; k <= hi; ++k) wts.push_back(row[k]);
    }
    (void)hipFree(h->d_wts);
    h->d_wts = nullptr;
    h->nnz = (int)wts.size();
    if (h->nnz > 0 && hipMalloc(&h->d_wts, wts.size() * sizeof(float)) != hipSuccess)
      fail(CFM_ERR_NOMEM, "cfm_mel_set_tables: hipMalloc failed");
    HIP_OK(hipMemcpy(h->d_win, wfull.data(), wfull.size() * sizeof(float), hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(h->d_band, band.data(), band.size() * sizeof(int), hipMemcpyHostToDevice));
    if (h->nnz) HIP_OK(hipMemcpy(h->d_wts, wts.data(), wts.size() * sizeof(float), hipMemcpyHostToDevice));
    const int N2 = c.n_fft / 2;
    h->lds_bytes = (size_t)(N2 + 1) * sizeof(float2) + (size_t)3 * c.nfilt * sizeof(int) +
                   (size_t)((h->nnz + 3) & ~3) * sizeof(float) + (size_t)c.nfilt * kFramesPerBlock * sizeof(float) +
                   (size_t)kWaves * 2 * N2 * sizeof(float2);
    if (h->lds_bytes > 160 * 1024) fail(CFM_ERR_UNSUPPORTED, "cfm_mel_set_tables: tables exceed the 160 KB LDS");
    (void)hipFuncSetAttribute((const void*)mel_frames_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)h->lds_bytes);
    h->tables_set = true;
  });
}

long cfm_mel_num_frames(const cfm_mel* h, long n) { return h ? num_frames(h->c, n) : -1; }
long cfm_mel_output_frames(const cfm_mel* h, long n) { return h ? output_frames(h->c, n) : -1; }

cfm_status cfm_mel_forward(cfm_mel* h, const float* x, const int64_t* len, int B, long N, float dither, uint64_t seed,
                           const uint8_t* nb_mask, int nb_max_bin, float* out, int64_t* out_len, void* stream) {
  return guarded([&] {
    if (!h || !h->tables_set) fail(CFM_ERR_WEIGHTS, "cfm_mel_forward: cfm_mel_set_tables not called");
    if (B < 0 || N < 1 || !x || !len || !out || !out_len) fail(CFM_ERR_INVALID_ARG, "cfm_mel_forward: bad arguments");
    const cfm_mel_cfg& c = h->c;
    const int P = c.exact_pad ? (c.n_fft - c.n_window_stride) / 2 : 0;
    if (c.exact_pad && P >= N) fail(CFM_ERR_INVALID_ARG, "cfm_mel_forward: reflect pad needs more samples than the pad");
    const long Ns = N + 2L * P;
    if (!c.exact_pad && c.n_fft / 2 >= Ns)
      fail(CFM_ERR_INVALID_ARG, "cfm_mel_forward: the stft center reflect pad needs more than n_fft/2 samples");
    const long T = num_frames(c, N), Tout = output_frames(c, N);
    if (T < 1) fail(CFM_ERR_INVALID_ARG, "cfm_mel_forward: signal shorter than one frame");
    if (B == 0) return;
    HIP_OK(hipSetDevice(h->device));
    hipStream_t st = (hipStream_t)stream;
    MelGeom g{};
    g.N = N;
    g.Ns = Ns;
    g.P = P;
    g.cpad = c.exact_pad ? 0 : c.n_fft / 2;
    g.hop = c.n_window_stride;
    g.n_fft = c.n_fft;
    g.nfilt = c.nfilt;
    g.nbins = h->nbins;
    g.use_pre = c.use_preemph;
    g.pre = c.preemph;
    g.mag_mode = c.mag_power == 1.0f ? 0 : (c.mag_power == 2.0f ? 1 : 2);
    g.mag_power = c.mag_power;
    g.log = c.log;
    g.guard_type = c.log_zero_guard_type;
    g.guard = c.log_zero_guard_value;
    g.dither = dither;
    g.seed = seed;
    dim3 grid((unsigned)((T + kFramesPerBlock - 1) / kFramesPerBlock), (unsigned)B);
    hipLaunchKernelGGL(mel_frames_kernel, grid, dim3(64 * kWaves), h->lds_bytes, st, x, (int)T, Tout, g, h->d_win,
                       h->d_tw, h->d_band, h->d_wts, h->nnz, nb_mask, nb_max_bin, out);
    HIP_OK(hipGetLastError());
    const LenRule r = len_rule(c);
    if (c.normalize == CFM_NORM_ALL_FEATURES)
      hipLaunchKernelGGL(mel_norm_all_kernel, dim3(B), dim3(256), 0, st, out, out, len, 1, r, c.nfilt, (int)T, Tout,
                         Tout, 1, c.pad_value, out_len);
    else
      hipLaunchKernelGGL(mel_norm_rows_kernel, dim3((unsigned)(((long)B * c.nfilt + 3) / 4)), dim3(256), 0, st, out,
                         out, len, 1, r, B, c.nfilt, (int)T, Tout, Tout, c.normalize, 1, c.pad_value, out_len);
    HIP_OK(hipGetLastError());
  });
}

cfm_status cfm_normalize_batch(const float* x, const int64_t* seq_len, int B, int F, int T, int type, float* out,
                               void* stream) {
  return guarded([&] {
    if (B < 0 || F < 1 || T < 1 || !x || !seq_len || !out) fail(CFM_ERR_INVALID_ARG, "cfm_normalize_batch: bad arguments");
    if (type != CFM_NORM_PER_FEATURE && type != CFM_NORM_ALL_FEATURES)
      fail(CFM_ERR_INVALID_ARG, "cfm_normalize_batch: type must be per_feature or all_features");
    if (B == 0) return;
    hipStream_t st = (hipStream_t)stream;
    const LenRule r{0, 0, 1};
    if (type == CFM_NORM_ALL_FEATURES)
      hipLaunchKernelGGL(mel_norm_all_kernel, dim3(B), dim3(256), 0, st, x, out, seq_len, 0, r, F, T, (long)T, (long)T,
                         0, 0.0f, (int64_t*)nullptr);
    else
      hipLaunchKernelGGL(mel_norm_rows_kernel, dim3((unsigned)(((long)B * F + 3) / 4)), dim3(256), 0, st, x, out,
                         seq_len, 0, r, B, F, T, (long)T, (long)T, CFM_NORM_PER_FEATURE, 0, 0.0f, (int64_t*)nullptr);
    HIP_OK(hipGetLastError());
  });
}

}  // extern "C"
