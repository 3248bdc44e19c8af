// LayerNorm of one row by one wave (torch.nn.LayerNorm semantics: biased variance, eps 1e-5;
// conformer_modules.py:66-70, 120).  Lane l holds float4 chunks l, l+64, ... of the row (E4 chunks,
// d % 4 == 0, d <= 256 * E4).  Optional second LayerNorm applied to the first's result (norm_out of
// layer l feeding norm_feed_forward1 of layer l+1) and optional Swish on the compute-type output.
// All loads are unconditional (clamped address, value selected afterwards).
#pragma once
#include "cfm_common.h"

namespace cfm {

template <int E4>
CFM_DEV void ln_load(const float* xr_, int d, int lane, float4 (&v)[E4]) {
  const int d4 = d >> 2;
  const float4* xr = (const float4*)xr_;
#pragma unroll
  for (int e = 0; e < E4; ++e) {
    const int g = lane + 64 * e;
    const float4 t = xr[min(g, d4 - 1)];
    v[e] = (g < d4) ? t : make_float4(0, 0, 0, 0);
  }
}

// LayerNorm(s) of a row already in registers (ln_load layout), then the stores.
template <typename T, int E4>
CFM_DEV void ln_apply(float4 (&v)[E4], int d, int lane, const float* w, const float* b, float* out_x,
                      const float* w2, const float* b2, T* out_t, int swish_out) {
  // no implicit FMA contraction: several rows per wave run unrolled copies of this body, and every
  // copy must round identically (bitwise batch invariance)
#pragma clang fp contract(off)
  const int d4 = d >> 2;
  float s = 0.0f;
#pragma unroll
  for (int e = 0; e < E4; ++e) s += v[e].x + v[e].y + v[e].z + v[e].w;
  const float inv_d = 1.0f / (float)d;
  auto normalize = [&](const float* ww, const float* bbp) {
    const float mean = wave_sum(s) * inv_d;
    float q = 0.0f;
#pragma unroll
    for (int e = 0; e < E4; ++e) {
      const int g = lane + 64 * e;
      if (g < d4) {
        const float a0 = v[e].x - mean, a1 = v[e].y - mean, a2 = v[e].z - mean, a3 = v[e].w - mean;
        q += a0 * a0 + a1 * a1 + a2 * a2 + a3 * a3;
      }
    }
    const float rstd = 1.0f / sqrtf(wave_sum(q) * inv_d + 1e-5f);
    s = 0.0f;
#pragma unroll
    for (int e = 0; e < E4; ++e) {
      const int g = lane + 64 * e;
      const float4 wv = ((const float4*)ww)[min(g, d4 - 1)], bv = ((const float4*)bbp)[min(g, d4 - 1)];
      if (g < d4) {
        v[e].x = (v[e].x - mean) * rstd * wv.x + bv.x;
        v[e].y = (v[e].y - mean) * rstd * wv.y + bv.y;
        v[e].z = (v[e].z - mean) * rstd * wv.z + bv.z;
        v[e].w = (v[e].w - mean) * rstd * wv.w + bv.w;
        s += v[e].x + v[e].y + v[e].z + v[e].w;
      }
    }
  };
  normalize(w, b);
  if (out_x) {
    float4* o = (float4*)out_x;
#pragma unroll
    for (int e = 0; e < E4; ++e) {
      const int g = lane + 64 * e;
      if (g < d4) o[g] = v[e];
    }
  }
  if (w2) normalize(w2, b2);
  if (out_t) {
#pragma unroll
    for (int e = 0; e < E4; ++e) {
      const int g = lane + 64 * e;
      if (g < d4) {
        float f[4] = {v[e].x, v[e].y, v[e].z, v[e].w};
        if (swish_out) {
#pragma unroll
          for (int i = 0; i < 4; ++i) f[i] = swishf(f[i]);
        }
        if constexpr (sizeof(T) == 2) {
          *(uint2*)(out_t + 4 * g) = make_uint2((uint32_t)f2bf(f[0]) | ((uint32_t)f2bf(f[1]) << 16),
                                                (uint32_t)f2bf(f[2]) | ((uint32_t)f2bf(f[3]) << 16));
        } else {
          *(float4*)(out_t + 4 * g) = make_float4(f[0], f[1], f[2], f[3]);
        }
      }
    }
  }
}

template <typename T, int E4>
CFM_DEV void ln_row(const float* xr, int d, int lane, const float* w, const float* b, float* out_x,
                    const float* w2, const float* b2, T* out_t, int swish_out) {
  float4 v[E4];
  ln_load<E4>(xr, d, lane, v);
  ln_apply<T, E4>(v, d, lane, w, b, out_x, w2, b2, out_t, swish_out);
}

}  // namespace cfm
