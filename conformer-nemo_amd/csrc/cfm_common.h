// Shared device helpers for the gfx950 (CDNA4) Conformer encoder kernels.
//
// Compute-type abstraction used by every MFMA kernel in this library
// ------------------------------------------------------------------
// All MFMA operands are staged as 32-byte "k-slabs" per matrix row: lane l of a wave supplies
// row (l & 31) and the 16 bytes at offset 16*(l >> 5) of the slab.
//   * bf16 : 16 bytes = 8 bf16 = exactly the A/B fragment of v_mfma_f32_32x32x16_bf16
//            (lane holds A[row l&31][k = 8*(l>>5) + j]).
//   * fp32 : 16 bytes = 4 floats, consumed by 4 x v_mfma_f32_32x32x2_f32, MFMA e taking element e
//            (lane half h then contributes logical k = 4h + e; A and B agree, so the sum is the
//            same dot product in a different order).
// Loaders, LDS images and swizzles are therefore byte-identical for both compute types; only the
// per-slab MFMA micro-step differs (`mfma_slab`).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define CFM_DEV __device__ __forceinline__

// The 16-bit compute type.  `bf16_t` is its 16-bit storage: bfloat16 in libcfm.so, IEEE fp16 in
// libcfm_f16.so (the same sources built with CFM_HALF_F16: the fp16 compute mode, 3 more mantissa
// bits at the same MFMA rate).  Only the conversions below, Vec16<bf16_t> and the two MFMA
// wrappers see the format; every loader, LDS image, swizzle and packing trick is format-agnostic.
typedef uint16_t bf16_t;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) float f32x4;
#ifdef CFM_HALF_F16
typedef __attribute__((ext_vector_type(8))) _Float16 h16x8;
CFM_DEV float bf2f(bf16_t v) { return (float)__builtin_bit_cast(_Float16, v); }
CFM_DEV bf16_t f2bf(float f) {
  // saturate to the fp16 range (v_med3_f32) so that an outlier cannot become inf, then round to nearest even
  return __builtin_bit_cast(bf16_t, (_Float16)__builtin_amdgcn_fmed3f(f, -65504.0f, 65504.0f));
}
CFM_DEV f32x16 mfma16_32x32x16(const uint4& a, const uint4& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(h16x8, a), __builtin_bit_cast(h16x8, b), c, 0, 0, 0);
}
CFM_DEV f32x4 mfma16_16x16x32(const uint4& a, const uint4& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h16x8, a), __builtin_bit_cast(h16x8, b), c, 0, 0, 0);
}
#else
typedef __attribute__((ext_vector_type(8))) __bf16 h16x8;
CFM_DEV float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }
CFM_DEV bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;  // lowers to v_cvt_pk_bf16_f32 (round-to-nearest-even, NaN-preserving)
  return __builtin_bit_cast(bf16_t, b);
}
CFM_DEV f32x16 mfma16_32x32x16(const uint4& a, const uint4& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(h16x8, a), __builtin_bit_cast(h16x8, b), c, 0, 0, 0);
}
CFM_DEV f32x4 mfma16_16x16x32(const uint4& a, const uint4& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(h16x8, a), __builtin_bit_cast(h16x8, b), c, 0, 0, 0);
}
#endif

// Scalar load / store in the compute type, math in fp32.
template <typename T> CFM_DEV float ld_f(const T* p);
template <> CFM_DEV float ld_f<float>(const float* p) { return *p; }
template <> CFM_DEV float ld_f<bf16_t>(const bf16_t* p) { return bf2f(*p); }
template <typename T> CFM_DEV void st_f(T* p, float v);
template <> CFM_DEV void st_f<float>(float* p, float v) { *p = v; }
template <> CFM_DEV void st_f<bf16_t>(bf16_t* p, float v) { *p = f2bf(v); }

// One 32-byte k-slab of a 32x32 output tile: acc += A_slab * B_slab.
template <typename T> CFM_DEV void mfma_slab(f32x16& acc, const uint4& a, const uint4& b);
template <> CFM_DEV void mfma_slab<bf16_t>(f32x16& acc, const uint4& a, const uint4& b) {
  acc = mfma16_32x32x16(a, b, acc);
}
template <> CFM_DEV void mfma_slab<float>(f32x16& acc, const uint4& a, const uint4& b) {
  acc = __builtin_amdgcn_mfma_f32_32x32x2f32(__uint_as_float(a.x), __uint_as_float(b.x), acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x2f32(__uint_as_float(a.y), __uint_as_float(b.y), acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x2f32(__uint_as_float(a.z), __uint_as_float(b.z), acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x2f32(__uint_as_float(a.w), __uint_as_float(b.w), acc, 0, 0, 0);
}

// C/D layout of a 32x32 MFMA accumulator: element r of lane l sits at
//   row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5),  col = l & 31.
CFM_DEV int acc_row(int r, int lane) { return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); }

// 16 bytes of compute-type values -> / <- fp32.
template <typename T> struct Vec16;
template <> struct Vec16<float> {
  static constexpr int N = 4;
  static CFM_DEV void to_f32(const uint4& u, float* f) {
    f[0] = __uint_as_float(u.x); f[1] = __uint_as_float(u.y); f[2] = __uint_as_float(u.z); f[3] = __uint_as_float(u.w);
  }
  static CFM_DEV uint4 from_f32(const float* f) {
    return make_uint4(__float_as_uint(f[0]), __float_as_uint(f[1]), __float_as_uint(f[2]), __float_as_uint(f[3]));
  }
};
template <> struct Vec16<bf16_t> {
  static constexpr int N = 8;
  static CFM_DEV void to_f32(const uint4& u, float* f) {
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) { f[2 * i] = bf2f((bf16_t)(w[i] & 0xffffu)); f[2 * i + 1] = bf2f((bf16_t)(w[i] >> 16)); }
  }
  static CFM_DEV uint4 from_f32(const float* f) {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = (uint32_t)f2bf(f[2 * i]) | ((uint32_t)f2bf(f[2 * i + 1]) << 16);
    return make_uint4(w[0], w[1], w[2], w[3]);
  }
};

CFM_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
// x * sigmoid(x) and sigmoid(x) with v_exp_f32 + v_rcp_f32 (~1 ulp each) instead of an IEEE
// divide sequence: the epilogues apply these to every output element.
CFM_DEV float sigmoidf_(float x) { return __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }
CFM_DEV float swishf(float x) { return x * sigmoidf_(x); }

// Asynchronous 16-byte global -> LDS copy (global_load_lds_dwordx4). The LDS destination is the
// wave-uniform `lds_base` + 16 * lane; the global source is per lane.
CFM_DEV void glds16(const void* gsrc, void* lds_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)gsrc,
                                   (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
}

namespace cfm {
// 16-byte store with the sc1 (write-through) cache policy, through a raw buffer descriptor built
// from the wave-uniform tensor base: the line goes to memory as it is written, so the kernel leaves
// no dirty L2 lines for the launch boundary to write back (MI355X_MICROARCH.md, boundary row).
CFM_DEV void store16_wt(const void* base, long byte_off, uint4 v) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)0x7fffffff, 0x00020000);
  u32x4 d = {v.x, v.y, v.z, v.w};
  __builtin_amdgcn_raw_buffer_store_b128(d, rs, (int)byte_off, 0, 16);
}
// LDS-DMA issued from inline asm (hipcc's waitcnt pass does not see it, so it does not put a
// vmcnt(0) in front of every ds_read), counted waits, a raw barrier and LDS byte addresses.
CFM_DEV void glds16_asm(const void* gsrc, uint32_t lds_dst) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(lds_dst) : "memory");
}
template <int N> CFM_DEV void wait_vmcnt() {
  static_assert(N >= 0 && N <= 63, "vmcnt");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
CFM_DEV void wait_lgkm0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
CFM_DEV void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
CFM_DEV uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

}  // namespace cfm
