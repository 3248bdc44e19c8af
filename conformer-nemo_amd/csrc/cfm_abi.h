// Host-side error plumbing shared by the C-ABI translation units (encoder.hip, ctc.hip): no C++
// exception crosses the ABI; every entry point runs its body in guarded(), which turns a thrown
// CfmError into a status code and a thread-local message for cfm_last_error().
#pragma once
#include <hip/hip_runtime.h>

#include <cstring>
#include <exception>
#include <string>

#include "../../include/cfm_encoder.h"

namespace cfm {

extern thread_local std::string g_last_error;

struct CfmError {
  cfm_status code;
  std::string msg;
};

[[noreturn]] inline void fail(cfm_status code, const std::string& msg) { throw CfmError{code, msg}; }

#define HIP_OK(expr)                                                                               \
  do {                                                                                             \
    hipError_t _e = (expr);                                                                        \
    if (_e != hipSuccess) ::cfm::fail(CFM_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

template <class F>
cfm_status guarded(F&& f) {
  try {
    f();
    return CFM_OK;
  } catch (const CfmError& e) {
    g_last_error = e.msg;
    return e.code;
  } catch (const std::exception& e) {
    g_last_error = e.what();
    return CFM_ERR_INVALID_ARG;
  } catch (...) {
    g_last_error = "unknown error";
    return CFM_ERR_INVALID_ARG;
  }
}

// The fp16 build (libcfm_f16.so, CFM_HALF_F16) is an inference build: its training and backward
// entry points refuse the 16-bit mode (fp16 gradients would need loss scaling, and several backward
// kernels - the weight-gradient TN kernel's bias sums, the attention-backward staging - decode their
// 16-bit operands as bf16).  fp32 mode stays available in either library; bf16 training: libcfm.so.
inline void refuse_half_training(bool is_f32, const char* what) {
#ifdef CFM_HALF_F16
  if (!is_f32) fail(CFM_ERR_UNSUPPORTED, std::string(what) + ": the fp16 library is inference-only; train in bf16 (libcfm.so) or fp32");
#else
  (void)is_f32; (void)what;
#endif
}

inline long round_up(long v, long m) { return (v + m - 1) / m * m; }

// host copies of the 16-bit compute type's conversions (cfm_common.h): bfloat16, or IEEE fp16 in
// the CFM_HALF_F16 build (round to nearest even, saturated to +-65504)
#ifdef CFM_HALF_F16
inline uint16_t host_f2bf(float f) {
  if (f == f) f = f > 65504.0f ? 65504.0f : (f < -65504.0f ? -65504.0f : f);
  const _Float16 h = (_Float16)f;
  uint16_t u;
  std::memcpy(&u, &h, 2);
  return u;
}
inline float host_bf2f(uint16_t v) {
  _Float16 h;
  std::memcpy(&h, &v, 2);
  return (float)h;
}
#else
inline uint16_t host_f2bf(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);  // NaN stays NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
inline float host_bf2f(uint16_t v) {
  const uint32_t u = (uint32_t)v << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}
#endif

}  // namespace cfm
