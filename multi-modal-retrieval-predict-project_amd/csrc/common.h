// Shared helpers for libmmr (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mmr.h"

namespace mmr {

void set_error(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
void clear_error();

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

__host__ __device__ inline int64_t round_up(int64_t x, int64_t m) { return (x + m - 1) / m * m; }
__host__ __device__ inline int64_t ceil_div(int64_t x, int64_t m) { return (x + m - 1) / m; }

// bf16 <-> f32 (bit patterns as uint16; RNE, inputs finite)
__device__ __forceinline__ float bf2f(uint16_t b) { return __uint_as_float(((uint32_t)b) << 16); }
__device__ __forceinline__ uint16_t f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

// two f32 -> packed bf16x2 (RNE) in one v_cvt_pk_bf16_f32
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pack2bf(float a, float b) {
  const bf16x2_t v = {(__bf16)a, (__bf16)b};
  return __builtin_bit_cast(uint32_t, v);
}

// GELU(erf) with erf from Abramowitz-Stegun 7.1.26 (|err| <= 1.5e-7): branch-free, one exp + one
// rcp instead of ocml's erff.
__device__ __forceinline__ float erf_as(float x) {
  const float a = fabsf(x);
  const float t = __frcp_rn(fmaf(0.3275911f, a, 1.0f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  const float y = 1.0f - p * t * __expf(-a * a);
  return copysignf(y, x);
}
__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.0f + erf_as(x * 0.70710678118654752f)); }

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
template <typename T>
__device__ __forceinline__ T wave_max(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

}  // namespace mmr

#define MMR_CHECK_HIP(expr)                                                                \
  do {                                                                                     \
    hipError_t _e = (expr);                                                                \
    if (_e != hipSuccess) {                                                                \
      mmr::set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e), __FILE__,      \
                     __LINE__);                                                            \
      return _e == hipErrorOutOfMemory ? MMR_ERR_OOM : MMR_ERR_HIP;                        \
    }                                                                                      \
  } while (0)

#define MMR_REQUIRE(cond, ...)      \
  do {                              \
    if (!(cond)) {                  \
      mmr::set_error(__VA_ARGS__);  \
      return MMR_ERR_INVALID;       \
    }                               \
  } while (0)

#define MMR_LAUNCH_CHECK()                                                                 \
  do {                                                                                     \
    hipError_t _e = hipGetLastError();                                                     \
    if (_e != hipSuccess) {                                                                \
      mmr::set_error("kernel launch failed: %s (%s:%d)", hipGetErrorString(_e), __FILE__,  \
                     __LINE__);                                                            \
      return MMR_ERR_HIP;                                                                  \
    }                                                                                      \
  } while (0)
