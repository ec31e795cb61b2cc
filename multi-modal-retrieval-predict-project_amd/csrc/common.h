// Shared helpers for libmmr (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>

#include "mmr.h"

namespace mmr {

void set_error(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
void clear_error();

// process-wide launch-variant pins (mmr_pin_variant; -1 = the launcher's own choice)
extern std::atomic<int> pin_gemm_bf16;
extern std::atomic<int> pin_x3_waves;
extern std::atomic<int> pin_x3_mlp;

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

__host__ __device__ inline int64_t round_up(int64_t x, int64_t m) { return (x + m - 1) / m * m; }
__host__ __device__ inline int64_t ceil_div(int64_t x, int64_t m) { return (x + m - 1) / m; }

// blockIdx -> work index such that the blocks the dispatcher places on one XCD (orig % 8) get a
// contiguous run of work indices (bijective for any n): neighbouring work units — the heads of
// one batch row, sharing 128-B lines of a fused QKV row — then meet in the same XCD's L2.
__device__ __forceinline__ int xcd_contiguous(int orig, int n) {
  const int q = n / 8, r8 = n % 8, xcd = orig % 8;
  return (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + orig / 8;
}

// bf16 <-> f32 (bit patterns as uint16; RNE, inputs finite)
__device__ __forceinline__ float bf2f(uint16_t b) { return __uint_as_float(((uint32_t)b) << 16); }
__device__ __forceinline__ uint16_t f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

// two f32 -> packed bf16x2 (RNE) in one v_cvt_pk_bf16_f32
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
// Pins a loaded value as used on every path: without it hipcc sinks a load whose value is later
// masked into the branch that consumes it, and then waits on each such load before issuing the next.
template <class T>
__device__ __forceinline__ void pin(T& v) {
  asm volatile("" : "+v"(v));
}
// a * b rounded to f32 on its own: HIP's __fmul_rn is a plain multiply (no OCML_BASIC_ROUNDED_OPERATIONS)
// that hipcc may contract with a following add into one fma; the pinned product cannot be
__device__ __forceinline__ float mul_rn(float a, float b) {
  float p = a * b;
  asm volatile("" : "+v"(p));
  return p;
}
// max over each 16-lane row by DPP: quad_perm [1,0,3,2] / [2,3,0,1] (xor 1 / 2), then row_half_mirror /
// row_mirror, which pair quads / halves whose lanes already agree — the xor-1/2/4/8 butterfly's result
// without its 4 LDS permutes
template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float row16_max(float v) {
  v = fmaxf(v, dppf<0xB1>(v));
  v = fmaxf(v, dppf<0x4E>(v));
  v = fmaxf(v, dppf<0x141>(v));
  return fmaxf(v, dppf<0x140>(v));
}
// the same butterfly for sums (bit-identical to the xor 1/2/4/8 shuffle order)
__device__ __forceinline__ float row16_sum(float v) {
  v += dppf<0xB1>(v);
  v += dppf<0x4E>(v);
  v += dppf<0x141>(v);
  return v + dppf<0x140>(v);
}

__device__ __forceinline__ uint32_t pack2bf(float a, float b) {
  const bf16x2_t v = {(__bf16)a, (__bf16)b};
  return __builtin_bit_cast(uint32_t, v);
}

// e^x for the x3 softmax (x = s - max <= 0; -inf is the caller's case): 2^t with t = RN(x log2 e) and t's
// rounding error carried to first order, 2^t (1 + ln 2 (fma(x, L2E, -t) + x L2E_lo)) — one v_exp_f32
// (1 ulp) and four FMA-class ops, <= ~2 ulp, against ocml expf's ~14 VALU (range reduction by rndne /
// ldexp and overflow / underflow selects the softmax never needs); results below 2^-126 may flush to 0.
// x is clamped at -104 (e^-104 is below the smallest f32 denormal): a masked score (HF's -FLT_MAX) would
// otherwise overflow x log2 e to -inf and turn the correction into inf * 0
__device__ __forceinline__ float exp_acc(float x) {
  constexpr float L2E = 1.44269504088896341f, L2E_LO = 1.925962991e-08f;  // log2 e = L2E + L2E_LO
  x = fmaxf(x, -104.0f);
  const float t = x * L2E;
  const float c = fmaf(x, L2E_LO, fmaf(x, L2E, -t));
  const float e = __builtin_amdgcn_exp2f(t);
  return fmaf(e, c * 0.69314718055994531f, e);
}

// GELU(erf) with erf from Abramowitz-Stegun 7.1.26 (|err| <= 1.5e-7): branch-free, one exp + one
// rcp instead of ocml's erff.
__device__ __forceinline__ float erf_as(float x) {
  const float a = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, a, 1.0f));  // v_rcp_f32 (1 ulp), not a division
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  const float y = fmaf(-p * t, __builtin_amdgcn_exp2f(-1.44269504088896341f * a * a), 1.0f);  // v_exp_f32
  return copysignf(y, x);
}
__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.0f + erf_as(x * 0.70710678118654752f)); }
// GELU(x) = x * Phi(x) as x * sigmoid(x * P(x^2)), P least-squares-fitted to the erf form on
// [-7, 7]: |err| < 1.2e-5 everywhere (40x below a bf16 half-ulp at |y| ~ 1), 7 VALU + v_exp + v_rcp
// instead of 11 VALU + v_exp + v_rcp.  Used where GELU output is rounded to bf16 (GEMM epilogues,
// fused Swin MLP); tools/gelu_fit.py holds the fit.
__device__ __forceinline__ float gelu_fast(float v) {
  const float x2 = v * v;
  float p = fmaf(3.275317185739523e-06f, x2, -7.756018138382363e-05f);
  p = fmaf(p, x2, -0.00016997469037563395f);
  p = fmaf(p, x2, 0.07280746695679054f);
  p = fmaf(p, x2, 1.5957042563586181f);
  const float e = __builtin_amdgcn_exp2f(-1.4426950408889634f * v * p);
  return v * __builtin_amdgcn_rcpf(1.0f + e);
}

// gelu_fast with -log2(e) folded into P (bitwise equal to one lane of gelu_fast2): for code where
// the GELU runs beside MFMAs, which packed f32 math slows (MI355X_MICROARCH.md, filler prices)
__device__ __forceinline__ float gelu_fast1(float v) {
  constexpr float L2E = -1.4426950408889634f;
  const float x2 = v * v;
  float p = fmaf(3.275317185739523e-06f * L2E, x2, -7.756018138382363e-05f * L2E);
  p = fmaf(p, x2, -0.00016997469037563395f * L2E);
  p = fmaf(p, x2, 0.07280746695679054f * L2E);
  p = fmaf(p, x2, 1.5957042563586181f * L2E);
  const float e = __builtin_amdgcn_exp2f(v * p);
  return v * __builtin_amdgcn_rcpf(e + 1.0f);
}

// gelu_fast on two values with packed f32 math (v_pk_fma / v_pk_mul / v_pk_add: half the VALU
// issues of two scalar calls), with -log2(e) folded into P's coefficients (one v_pk_mul fewer;
// equal to gelu_fast up to f32 rounding of the folded constants).
typedef float f32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2_t gelu_fast2(f32x2_t v) {
  constexpr float L2E = -1.4426950408889634f;
  const f32x2_t x2 = v * v;
  f32x2_t p = __builtin_elementwise_fma((f32x2_t)(3.275317185739523e-06f * L2E), x2, (f32x2_t)(-7.756018138382363e-05f * L2E));
  p = __builtin_elementwise_fma(p, x2, (f32x2_t)(-0.00016997469037563395f * L2E));
  p = __builtin_elementwise_fma(p, x2, (f32x2_t)(0.07280746695679054f * L2E));
  p = __builtin_elementwise_fma(p, x2, (f32x2_t)(1.5957042563586181f * L2E));
  const f32x2_t y = v * p;
  f32x2_t e;
  e.x = __builtin_amdgcn_exp2f(y.x);
  e.y = __builtin_amdgcn_exp2f(y.y);
  const f32x2_t d = e + 1.0f;
  f32x2_t r;
  r.x = __builtin_amdgcn_rcpf(d.x);
  r.y = __builtin_amdgcn_rcpf(d.y);
  return v * r;
}

// GELU for an MX-fp8 (e4m3) output: x sigmoid(x (a + b x^2)), (a, b) minimax-fitted to the erf form on
// [-12, 12] (tests/test_gelu_q8_cpu.py holds the fit's bounds): |err| <= 2.71e-4, relative <= 2.31 % wherever
// |GELU| >= 1e-2 — under the smallest e4m3 half-ulp (2^-5 relative) and ~2^-12 of a block's amax >= 1, while
// e4m3 keeps 3 mantissa bits.  4 packed f32 ops + 2 v_exp + 2 v_rcp per pair instead of gelu_fast2's 7 + 4: the
// fused FFN1 -> FFN2 operand epilogue (OUT8) runs it.
__device__ __forceinline__ f32x2_t gelu_q8x2(f32x2_t v) {
  constexpr float L2E = -1.4426950408889634f;
  const f32x2_t x2 = v * v;
  const f32x2_t p = __builtin_elementwise_fma((f32x2_t)(0.06940179f * L2E), x2, (f32x2_t)(1.60031416f * L2E));
  const f32x2_t y = v * p;
  f32x2_t e;
  e.x = __builtin_amdgcn_exp2f(y.x);
  e.y = __builtin_amdgcn_exp2f(y.y);
  const f32x2_t d = e + 1.0f;
  f32x2_t r;
  r.x = __builtin_amdgcn_rcpf(d.x);
  r.y = __builtin_amdgcn_rcpf(d.y);
  return v * r;
}

// lane-permuted copy of a 32- or 64-bit value by DPP (64-bit: both halves)
template <int CTRL, typename T>
__device__ __forceinline__ T dpp_mov(T v) {
  if constexpr (sizeof(T) == 4) {
    return __builtin_bit_cast(T, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
  } else {
    static_assert(sizeof(T) == 8, "dpp_mov: 32- or 64-bit values");
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)u, CTRL, 0xF, 0xF, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(u >> 32), CTRL, 0xF, 0xF, false);
    return __builtin_bit_cast(T, ((uint64_t)hi << 32) | lo);
  }
}
// Sum over the wave as the xor butterfly 32, 16, 8, 4, 2, 1 (each lane adds its own and its partner's
// value: the same tree, so the same bits, at every call site — the kNN norms and f64 re-scores rely on
// the order).  Levels 32 / 16 are LDS swaps; the in-row levels are DPP: row_ror:8 reads lane i ^ 8;
// row_ror:4 reads lane (i + 4) mod 16, which after the 8-level holds the same value as lane i ^ 4
// (the values are symmetric under ^8); quad_perm [2,3,0,1] / [1,0,3,2] are xor 2 / 1.  (Six dependent
// LDS round trips per call before; the f64 form cost the kNN selection's query norm ~0.3 us.)
template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
  v += __shfl_xor(v, 32, 64);
  v += __shfl_xor(v, 16, 64);
  v += dpp_mov<0x128>(v);
  v += dpp_mov<0x124>(v);
  v += dpp_mov<0x4E>(v);
  v += dpp_mov<0xB1>(v);
  return v;
}
// wave_sum of RB values at once (a[r] = lane's partial of row r): a reduce-scatter over the same xor
// 32 / 16 / 8 ... tree, so every row total is bit-identical to wave_sum(a[r]) (each level adds the same
// two partials; f64 / f32 addition is commutative).  The first log2(RB) levels halve the rows a lane
// carries (upper lanes keep the upper half), the rest are wave_sum's levels on one value: the levels'
// shuffles of all rows are independent, so a level costs one LDS round trip instead of RB.  Returns
// the total of row `row` (padding rows past RB: 0); lanes with (lane & ((64 >> LOG) - 1)) == 0 hold
// each row once.
template <int RB, typename T>
__device__ __forceinline__ T rows_wave_sum(const T (&a)[RB], int lane, int& row) {
  constexpr int LOG = RB > 4 ? 3 : RB > 2 ? 2 : RB > 1 ? 1 : 0;
  static_assert(RB <= 8, "rows_wave_sum: at most 8 rows");
  constexpr int P = 1 << LOG;
  T v[P];
#pragma unroll
  for (int r = 0; r < P; ++r) v[r] = r < RB ? a[r] : (T)0;
  row = 0;
#pragma unroll
  for (int s = 0; s < LOG; ++s) {
    const int m = 32 >> s, h = P >> (s + 1);
    const bool up = (lane & m) != 0;
    T sent[P / 2];
#pragma unroll
    for (int j = 0; j < h; ++j) sent[j] = __shfl_xor(up ? v[j] : v[h + j], m, 64);
#pragma unroll
    for (int j = 0; j < h; ++j) v[j] = (up ? v[h + j] : v[j]) + sent[j];
    row += up ? h : 0;
  }
  // the remaining butterfly levels as in wave_sum (row_ror:4 only when the 8-level was a butterfly
  // level: after a reduce-scatter 8-level, lanes i and i ^ 8 hold different rows)
  if constexpr (LOG == 0) v[0] += __shfl_xor(v[0], 32, 64);
  if constexpr (LOG <= 1) v[0] += __shfl_xor(v[0], 16, 64);
  if constexpr (LOG <= 2) {
    v[0] += dpp_mov<0x128>(v[0]);
    v[0] += dpp_mov<0x124>(v[0]);
  } else {
    v[0] += __shfl_xor(v[0], 4, 64);
  }
  v[0] += dpp_mov<0x4E>(v[0]);
  v[0] += dpp_mov<0xB1>(v[0]);
  return v[0];
}
template <typename T>
__device__ __forceinline__ T wave_max(T v) {  // max is order-free: the wave_sum lane pattern
  v = fmaxf(v, __shfl_xor(v, 32, 64));
  v = fmaxf(v, __shfl_xor(v, 16, 64));
  v = fmaxf(v, dpp_mov<0x128>(v));
  v = fmaxf(v, dpp_mov<0x124>(v));
  v = fmaxf(v, dpp_mov<0x4E>(v));
  return fmaxf(v, dpp_mov<0xB1>(v));
}

// MX-fp8 activation operand of an 8-value chunk (channels 8*ch .. 8*ch+7 of a row), written by the
// producer of the bf16 row (LayerNorm, add-pos): vb = the bf16-rounded values as stored, so the
// result is bit-identical to mmr_quantize_mxfp8 of the bf16 output.  A 32-block is 4 ADJACENT
// lanes' chunks (ch % 4 = lane % 4; every lane of the group calls it); its E8M0 scale goes to the
// layout-0 image [row/256][c/128][wr][fq][fr][ii] (see mmr_quantize_mxfp8).  valid masks the stores.
// E8M0 exponent of a 32-block from its max |value| (mmr_quantize_mxfp8's rule) and the e4m3 packing
__device__ __forceinline__ int q8_exp(float amax) {
  const uint32_t ab = __float_as_uint(amax);
  const int ex = (int)((ab >> 23) & 255) - 127 - 8 + ((ab & 0x7FFFFF) > 0x600000 ? 1 : 0);
  return ex < -127 ? -127 : (ex > 126 ? 126 : ex);
}
__device__ __forceinline__ float q8_inv(int ex) { return __uint_as_float((uint32_t)(127 - ex) << 23); }
__device__ __forceinline__ uint32_t q8_pack4(const float* v, float inv) {
  const uint32_t w = (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(v[0] * inv, v[1] * inv, 0, false);
  return (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(v[2] * inv, v[3] * inv, (int)w, true);
}
// byte offset of (row, 32-block of column col) in the layout-0 scale image of a c-column operand
__device__ __forceinline__ int64_t q8_soff(int64_t row, int col, int c) {
  const int kt = col / 128, fq = (col % 128) / 32;
  const int rr = (int)(row % 256), wr = rr / 128, ii = (rr % 128) / 16, fr = rr % 16;
  return ((row / 256) * (c / 128) + kt) * 1024 + ((wr * 4 + fq) * 16 + fr) * 8 + ii;
}

__device__ __forceinline__ void q8_chunk8(const float* vb, int64_t row, int ch, int c, uint8_t* q8,
                                          uint8_t* q8s, bool valid) {
  float amax = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(vb[j]));
  amax = fmaxf(amax, __shfl_xor(amax, 1, 64));
  amax = fmaxf(amax, __shfl_xor(amax, 2, 64));
  const int ex = q8_exp(amax);
  const float inv = q8_inv(ex);
  const uint32_t w0 = q8_pack4(vb, inv), w1 = q8_pack4(vb + 4, inv);
  if (valid) {
    *(uint2*)(q8 + row * c + ch * 8) = make_uint2(w0, w1);
    if ((ch & 3) == 0) q8s[q8_soff(row, ch * 8, c)] = (uint8_t)(ex + 127);
  }
}

// Fused-MLP weight images (swin_mlp.hip, x3_mlp.hip):
// physical 16-B unit of logical unit q in row r (conflict-free for the b128 lane groups; checked
// exhaustively for the 32x32x16 A-operand access pattern)
template <int U>
__host__ __device__ __forceinline__ int unit_swz(int r, int q) {
  if constexpr (U == 12) return (q + ((r >> 2) & 3)) % 12;
  else if constexpr (U == 4) return q ^ ((r >> 2) & 3);
  else return q ^ ((r >> 1) & 7);  // U = 8, 24
}

// W2 column order inside each 16-wide group: stored position 8h + j holds hidden
// 8(j>>2) + 4h + (j&3) — the order in which fc1's 32x32 C fragment leaves GELU'd values in lane
// half h, so one ds_read_b128 fetches the A fragment that matches the packed B fragment.
__host__ __device__ __forceinline__ int w2_hidden(int pos) {
  const int h = (pos >> 3) & 1, j = pos & 7;
  return (pos & ~15) + 8 * (j >> 2) + 4 * h + (j & 3);
}

}  // namespace mmr

#define MMR_CHECK_HIP(expr)                                                                \
  do {                                                                                     \
    hipError_t _e = (expr);                                                                \
    if (_e != hipSuccess) {                                                                \
      (void)hipGetLastError(); /* clear the sticky error: the next launch check is clean */ \
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
