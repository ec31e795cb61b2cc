// Brute-force batched cosine top-K over a row-major gallery (gfx950).
//
// Reference semantics (what this replaces): sklearn cosine_similarity(Q, G) + per-row
// np.argsort(sim[i])[::-1][:K]  — src/Evaluate/retrieval_overlap.py:84-90, same idiom in
// src/Retrieval/retrieval.py:128-137.  Here: exact cosine in f64, ties -> lower index.
//
// Pipeline per search (all on the caller's stream):
//   1. knn_prep_queries   q -> qn = q/|q| (f32, padded [Qp][Dp]) + |q| in f64.
//   (Q <= 32, mode x3)    skinny path instead of 2.: knn_scan_f32_gmax streams the tile16 copy of the
//                         gallery once on f32 MFMA (HBM-bound, ~5.3 TB/s at 100k x 768) into the
//                         same row-group maxima, then knn_select_groups with the f32-mode delta.
//   2. knn_scores_x3_gmax (default) S = (qn . g) / |g| as a bf16 "3-term split" MFMA GEMM: every
//                         operand is split into hi + lo bf16 (hi = bf16(x), lo = bf16(x - hi)) and
//                         s ~= q_hi.g_hi + q_hi.g_lo + q_lo.g_hi (dropped terms <= 3*2^-16 |q||g|),
//                         run as ONE K' = 3D GEMM on v_mfma_f32_16x16x32_bf16 (16x the f32 MFMA
//                         rate; 5.3x after the 3 terms).  Gallery stored [hi c | lo c] per
//                         64-wide chunk c (4 B/element, the f32 byte count); the k-tile 3c+2 re-reads
//                         hi c from L2.  Queries stored [hi c | hi c | lo c].  The epilogue keeps
//                         only the max of each lane's 4-row group per query (gmax, 1/4 of the
//                         score bytes; the score matrix is never written) and
//                         knn_select_groups re-scores every row of the groups whose max clears
//                         b - 2*delta (same bound, argued at the kernel).
//      knn_scores         (mode f32) S[Qp][Np] = (qn . g) * (1/|g|) with v_mfma_f32_32x32x2_f32 (exact f32
//                         products, f32 accumulate).  MFMA-bound for Q >~ 40, HBM-bound below.
//                         Wave tile 64 queries x 64 gallery rows (2x2 MFMA tiles, 64 acc regs);
//                         operands loaded straight to VGPRs as float4 with a k-permutation (lane
//                         half h owns k = kb+8h..kb+8h+7), which the dot product does not see.
//   3. knn_select         (mode f32) one 1024-thread workgroup per query: (A) per-thread max over a strided
//                         slice of the row; (B) b = K-th largest of the 1024 maxima (a lower bound
//                         of the K-th largest score); (C) collect every s >= b - 2*delta into LDS;
//                         (D) rare fallback: exact radix select over the row if (C) overflowed;
//                         (E) re-score candidates in f64 from the raw rows, rank by
//                         (score desc, index asc), write the top K.
//      delta bounds |s_approx - s_f64| (f32: (D+16) 2^-24; x3: (3D+16) 2^-24 + 4 2^-16), so every
//      true top-K row is a candidate:
//      the K rows with s32 >= t (t = K-th largest s32) all have s64 >= t - delta, hence the K-th
//      largest s64 is >= t - delta and any true top-K row has s32 >= t - 2 delta >= b - 2 delta.
#include <float.h>
#include <math.h>
#include <mutex>
#include <vector>

#include "common.h"

namespace mmr {
hipError_t knn_scan_p8(const uint16_t* qh, const uint16_t* gh, int K, int tiles_n, int64_t nval, float* gm,
                       int64_t ldG, float* bm, int64_t ldB, int unit_rows, hipStream_t st,
                       int tiles_m = 1, const float* rs = nullptr);  // gemm.hip
}

namespace {

using mmr::ceil_div;
using mmr::round_up;

constexpr int kSelThreads = 1024;
constexpr int kCandCap = 2048;
constexpr int kMaxK = 256;
constexpr int kRowPad = 256;  // gallery rows padded to this (covers every scores tile width)

typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ uint32_t f2key(float f) {
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key2f(uint32_t k) {
  uint32_t u = (k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k;
  return __uint_as_float(u);
}

// ------------------------------------------------------------------ gallery / query preparation
// One wave per row: copy into the padded layout, f64 norm, f32 inverse norm.
__global__ __launch_bounds__(256) void knn_prep_gallery(const float* __restrict__ src, int64_t n,
                                                        int d, float* __restrict__ dst, int Dp,
                                                        int64_t Np, float* __restrict__ inv_norm,
                                                        double* __restrict__ norm64) {
  int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  int lane = threadIdx.x & 63;
  if (row >= Np) return;
  double ss = 0.0;
  float* out = dst + row * Dp;
  if (row < n) {
    const float* in = src + row * (int64_t)d;
    for (int k = lane; k < Dp; k += 64) {
      float v = k < d ? in[k] : 0.0f;
      out[k] = v;
      ss += (double)v * (double)v;
    }
  } else {
    for (int k = lane; k < Dp; k += 64) out[k] = 0.0f;
  }
  ss = mmr::wave_sum(ss);
  if (lane == 0) {
    double nrm = sqrt(ss);
    norm64[row] = nrm;
    inv_norm[row] = nrm > 0.0 ? (float)(1.0 / nrm) : 0.0f;
  }
}

// MFMA-native 16-row tile layout of knn_scan_f32_gmax: element (row, k) of a [rows][Dp] matrix at
// ((row/16)*(Dp/16) + k/16)*256 + ((k%16)/4*16 + row%16)*4 + k%4 — lane l = 16h + r of a wave then
// reads rows r, floats 4h..4h+3 of a 16-float chunk as one contiguous 1-KB wave load.
__host__ __device__ __forceinline__ int64_t tile16_index(int64_t row, int k, int Dp) {
  return ((row >> 4) * (Dp >> 4) + (k >> 4)) * 256 + ((((k & 15) >> 2) << 4) + (row & 15)) * 4 + (k & 3);
}

// fp16 variant (skinny f16 scan): 16-row x 32-half pieces of 1 KB, lane l = 16h + r holding halfs
// 8h..8h+7 of row r (the v_mfma_f32_16x16x32_f16 operand layout):
// ((row/16)*(Dp/32) + k/32)*512 + ((k%32)/8*16 + row%16)*8 + k%8.
__host__ __device__ __forceinline__ int64_t tile32h_index(int64_t row, int k, int Dp) {
  return ((row >> 4) * (Dp >> 5) + (k >> 5)) * 512 + ((((k & 31) >> 3) << 4) + (row & 15)) * 8 + (k & 7);
}

// 4 fp16 (one 8-B load) -> float4 (exact)
__device__ __forceinline__ float4 h4_to_f4(uint2 u) {
  typedef _Float16 h4 __attribute__((ext_vector_type(4)));
  const h4 v = __builtin_bit_cast(h4, u);
  return make_float4((float)v[0], (float)v[1], (float)v[2], (float)v[3]);
}

// element (row, k) of the gallery as f64: the f32 rows, or the native fp16 index's raw tile32h rows
__device__ __forceinline__ double gal_elem(const float* gal, const uint16_t* galh, int64_t row, int k, int Dp) {
  if (galh) return (double)(float)__builtin_bit_cast(_Float16, galh[tile32h_index(row, k, Dp)]);
  return (double)gal[row * Dp + k];
}

// native fp16 gallery (mmr_index_create with MMR_F16): the raw rows [n][d] fp16 -> the tile32h image
// gh [Np][Dp] (zero padded; it is both the scan operand and the exact rows of the f64 re-score) + the
// f64 norms / f32 inverse norms of the f32-upcast values, summed in knn_prep_gallery's order (so an
// fp16 index and an f32 index of the upcast rows hold bit-identical norms).  One wave per row.
__global__ __launch_bounds__(256) void knn_prep_gallery_f16(const uint16_t* __restrict__ src, int64_t n, int d,
                                                            uint16_t* __restrict__ gh, int Dp, int64_t Np,
                                                            float* __restrict__ inv_norm, double* __restrict__ norm64) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= Np) return;
  double ss = 0.0;
  for (int k = lane; k < Dp; k += 64) {
    const uint16_t v = (row < n && k < d) ? src[row * (int64_t)d + k] : (uint16_t)0;
    gh[tile32h_index(row, k, Dp)] = v;
    const double x = (double)(float)__builtin_bit_cast(_Float16, v);
    ss += x * x;
  }
  ss = mmr::wave_sum(ss);
  if (lane == 0) {
    const double nrm = sqrt(ss);
    norm64[row] = nrm;
    inv_norm[row] = nrm > 0.0 ? (float)(1.0 / nrm) : 0.0f;
  }
}

// rows [row0, row0 + nrows) of a native fp16 index -> f32 [nrows][d] (the link graph's self-join queries)
__global__ __launch_bounds__(256) void knn_rows_from_f16(const uint16_t* __restrict__ gh, int64_t row0, int64_t nrows,
                                                         int d, int Dp, float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= nrows * d) return;
  const int64_t r = i / d;
  const int k = (int)(i % d);
  out[i] = (float)__builtin_bit_cast(_Float16, gh[tile32h_index(row0 + r, k, Dp)]);
}

__global__ __launch_bounds__(256) void knn_prep_queries(const float* __restrict__ q, int64_t nq,
                                                        int d, float* __restrict__ qn, int Dp,
                                                        int64_t Qp, double* __restrict__ qnorm64,
                                                        int tiled = 0) {
  int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  int lane = threadIdx.x & 63;
  if (row >= Qp) return;
  // tiled: 0 row-major f32, 1 tile16 f32, 2 tile32h fp16, 3 row-major fp16 (qn reinterpreted as halfs;
  // 3 needs Dp <= 1024)
  auto put = [&](int k, float v) {
    if (tiled == 2) ((_Float16*)qn)[tile32h_index(row, k, Dp)] = (_Float16)v;
    else if (tiled == 1) qn[tile16_index(row, k, Dp)] = v;
    else qn[row * Dp + k] = v;
  };
  if ((tiled == 2 || tiled == 3) && Dp <= 1024) {
    // fp16 tile32h: lane owns the 8-half groups g = lane + 64j (j < 2) of the row — 16-B stores
    // (one (row, 8-half) run is contiguous in tile32h) instead of 2-B scatters; loads unconditional
    typedef _Float16 h8 __attribute__((ext_vector_type(8)));
    const float* in = q + (row < nq ? row : 0) * (int64_t)d;
    float v[2][8];
    double ss = 0.0;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int k = 8 * (lane + 64 * j) + e;
        const float x = in[k < d ? k : d - 1];
        v[j][e] = (row < nq && k < d) ? x : 0.0f;
        ss += (double)v[j][e] * (double)v[j][e];
      }
    ss = mmr::wave_sum(ss);
    const double nrm = sqrt(ss);
    const float inv = nrm > 0.0 ? (float)(1.0 / nrm) : 0.0f;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int k0 = 8 * (lane + 64 * j);
      if (k0 >= Dp) continue;
      h8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = (_Float16)(v[j][e] * inv);
      *(h8*)((_Float16*)qn + (tiled == 2 ? tile32h_index(row, k0, Dp) : row * (int64_t)Dp + k0)) = o;
    }
    if (lane == 0) qnorm64[row] = row < nq ? nrm : 0.0;
    return;
  }
  if (row >= nq) {
    for (int k = lane; k < Dp; k += 64) put(k, 0.0f);
    return;
  }
  const float* in = q + row * (int64_t)d;
  double ss = 0.0;
  if (Dp <= 1024) {
    // all loads of the row issued together (a runtime-count loop waits for each load in turn)
    // unconditional loads (index clamped, value masked): a "load or zero" select makes hipcc branch
    // around each load and wait for it before the next, 16 serial round trips
    float v[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      const int k = lane + 64 * c;
      const float x = in[k < d ? k : d - 1];
      v[c] = k < d ? x : 0.0f;
    }
#pragma unroll
    for (int c = 0; c < 16; ++c) ss += (double)v[c] * (double)v[c];
    ss = mmr::wave_sum(ss);
    const double nrm = sqrt(ss);
    const float inv = nrm > 0.0 ? (float)(1.0 / nrm) : 0.0f;
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      const int k = lane + 64 * c;
      if (k < Dp) put(k, v[c] * inv);
    }
    if (lane == 0) qnorm64[row] = nrm;
    return;
  }
  for (int k = lane; k < d; k += 64) ss += (double)in[k] * (double)in[k];
  ss = mmr::wave_sum(ss);
  double nrm = sqrt(ss);
  float inv = nrm > 0.0 ? (float)(1.0 / nrm) : 0.0f;
  for (int k = lane; k < Dp; k += 64) put(k, k < d ? in[k] * inv : 0.0f);
  if (lane == 0) qnorm64[row] = nrm;
}

// ------------------------------------------------------------------ scores GEMM (f32 MFMA)
// Workgroup = 4 waves arranged WQ x WN; wave tile 64 x 64; workgroup tile (64WQ) x (64WN).
// Block id -> (gallery tile t, query block j) keeps all query blocks of one gallery tile on the
// same XCD (ids congruent mod 8) so the gallery rows are fetched from HBM once per XCD L2.
template <int WQ, int WN>
__global__ __launch_bounds__(256) void knn_scores(const float* __restrict__ qn,
                                                  const float* __restrict__ gal,
                                                  const float* __restrict__ inv_g,
                                                  float* __restrict__ scores, int Dp, int64_t ldS,
                                                  int n_gtiles, int n_qblocks) {
  const int b = blockIdx.x;
  const int per = 8 * n_qblocks;
  const int t = (b / per) * 8 + (b % 8);
  const int j = (b % per) / 8;
  if (t >= n_gtiles) return;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wq = wave / WN, wn = wave % WN;
  const int64_t q0 = (int64_t)j * (64 * WQ) + wq * 64;
  const int64_t g0 = (int64_t)t * (64 * WN) + wn * 64;
  const int r = lane & 31, h = lane >> 5;

  const float* pa0 = qn + (q0 + r) * Dp + 8 * h;
  const float* pa1 = pa0 + 32 * (int64_t)Dp;
  const float* pb0 = gal + (g0 + r) * Dp + 8 * h;
  const float* pb1 = pb0 + 32 * (int64_t)Dp;

  f32x16 c00 = {0}, c01 = {0}, c10 = {0}, c11 = {0};
  float4 a0l = *(const float4*)(pa0), a0h = *(const float4*)(pa0 + 4);
  float4 a1l = *(const float4*)(pa1), a1h = *(const float4*)(pa1 + 4);
  float4 b0l = *(const float4*)(pb0), b0h = *(const float4*)(pb0 + 4);
  float4 b1l = *(const float4*)(pb1), b1h = *(const float4*)(pb1 + 4);
  for (int kb = 0; kb < Dp; kb += 16) {
    float4 na0l, na0h, na1l, na1h, nb0l, nb0h, nb1l, nb1h;
    const bool more = kb + 16 < Dp;
    if (more) {
      na0l = *(const float4*)(pa0 + kb + 16); na0h = *(const float4*)(pa0 + kb + 20);
      na1l = *(const float4*)(pa1 + kb + 16); na1h = *(const float4*)(pa1 + kb + 20);
      nb0l = *(const float4*)(pb0 + kb + 16); nb0h = *(const float4*)(pb0 + kb + 20);
      nb1l = *(const float4*)(pb1 + kb + 16); nb1h = *(const float4*)(pb1 + kb + 20);
    }
    const float a0[8] = {a0l.x, a0l.y, a0l.z, a0l.w, a0h.x, a0h.y, a0h.z, a0h.w};
    const float a1[8] = {a1l.x, a1l.y, a1l.z, a1l.w, a1h.x, a1h.y, a1h.z, a1h.w};
    const float b0[8] = {b0l.x, b0l.y, b0l.z, b0l.w, b0h.x, b0h.y, b0h.z, b0h.w};
    const float b1[8] = {b1l.x, b1l.y, b1l.z, b1l.w, b1h.x, b1h.y, b1h.z, b1h.w};
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      c00 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[s], b0[s], c00, 0, 0, 0);
      c01 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[s], b1[s], c01, 0, 0, 0);
      c10 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[s], b0[s], c10, 0, 0, 0);
      c11 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[s], b1[s], c11, 0, 0, 0);
    }
    if (more) {
      a0l = na0l; a0h = na0h; a1l = na1l; a1h = na1h;
      b0l = nb0l; b0h = nb0h; b1l = nb1l; b1h = nb1h;
    }
  }
  // C[i][j]: j = lane&31 (gallery row), i = (reg&3) + 8*(reg>>2) + 4*(lane>>5) (query)
  const float ig0 = inv_g[g0 + r], ig1 = inv_g[g0 + 32 + r];
#pragma unroll
  for (int reg = 0; reg < 16; ++reg) {
    const int i = (reg & 3) + 8 * (reg >> 2) + 4 * h;
    float* s0 = scores + (q0 + i) * ldS + g0 + r;
    float* s1 = scores + (q0 + 32 + i) * ldS + g0 + r;
    s0[0] = c00[reg] * ig0;
    s0[32] = c01[reg] * ig1;
    s1[0] = c10[reg] * ig0;
    s1[32] = c11[reg] * ig1;
  }
}

// ------------------------------------------------------------------ bf16x3 split scores GEMM
typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;

__device__ __forceinline__ void split_bf16(float x, uint16_t& hi, uint16_t& lo) {
  hi = mmr::f2bf(x);
  lo = mmr::f2bf(x - mmr::bf2f(hi));
}

// gal f32 [Np][Dp] -> gs bf16 [Np][2Dp], chunk c (64 wide): [hi c | lo c]
__global__ __launch_bounds__(256) void knn_split_gallery(const float* __restrict__ gal, int Dp,
                                                         int64_t total, uint16_t* __restrict__ gs) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;  // element index in [Np][Dp]
  if (i >= total) return;
  const int64_t row = i / Dp;
  const int k = (int)(i % Dp);
  uint16_t hi, lo;
  split_bf16(gal[i], hi, lo);
  uint16_t* o = gs + row * 2 * Dp + (k / 64) * 128 + (k % 64);
  o[0] = hi;
  o[64] = lo;
}

// qn f32 [Qp][Dp] -> qs bf16 [Qp][3Dp], chunk c: [hi c | hi c | lo c]
__global__ __launch_bounds__(256) void knn_split_queries(const float* __restrict__ qn, int Dp,
                                                         int64_t total, uint16_t* __restrict__ qs) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int64_t row = i / Dp;
  const int k = (int)(i % Dp);
  uint16_t hi, lo;
  split_bf16(qn[i], hi, lo);
  uint16_t* o = qs + row * 3 * Dp + (k / 64) * 192 + (k % 64);
  o[0] = hi;
  o[64] = hi;
  o[128] = lo;
}

// gal f32 [Np][Dp] -> gt (tile16 layout), one thread per float4 of the output
__global__ __launch_bounds__(256) void knn_tile_gallery(const float* __restrict__ gal, int Dp,
                                                        int64_t total4, float* __restrict__ gt) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;  // float4 index in gt
  if (i >= total4) return;
  const int64_t piece = i >> 6;  // 1-KB piece = (16-row tile, 16-float chunk)
  const int l = (int)(i & 63), r = l & 15, h = l >> 4;
  const int64_t tile = piece / (Dp >> 4);
  const int c = (int)(piece % (Dp >> 4));
  const int64_t row = tile * 16 + r;
  ((float4*)gt)[i] = *(const float4*)(gal + row * Dp + c * 16 + 4 * h);
}

// gal f32 [Np][Dp] -> gh: fp16 of the unit rows g/|g| in the tile32h layout, one thread per 8 halfs
__global__ __launch_bounds__(256) void knn_tile_gallery_f16(const float* __restrict__ gal,
                                                            const float* __restrict__ inv_g, int Dp,
                                                            int64_t total8, uint16_t* __restrict__ gh) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;  // 16-B unit index in gh
  if (i >= total8) return;
  const int64_t piece = i >> 6;
  const int l = (int)(i & 63), r = l & 15, h = l >> 4;
  const int64_t tile = piece / (Dp >> 5);
  const int c = (int)(piece % (Dp >> 5));
  const int64_t row = tile * 16 + r;
  const float ig = inv_g[row];
  const float* src = gal + row * Dp + c * 32 + 8 * h;
  typedef _Float16 h8 __attribute__((ext_vector_type(8)));
  h8 v;
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = (_Float16)(src[e] * ig);
  ((h8*)gh)[i] = v;
}

__device__ __forceinline__ int xswz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

// S[m][n] = inv_g[n] * sum_k' Qs[m][k'] Gs'[n][k'] over K' = 3 Dp; tile 128 x 128 x 64, 4 waves
// (2x2) of 64x64, glds-staged double buffer with source-address swizzle (same structure as
// gemm.hip).  Rows of the query block past Qp / gallery past Np never exist (both padded).
// Gallery tiles outer, query tiles inner: the tiles_m query blocks of one gallery tile are
// consecutive in the remapped order and share the XCD (and its L2) -> gallery read once.
// Same GEMM, fused epilogue: instead of the (Qp x Np) score matrix, each lane keeps the max of its
// 4 gallery rows {B + fr + 16j : j < 4} (B = the wave's 64-row block) per query — a "row group" —
// and writes one float per (query, group): gmax[m][g], g = (B/64)*16 + fr, ldG = Np/4.  Rows >= n
// (padding) are -inf.  4x fewer bytes than the scores and no extra VALU beyond 3 max per value.
__global__ __launch_bounds__(256, 2) void knn_scores_x3_gmax(const uint16_t* __restrict__ qs,
                                                              const uint16_t* __restrict__ gs,
                                                              const float* __restrict__ inv_g,
                                                              float* __restrict__ gmax, int Dp,
                                                              int64_t ldG, int64_t n, int tiles_m,
                                                              int tiles_n) {
  constexpr int BK = 64, TILE = 128 * 64;
  __shared__ __attribute__((aligned(16))) uint16_t lds[2 * 2 * TILE];
  const int nwg = tiles_m * tiles_n;
  const int orig = blockIdx.x;
  const int q8 = nwg / 8, r8 = nwg % 8, xcd = orig % 8;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
  const int tn = wg / tiles_m, tm = wg % tiles_m;
  const int64_t m0 = (int64_t)tm * 128, n0 = (int64_t)tn * 128;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int K3 = 3 * Dp;
  const int prow_in = lane >> 3, pch = lane & 7;
  const uint16_t* srcA[4];
  const uint16_t* srcB[4];
  int lchk[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int row = wave * 32 + j * 8 + prow_in;
    lchk[j] = xswz(row, pch) * 8;
    srcA[j] = qs + (m0 + row) * K3;
    srcB[j] = gs + (n0 + row) * 2 * Dp;
  }
  auto stage = [&](int sbuf, int t) {
    const int c = t / 3, part = t % 3;
    const int ka = t * BK;
    const int kb = c * 128 + (part == 1 ? 64 : 0);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      uint16_t* la = lds + (sbuf * 2 + 0) * TILE + (wave * 32 + j * 8) * BK;
      uint16_t* lb = lds + (sbuf * 2 + 1) * TILE + (wave * 32 + j * 8) * BK;
      __builtin_amdgcn_global_load_lds((const void*)(srcA[j] + ka + lchk[j]), (lds_ptr_t)la, 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(srcB[j] + kb + lchk[j]), (lds_ptr_t)lb, 16, 0, 0);
    }
  };
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const int nk = K3 / BK;
  const int fr = lane & 15, fq = lane >> 4;
  stage(0, 0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int sb = kt & 1;
    if (kt + 1 < nk) stage(sb ^ 1, kt + 1);
    const uint16_t* la = lds + (sb * 2 + 0) * TILE;
    const uint16_t* lb = lds + (sb * 2 + 1) * TILE;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 a[4], b[4];
      const int ch = ks * 4 + fq;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int rowa = wm * 64 + i * 16 + fr;
        const int rowb = wn * 64 + i * 16 + fr;
        a[i] = *(const bf16x8*)(la + rowa * BK + xswz(rowa, ch) * 8);
        b[i] = *(const bf16x8*)(lb + rowb * BK + xswz(rowb, ch) * 8);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }
  // C[row][col]: col = lane&15 (gallery row), row = 4*(lane>>4) + reg (query)
  float ig[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t g = n0 + wn * 64 + j * 16 + fr;
    ig[j] = g < n ? inv_g[g] : 0.f;
    if (g >= n) ig[j] = -INFINITY;  // marks padding rows (never a candidate)
  }
  const int64_t gcol = (n0 + wn * 64) / 64 * 16 + fr;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int rg = 0; rg < 4; ++rg) {
      float mx = -INFINITY;
#pragma unroll
      for (int j = 0; j < 4; ++j) mx = fmaxf(mx, ig[j] == -INFINITY ? -INFINITY : acc[i][j][rg] * ig[j]);
      const int64_t m = m0 + wm * 64 + i * 16 + fq * 4 + rg;
      gmax[m * ldG + gcol] = mx;
    }
  }
}

// ------------------------------------------------------------------ fp16 scan (mode f16)
// The gallery scanned as fp16 unit rows (gh = fp16(g/|g|), 2 B per element: half the bytes of every
// f32 copy) against fp16 unit queries on v_mfma_f32_16x16x32_f16 (exact products, f32 accumulate);
// the f64 re-score from the raw f32 rows (knn_select_groups) keeps the result exact, with the
// candidate margin 2*delta_f16 (delta_f16 argued at mmr_index_search).  Same streaming structure as
// knn_scan_f32_gmax: one wave per 64-row block, lane l = 16h + r on row r of each 16-row tile, every
// wave load one contiguous 1-KB tile32h piece; QT query tiles of 16 from L2 (16*QT <= 256 queries per
// pass, so the gallery is read from HBM once per 256 queries).  At QT = 16 the accumulators (256 f32)
// sit in AGPRs.
// Measured and dropped (MI355X, 100k x 768, 256 queries): splitting the query tiles over 2 or 4 waves
// of one workgroup on the same 64-row block (more waves in flight, the block's gallery pieces re-read
// from L2 by the sibling waves) — 4 waves x 4 tiles 102 us vs 68 us for one wave x 16 tiles.
//
// RAW (Q <= 32, d % 8 == 0, 16-B aligned rows): no query-prep launch — lane (h, r) reads k = 8h..8h+7 of
// each 32-k piece of query row 16t + r straight from the caller's f32 rows (4 lanes = one 128-B line),
// one chunk ahead like the gallery, and converts them to fp16 at the MFMA: the scores are q . g^ for
// the UNNORMALISED query (|q| times the cosine; the order within a query is the same).  The selection
// then uses the per-query margin 2 (|q| delta_rel + delta_abs) (argued at mmr_index_search), and takes
// the exact path over every row if a component of q does not fit fp16.
// Block maxima: besides the per-(query, unit) maxima, each (query, 64-row block) max goes to bmax —
// the selection reads these 1/16-size rows first and touches unit maxima only inside blocks that can
// hold a top-K row.
template <int QT, int KC, int WQ = 1, bool RAW = false>
__global__ __launch_bounds__(64 * WQ) void knn_scan_f16_gmax(const uint16_t* __restrict__ qh,
                                                        const float* __restrict__ qraw, int64_t nq, int d,
                                                        const uint16_t* __restrict__ gh,
                                                        float* __restrict__ gmax, float* __restrict__ bmax,
                                                        int Dp, int64_t ldG, int64_t ldB, int64_t n,
                                                        const float* __restrict__ rs = nullptr) {
  typedef _Float16 h8 __attribute__((ext_vector_type(8)));
  constexpr int L = KC / 32;  // 1-KB pieces per tile per chunk
  static_assert(!RAW || WQ == 1, "raw queries: one wave per block");
  const int lane = threadIdx.x & 63, wq = threadIdx.x >> 6;
  const int64_t blk = blockIdx.x;
  const int r = lane & 15, h = lane >> 4;
  const int64_t g0 = blk * 64;
  const int64_t tileB = 16 * (int64_t)Dp;  // halfs per 16-row tile
  const uint16_t* pb = gh + g0 * Dp + 8 * lane;
  const uint16_t* pa = qh + (int64_t)wq * QT * tileB + 8 * lane;
  // RAW query rows: clamped row pointer + row mask per query tile
  constexpr int QR = RAW ? QT : 1;
  const float* qrow[QR];
  bool qok[QR];
  if constexpr (RAW) {
#pragma unroll
    for (int t = 0; t < QT; ++t) {
      const int64_t row = 16 * t + r;
      qok[t] = row < nq;
      qrow[t] = qraw + (qok[t] ? row : nq - 1) * (int64_t)d;
    }
  }
  // raw: the 8 floats k0..k0+7 (k0 = chunk + 32e + 8h; d % 8 == 0, so a group is all in or all out)
  auto qload = [&](int t, int k0, float4 (&x)[2]) {
    const int kk = k0 < d ? k0 : d - 8;  // unconditional load, value masked at the conversion
    x[0] = *(const float4*)(qrow[t] + kk);
    x[1] = *(const float4*)(qrow[t] + kk + 4);
  };
  auto qcvt = [&](int t, int k0, const float4 (&x)[2]) -> h8 {
    const bool ok = qok[t] && k0 < d;
    h8 o;
    o[0] = (_Float16)x[0].x; o[1] = (_Float16)x[0].y; o[2] = (_Float16)x[0].z; o[3] = (_Float16)x[0].w;
    o[4] = (_Float16)x[1].x; o[5] = (_Float16)x[1].y; o[6] = (_Float16)x[1].z; o[7] = (_Float16)x[1].w;
    return ok ? o : (h8){0, 0, 0, 0, 0, 0, 0, 0};
  };
  f32x4 acc[QT][4];
#pragma unroll
  for (int t = 0; t < QT; ++t)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[t][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  constexpr int LA = RAW ? 1 : L, LR = RAW ? L : 1;
  f32x4 b[4][L], a[QT][LA];
  float4 ra[QT][LR][2];
#pragma unroll
  for (int e = 0; e < L; ++e) {
#pragma unroll
    for (int t = 0; t < QT; ++t) {
      if constexpr (RAW) qload(t, 32 * e + 8 * h, ra[t][e]);
      else a[t][e] = *(const f32x4*)(pa + t * tileB + 512 * e);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) b[j][e] = __builtin_nontemporal_load((const f32x4*)(pb + j * tileB + 512 * e));
  }
  auto mma = [&](int kc) {
#pragma unroll
    for (int e = 0; e < L; ++e)
#pragma unroll
      for (int t = 0; t < QT; ++t) {
        h8 av;
        if constexpr (RAW) av = qcvt(t, kc + 32 * e + 8 * h, ra[t][e]);
        else av = __builtin_bit_cast(h8, a[t][e]);
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[t][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(av, __builtin_bit_cast(h8, b[j][e]), acc[t][j], 0, 0, 0);
      }
  };
  // both operands of the NEXT chunk are issued before this chunk's MFMAs (queries first: vmcnt
  // retires in issue order); the current ones were issued one iteration earlier.  The last chunk is
  // peeled (no loads: an unconditional re-read of itself cost ~1/7 more load instructions at Dp = 768).
  int kc = 0;
#pragma unroll 1
  for (; kc + KC < Dp; kc += KC) {
    const int kn = kc + KC;
    f32x4 na[QT][LA], nb[4][L];
    float4 nra[QT][LR][2];
#pragma unroll
    for (int e = 0; e < L; ++e)
#pragma unroll
      for (int t = 0; t < QT; ++t) {
        if constexpr (RAW) qload(t, kn + 32 * e + 8 * h, nra[t][e]);
        else na[t][e] = *(const f32x4*)(pa + t * tileB + 16 * kn + 512 * e);
      }
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < L; ++e)
        nb[j][e] = __builtin_nontemporal_load((const f32x4*)(pb + j * tileB + 16 * kn + 512 * e));
    __builtin_amdgcn_sched_barrier(0);
    mma(kc);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int e = 0; e < L; ++e) {
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j][e] = nb[j][e];
#pragma unroll
      for (int t = 0; t < QT; ++t) {
        if constexpr (RAW) {
          ra[t][e][0] = nra[t][e][0];
          ra[t][e][1] = nra[t][e][1];
        } else {
          a[t][e] = na[t][e];
        }
      }
    }
  }
  mma(kc);
  const int64_t gcol = blk * 16 + r;
  bool pad[4];
  float rsv[4];  // raw-row (native fp16) gallery: 1 / |g| per row, else 1
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    pad[j] = g0 + 16 * j + r >= n;
    rsv[j] = rs ? rs[g0 + 16 * j + r] : 1.f;
  }
#pragma unroll
  for (int t = 0; t < QT; ++t)
#pragma unroll
    for (int rg = 0; rg < 4; ++rg) {
      float mx = -INFINITY;
#pragma unroll
      for (int j = 0; j < 4; ++j) mx = fmaxf(mx, pad[j] ? -INFINITY : acc[t][j][rg] * rsv[j]);
      const int64_t qrw = 16 * (wq * QT + t) + 4 * h + rg;
      gmax[qrw * ldG + gcol] = mx;
      // block max over the 16 lanes of this h (rows r of the block's 4 tiles)
      float bm = mx;
      bm = mmr::row16_max(bm);
      if (r == 0) bmax[qrw * ldB + blk] = bm;
    }
}

// LQ (Q <= 32, raw queries, d % 8 == 0): the knn_scan_f16_gmax<RAW> stream with the query operand
// converted ONCE per workgroup into LDS (tile32h fp16 pieces, the MFMA operand layout) instead of once
// per 64-row block from the caller's f32 rows in L2: a block then moves its 96 KB of gallery and no
// query bytes through the CU's load path (RAW: + 48 KB of f32 queries per block at QT = 1).
// Persistent: workgroup w owns the 64-row blocks [nblk*w/G, nblk*(w+1)/G) (one workgroup per CU),
// its NWV waves take them round-robin; same unit / block maxima as knn_scan_f16_gmax<RAW>.
template <int QT, int KC, int NWV>
__global__ __launch_bounds__(64 * NWV) void knn_scan_f16_lq(const float* __restrict__ qraw, int64_t nq, int d,
                                                          const uint16_t* __restrict__ gh,
                                                          float* __restrict__ gmax, float* __restrict__ bmax,
                                                          int Dp, int64_t ldG, int64_t ldB, int64_t n, int64_t nblk,
                                                          double* __restrict__ qpre, const float* __restrict__ rs) {
  typedef _Float16 h8 __attribute__((ext_vector_type(8)));
  constexpr int L = KC / 32;  // 1-KB pieces per tile per chunk
  extern __shared__ __attribute__((aligned(16))) uint16_t qs[];  // [QT][Dp/32][512] halfs
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int KP = Dp / 32;
  {
    // |q| (f64, the select's canonical order: lane sums elements lane + 64c, c < 16, then the xor
    // tree — bit-identical to knn_select_t's own query_norm) and max |q_k| per query, for the select:
    // row r by the LAST wave of workgroup r, which takes a gallery block only when its workgroup has
    // more than NWV - 1 of them (100k rows: 6-7 per workgroup) — workgroup 0's waves computing every
    // row first delayed its blocks, the scan's tail
    for (int row = blockIdx.x; wave == NWV - 1 && row < nq; row += gridDim.x) {
      double ss = 0.0;
      float am = 0.f;
      float xv[16];  // every load issued before any use (clamped index, masked value: a "load if in
                     // range" compiles into a branch and a wait per load)
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        const int e = lane + 64 * c;
        xv[c] = qraw[(int64_t)row * d + (e < d ? e : d - 1)];
      }
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        const float x = lane + 64 * c < d ? xv[c] : 0.f;
        ss += (double)x * (double)x;
        am = fmaxf(am, fabsf(x));
      }
      ss = mmr::wave_sum(ss);
      am = mmr::wave_max(am);
      if (lane == 0) {
        qpre[2 * row] = sqrt(ss);
        qpre[2 * row + 1] = (double)am;
      }
    }
  }
  // (1) queries -> fp16 tile32h in LDS: one (row, 8-k group) per item, 16-B store; rows >= nq and
  //     k >= d are zero (unconditional clamped loads, masked at the conversion)
  const int groups = QT * 16 * (Dp / 8);
  for (int gi = tid; gi < groups; gi += 64 * NWV) {
    const int row = gi / (Dp / 8), k0 = (gi % (Dp / 8)) * 8;
    const bool ok = row < nq && k0 < d;
    const float* src = qraw + (int64_t)(row < nq ? row : nq - 1) * d + (k0 < d ? k0 : d - 8);
    const float4 x0 = *(const float4*)src, x1 = *(const float4*)(src + 4);
    h8 o;
    o[0] = (_Float16)x0.x; o[1] = (_Float16)x0.y; o[2] = (_Float16)x0.z; o[3] = (_Float16)x0.w;
    o[4] = (_Float16)x1.x; o[5] = (_Float16)x1.y; o[6] = (_Float16)x1.z; o[7] = (_Float16)x1.w;
    *(h8*)(qs + tile32h_index(row, k0, Dp)) = ok ? o : (h8){0, 0, 0, 0, 0, 0, 0, 0};
  }
  __syncthreads();
  const int r = lane & 15, h = lane >> 4;
  const int64_t tileB = 16 * (int64_t)Dp;  // halfs per 16-row tile
  const int64_t b_lo = nblk * blockIdx.x / gridDim.x, b_hi = nblk * (blockIdx.x + 1) / gridDim.x;
  const char* qbase = (const char*)qs + lane * 16;
  for (int64_t blk = b_lo + wave; blk < b_hi; blk += NWV) {
    const int64_t g0 = blk * 64;
    const uint16_t* pb = gh + g0 * Dp + 8 * lane;
    f32x4 acc[QT][4];
#pragma unroll
    for (int t = 0; t < QT; ++t)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[t][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    f32x4 b[4][L];
#pragma unroll
    for (int e = 0; e < L; ++e)
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j][e] = __builtin_nontemporal_load((const f32x4*)(pb + j * tileB + 512 * e));
    auto mma = [&](int kc) {
#pragma unroll
      for (int e = 0; e < L; ++e)
#pragma unroll
        for (int t = 0; t < QT; ++t) {
          const h8 av = *(const h8*)(qbase + ((int64_t)t * KP + kc / 32 + e) * 1024);
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[t][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(av, __builtin_bit_cast(h8, b[j][e]), acc[t][j], 0, 0, 0);
        }
    };
    // the next chunk's gallery pieces are issued before this chunk's MFMAs; the last chunk is peeled
    // (no loads: an unconditional re-read of itself cost ~1/7 more load instructions at Dp = 768)
    int kc = 0;
#pragma unroll 1
    for (; kc + KC < Dp; kc += KC) {
      f32x4 nb[4][L];
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int e = 0; e < L; ++e)
          nb[j][e] = __builtin_nontemporal_load((const f32x4*)(pb + j * tileB + 16 * (kc + KC) + 512 * e));
      __builtin_amdgcn_sched_barrier(0);
      mma(kc);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int e = 0; e < L; ++e)
#pragma unroll
        for (int j = 0; j < 4; ++j) b[j][e] = nb[j][e];
    }
    mma(kc);
    const int64_t gcol = blk * 16 + r;
    bool pad[4];
    float rsv[4];  // raw-row (native fp16) gallery: 1 / |g| per row, else 1
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      pad[j] = g0 + 16 * j + r >= n;
      rsv[j] = rs ? rs[g0 + 16 * j + r] : 1.f;
    }
#pragma unroll
    for (int t = 0; t < QT; ++t)
#pragma unroll
      for (int rg = 0; rg < 4; ++rg) {
        float mx = -INFINITY;
#pragma unroll
        for (int j = 0; j < 4; ++j) mx = fmaxf(mx, pad[j] ? -INFINITY : acc[t][j][rg] * rsv[j]);
        const int64_t qrw = 16 * t + 4 * h + rg;
        gmax[qrw * ldG + gcol] = mx;
        float bm = mx;
        bm = mmr::row16_max(bm);
        if (r == 0) bmax[qrw * ldB + blk] = bm;
      }
  }
}

// ------------------------------------------------------------------ fp16 tile scan (mode f16, Q > 32)
// The same fp16 product as knn_scan_f16_gmax, as an LDS-staged MFMA GEMM for query passes of 64-256
// queries.  Workgroup tile: RT = WR*MR gallery row tiles (16 rows each) x QT = WQ*MQ query tiles, one
// 32-deep k-piece per slice; wave (wq, wr) computes MQ query tiles x MR row tiles.  Every operand is
// a tile32h 1-KB piece (16 rows x 32 halfs, lane l holding 8 halfs of row l&15 — the
// v_mfma_f32_16x16x32_f16 operand layout), so each piece lands in LDS by ONE global_load_lds
// (lane-linear, no swizzle) and each fragment read is one conflict-free ds_read_b128.
// The gallery is the A operand and the queries the B operand, so a lane's 4 accumulators are 4
// CONSECUTIVE gallery rows of one query: the epilogue keeps their max (a contiguous 4-row unit,
// knn_select_t<2>), one float per (query, 4 rows).
// Schedule: an LDS ring of STAGES slices filled by glds (a wave issues either gallery or query pieces,
// PW per slice); at each step the wave waits for the slice it needs next (own vmcnt, then one barrier
// for every wave's pieces), refills the ring slot freed by the previous step and runs its MFMAs.  PF:
// the fragments of slice s+1 are read during slice s's MFMAs (one fewer ring slot in flight).
// Per-slice bookkeeping is incremental (uniform slice cursors, per-lane piece offsets computed once
// per tile, a constant vmcnt in steady state): a first version computed tile / slice / ring indices by
// division and 64-bit address math per piece per slice, and its instruction issue (SQ_ACTIVE_INST_ANY)
// was 3-6x its MFMA time.
// Persistent: workgroup w owns the 16-row tiles [n_rt*w/G, n_rt*(w+1)/G) (balanced to one row tile),
// walked in tiles of RT row tiles; the ring runs across tile boundaries, so the next tile's slices
// load under the epilogue.  In the last (partial) tile, row tiles past the range are clamped to its
// last one (valid memory, results discarded) and a wave whose row tiles are all past it skips its MFMAs.
// Epilogue: a 4x4 lane transpose (lanes qc + 16h x 4 row tiles) turns each lane's maxima of units
// {4i + h} into 4 consecutive units, one 16-B store per (query tile, 4 row tiles): NST stores per wave
// per tile, counted out of the next step's vmcnt wait instead of drained.
template <int WQ, int MQ, int WR, int MR, bool PF>
struct F16TileCfg {
  static constexpr int NW = WQ * WR;             // waves
  static constexpr int RT = WR * MR;             // gallery row tiles per tile
  static constexpr int QT = WQ * MQ;             // query tiles
  static constexpr int P = RT + QT;              // 1-KB pieces per slice
  static constexpr int PW = P / NW;              // glds per wave per slice
  static constexpr int SLICE_B = P * 1024;
  static constexpr int STAGES = 163840 / SLICE_B > 8 ? 8 : 163840 / SLICE_B;
  static constexpr int AHEAD = STAGES - (PF ? 3 : 2);  // slices in flight beyond the one waited for
  static constexpr int NST = 2 * (MQ * MR / 4);  // epilogue stores per wave per tile (unit + block maxima)
  static_assert(P % NW == 0 && MR % 4 == 0, "tile shape");
  static_assert(AHEAD >= 1 && PW * AHEAD + NST <= 63, "ring depth / vmcnt range");
};

__device__ __forceinline__ void wait_vm(int n) {
  // s_waitcnt vmcnt(n) for a wave-uniform runtime n in [0, 63] (rare path: the end of the stream)
  switch (n) {
#define MMR_VM(N) case N: __builtin_amdgcn_s_waitcnt(((N) & 15) | (7 << 4) | (15 << 8) | (((N) >> 4) << 14)); break;
    MMR_VM(0) MMR_VM(1) MMR_VM(2) MMR_VM(3) MMR_VM(4) MMR_VM(5) MMR_VM(6) MMR_VM(7) MMR_VM(8) MMR_VM(9)
    MMR_VM(10) MMR_VM(11) MMR_VM(12) MMR_VM(13) MMR_VM(14) MMR_VM(15) MMR_VM(16) MMR_VM(17) MMR_VM(18)
    MMR_VM(19) MMR_VM(20) MMR_VM(21) MMR_VM(22) MMR_VM(23) MMR_VM(24) MMR_VM(25) MMR_VM(26) MMR_VM(27)
    MMR_VM(28) MMR_VM(29) MMR_VM(30) MMR_VM(31) MMR_VM(32) MMR_VM(33) MMR_VM(34) MMR_VM(35) MMR_VM(36)
    MMR_VM(37) MMR_VM(38) MMR_VM(39) MMR_VM(40) MMR_VM(41) MMR_VM(42) MMR_VM(43) MMR_VM(44) MMR_VM(45)
    MMR_VM(46) MMR_VM(47) MMR_VM(48) MMR_VM(49) MMR_VM(50) MMR_VM(51) MMR_VM(52) MMR_VM(53) MMR_VM(54)
    MMR_VM(55) MMR_VM(56) MMR_VM(57) MMR_VM(58) MMR_VM(59) MMR_VM(60) MMR_VM(61) MMR_VM(62)
#undef MMR_VM
    default: break;
  }
}
template <int N>
__device__ __forceinline__ void wait_vm_c() {
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

// v[h] of lane (qc + 16c) -> out[c] of lane (qc + 16h): the 4x4 transpose of the epilogue
__device__ __forceinline__ f32x4 transpose4(const float (&v)[4], int h, int qc) {
  f32x4 out;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int give = (h - r) & 3, from = (h + r) & 3;  // this lane provides v[give], receives from lane `from`
    const float send = give == 0 ? v[0] : give == 1 ? v[1] : give == 2 ? v[2] : v[3];
    const float got = __shfl(send, qc + 16 * from, 64);
    if (from == 0) out[0] = got;
    else if (from == 1) out[1] = got;
    else if (from == 2) out[2] = got;
    else out[3] = got;
  }
  return out;
}

template <int WQ, int MQ, int WR, int MR, bool PF>
__global__ __launch_bounds__(64 * WQ * WR) void knn_scan_f16_tile(const uint16_t* __restrict__ qh,
                                                                  const uint16_t* __restrict__ gh,
                                                                  float* __restrict__ gmax, float* __restrict__ bmax,
                                                                  int Dp, int64_t ldG, int64_t ldB, int64_t n,
                                                                  int64_t n_rt, const float* __restrict__ rs) {
  using C = F16TileCfg<WQ, MQ, WR, MR, PF>;
  typedef _Float16 h8 __attribute__((ext_vector_type(8)));
  extern __shared__ __attribute__((aligned(16))) uint16_t dsm[];  // [STAGES][P][512] halfs
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave / WQ, wq = wave % WQ;
  // ranges of whole 64-row blocks (4 row tiles; n_rt % 4 == 0), so every block max is one lane group's
  const int64_t nb4 = n_rt / 4;
  const int64_t lo = 4 * (nb4 * blockIdx.x / gridDim.x), hi = 4 * (nb4 * (blockIdx.x + 1) / gridDim.x);
  if (lo >= hi) return;
  const int KP = Dp / 32;                          // k-pieces = slices per tile
  const int ntiles = (int)((hi - lo + C::RT - 1) / C::RT);
  const int64_t tile_b = (int64_t)KP * 1024;       // bytes of one 16-row tile (all k-pieces)
  // this wave's glds pieces p0 .. p0+PW-1: gallery row tiles (p < RT), then query tiles
  const int p0 = wave * C::PW;
  uint32_t off[C::PW];  // per-lane byte offsets of the pieces inside the current tile's k-piece 0
  auto set_offsets = [&](int64_t rt0) {
    const int valid = (int)(hi - rt0 < C::RT ? hi - rt0 : C::RT);  // row tiles of this tile in range
#pragma unroll
    for (int i = 0; i < C::PW; ++i) {
      const int p = p0 + i;
      const int piece = p < C::RT ? (p < valid ? p : valid - 1) : p - C::RT;
      off[i] = (uint32_t)(piece * tile_b) + lane * 16;
    }
  };
  // issue cursor: the next slice to load (uniform bases of its gallery and query pieces)
  int ic_tile = 0, ic_kp = 0, ic_stage = 0;
  const char* ic_gbase = (const char*)gh + lo * tile_b;
  const char* ic_qbase = (const char*)qh;
  set_offsets(lo);
  auto issue_next = [&]() {
    if (ic_tile >= ntiles) return;
    char* dst = (char*)dsm + ic_stage * C::SLICE_B + p0 * 1024;
#pragma unroll
    for (int i = 0; i < C::PW; ++i)
      __builtin_amdgcn_global_load_lds((const void*)((p0 + i < C::RT ? ic_gbase : ic_qbase) + off[i]),
                                       (lds_ptr_t)(dst + i * 1024), 16, 0, 0);
    ic_stage = ic_stage + 1 == C::STAGES ? 0 : ic_stage + 1;
    ic_gbase += 1024;
    ic_qbase += 1024;
    if (++ic_kp == KP) {
      ic_kp = 0;
      ++ic_tile;
      const int64_t rt0 = lo + (int64_t)C::RT * ic_tile;
      ic_gbase = (const char*)gh + rt0 * tile_b;
      ic_qbase = (const char*)qh;
      if (ic_tile < ntiles) set_offsets(rt0);
    }
  };
  const uint32_t lane_b = lane * 16;
  auto frag = [&](int stage, int piece) {
    return *(const h8*)((const char*)dsm + stage * C::SLICE_B + piece * 1024 + lane_b);
  };
  // wait until this wave's pieces of the slice `ahead_of` slices before the cursor end landed
  int waited = 0;  // slices whose pieces this wave has waited for
  bool stores_out = false;
  auto wait_slice = [&]() {
    const int issued_after = (ic_tile * KP + ic_kp) - (waited + 1);  // slices issued after the awaited one
    if (issued_after == C::AHEAD) {
      if (stores_out) wait_vm_c<C::PW * C::AHEAD + C::NST>();
      else wait_vm_c<C::PW * C::AHEAD>();
    } else {
      wait_vm(C::PW * issued_after + (stores_out ? C::NST : 0));
    }
    stores_out = false;
    ++waited;
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave's pieces landed; every wave is past the previous step
    asm volatile("" ::: "memory");
  };
  h8 fa[MR], fb0[MQ], fb1[MQ];
  f32x4 acc[MQ][MR];
  // prologue: STAGES-1 slices in flight
#pragma unroll
  for (int p = 0; p < C::STAGES - 1; ++p) issue_next();
  int stage = 0;  // ring slot of the slice being computed
  if constexpr (PF) {
    wait_slice();  // slice 0
#pragma unroll
    for (int i = 0; i < MR; ++i) fa[i] = frag(0, wr * MR + i);
#pragma unroll
    for (int t = 0; t < MQ; ++t) fb0[t] = frag(0, C::RT + wq * MQ + t);
  }
  // one step: slice (tile, kp) in ring slot `stage`; with PF its fragments are in (fa, fb) and the
  // next slice's are read into (fa, nb)
  auto step = [&](int tile, int kp, int64_t rt0, bool active, h8 (&fb)[MQ], h8 (&nb)[MQ]) {
    const bool more = tile + 1 < ntiles || kp + 1 < KP;
    if (PF) {
      if (more) wait_slice();  // slice s+1 (for the fragment prefetch)
    } else {
      wait_slice();            // slice s
    }
    issue_next();  // into the slot the previous step used
    const int nstage = stage + 1 == C::STAGES ? 0 : stage + 1;
    if (active) {
      if (!PF) {
#pragma unroll
        for (int i = 0; i < MR; ++i) fa[i] = frag(stage, wr * MR + i);
#pragma unroll
        for (int t = 0; t < MQ; ++t) fb[t] = frag(stage, C::RT + wq * MQ + t);
      }
#pragma unroll
      for (int i = 0; i < MR; ++i) {
#pragma unroll
        for (int t = 0; t < MQ; ++t) acc[t][i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[i], fb[t], acc[t][i], 0, 0, 0);
        if (PF && more) {
          fa[i] = frag(nstage, wr * MR + i);
#pragma unroll
          for (int t = i * MQ / MR; t < (i + 1) * MQ / MR; ++t) nb[t] = frag(nstage, C::RT + wq * MQ + t);
        }
      }
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this step's fragment reads returned
    stage = nstage;
    if (kp == KP - 1 && active) {
      // epilogue: lane (query tile t, query qc, rows 16 rt + 4h .. +3) -> unit max; 4x4 lane transpose
      // -> 4 consecutive units per lane -> one 16-B store per (t, block of 4 row tiles)
      const int h = lane >> 4, qc = lane & 15;
#pragma unroll
      for (int t = 0; t < MQ; ++t) {
        float* orow = gmax + (int64_t)(16 * (wq * MQ + t) + qc) * ldG;
#pragma unroll
        for (int b4 = 0; b4 < MR / 4; ++b4) {
          const int64_t rtb = rt0 + wr * MR + 4 * b4;
          float v[4];
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const int64_t r0 = (rtb + c) * 16 + 4 * h;
            const int64_t rc = r0 < 16 * n_rt ? r0 : 16 * n_rt - 4;  // past-range row tiles: clamped (discarded)
            const f32x4 rv = rs ? *(const f32x4*)(rs + rc) : (f32x4){1.f, 1.f, 1.f, 1.f};
            float mx = -INFINITY;
#pragma unroll
            for (int rg = 0; rg < 4; ++rg) mx = fmaxf(mx, r0 + rg < n ? acc[t][4 * b4 + c][rg] * rv[rg] : -INFINITY);
            v[c] = mx;
          }
          const f32x4 o = transpose4(v, h, qc);
          if (rtb + h < hi) *(f32x4*)(orow + (rtb + h) * 4) = o;
          // block max of rows 16 rtb .. +63 (rtb % 4 == 0): this lane's 4 units, then over h
          float bm = fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3]));
          bm = fmaxf(bm, __shfl_xor(bm, 16, 64));
          bm = fmaxf(bm, __shfl_xor(bm, 32, 64));
          if (h == 0 && rtb < hi) bmax[(int64_t)(16 * (wq * MQ + t) + qc) * ldB + rtb / 4] = bm;
        }
      }
      stores_out = tile + 1 < ntiles;
    }
  };
  for (int tile = 0; tile < ntiles; ++tile) {
    const int64_t rt0 = lo + (int64_t)C::RT * tile;
    const bool active = rt0 + wr * MR < hi;  // wave-uniform: some of this wave's row tiles are real
#pragma unroll
    for (int t = 0; t < MQ; ++t)
#pragma unroll
      for (int i = 0; i < MR; ++i) acc[t][i] = (f32x4){0.f, 0.f, 0.f, 0.f};
    for (int kp = 0; kp < KP; kp += 2) {
      step(tile, kp, rt0, active, fb0, fb1);
      if (kp + 1 < KP) step(tile, kp + 1, rt0, active, fb1, fb0);
    }
    if (KP & 1) {  // odd slice count: the next tile starts with the sets swapped — keep fb0 current
#pragma unroll
      for (int t = 0; t < MQ; ++t) fb0[t] = fb1[t];
    }
  }
  __builtin_amdgcn_s_waitcnt(0 | (7 << 4) | (15 << 8));  // vmcnt(0): no LDS-DMA may land after the workgroup retires
}

// ------------------------------------------------------------------ skinny-Q scan (f32 MFMA)
// Few queries (Q <= 16*QT, QT <= 4): the gallery read (N*Dp*4 B) is the whole cost, so the scan is a
// streaming kernel — every gallery byte from HBM exactly once, no LDS, no barriers — on exact-product
// v_mfma_f32_16x16x4_f32 (f32 accumulate: the f32-mode delta applies).  One wave per 64-row block
// (the gmax group format of knn_scores_x3_gmax, so knn_select_groups consumes it unchanged): lane
// l = 16h + r owns row r of each of the 4 16-row tiles.  Gallery and queries are read from the
// tile16 copies (tile16_index): load e of a KC-wide chunk gives lane l floats kc + 16e + 4h .. +3 of
// its row, and the 64 lanes' float4 are one contiguous 1-KB piece — full-line, one-pass-per-16-lanes
// loads straight into the MFMA operand layout (a row-major read would touch 16 rows per 16 lanes).
// The MFMA k index of product (e, s) is kc + 16e + 4h + s for both operands (a permutation the dot
// product does not see).  Queries (<= 196 KB, L2-resident) are loaded before the next chunk's gallery
// loads: one chunk in flight while the current one is multiplied (sched_barrier keeps the order).
template <int QT, int KC>
__global__ __launch_bounds__(64) void knn_scan_f32_gmax(const float* __restrict__ qt16,
                                                        const float* __restrict__ gt,
                                                        const float* __restrict__ inv_g,
                                                        float* __restrict__ gmax, int Dp, int64_t ldG,
                                                        int64_t n) {
  constexpr int L = KC / 16;  // 1-KB pieces per tile per chunk
  const int lane = threadIdx.x;
  const int64_t blk = blockIdx.x;
  const int r = lane & 15, h = lane >> 4;
  const int64_t g0 = blk * 64;
  const int64_t tileB = 16 * (int64_t)Dp;  // floats per 16-row tile
  const float* pb = gt + g0 * Dp + 4 * lane;
  const float* pa = qt16 + 4 * lane;
  f32x4 acc[QT][4];
#pragma unroll
  for (int t = 0; t < QT; ++t)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[t][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  f32x4 b[4][L];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int e = 0; e < L; ++e) b[j][e] = __builtin_nontemporal_load((const f32x4*)(pb + j * tileB + 256 * e));
  // queries first: vmcnt retires loads in issue order, so loads issued after the next chunk's
  // gallery loads would make the MFMAs below wait for that chunk too
  auto qload = [&](int kc, f32x4 (&a)[QT][L]) {
#pragma unroll
    for (int t = 0; t < QT; ++t)
#pragma unroll
      for (int e = 0; e < L; ++e) a[t][e] = *(const f32x4*)(pa + t * tileB + 16 * kc + 256 * e);
  };
  auto mma = [&](const f32x4 (&a)[QT][L]) {
#pragma unroll
    for (int e = 0; e < L; ++e) {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
#pragma unroll
        for (int t = 0; t < QT; ++t) {
          const float av = a[t][e][s];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float bv = b[j][e][s];
            acc[t][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[t][j], 0, 0, 0);
          }
        }
      }
    }
  };
  // the next chunk's gallery pieces are issued ahead of this chunk's MFMAs; the last chunk is peeled
  // (no gallery loads: an unconditional re-read of itself cost extra load instructions per chunk)
  int kc = 0;
  for (; kc + KC < Dp; kc += KC) {
    f32x4 a[QT][L];
    qload(kc, a);
    f32x4 nb[4][L];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < L; ++e)
        nb[j][e] = __builtin_nontemporal_load((const f32x4*)(pb + j * tileB + 16 * (kc + KC) + 256 * e));
    __builtin_amdgcn_sched_barrier(0);  // keep the whole next chunk issued ahead of the MFMAs
    mma(a);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < L; ++e) b[j][e] = nb[j][e];
  }
  {
    f32x4 a[QT][L];
    qload(kc, a);
    mma(a);
  }
  // C[i][c]: c = lane&15 (gallery row r of tile j), i = 4h + reg (query of tile t)
  float ig[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t g = g0 + 16 * j + r;
    ig[j] = g < n ? inv_g[g] : -INFINITY;  // -inf marks padding rows (never a candidate)
  }
  const int64_t gcol = blk * 16 + r;
#pragma unroll
  for (int t = 0; t < QT; ++t)
#pragma unroll
    for (int rg = 0; rg < 4; ++rg) {
      float mx = -INFINITY;
#pragma unroll
      for (int j = 0; j < 4; ++j) mx = fmaxf(mx, ig[j] == -INFINITY ? -INFINITY : acc[t][j][rg] * ig[j]);
      gmax[(int64_t)(16 * t + 4 * h + rg) * ldG + gcol] = mx;
    }
}

// ------------------------------------------------------------------ per-query selection
// Digit pick of one radix pass, by wave 0: the largest digit dg whose bins [dg..255] hold >= krem
// keys, and the rank left inside that bin.  Lane l owns bins 4l..4l+3; a suffix sum over the
// lanes (shuffles) replaces a 256-step serial walk of the histogram.
__device__ __forceinline__ void pick_digit(const uint32_t* hist, uint32_t krem, uint32_t prefix, int shift,
                                           uint32_t* bcast) {
  if (threadIdx.x >= 64) return;
  const int l = threadIdx.x;
  const uint32_t h0 = hist[4 * l], h1 = hist[4 * l + 1], h2 = hist[4 * l + 2], h3 = hist[4 * l + 3];
  const uint32_t own = h0 + h1 + h2 + h3;
  uint32_t suf = own;  // inclusive suffix sum over lanes >= l
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t v = __shfl_down(suf, o, 64);
    if (l + o < 64) suf += v;
  }
  const uint32_t above = suf - own;  // keys in bins of higher lanes
  const uint32_t total = __shfl(suf, 0, 64);
  if (krem > total) {  // fewer keys than the rank asked for: digit 0 (as a full downward walk ends)
    if (l == 0) {
      bcast[0] = prefix;
      bcast[1] = krem - (total - h0);
    }
    return;
  }
  if (above < krem && krem <= suf) {  // exactly one lane
    uint32_t acc = above;
    int dg = 4 * l + 3;
    const uint32_t hb[4] = {h0, h1, h2, h3};
    for (int e = 3; e > 0; --e) {
      if (acc + hb[e] >= krem) break;
      acc += hb[e];
      dg = 4 * l + e - 1;
    }
    bcast[0] = prefix | ((uint32_t)dg << shift);
    bcast[1] = krem - acc;
  }
}

// Block-wide radix select: the kth (1-based) largest key among keys[0..m) (LDS).  All threads
// return the same key.  hist: 256-entry LDS scratch.
// passes < 4: only the top 8*passes bits are resolved and the smallest key with that prefix is
// returned — a lower bound of the kth key (all a threshold needs), one radix pass (~1 us) less each.
__device__ uint32_t block_select_kth(const uint32_t* keys, int m, int kth, uint32_t* hist,
                                     uint32_t* bcast, int passes = 4) {
  uint32_t prefix = 0, pmask = 0;
  uint32_t krem = (uint32_t)kth;
  for (int pass = 0; pass < passes; ++pass) {
    const int shift = 24 - 8 * pass;
    for (int i = threadIdx.x; i < 256; i += blockDim.x) hist[i] = 0;
    __syncthreads();
    for (int i = threadIdx.x; i < m; i += blockDim.x) {
      uint32_t key = keys[i];
      if ((key & pmask) == prefix) atomicAdd(&hist[(key >> shift) & 255u], 1u);
    }
    __syncthreads();
    pick_digit(hist, krem, prefix, shift, bcast);
    __syncthreads();
    prefix = bcast[0];
    krem = bcast[1];
    pmask |= 0xFFu << shift;
    __syncthreads();
  }
  return prefix;
}

// Same over a global row (fallback path, all N elements each pass).
__device__ uint32_t row_select_kth(const float* row, int64_t n, int kth, uint32_t* hist,
                                   uint32_t* bcast) {
  uint32_t prefix = 0, pmask = 0;
  uint32_t krem = (uint32_t)kth;
  for (int pass = 0; pass < 4; ++pass) {
    const int shift = 24 - 8 * pass;
    for (int i = threadIdx.x; i < 256; i += blockDim.x) hist[i] = 0;
    __syncthreads();
    for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
      uint32_t key = f2key(row[i]);
      if ((key & pmask) == prefix) atomicAdd(&hist[(key >> shift) & 255u], 1u);
    }
    __syncthreads();
    pick_digit(hist, krem, prefix, shift, bcast);
    __syncthreads();
    prefix = bcast[0];
    krem = bcast[1];
    pmask |= 0xFFu << shift;
    __syncthreads();
  }
  return prefix;
}

__device__ __forceinline__ float lower_threshold(float t, float two_delta) {
  double thr_d = (double)t - (double)two_delta;
  float thr = (float)thr_d;
  if ((double)thr > thr_d) thr = nextafterf(thr, -INFINITY);
  return thr;
}

// Per-query selection, one 1024-thread workgroup per query, over the scan's per-query value row.
// Units (what one value covers): MODE 0 = one gallery row (f32-mode score matrix, knn_scores);
// MODE 1 = a strided 4-row group {(u>>4)*64 + (u&15) + 16m : m < 4} (the gmax of knn_scores_x3_gmax /
// knn_scan_f32_gmax / knn_scan_f16_gmax: one lane's 4 rows of a 64-row block); MODE 2 = 4 consecutive
// rows {4u + m} (knn_scan_f16_tile); MODE 3 = 2 consecutive rows {2u + m} (the 8-phase GEMM scan,
// gemm_bf16_tn_p8<KNN>: half the rows to re-score per candidate unit).  A unit's value is >= the approximate score of each of its rows.
// (A) per-thread max over a strided slice; (B) b = a lower bound of the K-th largest unit value (each
// unit value is a distinct row's score, so b <= t, the K-th largest approximate row score); (C)
// collect every unit with value >= b - 2 delta: a true top-K row j has s(j) >= t - 2 delta >= b - 2
// delta, and its unit's value >= s(j); (D) more than kCandCap/GS units: the exact K-th largest unit
// value replaces b (same argument) and the set is rebuilt; still more (massive near-ties): the units
// are processed in position order, kCandCap/GS at a time, each batch re-scored and merged into a
// carried exact top-K — slower, never inexact, so the status output is always 0; (E) every row of
// the collected units is re-scored in f64 from the raw rows and (F) ranked by (score desc, index asc).
constexpr int kSlotCap = kMaxK + kCandCap;  // [0, kMaxK): carried top-K; [kMaxK, +kCandCap): one batch

// Phase clock of block 0 (tools/select_trace.hip builds this file with MMR_SELECT_TRACE; off in libmmr)
#ifdef MMR_SELECT_TRACE
__device__ long long g_sel_trace[24];
#define SEL_MARK(i) \
  if (blockIdx.x == 0 && threadIdx.x == 0) g_sel_trace[i] = wall_clock64();
#define SEL_VAL(i, v) \
  if (blockIdx.x == 0 && threadIdx.x == 0) g_sel_trace[i] = (long long)(v);
#else
#define SEL_MARK(i)
#define SEL_VAL(i, v)
#endif

template <int MODE>
__device__ __forceinline__ int64_t unit_row(int64_t u, int m) {
  if (MODE == 0) return u;
  if (MODE == 1) return (u >> 4) * 64 + (u & 15) + 16 * m;
  if (MODE == 3) return 2 * u + m;
  return 4 * u + m;
}

constexpr int kBlkCap = 1024;
// the select's first bound from per-wave top-4 keys (K <= 32; else the 2-pass radix)
__device__ __forceinline__ constexpr bool top4_bound_enabled() { return true; }

template <int T>
struct SelLds {
  float qrow[1024];  // raw query row (d <= 1024), first member: 16-B aligned
  uint32_t tmax[T];
  uint32_t hist[256];
  uint32_t bcast[4];
  int cand_b[kBlkCap];   // coarse pass: collected blocks (also the compaction buffer of the tightening)
  uint32_t ukey[kCandCap];  // keys of the collected units' values (tightening)
  int cand_u[kCandCap];
  double cand_d[kSlotCap];
  int rank_s[kSlotCap];
  int row_s[kSlotCap];
  double tmp_d[kMaxK];
  int tmp_r[kMaxK];
  double qn;
  float qmax;
};

// one 8-bit radix pass over the block's 1024 keys on the digit just below their common prefix
// (from the block max / min): the smallest key of the digit bin holding the kth largest key — a
// lower bound of it, resolved to 2^-8 of the keys' spread (a fixed top-down radix spends its first
// passes on bits every key shares, with all 1024 LDS atomics on one bin)
// PASSES = 2: a second 8-bit pass inside the chosen bin (2^-16 of the spread) — needed when the keys
// span several binary exponents (unnormalised RAW scores: one pass then resolves only to the exponent)
template <int T, int PASSES = 1>
__device__ uint32_t block_kth_lower(uint32_t key, int kth, uint32_t* hist, uint32_t* bcast) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  uint32_t mx = key, mn = key;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    mx = max(mx, (uint32_t)__shfl_xor((int)mx, o, 64));
    mn = min(mn, (uint32_t)__shfl_xor((int)mn, o, 64));
  }
  if (lane == 0) {
    hist[wave] = mx;
    hist[32 + wave] = mn;
  }
  __syncthreads();
  if (tid < 64) {
    const int nw = T / 64;
    uint32_t a = lane < nw ? hist[lane] : 0u, b = lane < nw ? hist[32 + lane] : 0xFFFFFFFFu;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      a = max(a, (uint32_t)__shfl_xor((int)a, o, 64));
      b = min(b, (uint32_t)__shfl_xor((int)b, o, 64));
    }
    if (lane == 0) {
      bcast[0] = a;
      bcast[1] = b;
    }
  }
  __syncthreads();
  const uint32_t kmax = bcast[0], diff = kmax ^ bcast[1];
  __syncthreads();
  if (diff == 0) return kmax;  // all keys equal (uniform)
  const int p = 31 - __builtin_clz(diff);
  const int shift = p > 7 ? p - 7 : 0;
  const uint32_t prefix = shift + 8 >= 32 ? 0u : kmax & ~((1u << (shift + 8)) - 1u);
  for (int i = tid; i < 256; i += T) hist[i] = 0;
  __syncthreads();
  atomicAdd(&hist[(key >> shift) & 255u], 1u);
  __syncthreads();
  pick_digit(hist, (uint32_t)kth, prefix, shift, bcast);
  __syncthreads();
  uint32_t r = bcast[0];
  if (PASSES > 1 && shift >= 8) {
    const uint32_t krem = bcast[1];
    const int shift2 = shift - 8;
    __syncthreads();
    for (int i = tid; i < 256; i += T) hist[i] = 0;
    __syncthreads();
    if ((key >> shift) == (r >> shift)) atomicAdd(&hist[(key >> shift2) & 255u], 1u);
    __syncthreads();
    pick_digit(hist, krem, r, shift2, bcast);
    __syncthreads();
    r = bcast[0];
  }
  __syncthreads();
  return r;
}

// Lower bound of the kth largest of the block's keys (kth <= 4 * waves) without a radix pass: each
// wave's 4 largest keys (4 distinct threads: lanes removed one at a time), then the kth largest of
// those 4 * T/64 values — kth values from distinct threads, so kth distinct rows score at least it.
// Usually the kth largest overall (a wave holds > 4 of the top keys rarely); ~0.4 us against the
// 2-pass radix's ~2.7 (select phase clock, Q = 16).
template <int T>
__device__ uint32_t block_kth_lower_top4(uint32_t key, int kth, uint32_t* vals, uint32_t* bcast) {
  constexpr int NV = 4 * (T / 64);
  static_assert(NV <= 64, "one wave ranks the candidates");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  uint32_t v = key;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    // wave max: DPP within each 16-lane row, then the four rows' lanes 0 / 16 / 32 / 48 read into
    // scalars (a 6-level shuffle butterfly paid 6 LDS round trips per round: 24 per call)
    uint32_t mx = v;
    mx = max(mx, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)mx, 0xB1, 0xF, 0xF, false));
    mx = max(mx, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)mx, 0x4E, 0xF, 0xF, false));
    mx = max(mx, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)mx, 0x141, 0xF, 0xF, false));
    mx = max(mx, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)mx, 0x140, 0xF, 0xF, false));
    mx = max(max((uint32_t)__builtin_amdgcn_readlane((int)mx, 0), (uint32_t)__builtin_amdgcn_readlane((int)mx, 16)),
             max((uint32_t)__builtin_amdgcn_readlane((int)mx, 32), (uint32_t)__builtin_amdgcn_readlane((int)mx, 48)));
    const uint64_t hit = __ballot(v == mx);
    if (lane == (int)__builtin_ctzll(hit)) v = 0u;  // key 0 sorts below every float key
    if (lane == 0) vals[wave * 4 + j] = mx;
  }
  __syncthreads();
  // every wave ranks the NV candidates itself from LDS broadcast reads (one wave ranking them by lane
  // swaps, then two more barriers to broadcast its pick, cost ~0.5 us of the phase)
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  const uint32_t mine = lane < NV ? vals[lane] : 0u;
  int rank = 0;  // values ahead of mine (larger, or equal at a lower position)
#pragma unroll
  for (int j4 = 0; j4 < NV / 4; ++j4) {
    const u32x4 o4 = *(const u32x4*)(vals + 4 * j4);
#pragma unroll
    for (int e = 0; e < 4; ++e) rank += (o4[e] > mine) || (o4[e] == mine && 4 * j4 + e < lane);
  }
  // ranks are a permutation of 0 .. NV-1 and kth <= NV: exactly one lane holds the kth largest
  const uint64_t hit = __ballot(lane < NV && rank == kth - 1);
  (void)bcast;
  return (uint32_t)__builtin_amdgcn_readlane((int)mine, (int)__builtin_ctzll(hit));
}

// COARSE (MODE 1 / 2: 16 units = one 64-row block; MODE 3: 32): the scan also wrote per-(query, block) maxima
// bvals; (A)-(C) run on those first — the K-th largest thread max over block maxima is a lower bound
// b of t (each block max is a distinct row's score), and only blocks whose max clears b - 2 delta have
// their 16 unit maxima read; when more units than 2K + 32 qualify, the K-th largest of THEIR values
// (again a distinct-row bound, >= b) tightens the threshold before the re-score.
// RAW: the scan scored the unnormalised query (knn_scan_f16_gmax<RAW>): the margin is per query,
// two_delta * |q| + two_delta_abs, |q| computed first (wave 0, canonical order); a query with a
// component outside fp16 range takes the exact every-row path; |q| = 0 scores every row 0 (rows
// 0..K-1).
template <int MODE, int NC, int T, bool COARSE = false, bool RAW = false>
__global__ __launch_bounds__(T) void knn_select_t(
    const float* __restrict__ vals, int64_t ldV, int64_t nunits, int64_t n, int k, float two_delta,
    const float* __restrict__ bvals, int64_t ldB, float two_delta_abs,
    const float* __restrict__ q_raw, int d, const double* __restrict__ qnorm64,
    const float* __restrict__ gal, int Dp, const double* __restrict__ gnorm64, int64_t idx_base,
    const uint16_t* __restrict__ galh,
    int64_t* __restrict__ out_idx, float* __restrict__ out_score, double* __restrict__ out_score64,
    int32_t* __restrict__ status, const double* __restrict__ qpre = nullptr) {
  constexpr int GS = MODE == 0 ? 1 : MODE == 3 ? 2 : 4;  // rows per unit
  constexpr int UPB = 64 / GS;               // units per 64-row block (COARSE)
  constexpr int UC = kCandCap / GS;          // units per batch
  __shared__ __attribute__((aligned(16))) SelLds<T> L;

  SEL_MARK(0)
  const int64_t qi = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (SGPR)
  const float* row = vals + qi * ldV;
  const int kk = (int)(n < (int64_t)k ? n : (int64_t)k);
  int64_t* oi = out_idx + qi * k;
  float* os = out_score ? out_score + qi * k : nullptr;
  double* os64 = out_score64 ? out_score64 + qi * k : nullptr;
  (void)qnorm64;
  for (int r = kk + tid; r < k; r += T) {
    oi[r] = -1;
    if (os) os[r] = -INFINITY;
    if (os64) os64[r] = -INFINITY;
  }
  if (tid == 0 && status) status[qi] = 0;
  if (kk <= 0) return;
  // the raw query row (f64 re-score, phase E) is staged in LDS first: its latency hides under
  // phases A-D and it holds no registers meanwhile
  const float* qr = q_raw + qi * (int64_t)d;
  if (NC > 0) {
    for (int e = tid; e < 1024; e += T) {
      const float x = qr[e < d ? e : d - 1];  // unconditional load (see knn_prep_queries)
      L.qrow[e] = e < d ? x : 0.f;
    }
  }
  const int64_t n4 = nunits >> 2;
  // the first kRegF4 float4 of each thread's strided slice stay in registers for (C): one HBM/L2
  // round trip for rows up to kRegF4 * 4 * 1024 = 32k units, all loads issued together
  constexpr int kRegF4 = COARSE ? 1 : 8;
  float4 cache[kRegF4];
  float m = -INFINITY;
  // COARSE: the block maxima (nunits / 16 per query; the first kRegB per thread kept for (C))
  constexpr int kRegB = 4;
  const int64_t nblk = nunits / UPB;
  const float* brow = COARSE ? bvals + qi * ldB : nullptr;
  float bc[kRegB];
  if constexpr (COARSE) {
#pragma unroll
    for (int it = 0; it < kRegB; ++it) {
      const int64_t i = tid + (int64_t)it * T;
      const float v = brow[i < nblk ? i : (nblk > 0 ? nblk - 1 : 0)];
      bc[it] = i < nblk ? v : -INFINITY;
    }
#pragma unroll
    for (int it = 0; it < kRegB; ++it) m = fmaxf(m, bc[it]);
    for (int64_t i = tid + (int64_t)kRegB * T; i < nblk; i += T) m = fmaxf(m, brow[i]);
  } else {
#pragma unroll
    for (int it = 0; it < kRegF4; ++it) {
      // unconditional loads (clamped index, masked value): see knn_prep_queries
      const int64_t i = tid + (int64_t)it * T;
      const float4 v = ((const float4*)row)[i < n4 ? i : (n4 > 0 ? n4 - 1 : 0)];
      cache[it] = i < n4 ? v : make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
    }
#pragma unroll
    for (int it = 0; it < kRegF4; ++it)
      m = fmaxf(m, fmaxf(fmaxf(cache[it].x, cache[it].y), fmaxf(cache[it].z, cache[it].w)));
    for (int64_t i = tid + (int64_t)kRegF4 * T; i < n4; i += T) {
      const float4 v = ((const float4*)row)[i];
      m = fmaxf(m, fmaxf(fmaxf(v.x, v.y), fmaxf(v.z, v.w)));
    }
    for (int64_t i = (n4 << 2) + tid; i < nunits; i += T) m = fmaxf(m, row[i]);
  }
  if (tid == 0) {
    L.bcast[2] = 0;
    L.bcast[3] = 0;
  }
  // |q| in f64 in the gallery norms' order (knn_prep_gallery: lane sums elements lane + 64c over c,
  // then the xor tree), so a query equal to a gallery row scores exactly 1 whatever the scan path;
  // RAW also needs max |q_k| (fp16 range of the scan's operand)
  double qn = 0.0;
  auto query_norm = [&]() {
    if (wave == 0) {
      double ss = 0.0;
      float am = 0.f;
      if constexpr (NC > 0) {
        for (int e = lane; e < 1024; e += 64) {
          const float x = L.qrow[e];
          ss += (double)x * (double)x;
          am = fmaxf(am, fabsf(x));
        }
      } else {
        for (int e = lane; e < Dp; e += 64) {
          const float x = e < d ? qr[e] : 0.f;
          ss += (double)x * (double)x;
          am = fmaxf(am, fabsf(x));
        }
      }
      ss = mmr::wave_sum(ss);
      if (RAW) am = mmr::wave_max(am);
      if (lane == 0) {
        L.qn = sqrt(ss);
        L.qmax = am;
      }
    }
  };
  if (RAW) {
    if (qpre != nullptr) {  // computed by the scan (knn_scan_f16_lq), same order and bits
      if (tid == 0) {
        L.qn = qpre[2 * qi];
        L.qmax = (float)qpre[2 * qi + 1];
      }
    } else {
      __syncthreads();  // qrow staged
      query_norm();
    }
    // L.qn / L.qmax visible after the first bound's first barrier
  }
  SEL_MARK(1)
  // (B) lower bound of the K-th largest thread max, clamped to -inf's key (smaller keys are NaNs)
  uint32_t bkey = COARSE && kk <= 4 * (T / 64) && top4_bound_enabled()
                      ? block_kth_lower_top4<T>(f2key(m), kk, L.tmax, L.bcast)
                      : block_kth_lower<T, COARSE ? 2 : 1>(f2key(m), kk, L.hist, L.bcast);
  if (bkey < f2key(-INFINITY)) bkey = f2key(-INFINITY);
  float tdel = two_delta;
  bool take_all = false;  // RAW, q outside fp16 range: every unit is a candidate (exact, slow)
  if (RAW) {
    const double qn0 = L.qn;
    if (qn0 == 0.0) {
      // s(q, g) = 0 for every row: rows 0 .. kk-1 (ties by lower index)
      for (int r = tid; r < kk; r += T) {
        oi[r] = (int64_t)r + idx_base;
        if (os) os[r] = 0.f;
        if (os64) os64[r] = 0.0;
      }
      return;
    }
    const double td = (double)two_delta * qn0 + (double)two_delta_abs;
    tdel = (float)td;
    if ((double)tdel < td) tdel = nextafterf(tdel, INFINITY);
    take_all = !(L.qmax < 32768.f);
  }
  float thr = take_all ? -INFINITY : lower_threshold(key2f(bkey), tdel);
  SEL_MARK(2)
  auto take = [&](int64_t u, float v, float th) {
    if (take_all || (v >= th && v > -INFINITY)) {
      const uint32_t p = atomicAdd(&L.bcast[2], 1u);
      if (p < (uint32_t)UC) {
        L.cand_u[p] = (int)u;
        L.ukey[p] = f2key(v);
      }
    }
  };
  // collect the units of [lo, hi) (float4-aligned lo) with value >= th into cand_u; returns the count
  auto collect = [&](float th, bool cached, int64_t lo, int64_t hi) -> int {
    const int64_t h4 = hi >> 2;
    if (cached) {
#pragma unroll
      for (int it = 0; it < kRegF4; ++it) {
        const int64_t i = tid + (int64_t)it * T;
        take(4 * i, cache[it].x, th);
        take(4 * i + 1, cache[it].y, th);
        take(4 * i + 2, cache[it].z, th);
        take(4 * i + 3, cache[it].w, th);
      }
    }
    for (int64_t i = (lo >> 2) + tid + (cached ? (int64_t)kRegF4 * T : 0); i < h4; i += T) {
      const float4 v = ((const float4*)row)[i];
      take(4 * i, v.x, th);
      take(4 * i + 1, v.y, th);
      take(4 * i + 2, v.z, th);
      take(4 * i + 3, v.w, th);
    }
    for (int64_t i = (h4 << 2 > lo ? h4 << 2 : lo) + tid; i < hi; i += T) take(i, row[i], th);
    __syncthreads();
    const int c = (int)L.bcast[2];
    __syncthreads();
    if (tid == 0) L.bcast[2] = 0;
    __syncthreads();  // reset visible before any thread's next take()
    return c;
  };
  // (E) re-score the rows of cnt collected units in f64 into slots [kMaxK, ...)
  auto rescore = [&](int cnt) -> int {
    const int nslot = GS * cnt;
    for (int s = tid; s < nslot; s += T) {
      const int64_t g = unit_row<MODE>(L.cand_u[s / GS], s % GS);
      L.row_s[kMaxK + s] = (int)(g < n ? g : n);
    }
    // the loads below compute their rows from cand_u themselves (row_s is for the rank, behind the
    // caller's barrier); only a non-RAW selection waits here, for wave 0's |q|
    if (!RAW) __syncthreads();
    qn = L.qn;
    SEL_MARK(8)
    if constexpr (NC > 0) {
      // latency-bound: each wave issues the float4 loads of its RB rows (NC 256-float chunks each)
      // before reducing any of them, so up to 16*RB rows (48 at Dp = 768: a usual 11-unit candidate
      // set) take one round trip; the query row from LDS (lane owns elements 4(64c + lane) .. +3)
      // (1024 threads; a 256-thread variant with 8-12 rows per wave: 2x slower); 512 threads: 8 rows at NC 3
      // (64 rows, a usual 13-unit candidate set, in one round trip)
      constexpr int RB = T >= 1024 ? (NC <= 2 ? 4 : NC == 3 ? 3 : 2) : (NC <= 2 ? 8 : NC == 3 ? 8 : 6);
      for (int s0 = wave * RB; s0 < nslot; s0 += (T / 64) * RB) {
        float4 gv[RB][NC];
        double gnr[RB];  // row norms loaded with the rows (not after the reduction: one round trip)
        int64_t gir[RB];
        // every load unconditional (a "load or zero" select makes hipcc branch around each load and
        // wait for it before the next — 9 serial round trips, measured 5 us of the 12 us select):
        // padding slots read row 0 (score discarded), lanes past Dp re-read the row's last float4
        // (their query elements in LDS are 0, so the product is 0)
        if (galh) {  // native fp16 gallery: the raw rows from the tile32h image (4 halfs = 8 B per load)
#pragma unroll
          for (int r = 0; r < RB; ++r) {
            const int s = s0 + r;
            const int64_t gu = s < nslot ? unit_row<MODE>(L.cand_u[s / GS], s % GS) : n;
            const int64_t gi = gu < n ? gu : n;
            gir[r] = gi;
            const int64_t gl = gi < n ? gi : 0;
            gnr[r] = gnorm64[gl];
#pragma unroll
            for (int c = 0; c < NC; ++c) {
              const int e = c * 256 + lane * 4;
              gv[r][c] = h4_to_f4(*(const uint2*)(galh + tile32h_index(gl, e < Dp ? e : Dp - 4, Dp)));
            }
          }
        } else {
#pragma unroll
          for (int r = 0; r < RB; ++r) {
            const int s = s0 + r;
            const int64_t gu = s < nslot ? unit_row<MODE>(L.cand_u[s / GS], s % GS) : n;
            const int64_t gi = gu < n ? gu : n;
            gir[r] = gi;
            const int64_t gl = gi < n ? gi : 0;
            gnr[r] = gnorm64[gl];
            const float* gr = gal + gl * Dp;
#pragma unroll
            for (int c = 0; c < NC; ++c) {
              const int e = c * 256 + lane * 4;
              gv[r][c] = *(const float4*)(gr + (e < Dp ? e : Dp - 4));
            }
          }
        }
        double part[RB];
#pragma unroll
        for (int r = 0; r < RB; ++r) {
          double acc = 0.0;
#pragma unroll
          for (int c = 0; c < NC; ++c) {
            const float4 qv = *(const float4*)(L.qrow + (c * 64 + lane) * 4);
            acc += (double)qv.x * gv[r][c].x + (double)qv.y * gv[r][c].y + (double)qv.z * gv[r][c].z +
                   (double)qv.w * gv[r][c].w;
          }
          part[r] = acc;
        }
        // the RB rows' wave sums together (bit-identical to one wave_sum per row, which paid RB x 6
        // dependent LDS round trips after the fetch)
        int rr;
        const double acc = mmr::rows_wave_sum<RB>(part, lane, rr);
        constexpr int LOG = RB > 4 ? 3 : RB > 2 ? 2 : RB > 1 ? 1 : 0;
        if ((lane & ((64 >> LOG) - 1)) == 0 && rr < RB && s0 + rr < nslot) {
          double gn = gnr[0];
          int64_t gi = gir[0];
#pragma unroll
          for (int r = 1; r < RB; ++r)
            if (rr == r) {
              gn = gnr[r];
              gi = gir[r];
            }
          L.cand_d[kMaxK + s0 + rr] = gi >= n ? -INFINITY : ((qn > 0.0 && gn > 0.0) ? acc / (qn * gn) : 0.0);
        }
      }
    } else {
      for (int s = wave; s < nslot; s += T / 64) {
        const int64_t gu = unit_row<MODE>(L.cand_u[s / GS], s % GS);
        const int64_t gi = gu < n ? gu : n;
        double sc = -INFINITY;
        if (gi < n) {
          double acc = 0.0;
          for (int kq = lane; kq < d; kq += 64) acc += (double)qr[kq] * gal_elem(gal, galh, gi, kq, Dp);
          acc = mmr::wave_sum(acc);
          const double gn = gnorm64[gi];
          sc = (qn > 0.0 && gn > 0.0) ? acc / (qn * gn) : 0.0;
        }
        if (lane == 0) L.cand_d[kMaxK + s] = sc;
      }
    }
    SEL_MARK(9)
    return nslot;
  };
  // (F) rank the carried rows [0, carry) with the re-scored slots [kMaxK, +nslot): a thread per slot
  // counts the slots ahead of it (score desc, row asc) in a register, every thread reading the same
  // other slot at each step (LDS broadcast); `direct` writes the first kk to the outputs, else they
  // become the new carried top-K in [0, kk).  (A first version spread the m^2 pairs over all threads
  // with an LDS atomic per pair: consecutive threads hit the same counter, 45 us at m = 272 —
  // K = 50 over 1M rows; a one-read-per-step loop then paid the LDS latency per step, 21 us.)
  auto rank = [&](int carry, int nslot, bool direct) -> int {
    const int mtot = carry + nslot;
    auto slot = [&](int u) { return u < carry ? u : kMaxK + u - carry; };
    // G threads per slot (a power of two, G * mtot <= T, G <= 64: one wave's lanes), each counting a
    // contiguous share of the others, summed by lane swaps
    int G = 1, lgG = 0;
    while (G < 64 && 2 * G * mtot <= T) {
      G *= 2;
      ++lgG;
    }
    const int per = (mtot + G - 1) / G;
    const int rounds = (mtot * G + T - 1) / T;  // block-uniform
    for (int rd = 0; rd < rounds; ++rd) {
      const int w = rd * T + tid, u = w >> lgG, g = w & (G - 1);  // G a power of two: no divides
      const int a = slot(u < mtot ? u : 0);
      const double sa = L.cand_d[a];
      const int ra = L.row_s[a];
      const int v0 = g * per, v1 = v0 + per < mtot ? v0 + per : mtot;
      int rk = 0;
      for (int v = v0; v < v1; v += 8) {  // 8 independent LDS reads in flight per step (the tail
                                          // predicated: a serial tail paid one LDS round trip per slot)
        double sb[8];
        int rb[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int b = slot(v + e < v1 ? v + e : v1 - 1);
          sb[e] = L.cand_d[b];
          rb[e] = L.row_s[b];
        }
#pragma unroll
        for (int e = 0; e < 8; ++e)  // bitwise, not short-circuit: hipcc branched on each && / ||
          rk += (int)((v + e < v1) & ((sb[e] > sa) | ((sb[e] == sa) & (rb[e] < ra))));
      }
      // group sum (G consecutive lanes, power of two): DPP xor 1 / 2, then row_half_mirror / row_mirror
      // (pairing quads / halves whose lanes already agree), LDS swaps only across 16-lane rows
      if (G > 1) rk += __builtin_amdgcn_update_dpp(0, rk, 0xB1, 0xF, 0xF, false);
      if (G > 2) rk += __builtin_amdgcn_update_dpp(0, rk, 0x4E, 0xF, 0xF, false);
      if (G > 4) rk += __builtin_amdgcn_update_dpp(0, rk, 0x141, 0xF, 0xF, false);
      if (G > 8) rk += __builtin_amdgcn_update_dpp(0, rk, 0x140, 0xF, 0xF, false);
      for (int o = 16; o < G; o <<= 1) rk += __shfl_xor(rk, o, 64);
      if (u < mtot && g == 0) L.rank_s[a] = rk;
    }
    SEL_MARK(15)
    __syncthreads();
    SEL_MARK(16)
    for (int u = tid; u < mtot; u += T) {
      const int sl = slot(u);
      const int rk = L.rank_s[sl];
      const double sc = L.cand_d[sl];
      if (sc == -INFINITY || rk >= kk) continue;
      if (direct) {
        oi[rk] = (int64_t)L.row_s[sl] + idx_base;
        if (os) os[rk] = (float)sc;
        if (os64) os64[rk] = sc;
      } else {
        L.tmp_d[rk] = sc;
        L.tmp_r[rk] = L.row_s[sl];
        atomicAdd(&L.bcast[3], 1u);
      }
    }
    if (direct) return kk;
    __syncthreads();
    const int kept = (int)L.bcast[3];
    for (int r = tid; r < kept; r += T) {
      L.cand_d[r] = L.tmp_d[r];
      L.row_s[r] = L.tmp_r[r];
    }
    __syncthreads();
    if (tid == 0) L.bcast[3] = 0;
    __syncthreads();
    return kept;
  };
  int cnt;
  bool coarse_ok = COARSE && !take_all;
  if (COARSE && !take_all) {
    // (C, coarse) blocks whose max clears thr, then their units
    for (int it = 0; it < kRegB; ++it) {
      const int64_t i = tid + (int64_t)it * T;
      if (i < nblk && bc[it] >= thr && bc[it] > -INFINITY) {
        const uint32_t p = atomicAdd(&L.bcast[3], 1u);
        if (p < (uint32_t)kBlkCap) {
          L.cand_b[p] = (int)i;
          L.ukey[p] = f2key(bc[it]);
        }
      }
    }
    for (int64_t i = tid + (int64_t)kRegB * T; i < nblk; i += T) {
      const float v = brow[i];
      if (v >= thr && v > -INFINITY) {
        const uint32_t p = atomicAdd(&L.bcast[3], 1u);
        if (p < (uint32_t)kBlkCap) {
          L.cand_b[p] = (int)i;
          L.ukey[p] = f2key(v);
        }
      }
    }
    __syncthreads();
    int nb = (int)L.bcast[3];
    SEL_MARK(17)
    SEL_VAL(10, nb)
    __syncthreads();
    if (tid == 0) L.bcast[3] = 0;
    if (nb <= kBlkCap && nb > 2 * kk + 32) {
      // block-level tightening (large K: the first bound comes from thread maxima, each over ~nblk/T
      // blocks, and admits many blocks — K = 50 over 1M rows: ~100 blocks, ~1700 units, past the unit
      // buffer, which sent every query through the all-units path): the exact kth largest of the
      // collected blocks' maxima is again a distinct-row bound (>= thr), and only blocks clearing
      // it - 2 delta keep their units
      const float t2 = key2f(block_select_kth(L.ukey, nb, kk, L.hist, L.bcast, 4));
      const float thr2 = lower_threshold(t2, tdel);
      if (thr2 > thr) {
        const uint32_t k2 = f2key(thr2);
        __syncthreads();
        for (int p = tid; p < nb; p += T)  // compacted into cand_u (nb <= kBlkCap <= kCandCap), then back
          if (L.ukey[p] >= k2) L.cand_u[atomicAdd(&L.bcast[3], 1u)] = L.cand_b[p];
        __syncthreads();
        const int nb2 = (int)L.bcast[3];
        for (int p = tid; p < nb2; p += T) L.cand_b[p] = L.cand_u[p];
        __syncthreads();
        if (tid == 0) L.bcast[3] = 0;
        nb = nb2;
        thr = thr2;
        __syncthreads();
      }
    }
    if (nb > kBlkCap) {
      coarse_ok = false;
      cnt = collect(thr, false, 0, nunits);
    } else {
      // one unit per thread-slot: all loads of a pass issued together
      for (int s0 = 0; s0 < nb * UPB; s0 += T) {
        const int s = s0 + tid;
        const int64_t u = (int64_t)L.cand_b[(s < nb * UPB ? s : 0) / UPB] * UPB + (s % UPB);
        const float v = row[u];
        if (s < nb * UPB) take(u, v, thr);
      }
      __syncthreads();
      cnt = (int)L.bcast[2];
      SEL_MARK(18)
      __syncthreads();
      if (tid == 0) L.bcast[2] = 0;
      __syncthreads();
    }
    SEL_VAL(11, cnt)
    if (coarse_ok && cnt <= UC && cnt > 2 * kk + 32) {
      // tighten: the exact K-th largest of the collected units' values (distinct rows: <= t)
      const float t2 = key2f(block_select_kth(L.ukey, cnt, kk, L.hist, L.bcast, 4));
      const float thr2 = lower_threshold(t2, tdel);
      if (thr2 > thr) {
        const uint32_t k2 = f2key(thr2);
        for (int p = tid; p < cnt; p += T)
          if (L.ukey[p] >= k2 && key2f(L.ukey[p]) > -INFINITY) {
            const uint32_t o = atomicAdd(&L.bcast[2], 1u);
            L.cand_b[o] = L.cand_u[p];  // cnt <= UC <= kBlkCap
          }
        __syncthreads();
        cnt = (int)L.bcast[2];
        for (int p = tid; p < cnt; p += T) L.cand_u[p] = L.cand_b[p];
        thr = thr2;
        __syncthreads();
        if (tid == 0) L.bcast[2] = 0;
        __syncthreads();
      }
    }
  } else {
    cnt = collect(thr, !COARSE, 0, nunits);
  }
  if (!RAW) query_norm();  // read after rescore's first barrier
  SEL_VAL(12, cnt)
  SEL_VAL(13, take_all)
  SEL_VAL(14, __float_as_int(thr))
  SEL_MARK(3)
  if (cnt > UC && !take_all) {
    const float t = key2f(row_select_kth(row, nunits, kk, L.hist, L.bcast));
    thr = lower_threshold(t, two_delta);
    cnt = collect(thr, false, 0, nunits);
  }
  if (cnt <= UC) {
    const int ns = rescore(cnt);
    __syncthreads();
    SEL_MARK(4)
    rank(0, ns, true);
  } else {
    // massive near-ties: batches of UC units in position order (a batch cannot overflow), each
    // merged into the carried exact top-K
    int kept = 0;
    for (int64_t lo = 0; lo < nunits; lo += UC) {
      const int c = collect(thr, false, lo, lo + UC < nunits ? lo + UC : nunits);
      if (c == 0) continue;
      const int ns = rescore(c);
      __syncthreads();
      kept = rank(kept, ns, false);
    }
    SEL_MARK(4)
    for (int r = tid; r < kept; r += T) {
      oi[r] = (int64_t)L.row_s[r] + idx_base;
      if (os) os[r] = (float)L.cand_d[r];
      if (os64) os64[r] = L.cand_d[r];
    }
  }
  SEL_MARK(5)
#ifdef MMR_SELECT_TRACE
  if (blockIdx.x == 0 && threadIdx.x == 0) g_sel_trace[6] = cnt;
#endif
}

// ------------------------------------------------------------------ shard merge
// Lists [n_lists][nq_total][k_in]; workgroup qi merges query q0 + qi.  Optional payload
// pay [n_lists][nq_total][k_in][P] f64 rides with each entry into out_pay [nq][k_out][P] (the
// sharded rerank's per-candidate components, computed on the shard that owns the row).  Entry e's
// score / index / payload sit at scores[e * ss], idx[e * si], pay[e * sp + p]: separate arrays
// (1, 1, P) or ONE packed all-gather buffer of 8-byte words [n_lists][nq_total][k_in][W] = {f64 score,
// int64 index, P f64 payload} (W, W, W: mmr_merge_topk_packed).
__global__ __launch_bounds__(256) void knn_merge(const double* __restrict__ scores,
                                                 const int64_t* __restrict__ idx, int n_lists,
                                                 int64_t nq_total, int64_t q0, int k_in, int k_out,
                                                 int64_t* __restrict__ out_idx,
                                                 float* __restrict__ out_score,
                                                 double* __restrict__ out_score64,
                                                 const double* __restrict__ pay, int P,
                                                 double* __restrict__ out_pay, int64_t ss, int64_t si, int64_t sp) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* cs = (double*)smem;
  int64_t* ci = (int64_t*)(smem + sizeof(double) * n_lists * k_in);
  const int64_t qi = blockIdx.x;
  const int m = n_lists * k_in;
  auto src = [&](int c) { return ((int64_t)(c / k_in) * nq_total + q0 + qi) * k_in + c % k_in; };
  for (int c = threadIdx.x; c < m; c += blockDim.x) {
    const int64_t off = src(c);
    cs[c] = scores[off * ss];
    ci[c] = idx[off * si];
  }
  __syncthreads();
  int nvalid = 0;
  for (int c = 0; c < m; ++c) nvalid += ci[c] >= 0;
  for (int c = threadIdx.x; c < m; c += blockDim.x) {
    const int64_t ic = ci[c];
    if (ic < 0) continue;
    const double sc = cs[c];
    int rank = 0;
    for (int j = 0; j < m; ++j) {
      const int64_t ij = ci[j];
      if (ij < 0) continue;
      const double sj = cs[j];
      rank += (sj > sc) || (sj == sc && ij < ic);
    }
    if (rank < k_out) {
      out_idx[qi * k_out + rank] = ic;
      if (out_score) out_score[qi * k_out + rank] = (float)sc;
      if (out_score64) out_score64[qi * k_out + rank] = sc;
      if (out_pay)
        for (int p = 0; p < P; ++p) out_pay[(qi * k_out + rank) * P + p] = pay[src(c) * sp + p];
    }
  }
  for (int r = nvalid + threadIdx.x; r < k_out; r += blockDim.x) {
    out_idx[qi * k_out + r] = -1;
    if (out_score) out_score[qi * k_out + r] = -INFINITY;
    if (out_score64) out_score64[qi * k_out + r] = -INFINITY;
    if (out_pay)
      for (int p = 0; p < P; ++p) out_pay[(qi * k_out + r) * P + p] = 0.0;
  }
}

// ------------------------------------------------------------------ DLS link-graph filter
// Row i of a self-join (queries = gallery rows r0..r0+nq): drop i itself (the reference sets the
// diagonal to -1), keep neighbours with exact score >= threshold in rank order (score desc, index
// asc), first max_links (DLSRetrievalEngine._build_link_graph, retrieval.py:121-138).
__global__ __launch_bounds__(256) void knn_link_filter(const int64_t* __restrict__ idx,
                                                       const double* __restrict__ s64, int k,
                                                       int64_t nq, int64_t r0, int64_t idx_base,
                                                       double threshold, int max_links,
                                                       int64_t* __restrict__ nbr,
                                                       int32_t* __restrict__ cnt) {
  const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (q >= nq) return;
  const int64_t self = r0 + q;
  int c = 0;
  for (int j = 0; j < k && c < max_links; ++j) {
    const int64_t g = idx[q * k + j];
    if (g < 0) break;
    const int64_t loc = g - idx_base;
    if (loc == self) continue;
    if (!(s64[q * k + j] >= threshold)) break;  // ranked: nothing later passes either
    nbr[q * max_links + c++] = loc;
  }
  for (int j = c; j < max_links; ++j) nbr[q * max_links + j] = -1;
  cnt[q] = c;
}

// ------------------------------------------------------------------ KG / label reranker
// Reranker.rerank (src/Retrieval/reranker.py:240-333) fused after the top-K, one wave per query,
// one candidate per lane (kc <= 64): embedding cosine (exact f64 of the raw f32 rows; 0 for a
// zero norm, safe_cos :134-142), label Jaccard on 64-bit label sets (:144-149), KG-vector cosine,
// each min-max scaled over the valid candidates (:151-159, constant -> 0), final = a*e + b*l + g*k,
// ranked by final desc with equal finals -> later candidate first (the reference's
// np.argsort(final)[::-1] over a short, insertion-sorted list), first topk written.
__device__ __forceinline__ double wave_min_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ double wave_max_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
  return v;
}

__device__ __forceinline__ double minmax_lane(double x, bool valid) {
  const double lo = wave_min_d(valid ? x : INFINITY), hi = wave_max_d(valid ? x : -INFINITY);
  return (hi - lo == 0.0) ? 0.0 : (x - lo) / (hi - lo);
}

// The three raw components of candidate `lane` of query qi (lane < kc): e = emb cosine, lab =
// label Jaccard, kg = KG cosine; my = its local row (-1: empty or not in this index).  One wave.
struct RerankRaw {
  double e, lab, kg;
  int64_t my;
};
__device__ RerankRaw rerank_raw(const float* __restrict__ qe, int d, const float* __restrict__ gal,
                                const uint16_t* __restrict__ galh, int Dp,
                                const double* __restrict__ gnorm64, int64_t n, int64_t idx_base,
                                const int64_t* __restrict__ cand, int kc, const uint64_t* __restrict__ qlab,
                                const uint64_t* __restrict__ glab, const float* __restrict__ qkg,
                                const float* __restrict__ gkg, int dk, int64_t qi, int lane) {
  const int64_t* cq = cand + qi * kc;
  const float* qr = qe + qi * (int64_t)d;
  const float* qk = qkg + qi * (int64_t)dk;
  double qq = 0.0, kk = 0.0;
  for (int t = lane; t < d; t += 64) qq += (double)qr[t] * (double)qr[t];
  for (int t = lane; t < dk; t += 64) kk += (double)qk[t] * (double)qk[t];
  const double qn = sqrt(mmr::wave_sum(qq)), qkn = sqrt(mmr::wave_sum(kk));
  RerankRaw r = {0.0, 0.0, 0.0, -1};
  for (int c = 0; c < kc; ++c) {  // wave-cooperative dot products, candidate c lands on lane c
    const int64_t g = cq[c] - idx_base;
    const bool ok = cq[c] >= 0 && g >= 0 && g < n;
    double de = 0.0, dkg = 0.0, gk = 0.0;
    if (ok) {
      const float* gq = gkg + g * (int64_t)dk;
      for (int t = lane; t < d; t += 64) de += (double)qr[t] * gal_elem(gal, galh, g, t, Dp);
      for (int t = lane; t < dk; t += 64) {
        dkg += (double)qk[t] * (double)gq[t];
        gk += (double)gq[t] * (double)gq[t];
      }
    }
    de = mmr::wave_sum(de);
    dkg = mmr::wave_sum(dkg);
    gk = mmr::wave_sum(gk);
    if (lane == c && ok) {
      r.my = g;
      const double gn = gnorm64[g];
      r.e = (qn > 0.0 && gn > 0.0) ? de / (qn * gn) : 0.0;
      const double gkn = sqrt(gk);
      r.kg = (qkn > 0.0 && gkn > 0.0) ? dkg / (qkn * gkn) : 0.0;
    }
  }
  if (lane < kc && r.my >= 0) {
    const uint64_t a = qlab[qi], b = glab[r.my];
    const int u = __popcll(a | b);
    r.lab = u == 0 ? 0.0 : (double)__popcll(a & b) / (double)u;
  }
  return r;
}

// min-max over the valid lanes, mix, rank (final desc, equal finals: later candidate first), write
__device__ void rerank_mix_out(double e, double lab, double kgs, bool valid, int64_t gidx, double wa, double wb,
                               double wg, int topk, int64_t qi, int lane, int64_t* __restrict__ out_idx,
                               double* __restrict__ out_final, double* __restrict__ out_emb,
                               double* __restrict__ out_lab, double* __restrict__ out_kg) {
  const double en = minmax_lane(e, valid), ln = minmax_lane(lab, valid), kn = minmax_lane(kgs, valid);
  const double f = wa * en + wb * ln + wg * kn;
  int rank = 0;
  for (int j = 0; j < 64; ++j) {
    const double fj = __shfl(f, j, 64);
    const bool vj = __shfl((int)valid, j, 64) != 0;
    rank += vj && (fj > f || (fj == f && j > lane));
  }
  if (valid && rank < topk) {
    const int64_t o = qi * topk + rank;
    out_idx[o] = gidx;
    if (out_final) out_final[o] = f;
    if (out_emb) out_emb[o] = en;
    if (out_lab) out_lab[o] = ln;
    if (out_kg) out_kg[o] = kn;
  }
  int nvalid = 0;
  for (int j = 0; j < 64; ++j) nvalid += __shfl((int)valid, j, 64);
  for (int r = nvalid + lane; r < topk; r += 64) out_idx[qi * topk + r] = -1;
}

__global__ __launch_bounds__(64) void knn_rerank(
    const float* __restrict__ qe, int d, const float* __restrict__ gal, const uint16_t* __restrict__ galh, int Dp,
    const double* __restrict__ gnorm64, int64_t n, int64_t idx_base, const int64_t* __restrict__ cand,
    int kc, const uint64_t* __restrict__ qlab, const uint64_t* __restrict__ glab,
    const float* __restrict__ qkg, const float* __restrict__ gkg, int dk, double wa, double wb,
    double wg, int topk, int64_t* __restrict__ out_idx, double* __restrict__ out_final,
    double* __restrict__ out_emb, double* __restrict__ out_lab, double* __restrict__ out_kg) {
  const int64_t qi = blockIdx.x;
  const int lane = threadIdx.x;
  const RerankRaw r = rerank_raw(qe, d, gal, galh, Dp, gnorm64, n, idx_base, cand, kc, qlab, glab, qkg, gkg, dk, qi, lane);
  rerank_mix_out(r.e, r.lab, r.kg, lane < kc && r.my >= 0, r.my + idx_base, wa, wb, wg, topk, qi, lane, out_idx,
                 out_final, out_emb, out_lab, out_kg);
}

// Sharded rerank, shard side: the raw components of this shard's candidates -> comp [nq][kc][3]
// (zeros for an empty slot).
__global__ __launch_bounds__(64) void knn_rerank_comp(
    const float* __restrict__ qe, int d, const float* __restrict__ gal, const uint16_t* __restrict__ galh, int Dp,
    const double* __restrict__ gnorm64, int64_t n, int64_t idx_base, const int64_t* __restrict__ cand,
    int kc, const uint64_t* __restrict__ qlab, const uint64_t* __restrict__ glab,
    const float* __restrict__ qkg, const float* __restrict__ gkg, int dk, double* __restrict__ comp) {
  const int64_t qi = blockIdx.x;
  const int lane = threadIdx.x;
  const RerankRaw r = rerank_raw(qe, d, gal, galh, Dp, gnorm64, n, idx_base, cand, kc, qlab, glab, qkg, gkg, dk, qi, lane);
  if (lane < kc) {
    double* o = comp + (qi * kc + lane) * 3;
    o[0] = r.e;
    o[1] = r.lab;
    o[2] = r.kg;
  }
}

// Sharded rerank, after the merge: cand (global indices, -1 empty) + their merged components.
__global__ __launch_bounds__(64) void knn_rerank_mix(const int64_t* __restrict__ cand, const double* __restrict__ comp,
                                                     int kc, double wa, double wb, double wg, int topk,
                                                     int64_t* __restrict__ out_idx, double* __restrict__ out_final,
                                                     double* __restrict__ out_emb, double* __restrict__ out_lab,
                                                     double* __restrict__ out_kg) {
  const int64_t qi = blockIdx.x;
  const int lane = threadIdx.x;
  const int64_t g = lane < kc ? cand[qi * kc + lane] : -1;
  const bool valid = g >= 0;
  const double* c = comp + (qi * kc + (lane < kc ? lane : 0)) * 3;
  rerank_mix_out(valid ? c[0] : 0.0, valid ? c[1] : 0.0, valid ? c[2] : 0.0, valid, g, wa, wb, wg, topk, qi, lane,
                 out_idx, out_final, out_emb, out_lab, out_kg);
}

}  // namespace

// ------------------------------------------------------------------ index object
struct mmr_index {
  int device = 0;
  int64_t n = 0, Np = 0, idx_base = 0;
  int d = 0, Dp = 0;
  int dtype = 0;              // MMR_F32 (f32 rows in gal) | MMR_F16 (native fp16: raw rows in gh, no gal)
  float* gal = nullptr;       // [Np][Dp] f32 rows (MMR_F32 index)
  float* inv_norm = nullptr;  // [Np]
  double* norm64 = nullptr;   // [Np]
  uint16_t* gs = nullptr;     // [Np][2Dp] bf16 hi/lo split (mode x3)
  float* gt = nullptr;        // [Np][Dp] f32 in the tile16 layout (skinny scan)
  // [Np][Dp] fp16 in the tile32h layout, the operand of every fp16 scan (lq / gmax / tile / p8): the unit
  // rows g/|g| of an MMR_F32 index in mode f16 (built on first use), or the raw rows of an MMR_F16 index
  // (its only copy of the gallery: 2 B per element; scans scale by inv_norm per row)
  uint16_t* gh = nullptr;
  int mode = 1;               // 0: f32 MFMA scores, 1: bf16x3 split scores, 2: fp16 scan
  // Workspace: one set per index, sized by what the mode needs (grown on demand).  `mu` serialises
  // the enqueue of searches; across streams the workspace follows the stream: a search on another
  // stream records ws_event on ws_stream (the last user's) and waits for it, so two streams never race
  // on it (and a realloc waits for the last user the same way).  Recorded at the switch, not after
  // every search: an event record per search cost 3-5 us of device time (16-query search 50.3 ->
  // 47.2 us back to back).
  std::mutex mu;
  int64_t ws_qrows = 0;       // query rows in qn / qnorm64
  int64_t ws_vals = 0;        // floats in vals
  int64_t ws_qsrows = 0;      // query rows in qs
  float* qn = nullptr;        // [rows][Dp] f32 (or fp16 / tile layouts, same bytes or fewer)
  double* qnorm64 = nullptr;  // [rows]
  float* vals = nullptr;      // scores (f32 mode) or per-(query, unit) maxima
  int64_t ws_bvals = 0;       // floats in bvals
  float* bvals = nullptr;     // mode f16: per-(query, 64-row block) maxima [256][Np/64]
  uint16_t* qs = nullptr;     // [rows][3Dp] bf16 split queries (x3 GEMM)
  int n_cu = 256;             // compute units of `device` (persistent grids)
  hipEvent_t ws_event = nullptr;
  hipStream_t ws_stream = nullptr;
  bool ws_used = false;
};

namespace {

constexpr int64_t kScoresBudget = int64_t(4) << 30;  // bytes of value workspace per query chunk

// Queries per chunk: bounded by the value workspace (f32 mode: Np floats per query; x3: Np / 4).
// The f16 scan runs passes of <= 256 queries whatever the chunk.
int64_t chunk_queries(const mmr_index* ix) {
  const int64_t per = (ix->mode == 0 ? ix->Np : ix->Np / 4) * (int64_t)sizeof(float);
  int64_t c = kScoresBudget / per;
  c = c / 256 * 256;
  return c < 256 ? 256 : c;
}

// the p8 GEMM scan takes the fp16 passes of > 128 queries when the row length fits its K tiles
bool p8_ok(const mmr_index* ix) { return ix->Dp % 128 == 0 && ix->Dp <= 1024; }

// raw-row galleries (native fp16 index): the scans' per-row 1 / |g|; unit-row copies: none
const float* scan_rscale(const mmr_index* ix) { return ix->dtype == MMR_F16 ? ix->inv_norm : nullptr; }

template <class T>
mmr_status grow(mmr_index* ix, T*& buf, int64_t& have, int64_t want, size_t elem_bytes) {
  if (want <= have) return MMR_OK;
  if (buf) {
    if (ix->ws_used) {  // the last search has released it
      (void)hipEventRecord(ix->ws_event, ix->ws_stream);
      (void)hipEventSynchronize(ix->ws_event);
    }
    (void)hipFree(buf);
  }
  buf = nullptr;
  have = 0;
  MMR_CHECK_HIP(hipMalloc((void**)&buf, elem_bytes * want));
  have = want;
  return MMR_OK;
}

// Workspace for a search of nq queries in the current mode (rows rounded to 256).
mmr_status ensure_ws(mmr_index* ix, int64_t nq) {
  const int64_t cq = round_up(nq < chunk_queries(ix) ? nq : chunk_queries(ix), 256);
  int64_t rows = cq, vals = 0, qs = 0, bvals = 0;
  if (ix->mode == 0) {
    vals = cq * ix->Np;
  } else if (ix->mode == 1) {
    vals = cq * (ix->Np / 4);
    qs = cq;
  } else {
    // passes of <= 256 queries, or on the p8 scan 512 (2-row units) / 1024 (4-row units): the same
    // unit-maxima bytes; fp16 query rows of a pass take half the f32 rows of qn
    rows = 1024;
    const int64_t nr = ix->Np;  // a multiple of 256: the p8 scan's whole gallery tiles
    vals = p8_ok(ix) ? 512 * (nr / 2) : 256 * (nr / 4);  // p8: up to 512 queries of 2-row unit maxima
    bvals = 1024 * (nr / 64);
  }
  int64_t hq = ix->ws_qrows, hq2 = ix->ws_qrows;
  mmr_status s = grow(ix, ix->qn, hq, rows, sizeof(float) * ix->Dp);
  if (s == MMR_OK) s = grow(ix, ix->qnorm64, hq2, rows, sizeof(double));
  if (s != MMR_OK) return s;
  ix->ws_qrows = hq < hq2 ? hq : hq2;
  if ((s = grow(ix, ix->vals, ix->ws_vals, vals, sizeof(float))) != MMR_OK) return s;
  if (qs > 0 && (s = grow(ix, ix->qs, ix->ws_qsrows, qs, sizeof(uint16_t) * 3 * ix->Dp)) != MMR_OK) return s;
  if (bvals > 0 && (s = grow(ix, ix->bvals, ix->ws_bvals, bvals, sizeof(float))) != MMR_OK) return s;
  return MMR_OK;
}

// Largest query chunk routed to the skinny scan in mode x3.  Measured (100k x 768, MI355X): Q <= 16 scan
// 58 us (5.3 TB/s) vs the x3 GEMM's ~110 us; Q = 32 132 vs ~145 us per search; Q = 64 (4 query tiles,
// MFMA-paced with ~1.5 waves per SIMD) 196 vs ~145.
constexpr int64_t kSkinnyMaxQ = 32;
// query tiles per p8 pass with 4-row units (2 / 4 measured: 4, profiles/r03_s4_knn_pair_ab.txt)
constexpr int kP8PairTiles = 4;

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

template <int WQ, int MQ, int WR, int MR, bool PF>
void launch_f16_tile(hipStream_t st, const mmr_index* ix, const uint16_t* qh, float* gm, float* bm, int64_t ldG,
                     int64_t ldB, int64_t n_rt) {
  using C = F16TileCfg<WQ, MQ, WR, MR, PF>;
  const size_t lds = (size_t)C::STAGES * C::SLICE_B;
  knn_scan_f16_tile<WQ, MQ, WR, MR, PF><<<dim3((unsigned)ix->n_cu), dim3(64 * C::NW), lds, st>>>(
      qh, ix->gh, gm, bm, ix->Dp, ldG, ldB, ix->n, n_rt, scan_rscale(ix));
}

// COARSE selections (block maxima first) run 512-thread workgroups, the unit-level ones 1024
template <int MODE, bool COARSE = false, bool RAW = false>
void launch_select(hipStream_t st, int64_t nq, const float* vals, int64_t ldV, int64_t nunits, const mmr_index* ix,
                   int k, float two_delta, const float* q_raw, const double* qnorm64, int64_t* oi, float* os,
                   double* os64, int32_t* ost, const float* bvals = nullptr, int64_t ldB = 0,
                   float two_delta_abs = 0.f, const double* qpre = nullptr) {
  constexpr int T = COARSE ? 512 : kSelThreads;
  const dim3 g((unsigned)nq), b(T);
#define MMR_SEL(NC)                                                                                              \
  knn_select_t<MODE, NC, T, COARSE, RAW><<<g, b, 0, st>>>(vals, ldV, nunits, ix->n, k, two_delta, bvals, ldB,    \
                                                          two_delta_abs, q_raw, ix->d, qnorm64, ix->gal, ix->Dp,  \
                                                          ix->norm64, ix->idx_base,                               \
                                                          ix->dtype == MMR_F16 ? ix->gh : nullptr, oi, os, os64,  \
                                                          ost, qpre)
  // NC = 256-float chunks of a row in the f64 re-score (0: d > 1024, strided loop)
  switch (ix->d > 1024 ? 0 : (int)ceil_div(ix->Dp, 256)) {
    case 1: MMR_SEL(1); break;
    case 2: MMR_SEL(2); break;
    case 3: MMR_SEL(3); break;
    case 4: MMR_SEL(4); break;
    default: MMR_SEL(0); break;
  }
#undef MMR_SEL
}

// Mode-specific scan copies, built when a mode first needs them (mmr_index_set_mode / the first
// search): x3 = the bf16 hi/lo split [Np][2Dp] + the tile16 f32 copy of the skinny scan (8 B per
// element); f16 = the tile32h fp16 unit rows + (Dp % 128 == 0, Dp <= 1024) the row-major fp16 copy
// of the p8 scan (4 B per element).  A switch to f16 / f32 frees the x3 copies (an fp16 gallery
// index holds f32 rows + fp16 copies only); a switch away from f16 frees the fp16 copies.
mmr_status build_x3_copies(mmr_index* ix) {
  if (ix->gs != nullptr && ix->gt != nullptr) return MMR_OK;
  DeviceGuard g(ix->device);
  hipError_t e;
  if ((ix->gs == nullptr && (e = hipMalloc(&ix->gs, sizeof(uint16_t) * ix->Np * 2 * ix->Dp)) != hipSuccess) ||
      (ix->gt == nullptr && (e = hipMalloc(&ix->gt, sizeof(float) * ix->Np * ix->Dp)) != hipSuccess)) {
    (void)hipGetLastError();  // a failed hipMalloc leaves a sticky error the next launch check would report
    mmr::set_error("mmr_index: hipMalloc(x3 scan copies) failed: %s", hipGetErrorString(e));
    return MMR_ERR_OOM;
  }
  const int64_t total = ix->Np * ix->Dp;
  knn_split_gallery<<<dim3((unsigned)ceil_div(total, 256)), dim3(256)>>>(ix->gal, ix->Dp, total, ix->gs);
  e = hipGetLastError();
  if (e == hipSuccess) {
    const int64_t total4 = total / 4;
    knn_tile_gallery<<<dim3((unsigned)ceil_div(total4, 256)), dim3(256)>>>(ix->gal, ix->Dp, total4, ix->gt);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e != hipSuccess) {
    mmr::set_error("mmr_index: x3 scan copy kernels failed: %s", hipGetErrorString(e));
    return MMR_ERR_HIP;
  }
  return MMR_OK;
}

mmr_status build_f16_copies(mmr_index* ix) {
  if (ix->gh != nullptr) return MMR_OK;  // built, or the native fp16 index's own rows
  DeviceGuard g(ix->device);
  hipError_t e;
  if ((e = hipMalloc(&ix->gh, sizeof(uint16_t) * ix->Np * ix->Dp)) != hipSuccess) {
    ix->gh = nullptr;
    (void)hipGetLastError();
    mmr::set_error("mmr_index: hipMalloc(fp16 copy) failed: %s", hipGetErrorString(e));
    return MMR_ERR_OOM;
  }
  const int64_t total8 = ix->Np * ix->Dp / 8;
  knn_tile_gallery_f16<<<dim3((unsigned)ceil_div(total8, 256)), dim3(256)>>>(ix->gal, ix->inv_norm, ix->Dp, total8,
                                                                           ix->gh);
  e = hipGetLastError();
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e != hipSuccess) {
    mmr::set_error("mmr_index: fp16 copy kernel failed: %s", hipGetErrorString(e));
    return MMR_ERR_HIP;
  }
  return MMR_OK;
}

void free_copies(mmr_index* ix, bool x3, bool f16) {
  DeviceGuard g(ix->device);
  if (x3 || f16) (void)hipDeviceSynchronize();  // no search still reads them
  if (x3) {
    if (ix->gs) (void)hipFree(ix->gs);
    if (ix->gt) (void)hipFree(ix->gt);
    ix->gs = nullptr;
    ix->gt = nullptr;
  }
  if (f16 && ix->dtype != MMR_F16) {  // a native fp16 index's gh IS its gallery
    if (ix->gh) (void)hipFree(ix->gh);
    ix->gh = nullptr;
  }
}

}  // namespace

extern "C" {

int mmr_max_k(void) { return kMaxK; }

mmr_status mmr_index_create(const void* gallery, int64_t n, int32_t d, mmr_dtype dtype,
                            int gallery_is_host, int64_t idx_base, int device, mmr_index** out) {
  mmr::clear_error();
  MMR_REQUIRE(out != nullptr, "mmr_index_create: out is NULL");
  MMR_REQUIRE(n >= 0 && d > 0, "mmr_index_create: bad shape n=%lld d=%d", (long long)n, d);
  MMR_REQUIRE(n == 0 || gallery != nullptr, "mmr_index_create: gallery is NULL");
  MMR_REQUIRE(n < (int64_t(1) << 31), "mmr_index_create: n=%lld exceeds 2^31 rows per shard",
              (long long)n);
  if (dtype != MMR_F32 && dtype != MMR_F16) {
    mmr::set_error("mmr_index_create: dtype %d not built (MMR_F32 | MMR_F16)", (int)dtype);
    return MMR_ERR_UNSUPPORTED;
  }
  DeviceGuard g(device);
  mmr_index* ix = new mmr_index();
  ix->device = device;
  ix->n = n;
  ix->d = d;
  ix->Dp = (int)round_up(d, 64);
  ix->Np = round_up(n > 0 ? n : 1, kRowPad);
  ix->idx_base = idx_base;
  ix->dtype = dtype;
  auto fail = [&](mmr_status s) {
    mmr_index_destroy(ix);
    return s;
  };
  hipError_t e;
  if (hipDeviceGetAttribute(&ix->n_cu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || ix->n_cu <= 0)
    ix->n_cu = 256;
  if ((e = hipEventCreateWithFlags(&ix->ws_event, hipEventDisableTiming)) != hipSuccess) {
    ix->ws_event = nullptr;
    mmr::set_error("mmr_index_create: hipEventCreate failed: %s", hipGetErrorString(e));
    return fail(MMR_ERR_HIP);
  }
  const size_t esz = dtype == MMR_F16 ? sizeof(uint16_t) : sizeof(float);
  if ((dtype == MMR_F16 ? (e = hipMalloc(&ix->gh, sizeof(uint16_t) * ix->Np * ix->Dp))
                        : (e = hipMalloc(&ix->gal, sizeof(float) * ix->Np * ix->Dp))) != hipSuccess ||
      (e = hipMalloc(&ix->inv_norm, sizeof(float) * ix->Np)) != hipSuccess ||
      (e = hipMalloc(&ix->norm64, sizeof(double) * ix->Np)) != hipSuccess) {
    mmr::set_error("mmr_index_create: hipMalloc failed: %s", hipGetErrorString(e));
    return fail(MMR_ERR_OOM);
  }
  // stage the raw rows into a contiguous device buffer, then pad + norm in one kernel
  void* raw = nullptr;
  if (n > 0) {
    if ((e = hipMalloc(&raw, esz * n * d)) != hipSuccess) {
      mmr::set_error("mmr_index_create: hipMalloc(raw) failed: %s", hipGetErrorString(e));
      return fail(MMR_ERR_OOM);
    }
    e = hipMemcpy(raw, gallery, esz * n * d, gallery_is_host ? hipMemcpyHostToDevice : hipMemcpyDeviceToDevice);
    if (e != hipSuccess) {
      (void)hipFree(raw);
      mmr::set_error("mmr_index_create: hipMemcpy failed: %s", hipGetErrorString(e));
      return fail(MMR_ERR_HIP);
    }
  }
  if (dtype == MMR_F16) {
    // native fp16 gallery: the raw rows ARE the scan operand (tile32h) and the exact re-score rows; the
    // index runs the fp16 scan only (mode 2)
    knn_prep_gallery_f16<<<dim3((unsigned)ceil_div(ix->Np, 4)), dim3(256)>>>(
        (const uint16_t*)raw, n, d, ix->gh, ix->Dp, ix->Np, ix->inv_norm, ix->norm64);
    ix->mode = 2;
  } else {
    knn_prep_gallery<<<dim3((unsigned)ceil_div(ix->Np, 4)), dim3(256)>>>(
        (const float*)raw, n, d, ix->gal, ix->Dp, ix->Np, ix->inv_norm, ix->norm64);
  }
  e = hipGetLastError();
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (raw) (void)hipFree(raw);
  if (e != hipSuccess) {
    mmr::set_error("mmr_index_create: prep kernel failed: %s", hipGetErrorString(e));
    return fail(MMR_ERR_HIP);
  }
  *out = ix;
  return MMR_OK;
}

mmr_status mmr_index_destroy(mmr_index* ix) {
  if (!ix) return MMR_OK;
  DeviceGuard g(ix->device);
  if (ix->gal) (void)hipFree(ix->gal);
  if (ix->inv_norm) (void)hipFree(ix->inv_norm);
  if (ix->norm64) (void)hipFree(ix->norm64);
  if (ix->gs) (void)hipFree(ix->gs);
  if (ix->gt) (void)hipFree(ix->gt);
  if (ix->gh) (void)hipFree(ix->gh);
  if (ix->qs) (void)hipFree(ix->qs);
  if (ix->qn) (void)hipFree(ix->qn);
  if (ix->qnorm64) (void)hipFree(ix->qnorm64);
  if (ix->vals) (void)hipFree(ix->vals);
  if (ix->bvals) (void)hipFree(ix->bvals);
  if (ix->ws_event) (void)hipEventDestroy(ix->ws_event);
  delete ix;
  return MMR_OK;
}

mmr_status mmr_index_device_bytes(const mmr_index* ix, int64_t* gallery_bytes, int64_t* workspace_bytes) {
  mmr::clear_error();
  MMR_REQUIRE(ix != nullptr, "mmr_index_device_bytes: index is NULL");
  const int64_t e = ix->Np * ix->Dp;
  int64_t gb = (ix->gal ? e * 4 : 0) + ix->Np * (4 + 8);
  if (ix->gs) gb += e * 2 * 2;
  if (ix->gt) gb += e * 4;
  if (ix->gh) gb += e * 2;
  const int64_t wb = ix->ws_qrows * (ix->Dp * 4 + 8) + ix->ws_vals * 4 + ix->ws_bvals * 4 + ix->ws_qsrows * 3 * ix->Dp * 2;
  if (gallery_bytes) *gallery_bytes = gb;
  if (workspace_bytes) *workspace_bytes = wb;
  return MMR_OK;
}

mmr_status mmr_index_info(const mmr_index* ix, int64_t* n, int32_t* d, int64_t* idx_base) {
  mmr::clear_error();
  MMR_REQUIRE(ix != nullptr, "mmr_index_info: index is NULL");
  if (n) *n = ix->n;
  if (d) *d = ix->d;
  if (idx_base) *idx_base = ix->idx_base;
  return MMR_OK;
}

mmr_status mmr_index_reserve(mmr_index* ix, int64_t max_q) {
  mmr::clear_error();
  MMR_REQUIRE(ix != nullptr && max_q > 0, "mmr_index_reserve: bad arguments");
  DeviceGuard g(ix->device);
  std::lock_guard<std::mutex> lk(ix->mu);
  return ensure_ws(ix, max_q);
}

mmr_status mmr_index_search(mmr_index* ix, const float* q, int64_t nq, int32_t k,
                            int64_t* out_idx, float* out_score, double* out_score64,
                            int32_t* out_status, void* stream) {
  mmr::clear_error();
  MMR_REQUIRE(ix != nullptr, "mmr_index_search: index is NULL");
  MMR_REQUIRE(nq >= 0, "mmr_index_search: nq < 0");
  MMR_REQUIRE(k >= 1 && k <= kMaxK, "mmr_index_search: K=%d outside [1, %d]", k, kMaxK);
  if (nq == 0) return MMR_OK;
  MMR_REQUIRE(q != nullptr && out_idx != nullptr, "mmr_index_search: NULL query/output");
  DeviceGuard g(ix->device);
  std::lock_guard<std::mutex> lk(ix->mu);
  hipStream_t st = mmr::as_stream(stream);
  // the workspace follows the stream: wait for the previous search if it ran on another stream
  if (ix->ws_used && ix->ws_stream != st) {
    MMR_CHECK_HIP(hipEventRecord(ix->ws_event, ix->ws_stream));
    MMR_CHECK_HIP(hipStreamWaitEvent(st, ix->ws_event, 0));
  }
  mmr_status s = ensure_ws(ix, nq);
  if (s != MMR_OK) return s;
  if (ix->mode == 1 && (s = build_x3_copies(ix)) != MMR_OK) return s;  // default mode, first search
  if (ix->mode == 2 && (s = build_f16_copies(ix)) != MMR_OK) return s;  // never scan a missing copy
  // |s_approx - s64| <= delta; threshold margin 2*delta.
  //  f32 (knn_scores, knn_scan_f32_gmax): (Dp + 16) 2^-24 — f32 products accumulated in f32 over Dp
  //      terms of a unit query against g/|g| (|sum| <= 1), plus the normalisations;
  //  x3: + the dropped lo*lo bf16 terms and the bf16 rounding of the split, (3Dp + 16) 2^-24 + 4 2^-16;
  //  f16: fp16 rounding of both unit vectors, 2 * 2^-11 relative with sum |q_k g_k| <= 1
  //      (Cauchy-Schwarz) -> 2^-10; fp16 subnormal half-ulps (components below 2^-14 are held to
  //      2^-25 absolute): sum_k (|q_k| + |g_k|) 2^-25 <= 2 sqrt(Dp) 2^-25 (Cauchy-Schwarz again),
  //      computed from Dp below; f32 accumulation (Dp terms) and the f32 normalisation of both
  //      operands (the f32-mode bound, doubled: (2Dp + 64) 2^-24).
  const float two_delta32 = 2.0f * (float)(ix->Dp + 16) * 5.9604645e-8f;
  const float two_delta3 = 2.0f * ((float)(3 * ix->Dp + 16) * 5.9604645e-8f + 4.0f * 1.5258789e-5f);
  const float two_delta16 = 2.0f * (9.765625e-4f + 2.0f * sqrtf((float)ix->Dp) * 2.9802322e-8f +
                                    (float)(2 * ix->Dp + 64) * 5.9604645e-8f);
  //  f16 RAW (knn_scan_f16_gmax<RAW>: fp16(q) . g^ for the unnormalised q): the same terms scaled by |q|
  //      — fp16 rounding 2^-10 |q| (Cauchy-Schwarz over |q| |g^|), g^'s subnormal half-ulps
  //      sum |q_k| 2^-25 <= sqrt(Dp) |q| 2^-25, f32 accumulation (2Dp + 64) 2^-24 |q| — plus q's own
  //      subnormal half-ulps sum |g^_k| 2^-25 <= sqrt(Dp) 2^-25, independent of |q|:
  //      delta = |q| two_delta16r / 2 + two_delta16a / 2 (the selection computes |q| first).
  const float two_delta16r = 2.0f * (9.765625e-4f + sqrtf((float)ix->Dp) * 2.9802322e-8f +
                                     (float)(2 * ix->Dp + 64) * 5.9604645e-8f);
  const float two_delta16a = 2.0f * sqrtf((float)ix->Dp) * 2.9802322e-8f;
  const int64_t chunk = chunk_queries(ix);
  for (int64_t c0 = 0; c0 < nq; c0 += chunk) {
    const int64_t cq = nq - c0 < chunk ? nq - c0 : chunk;
    const float* qc = q + c0 * ix->d;
    int64_t* oi = out_idx + c0 * k;
    float* os = out_score ? out_score + c0 * k : nullptr;
    double* os64 = out_score64 ? out_score64 + c0 * k : nullptr;
    int32_t* ost = out_status ? out_status + c0 : nullptr;
    if (ix->mode == 2) {
      // fp16 scan, passes of <= 256 queries (16 * QT, QT a power of two), or on the p8 scan <= 512
      // (2-row units) / 1024 (4-row units): its query tiles share every gallery tile read (cfg5: Q =
      // 2048 over 1M rows reads the 2 GB fp16 gallery twice instead of 8 times).  Every scan reads the
      // tile32h fp16 image gh; rs scales raw rows (native fp16 index) by 1 / |g|.
      const bool p8 = p8_ok(ix);
      const float* rs = scan_rscale(ix);
      const bool u2 = ix->n <= (int64_t(1) << 18) || k >= 32;
      const int64_t pass = p8 ? 256 * (u2 ? 2 : kP8PairTiles) : 256;
      for (int64_t p0 = 0; p0 < cq; p0 += pass) {
        const int64_t pq = cq - p0 < pass ? cq - p0 : pass;
        int qt = 1;
        while (16 * qt < pq) qt *= 2;
        const int64_t Qp = 16 * qt;
        const float* qp = qc + p0 * ix->d;
        const uint16_t* qh = (const uint16_t*)ix->qn;
        float* gm = ix->vals;
        float* bm = ix->bvals;
        const int64_t ldG = ix->Np / 4, ldB = ix->Np / 64;
        if (pq > 128 && p8) {
          // 129-1024 queries: the persistent 8-phase GEMM (gemm.hip) with the unit-max epilogue —
          // 256-query M tiles x 256-row gallery tiles, row-major fp16 queries, the tile32h gallery.
          // (It computes all 256 query rows; at 100k x 768 it beats the LDS-ring tile scan from Q ~ 160:
          // Q = 64 / 128 / 192 / 256: 81 / 83 / 86 / 88 us vs 62 / 69 / 96 / 100.)
          const int tm = (int)((pq + 255) / 256);  // query tiles of this pass
          knn_prep_queries<<<dim3(64 * tm), dim3(256), 0, st>>>(qp, pq, ix->d, ix->qn, ix->Dp, 256 * tm, ix->qnorm64, 3);
          MMR_LAUNCH_CHECK();
          // unit size: 2 rows halves the rows the select re-scores per candidate unit, 4 rows halves
          // the unit maxima the scan writes (512 vs 256 MB per pass at 1M rows): 2 for small
          // galleries or large K (cfg2 100k / K 10: select 22 -> 16 us; cfg3 1M / K 50: 104 -> 65 us for
          // +30 us of scan), 4 for large galleries at small K (cfg5 1M / K 10: +37 us scan, -9 select)
          const int64_t ldG8 = ix->Np / (u2 ? 2 : 4), ldB8 = ix->Np / 64;
          MMR_CHECK_HIP(mmr::knn_scan_p8(qh, ix->gh, ix->Dp, (int)(ix->Np / 256), ix->n, gm, ldG8, bm, ldB8,
                                         u2 ? 2 : 4, st, tm, rs));
          if (u2)
            launch_select<3, true>(st, pq, gm, ldG8, ldG8, ix, k, two_delta16, qp, ix->qnorm64, oi + p0 * k,
                                   os ? os + p0 * k : nullptr, os64 ? os64 + p0 * k : nullptr, ost ? ost + p0 : nullptr,
                                   bm, ldB8);
          else
            launch_select<2, true>(st, pq, gm, ldG8, ldG8, ix, k, two_delta16, qp, ix->qnorm64, oi + p0 * k,
                                   os ? os + p0 * k : nullptr, os64 ? os64 + p0 * k : nullptr, ost ? ost + p0 : nullptr,
                                   bm, ldB8);
          MMR_LAUNCH_CHECK();
          continue;
        }
        if (pq > 32) {
          // 33-256 queries: the LDS-staged tile scan (64 / 128 / 256-query tiles), contiguous units
          const int wq = pq <= 64 ? 1 : pq <= 128 ? 2 : 4;
          const int64_t Qt = 64 * wq;
          knn_prep_queries<<<dim3((unsigned)ceil_div(Qt, 4)), dim3(256), 0, st>>>(
              qp, pq, ix->d, ix->qn, ix->Dp, Qt, ix->qnorm64, 2);
          MMR_LAUNCH_CHECK();
          const int64_t n_rt = ix->Np / 16;
          if (wq == 1) launch_f16_tile<1, 4, 4, 4, false>(st, ix, qh, gm, bm, ldG, ldB, n_rt);
          else if (wq == 2) launch_f16_tile<2, 4, 4, 4, false>(st, ix, qh, gm, bm, ldG, ldB, n_rt);
          else launch_f16_tile<4, 4, 2, 8, false>(st, ix, qh, gm, bm, ldG, ldB, n_rt);
          MMR_LAUNCH_CHECK();
          launch_select<2, true>(st, pq, gm, ldG, ldG, ix, k, two_delta16, qp, ix->qnorm64, oi + p0 * k,
                                 os ? os + p0 * k : nullptr, os64 ? os64 + p0 * k : nullptr, ost ? ost + p0 : nullptr,
                                 bm, ldB);
          MMR_LAUNCH_CHECK();
          continue;
        }
        const dim3 grid((unsigned)(ix->Np / 64));
        if (qt <= 2 && ix->d % 8 == 0 && ((uintptr_t)qp & 15) == 0) {
          // <= 32 queries: the scan reads the caller's f32 rows itself (no prep launch), per-query margin
          const int64_t nqp = pq;
          const bool lq = ix->Dp <= 1024;
          if (lq) {
            const size_t lds = (size_t)qt * 16 * ix->Dp * 2;
            const int64_t nblk = ix->Np / 64;
            const dim3 g2((unsigned)ix->n_cu);
            if (qt == 1) {
              if (ix->Dp % 128 == 0)
                knn_scan_f16_lq<1, 128, 8><<<g2, 512, lds, st>>>(qp, nqp, ix->d, ix->gh, gm, bm, ix->Dp, ldG, ldB, ix->n, nblk, ix->qnorm64, rs);
              else
                knn_scan_f16_lq<1, 64, 8><<<g2, 512, lds, st>>>(qp, nqp, ix->d, ix->gh, gm, bm, ix->Dp, ldG, ldB, ix->n, nblk, ix->qnorm64, rs);
            } else {
              knn_scan_f16_lq<2, 64, 8><<<g2, 512, lds, st>>>(qp, nqp, ix->d, ix->gh, gm, bm, ix->Dp, ldG, ldB, ix->n, nblk, ix->qnorm64, rs);
            }
          } else if (qt == 1) {
            if (ix->Dp % 128 == 0)
              knn_scan_f16_gmax<1, 128, 1, true><<<grid, 64, 0, st>>>(nullptr, qp, nqp, ix->d, ix->gh, gm, bm, ix->Dp, ldG, ldB, ix->n, rs);
            else
              knn_scan_f16_gmax<1, 64, 1, true><<<grid, 64, 0, st>>>(nullptr, qp, nqp, ix->d, ix->gh, gm, bm, ix->Dp, ldG, ldB, ix->n, rs);
          } else {
            knn_scan_f16_gmax<2, 64, 1, true><<<grid, 64, 0, st>>>(nullptr, qp, nqp, ix->d, ix->gh, gm, bm, ix->Dp, ldG, ldB, ix->n, rs);
          }
          MMR_LAUNCH_CHECK();
          launch_select<1, true, true>(st, pq, gm, ldG, ldG, ix, k, two_delta16r, qp, ix->qnorm64, oi + p0 * k,
                                       os ? os + p0 * k : nullptr, os64 ? os64 + p0 * k : nullptr,
                                       ost ? ost + p0 : nullptr, bm, ldB, two_delta16a, lq ? ix->qnorm64 : nullptr);
          MMR_LAUNCH_CHECK();
          continue;
        }
        // <= 32 queries whose rows are not 16-B aligned / d % 8 != 0: prep + the one-wave stream
        knn_prep_queries<<<dim3((unsigned)ceil_div(Qp, 4)), dim3(256), 0, st>>>(
            qp, pq, ix->d, ix->qn, ix->Dp, Qp, ix->qnorm64, 2);
        MMR_LAUNCH_CHECK();
        if (qt == 1) {
          if (ix->Dp % 128 == 0) knn_scan_f16_gmax<1, 128><<<grid, 64, 0, st>>>(qh, nullptr, 0, ix->d, ix->gh, gm, bm, ix->Dp, ldG, ldB, ix->n, rs);
          else knn_scan_f16_gmax<1, 64><<<grid, 64, 0, st>>>(qh, nullptr, 0, ix->d, ix->gh, gm, bm, ix->Dp, ldG, ldB, ix->n, rs);
        } else {
          if (ix->Dp % 128 == 0) knn_scan_f16_gmax<2, 128><<<grid, 64, 0, st>>>(qh, nullptr, 0, ix->d, ix->gh, gm, bm, ix->Dp, ldG, ldB, ix->n, rs);
          else knn_scan_f16_gmax<2, 64><<<grid, 64, 0, st>>>(qh, nullptr, 0, ix->d, ix->gh, gm, bm, ix->Dp, ldG, ldB, ix->n, rs);
        }
        MMR_LAUNCH_CHECK();
        launch_select<1, true>(st, pq, gm, ldG, ldG, ix, k, two_delta16, qp, ix->qnorm64, oi + p0 * k,
                               os ? os + p0 * k : nullptr, os64 ? os64 + p0 * k : nullptr, ost ? ost + p0 : nullptr,
                               bm, ldB);
        MMR_LAUNCH_CHECK();
      }
    } else if (ix->mode == 1 && cq <= kSkinnyMaxQ) {
      // skinny scan: HBM-streaming f32 MFMA, f32-mode delta
      const int qt = cq <= 16 ? 1 : cq <= 32 ? 2 : 4;
      const int64_t Qp = 16 * qt;
      knn_prep_queries<<<dim3((unsigned)ceil_div(Qp, 4)), dim3(256), 0, st>>>(
          qc, cq, ix->d, ix->qn, ix->Dp, Qp, ix->qnorm64, 1);
      MMR_LAUNCH_CHECK();
      const dim3 grid((unsigned)(ix->Np / 64));
      const int64_t ldG = ix->Np / 4;
      if (qt == 1)
        knn_scan_f32_gmax<1, 64><<<grid, 64, 0, st>>>(ix->qn, ix->gt, ix->inv_norm, ix->vals, ix->Dp, ldG, ix->n);
      else if (qt == 2)
        knn_scan_f32_gmax<2, 64><<<grid, 64, 0, st>>>(ix->qn, ix->gt, ix->inv_norm, ix->vals, ix->Dp, ldG, ix->n);
      else
        knn_scan_f32_gmax<4, 32><<<grid, 64, 0, st>>>(ix->qn, ix->gt, ix->inv_norm, ix->vals, ix->Dp, ldG, ix->n);
      MMR_LAUNCH_CHECK();
      launch_select<1>(st, cq, ix->vals, ldG, ldG, ix, k, two_delta32, qc, ix->qnorm64, oi, os, os64, ost);
      MMR_LAUNCH_CHECK();
    } else if (ix->mode == 1) {
      const int64_t Qp = round_up(cq, 128);
      knn_prep_queries<<<dim3((unsigned)ceil_div(Qp, 4)), dim3(256), 0, st>>>(
          qc, cq, ix->d, ix->qn, ix->Dp, Qp, ix->qnorm64);
      MMR_LAUNCH_CHECK();
      const int64_t total = Qp * ix->Dp;
      knn_split_queries<<<dim3((unsigned)ceil_div(total, 256)), dim3(256), 0, st>>>(ix->qn, ix->Dp, total, ix->qs);
      MMR_LAUNCH_CHECK();
      const int tiles_m = (int)(Qp / 128), tiles_n = (int)(ix->Np / 128);
      const int64_t ldG = ix->Np / 4;
      knn_scores_x3_gmax<<<dim3((unsigned)(tiles_m * tiles_n)), dim3(256), 0, st>>>(
          ix->qs, ix->gs, ix->inv_norm, ix->vals, ix->Dp, ldG, ix->n, tiles_m, tiles_n);
      MMR_LAUNCH_CHECK();
      launch_select<1>(st, cq, ix->vals, ldG, ldG, ix, k, two_delta3, qc, ix->qnorm64, oi, os, os64, ost);
      MMR_LAUNCH_CHECK();
    } else {
      int wq, wn;
      if (cq <= 64) { wq = 1; wn = 4; } else if (cq <= 128) { wq = 2; wn = 2; } else { wq = 4; wn = 1; }
      const int64_t Qp = round_up(cq, 64 * wq);
      knn_prep_queries<<<dim3((unsigned)ceil_div(Qp, 4)), dim3(256), 0, st>>>(
          qc, cq, ix->d, ix->qn, ix->Dp, Qp, ix->qnorm64);
      MMR_LAUNCH_CHECK();
      const int n_qblocks = (int)(Qp / (64 * wq));
      const int n_gtiles = (int)ceil_div(ix->Np, 64 * wn);
      const unsigned grid = (unsigned)(round_up(n_gtiles, 8) * n_qblocks);
      if (wq == 1)
        knn_scores<1, 4><<<grid, 256, 0, st>>>(ix->qn, ix->gal, ix->inv_norm, ix->vals, ix->Dp, ix->Np, n_gtiles, n_qblocks);
      else if (wq == 2)
        knn_scores<2, 2><<<grid, 256, 0, st>>>(ix->qn, ix->gal, ix->inv_norm, ix->vals, ix->Dp, ix->Np, n_gtiles, n_qblocks);
      else
        knn_scores<4, 1><<<grid, 256, 0, st>>>(ix->qn, ix->gal, ix->inv_norm, ix->vals, ix->Dp, ix->Np, n_gtiles, n_qblocks);
      MMR_LAUNCH_CHECK();
      launch_select<0>(st, cq, ix->vals, ix->Np, ix->n, ix, k, two_delta32, qc, ix->qnorm64, oi, os, os64, ost);
      MMR_LAUNCH_CHECK();
    }
  }
  ix->ws_stream = st;
  ix->ws_used = true;
  return MMR_OK;
}

mmr_status mmr_index_link_graph(mmr_index* ix, double threshold, int32_t max_links, int64_t row0,
                                 int64_t nrows, int64_t* out_nbr, int32_t* out_cnt, void* stream) {
  mmr::clear_error();
  MMR_REQUIRE(ix != nullptr, "mmr_index_link_graph: index is NULL");
  MMR_REQUIRE(max_links >= 1 && max_links < kMaxK, "mmr_index_link_graph: max_links=%d outside [1, %d)", max_links, kMaxK);
  MMR_REQUIRE(row0 >= 0 && nrows >= 0 && row0 + nrows <= ix->n, "mmr_index_link_graph: rows [%lld, +%lld) outside the gallery",
              (long long)row0, (long long)nrows);
  if (nrows == 0) return MMR_OK;
  MMR_REQUIRE(out_nbr && out_cnt, "mmr_index_link_graph: NULL output");
  DeviceGuard g(ix->device);
  hipStream_t st = mmr::as_stream(stream);
  const int k = max_links + 1;  // + the row itself
  int64_t* ti = nullptr;
  double* ts = nullptr;
  float* qc = nullptr;
  MMR_CHECK_HIP(hipMallocAsync((void**)&ti, sizeof(int64_t) * nrows * k, st));
  MMR_CHECK_HIP(hipMallocAsync((void**)&ts, sizeof(double) * nrows * k, st));
  const float* q = ix->gal ? ix->gal + row0 * ix->Dp : nullptr;  // padded rows double as queries when d == Dp
  if (ix->dtype == MMR_F16) {  // native fp16 rows -> f32 query rows (exact)
    MMR_CHECK_HIP(hipMallocAsync((void**)&qc, sizeof(float) * nrows * ix->d, st));
    knn_rows_from_f16<<<dim3((unsigned)ceil_div(nrows * ix->d, 256)), dim3(256), 0, st>>>(ix->gh, row0, nrows, ix->d,
                                                                                         ix->Dp, qc);
    MMR_LAUNCH_CHECK();
    q = qc;
  } else if (ix->d != ix->Dp) {
    MMR_CHECK_HIP(hipMallocAsync((void**)&qc, sizeof(float) * nrows * ix->d, st));
    MMR_CHECK_HIP(hipMemcpy2DAsync(qc, sizeof(float) * ix->d, q, sizeof(float) * ix->Dp, sizeof(float) * ix->d,
                                   nrows, hipMemcpyDeviceToDevice, st));
    q = qc;
  }
  mmr_status s = mmr_index_search(ix, q, nrows, k, ti, nullptr, ts, nullptr, stream);
  if (s == MMR_OK) {
    knn_link_filter<<<dim3((unsigned)ceil_div(nrows, 256)), dim3(256), 0, st>>>(
        ti, ts, k, nrows, row0, ix->idx_base, threshold, max_links, out_nbr, out_cnt);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
      mmr::set_error("knn_link_filter launch failed: %s", hipGetErrorString(e));
      s = MMR_ERR_HIP;
    }
  }
  (void)hipFreeAsync(ti, st);
  (void)hipFreeAsync(ts, st);
  if (qc) (void)hipFreeAsync(qc, st);
  return s;
}

mmr_status mmr_index_rerank(const mmr_index* ix, const float* q_emb, int64_t nq, const int64_t* cand,
                            int32_t kc, const uint64_t* q_labels, const uint64_t* g_labels, const float* q_kg,
                            const float* g_kg, int32_t dk, double alpha, double beta, double gamma,
                            int32_t topk, int64_t* out_idx, double* out_final, double* out_emb,
                            double* out_lab, double* out_kg, void* stream) {
  mmr::clear_error();
  MMR_REQUIRE(ix != nullptr, "mmr_index_rerank: index is NULL");
  MMR_REQUIRE(kc >= 1 && kc <= 64 && topk >= 1 && topk <= kc && dk >= 1 && nq >= 0,
              "mmr_index_rerank: kc=%d (1..64), topk=%d (1..kc), dk=%d", kc, topk, dk);
  if (nq == 0) return MMR_OK;
  MMR_REQUIRE(q_emb && cand && q_labels && g_labels && q_kg && g_kg && out_idx, "mmr_index_rerank: NULL pointer");
  DeviceGuard g(ix->device);
  knn_rerank<<<dim3((unsigned)nq), dim3(64), 0, mmr::as_stream(stream)>>>(
      q_emb, ix->d, ix->gal, ix->dtype == MMR_F16 ? ix->gh : nullptr, ix->Dp, ix->norm64, ix->n, ix->idx_base, cand, kc, q_labels, g_labels, q_kg,
      g_kg, dk, alpha, beta, gamma, topk, out_idx, out_final, out_emb, out_lab, out_kg);
  MMR_LAUNCH_CHECK();
  return MMR_OK;
}

mmr_status mmr_index_set_mode(mmr_index* ix, int32_t mode) {
  mmr::clear_error();
  MMR_REQUIRE(ix != nullptr && mode >= 0 && mode <= 2, "mmr_index_set_mode: bad arguments");
  std::lock_guard<std::mutex> lk(ix->mu);
  if (ix->dtype == MMR_F16 && mode != 2) {
    mmr::set_error("mmr_index_set_mode: a native fp16 index (MMR_F16) scans its fp16 rows only (mode 2)");
    return MMR_ERR_UNSUPPORTED;
  }
  if (mode == ix->mode && (mode != 1 || ix->gs != nullptr) && (mode != 2 || ix->gh != nullptr)) return MMR_OK;
  // the new mode's copies are built BEFORE the old mode's are freed: on a failure (e.g. an OOM on a
  // shard sized for fp16) the index stays in its previous mode with its copies intact, and only the
  // partial new copies are released (freeing first left mode 2 with a null gh)
  mmr_status s = mode == 1 ? build_x3_copies(ix) : mode == 2 ? build_f16_copies(ix) : MMR_OK;
  if (s != MMR_OK) {
    if (ix->mode != mode) free_copies(ix, mode == 1, mode == 2);
    return s;
  }
  free_copies(ix, mode != 1, mode != 2);
  ix->mode = mode;
  return MMR_OK;
}

mmr_status mmr_merge_topk(const double* scores, const int64_t* idx, int32_t n_lists, int64_t nq,
                          int32_t k_in, int32_t k_out, int64_t* out_idx, float* out_score,
                          double* out_score64, void* stream) {
  return mmr_merge_topk_payload(scores, idx, nullptr, 0, n_lists, nq, 0, nq, k_in, k_out, out_idx, out_score,
                                out_score64, nullptr, stream);
}

mmr_status mmr_merge_topk_payload(const double* scores, const int64_t* idx, const double* payload,
                                  int32_t payload_width, int32_t n_lists, int64_t nq_total, int64_t q0, int64_t nq,
                                  int32_t k_in, int32_t k_out, int64_t* out_idx, float* out_score,
                                  double* out_score64, double* out_payload, void* stream) {
  mmr::clear_error();
  MMR_REQUIRE(n_lists >= 1 && k_in >= 1 && k_out >= 1 && nq >= 0 && q0 >= 0 && q0 + nq <= nq_total,
              "mmr_merge_topk: bad sizes");
  MMR_REQUIRE((int64_t)n_lists * k_in <= 4096, "mmr_merge_topk: n_lists*k_in > 4096");
  MMR_REQUIRE(payload_width >= 0 && payload_width <= 16 && ((payload == nullptr) == (out_payload == nullptr)) &&
                  (payload == nullptr || payload_width > 0),
              "mmr_merge_topk_payload: payload / out_payload / width disagree");
  if (nq == 0) return MMR_OK;
  MMR_REQUIRE(scores && idx && out_idx, "mmr_merge_topk: NULL pointer");
  const size_t lds = (sizeof(double) + sizeof(int64_t)) * (size_t)n_lists * k_in;
  knn_merge<<<dim3((unsigned)nq), dim3(256), lds, mmr::as_stream(stream)>>>(
      scores, idx, n_lists, nq_total, q0, k_in, k_out, out_idx, out_score, out_score64, payload, payload_width,
      out_payload, 1, 1, payload_width);
  MMR_LAUNCH_CHECK();
  return MMR_OK;
}

mmr_status mmr_merge_topk_packed(const void* packed, int32_t payload_width, int32_t n_lists, int64_t nq_total,
                                 int64_t q0, int64_t nq, int32_t k_in, int32_t k_out, int64_t* out_idx,
                                 float* out_score, double* out_score64, double* out_payload, void* stream) {
  mmr::clear_error();
  MMR_REQUIRE(n_lists >= 1 && k_in >= 1 && k_out >= 1 && nq >= 0 && q0 >= 0 && q0 + nq <= nq_total,
              "mmr_merge_topk_packed: bad sizes");
  MMR_REQUIRE((int64_t)n_lists * k_in <= 4096, "mmr_merge_topk_packed: n_lists*k_in > 4096");
  MMR_REQUIRE(payload_width >= 0 && payload_width <= 16 && (out_payload == nullptr || payload_width > 0),
              "mmr_merge_topk_packed: payload width %d", payload_width);
  if (nq == 0) return MMR_OK;
  MMR_REQUIRE(packed && out_idx, "mmr_merge_topk_packed: NULL pointer");
  MMR_REQUIRE(((uintptr_t)packed & 7u) == 0, "mmr_merge_topk_packed: packed buffer must be 8-B aligned");
  const int64_t W = 2 + payload_width;
  const double* base = (const double*)packed;
  const size_t lds = (sizeof(double) + sizeof(int64_t)) * (size_t)n_lists * k_in;
  knn_merge<<<dim3((unsigned)nq), dim3(256), lds, mmr::as_stream(stream)>>>(
      base, (const int64_t*)(base + 1), n_lists, nq_total, q0, k_in, k_out, out_idx, out_score, out_score64,
      out_payload ? base + 2 : nullptr, payload_width, out_payload, W, W, W);
  MMR_LAUNCH_CHECK();
  return MMR_OK;
}

mmr_status mmr_index_rerank_components(const mmr_index* ix, const float* q_emb, int64_t nq, const int64_t* cand,
                                       int32_t kc, const uint64_t* q_labels, const uint64_t* g_labels,
                                       const float* q_kg, const float* g_kg, int32_t dk, double* out_comp,
                                       void* stream) {
  mmr::clear_error();
  MMR_REQUIRE(ix != nullptr, "mmr_index_rerank_components: index is NULL");
  MMR_REQUIRE(kc >= 1 && kc <= 64 && dk >= 1 && nq >= 0, "mmr_index_rerank_components: kc=%d (1..64), dk=%d", kc,
              dk);
  if (nq == 0) return MMR_OK;
  MMR_REQUIRE(q_emb && cand && q_labels && g_labels && q_kg && g_kg && out_comp,
              "mmr_index_rerank_components: NULL pointer");
  DeviceGuard g(ix->device);
  knn_rerank_comp<<<dim3((unsigned)nq), dim3(64), 0, mmr::as_stream(stream)>>>(
      q_emb, ix->d, ix->gal, ix->dtype == MMR_F16 ? ix->gh : nullptr, ix->Dp, ix->norm64, ix->n, ix->idx_base, cand, kc, q_labels, g_labels, q_kg, g_kg, dk,
      out_comp);
  MMR_LAUNCH_CHECK();
  return MMR_OK;
}

mmr_status mmr_rerank_mix(const int64_t* cand, const double* comp, int64_t nq, int32_t kc, double alpha,
                          double beta, double gamma, int32_t topk, int64_t* out_idx, double* out_final,
                          double* out_emb, double* out_lab, double* out_kg, void* stream) {
  mmr::clear_error();
  MMR_REQUIRE(kc >= 1 && kc <= 64 && topk >= 1 && topk <= kc && nq >= 0, "mmr_rerank_mix: kc=%d (1..64), topk=%d",
              kc, topk);
  if (nq == 0) return MMR_OK;
  MMR_REQUIRE(cand && comp && out_idx, "mmr_rerank_mix: NULL pointer");
  knn_rerank_mix<<<dim3((unsigned)nq), dim3(64), 0, mmr::as_stream(stream)>>>(
      cand, comp, kc, alpha, beta, gamma, topk, out_idx, out_final, out_emb, out_lab, out_kg);
  MMR_LAUNCH_CHECK();
  return MMR_OK;
}

}  // extern "C"
