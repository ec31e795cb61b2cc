// fp32-faithful (x3) fused Swin MLP sub-block for the narrow, memory-bound stages (C = 96, 192):
//   y = x + fc2(GELU(fc1(LN2(x))))            (timm SwinTransformerBlock, fusion.py:198-199)
// in f32 with both linears on bf16x3 MFMA (a.b ~= a_hi.b_hi + a_hi.b_lo + a_lo.b_hi, f32 accumulate) and
// torch's erf GELU (ocml erff), the 4C-wide hidden activation never leaving the CU.  The unfused x3
// chain (LayerNorm split pass -> fc1 GEMM writing the hidden as split rows -> fc2 GEMM + residual) moves
// 2 x 4 x 4C bytes of hidden per token through HBM and runs its short-K GEMMs at ~3.5 TB/s: at stage 1
// 1.17 ms per block for 355 GF of bf16 MFMA work.
// Structure (the bf16 streamed form of swin_mlp.hip on split operands): each wave owns 32 tokens,
// LayerNorms them in f32 registers (row split over the lane pair sharing a token) straight into the
// fc1 B operand as hi / lo fragments, and walks the hidden dimension 32 units at a time: fc1 in the
// C^T orientation on v_mfma_f32_32x32x16_bf16 (3 products per k-step, bias in the accumulator), GELU,
// the hidden split in registers into the hi / lo B operands of fc2 (C^T, A = W2 from LDS under the
// k-permutation w2_hidden mirrors).  Weights are split and repacked once at load into per-HC-hidden-
// unit chunks [W1_hi | W1_lo | W2_hi | W2_lo] — exact, bank-conflict-free LDS images — streamed through
// an R-deep LDS ring by global_load_lds and shared by the workgroup's 32 NW tokens.  The residual x is
// re-read (L2) in the epilogue; y is f32.
#include <algorithm>
#include <float.h>
#include <math.h>

#include "common.h"

namespace {

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;

constexpr int vmcnt_n(int n) { return (n & 15) | (7 << 4) | (15 << 8) | ((n >> 4) << 14); }

template <int C, int NW, int HC, int R>
struct X3MlpGeo {
  static constexpr int U1 = C / 8;        // 16-B units per W1 row
  static constexpr int U2 = HC / 8;       // 16-B units per W2 row (chunk columns)
  static constexpr int KS1 = C / 16;      // fc1 k-steps
  static constexpr int NU = C / 32;       // fc2 output tiles (32 channels)
  static constexpr int NT = HC / 32;      // 32-wide hidden tiles per chunk
  static constexpr int NCH = 4 * C / HC;  // chunks
  static constexpr int W1B = HC * C * 2;  // bytes of one bf16 image (W1 rows or W2 columns of a chunk)
  static constexpr int CHUNK_B = 4 * W1B;
  static constexpr int PW = CHUNK_B / 1024 / NW;  // glds pieces per wave per chunk
  static constexpr int TOK = 32 * NW;
  static constexpr int LDS_B = R * CHUNK_B;
  static_assert(CHUNK_B % (1024 * NW) == 0, "chunk must split evenly over the waves");
  static_assert(R == 2 || R == 3, "ring depth");
};

// f32 w1 [4C][C], w2 [C][4C] -> chunk images [W1_hi | W1_lo | W2_hi | W2_lo] (hi = bf16(w), lo = bf16(w - hi))
template <int C, int HC>
__global__ __launch_bounds__(256) void x3_swin_mlp_pack(const float* __restrict__ w1, const float* __restrict__ w2,
                                                        uint16_t* __restrict__ pack) {
  constexpr int W1E = HC * C, CE = 4 * W1E;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;  // destination element
  if (i >= (int64_t)16 * C * C) return;
  const int ch = (int)(i / CE), e = (int)(i % CE), part = e / W1E, e2 = e % W1E;
  float v;
  int dst;
  if (part < 2) {
    const int rr = e2 / C, k = e2 % C;
    dst = rr * C + 8 * mmr::unit_swz<C / 8>(rr, k >> 3) + (k & 7);
    v = w1[(int64_t)(HC * ch + rr) * C + k];
  } else {
    const int c = e2 / HC, pos = e2 % HC;
    dst = c * HC + 8 * mmr::unit_swz<HC / 8>(c, pos >> 3) + (pos & 7);
    v = w2[(int64_t)c * 4 * C + HC * ch + mmr::w2_hidden(pos)];
  }
  const uint16_t hi = mmr::f2bf(v);
  pack[(int64_t)ch * CE + part * W1E + dst] = (part & 1) ? mmr::f2bf(v - mmr::bf2f(hi)) : hi;
}

// GELU(erf) with erf by Abramowitz-Stegun 7.1.26 (mmr::gelu_erf: |erf err| <= 1.5e-7, one v_exp + one
// v_rcp, branch-free): the GELU's absolute error <= 0.75e-7 |x|, 100x below the x3 products' 2^-17.  ocml
// erff (a branchy polynomial) made the kernel VALU-bound: stage 1 615 vs 529 us, stage 2 587 vs 464 us at
// B = 256, the same max deviation from the unfused chain (profiles/r05_x3_mlp_ab.txt)
__device__ __forceinline__ float gelu_exact(float v) { return mmr::gelu_erf(v); }

// two f32 -> (hi, lo) packed bf16 pairs
__device__ __forceinline__ void split2(float a, float b, uint32_t& hi, uint32_t& lo) {
  hi = mmr::pack2bf(a, b);
  lo = mmr::pack2bf(a - __uint_as_float(hi << 16), b - __uint_as_float(hi & 0xFFFF0000u));
}

template <int C, int NW, int HC, int R>
__global__ __launch_bounds__(64 * NW) void x3_swin_mlp(const float* __restrict__ x, const float* __restrict__ lng,
                                                       const float* __restrict__ lnb, const uint16_t* __restrict__ pack,
                                                       const float* __restrict__ b1, const float* __restrict__ b2,
                                                       float* __restrict__ y, int64_t T, float eps) {
  using G = X3MlpGeo<C, NW, HC, R>;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];  // the weight ring only
  __shared__ __attribute__((aligned(16))) float Pg[6 * C];               // gamma | beta | b1
  const float* Pb = Pg + C;
  const float* Pb1 = Pg + 2 * C;

  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 31, h = lane >> 5;
  const int64_t tok = (int64_t)blockIdx.x * G::TOK + wave * 32 + r;
  const bool ok = tok < T;
  const float* xr = x + (ok ? tok : 0) * C;

  for (int i = threadIdx.x; i < 6 * C; i += 64 * NW)
    Pg[i] = i < C ? lng[i] : (i < 2 * C ? lnb[i - C] : b1[i - 2 * C]);
  // lane half h: columns 16 ks + 8 h .. + 7 of its token (clamped row: unconditional loads)
  f32x4 xv[2 * G::KS1];
#pragma unroll
  for (int ks = 0; ks < G::KS1; ++ks) {
    xv[2 * ks] = *(const f32x4*)(xr + 16 * ks + 8 * h);
    xv[2 * ks + 1] = *(const f32x4*)(xr + 16 * ks + 8 * h + 4);
  }

  auto stage = [&](int ch) {
    const unsigned char* src = (const unsigned char*)pack + (size_t)ch * G::CHUNK_B;
    unsigned char* dst = smem + (ch % R) * G::CHUNK_B;
#pragma unroll
    for (int p = 0; p < G::PW; ++p) {
      const int piece = wave * G::PW + p;
      __builtin_amdgcn_global_load_lds((const void*)(src + piece * 1024 + lane * 16), (lds_ptr_t)(dst + piece * 1024),
                                       16, 0, 0);
    }
  };
  stage(0);
  if constexpr (R == 3) stage(1);
  __builtin_amdgcn_s_waitcnt(vmcnt_n((R - 1) * G::PW));  // x and chunk 0 landed
  __builtin_amdgcn_s_waitcnt(0xC07F);                    // lgkmcnt(0): parameter stores landed
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  // LayerNorm (f32, two-pass, row split over the lane pair) -> the fc1 B operand as hi / lo fragments
  bf16x8 xh[G::KS1], xl[G::KS1];
  {
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < 2 * G::KS1; ++q) s += (xv[q][0] + xv[q][1]) + (xv[q][2] + xv[q][3]);
    s += __shfl_xor(s, 32, 64);
    const float mean = s * (1.0f / C);
    float ss = 0.f;
#pragma unroll
    for (int q = 0; q < 2 * G::KS1; ++q)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float d = xv[q][j] - mean;
        ss += d * d;
      }
    ss += __shfl_xor(ss, 32, 64);
    const float rstd = rsqrtf(ss * (1.0f / C) + eps);
#pragma unroll
    for (int ks = 0; ks < G::KS1; ++ks) {
      const int k0 = 16 * ks + 8 * h;
      uint32_t hh[4], ll[4];
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const f32x4 g4 = *(const f32x4*)(Pg + k0 + 4 * p), c4 = *(const f32x4*)(Pb + k0 + 4 * p);
        const f32x4 v = xv[2 * ks + p];
        split2((v[0] - mean) * rstd * g4[0] + c4[0], (v[1] - mean) * rstd * g4[1] + c4[1], hh[2 * p], ll[2 * p]);
        split2((v[2] - mean) * rstd * g4[2] + c4[2], (v[3] - mean) * rstd * g4[3] + c4[3], hh[2 * p + 1],
               ll[2 * p + 1]);
      }
      xh[ks] = __builtin_bit_cast(bf16x8, make_uint4(hh[0], hh[1], hh[2], hh[3]));
      xl[ks] = __builtin_bit_cast(bf16x8, make_uint4(ll[0], ll[1], ll[2], ll[3]));
    }
  }

  f32x16 acc2[G::NU];
#pragma unroll
  for (int u = 0; u < G::NU; ++u) acc2[u] = (f32x16){0};

  for (int ch = 0; ch < G::NCH; ++ch) {
    if (R == 3 && ch + 1 < G::NCH) __builtin_amdgcn_s_waitcnt(vmcnt_n(G::PW));  // chunk ch landed
    else __builtin_amdgcn_s_waitcnt(vmcnt_n(0));
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave's pieces landed; the slot refilled next is free
    asm volatile("" ::: "memory");
    if (ch + R - 1 < G::NCH) stage(ch + R - 1);
    const unsigned char* W1h = smem + (ch % R) * G::CHUNK_B;
    const unsigned char* W1l = W1h + G::W1B;
    const unsigned char* W2h = W1h + 2 * G::W1B;
    const unsigned char* W2l = W1h + 3 * G::W1B;
#pragma unroll
    for (int t = 0; t < G::NT; ++t) {  // 32 hidden units per step
      f32x16 a1;  // starts at fc1's bias (lane: hidden HC ch + 32 t + 8 i + 4 h + rr of token r)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const f32x4 bb = *(const f32x4*)(Pb1 + HC * ch + 32 * t + 8 * i + 4 * h);
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) a1[4 * i + rr] = bb[rr];
      }
      const int row = 32 * t + r;
#pragma unroll
      for (int ks = 0; ks < G::KS1; ++ks) {
        const int off = (row * G::U1 + mmr::unit_swz<G::U1>(row, 2 * ks + h)) * 16;
        const bf16x8 wh = *(const bf16x8*)(W1h + off), wl = *(const bf16x8*)(W1l + off);
        a1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh, xh[ks], a1, 0, 0, 0);
        a1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh, xl[ks], a1, 0, 0, 0);
        a1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wl, xh[ks], a1, 0, 0, 0);
      }
      uint32_t hph[8], hpl[8];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        split2(gelu_exact(a1[4 * i]), gelu_exact(a1[4 * i + 1]), hph[2 * i], hpl[2 * i]);
        split2(gelu_exact(a1[4 * i + 2]), gelu_exact(a1[4 * i + 3]), hph[2 * i + 1], hpl[2 * i + 1]);
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {  // k-step over hidden 32 t + 16 s2 .. + 15
        const bf16x8 hfh = __builtin_bit_cast(bf16x8, make_uint4(hph[4 * s2], hph[4 * s2 + 1], hph[4 * s2 + 2],
                                                                 hph[4 * s2 + 3]));
        const bf16x8 hfl = __builtin_bit_cast(bf16x8, make_uint4(hpl[4 * s2], hpl[4 * s2 + 1], hpl[4 * s2 + 2],
                                                                 hpl[4 * s2 + 3]));
        const int q = 2 * (2 * t + s2) + h;
#pragma unroll
        for (int u = 0; u < G::NU; ++u) {
          const int c = 32 * u + r;
          const int off = (c * G::U2 + mmr::unit_swz<G::U2>(c, q)) * 16;
          const bf16x8 wh = *(const bf16x8*)(W2h + off), wl = *(const bf16x8*)(W2l + off);
          acc2[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh, hfh, acc2[u], 0, 0, 0);
          acc2[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh, hfl, acc2[u], 0, 0, 0);
          acc2[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wl, hfh, acc2[u], 0, 0, 0);
        }
      }
    }
  }

  // y[tok][c] = x + (fc2 + b2), c = 32 u + 8 i + 4 h + rr: each 32-channel slice of the wave's 32
  // (consecutive) tokens staged through the then idle weight ring, so the residual re-read and the
  // store move whole 128-B row segments (8 per instruction) instead of 32 scattered 16-B pieces
  __builtin_amdgcn_s_waitcnt(vmcnt_n(0));
  __syncthreads();  // every wave done with the ring
  float* sw = (float*)smem + wave * 32 * 36;
  const int64_t tok0 = (int64_t)blockIdx.x * G::TOK + wave * 32;
#pragma unroll
  for (int u = 0; u < G::NU; ++u) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = 32 * u + 8 * i + 4 * h;
      const f32x4 bb = *(const f32x4*)(b2 + c);
      f32x4 v;
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) v[rr] = acc2[u][4 * i + rr] + bb[rr];
      *(f32x4*)(sw + r * 36 + 8 * i + 4 * h) = v;
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the slice is in LDS
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int k = 0; k < 4; ++k) {  // lane: token 8 k + lane / 8, channels 4 (lane % 8) .. + 3 of the slice
      const int t = 8 * k + (lane >> 3), c4 = (lane & 7) * 4;
      if (tok0 + t < T) {
        const int64_t o = (tok0 + t) * C + 32 * u + c4;
        const f32x4 xq = *(const f32x4*)(x + o);
        *(f32x4*)(y + o) = *(const f32x4*)(sw + t * 36 + c4) + xq;
      }
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_wave_barrier();
  }
}

// ------------------------------------------------------------------ x3 row-linear (narrow Swin stages)
// y = LN?(x) W^T + b (+ r) for the short-K Swin linears of stages 1-2 (C = 96 / 192: qkv N = 3C with the
// block's norm1 fused, proj N = C + residual reading the window attention's split-row output), whose
// K' = 3 kp split GEMMs on the 8-phase kernel run HBM-bound at ~3.5 TB/s with padded tiles (stage-1 qkv
// N 288 -> 384, proj N 96 -> 192).  The MLP kernel's structure without the hidden: each wave LayerNorms
// (or loads as split rows) its 32 tokens into the hi / lo B operand in registers, and walks the output
// features 32 at a time against W^T chunks [W_hi 64 x C | W_lo 64 x C] streamed through an R-deep LDS
// ring (bias in the accumulator; f32 output rows, the residual added in the epilogue).
template <int C, int NW, int R>
struct X3RowGeo {
  static constexpr int U1 = C / 8, KS1 = C / 16;
  static constexpr int WB = 64 * C * 2;  // one bf16 image of a 64-row chunk
  static constexpr int CHUNK_B = 2 * WB;
  static constexpr int PW = CHUNK_B / 1024 / NW;
  static constexpr int TOK = 32 * NW;
  static constexpr int LDS_B = R * CHUNK_B;
  static_assert(CHUNK_B % (1024 * NW) == 0, "chunk must split evenly over the waves");
};

// f32 W [n][C] -> 64-row chunks [W_hi | W_lo] (rows >= n zero), the fc1 image layout of the MLP pack
template <int C>
__global__ __launch_bounds__(256) void x3_rowlin_pack(const float* __restrict__ w, uint16_t* __restrict__ pack, int n,
                                                      int64_t total) {
  constexpr int WE = 64 * C;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int ch = (int)(i / (2 * WE)), e = (int)(i % (2 * WE)), part = e / WE, e2 = e % WE;
  const int rr = e2 / C, k = e2 % C;
  const int row = 64 * ch + rr;
  const float v = row < n ? w[(int64_t)row * C + k] : 0.f;
  const uint16_t hi = mmr::f2bf(v);
  pack[(int64_t)ch * 2 * WE + part * WE + rr * C + 8 * mmr::unit_swz<C / 8>(rr, k >> 3) + (k & 7)] =
      part ? mmr::f2bf(v - mmr::bf2f(hi)) : hi;
}

template <int C, int NW, int R, bool LN, bool RES>
__global__ __launch_bounds__(64 * NW) void x3_rowlin(const float* __restrict__ x, const uint16_t* __restrict__ xs,
                                                     int kp, const float* __restrict__ lng, const float* __restrict__ lnb,
                                                     const uint16_t* __restrict__ pack, const float* __restrict__ bias,
                                                     const float* __restrict__ res, float* __restrict__ y, int64_t T,
                                                     int N, float eps) {
  using G = X3RowGeo<C, NW, R>;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];  // ring | bias [N] | gamma, beta
  float* Pbias = (float*)(smem + G::LDS_B);
  float* Pg = Pbias + N;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 31, h = lane >> 5;
  const int64_t tok = (int64_t)blockIdx.x * G::TOK + wave * 32 + r;
  const bool ok = tok < T;
  const int64_t tk = ok ? tok : 0;
  const int nch = (N + 63) / 64;

  for (int i = threadIdx.x; i < N; i += 64 * NW) Pbias[i] = bias[i];
  if constexpr (LN)
    for (int i = threadIdx.x; i < 2 * C; i += 64 * NW) Pg[i] = i < C ? lng[i] : lnb[i - C];
  bf16x8 xh[G::KS1], xl[G::KS1];
  f32x4 xv[LN ? 2 * G::KS1 : 1];
  if constexpr (LN) {
#pragma unroll
    for (int ks = 0; ks < G::KS1; ++ks) {
      xv[2 * ks] = *(const f32x4*)(x + tk * C + 16 * ks + 8 * h);
      xv[2 * ks + 1] = *(const f32x4*)(x + tk * C + 16 * ks + 8 * h + 4);
    }
  } else {
#pragma unroll
    for (int ks = 0; ks < G::KS1; ++ks) {
      xh[ks] = *(const bf16x8*)(xs + tk * 2 * kp + 16 * ks + 8 * h);
      xl[ks] = *(const bf16x8*)(xs + tk * 2 * kp + kp + 16 * ks + 8 * h);
    }
  }
  auto stage = [&](int ch) {
    const unsigned char* src = (const unsigned char*)pack + (size_t)ch * G::CHUNK_B;
    unsigned char* dst = smem + (ch % R) * G::CHUNK_B;
#pragma unroll
    for (int p = 0; p < G::PW; ++p) {
      const int piece = wave * G::PW + p;
      __builtin_amdgcn_global_load_lds((const void*)(src + piece * 1024 + lane * 16), (lds_ptr_t)(dst + piece * 1024),
                                       16, 0, 0);
    }
  };
  // (nch >= R - 1 is required by the launcher: every issued stage is waited for below)
  stage(0);
  if constexpr (R == 3) stage(1);
  __builtin_amdgcn_s_waitcnt(vmcnt_n((R - 1) * G::PW));  // x and chunk 0 landed
  __builtin_amdgcn_s_waitcnt(0xC07F);
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  if constexpr (LN) {
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < 2 * G::KS1; ++q) s += (xv[q][0] + xv[q][1]) + (xv[q][2] + xv[q][3]);
    s += __shfl_xor(s, 32, 64);
    const float mean = s * (1.0f / C);
    float ss = 0.f;
#pragma unroll
    for (int q = 0; q < 2 * G::KS1; ++q)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float d = xv[q][j] - mean;
        ss += d * d;
      }
    ss += __shfl_xor(ss, 32, 64);
    const float rstd = rsqrtf(ss * (1.0f / C) + eps);
#pragma unroll
    for (int ks = 0; ks < G::KS1; ++ks) {
      const int k0 = 16 * ks + 8 * h;
      uint32_t hh[4], ll[4];
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const f32x4 g4 = *(const f32x4*)(Pg + k0 + 4 * p), c4 = *(const f32x4*)(Pg + C + k0 + 4 * p);
        const f32x4 v = xv[2 * ks + p];
        split2((v[0] - mean) * rstd * g4[0] + c4[0], (v[1] - mean) * rstd * g4[1] + c4[1], hh[2 * p], ll[2 * p]);
        split2((v[2] - mean) * rstd * g4[2] + c4[2], (v[3] - mean) * rstd * g4[3] + c4[3], hh[2 * p + 1],
               ll[2 * p + 1]);
      }
      xh[ks] = __builtin_bit_cast(bf16x8, make_uint4(hh[0], hh[1], hh[2], hh[3]));
      xl[ks] = __builtin_bit_cast(bf16x8, make_uint4(ll[0], ll[1], ll[2], ll[3]));
    }
  }
  for (int ch = 0; ch < nch; ++ch) {
    if (R == 3 && ch + 1 < nch) __builtin_amdgcn_s_waitcnt(vmcnt_n(G::PW));  // chunk ch landed
    else __builtin_amdgcn_s_waitcnt(vmcnt_n(0));
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (ch + R - 1 < nch) stage(ch + R - 1);
    const unsigned char* Wh = smem + (ch % R) * G::CHUNK_B;
    const unsigned char* Wl = Wh + G::WB;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int u = 2 * ch + t;
      if (32 * u >= N) break;  // wave-uniform (N % 32 == 0)
      f32x16 acc;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const f32x4 bb = *(const f32x4*)(Pbias + 32 * u + 8 * i + 4 * h);
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) acc[4 * i + rr] = bb[rr];
      }
      const int row = 32 * t + r;
#pragma unroll
      for (int ks = 0; ks < G::KS1; ++ks) {
        const int off = (row * G::U1 + mmr::unit_swz<G::U1>(row, 2 * ks + h)) * 16;
        const bf16x8 wh = *(const bf16x8*)(Wh + off), wl = *(const bf16x8*)(Wl + off);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh, xh[ks], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh, xl[ks], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wl, xh[ks], acc, 0, 0, 0);
      }
      // lane: channels 32 u + 8 i + 4 h + rr of token r
      if (ok) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int c = 32 * u + 8 * i + 4 * h;
          f32x4 v = {acc[4 * i], acc[4 * i + 1], acc[4 * i + 2], acc[4 * i + 3]};
          if constexpr (RES) v += *(const f32x4*)(res + tok * N + c);
          *(f32x4*)(y + tok * N + c) = v;
        }
      }
    }
  }
}

template <int C, int HC>
mmr_status launch_x3_pack(const float* w1, const float* w2, uint16_t* pack, hipStream_t st) {
  const int64_t n = (int64_t)16 * C * C;
  x3_swin_mlp_pack<C, HC><<<dim3((unsigned)mmr::ceil_div(n, 256)), 256, 0, st>>>(w1, w2, pack);
  MMR_LAUNCH_CHECK();
  return MMR_OK;
}

template <int C, int NW, int HC, int R>
mmr_status launch_x3_mlp(const float* x, const float* g, const float* b, const uint16_t* pack, const float* b1,
                         const float* b2, float* y, int64_t T, float eps, hipStream_t st) {
  using G = X3MlpGeo<C, NW, HC, R>;
  const dim3 grid((unsigned)mmr::ceil_div(T, G::TOK));
  x3_swin_mlp<C, NW, HC, R><<<grid, 64 * NW, G::LDS_B, st>>>(x, g, b, pack, b1, b2, y, T, eps);
  MMR_LAUNCH_CHECK();
  return MMR_OK;
}

constexpr int X3MLP_HC = 32;

template <int C, bool LN, bool RES>
mmr_status launch_rowlin(const float* x, const uint16_t* xs, int kp, const float* g, const float* b,
                         const uint16_t* pack, const float* bias, const float* res, float* y, int64_t T, int N,
                         float eps, hipStream_t st) {
  constexpr int R = C == 96 ? 3 : 2;
  using G = X3RowGeo<C, 8, R>;
  const size_t lds = G::LDS_B + (size_t)(N + 2 * C) * 4;
  x3_rowlin<C, 8, R, LN, RES><<<dim3((unsigned)mmr::ceil_div(T, G::TOK)), 512, lds, st>>>(x, xs, kp, g, b, pack, bias,
                                                                                         res, y, T, N, eps);
  MMR_LAUNCH_CHECK();
  return MMR_OK;
}

// ------------------------------------------------------------------ x3 patch embed (the Swin stem)
// y = LayerNorm(conv4x4/s4(img) + b) for timm's PatchEmbed (Conv2d(3, 96, 4, 4) + LayerNorm(96), reached
// through fusion.py:198-199) in f32, the conv on bf16x3 MFMA, in one pass: the unfused x3 stem wrote the
// im2col rows (4 B x 64 per token), re-read them in a 128 x 128-tile GEMM with N = 96 (25 % of each tile
// idle, column stores) and ran the LayerNorm as a third pass (56 + 228 + 128 us at B = 256).  Each wave
// owns 32 tokens (the N side of v_mfma_f32_32x32x16_bf16, C^T orientation): for k-step s (= input
// channel s, k = 16 s + 4 ky + kx, PyTorch's flattened conv weight order) lane (token r, half h) loads
// the two 16-B pixel rows ky = 2h, 2h + 1 of its patch — exactly its 8 B-operand k values — and splits
// them into hi / lo fragments; A = the weight image in fragment order (LDS, 18 KB, [hi | lo]); bias in
// the accumulators; the LayerNorm over the 96 outputs a lane pair holds (two-pass, f32), 16-B stores.
constexpr int PE_E = 96, PE_K = 48;
constexpr int PE_IMG_E = 3 * 3 * 64 * 8;  // bf16 per image: (3 output tiles x 3 k-steps) fragments

__global__ __launch_bounds__(256) void x3_patch_embed_pack(const float* __restrict__ w, uint16_t* __restrict__ pack) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= PE_IMG_E) return;
  const int j = i & 7, l = (i >> 3) & 63, f = i >> 9, u = f / 3, s = f % 3;
  const float v = w[(32 * u + (l & 31)) * PE_K + 16 * s + 8 * (l >> 5) + j];
  const uint16_t hi = mmr::f2bf(v);
  pack[i] = hi;
  pack[PE_IMG_E + i] = mmr::f2bf(v - mmr::bf2f(hi));
}

// X3 = false: the bf16 towers' stem — one product of the bf16-rounded pixels with the hi image (= the
// bf16 weight), the bias and LayerNorm on the f32 accumulators (no bf16 rounding of the conv output in
// between), bf16 tokens out; replaces im2col + GEMM + LayerNorm (39 + 49 + 43 us at B = 256).
template <int NW, bool X3>
__global__ __launch_bounds__(64 * NW, 4) void x3_patch_embed_ln(const float* __restrict__ img,
                                                             const uint16_t* __restrict__ pack,
                                                             const float* __restrict__ bias,
                                                             const float* __restrict__ lng,
                                                             const float* __restrict__ lnb, void* __restrict__ yv,
                                                             int64_t ntile, int hw, float eps) {
  __shared__ __attribute__((aligned(16))) uint16_t W[2 * PE_IMG_E];
  __shared__ __attribute__((aligned(16))) float Pp[3 * PE_E];  // bias | gamma | beta
  // per wave: one 32-channel slice of its 32 tokens' outputs (row stride 36 f32: conflict-free 16-B
  // writes), written back as whole 128-B (f32) / 64-B (bf16) row segments — the tile's rows are
  // consecutive tokens, so each store instruction covers 8 / 16 complete segments instead of 32
  // scattered 16-B (f32) / 8-B (bf16) pieces
  __shared__ __attribute__((aligned(16))) float stg[NW][32 * 36];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 31, h = lane >> 5;
  for (int i = threadIdx.x; i < 2 * PE_IMG_E / 8; i += 64 * NW) ((uint4*)W)[i] = ((const uint4*)pack)[i];
  for (int i = threadIdx.x; i < 3 * PE_E; i += 64 * NW)
    Pp[i] = i < PE_E ? bias[i] : (i < 2 * PE_E ? lng[i - PE_E] : lnb[i - 2 * PE_E]);
  __syncthreads();
  const int g = hw / 4, per_img = g * g;
  for (int64_t tile = (int64_t)blockIdx.x * NW + wave; tile < ntile; tile += (int64_t)gridDim.x * NW) {
    const int64_t tok = tile * 32 + r;
    const int64_t b = tok / per_img;
    const int p = (int)(tok - b * per_img), py = p / g, px = p - py * g;
    const float* base = img + ((b * 3) * hw + 4 * py + 2 * h) * (int64_t)hw + 4 * px;
    f32x4 xv[3][2];
#pragma unroll
    for (int s = 0; s < 3; ++s)
#pragma unroll
      for (int j = 0; j < 2; ++j) xv[s][j] = *(const f32x4*)(base + ((int64_t)s * hw + j) * hw);
    bf16x8 xh[3], xl[3];
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      uint32_t hh[4], ll[4];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        split2(xv[s][j][0], xv[s][j][1], hh[2 * j], ll[2 * j]);
        split2(xv[s][j][2], xv[s][j][3], hh[2 * j + 1], ll[2 * j + 1]);
      }
      xh[s] = __builtin_bit_cast(bf16x8, make_uint4(hh[0], hh[1], hh[2], hh[3]));
      xl[s] = __builtin_bit_cast(bf16x8, make_uint4(ll[0], ll[1], ll[2], ll[3]));
    }
    f32x16 acc[3];
    // an opaque per-tile zero on the weight-image address: hipcc otherwise hoists the 18 loop-invariant
    // fragment reads out of the tile loop (72 more VGPRs live: 1 wave per SIMD)
    int wz = 0;
    asm volatile("" : "+v"(wz));
#pragma unroll
    for (int u = 0; u < 3; ++u) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const f32x4 bb = *(const f32x4*)(Pp + 32 * u + 8 * i + 4 * h);
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) acc[u][4 * i + rr] = bb[rr];
      }
#pragma unroll
      for (int s = 0; s < 3; ++s) {
        const bf16x8 wh = *(const bf16x8*)(W + wz + ((u * 3 + s) * 64 + lane) * 8);
        const bf16x8 wl = *(const bf16x8*)(W + wz + PE_IMG_E + ((u * 3 + s) * 64 + lane) * 8);
        acc[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh, xh[s], acc[u], 0, 0, 0);
        if constexpr (X3) {
          acc[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh, xl[s], acc[u], 0, 0, 0);
          acc[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wl, xh[s], acc[u], 0, 0, 0);
        }
      }
    }
    // LayerNorm over the token's 96 outputs (lane half h holds 48 of them: channels 32 u + 8 i + 4 h + rr)
    float sm = 0.f;
#pragma unroll
    for (int u = 0; u < 3; ++u)
#pragma unroll
      for (int e = 0; e < 16; ++e) sm += acc[u][e];
    sm += __shfl_xor(sm, 32, 64);
    const float mean = sm * (1.0f / PE_E);
    float ss = 0.f;
#pragma unroll
    for (int u = 0; u < 3; ++u)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const float d = acc[u][e] - mean;
        ss += d * d;
      }
    ss += __shfl_xor(ss, 32, 64);
    const float rstd = rsqrtf(ss * (1.0f / PE_E) + eps);
    float* sw = stg[wave];
    const int64_t tok0 = tile * 32;
#pragma unroll
    for (int u = 0; u < 3; ++u) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = 32 * u + 8 * i + 4 * h;
        const f32x4 g4 = *(const f32x4*)(Pp + PE_E + c), b4 = *(const f32x4*)(Pp + 2 * PE_E + c);
        f32x4 v;
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) v[rr] = (acc[u][4 * i + rr] - mean) * rstd * g4[rr] + b4[rr];
        *(f32x4*)(sw + r * 36 + 8 * i + 4 * h) = v;
      }
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the slice is in LDS
      __builtin_amdgcn_wave_barrier();
      if constexpr (X3) {  // lane: token 8 k + lane / 8, channels 4 (lane % 8) .. + 3 of the slice
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int t = 8 * k + (lane >> 3), c4 = (lane & 7) * 4;
          *(f32x4*)((float*)yv + (tok0 + t) * PE_E + 32 * u + c4) = *(const f32x4*)(sw + t * 36 + c4);
        }
      } else {  // lane: token 16 k + lane / 4, channels 8 (lane % 4) .. + 7
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const int t = 16 * k + (lane >> 2), c8 = (lane & 3) * 8;
          const f32x4 a = *(const f32x4*)(sw + t * 36 + c8), b2 = *(const f32x4*)(sw + t * 36 + c8 + 4);
          *(uint4*)((uint16_t*)yv + (tok0 + t) * PE_E + 32 * u + c8) =
              make_uint4(mmr::pack2bf(a[0], a[1]), mmr::pack2bf(a[2], a[3]), mmr::pack2bf(b2[0], b2[1]),
                         mmr::pack2bf(b2[2], b2[3]));
        }
      }
      __builtin_amdgcn_s_waitcnt(0xC07F);  // this slice's reads done before the next slice's writes
      __builtin_amdgcn_wave_barrier();
    }
  }
}

}  // namespace

extern "C" {

int64_t mmr_x3_swin_mlp_pack_elems(int32_t c) { return (c == 96 || c == 192) ? (int64_t)16 * c * c : 0; }

mmr_status mmr_x3_swin_mlp_pack(const float* w1, const float* w2, uint16_t* pack, int32_t c, void* stream) {
  mmr::clear_error();
  MMR_REQUIRE(w1 && w2 && pack, "mmr_x3_swin_mlp_pack: NULL pointer");
  hipStream_t st = mmr::as_stream(stream);
  if (c == 96) return launch_x3_pack<96, X3MLP_HC>(w1, w2, pack, st);
  if (c == 192) return launch_x3_pack<192, X3MLP_HC>(w1, w2, pack, st);
  mmr::set_error("mmr_x3_swin_mlp_pack: C=%d not built (96, 192)", c);
  return MMR_ERR_UNSUPPORTED;
}

mmr_status mmr_x3_swin_mlp(const float* x, const float* ln_g, const float* ln_b, const uint16_t* pack, const float* b1,
                           const float* b2, float* y, int64_t tokens, int32_t c, float eps, void* stream) {
  mmr::clear_error();
  MMR_REQUIRE(x && ln_g && ln_b && pack && b1 && b2 && y, "mmr_x3_swin_mlp: NULL pointer");
  MMR_REQUIRE(tokens >= 0 && x != y, "mmr_x3_swin_mlp: tokens < 0 or in place");
  MMR_REQUIRE(((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 15) == 0 && ((uintptr_t)b2 & 15) == 0,
              "mmr_x3_swin_mlp: x / y / b2 must be 16-B aligned");
  if (tokens == 0) return MMR_OK;
  hipStream_t st = mmr::as_stream(stream);
  if (c == 96) {
    // 4-wave workgroups, two per CU (their chunk barriers and prologue / epilogue latencies independent):
    // 491 vs 516 us for the 8-wave one at stage 1, B = 256 (profiles/r06_x3_mlp_walk_ab.txt); a test / A-B
    // pins the 8-wave form through mmr_pin_variant
    if (mmr::pin_x3_mlp.load(std::memory_order_relaxed) == 0)
      return launch_x3_mlp<96, 8, X3MLP_HC, 3>(x, ln_g, ln_b, pack, b1, b2, y, tokens, eps, st);
    return launch_x3_mlp<96, 4, X3MLP_HC, 3>(x, ln_g, ln_b, pack, b1, b2, y, tokens, eps, st);
  }
  if (c == 192) return launch_x3_mlp<192, 8, X3MLP_HC, 2>(x, ln_g, ln_b, pack, b1, b2, y, tokens, eps, st);
  mmr::set_error("mmr_x3_swin_mlp: C=%d not built (96, 192)", c);
  return MMR_ERR_UNSUPPORTED;
}

int64_t mmr_x3_rowlin_pack_elems(int32_t n, int32_t c) {
  return (c == 96 || c == 192) && n > 0 && n % 32 == 0 && n <= 4096 ? (int64_t)(n + 63) / 64 * 128 * c : 0;
}

mmr_status mmr_x3_rowlin_pack(const float* w, uint16_t* pack, int32_t n, int32_t c, void* stream) {
  mmr::clear_error();
  const int64_t total = mmr_x3_rowlin_pack_elems(n, c);
  MMR_REQUIRE(w && pack, "mmr_x3_rowlin_pack: NULL pointer");
  if (total <= 0) {
    mmr::set_error("mmr_x3_rowlin_pack: n=%d c=%d not built (c 96 / 192, n %% 32 == 0, n <= 4096)", n, c);
    return MMR_ERR_UNSUPPORTED;
  }
  const dim3 grid((unsigned)mmr::ceil_div(total, 256));
  hipStream_t st = mmr::as_stream(stream);
  if (c == 96) x3_rowlin_pack<96><<<grid, 256, 0, st>>>(w, pack, n, total);
  else x3_rowlin_pack<192><<<grid, 256, 0, st>>>(w, pack, n, total);
  MMR_LAUNCH_CHECK();
  return MMR_OK;
}

mmr_status mmr_x3_rowlin(const float* x, const uint16_t* xs, const float* ln_g, const float* ln_b, const uint16_t* pack,
                         const float* bias, const float* residual, float* y, int64_t tokens, int32_t n, int32_t c,
                         float eps, void* stream) {
  mmr::clear_error();
  MMR_REQUIRE(mmr_x3_rowlin_pack_elems(n, c) > 0, "mmr_x3_rowlin: n=%d c=%d not built", n, c);
  MMR_REQUIRE((x != nullptr) != (xs != nullptr), "mmr_x3_rowlin: exactly one of x (f32 rows) / xs (split rows)");
  MMR_REQUIRE(!x || (ln_g && ln_b), "mmr_x3_rowlin: f32 rows are taken with their LayerNorm");
  MMR_REQUIRE(pack && bias && y && tokens >= 0 && y != residual && (const void*)y != (const void*)x,
              "mmr_x3_rowlin: bad arguments");
  auto al = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  MMR_REQUIRE(al(x) && al(xs) && al(y) && al(residual) && al(bias), "mmr_x3_rowlin: 16-B aligned pointers");
  MMR_REQUIRE(c != 96 || n > 64, "mmr_x3_rowlin: c=96 takes n > 64 (its 3-deep weight ring)");
  if (tokens == 0) return MMR_OK;
  hipStream_t st = mmr::as_stream(stream);
  const int kp = mmr_x3_p8_kpad(c);
  if (c == 96) {
    if (x) return residual ? launch_rowlin<96, true, true>(x, xs, kp, ln_g, ln_b, pack, bias, residual, y, tokens, n, eps, st)
                           : launch_rowlin<96, true, false>(x, xs, kp, ln_g, ln_b, pack, bias, residual, y, tokens, n, eps, st);
    return residual ? launch_rowlin<96, false, true>(x, xs, kp, ln_g, ln_b, pack, bias, residual, y, tokens, n, eps, st)
                    : launch_rowlin<96, false, false>(x, xs, kp, ln_g, ln_b, pack, bias, residual, y, tokens, n, eps, st);
  }
  if (x) return residual ? launch_rowlin<192, true, true>(x, xs, kp, ln_g, ln_b, pack, bias, residual, y, tokens, n, eps, st)
                         : launch_rowlin<192, true, false>(x, xs, kp, ln_g, ln_b, pack, bias, residual, y, tokens, n, eps, st);
  return residual ? launch_rowlin<192, false, true>(x, xs, kp, ln_g, ln_b, pack, bias, residual, y, tokens, n, eps, st)
                  : launch_rowlin<192, false, false>(x, xs, kp, ln_g, ln_b, pack, bias, residual, y, tokens, n, eps, st);
}

int64_t mmr_x3_patch_embed_pack_elems(void) { return 2 * PE_IMG_E; }

mmr_status mmr_x3_patch_embed_pack(const float* w, uint16_t* pack, void* stream) {
  mmr::clear_error();
  MMR_REQUIRE(w && pack, "mmr_x3_patch_embed_pack: NULL pointer");
  x3_patch_embed_pack<<<dim3((unsigned)mmr::ceil_div(PE_IMG_E, 256)), 256, 0, mmr::as_stream(stream)>>>(w, pack);
  MMR_LAUNCH_CHECK();
  return MMR_OK;
}

static mmr_status patch_embed_ln(const char* who, bool x3, const float* img, int32_t b, int32_t hw,
                                 const uint16_t* pack, const float* bias, const float* ln_g, const float* ln_b,
                                 float eps, void* y, void* stream) {
  mmr::clear_error();
  MMR_REQUIRE(img && pack && bias && ln_g && ln_b && y, "%s: NULL pointer", who);
  MMR_REQUIRE(b >= 0 && hw > 0 && hw % 4 == 0 && ((hw / 4) * (hw / 4)) % 32 == 0,
              "%s: b=%d hw=%d (hw %% 4 == 0, (hw/4)^2 %% 32 == 0)", who, b, hw);
  auto al = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  MMR_REQUIRE(al(img) && al(y) && al(bias) && al(ln_g) && al(ln_b) && al(pack), "%s: 16-B aligned pointers", who);
  if (b == 0) return MMR_OK;
  const int64_t ntile = (int64_t)b * (hw / 4) * (hw / 4) / 32;
  const int64_t grid = std::min<int64_t>(2048, mmr::ceil_div(ntile, 4));
  if (x3)
    x3_patch_embed_ln<4, true><<<dim3((unsigned)grid), 256, 0, mmr::as_stream(stream)>>>(img, pack, bias, ln_g, ln_b, y,
                                                                                        ntile, hw, eps);
  else
    x3_patch_embed_ln<4, false><<<dim3((unsigned)grid), 256, 0, mmr::as_stream(stream)>>>(img, pack, bias, ln_g, ln_b, y,
                                                                                         ntile, hw, eps);
  MMR_LAUNCH_CHECK();
  return MMR_OK;
}

mmr_status mmr_x3_patch_embed_ln(const float* img, int32_t b, int32_t hw, const uint16_t* pack, const float* bias,
                                 const float* ln_g, const float* ln_b, float eps, float* y, void* stream) {
  return patch_embed_ln("mmr_x3_patch_embed_ln", true, img, b, hw, pack, bias, ln_g, ln_b, eps, y, stream);
}

mmr_status mmr_patch_embed_ln_bf16(const float* img, int32_t b, int32_t hw, const uint16_t* pack, const float* bias,
                                   const float* ln_g, const float* ln_b, float eps, uint16_t* y, void* stream) {
  return patch_embed_ln("mmr_patch_embed_ln_bf16", false, img, b, hw, pack, bias, ln_g, ln_b, eps, y, stream);
}

}  // extern "C"
