// Fused Swin MLP sub-block for the narrow, memory-bound stages (C = 96, 192):
//   y = x + fc2(GELU(fc1(LN2(x))))            (timm SwinTransformerBlock, fusion.py:198-199)
// The 4C-wide hidden activation never leaves the CU.  Each wave owns 32 tokens, LayerNorms them in
// registers (row split over the lane pair that shares a token) straight into the fc1 B operand,
// and walks the hidden dimension 32 units at a time: fc1 (C^T orientation, 32x32x16 MFMA, so the
// GELU'd hidden values land in exactly the registers fc2 needs as its B operand under a
// k-permutation that the packed W2 columns mirror), bias + GELU, then accumulate fc2 (C^T, A = W2
// from LDS).  Weights are repacked once at load into per-64-hidden-unit chunks
// [W1 rows | W2 columns] that are exact, bank-conflict-free LDS images.
//   C = 96  (swin_mlp_sp): all of W1 + W2 (147 KiB) resident in LDS, one persistent workgroup per
//           CU, waves walk token tiles independently (no barriers), software-pipelined fc1 / GELU / fc2.
//   C = 192 (swin_mlp): 590 KiB of weights streamed through a 3-deep LDS ring by global_load_lds,
//           shared by the workgroup's 256 tokens.
// HBM traffic per token: 2C (x) + 2C (y) bytes, vs ~24C for the LN -> GEMM -> GEMM chain.
// The kernel is VALU-bound on GELU (308M evaluations per stage-1 call), hence the
// x*sigmoid(x*P(x^2)) form below.
#include <algorithm>
#include <float.h>
#include <math.h>

#include "common.h"

namespace {

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
// NOTE: LDS reads below use native vector types on purpose.  A HIP float4 (struct) load carries no
// TBAA info, and hipcc then makes every such ds_read wait vmcnt(0) for all in-flight
// global_load_lds — draining the weight ring each time.
typedef __attribute__((address_space(3))) void* lds_ptr_t;

constexpr int vmcnt_n(int n) { return (n & 15) | (7 << 4) | (15 << 8) | ((n >> 4) << 14); }

// Geometry.  NW waves per workgroup, 32 tokens per wave (the N side of
// v_mfma_f32_32x32x16_bf16).  Hidden units are walked in HC-wide chunks; a chunk is
// [W1 rows HC*ch.. : HC x C][W2 columns HC*ch.. : C x HC] = 4*HC*C bytes, an exact LDS image (16-B
// units permuted so every ds_read_b128 is bank-conflict-free, no padding), loaded as 1-KiB
// global_load_lds pieces spread evenly over the waves, through an R-deep ring.  The f32
// parameters (LN gamma/beta, fc1 bias) sit in a separate static LDS array.
template <int C, int NW, int HC, int R>
struct MlpGeo {
  static constexpr int U1 = C / 8;        // 16-B units per W1 row
  static constexpr int U2 = HC / 8;       // 16-B units per W2 row
  static constexpr int KS1 = C / 16;      // fc1 k-steps (k = 16)
  static constexpr int NU = C / 32;       // fc2 output tiles (32 channels)
  static constexpr int NT = HC / 32;      // 32-wide hidden tiles per chunk
  static constexpr int NCH = 4 * C / HC;  // chunks
  static constexpr int W1B = HC * C * 2;
  static constexpr int CHUNK_B = 2 * W1B;
  static constexpr int PW = CHUNK_B / 1024 / NW;  // glds pieces per wave per chunk
  static constexpr int TOK = 32 * NW;     // tokens per workgroup
  static constexpr int LDS_B = R * CHUNK_B;
  static_assert(CHUNK_B % (1024 * NW) == 0, "chunk must split evenly over the waves");
  static_assert(R == 2 || R == 3, "ring depth");
};

using mmr::unit_swz;
using mmr::w2_hidden;

// Output-row order for the resident kernel: MFMA C row 8i + 4h + rr of output tile u holds channel
// 32u + 16(i>>1) + 8h + 4(i&1) + rr, so lane half h ends up with channels 32u + 8h + 0..7 and
// 32u + 16 + 8h + 0..7 — exactly the channels it loaded for LayerNorm (residual from registers,
// 16-B stores).
__host__ __device__ __forceinline__ int w2_channel(int row) {
  const int u = row >> 5, rho = row & 31, i = rho >> 3, h = (rho >> 2) & 1, rr = rho & 3;
  return 32 * u + 16 * (i >> 1) + 8 * h + 4 * (i & 1) + rr;
}

template <int C, int HC, bool PERM>
__global__ __launch_bounds__(256) void swin_mlp_pack(const uint16_t* __restrict__ w1,
                                                     const uint16_t* __restrict__ w2,
                                                     uint16_t* __restrict__ pack) {
  constexpr int CE = 2 * HC * C, W1E = HC * C;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;  // logical element
  if (i >= (int64_t)8 * C * C) return;
  const int ch = (int)(i / CE), e = (int)(i % CE);
  if (e < W1E) {
    const int r = e / C, k = e % C, q = k >> 3;
    pack[(int64_t)ch * CE + r * C + 8 * unit_swz<C / 8>(r, q) + (k & 7)] = w1[(int64_t)(HC * ch + r) * C + k];
  } else {
    const int e2 = e - W1E, c = e2 / HC, pos = e2 % HC, q = pos >> 3;
    pack[(int64_t)ch * CE + W1E + c * HC + 8 * unit_swz<HC / 8>(c, q) + (pos & 7)] =
        w2[(int64_t)(PERM ? w2_channel(c) : c) * 4 * C + HC * ch + w2_hidden(pos)];
  }
}

template <bool FAST>
__device__ __forceinline__ float gelu_t(float v) {
  if constexpr (FAST) return mmr::gelu_fast(v);
  else return mmr::gelu_erf(v);
}

// GELU of two hidden values whose bias is already in the accumulator -> packed bf16 pair
template <bool FAST>
__device__ __forceinline__ uint32_t gelu_pack2(float a0, float a1) {
  if constexpr (FAST) {
    const mmr::f32x2_t u = mmr::gelu_fast2((mmr::f32x2_t){a0, a1});
    return mmr::pack2bf(u.x, u.y);
  } else {
    return mmr::pack2bf(gelu_t<FAST>(a0), gelu_t<FAST>(a1));
  }
}

template <int C, int NW, int HC, int R, bool FAST>
__global__ __launch_bounds__(64 * NW) void swin_mlp(const uint16_t* __restrict__ x,
                                                         const float* __restrict__ lng,
                                                         const float* __restrict__ lnb,
                                                         const uint16_t* __restrict__ pack,
                                                         const float* __restrict__ b1,
                                                         const float* __restrict__ b2,
                                                         uint16_t* __restrict__ y, int64_t T, float eps) {
  using G = MlpGeo<C, NW, HC, R>;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];  // the weight ring only
  __shared__ __attribute__((aligned(16))) float Pg[6 * C];
  const float* Pb = Pg + C;
  const float* Pb1 = Pg + 2 * C;

  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 31, h = lane >> 5;
  const int64_t tok = (int64_t)blockIdx.x * G::TOK + wave * 32 + r;
  const bool ok = tok < T;
  const uint16_t* xr = x + (ok ? tok : 0) * C;

  for (int i = threadIdx.x; i < 6 * C; i += 64 * NW)
    Pg[i] = i < C ? lng[i] : (i < 2 * C ? lnb[i - C] : b1[i - 2 * C]);
  bf16x8 xb[G::KS1];
#pragma unroll
  for (int ks = 0; ks < G::KS1; ++ks)
    xb[ks] = ok ? *(const bf16x8*)(xr + 16 * ks + 8 * h) : (bf16x8){0, 0, 0, 0, 0, 0, 0, 0};

  auto stage = [&](int ch) {
    const unsigned char* src = (const unsigned char*)pack + (size_t)ch * G::CHUNK_B;
    unsigned char* dst = smem + (ch % R) * G::CHUNK_B;
#pragma unroll
    for (int p = 0; p < G::PW; ++p) {
      const int piece = wave * G::PW + p;
      __builtin_amdgcn_global_load_lds((const void*)(src + piece * 1024 + lane * 16),
                                       (lds_ptr_t)(dst + piece * 1024), 16, 0, 0);
    }
  };
  stage(0);
  if constexpr (R == 3) stage(1);
  // x and the parameters were issued before the chunk(s): wait for them only
  __builtin_amdgcn_s_waitcnt(vmcnt_n((R - 1) * G::PW));
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): parameter stores landed
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  // LayerNorm (row split over the lane pair h = 0, 1), written back over xb as the fc1 B operand
  {
    float s = 0.f;
#pragma unroll
    for (int ks = 0; ks < G::KS1; ++ks)
#pragma unroll
      for (int j = 0; j < 8; ++j) s += mmr::bf2f((uint16_t)xb[ks][j]);
    s += __shfl_xor(s, 32, 64);
    const float mean = s * (1.0f / C);
    float ss = 0.f;
#pragma unroll
    for (int ks = 0; ks < G::KS1; ++ks)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = mmr::bf2f((uint16_t)xb[ks][j]) - mean;
        ss += d * d;
      }
    ss += __shfl_xor(ss, 32, 64);
    const float rstd = rsqrtf(ss * (1.0f / C) + eps);
#pragma unroll
    for (int ks = 0; ks < G::KS1; ++ks) {
      const int k0 = 16 * ks + 8 * h;
      const f32x4 g0 = *(const f32x4*)(Pg + k0), g1 = *(const f32x4*)(Pg + k0 + 4);
      const f32x4 c0 = *(const f32x4*)(Pb + k0), c1 = *(const f32x4*)(Pb + k0 + 4);
      const float gg[8] = {g0[0], g0[1], g0[2], g0[3], g1[0], g1[1], g1[2], g1[3]};
      const float cc[8] = {c0[0], c0[1], c0[2], c0[3], c1[0], c1[1], c1[2], c1[3]};
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (mmr::bf2f((uint16_t)xb[ks][j]) - mean) * rstd * gg[j] + cc[j];
      xb[ks] = __builtin_bit_cast(bf16x8, make_uint4(mmr::pack2bf(v[0], v[1]), mmr::pack2bf(v[2], v[3]),
                                                     mmr::pack2bf(v[4], v[5]), mmr::pack2bf(v[6], v[7])));
    }
  }

  f32x16 acc2[G::NU];
#pragma unroll
  for (int u = 0; u < G::NU; ++u)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc2[u][e] = 0.f;

  for (int ch = 0; ch < G::NCH; ++ch) {
    if (R == 3 && ch + 1 < G::NCH) __builtin_amdgcn_s_waitcnt(vmcnt_n(G::PW));  // chunk ch landed
    else __builtin_amdgcn_s_waitcnt(vmcnt_n(0));
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave's pieces landed; the slot refilled next is free
    asm volatile("" ::: "memory");
    if (ch + R - 1 < G::NCH) stage(ch + R - 1);
    const unsigned char* W1s = smem + (ch % R) * G::CHUNK_B;
    const unsigned char* W2s = W1s + G::W1B;
#pragma unroll
    for (int t = 0; t < G::NT; ++t) {  // 32 hidden units per step
      f32x16 a1;  // starts at fc1's bias (lane: hidden HC*ch + 32t + 8i + 4h + rr)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const f32x4 bb = *(const f32x4*)(Pb1 + HC * ch + 32 * t + 8 * i + 4 * h);
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) a1[4 * i + rr] = bb[rr];
      }
      const int row = 32 * t + r;
#pragma unroll
      for (int ks = 0; ks < G::KS1; ++ks) {
        const bf16x8 w = *(const bf16x8*)(W1s + (row * G::U1 + unit_swz<G::U1>(row, 2 * ks + h)) * 16);
        a1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w, xb[ks], a1, 0, 0, 0);
      }
      // lane holds hidden HC*ch + 32t + 8i + 4h + rr (i, rr = 0..3) of token r
      uint32_t hp[8];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        hp[2 * i] = gelu_pack2<FAST>(a1[4 * i], a1[4 * i + 1]);
        hp[2 * i + 1] = gelu_pack2<FAST>(a1[4 * i + 2], a1[4 * i + 3]);
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {  // k-step over hidden 32t + 16 s2 .. +15
        const bf16x8 hf = __builtin_bit_cast(bf16x8, make_uint4(hp[4 * s2], hp[4 * s2 + 1], hp[4 * s2 + 2],
                                                                hp[4 * s2 + 3]));
        const int q = 2 * (2 * t + s2) + h;
#pragma unroll
        for (int u = 0; u < G::NU; ++u) {
          const int c = 32 * u + r;
          const bf16x8 w = *(const bf16x8*)(W2s + (c * G::U2 + unit_swz<G::U2>(c, q)) * 16);
          acc2[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w, hf, acc2[u], 0, 0, 0);
        }
      }
    }
  }

  // y[tok][c] = x + b2 + fc2, c = 32u + 8i + 4h + rr
  if (ok) {
#pragma unroll
    for (int u = 0; u < G::NU; ++u)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = 32 * u + 8 * i + 4 * h;
        const float4 bb = *(const float4*)(b2 + c);
        const uint2 xv = *(const uint2*)(xr + c);
        const float v0 = acc2[u][4 * i] + bb.x + __uint_as_float(xv.x << 16);
        const float v1 = acc2[u][4 * i + 1] + bb.y + __uint_as_float(xv.x & 0xFFFF0000u);
        const float v2 = acc2[u][4 * i + 2] + bb.z + __uint_as_float(xv.y << 16);
        const float v3 = acc2[u][4 * i + 3] + bb.w + __uint_as_float(xv.y & 0xFFFF0000u);
        *(uint2*)(y + tok * C + c) = make_uint2(mmr::pack2bf(v0, v1), mmr::pack2bf(v2, v3));
      }
  }
}


// Software-pipelined resident variant (C = 96): iteration t runs fc1 of hidden block t+1 and fc2 of
// block t-1 (12 MFMAs) beside the bias'd GELU of block t (VALU) — three mutually independent
// streams in one basic block, so the matrix pipe works under the GELU instead of waiting for it
// (the forms above serialise fc1 -> GELU -> fc2 inside a wave and rely on other waves to fill the
// gaps).  2 waves per SIMD (<= 256 VGPRs: two fc1 accumulators, both packed hidden sets, the fc2
// accumulators, the LN'd x of this tile and the next tile's x; the residual is re-read from L2).
template <int C, int NW, bool FAST>
__global__ __launch_bounds__(64 * NW) void swin_mlp_sp(const uint16_t* __restrict__ x,
                                                       const float* __restrict__ lng,
                                                       const float* __restrict__ lnb,
                                                       const uint16_t* __restrict__ pack,
                                                       const float* __restrict__ b1,
                                                       const float* __restrict__ b2,
                                                       uint16_t* __restrict__ y, int64_t T, float eps) {
  using G = MlpGeo<C, NW, 64, 2>;
  constexpr int WB = G::NCH * G::CHUNK_B;
  constexpr int PWW = WB / 1024 / NW;
  constexpr int NB = 4 * C / 32;  // 32-wide hidden blocks
  static_assert(WB % (1024 * NW) == 0, "weights must split evenly over the waves");
  static_assert(NB >= 3, "pipeline depth");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* Pg = (float*)(smem + WB);
  const float* Pb = Pg + C;
  const float* Pb1 = Pg + 2 * C;
  const float* Pb2 = Pg + 6 * C;

  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 31, h = lane >> 5;
  const int64_t ntile = (T + 31) / 32, stride = (int64_t)gridDim.x * NW;
  int64_t tile = (int64_t)blockIdx.x * NW + wave;

  for (int i = threadIdx.x; i < 7 * C; i += 64 * NW)
    Pg[i] = i < C ? lng[i] : (i < 2 * C ? lnb[i - C] : (i < 6 * C ? b1[i - 2 * C] : b2[i - 6 * C]));
#pragma unroll
  for (int p = 0; p < PWW; ++p) {
    const int piece = wave * PWW + p;
    __builtin_amdgcn_global_load_lds((const void*)((const unsigned char*)pack + piece * 1024 + lane * 16),
                                     (lds_ptr_t)(smem + piece * 1024), 16, 0, 0);
  }
  auto load_x = [&](int64_t tl, bf16x8* dst) {
    const int64_t tk = tl * 32 + r;
    const bool ok = tl < ntile && tk < T;
    const uint16_t* xr = x + (ok ? tk : 0) * C;
#pragma unroll
    for (int ks = 0; ks < G::KS1; ++ks) {
      const bf16x8 v = *(const bf16x8*)(xr + 16 * ks + 8 * h);  // clamped row: unconditional load
      dst[ks] = ok ? v : (bf16x8){0, 0, 0, 0, 0, 0, 0, 0};
    }
  };
  bf16x8 xn[G::KS1];
  load_x(tile, xn);
  __builtin_amdgcn_s_waitcnt(vmcnt_n(0));
  __builtin_amdgcn_s_waitcnt(0xC07F);
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  // fc1 of hidden block t (bias in the accumulator): lane holds hidden 32t + 8i + 4h + rr of token r
  auto fc1 = [&](int t, const bf16x8* xb) {
    f32x16 a;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const f32x4 bb = *(const f32x4*)(Pb1 + 32 * t + 8 * i + 4 * h);
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) a[4 * i + rr] = bb[rr];
    }
    const unsigned char* W1s = smem + (t >> 1) * G::CHUNK_B;
    const int row = 32 * (t & 1) + r;
    bf16x8 w[G::KS1];
#pragma unroll
    for (int ks = 0; ks < G::KS1; ++ks)
      w[ks] = *(const bf16x8*)(W1s + (row * G::U1 + unit_swz<G::U1>(row, 2 * ks + h)) * 16);
#pragma unroll
    for (int ks = 0; ks < G::KS1; ++ks) a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[ks], xb[ks], a, 0, 0, 0);
    return a;
  };
  auto gelu = [&](const f32x16& a, uint32_t* hp) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      hp[2 * i] = gelu_pack2<FAST>(a[4 * i], a[4 * i + 1]);
      hp[2 * i + 1] = gelu_pack2<FAST>(a[4 * i + 2], a[4 * i + 3]);
    }
  };
  auto fc2 = [&](int t, const uint32_t* hp, f32x16* acc2) {
    const unsigned char* W2s = smem + (t >> 1) * G::CHUNK_B + G::W1B;
    bf16x8 w[2 * G::NU];
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int u = 0; u < G::NU; ++u) {
        const int c = 32 * u + r, q = 2 * (2 * (t & 1) + s2) + h;
        w[s2 * G::NU + u] = *(const bf16x8*)(W2s + (c * G::U2 + unit_swz<G::U2>(c, q)) * 16);
      }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const bf16x8 hf = __builtin_bit_cast(bf16x8, make_uint4(hp[4 * s2], hp[4 * s2 + 1], hp[4 * s2 + 2], hp[4 * s2 + 3]));
#pragma unroll
      for (int u = 0; u < G::NU; ++u)
        acc2[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[s2 * G::NU + u], hf, acc2[u], 0, 0, 0);
    }
  };

  for (; tile < ntile; tile += stride) {
    asm volatile("" ::: "memory");  // keep the parameter reads in the loop (LICM would pin them)
    bf16x8 xr[G::KS1], xb[G::KS1];
#pragma unroll
    for (int ks = 0; ks < G::KS1; ++ks) xr[ks] = xn[ks];
    load_x(tile + stride, xn);  // next tile's x in flight during this one
    const int64_t tok = tile * 32 + r;

    // LayerNorm (row split over the lane pair h = 0, 1) -> fc1 B operand
    {
      float s = 0.f;
#pragma unroll
      for (int ks = 0; ks < G::KS1; ++ks)
#pragma unroll
        for (int j = 0; j < 8; ++j) s += mmr::bf2f((uint16_t)xr[ks][j]);
      s += __shfl_xor(s, 32, 64);
      const float mean = s * (1.0f / C);
      float ss = 0.f;
#pragma unroll
      for (int ks = 0; ks < G::KS1; ++ks)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float d = mmr::bf2f((uint16_t)xr[ks][j]) - mean;
          ss += d * d;
        }
      ss += __shfl_xor(ss, 32, 64);
      const float rstd = rsqrtf(ss * (1.0f / C) + eps);
#pragma unroll
      for (int ks = 0; ks < G::KS1; ++ks) {
        const int k0 = 16 * ks + 8 * h;
        const f32x4 g0 = *(const f32x4*)(Pg + k0), g1 = *(const f32x4*)(Pg + k0 + 4);
        const f32x4 c0 = *(const f32x4*)(Pb + k0), c1 = *(const f32x4*)(Pb + k0 + 4);
        const float gg[8] = {g0[0], g0[1], g0[2], g0[3], g1[0], g1[1], g1[2], g1[3]};
        const float cc[8] = {c0[0], c0[1], c0[2], c0[3], c1[0], c1[1], c1[2], c1[3]};
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = (mmr::bf2f((uint16_t)xr[ks][j]) - mean) * rstd * gg[j] + cc[j];
        xb[ks] = __builtin_bit_cast(bf16x8, make_uint4(mmr::pack2bf(v[0], v[1]), mmr::pack2bf(v[2], v[3]),
                                                       mmr::pack2bf(v[4], v[5]), mmr::pack2bf(v[6], v[7])));
      }
    }

    f32x16 acc2[G::NU];
#pragma unroll
    for (int u = 0; u < G::NU; ++u)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc2[u][e] = 0.f;

    // pipeline: a1 = fc1(t) ready at the top of iteration t; hp = GELU(t - 1) packed
    f32x16 a1 = fc1(0, xb);
    uint32_t hp[8];
    {
      const f32x16 an = fc1(1, xb);
      gelu(a1, hp);
      a1 = an;
    }
#pragma unroll 1
    for (int t = 1; t < NB - 1; ++t) {
      const f32x16 an = fc1(t + 1, xb);
      uint32_t hn[8];
      gelu(a1, hn);
      fc2(t - 1, hp, acc2);
#pragma unroll
      for (int e = 0; e < 8; ++e) hp[e] = hn[e];
      a1 = an;
    }
    {
      uint32_t hn[8];
      gelu(a1, hn);
      fc2(NB - 2, hp, acc2);
      fc2(NB - 1, hn, acc2);
    }

    // y = x + b2 + fc2: lane half h holds channels 32u + 16 half + 8h + 0..7 (w2_channel order)
    if (tok < T) {
#pragma unroll
      for (int u = 0; u < G::NU; ++u)
#pragma unroll
        for (int hf2 = 0; hf2 < 2; ++hf2) {
          const int c0 = 32 * u + 16 * hf2 + 8 * h;
          const f32x4 bl = *(const f32x4*)(Pb2 + c0), bh = *(const f32x4*)(Pb2 + c0 + 4);
          const bf16x8 xv = *(const bf16x8*)(x + tok * C + c0);  // residual re-read (L2): no registers held
          float v[8];
#pragma unroll
          for (int j = 0; j < 8; ++j)
            v[j] = acc2[u][8 * hf2 + j] + (j < 4 ? bl[j] : bh[j - 4]) + mmr::bf2f((uint16_t)xv[j]);
          *(uint4*)(y + tok * C + c0) = make_uint4(mmr::pack2bf(v[0], v[1]), mmr::pack2bf(v[2], v[3]),
                                                   mmr::pack2bf(v[4], v[5]), mmr::pack2bf(v[6], v[7]));
        }
    }
  }
}

int cu_count() {
  static int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
      v = 256;
    return v;
  }();
  return n;
}

template <int C, int NW, bool FAST>
mmr_status launch_sp(const uint16_t* x, const float* g, const float* b, const uint16_t* pack,
                     const float* b1, const float* b2, uint16_t* y, int64_t T, float eps, hipStream_t st) {
  using G = MlpGeo<C, NW, 64, 2>;
  const int64_t wave_tiles = (T + 31) / 32;
  const int64_t grid = std::min<int64_t>(cu_count(), (wave_tiles + NW - 1) / NW);
  swin_mlp_sp<C, NW, FAST><<<dim3((unsigned)grid), 64 * NW, G::NCH * G::CHUNK_B + 7 * C * 4, st>>>(
      x, g, b, pack, b1, b2, y, T, eps);
  MMR_LAUNCH_CHECK();
  return MMR_OK;
}

template <int C, int HC, bool PERM>
mmr_status launch_pack(const uint16_t* w1, const uint16_t* w2, uint16_t* pack, hipStream_t st) {
  const int64_t n = (int64_t)8 * C * C;
  swin_mlp_pack<C, HC, PERM><<<dim3((unsigned)mmr::ceil_div(n, 256)), 256, 0, st>>>(w1, w2, pack);
  MMR_LAUNCH_CHECK();
  return MMR_OK;
}

template <int C, int NW, int HC, int R, bool FAST>
mmr_status launch_stream(const uint16_t* x, const float* g, const float* b, const uint16_t* pack,
                         const float* b1, const float* b2, uint16_t* y, int64_t T, float eps,
                         hipStream_t st) {
  using G = MlpGeo<C, NW, HC, R>;
  swin_mlp<C, NW, HC, R, FAST><<<dim3((unsigned)mmr::ceil_div(T, G::TOK)), 64 * NW, G::LDS_B, st>>>(
      x, g, b, pack, b1, b2, y, T, eps);
  MMR_LAUNCH_CHECK();
  return MMR_OK;
}

}  // namespace

extern "C" {

int64_t mmr_swin_mlp_pack_elems(int32_t c) {
  return (c == 96 || c == 192) ? (int64_t)8 * c * c : 0;
}

mmr_status mmr_swin_mlp_pack(const uint16_t* w1, const uint16_t* w2, uint16_t* pack, int32_t c,
                             void* stream) {
  mmr::clear_error();
  MMR_REQUIRE(w1 && w2 && pack, "mmr_swin_mlp_pack: NULL pointer");
  hipStream_t st = mmr::as_stream(stream);
  // C = 96: resident kernel (W2 rows in w2_channel order); C = 192: streamed chunks
  if (c == 96) return launch_pack<96, 64, true>(w1, w2, pack, st);
  if (c == 192) return launch_pack<192, 64, false>(w1, w2, pack, st);
  mmr::set_error("mmr_swin_mlp_pack: C=%d not built (96, 192)", c);
  return MMR_ERR_UNSUPPORTED;
}

mmr_status mmr_swin_mlp(const uint16_t* x, const float* ln_g, const float* ln_b,
                        const uint16_t* pack, const float* b1, const float* b2, uint16_t* y,
                        int64_t tokens, int32_t c, float eps, void* stream) {
  mmr::clear_error();
  MMR_REQUIRE(x && ln_g && ln_b && pack && b1 && b2 && y, "mmr_swin_mlp: NULL pointer");
  MMR_REQUIRE(tokens >= 0, "mmr_swin_mlp: tokens < 0");
  MMR_REQUIRE(x != y, "mmr_swin_mlp: in-place not supported");
  if (tokens == 0) return MMR_OK;
  hipStream_t st = mmr::as_stream(stream);
  // C = 96: the software-pipelined resident form, 2 waves per SIMD (215 -> 199 us at B = 256 over the
  // serial resident forms, which were removed: profiles/r03_swin_mlp_sp_ab.txt, r03_swin_mlp_ab.txt);
  // C = 192: the streamed form (its software-pipelined twin measured equal and was removed)
  if (c == 96) return launch_sp<96, 8, true>(x, ln_g, ln_b, pack, b1, b2, y, tokens, eps, st);
  if (c == 192) return launch_stream<192, 8, 64, 3, true>(x, ln_g, ln_b, pack, b1, b2, y, tokens, eps, st);
  mmr::set_error("mmr_swin_mlp: C=%d not built (96, 192)", c);
  return MMR_ERR_UNSUPPORTED;
}

}  // extern "C"
