// Fused Swin MLP sub-block for the narrow, memory-bound stages (C = 96, 192):
//   y = x + fc2(GELU(fc1(LN2(x))))            (timm SwinTransformerBlock, fusion.py:198-199)
// The 4C-wide hidden activation never leaves the CU: per 64-token tile, each wave owns 16 tokens,
// LayerNorms them in registers (row split over the 4 lanes that share a token), and walks the
// hidden dimension in HC-wide chunks: fc1 (C^T orientation, so the GELU'd hidden values land in
// exactly the registers fc2 needs as its B operand under a k-permutation that the A operand —
// W2 read from LDS — mirrors), bias + GELU, then accumulate fc2.  Weights are repacked once at
// load into per-chunk [W1 rows | W2 columns] slabs with padded rows (conflict-free ds_read_b128 /
// ds_read_b64) and streamed through a 2-deep LDS ring by global_load_lds.
// HBM traffic per token: 2C (x) + 2C (y) bytes, vs 2C + 8C + 8C + 2C + 2C (+LN pass) for the
// LN -> GEMM -> GEMM chain.
#include <float.h>
#include <math.h>

#include "common.h"

namespace {

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;

template <int C, int HC>
struct MlpCfg {
  static constexpr int LD1 = C + 8;        // W1 chunk row stride (elements): 16-row reads conflict-free
  static constexpr int LD2 = HC + 4;       // W2 chunk row stride: 8-B reads conflict-free
  static constexpr int W1E = HC * LD1;
  static constexpr int W2E = C * LD2;
  static constexpr int CHUNK_E = (W1E + W2E + 511) / 512 * 512;  // whole 1-KiB glds pieces
  static constexpr int NCH = 4 * C / HC;
};

template <int C, int HC>
__global__ __launch_bounds__(256) void swin_mlp_pack(const uint16_t* __restrict__ w1,
                                                     const uint16_t* __restrict__ w2,
                                                     uint16_t* __restrict__ pack) {
  using Cf = MlpCfg<C, HC>;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)Cf::NCH * Cf::CHUNK_E) return;
  const int ch = (int)(i / Cf::CHUNK_E), e = (int)(i % Cf::CHUNK_E);
  uint16_t v = 0;
  if (e < Cf::W1E) {
    const int r = e / Cf::LD1, k = e % Cf::LD1;
    if (k < C) v = w1[(int64_t)(ch * HC + r) * C + k];  // fc1.weight [4C][C]
  } else if (e < Cf::W1E + Cf::W2E) {
    const int e2 = e - Cf::W1E;
    const int c = e2 / Cf::LD2, j = e2 % Cf::LD2;
    if (j < HC) v = w2[(int64_t)c * 4 * C + ch * HC + j];  // fc2.weight [C][4C]
  }
  pack[i] = v;
}

template <int C, int HC>
__global__ __launch_bounds__(256) void swin_mlp(const uint16_t* __restrict__ x,
                                                const float* __restrict__ lng,
                                                const float* __restrict__ lnb,
                                                const uint16_t* __restrict__ pack,
                                                const float* __restrict__ b1,
                                                const float* __restrict__ b2,
                                                uint16_t* __restrict__ y, int64_t T, float eps) {
  using Cf = MlpCfg<C, HC>;
  constexpr int KS1 = C / 32;       // fc1 k-steps
  constexpr int NT1 = HC / 16;      // fc1 n-tiles per chunk
  constexpr int KS2 = HC / 32;      // fc2 k-steps per chunk
  constexpr int NU = C / 16;        // fc2 output tiles
  constexpr int PIECES = Cf::CHUNK_E / 512;
  extern __shared__ __attribute__((aligned(16))) uint16_t sm[];  // [2][CHUNK_E]

  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int fr = lane & 15, g4 = lane >> 4;
  const int64_t m = (int64_t)blockIdx.x * 64 + wave * 16 + fr;
  const bool mok = m < T;
  const uint16_t* xr = x + (mok ? m : 0) * C;

  auto stage = [&](int ch, int buf) {
    const uint16_t* src = pack + (int64_t)ch * Cf::CHUNK_E;
    uint16_t* dst = sm + buf * Cf::CHUNK_E;
    for (int p = wave; p < PIECES; p += 4)
      __builtin_amdgcn_global_load_lds((const void*)(src + p * 512 + lane * 8), (lds_ptr_t)(dst + p * 512),
                                       16, 0, 0);
  };
  stage(0, 0);

  // LayerNorm of this lane's token (row split over the 4 lanes g4 = 0..3 sharing fr)
  float xv[KS1][8];
  float s = 0.f;
#pragma unroll
  for (int ks = 0; ks < KS1; ++ks) {
    const bf16x8 v = mok ? *(const bf16x8*)(xr + 32 * ks + 8 * g4) : (bf16x8){0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      xv[ks][j] = mmr::bf2f((uint16_t)v[j]);
      s += xv[ks][j];
    }
  }
  s += __shfl_xor(s, 16, 64);
  s += __shfl_xor(s, 32, 64);
  const float mean = s / C;
  float ss = 0.f;
#pragma unroll
  for (int ks = 0; ks < KS1; ++ks)
#pragma unroll
    for (int j = 0; j < 8; ++j) ss += (xv[ks][j] - mean) * (xv[ks][j] - mean);
  ss += __shfl_xor(ss, 16, 64);
  ss += __shfl_xor(ss, 32, 64);
  const float rstd = rsqrtf(ss / C + eps);
  bf16x8 hB[KS1];
#pragma unroll
  for (int ks = 0; ks < KS1; ++ks) {
    const int k0 = 32 * ks + 8 * g4;
    float h[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) h[j] = (xv[ks][j] - mean) * rstd * lng[k0 + j] + lnb[k0 + j];
    hB[ks] = __builtin_bit_cast(bf16x8, make_uint4(mmr::pack2bf(h[0], h[1]), mmr::pack2bf(h[2], h[3]),
                                                   mmr::pack2bf(h[4], h[5]), mmr::pack2bf(h[6], h[7])));
  }

  f32x4 acc2[NU];
#pragma unroll
  for (int u = 0; u < NU; ++u) acc2[u] = (f32x4){0.f, 0.f, 0.f, 0.f};

  for (int ch = 0; ch < Cf::NCH; ++ch) {
    __builtin_amdgcn_s_waitcnt(0x0070 | 0x0F00);  // vmcnt(0): this wave's pieces of chunk ch landed
    __syncthreads();                                 // ... and every wave's; buffer ch+1 is free
    if (ch + 1 < Cf::NCH) stage(ch + 1, (ch + 1) & 1);
    const uint16_t* W1s = sm + (ch & 1) * Cf::CHUNK_E;
    const uint16_t* W2s = W1s + Cf::W1E;
    // fc1 (C^T): hidden n = ch*HC + 16t + 4*g4 + rg for token fr
    float hv[NT1][4];
#pragma unroll
    for (int t = 0; t < NT1; ++t) {
      f32x4 a1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS1; ++ks) {
        const bf16x8 w = *(const bf16x8*)(W1s + (16 * t + fr) * Cf::LD1 + 32 * ks + 8 * g4);
        a1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w, hB[ks], a1, 0, 0, 0);
      }
      const float4 bb = *(const float4*)(b1 + ch * HC + 16 * t + 4 * g4);
      hv[t][0] = mmr::gelu_erf(a1[0] + bb.x);
      hv[t][1] = mmr::gelu_erf(a1[1] + bb.y);
      hv[t][2] = mmr::gelu_erf(a1[2] + bb.z);
      hv[t][3] = mmr::gelu_erf(a1[3] + bb.w);
    }
    // fc2 (C^T): k-step s covers hidden 32s + 16(j>>2) + 4*g4 + (j&3) for fragment element j
#pragma unroll
    for (int s2 = 0; s2 < KS2; ++s2) {
      const bf16x8 hf = __builtin_bit_cast(
          bf16x8, make_uint4(mmr::pack2bf(hv[2 * s2][0], hv[2 * s2][1]), mmr::pack2bf(hv[2 * s2][2], hv[2 * s2][3]),
                             mmr::pack2bf(hv[2 * s2 + 1][0], hv[2 * s2 + 1][1]),
                             mmr::pack2bf(hv[2 * s2 + 1][2], hv[2 * s2 + 1][3])));
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        const uint16_t* wr = W2s + (16 * u + fr) * Cf::LD2 + 32 * s2 + 4 * g4;
        const bf16x4 lo = *(const bf16x4*)(wr);
        const bf16x4 hi = *(const bf16x4*)(wr + 16);
        const bf16x8 wf = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        acc2[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf, hf, acc2[u], 0, 0, 0);
      }
    }
  }

  // y[m][c] = x + b2 + fc2; lane holds c = 16u + 4*g4 + 0..3 of token fr
  if (mok) {
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int c = 16 * u + 4 * g4;
      const float4 bb = *(const float4*)(b2 + c);
      const uint2 xr2 = *(const uint2*)(xr + c);
      const float v0 = acc2[u][0] + bb.x + __uint_as_float(xr2.x << 16);
      const float v1 = acc2[u][1] + bb.y + __uint_as_float(xr2.x & 0xFFFF0000u);
      const float v2 = acc2[u][2] + bb.z + __uint_as_float(xr2.y << 16);
      const float v3 = acc2[u][3] + bb.w + __uint_as_float(xr2.y & 0xFFFF0000u);
      *(uint2*)(y + m * C + c) = make_uint2(mmr::pack2bf(v0, v1), mmr::pack2bf(v2, v3));
    }
  }
}

template <int C, int HC>
mmr_status launch_pack(const uint16_t* w1, const uint16_t* w2, uint16_t* pack, hipStream_t st) {
  using Cf = MlpCfg<C, HC>;
  const int64_t n = (int64_t)Cf::NCH * Cf::CHUNK_E;
  swin_mlp_pack<C, HC><<<dim3((unsigned)mmr::ceil_div(n, 256)), 256, 0, st>>>(w1, w2, pack);
  MMR_LAUNCH_CHECK();
  return MMR_OK;
}

template <int C, int HC>
mmr_status launch_mlp(const uint16_t* x, const float* g, const float* b, const uint16_t* pack,
                      const float* b1, const float* b2, uint16_t* y, int64_t T, float eps,
                      hipStream_t st) {
  using Cf = MlpCfg<C, HC>;
  const size_t lds = 2 * Cf::CHUNK_E * sizeof(uint16_t);
  swin_mlp<C, HC><<<dim3((unsigned)mmr::ceil_div(T, 64)), 256, lds, st>>>(x, g, b, pack, b1, b2, y, T, eps);
  MMR_LAUNCH_CHECK();
  return MMR_OK;
}

}  // namespace

extern "C" {

int64_t mmr_swin_mlp_pack_elems(int32_t c) {
  if (c == 96) return (int64_t)MlpCfg<96, 64>::NCH * MlpCfg<96, 64>::CHUNK_E;
  if (c == 192) return (int64_t)MlpCfg<192, 32>::NCH * MlpCfg<192, 32>::CHUNK_E;
  return 0;
}

mmr_status mmr_swin_mlp_pack(const uint16_t* w1, const uint16_t* w2, uint16_t* pack, int32_t c,
                             void* stream) {
  mmr::clear_error();
  MMR_REQUIRE(w1 && w2 && pack, "mmr_swin_mlp_pack: NULL pointer");
  hipStream_t st = mmr::as_stream(stream);
  if (c == 96) return launch_pack<96, 64>(w1, w2, pack, st);
  if (c == 192) return launch_pack<192, 32>(w1, w2, pack, st);
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
  if (c == 96) return launch_mlp<96, 64>(x, ln_g, ln_b, pack, b1, b2, y, tokens, eps, st);
  if (c == 192) return launch_mlp<192, 32>(x, ln_g, ln_b, pack, b1, b2, y, tokens, eps, st);
  mmr::set_error("mmr_swin_mlp: C=%d not built (96, 192)", c);
  return MMR_ERR_UNSUPPORTED;
}

}  // extern "C"
