// Per-query f32 linears of the multimodal head on bf16 MFMA with three-term splits (bf16x3):
//   Y[b][o] = act(sum_i X[b][i] W[o][i] + bias[o]) (+ R[b][o])
// X f32 is split in registers into hi = bf16(x), lo = bf16(x - hi); W comes pre-split (hi / lo bf16
// copies made once at load); each 16x16x32 k-step runs hi*hi + hi*lo + lo*hi on
// v_mfma_f32_16x16x32_bf16 with f32 accumulation.  The dropped lo*lo term and the bf16 rounding of the
// lo parts leave ~2^-17 relative error per product (vs 2^-24 for f32 products) — two orders of
// magnitude below the bf16 tower activations these vectors are computed from, at 1/5 of the f32
// MFMA time (16x16x32 bf16: 8192 MACs in 16 cycles, x3, vs v_mfma_f32_32x32x2_f32: 2048 in 64).
// Reference semantics: the fusion head's nn.Linear chain in fp32 (model.py:375-459, MultiHeadMLP
// model.py:61-75, adapters :262-268); linear_f32 (tower.hip) stays the exact-f32 path.
//
// Geometry: one 32x32 output tile per workgroup of NW waves, the K range split over the waves
// (cin % (32 NW) == 0; NW = 8 when the launch has too few tiles to fill the chip, which halves each
// wave's serial K chain), partial tiles summed in LDS in a fixed order (deterministic); every load of a
// 3-step chunk issued before its MFMAs; rows >= nb clamped (loaded, never stored).  blockIdx.y is the
// problem index of the batched form (independent problems at fixed element strides).
#include "common.h"

namespace {

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int X3_CH = 3;  // k-steps (32 k each) per load chunk

__device__ __forceinline__ void split8(const float4& p, const float4& q, bf16x8& hi, bf16x8& lo) {
  const float v[8] = {p.x, p.y, p.z, p.w, q.x, q.y, q.z, q.w};
  uint32_t h[4], l[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    h[j] = mmr::pack2bf(v[2 * j], v[2 * j + 1]);
    const float r0 = v[2 * j] - __uint_as_float(h[j] << 16);
    const float r1 = v[2 * j + 1] - __uint_as_float(h[j] & 0xFFFF0000u);
    l[j] = mmr::pack2bf(r0, r1);
  }
  hi = __builtin_bit_cast(bf16x8, make_uint4(h[0], h[1], h[2], h[3]));
  lo = __builtin_bit_cast(bf16x8, make_uint4(l[0], l[1], l[2], l[3]));
}

template <int ACT, bool BIAS, bool RES, int NW>
__global__ __launch_bounds__(64 * NW) void linear_x3(const float* __restrict__ X, int64_t ldx,
                                                 const uint16_t* __restrict__ Wh,
                                                 const uint16_t* __restrict__ Wl,
                                                 const float* __restrict__ bias, const float* R,
                                                 int64_t ldr, float* Y, int64_t ldy, int nb, int cin,
                                                 int cout, int64_t bsx, int64_t bsw, int64_t bsb,
                                                 int64_t bsr, int64_t bsy) {
  __shared__ float part[NW][32][33];
  X += blockIdx.y * bsx;
  Wh += blockIdx.y * bsw;
  Wl += blockIdx.y * bsw;
  if (BIAS) bias += blockIdx.y * bsb;
  if (RES) R += blockIdx.y * bsr;
  Y += blockIdx.y * bsy;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int tiles_o = cout / 32;
  const int tb = blockIdx.x / tiles_o, to = blockIdx.x % tiles_o;
  const int r = lane & 15, g = lane >> 4;
  const float* xa[2];
  const uint16_t* wh[2];
  const uint16_t* wl[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int row = tb * 32 + 16 * t + r;
    xa[t] = X + (int64_t)(row < nb ? row : nb - 1) * ldx + 8 * g;
    wh[t] = Wh + (int64_t)(to * 32 + 16 * t + r) * cin + 8 * g;
    wl[t] = Wl + (int64_t)(to * 32 + 16 * t + r) * cin + 8 * g;
  }
  const int kw = cin / NW, k0 = wave * kw, nsteps = kw / 32;
  f32x4 acc[2][2];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n) acc[m][n] = (f32x4){0.f, 0.f, 0.f, 0.f};
  for (int s0 = 0; s0 < nsteps; s0 += X3_CH) {
    float4 xv[X3_CH][2][2];
    bf16x8 bh[X3_CH][2], bl[X3_CH][2];
#pragma unroll
    for (int c = 0; c < X3_CH; ++c) {
      const int kk = k0 + 32 * (s0 + c < nsteps ? s0 + c : nsteps - 1);  // clamped: loads unconditional
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        xv[c][t][0] = *(const float4*)(xa[t] + kk);
        xv[c][t][1] = *(const float4*)(xa[t] + kk + 4);
        bh[c][t] = *(const bf16x8*)(wh[t] + kk);
        bl[c][t] = *(const bf16x8*)(wl[t] + kk);
      }
    }
#pragma unroll
    for (int c = 0; c < X3_CH; ++c) {
      if (s0 + c < nsteps) {
        bf16x8 ah[2], al[2];
#pragma unroll
        for (int t = 0; t < 2; ++t) split8(xv[c][t][0], xv[c][t][1], ah[t], al[t]);
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
          for (int n = 0; n < 2; ++n) {
            acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[m], bh[c][n], acc[m][n], 0, 0, 0);
            acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[m], bl[c][n], acc[m][n], 0, 0, 0);
            acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[m], bh[c][n], acc[m][n], 0, 0, 0);
          }
      }
    }
  }
  // lane: output column 16 n + r, rows 16 m + 4 g + i
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int i = 0; i < 4; ++i) part[wave][16 * m + 4 * g + i][16 * n + r] = acc[m][n][i];
  __syncthreads();
#pragma unroll
  for (int e4 = 0; e4 < 16 / NW; ++e4) {
    const int e = threadIdx.x + 64 * NW * e4, row = e >> 5, col = e & 31;
    const int bb = tb * 32 + row, o = to * 32 + col;
    float v = part[0][row][col];
#pragma unroll
    for (int w = 1; w < NW; ++w) v += part[w][row][col];
    if (bb >= nb) continue;
    if (BIAS) v += bias[o];
    if (ACT == 1) v = mmr::gelu_erf(v);
    if (RES) v += R[(int64_t)bb * ldr + o];
    Y[(int64_t)bb * ldy + o] = v;
  }
}

}  // namespace

extern "C" mmr_status mmr_linear_x3(const float* x, int64_t ldx, int64_t bsx, const uint16_t* w_hi,
                                    const uint16_t* w_lo, int64_t bsw, const float* bias, int64_t bsb,
                                    const float* residual, int64_t ldr, int64_t bsr, float* y, int64_t ldy,
                                    int64_t bsy, int32_t nbatch, int32_t b, int32_t cin, int32_t cout,
                                    int32_t act, void* stream) {
  mmr::clear_error();
  MMR_REQUIRE(x && w_hi && w_lo && y && b >= 0 && nbatch >= 1, "mmr_linear_x3: bad arguments");
  MMR_REQUIRE(cin > 0 && cin % 128 == 0 && cout > 0 && cout % 32 == 0,
              "mmr_linear_x3: cin=%d must be a multiple of 128, cout=%d of 32", cin, cout);
  MMR_REQUIRE(ldx >= cin && ldx % 4 == 0 && bsx % 4 == 0 && bsw % 8 == 0 && ldy >= cout && (!residual || ldr >= cout),
              "mmr_linear_x3: bad strides");
  MMR_REQUIRE(((uintptr_t)x & 15u) == 0 && ((uintptr_t)w_hi & 15u) == 0 && ((uintptr_t)w_lo & 15u) == 0,
              "mmr_linear_x3: x / w must be 16-B aligned");
  MMR_REQUIRE(act == 0 || act == 1, "mmr_linear_x3: act=%d", act);
  if (b == 0) return MMR_OK;
  const dim3 grid((unsigned)(mmr::ceil_div(b, 32) * (cout / 32)), (unsigned)nbatch);
  hipStream_t st = mmr::as_stream(stream);
  const bool hb = bias != nullptr, hr = residual != nullptr;
  // 8 waves per tile when the launch has fewer than 2 tiles per CU (the joint chain at B = 256:
  // 96-384 tiles) and the K range splits evenly into 8
  int nw = (cin % 256 == 0 && (int64_t)grid.x * grid.y < 512) ? 8 : 4;
  const int pin = mmr::pin_x3_waves.load(std::memory_order_relaxed);  // mmr_pin_variant (tests)
  if (pin == 4 || (pin == 8 && cin % 256 == 0)) nw = pin;
#define X3_L(A, B_, R_)                                                                                          \
  (nw == 8 ? linear_x3<A, B_, R_, 8><<<grid, 512, 0, st>>>(x, ldx, w_hi, w_lo, bias, residual, ldr, y, ldy, b, cin, \
                                                         cout, bsx, bsw, bsb, bsr, bsy)                          \
           : linear_x3<A, B_, R_, 4><<<grid, 256, 0, st>>>(x, ldx, w_hi, w_lo, bias, residual, ldr, y, ldy, b, cin, \
                                                         cout, bsx, bsw, bsb, bsr, bsy))
  if (act == 1) {
    if (hb && hr) X3_L(1, true, true);
    else if (hb) X3_L(1, true, false);
    else if (hr) X3_L(1, false, true);
    else X3_L(1, false, false);
  } else {
    if (hb && hr) X3_L(0, true, true);
    else if (hb) X3_L(0, true, false);
    else if (hr) X3_L(0, false, true);
    else X3_L(0, false, false);
  }
#undef X3_L
  MMR_LAUNCH_CHECK();
  return MMR_OK;
}
