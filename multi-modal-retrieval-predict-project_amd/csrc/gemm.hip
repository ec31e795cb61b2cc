// bf16 "linear" GEMM with fused epilogue for the towers (gfx950):
//   Y[m][n] = act(sum_k X[m][k] * W[n][k] + bias[n]) (+ R[m][n]),  X, W, R, Y bf16, f32 accumulate.
// nn.Linear layout (W = [out][in], both operands K-contiguous), so both MFMA fragments are
// 16-byte contiguous row reads.  Replaces every nn.Linear of timm Swin / HF BERT on the path
// (fusion.py:198-199, 322-325) — QKV, attention output (+residual), FFN1 (+GELU), FFN2 (+residual),
// PatchMerging reduction, patch-embed conv as im2col GEMM.
//
// Tile 128x128x64, 256 threads = 4 waves (2x2), wave tile 64x64 = 4x4 v_mfma_f32_16x16x32_bf16.
// LDS: double-buffered A/B tiles, 128-B rows, 16-B chunk c of row r stored at chunk
// c ^ ((r>>1)&7) — conflict-free ds_read_b128 for the 16-row fragment reads.  Register-staged
// global loads of tile k+1 are issued before the MFMAs of tile k (T14 issue-early/write-late).
// Block ids are remapped so each XCD walks a contiguous range of (m, n) tiles, n fastest: the
// N/128 tiles that share one 128-row X panel run on one XCD and reuse it from that XCD's L2.
#include "common.h"

namespace {

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int BM = 128, BN = 128, BK = 64;
constexpr int TILE_ELEMS = BM * BK;  // per operand per buffer (bf16)

__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

template <int ACT, bool HAS_BIAS, bool HAS_RES>
__global__ __launch_bounds__(256, 2) void gemm_bf16_tn(const uint16_t* __restrict__ X,
                                                        const uint16_t* __restrict__ W,
                                                        const float* __restrict__ bias,
                                                        const uint16_t* __restrict__ R,
                                                        uint16_t* __restrict__ Y, int64_t M, int N,
                                                        int K, int tiles_m, int tiles_n) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[2][2][TILE_ELEMS];  // 64 KiB

  // XCD-aware bijective remap (cdna_hip_programming.md §5, "XCD swizzle must be bijective")
  const int nwg = tiles_m * tiles_n;
  const int orig = blockIdx.x;
  const int q = nwg / 8, r8 = nwg % 8, xcd = orig % 8;
  const int wg = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + orig / 8;
  const int tm = wg / tiles_n, tn = wg % tiles_n;
  const int64_t m0 = (int64_t)tm * BM;
  const int n0 = tn * BN;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  // staging: 128 rows x 8 chunks = 1024 chunks per operand, 4 per thread
  bf16x8 ra[4], rb[4];
  auto gload = [&](int k0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = tid + 256 * i;
      const int row = c >> 3, ch = c & 7;
      const int k = k0 + ch * 8;
      const int64_t gm = m0 + row;
      const int gn = n0 + row;
      bf16x8 z = {0, 0, 0, 0, 0, 0, 0, 0};
      ra[i] = (gm < M && k < K) ? *(const bf16x8*)(X + gm * K + k) : z;
      rb[i] = (gn < N && k < K) ? *(const bf16x8*)(W + (int64_t)gn * K + k) : z;
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = tid + 256 * i;
      const int row = c >> 3, ch = c & 7;
      const int off = row * BK + swz(row, ch) * 8;
      *(bf16x8*)(&lds[buf][0][off]) = ra[i];
      *(bf16x8*)(&lds[buf][1][off]) = rb[i];
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int nk = (K + BK - 1) / BK;
  gload(0);
  lstore(0);
  __syncthreads();
  const int fr = lane & 15, fq = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) gload((kt + 1) * BK);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 a[4], b[4];
      const int ch = s * 4 + fq;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int rowa = wm * 64 + i * 16 + fr;
        const int rowb = wn * 64 + i * 16 + fr;
        a[i] = *(const bf16x8*)(&lds[buf][0][rowa * BK + swz(rowa, ch) * 8]);
        b[i] = *(const bf16x8*)(&lds[buf][1][rowb * BK + swz(rowb, ch) * 8]);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) lstore(buf ^ 1);
    __syncthreads();
  }

  // epilogue: C[row][col], col = lane&15, row = 4*(lane>>4) + reg
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = n0 + wn * 64 + j * 16 + fr;
    if (n >= N) continue;
    const float bv = HAS_BIAS ? bias[n] : 0.0f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int rg = 0; rg < 4; ++rg) {
        const int64_t m = m0 + wm * 64 + i * 16 + fq * 4 + rg;
        if (m >= M) continue;
        float v = acc[i][j][rg] + bv;
        if (ACT == 1) v = mmr::gelu_erf(v);
        if (HAS_RES) v += mmr::bf2f(R[m * N + n]);
        Y[m * N + n] = mmr::f2bf(v);
      }
    }
  }
}

template <int ACT, bool HB, bool HR>
void launch(const uint16_t* x, const uint16_t* w, const float* b, const uint16_t* r, uint16_t* y,
            int64_t m, int n, int k, hipStream_t st) {
  const int tm = (int)mmr::ceil_div(m, BM), tn = (int)mmr::ceil_div(n, BN);
  gemm_bf16_tn<ACT, HB, HR><<<dim3(tm * tn), dim3(256), 0, st>>>(x, w, b, r, y, m, n, k, tm, tn);
}

}  // namespace

extern "C" mmr_status mmr_linear_bf16(const uint16_t* x, const uint16_t* w, const float* bias,
                                      const uint16_t* residual, uint16_t* y, int64_t m, int32_t n,
                                      int32_t k, int32_t act, void* stream) {
  mmr::clear_error();
  MMR_REQUIRE(x && w && y, "mmr_linear_bf16: NULL pointer");
  MMR_REQUIRE(m >= 0 && n > 0 && k > 0, "mmr_linear_bf16: bad shape");
  MMR_REQUIRE(k % 8 == 0, "mmr_linear_bf16: K=%d must be a multiple of 8", k);
  MMR_REQUIRE(act == 0 || act == 1, "mmr_linear_bf16: act=%d", act);
  MMR_REQUIRE(m * (int64_t)mmr::ceil_div(n, BN) / BM < (int64_t(1) << 31), "mmr_linear_bf16: grid too large");
  if (m == 0) return MMR_OK;
  hipStream_t st = mmr::as_stream(stream);
  const bool hb = bias != nullptr, hr = residual != nullptr;
  if (act == 0) {
    if (hb && hr) launch<0, true, true>(x, w, bias, residual, y, m, n, k, st);
    else if (hb) launch<0, true, false>(x, w, bias, residual, y, m, n, k, st);
    else if (hr) launch<0, false, true>(x, w, bias, residual, y, m, n, k, st);
    else launch<0, false, false>(x, w, bias, residual, y, m, n, k, st);
  } else {
    if (hb && hr) launch<1, true, true>(x, w, bias, residual, y, m, n, k, st);
    else if (hb) launch<1, true, false>(x, w, bias, residual, y, m, n, k, st);
    else if (hr) launch<1, false, true>(x, w, bias, residual, y, m, n, k, st);
    else launch<1, false, false>(x, w, bias, residual, y, m, n, k, st);
  }
  MMR_LAUNCH_CHECK();
  return MMR_OK;
}
