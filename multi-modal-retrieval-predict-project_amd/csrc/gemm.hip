// bf16 "linear" GEMM with fused epilogue for the towers (gfx950):
//   Y[m][n] = act(sum_k X[m][k] * W[n][k] + bias[n]) (+ R[m][n]),  X, W, R, Y bf16, f32 accumulate.
// nn.Linear layout (W = [out][in]): both operands K-contiguous, so both MFMA fragments are 16-byte
// row reads.  Replaces every nn.Linear of timm Swin / HF BERT on the path (fusion.py:198-199,
// 322-325): QKV, attention output (+residual), FFN1 (+GELU), FFN2 (+residual), PatchMerging
// reduction, and the 4x4/s4 patch-embed conv as an im2col GEMM.
//
// Structure (cdna_hip_programming.md §5 "minimum 2-phase" + glds + T1/T2):
//  * tile 128x128x64, 256 threads = 4 waves (2x2), wave tile 64x64 = 4x4 v_mfma_f32_16x16x32_bf16;
//  * operands go HBM -> LDS with global_load_lds_dwordx4 (no VGPR staging); the LDS image is
//    lane-linear per wave instruction (8 rows x 128 B), and the bank-conflict swizzle
//    (16-B chunk c of row r lives at chunk c ^ ((r>>1)&7)) is applied on the per-lane SOURCE
//    address and again on the ds_read_b128 fragment read (rule 21: same involution both sides);
//  * rows past M / N and chunks past K read a 16-byte zero page, so tails need no branches;
//  * two LDS stages: the loads of k-tile t+1 are issued before the MFMAs of tile t;
//  * XCD-aware bijective block remap: the N/128 tiles sharing one 128-row X panel run on one XCD;
//  * epilogue: bias + GELU in registers, tile staged through LDS as bf16, then written (with the
//    residual add) as 16-byte row chunks — coalesced 128-B rows instead of 2-byte scatters.
#include "common.h"

namespace {

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int BM = 128, BN = 128, BK = 64;
constexpr int TILE = BM * BK;          // bf16 elements per operand per stage (16 KiB)
constexpr int EPI_LD = 64 + 8;         // bf16 row stride of a wave's 64x64 epilogue tile

__device__ __attribute__((aligned(16))) uint4 g_zero_page[4];  // zero-initialised

__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

typedef __attribute__((address_space(3))) void* lds_ptr_t;

template <int ACT, bool HAS_BIAS, bool HAS_RES>
__global__ __launch_bounds__(256, 2) void gemm_bf16_tn(const uint16_t* __restrict__ X,
                                                        const uint16_t* __restrict__ W,
                                                        const float* __restrict__ bias,
                                                        const uint16_t* __restrict__ R,
                                                        uint16_t* __restrict__ Y, int64_t M, int N,
                                                        int K, int tiles_m, int tiles_n) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[2 * 2 * TILE];  // [stage][A|B][128][64]

  const int nwg = tiles_m * tiles_n;
  const int orig = blockIdx.x;
  const int q = nwg / 8, r8 = nwg % 8, xcd = orig % 8;
  const int wg = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + orig / 8;
  const int tm = wg / tiles_n, tn = wg % tiles_n;
  const int64_t m0 = (int64_t)tm * BM;
  const int n0 = tn * BN;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  // glds addressing: wave w stages rows [32w, 32w+32) of each operand, 4 instructions of 8 rows;
  // lane i of instruction j writes LDS row 32w + 8j + i/8, physical chunk i%8.
  const int prow_in = lane >> 3, pch = lane & 7;
  const uint16_t* srcA[4];
  const uint16_t* srcB[4];
  int lchk[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int row = wave * 32 + j * 8 + prow_in;
    lchk[j] = swz(row, pch) * 8;  // logical k offset (elements) this lane fetches within a k-tile
    const int64_t gm = m0 + row;
    const int gn = n0 + row;
    srcA[j] = gm < M ? X + gm * K : nullptr;
    srcB[j] = gn < N ? W + (int64_t)gn * K : nullptr;
  }
  const uint16_t* zp = (const uint16_t*)g_zero_page;

  auto stage = [&](int s, int k0) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = k0 + lchk[j];
      const bool kin = k < K;
      const uint16_t* a = (srcA[j] && kin) ? srcA[j] + k : zp;
      const uint16_t* b = (srcB[j] && kin) ? srcB[j] + k : zp;
      uint16_t* la = lds + (s * 2 + 0) * TILE + (wave * 32 + j * 8) * BK;
      uint16_t* lb = lds + (s * 2 + 1) * TILE + (wave * 32 + j * 8) * BK;
      __builtin_amdgcn_global_load_lds((const void*)a, (lds_ptr_t)la, 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)b, (lds_ptr_t)lb, 16, 0, 0);
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int nk = (K + BK - 1) / BK;
  const int fr = lane & 15, fq = lane >> 4;
  stage(0, 0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int s = kt & 1;
    if (kt + 1 < nk) stage(s ^ 1, (kt + 1) * BK);
    const uint16_t* la = lds + (s * 2 + 0) * TILE;
    const uint16_t* lb = lds + (s * 2 + 1) * TILE;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 a[4], b[4];
      const int ch = ks * 4 + fq;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int rowa = wm * 64 + i * 16 + fr;
        const int rowb = wn * 64 + i * 16 + fr;
        a[i] = *(const bf16x8*)(la + rowa * BK + swz(rowa, ch) * 8);
        b[i] = *(const bf16x8*)(lb + rowb * BK + swz(rowb, ch) * 8);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();  // waits the in-flight glds (vmcnt(0)) and every wave's reads of stage s
  }

  // ---- epilogue: bias/act in registers -> bf16 tile in LDS -> 16-B row chunks (+ residual)
  uint16_t* et = lds + wave * 64 * EPI_LD;  // reuses the (now idle) staging buffers
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int nl = j * 16 + fr;
    const int n = n0 + wn * 64 + nl;
    const float bv = (HAS_BIAS && n < N) ? bias[n] : 0.0f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int rg = 0; rg < 4; ++rg) {
        float v = acc[i][j][rg] + bv;
        if (ACT == 1) v = mmr::gelu_erf(v);
        et[(i * 16 + fq * 4 + rg) * EPI_LD + nl] = mmr::f2bf(v);
      }
    }
  }
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's LDS writes landed
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int c = it * 64 + lane;
    const int rl = c >> 3, cc = (c & 7) * 8;
    const int64_t m = m0 + wm * 64 + rl;
    const int n = n0 + wn * 64 + cc;
    if (m >= M || n >= N) continue;
    bf16x8 v = *(const bf16x8*)(et + rl * EPI_LD + cc);
    if (HAS_RES) {
      const bf16x8 rr = *(const bf16x8*)(R + m * N + n);
#pragma unroll
      for (int e = 0; e < 8; ++e)
        v[e] = (short)mmr::f2bf(mmr::bf2f((uint16_t)v[e]) + mmr::bf2f((uint16_t)rr[e]));
    }
    *(bf16x8*)(Y + m * N + n) = v;
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
  MMR_REQUIRE(k % 8 == 0 && n % 8 == 0, "mmr_linear_bf16: K=%d and N=%d must be multiples of 8", k, n);
  MMR_REQUIRE(act == 0 || act == 1, "mmr_linear_bf16: act=%d", act);
  MMR_REQUIRE(mmr::ceil_div(m, BM) * mmr::ceil_div(n, BN) < (int64_t(1) << 31), "mmr_linear_bf16: grid too large");
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
