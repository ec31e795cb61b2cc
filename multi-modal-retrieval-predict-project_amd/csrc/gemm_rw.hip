// Resident-weight streaming GEMM for the short-K, narrow-N tower linears (Swin patch embed, stage-2
// qkv / proj, the stage-1 -> 2 PatchMerging reduction):  Y = X W^T + b (+ R), X [M][K] bf16,
// W [N][K] bf16 (nn.Linear), K in {64, 192}.  These shapes are HBM-bound (K = 64 ... 192:
// 2K bytes read and 2N written per token against 2NK flops), and the general GEMM tiles re-stream
// W per 256-row tile and pay a K-loop prologue per tile that such short K never amortises
// (M = 200704, N = 576, K = 192: 124 us = 2.5 TB/s).
//
// Here W stays in LDS for the whole launch: the launcher splits N into P parts of NO = N / P
// channels (NO * K * 2 <= 150 KiB), each part's image loaded once per workgroup; workgroups are
// persistent (a part per blockIdx.y) and every wave walks 32-token tiles on its own (no barrier
// after the image load).  C^T orientation (v_mfma_f32_32x32x16_bf16, A = W rows from LDS, B = the
// tile's X rows straight from HBM into registers, the next tile's issued before this one's MFMAs),
// so the bf16 output leaves from registers: the image's rows are stored in the order that gives
// each lane half 8 consecutive channels per (tile, i-pair) (w2_channel of swin_mlp.hip) -> 16-B
// stores, residual read in the same chunks.  HBM per token: 2K * P + 2N (+ 2N residual) bytes.
#include <algorithm>

#include "common.h"

namespace {

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;

constexpr int vmcnt_n(int n) { return (n & 15) | (7 << 4) | (15 << 8) | ((n >> 4) << 14); }

// physical 16-B unit of logical unit q in image row r: conflict-free ds_read_b128 for the 32x32x16
// A-fragment pattern (rows lane & 31, unit 2ks + lane / 32), as swin_mlp.hip's unit_swz for 8n units
template <int U>
__host__ __device__ __forceinline__ int rw_swz(int r, int q) {
  if constexpr (U == 4) return q ^ ((r >> 2) & 3);
  else return q ^ ((r >> 1) & 7);
}
// MFMA C row 8i + 4h + rr of a 32-row tile holds channel 16(i>>1) + 8h + 4(i&1) + rr of that tile
__host__ __device__ __forceinline__ int rw_channel(int row) {
  const int u = row >> 5, rho = row & 31, i = rho >> 3, h = (rho >> 2) & 1, rr = rho & 3;
  return 32 * u + 16 * (i >> 1) + 8 * h + 4 * (i & 1) + rr;
}

// image [P][NO][K] (+ f32 bias [P][NO] after it when given): row r of part p = channel
// p * NO + rw_channel(r), 16-B units swizzled
template <int K>
__global__ __launch_bounds__(256) void rw_pack(const uint16_t* __restrict__ w, int n, int no,
                                               uint16_t* __restrict__ img) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)n * K) return;
  const int row = (int)(i / K), k = (int)(i % K);  // image row (over all parts)
  const int p = row / no, r = row % no;
  const int ch = p * no + rw_channel(r);
  img[(int64_t)row * K + 8 * rw_swz<K / 8>(r, k >> 3) + (k & 7)] = w[(int64_t)ch * K + k];
}

// NW waves, each owning whole 32-token tiles; CT output tiles (32 channels) per accumulation pass
template <int K, int CT, bool BIAS, bool RES, int NW>
__global__ __launch_bounds__(64 * NW) void gemm_rw(const uint16_t* __restrict__ X,
                                                   const uint16_t* __restrict__ img,
                                                   const float* __restrict__ bias,
                                                   const uint16_t* __restrict__ R,
                                                   uint16_t* __restrict__ Y, int64_t M, int N, int no) {
  constexpr int KS = K / 16, U = K / 8;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int part = blockIdx.y;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 31, h = lane >> 5;
  const int ntl = no / 32;  // output tiles of this part
  float* lb = (float*)(smem + (size_t)no * K * 2);
  {  // the part's image (+ bias) -> LDS by 1-KiB LDS-DMA pieces, spread over the waves
    const unsigned char* src = (const unsigned char*)(img + (int64_t)part * no * K);
    const int pieces = no * K * 2 / 1024;
    for (int pc = wave; pc < pieces; pc += NW)
      __builtin_amdgcn_global_load_lds((const void*)(src + pc * 1024 + lane * 16), (lds_ptr_t)(smem + pc * 1024), 16, 0, 0);
    if (BIAS)
      for (int c = threadIdx.x; c < no; c += 64 * NW) lb[c] = bias[part * no + c];
  }
  const int64_t ntile = (M + 31) / 32, stride = (int64_t)gridDim.x * NW;
  int64_t tile = (int64_t)blockIdx.x * NW + wave;
  auto load_x = [&](int64_t tl, bf16x8* dst) {
    int64_t tok = tl * 32 + r;
    tok = tok < M ? tok : M - 1;  // clamped row: unconditional loads (tail rows never stored)
    const uint16_t* xr = X + tok * K + 8 * h;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) dst[ks] = *(const bf16x8*)(xr + 16 * ks);
  };
  bf16x8 xn[KS];
  if (tile < ntile) load_x(tile, xn);
  __builtin_amdgcn_s_waitcnt(vmcnt_n(0));  // the image's LDS-DMA landed
  __builtin_amdgcn_s_waitcnt(0xC07F);      // lgkmcnt(0): the bias stores
  asm volatile("" ::: "memory");
  __syncthreads();
  asm volatile("" ::: "memory");
  // A-fragment base of image row r (unit 2 ks + h, swizzled per row)
  const unsigned char* wrow = smem + (size_t)r * K * 2;
  for (; tile < ntile; tile += stride) {
    bf16x8 xb[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) xb[ks] = xn[ks];
    if (tile + stride < ntile) load_x(tile + stride, xn);  // next tile's rows in flight meanwhile
    const int64_t tok = tile * 32 + r;
    for (int t0 = 0; t0 < ntl; t0 += CT) {
      uint4 rv[CT][2];
      if constexpr (RES) {  // residual chunks first: their latency hides under the MFMAs
        const int64_t tr = tok < M ? tok : M - 1;
#pragma unroll
        for (int c = 0; c < CT; ++c)
#pragma unroll
          for (int hf = 0; hf < 2; ++hf)
            rv[c][hf] = *(const uint4*)(R + tr * N + part * no + 32 * (t0 + c) + 16 * hf + 8 * h);
      }
      f32x16 acc[CT];
#pragma unroll
      for (int c = 0; c < CT; ++c) acc[c] = (f32x16){0};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int c = 0; c < CT; ++c) {
          const int row = 32 * (t0 + c);
          const bf16x8 a = *(const bf16x8*)(wrow + (size_t)row * K * 2 + rw_swz<U>(r, 2 * ks + h) * 16);
          acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, xb[ks], acc[c], 0, 0, 0);
        }
      if (tok < M) {
#pragma unroll
        for (int c = 0; c < CT; ++c)
#pragma unroll
          for (int hf = 0; hf < 2; ++hf) {  // channels 32 (t0 + c) + 16 hf + 8 h + 0..7 = acc i = 2 hf, 2 hf + 1
            const int cl = 32 * (t0 + c) + 16 * hf + 8 * h;
            float v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = acc[c][8 * hf + j] + (BIAS ? lb[cl + j] : 0.f);
            if constexpr (RES) {
              const uint32_t rw[4] = {rv[c][hf].x, rv[c][hf].y, rv[c][hf].z, rv[c][hf].w};
#pragma unroll
              for (int j = 0; j < 4; ++j) {
                v[2 * j] += __uint_as_float(rw[j] << 16);
                v[2 * j + 1] += __uint_as_float(rw[j] & 0xFFFF0000u);
              }
            }
            *(uint4*)(Y + tok * N + part * no + cl) =
                make_uint4(mmr::pack2bf(v[0], v[1]), mmr::pack2bf(v[2], v[3]), mmr::pack2bf(v[4], v[5]), mmr::pack2bf(v[6], v[7]));
          }
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

constexpr int RW_MAX_IMG = 150 * 1024;

int rw_parts(int n, int k) {
  for (int p = 1; p <= n / 32; ++p)
    if (n % p == 0 && (n / p) % 32 == 0 && (int64_t)(n / p) * k * 2 <= RW_MAX_IMG && ((n / p) / 32) % 3 == 0) return p;
  for (int p = 1; p <= n / 32; ++p)
    if (n % p == 0 && (n / p) % 32 == 0 && (int64_t)(n / p) * k * 2 <= RW_MAX_IMG) return p;
  return 0;
}

template <int K, bool B, bool RS>
void launch_rw(const uint16_t* x, const uint16_t* img, const float* bias, const uint16_t* res, uint16_t* y, int64_t m,
               int n, int parts, hipStream_t st) {
  const int no = n / parts;
  const size_t lds = (size_t)no * K * 2 + (B ? (size_t)no * 4 : 0);
  constexpr int NW = 8;
  const int per_cu = std::max(1, std::min(4, (int)((160 * 1024) / lds)));
  const int64_t tiles = (m + 31) / 32;
  const int64_t want = std::max<int64_t>(1, std::min<int64_t>((int64_t)cu_count() * per_cu / parts, (tiles + NW - 1) / NW));
  const dim3 grid((unsigned)want, (unsigned)parts);
  // CT (output tiles per accumulation pass) divides the part's tile count
  if ((no / 32) % 3 == 0)
    gemm_rw<K, 3, B, RS, NW><<<grid, dim3(64 * NW), lds, st>>>(x, img, bias, res, y, m, n, no);
  else if ((no / 32) % 2 == 0)
    gemm_rw<K, 2, B, RS, NW><<<grid, dim3(64 * NW), lds, st>>>(x, img, bias, res, y, m, n, no);
  else
    gemm_rw<K, 1, B, RS, NW><<<grid, dim3(64 * NW), lds, st>>>(x, img, bias, res, y, m, n, no);
}

}  // namespace

extern "C" int32_t mmr_linear_rw_parts(int32_t n, int32_t k) {
  // (K = 384 dropped: its 32-token tile needs more than 256 VGPRs — 21-143 spilled — and measured
  // slower than the GEMM, profiles/r03_s4_linear_rw.txt)
  if (!(k == 64 || k == 192) || n <= 0 || n % 32) return 0;
  return rw_parts(n, k);
}

extern "C" mmr_status mmr_linear_rw_pack(const uint16_t* w, int32_t n, int32_t k, uint16_t* img, void* stream) {
  mmr::clear_error();
  MMR_REQUIRE(w && img, "mmr_linear_rw_pack: NULL pointer");
  const int parts = mmr_linear_rw_parts(n, k);
  MMR_REQUIRE(parts > 0, "mmr_linear_rw_pack: N=%d K=%d not supported (K in {64, 192}, N %% 32 == 0, N/P * K * 2 <= 150 KiB)", n, k);
  const int no = n / parts;
  hipStream_t st = mmr::as_stream(stream);
  const dim3 grid((unsigned)mmr::ceil_div((int64_t)n * k, 256));
  if (k == 64) rw_pack<64><<<grid, 256, 0, st>>>(w, n, no, img);
  else rw_pack<192><<<grid, 256, 0, st>>>(w, n, no, img);
  MMR_LAUNCH_CHECK();
  return MMR_OK;
}

extern "C" mmr_status mmr_linear_rw(const uint16_t* x, const uint16_t* img, const float* bias, const uint16_t* residual,
                                    uint16_t* y, int64_t m, int32_t n, int32_t k, void* stream) {
  mmr::clear_error();
  MMR_REQUIRE(x && img && y, "mmr_linear_rw: NULL pointer");
  const int parts = mmr_linear_rw_parts(n, k);
  MMR_REQUIRE(parts > 0 && m >= 0, "mmr_linear_rw: M=%lld N=%d K=%d not supported", (long long)m, n, k);
  if (m == 0) return MMR_OK;
  hipStream_t st = mmr::as_stream(stream);
  const bool hb = bias != nullptr, hr = residual != nullptr;
#define RW_K(KK)                                                                         \
  if (k == KK) {                                                                         \
    if (hb && hr) launch_rw<KK, true, true>(x, img, bias, residual, y, m, n, parts, st);   \
    else if (hb) launch_rw<KK, true, false>(x, img, bias, residual, y, m, n, parts, st);   \
    else if (hr) launch_rw<KK, false, true>(x, img, bias, residual, y, m, n, parts, st);   \
    else launch_rw<KK, false, false>(x, img, bias, residual, y, m, n, parts, st);          \
  }
  RW_K(64)
  else RW_K(192)
#undef RW_K
  MMR_LAUNCH_CHECK();
  return MMR_OK;
}
