// Fused Swin attention sub-block for the narrow stage (C = 96, 3 heads of 32):
//   y = x + proj(W-MSA(LN1(x)))        (timm SwinTransformerBlock._attn + residual,
//                                        reference fusion.py:198-199 via timm Swin-T)
// including the cyclic shift (torch.roll), window partition / reverse, relative-position bias and
// the shifted-window mask.  The unfused chain moves ~2 GB per stage-1 block through HBM (LN1 out,
// 288-wide QKV, attention out, proj in/out); this kernel reads x once and writes y once.
//
// Layout: one workgroup of 4 waves per CU, persistent over windows; each wave owns whole windows
// (49 tokens, padded to 64 = two 32-token MFMA tiles) and needs no barrier after the one-time
// weight load.  All GEMMs are v_mfma_f32_32x32x16_bf16 in the C^T orientation (A = weight rows
// from LDS, B = tokens), so every intermediate — LN'd x, K^T, Q^T, V, S^T, P, O^T — is produced
// in exactly the register fragment the next MFMA consumes (one shared k-permutation
// 16s + 8(j>>2) + 4h + (j&3) on both operands; the proj weight columns are stored permuted to
// match).  The proj weight rows are stored in the order that leaves each lane half with 8
// consecutive output channels (16-B stores, residual read with the same chunking as LN).
// LDS: the packed weights + f32 parameters (76.8 KB, resident) and, per wave, a double-buffered
// copy of its window's x (gathered through the roll by global_load_lds, next window prefetched).
#include <float.h>
#include <math.h>

#include <algorithm>

#include "common.h"

namespace {

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;

constexpr int vmcnt_n(int n) { return (n & 15) | (7 << 4) | (15 << 8) | ((n >> 4) << 14); }

constexpr int AC = 96, AH = 3, ADH = 32, AWS = 7, ATOK = 49;
constexpr int QKV_E = 3 * AC * AC;            // bf16 elements of the QKV image
constexpr int PROJ_E = AC * AC;
constexpr int PAR_F = 3 * AC + AC + 2 * AC;   // qkv_b, proj_b, ln_g, ln_b (f32)
constexpr int IMG_B = 76800;                  // (QKV_E + PROJ_E) * 2 + PAR_F * 4 = 76032, padded to 1-KiB pieces
constexpr int XCH = 640;                      // 16-B chunks per x buffer (49 x 12 = 588 used)
constexpr int XBUF_B = XCH * 16;
constexpr int LDS_B = IMG_B + 4 * 2 * XBUF_B;
static_assert((QKV_E + PROJ_E) * 2 + PAR_F * 4 <= IMG_B, "image size");
static_assert(LDS_B <= 160 * 1024, "LDS budget");

// conflict-free 16-B unit permutation for 12-unit rows read as 32x32x16 A fragments (rows =
// lane & 31, unit 2ks + (lane >> 5)); checked exhaustively (see swin_mlp.hip)
__host__ __device__ __forceinline__ int u12(int r, int q) { return (q + ((r >> 2) & 3)) % 12; }
__host__ __device__ __forceinline__ int u12_inv(int r, int p) { return (p - ((r >> 2) & 3) + 12) % 12; }
// C-fragment k-permutation (see header) and the output-row order of the proj weight
__host__ __device__ __forceinline__ int kperm(int pos) {
  const int h = (pos >> 3) & 1, j = pos & 7;
  return (pos & ~15) + 8 * (j >> 2) + 4 * h + (j & 3);
}
__host__ __device__ __forceinline__ int chan_of_row(int row) {
  const int u = row >> 5, rho = row & 31, i = rho >> 3, h = (rho >> 2) & 1, rr = rho & 3;
  return 32 * u + 16 * (i >> 1) + 8 * h + 4 * (i & 1) + rr;
}

__global__ __launch_bounds__(256) void swin_attn_pack(const uint16_t* __restrict__ qkv_w,
                                                      const float* __restrict__ qkv_b,
                                                      const uint16_t* __restrict__ proj_w,
                                                      const float* __restrict__ proj_b,
                                                      const float* __restrict__ ln_g,
                                                      const float* __restrict__ ln_b,
                                                      unsigned char* __restrict__ img) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  uint16_t* e16 = (uint16_t*)img;
  float* pf = (float*)(img + (QKV_E + PROJ_E) * 2);
  if (i < QKV_E) {  // qkv.weight [3C][C], rows (q|k|v, head, dh)
    const int row = i / AC, col = i % AC, q = col >> 3;
    e16[row * AC + 8 * u12(row, q) + (col & 7)] = qkv_w[i];
  } else if (i < QKV_E + PROJ_E) {  // proj.weight [C][C], rows / columns permuted
    const int k = i - QKV_E, row = k / AC, pos = k % AC, q = pos >> 3;
    e16[QKV_E + row * AC + 8 * u12(row, q) + (pos & 7)] = proj_w[chan_of_row(row) * AC + kperm(pos)];
  } else if (i < QKV_E + PROJ_E + PAR_F) {
    const int k = i - QKV_E - PROJ_E;
    pf[k] = k < 3 * AC ? qkv_b[k] : k < 4 * AC ? proj_b[k - 3 * AC] : k < 5 * AC ? ln_g[k - 4 * AC] : ln_b[k - 5 * AC];
  } else if (i + PAR_F < IMG_B / 2) {
    e16[i + PAR_F] = 0;  // zero tail (the f32 block spans 2 bf16 slots per thread above)
  }
}

__device__ __forceinline__ bf16x8 pack_frag(const f32x16& a, int s) {
  return __builtin_bit_cast(bf16x8, make_uint4(mmr::pack2bf(a[8 * s + 0], a[8 * s + 1]), mmr::pack2bf(a[8 * s + 2], a[8 * s + 3]),
                                               mmr::pack2bf(a[8 * s + 4], a[8 * s + 5]), mmr::pack2bf(a[8 * s + 6], a[8 * s + 7])));
}

__global__ __launch_bounds__(256) void swin_attn_block(const uint16_t* __restrict__ x,
                                                       const unsigned char* __restrict__ img,
                                                       const float* __restrict__ bias,
                                                       uint16_t* __restrict__ y, int nimg, int H,
                                                       int shift, float eps) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const uint16_t* Wqkv = (const uint16_t*)smem;
  const uint16_t* Wproj = Wqkv + QKV_E;
  const float* P = (const float*)(smem + (QKV_E + PROJ_E) * 2);
  const float* Pqb = P;
  const float* Ppb = P + 3 * AC;
  const float* Pg = P + 4 * AC;
  const float* Pb = P + 5 * AC;

  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 31, h = lane >> 5;
  unsigned char* xb0 = smem + IMG_B + wave * 2 * XBUF_B;

  // one-time weight image load (75 pieces over 4 waves)
  for (int p = wave; p < IMG_B / 1024; p += 4)
    __builtin_amdgcn_global_load_lds((const void*)(img + p * 1024 + lane * 16), (lds_ptr_t)(smem + p * 1024), 16, 0, 0);

  const int nw1 = H / AWS, nwin = nw1 * nw1;
  const int64_t total = (int64_t)nimg * nwin;
  const int64_t stride = (int64_t)gridDim.x * 4;
  int64_t win = (int64_t)blockIdx.x * 4 + wave;

  // token -> row of x for window w (rolled by -shift: window token (hr, wr) reads (hr+s, wr+s))
  auto tok_row = [&](int64_t w, int t) -> int64_t {
    const int64_t bi = w / nwin;
    const int wi = (int)(w % nwin), wy = wi / nw1, wx = wi % nw1;
    const int hr = wy * AWS + t / AWS, wr = wx * AWS + t % AWS;
    const int h0 = (hr + shift) % H, w0 = (wr + shift) % H;
    return bi * H * H + (int64_t)h0 * H + w0;
  };
  // gather window w's x into buffer `buf`: LDS chunk p = token * 12 + u12(token, unit)
  auto gather = [&](int64_t w, int buf) {
    unsigned char* dst = xb0 + buf * XBUF_B;
#pragma unroll
    for (int it = 0; it < XCH / 64; ++it) {
      const int p = it * 64 + lane;
      int t = p / 12;
      int unit = u12_inv(t, p % 12);
      if (p >= ATOK * 12) t = 0, unit = 0;  // pad lanes re-read a valid chunk into the tail
      const uint16_t* src = x + tok_row(w, t) * AC + unit * 8;
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_ptr_t)(dst + it * 1024), 16, 0, 0);
    }
  };
  if (win < total) gather(win, 0);
  __builtin_amdgcn_s_waitcnt(vmcnt_n(0));
  __builtin_amdgcn_s_waitcnt(0xC07F);
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();  // weights visible to every wave; no barrier after this point
  asm volatile("" ::: "memory");

  const float scale = 0.17677669529663687f;  // 32^-0.5
  int buf = 0;
  for (; win < total; win += stride, buf ^= 1) {
    __builtin_amdgcn_s_waitcnt(vmcnt_n(0));  // this window's gather (and last window's stores)
    asm volatile("" ::: "memory");
    const unsigned char* xs = xb0 + buf * XBUF_B;
    const int wi = (int)(win % nwin), wy = wi / nw1, wx = wi % nw1;
    const int type = shift > 0 ? ((wy == nw1 - 1) ? 2 : 0) + ((wx == nw1 - 1) ? 1 : 0) : 0;

    // ---- LN1 -> hB[t2][ks]: B fragments, token t2*32 + r, channels 16ks + 8h + 0..7
    bf16x8 hB[2][AC / 16];
#pragma unroll
    for (int t2 = 0; t2 < 2; ++t2) {
      const int t = t2 * 32 + r;
      const bool ok = t < ATOK;
      float v[AC / 16][8];
      float s = 0.f;
#pragma unroll
      for (int ks = 0; ks < AC / 16; ++ks) {
        const bf16x8 raw = ok ? *(const bf16x8*)(xs + (t * 12 + u12(t, 2 * ks + h)) * 16) : (bf16x8){0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          v[ks][j] = mmr::bf2f((uint16_t)raw[j]);
          s += v[ks][j];
        }
      }
      s += __shfl_xor(s, 32, 64);
      const float mean = s * (1.0f / AC);
      float ss = 0.f;
#pragma unroll
      for (int ks = 0; ks < AC / 16; ++ks)
#pragma unroll
        for (int j = 0; j < 8; ++j) ss += (v[ks][j] - mean) * (v[ks][j] - mean);
      ss += __shfl_xor(ss, 32, 64);
      const float rstd = rsqrtf(ss * (1.0f / AC) + eps);
#pragma unroll
      for (int ks = 0; ks < AC / 16; ++ks) {
        const int k0 = 16 * ks + 8 * h;
        const f32x4 g0 = *(const f32x4*)(Pg + k0), g1 = *(const f32x4*)(Pg + k0 + 4);
        const f32x4 c0 = *(const f32x4*)(Pb + k0), c1 = *(const f32x4*)(Pb + k0 + 4);
        const float gg[8] = {g0[0], g0[1], g0[2], g0[3], g1[0], g1[1], g1[2], g1[3]};
        const float cc[8] = {c0[0], c0[1], c0[2], c0[3], c1[0], c1[1], c1[2], c1[3]};
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = (v[ks][j] - mean) * rstd * gg[j] + cc[j];
        hB[t2][ks] = __builtin_bit_cast(bf16x8, make_uint4(mmr::pack2bf(o[0], o[1]), mmr::pack2bf(o[2], o[3]),
                                                           mmr::pack2bf(o[4], o[5]), mmr::pack2bf(o[6], o[7])));
      }
    }

    // every head's O^T (bf16 fragments) is kept and the proj runs after the head loop, one token tile
    // at a time: 48 registers of packed O instead of 96 of proj accumulators live across the heads
    bf16x8 ost[AH][2][2];

    auto wrow = [&](const uint16_t* W, int row, int ks) {  // A/B fragment: weight row, k-step ks
      return *(const bf16x8*)(W + row * AC + 8 * u12(row, 2 * ks + h));
    };

#pragma unroll
    for (int hd = 0; hd < AH; ++hd) {
      const float* bt = bias + ((int64_t)type * AH + hd) * 4096;  // dense rel-pos + mask, L2-resident
      // K^T (C^T: lane (token r, half h) holds dh = 8i + 4h + rr) and V (swapped: lane (dh r,
      // half h) holds tokens 8i + 4h + rr) of both token tiles, packed into MFMA fragments
      bf16x8 kf[2][2], vf[2][2];
      // biases start the accumulators (no VALU pass over the MFMA results)
      f32x16 kb, vb;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const f32x4 bkk = *(const f32x4*)(Pqb + AC + hd * ADH + 8 * i + 4 * h);
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) kb[4 * i + rr] = bkk[rr];
      }
      {
        const float bv = Pqb[2 * AC + hd * ADH + r];
#pragma unroll
        for (int e = 0; e < 16; ++e) vb[e] = bv;
      }
#pragma unroll
      for (int t2 = 0; t2 < 2; ++t2) {
        f32x16 ak = kb;
#pragma unroll
        for (int ks = 0; ks < AC / 16; ++ks)
          ak = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wrow(Wqkv, AC + hd * ADH + r, ks), hB[t2][ks], ak, 0, 0, 0);
        kf[t2][0] = pack_frag(ak, 0);
        kf[t2][1] = pack_frag(ak, 1);
      }
#pragma unroll
      for (int t2 = 0; t2 < 2; ++t2) {
        f32x16 av = vb;
#pragma unroll
        for (int ks = 0; ks < AC / 16; ++ks)
          av = __builtin_amdgcn_mfma_f32_32x32x16_bf16(hB[t2][ks], wrow(Wqkv, 2 * AC + hd * ADH + r, ks), av, 0, 0, 0);
        vf[t2][0] = pack_frag(av, 0);
        vf[t2][1] = pack_frag(av, 1);
      }

#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        // this query tile's bias rows, in flight while Q^T is computed
        f32x4 bq[2][4];
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
          for (int i = 0; i < 4; ++i) bq[kt][i] = *(const f32x4*)(bt + (qt * 32 + r) * 64 + kt * 32 + 8 * i + 4 * h);
        if (hd == AH - 1 && qt == 1 && win + stride < total) gather(win + stride, buf ^ 1);  // after the last bias loads
        bf16x8 qf[2];
        {
          // q = (Wq x + bq) * scale before the bf16 rounding (timm scales q before q @ k^T), bias in
          // the accumulator
          f32x16 aq;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const f32x4 bqq = *(const f32x4*)(Pqb + hd * ADH + 8 * i + 4 * h);
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) aq[4 * i + rr] = bqq[rr];
          }
#pragma unroll
          for (int ks = 0; ks < AC / 16; ++ks)
            aq = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wrow(Wqkv, hd * ADH + r, ks), hB[qt][ks], aq, 0, 0, 0);
#pragma unroll
          for (int e = 0; e < 16; ++e) aq[e] *= scale;
          qf[0] = pack_frag(aq, 0);
          qf[1] = pack_frag(aq, 1);
        }
        // S^T[key][query] = K (scale Q)^T + bias (the rel-pos / mask rows start the accumulator);
        // softmax over the 64 keys of query r
        f32x16 s[2];
        float mx = -FLT_MAX;
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) s[kt][4 * i + rr] = bq[kt][i][rr];
#pragma unroll
          for (int k2 = 0; k2 < 2; ++k2) s[kt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf[kt][k2], qf[k2], s[kt], 0, 0, 0);
#pragma unroll
          for (int e = 0; e < 16; ++e) mx = fmaxf(mx, s[kt][e]);
        }
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        const float mxl = mx * 1.4426950408889634f;  // exp(s - mx) = exp2(s log2e - mx log2e): one fma
        float sum = 0.f;
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const float p = __builtin_amdgcn_exp2f(fmaf(s[kt][e], 1.4426950408889634f, -mxl));
            s[kt][e] = p;
            sum += p;
          }
        sum += __shfl_xor(sum, 32, 64);
        // O^T[dh][query] = V^T P^T
        f32x16 o = {0};
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
          for (int k2 = 0; k2 < 2; ++k2) o = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf[kt][k2], pack_frag(s[kt], k2), o, 0, 0, 0);
        const float inv = __builtin_amdgcn_rcpf(sum);
#pragma unroll
        for (int e = 0; e < 16; ++e) o[e] *= inv;
        ost[hd][qt][0] = pack_frag(o, 0);
        ost[hd][qt][1] = pack_frag(o, 1);
      }
    }

    // ---- proj: out^T[c][query] = Wproj[c][hd*32 + dh] O^T[dh][query] (+ proj_b in the accumulator);
    // y = x + out: lane half h holds channels 32u + 16 hf + 8h + 0..7 of token r
#pragma unroll
    for (int t2 = 0; t2 < 2; ++t2) {
      f32x16 acc[3];
#pragma unroll
      for (int u = 0; u < 3; ++u) {
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
          const int c0 = 32 * u + 16 * hf + 8 * h;
          const f32x4 b0 = *(const f32x4*)(Ppb + c0), b1 = *(const f32x4*)(Ppb + c0 + 4);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            acc[u][8 * hf + j] = b0[j];
            acc[u][8 * hf + 4 + j] = b1[j];
          }
        }
#pragma unroll
        for (int hd = 0; hd < AH; ++hd) {
          acc[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wrow(Wproj, 32 * u + r, 2 * hd), ost[hd][t2][0], acc[u], 0, 0, 0);
          acc[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wrow(Wproj, 32 * u + r, 2 * hd + 1), ost[hd][t2][1], acc[u], 0, 0, 0);
        }
      }
      const int t = t2 * 32 + r;
      if (t >= ATOK) continue;
      uint16_t* yr = y + tok_row(win, t) * AC;
#pragma unroll
      for (int u = 0; u < 3; ++u)
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
          const int c0 = 32 * u + 16 * hf + 8 * h;
          const bf16x8 xv = *(const bf16x8*)(xs + (t * 12 + u12(t, c0 >> 3)) * 16);
          float v[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = acc[u][8 * hf + j] + mmr::bf2f((uint16_t)xv[j]);
          *(uint4*)(yr + c0) = make_uint4(mmr::pack2bf(v[0], v[1]), mmr::pack2bf(v[2], v[3]),
                                          mmr::pack2bf(v[4], v[5]), mmr::pack2bf(v[6], v[7]));
        }
    }
  }
  __builtin_amdgcn_s_waitcnt(vmcnt_n(0));  // no LDS-DMA may land after the workgroup retires
}

int cu_count() {
  static int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
      v = 256;
    return v;
  }();
  return n;
}

}  // namespace

extern "C" {

int64_t mmr_swin_attn_block_pack_bytes(int32_t c) { return c == AC ? IMG_B : 0; }

mmr_status mmr_swin_attn_block_pack(const uint16_t* qkv_w, const float* qkv_b, const uint16_t* proj_w,
                                    const float* proj_b, const float* ln_g, const float* ln_b,
                                    void* pack, int32_t c, void* stream) {
  mmr::clear_error();
  MMR_REQUIRE(qkv_w && qkv_b && proj_w && proj_b && ln_g && ln_b && pack, "mmr_swin_attn_block_pack: NULL pointer");
  if (c != AC) {
    mmr::set_error("mmr_swin_attn_block_pack: C=%d not built (96)", c);
    return MMR_ERR_UNSUPPORTED;
  }
  swin_attn_pack<<<dim3((unsigned)mmr::ceil_div(IMG_B / 2, 256)), 256, 0, mmr::as_stream(stream)>>>(
      qkv_w, qkv_b, proj_w, proj_b, ln_g, ln_b, (unsigned char*)pack);
  MMR_LAUNCH_CHECK();
  return MMR_OK;
}

mmr_status mmr_swin_attn_block(const uint16_t* x, const void* pack, const float* bias, uint16_t* y,
                               int32_t b, int32_t hw, int32_t c, int32_t ws, int32_t shift, float eps,
                               void* stream) {
  mmr::clear_error();
  MMR_REQUIRE(x && pack && bias && y, "mmr_swin_attn_block: NULL pointer");
  MMR_REQUIRE(x != y, "mmr_swin_attn_block: in-place not supported");
  MMR_REQUIRE(b >= 0 && hw > 0 && hw % AWS == 0 && shift >= 0 && shift < AWS,
              "mmr_swin_attn_block: b=%d hw=%d shift=%d", b, hw, shift);
  if (c != AC || ws != AWS) {
    mmr::set_error("mmr_swin_attn_block: C=%d ws=%d not built (96, 7)", c, ws);
    return MMR_ERR_UNSUPPORTED;
  }
  if (b == 0) return MMR_OK;
  const int64_t wins = (int64_t)b * (hw / AWS) * (hw / AWS);
  const int64_t grid = std::min<int64_t>(cu_count(), (wins + 3) / 4);
  swin_attn_block<<<dim3((unsigned)grid), 256, LDS_B, mmr::as_stream(stream)>>>(x, (const unsigned char*)pack,
                                                                                 bias, y, b, hw, shift, eps);
  MMR_LAUNCH_CHECK();
  return MMR_OK;
}

}  // extern "C"
