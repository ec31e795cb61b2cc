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
// LDS: the packed weights in MFMA fragment order + f32 parameters (76.8 KB, resident) and, per
// wave, a double-buffered copy of its window's x (gathered through the roll by global_load_lds,
// next window prefetched; 208-B token rows).
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
constexpr int XCH = 640;                      // 16-B chunks per x buffer (49 tokens x 13 = 637 used)
constexpr int XT = 13;                        // chunks per token row in LDS: 12 + 1 pad (208-B stride
                                              // puts 16 consecutive tokens on distinct bank quads)
constexpr int XBUF_B = XCH * 16;
constexpr int GCO_B = (XCH / 64) * 64 * 4;     // per-lane gather coordinates (shared by the waves)
constexpr int NWV = 8;                        // waves per workgroup: 2 per SIMD (<= 256 registers)
constexpr int LDS_B = IMG_B + NWV * XBUF_B + GCO_B;
static_assert((QKV_E + PROJ_E) * 2 + PAR_F * 4 <= IMG_B, "image size");
static_assert(LDS_B <= 160 * 1024, "LDS budget");

// C-fragment k-permutation (see header) and the output-row order of the proj weight
__host__ __device__ __forceinline__ int kperm(int pos) {
  const int h = (pos >> 3) & 1, j = pos & 7;
  return (pos & ~15) + 8 * (j >> 2) + 4 * h + (j & 3);
}
__host__ __device__ __forceinline__ int chan_of_row(int row) {
  const int u = row >> 5, rho = row & 31, i = rho >> 3, h = (rho >> 2) & 1, rr = rho & 3;
  return 32 * u + 16 * (i >> 1) + 8 * h + 4 * (i & 1) + rr;
}

// weight images in MFMA fragment order: the 16-B slot of (32-row tile, k-step ks, lane) holds row
// 32 tile + (lane & 31), k = 16 ks + 8 (lane >> 5) + 0..7, so a fragment read is lane * 16 + an
// immediate (no per-lane address registers, conflict-free)
__host__ __device__ __forceinline__ int frag_pos(int row, int col) {
  return (((row >> 5) * (AC / 16) + (col >> 4)) * 64 + ((col >> 3) & 1) * 32 + (row & 31)) * 8 + (col & 7);
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
  if (i < QKV_E) {  // qkv.weight [3C][C], rows (q|k|v, head, dh), fragment order
    const int row = i / AC, col = i % AC;
    e16[frag_pos(row, col)] = qkv_w[i];
  } else if (i < QKV_E + PROJ_E) {  // proj.weight [C][C], rows / columns permuted, fragment order
    const int k = i - QKV_E, row = k / AC, pos = k % AC;
    e16[QKV_E + frag_pos(row, pos)] = proj_w[chan_of_row(row) * AC + kperm(pos)];
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

typedef float f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2 pk(float a, float b) { return (f2){a, b}; }
// two bf16 of a packed dword -> f32 pair (2 VALU: shift + and)
__device__ __forceinline__ f2 bf2x(uint32_t u) { return (f2){__uint_as_float(u << 16), __uint_as_float(u & 0xffff0000u)}; }
__device__ __forceinline__ f2 fma2(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
// reductions across the two lane halves (lane l and l ^ 32): v_permlane32_swap, no LDS round trip
__device__ __forceinline__ float half_sum(float v) {
  const auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(p[0]) + __uint_as_float(p[1]);
}
__device__ __forceinline__ float half_max(float v) {
  const auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(p[0]), __uint_as_float(p[1]));
}

// VALU budget (the kernel is VALU-issue-bound: one wave64 VALU op occupies the SIMD 4 cycles, a
// 32x32x16 MFMA 32): all index math is 32-bit with per-lane token coordinates hoisted out of the
// window loop; softmax, LN, the q scale and the 1/sum scale run on packed-f32 (v_pk_fma/mul/add).
__global__ __launch_bounds__(NWV * 64) __attribute__((amdgpu_waves_per_eu(2, 2))) void swin_attn_block(const uint16_t* __restrict__ x,
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

  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  unsigned char* xs = smem + IMG_B + wave * XBUF_B;
  uint32_t* gco = (uint32_t*)(smem + IMG_B + NWV * XBUF_B);

  // one-time weight image load (75 pieces over the waves)
  for (int p = wave; p < IMG_B / 1024; p += NWV)
    __builtin_amdgcn_global_load_lds((const void*)(img + p * 1024 + lane * 16), (lds_ptr_t)(smem + p * 1024), 16, 0, 0);

  const int nw1 = H / AWS, nwin = nw1 * nw1;
  const int total = nimg * nwin;  // host-checked < 2^31
  const int stride = gridDim.x * NWV;
  int win = blockIdx.x * NWV + wave;

  // per-lane window-token coordinates, fixed for the whole kernel: LDS chunk p holds token p / 13,
  // 16-B unit p % 13 (the pad unit 12 and the tail re-read token 0's unit 0); packed
  // (ty | tx << 8 | unit << 16), table [it][lane] in LDS
  for (int p = threadIdx.x; p < XCH; p += NWV * 64) {
    int t = p / XT, unit = p % XT;
    if (unit == XT - 1 || t >= ATOK) t = 0, unit = 0;
    gco[p] = (uint32_t)(t / AWS) | ((uint32_t)(t % AWS) << 8) | ((uint32_t)unit << 16);
  }
  // window token -> row of x inside the image (rolled by -shift: token (hr, wr) reads (hr+s, wr+s))
  // (wrap as an unsigned min: no VGPR copy of H for a v_cndmask — such copies were hoisted and spilled)
  auto img_row = [&](int hs, int ws_, int ty, int tx) -> int {
    uint32_t hh = (uint32_t)(hs + ty), ww = (uint32_t)(ws_ + tx);
    hh = min(hh, hh - (uint32_t)H);
    ww = min(ww, ww - (uint32_t)H);
    return (int)(hh * (uint32_t)H + ww);
  };
  struct Win {
    const uint16_t* xi;
    uint16_t* yi;
    int hs, ws_, type;
  };
  auto win_of = [&](int w) -> Win {
    // wave-uniform: pinned to SGPRs so the pointers below stay scalar
    const int bi = __builtin_amdgcn_readfirstlane(w / nwin), wi = w - bi * nwin;
    const int wy = __builtin_amdgcn_readfirstlane(wi / nw1), wx = wi - wy * nw1;
    const size_t ioff = (size_t)bi * H * H * AC;
    Win o;
    o.xi = x + ioff;
    o.yi = y + ioff;
    o.hs = wy * AWS + shift;
    o.ws_ = wx * AWS + shift;
    o.type = shift > 0 ? ((wy == nw1 - 1) ? 2 : 0) + ((wx == nw1 - 1) ? 1 : 0) : 0;
    return o;
  };
  // gather window w's x into this wave's buffer: LDS chunk p = token * 13 + unit
  auto gather = [&](const Win& wd, int ln) {
    unsigned char* dst = xs;
#pragma unroll
    for (int it = 0; it < XCH / 64; ++it) {
      const uint32_t c = gco[it * 64 + ln];
      const int row = img_row(wd.hs, wd.ws_, (int)(c & 0xff), (int)((c >> 8) & 0xff));
      const uint16_t* src = wd.xi + row * AC + (int)(c >> 16) * 8;
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_ptr_t)(dst + it * 1024), 16, 0, 0);
    }
  };
  __syncthreads();  // gather table
  if (win < total) gather(win_of(win), lane);
  __builtin_amdgcn_s_waitcnt(vmcnt_n(0));
  __builtin_amdgcn_s_waitcnt(0xC07F);
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();  // weights visible to every wave; no barrier after this point
  asm volatile("" ::: "memory");

  const float scale = 0.17677669529663687f;  // 32^-0.5
  const f2 L2E = pk(1.4426950408889634f, 1.4426950408889634f);
  for (; win < total; win += stride) {
    // this window's gather; the previous window's 12 row stores (issued after it) may stay in flight
    __builtin_amdgcn_s_waitcnt(vmcnt_n(12));
    asm volatile("" ::: "memory");
    const Win wd = win_of(win);
    // every lane-derived value is recomputed per window from an opaque lane id: held across the
    // loop they were spilled, and the reloads at the loop top (vmcnt ops) waited for the previous
    // window's row stores
    int lnv;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lnv));
    const int r = lnv & 31, h = lnv >> 5;
    const uint32_t boff = (uint32_t)(r * 64 + 4 * h);  // this lane's bias row / column offset
    float epsv;  // eps in a VGPR made per window (a hoisted copy was spilled)
    asm volatile("v_mov_b32 %0, %1" : "=v"(epsv) : "s"(eps));

    // ---- LN1 -> hB[t2][ks]: B fragments, token t2*32 + r, channels 16ks + 8h + 0..7
    bf16x8 hB[2][AC / 16];
#pragma unroll
    for (int t2 = 0; t2 < 2; ++t2) {
      const int t = t2 * 32 + r;
      const bool ok = t < ATOK;
      const unsigned char* xt = xs + (ok ? t : ATOK - 1) * (XT * 16) + 16 * h;  // pad tokens: zeroed below
      f2 v[AC / 16][4];
      f2 s2 = pk(0.f, 0.f);
#pragma unroll
      for (int ks = 0; ks < AC / 16; ++ks) {
        uint4 raw = *(const uint4*)(xt + 32 * ks);
        if (!ok) raw = make_uint4(0, 0, 0, 0);
        v[ks][0] = bf2x(raw.x);
        v[ks][1] = bf2x(raw.y);
        v[ks][2] = bf2x(raw.z);
        v[ks][3] = bf2x(raw.w);
#pragma unroll
        for (int j = 0; j < 4; ++j) s2 += v[ks][j];
      }
      float s = s2.x + s2.y;
      s = half_sum(s);
      const float mean = s * (1.0f / AC);
      const f2 nm = pk(-mean, -mean);
      f2 q2 = pk(0.f, 0.f);
#pragma unroll
      for (int ks = 0; ks < AC / 16; ++ks)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          v[ks][j] += nm;
          q2 = fma2(v[ks][j], v[ks][j], q2);
        }
      float ss = q2.x + q2.y;
      ss = half_sum(ss);
      const float rstd = rsqrtf(ss * (1.0f / AC) + epsv);
      const f2 rs = pk(rstd, rstd);
#pragma unroll
      for (int ks = 0; ks < AC / 16; ++ks) {
        const int k0 = 16 * ks + 8 * h;
        const f32x4 g0 = *(const f32x4*)(Pg + k0), g1 = *(const f32x4*)(Pg + k0 + 4);
        const f32x4 c0 = *(const f32x4*)(Pb + k0), c1 = *(const f32x4*)(Pb + k0 + 4);
        const f2 gg[4] = {pk(g0[0], g0[1]), pk(g0[2], g0[3]), pk(g1[0], g1[1]), pk(g1[2], g1[3])};
        const f2 cc[4] = {pk(c0[0], c0[1]), pk(c0[2], c0[3]), pk(c1[0], c1[1]), pk(c1[2], c1[3])};
        uint32_t o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const f2 n = fma2(v[ks][j] * rs, gg[j], cc[j]);
          o[j] = mmr::pack2bf(n.x, n.y);
        }
        hB[t2][ks] = __builtin_bit_cast(bf16x8, make_uint4(o[0], o[1], o[2], o[3]));
      }
    }

    // every head's O^T (bf16 fragments) is kept and the proj runs after the head loop, one token tile
    // at a time: 48 registers of packed O instead of 96 of proj accumulators live across the heads
    bf16x8 ost[AH][2][2];
    uint4 xv[2][3][2];  // residual rows (L2-hot), loaded before the next window's gather is issued
    uint32_t orow[2];   // element offset of each token tile's row in the image (residual + store)

    auto wfrag = [&](const uint16_t* W, int tile, int ks) {  // A/B fragment: 32-row tile, k-step ks
      return *(const bf16x8*)(W + lnv * 8 + (tile * (AC / 16) + ks) * 512);
    };

#pragma unroll
    for (int hd = 0; hd < AH; ++hd) {
      const float* bt = bias + (wd.type * AH + hd) * 4096;  // dense rel-pos + mask, L2-resident (uniform)
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
          ak = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wfrag(Wqkv, AC / 32 + hd, ks), hB[t2][ks], ak, 0, 0, 0);
        kf[t2][0] = pack_frag(ak, 0);
        kf[t2][1] = pack_frag(ak, 1);
      }
#pragma unroll
      for (int t2 = 0; t2 < 2; ++t2) {
        f32x16 av = vb;
#pragma unroll
        for (int ks = 0; ks < AC / 16; ++ks)
          av = __builtin_amdgcn_mfma_f32_32x32x16_bf16(hB[t2][ks], wfrag(Wqkv, 2 * AC / 32 + hd, ks), av, 0, 0, 0);
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
          for (int i = 0; i < 4; ++i) bq[kt][i] = *(const f32x4*)(bt + (boff + qt * 2048 + kt * 32 + 8 * i));
        __builtin_amdgcn_sched_barrier(0);  // keep the bias loads ahead of the Q chain
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
            aq = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wfrag(Wqkv, hd, ks), hB[qt][ks], aq, 0, 0, 0);
          uint32_t qp[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const f2 q = pk(aq[2 * e], aq[2 * e + 1]) * pk(scale, scale);
            qp[e] = mmr::pack2bf(q.x, q.y);
          }
          qf[0] = __builtin_bit_cast(bf16x8, make_uint4(qp[0], qp[1], qp[2], qp[3]));
          qf[1] = __builtin_bit_cast(bf16x8, make_uint4(qp[4], qp[5], qp[6], qp[7]));
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
        mx = half_max(mx);
        const float mxl = -mx * 1.4426950408889634f;  // exp(s - mx) = exp2(s log2e - mx log2e): one fma
        const f2 nmx = pk(mxl, mxl);
        f2 sum2 = pk(0.f, 0.f);
        uint32_t pp[2][8];
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const f2 a = fma2(pk(s[kt][2 * e], s[kt][2 * e + 1]), L2E, nmx);
            const f2 p2 = pk(__builtin_amdgcn_exp2f(a.x), __builtin_amdgcn_exp2f(a.y));
            sum2 += p2;
            pp[kt][e] = mmr::pack2bf(p2.x, p2.y);
          }
        float sum = sum2.x + sum2.y;
        sum = half_sum(sum);
        // O^T[dh][query] = V^T P^T
        f32x16 o = {0};
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
          for (int k2 = 0; k2 < 2; ++k2)
            o = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                vf[kt][k2], __builtin_bit_cast(bf16x8, make_uint4(pp[kt][4 * k2], pp[kt][4 * k2 + 1], pp[kt][4 * k2 + 2], pp[kt][4 * k2 + 3])),
                o, 0, 0, 0);
        const float inv = __builtin_amdgcn_rcpf(sum);
        uint32_t op[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const f2 v = pk(o[2 * e], o[2 * e + 1]) * pk(inv, inv);
          op[e] = mmr::pack2bf(v.x, v.y);
        }
        ost[hd][qt][0] = __builtin_bit_cast(bf16x8, make_uint4(op[0], op[1], op[2], op[3]));
        ost[hd][qt][1] = __builtin_bit_cast(bf16x8, make_uint4(op[4], op[5], op[6], op[7]));
      }
    }

    // every global load of this window is issued: the residual rows, then the next window's gather
    // (vmcnt retires in order, so the epilogue's wait on the residual never waits on the gather)
#pragma unroll
    for (int t2 = 0; t2 < 2; ++t2) {
      const int tc = t2 * 32 + r < ATOK ? t2 * 32 + r : 0;
      orow[t2] = (uint32_t)img_row(wd.hs, wd.ws_, tc / AWS, tc % AWS) * AC;
      const uint16_t* xr = wd.xi + orow[t2];
#pragma unroll
      for (int u = 0; u < 3; ++u)
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) xv[t2][u][hf] = *(const uint4*)(xr + 32 * u + 16 * hf + 8 * h);
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);  // LN's reads of the buffer (long done) before the DMA
    asm volatile("" ::: "memory");
    if (win + stride < total) gather(win_of(win + stride), lnv);
    // the proj's lane values from a fresh opaque lane id: an address kept from the LN phase was
    // spilled, and its reload here (a vmcnt op, younger than the gather) drained the gather
    int lnp;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lnp));
    const int rp = lnp & 31, hp = lnp >> 5;

    auto wfragp = [&](const uint16_t* W, int tile, int ks) {
      return *(const bf16x8*)(W + lnp * 8 + (tile * (AC / 16) + ks) * 512);
    };
    // ---- proj: out^T[c][query] = Wproj[c][hd*32 + dh] O^T[dh][query] (+ proj_b in the accumulator);
    // y = x + out: lane half h holds channels 32u + 16 hf + 8h + 0..7 of token r
#pragma unroll
    for (int t2 = 0; t2 < 2; ++t2) {
      const int t = t2 * 32 + rp;
      const bool tok_ok = t < ATOK;
      uint16_t* yr = wd.yi + orow[t2];
      f32x16 acc[3];
#pragma unroll
      for (int u = 0; u < 3; ++u) {
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
          const int c0 = 32 * u + 16 * hf + 8 * hp;
          const f32x4 b0 = *(const f32x4*)(Ppb + c0), b1 = *(const f32x4*)(Ppb + c0 + 4);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            acc[u][8 * hf + j] = b0[j];
            acc[u][8 * hf + 4 + j] = b1[j];
          }
        }
#pragma unroll
        for (int hd = 0; hd < AH; ++hd) {
          acc[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wfragp(Wproj, u, 2 * hd), ost[hd][t2][0], acc[u], 0, 0, 0);
          acc[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wfragp(Wproj, u, 2 * hd + 1), ost[hd][t2][1], acc[u], 0, 0, 0);
        }
      }
      if (!tok_ok) continue;
#pragma unroll
      for (int u = 0; u < 3; ++u)
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
          const int c0 = 32 * u + 16 * hf + 8 * hp;
          const uint32_t xw[4] = {xv[t2][u][hf].x, xv[t2][u][hf].y, xv[t2][u][hf].z, xv[t2][u][hf].w};
          uint32_t o[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const f2 v = pk(acc[u][8 * hf + 2 * j], acc[u][8 * hf + 2 * j + 1]) + bf2x(xw[j]);
            o[j] = mmr::pack2bf(v.x, v.y);
          }
          *(uint4*)(yr + c0) = make_uint4(o[0], o[1], o[2], o[3]);
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
  MMR_REQUIRE(wins < (int64_t)1 << 31, "mmr_swin_attn_block: %lld windows (32-bit window index)", (long long)wins);
  const int64_t grid = std::min<int64_t>(cu_count(), (wins + NWV - 1) / NWV);
  swin_attn_block<<<dim3((unsigned)grid), NWV * 64, LDS_B, mmr::as_stream(stream)>>>(x, (const unsigned char*)pack,
                                                                                 bias, y, b, hw, shift, eps);
  MMR_LAUNCH_CHECK();
  return MMR_OK;
}

}  // extern "C"
