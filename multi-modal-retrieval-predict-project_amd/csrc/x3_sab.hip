// fp32-faithful (x3) fused Swin attention sub-block for stage 1 (C = 96, 3 heads of 32, 7 x 7 windows):
//   y = x + proj(W-MSA(LN1(x)))        (timm SwinTransformerBlock attention half + residual, reached
//                                        through the reference's fusion.py:198-199 Swin-T forward_features)
// including the cyclic shift (torch.roll), window partition / reverse, the relative-position bias and the
// shifted-window mask (mmr_swin_attn_bias's dense [types][heads][64][64] table), in f32 with every
// contraction on bf16x3 MFMA (a.b ~= a_hi.b_hi + a_hi.b_lo + a_lo.b_hi, f32 accumulate) as the unfused x3
// chain computes it: x3_rowlin (norm1 + qkv) -> x3_mha<1, 2> (split q k^T, f32 softmax on mmr::exp_acc,
// split P V) -> x3_rowlin (proj + residual).  That chain moves ~3.4 GB per stage-1 block at B = 256
// through HBM (the 288-wide f32 QKV written and re-read, the split attention output written and re-read,
// the residual) at 0.81 ms per block; this kernel reads x once (+ the residual re-read, L2-hot) and
// writes y once.
//
// Structure: the bf16 fused block's (swin_attn.hip) on split operands.  One workgroup of 4 waves per
// CU (one per SIMD: the split fragments need ~400 registers), persistent over windows; each wave owns
// whole windows (49 tokens padded to 64 = two 32-token MFMA tiles) and needs no barrier after the
// one-time weight load.  Every GEMM is v_mfma_f32_32x32x16_bf16 in the C^T orientation (A = weight
// rows from LDS, B = tokens), so each intermediate — LN'd x, K^T, Q^T, V, S^T, P, O^T — lands in the
// register fragment the next MFMA consumes (the shared k-permutation 16s + 8(j>>2) + 4h + (j&3) of
// swin_attn.hip), and is split into hi / lo fragments in registers.  The weights live in LDS as hi and lo
// images in MFMA fragment order (qkv 3C x C, proj C x C with its columns permuted to the O^T
// fragments' order: 144 KB) + f32 parameters; x rows are read straight into registers, f32 y rows
// written with the residual.
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

constexpr int SC = 96, SNH = 3, SWS = 7, STOK = 49, SKS = SC / 16;
constexpr int S_QKV_E = 3 * SC * SC;  // bf16 elements of one qkv image
constexpr int S_PROJ_E = SC * SC;
constexpr int S_PAR_F = 6 * SC;       // qkv_b | proj_b | ln_g | ln_b (f32)
constexpr int S_PAR_OFF = (2 * S_QKV_E + 2 * S_PROJ_E) * 2;  // byte offset of the parameters
constexpr int S_IMG_B = (S_PAR_OFF + S_PAR_F * 4 + 1023) / 1024 * 1024;
constexpr int S_NWV = 4;
static_assert(S_IMG_B <= 160 * 1024, "LDS budget");

// the C-fragment k-permutation and the fragment-order position of (row, col) in a C-column image (see
// swin_attn.hip): the 16-B slot of (32-row tile, k-step ks, lane) holds row 32 tile + (lane & 31),
// k = 16 ks + 8 (lane >> 5) + 0..7
__host__ __device__ __forceinline__ int s_kperm(int pos) {
  const int h = (pos >> 3) & 1, j = pos & 7;
  return (pos & ~15) + 8 * (j >> 2) + 4 * h + (j & 3);
}
__host__ __device__ __forceinline__ int s_frag_pos(int row, int col) {
  return (((row >> 5) * SKS + (col >> 4)) * 64 + ((col >> 3) & 1) * 32 + (row & 31)) * 8 + (col & 7);
}

// f32 weights -> [Wqkv_hi | Wqkv_lo | Wproj_hi | Wproj_lo | params] (hi = bf16(w), lo = bf16(w - hi));
// proj columns in O^T fragment order (kperm within each 16-block of a head's 32 dims)
__global__ __launch_bounds__(256) void x3_sab_pack(const float* __restrict__ qkv_w, const float* __restrict__ qkv_b,
                                                   const float* __restrict__ proj_w, const float* __restrict__ proj_b,
                                                   const float* __restrict__ ln_g, const float* __restrict__ ln_b,
                                                   unsigned char* __restrict__ img) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  uint16_t* e16 = (uint16_t*)img;
  float* pf = (float*)(img + S_PAR_OFF);
  if (i < S_QKV_E) {
    const int row = i / SC, col = i % SC;
    const float v = qkv_w[i];
    const uint16_t hi = mmr::f2bf(v);
    e16[s_frag_pos(row, col)] = hi;
    e16[S_QKV_E + s_frag_pos(row, col)] = mmr::f2bf(v - mmr::bf2f(hi));
  } else if (i < S_QKV_E + S_PROJ_E) {
    const int k = i - S_QKV_E, row = k / SC, pos = k % SC;
    const float v = proj_w[row * SC + s_kperm(pos)];
    const uint16_t hi = mmr::f2bf(v);
    e16[2 * S_QKV_E + s_frag_pos(row, pos)] = hi;
    e16[2 * S_QKV_E + S_PROJ_E + s_frag_pos(row, pos)] = mmr::f2bf(v - mmr::bf2f(hi));
  } else if (i < S_QKV_E + S_PROJ_E + S_PAR_F) {
    const int k = i - S_QKV_E - S_PROJ_E;
    pf[k] = k < 3 * SC ? qkv_b[k] : k < 4 * SC ? proj_b[k - 3 * SC] : k < 5 * SC ? ln_g[k - 4 * SC] : ln_b[k - 5 * SC];
  } else {
    const int z = S_PAR_OFF + S_PAR_F * 4 + 4 * (i - S_QKV_E - S_PROJ_E - S_PAR_F);  // zero tail (4 B each)
    if (z < S_IMG_B) *(uint32_t*)(img + z) = 0u;
  }
}

// 16 f32 accumulators -> (hi, lo) fragments of k-step s (values 8 s .. 8 s + 7)
__device__ __forceinline__ void split_frag(const f32x16& a, int s, bf16x8& hi, bf16x8& lo) {
  uint32_t h[4], l[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float v0 = a[8 * s + 2 * j], v1 = a[8 * s + 2 * j + 1];
    h[j] = mmr::pack2bf(v0, v1);
    l[j] = mmr::pack2bf(v0 - __uint_as_float(h[j] << 16), v1 - __uint_as_float(h[j] & 0xFFFF0000u));
  }
  hi = __builtin_bit_cast(bf16x8, make_uint4(h[0], h[1], h[2], h[3]));
  lo = __builtin_bit_cast(bf16x8, make_uint4(l[0], l[1], l[2], l[3]));
}

__device__ __forceinline__ f32x16 mfma3(const bf16x8 ah, const bf16x8 al, const bf16x8 bh, const bf16x8 bl, f32x16 c) {
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, c, 0, 0, 0);
}

__device__ __forceinline__ float half_sum(float v) {
  const auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(p[0]) + __uint_as_float(p[1]);
}
__device__ __forceinline__ float half_max(float v) {
  const auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(p[0]), __uint_as_float(p[1]));
}

__global__ __launch_bounds__(S_NWV * 64, 1) void x3_swin_attn_block(const float* __restrict__ x,
                                                                   const unsigned char* __restrict__ img,
                                                                   const float* __restrict__ bias,
                                                                   float* __restrict__ y, int nimg, int H, int shift,
                                                                   float eps) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const uint16_t* Wqh = (const uint16_t*)smem;  // qkv hi image
  const uint16_t* Wql = Wqh + S_QKV_E;
  const uint16_t* Wph = Wql + S_QKV_E;           // proj hi image
  const uint16_t* Wpl = Wph + S_PROJ_E;
  const float* P = (const float*)(smem + S_PAR_OFF);
  const float* Pqb = P;
  const float* Ppb = P + 3 * SC;
  const float* Pg = P + 4 * SC;
  const float* Pb = P + 5 * SC;

  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int r = lane & 31, h = lane >> 5;

  for (int p = wave; p < S_IMG_B / 1024; p += S_NWV)
    __builtin_amdgcn_global_load_lds((const void*)(img + p * 1024 + lane * 16), (lds_ptr_t)(smem + p * 1024), 16, 0, 0);

  const int nw1 = H / SWS, nwin = nw1 * nw1;
  const int total = nimg * nwin;  // host-checked < 2^31
  const int stride = gridDim.x * S_NWV;
  int win = blockIdx.x * S_NWV + wave;

  // token t (< 49) of window w -> element offset of its row in x / y (rolled by -shift)
  auto row_off = [&](int w, int t) -> int64_t {
    const int bi = w / nwin, wi = w - bi * nwin;
    const int wy = wi / nw1, wx = wi - wy * nw1;
    const int ty = t / SWS, tx = t - ty * SWS;
    int hh = wy * SWS + shift + ty, ww = wx * SWS + shift + tx;
    hh = hh >= H ? hh - H : hh;
    ww = ww >= H ? ww - H : ww;
    return ((int64_t)bi * H * H + (int64_t)hh * H + ww) * SC;
  };
  // lane (token 32 t2 + r, half h) loads channels 16 ks + 8 h .. + 7 (pad tokens re-read token 48)
  f32x4 xv[2][2 * SKS];
  auto load_xt = [&](int w, int t2) {
    const int t = 32 * t2 + r < STOK ? 32 * t2 + r : STOK - 1;
    const float* xr = x + row_off(w, t) + 8 * h;
#pragma unroll
    for (int ks = 0; ks < SKS; ++ks) {
      xv[t2][2 * ks] = *(const f32x4*)(xr + 16 * ks);
      xv[t2][2 * ks + 1] = *(const f32x4*)(xr + 16 * ks + 4);
    }
  };
  __builtin_amdgcn_s_waitcnt(vmcnt_n(0));
  asm volatile("" ::: "memory");
  __syncthreads();  // the weight image visible to every wave; no barrier after this point

  const float scale = 0.17677669529663687f;  // 32^-0.5 (timm scales q before q @ k^T)
  for (; win < total; win += stride) {
    int type = 0;
    if (shift > 0) {
      const int wi = win % nwin, wy = wi / nw1, wx = wi - wy * nw1;
      type = ((wy == nw1 - 1) ? 2 : 0) + ((wx == nw1 - 1) ? 1 : 0);
    }
    // this window's x rows (a prefetch of the next window's under the attention needs 96 more registers
    // than the 512 of a wave at one per SIMD: it spilled)
    load_xt(win, 0);
    load_xt(win, 1);
    // ---- LN1 (f32, two-pass, row over the lane pair) -> hi / lo B fragments of both token tiles
    bf16x8 hbh[2][SKS], hbl[2][SKS];
#pragma unroll
    for (int t2 = 0; t2 < 2; ++t2) {
      float s = 0.f;
#pragma unroll
      for (int q = 0; q < 2 * SKS; ++q) s += (xv[t2][q][0] + xv[t2][q][1]) + (xv[t2][q][2] + xv[t2][q][3]);
      s = half_sum(s);
      const float mean = s * (1.0f / SC);
      float ss = 0.f;
#pragma unroll
      for (int q = 0; q < 2 * SKS; ++q)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float d = xv[t2][q][j] - mean;
          ss += d * d;
        }
      ss = half_sum(ss);
      const float rstd = rsqrtf(ss * (1.0f / SC) + eps);
#pragma unroll
      for (int ks = 0; ks < SKS; ++ks) {
        const int k0 = 16 * ks + 8 * h;
        f32x16 nv;  // 8 normalised values in slots 0..7
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          const f32x4 g4 = *(const f32x4*)(Pg + k0 + 4 * p), c4 = *(const f32x4*)(Pb + k0 + 4 * p);
          const f32x4 v = xv[t2][2 * ks + p];
#pragma unroll
          for (int j = 0; j < 4; ++j) nv[4 * p + j] = (v[j] - mean) * rstd * g4[j] + c4[j];
        }
        split_frag(nv, 0, hbh[t2][ks], hbl[t2][ks]);
      }
    }

    // proj accumulators (lane: channels 32 u + 8 i + 4 h + rr of token 32 qt + r), starting at proj_b
    f32x16 acc[2][SC / 32];
#pragma unroll
    for (int u = 0; u < SC / 32; ++u)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const f32x4 bb = *(const f32x4*)(Ppb + 32 * u + 8 * i + 4 * h);
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) acc[0][u][4 * i + rr] = acc[1][u][4 * i + rr] = bb[rr];
      }

    auto wfrag = [&](const uint16_t* W, int tile, int ks) {  // A / B fragment: 32-row tile, k-step ks
      return *(const bf16x8*)(W + lane * 8 + (tile * SKS + ks) * 512);
    };

    auto head = [&](const int hd) {
      const float* bt = bias + (type * SNH + hd) * 4096;  // dense rel-pos + mask + pad keys, L2-resident
      // K^T (lane: token r, dh 8i + 4h + rr) and V (swapped: lane dh r, tokens 8i + 4h + rr) of both
      // token tiles, and Q^T (scaled) of both query tiles, as hi / lo fragments; biases start the
      // accumulators
      bf16x8 kfh[2][2], kfl[2][2], vfh[2][2], vfl[2][2], qfh[2][2], qfl[2][2];
      // the score accumulators start at the bias rows (L2): query tile 0's loaded before the QKV products,
      // tile 1's before tile 0's scores, so neither round trip is waited for at the scores
      f32x4 bq[2][2][4];
      auto load_bias = [&](int qt) {
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
          for (int i = 0; i < 4; ++i) bq[qt][kt][i] = *(const f32x4*)(bt + (32 * qt + r) * 64 + 32 * kt + 8 * i + 4 * h);
      };
      load_bias(0);
#pragma unroll
      for (int t2 = 0; t2 < 2; ++t2) {
        f32x16 ak, aq;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const f32x4 bkk = *(const f32x4*)(Pqb + SC + hd * 32 + 8 * i + 4 * h);
          const f32x4 bqq = *(const f32x4*)(Pqb + hd * 32 + 8 * i + 4 * h);
#pragma unroll
          for (int rr = 0; rr < 4; ++rr) ak[4 * i + rr] = bkk[rr], aq[4 * i + rr] = bqq[rr];
        }
        f32x16 av;
        {
          const float bv = Pqb[2 * SC + hd * 32 + r];
#pragma unroll
          for (int e = 0; e < 16; ++e) av[e] = bv;
        }
#pragma unroll
        for (int ks = 0; ks < SKS; ++ks) {
          ak = mfma3(wfrag(Wqh, SNH + hd, ks), wfrag(Wql, SNH + hd, ks), hbh[t2][ks], hbl[t2][ks], ak);
          av = mfma3(hbh[t2][ks], hbl[t2][ks], wfrag(Wqh, 2 * SNH + hd, ks), wfrag(Wql, 2 * SNH + hd, ks), av);
          aq = mfma3(wfrag(Wqh, hd, ks), wfrag(Wql, hd, ks), hbh[t2][ks], hbl[t2][ks], aq);
          // fence: unfenced, the scheduler hoists every k-step's 6 weight fragments (144 registers) and spills
          __builtin_amdgcn_sched_barrier(0);
        }
        aq *= scale;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          split_frag(ak, s, kfh[t2][s], kfl[t2][s]);
          split_frag(av, s, vfh[t2][s], vfl[t2][s]);
          split_frag(aq, s, qfh[t2][s], qfl[t2][s]);
        }
      }

#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        // S^T[key][query] = K (scale Q)^T + bias (the rel-pos / mask rows start the accumulator)
        if (qt == 0) load_bias(1);
        f32x16 s[2];
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) s[kt][4 * i + rr] = bq[qt][kt][i][rr];
#pragma unroll
          for (int k2 = 0; k2 < 2; ++k2) s[kt] = mfma3(kfh[kt][k2], kfl[kt][k2], qfh[qt][k2], qfl[qt][k2], s[kt]);
        }
        // softmax over the 49 keys of query r (f32, mmr::exp_acc; pad keys exactly 0)
        float mx = -FLT_MAX;
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
          for (int e = 0; e < 16; ++e) mx = fmaxf(mx, s[kt][e]);
        mx = half_max(mx);
        float sum = 0.f;
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const int key = 32 * kt + 8 * (e >> 2) + 4 * h + (e & 3);
            const float p = key < STOK ? mmr::exp_acc(s[kt][e] - mx) : 0.f;
            s[kt][e] = p;
            sum += p;
          }
        sum = half_sum(sum);
        // O^T[dh][query] = V^T P^T (P split in registers)
        f32x16 o = (f32x16){0};
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
          for (int k2 = 0; k2 < 2; ++k2) {
            bf16x8 ph, pl;
            split_frag(s[kt], k2, ph, pl);
            o = mfma3(vfh[kt][k2], vfl[kt][k2], ph, pl, o);
          }
        const float inv = 1.0f / sum;
        o *= inv;
        // proj: out^T[c][query] += Wproj[c][32 hd + dh] O^T[dh][query]
#pragma unroll
        for (int k2 = 0; k2 < 2; ++k2) {
          bf16x8 oh, ol;
          split_frag(o, k2, oh, ol);
#pragma unroll
          for (int u = 0; u < SC / 32; ++u) {
            acc[qt][u] = mfma3(wfrag(Wph, u, 2 * hd + k2), wfrag(Wpl, u, 2 * hd + k2), oh, ol, acc[qt][u]);
          }
        }
      }
    };
    // the heads unrolled: rolled, the loop-carried proj accumulators and the AGPR-resident MFMA results cost
    // ~1.7k accvgpr moves / reads per window against ~0.8k unrolled, 453-481 -> 404-433 us per block
    // (profiles/r06_x3_sab_variants_ab.txt; SLP vectorisation off on top of it: slower)
    head(0);
    head(1);
    head(2);

    // ---- y = x + proj (f32 rows; the residual re-read is L2-hot)
#pragma unroll
    for (int t2 = 0; t2 < 2; ++t2) {
      const int t = 32 * t2 + r;
      if (t < STOK) {
        const int64_t o = row_off(win, t);
#pragma unroll
        for (int u = 0; u < SC / 32; ++u)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int c = 32 * u + 8 * i + 4 * h;
            const f32x4 xr = *(const f32x4*)(x + o + c);
            f32x4 v;
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) v[rr] = acc[t2][u][4 * i + rr] + xr[rr];
            *(f32x4*)(y + o + c) = v;
          }
      }
    }
  }
}

int sab_cu_count() {
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

int64_t mmr_x3_swin_attn_block_pack_bytes(int32_t c) { return c == SC ? S_IMG_B : 0; }

mmr_status mmr_x3_swin_attn_block_pack(const float* qkv_w, const float* qkv_b, const float* proj_w, const float* proj_b,
                                       const float* ln_g, const float* ln_b, void* pack, int32_t c, void* stream) {
  mmr::clear_error();
  MMR_REQUIRE(qkv_w && qkv_b && proj_w && proj_b && ln_g && ln_b && pack, "mmr_x3_swin_attn_block_pack: NULL pointer");
  if (c != SC) {
    mmr::set_error("mmr_x3_swin_attn_block_pack: C=%d not built (96)", c);
    return MMR_ERR_UNSUPPORTED;
  }
  const int n = S_QKV_E + S_PROJ_E + S_PAR_F + (S_IMG_B - S_PAR_OFF - S_PAR_F * 4) / 4;
  x3_sab_pack<<<dim3((unsigned)mmr::ceil_div(n, 256)), 256, 0, mmr::as_stream(stream)>>>(
      qkv_w, qkv_b, proj_w, proj_b, ln_g, ln_b, (unsigned char*)pack);
  MMR_LAUNCH_CHECK();
  return MMR_OK;
}

mmr_status mmr_x3_swin_attn_block(const float* x, const void* pack, const float* bias, float* y, int32_t b, int32_t hw,
                                  int32_t c, int32_t ws, int32_t shift, float eps, void* stream) {
  mmr::clear_error();
  MMR_REQUIRE(x && pack && bias && y, "mmr_x3_swin_attn_block: NULL pointer");
  MMR_REQUIRE(x != y, "mmr_x3_swin_attn_block: in-place not supported");
  MMR_REQUIRE(b >= 0 && hw > 0 && hw % SWS == 0 && shift >= 0 && shift < SWS,
              "mmr_x3_swin_attn_block: b=%d hw=%d shift=%d", b, hw, shift);
  if (c != SC || ws != SWS) {
    mmr::set_error("mmr_x3_swin_attn_block: C=%d ws=%d not built (96, 7)", c, ws);
    return MMR_ERR_UNSUPPORTED;
  }
  if (b == 0) return MMR_OK;
  const int64_t wins = (int64_t)b * (hw / SWS) * (hw / SWS);
  MMR_REQUIRE(wins < (int64_t)1 << 31 && (int64_t)b * hw * hw * SC < ((int64_t)1 << 40),
              "mmr_x3_swin_attn_block: %lld windows", (long long)wins);
  const int64_t grid = std::min<int64_t>(sab_cu_count(), (wins + S_NWV - 1) / S_NWV);
  x3_swin_attn_block<<<dim3((unsigned)grid), S_NWV * 64, S_IMG_B, mmr::as_stream(stream)>>>(
      x, (const unsigned char*)pack, bias, y, b, hw, shift, eps);
  MMR_LAUNCH_CHECK();
  return MMR_OK;
}

}  // extern "C"
