// Tower kernels for the Swin-Tiny image tower and the ClinicalBERT text tower (gfx950), plus the
// pooling / projection heads.  GEMM-shaped work is in gemm.hip (mmr_linear_bf16); this file holds
// the attention cores (MFMA, LDS-staged), LayerNorms, gathers and the heads.
//
// Reference (semantics): timm SwinTransformer.forward_features (fusion.py:198-199), HF BertModel
// last_hidden_state (fusion.py:322-325), Backbones.forward pooling (fusion.py:259-265),
// MultiModalRetrievalModel heads (model.py:365-373, 462-479), MultiHeadMLP (model.py:61-75).
#include <float.h>
#include <math.h>
#include <stdlib.h>

#include "common.h"

namespace {

using mmr::bf2f;
using mmr::f2bf;

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void load8(const uint16_t* p, float* v) {
  bf16x8 x = *(const bf16x8*)p;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = bf2f((uint16_t)x[j]);
}
__device__ __forceinline__ void store8(uint16_t* p, const float* v) {
  *(uint4*)p = make_uint4(mmr::pack2bf(v[0], v[1]), mmr::pack2bf(v[2], v[3]), mmr::pack2bf(v[4], v[5]),
                          mmr::pack2bf(v[6], v[7]));
}

// ------------------------------------------------------------------ LayerNorm
// LPR lanes per row (64/LPR rows per wave) so narrow Swin rows (C = 96..384) keep every lane busy;
// the row stays in registers (<= NC chunks of 8 per lane; NC sized to the launch so the register
// file, and with it the occupancy, follows the row width): one read, one write, exact two-pass
// (centred) variance like torch.
// Q8: also emit the row as the next GEMM's MX-fp8 activation operand (e4m3 q [rows][c] + E8M0
// scales in the layout-0 image, see mmr_quantize_mxfp8) from the bf16-rounded outputs — bit-identical
// to quantising y afterwards; a 32-block is 4 adjacent lanes' chunks (two lane swaps).
template <int LPR, int NC, bool ADD, bool Q8 = false>
__global__ __launch_bounds__(256) void layernorm_bf16(const uint16_t* __restrict__ x,
                                                      const uint16_t* __restrict__ r,
                                                      const float* __restrict__ g,
                                                      const float* __restrict__ b,
                                                      uint16_t* __restrict__ y, int64_t rows,
                                                      int c, float eps,
                                                      const float* __restrict__ alpha = nullptr,
                                                      uint8_t* __restrict__ q8 = nullptr,
                                                      uint8_t* __restrict__ q8s = nullptr, int kp = 0) {
  static_assert(!Q8 || LPR % 4 == 0, "Q8: a 32-block must be 4 lanes of one row");
  constexpr int RPW = 64 / LPR;
  const int lane = threadIdx.x & 63;
  const int sub = lane % LPR;
  const int64_t row = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW + lane / LPR;
  const bool ok = row < rows;
  const uint16_t* xr = x + (ok ? row : 0) * c;
  const int nch = c / 8;
  const float av = alpha ? *alpha : 1.f;  // learned scale of x (PreFusionEnhancer alpha, fusion.py:34)
  // every load unconditional (chunk index clamped, value masked): a "load if in range" branch makes
  // hipcc wait for each chunk's load before issuing the next — NC (x2 with ADD) serial round trips
  bf16x8 xa[NC], ra[NC];
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    const int ch = sub + i * LPR;
    const int chc = ch < nch ? ch : nch - 1;
    xa[i] = *(const bf16x8*)(xr + chc * 8);
    if (ADD) ra[i] = *(const bf16x8*)(r + (ok ? row : 0) * c + chc * 8);
  }
  f32x4 ga[NC][2], ba[NC][2];
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    const int ch = sub + i * LPR;
    const int chc = ch < nch ? ch : nch - 1;
    ga[i][0] = *(const f32x4*)(g + chc * 8);
    ga[i][1] = *(const f32x4*)(g + chc * 8 + 4);
    ba[i][0] = *(const f32x4*)(b + chc * 8);
    ba[i][1] = *(const f32x4*)(b + chc * 8 + 4);
  }
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    mmr::pin(xa[i]);
    if (ADD) mmr::pin(ra[i]);
  }
  float v[NC][8];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    const int ch = sub + i * LPR;
    const bool in = ok && ch < nch;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[i][j] = bf2f((uint16_t)xa[i][j]);
    if (ADD) {  // post-LN residual: LN(x + r), the sum kept in f32
#pragma unroll
      for (int j = 0; j < 8; ++j) v[i][j] = fmaf(v[i][j], av, bf2f((uint16_t)ra[i][j]));
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[i][j] *= av;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      v[i][j] = in ? v[i][j] : 0.f;
      s += v[i][j];
    }
  }
#pragma unroll
  for (int o = LPR / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  const float mean = s / c;
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    const int ch = sub + i * LPR;
    if (ok && ch < nch) {
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += (v[i][j] - mean) * (v[i][j] - mean);
    }
  }
#pragma unroll
  for (int o = LPR / 2; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 64);
  const float rstd = rsqrtf(ss / c + eps);
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    const int ch = sub + i * LPR;
    mmr::pin(ga[i][0]);
    mmr::pin(ga[i][1]);
    mmr::pin(ba[i][0]);
    mmr::pin(ba[i][1]);
    const f32x4 g0 = ga[i][0], g1 = ga[i][1], b0 = ba[i][0], b1 = ba[i][1];
    const float gg[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
    const float bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
    for (int j = 0; j < 8; ++j) v[i][j] = (v[i][j] - mean) * rstd * gg[j] + bb[j];
    if (y && ok && ch < nch) store8(y + row * c + ch * 8, v[i]);
    if constexpr (Q8) {
      float vb[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) vb[j] = bf2f(f2bf(v[i][j]));  // the stored bf16 value
      mmr::q8_chunk8(vb, row, ch, kp, q8, q8s, ok && ch < nch);
    }
  }
  if constexpr (Q8) {
    // K padded to kp (c = 384 -> 512: the stage-3 Swin linears): zero bytes and zero scale bytes for
    // the padding blocks, as mmr_quantize_mxfp8 writes them (amax 0 -> E8M0 byte 0)
    if (ok)
      for (int pc = nch + sub; pc < kp / 8; pc += LPR) {
        *(uint2*)(q8 + row * kp + pc * 8) = make_uint2(0u, 0u);
        if ((pc & 3) == 0) q8s[mmr::q8_soff(row, pc * 8, kp)] = 0;
      }
  }
}

// ------------------------------------------------------------------ BERT embeddings + LN
__global__ __launch_bounds__(256) void bert_embed(const int64_t* __restrict__ ids,
                                                  const float* __restrict__ word,
                                                  const float* __restrict__ pos,
                                                  const float* __restrict__ type0,
                                                  const float* __restrict__ g,
                                                  const float* __restrict__ b,
                                                  uint16_t* __restrict__ y, int64_t ntok, int l,
                                                  int c, float eps, uint8_t* __restrict__ q8 = nullptr,
                                                  uint8_t* __restrict__ q8s = nullptr) {
  // q8 (c % 256 == 0, ntok % 256 == 0): also the first QKV GEMM's MX-fp8 operand, bit-identical to
  // mmr_quantize_mxfp8 of y (a 32-block = 8 adjacent lanes' float4s)
  const int64_t tok = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (tok >= ntok) return;
  const int p = (int)(tok % l);
  const float* wr = word + ids[tok] * (int64_t)c;
  const float* pr = pos + (int64_t)p * c;
  if (c % 256 == 0 && c <= 1024) {
    // the row in registers: lane owns floats 4(64j + lane) .. +3, every load issued at once
    // (three runtime-count passes re-reading the row waited on each load in turn: 67 -> 34 us at 256 x 128)
    float4 v[4];
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = 4 * (64 * j + lane);
      if (k < c) {
        const float4 a = *(const float4*)(wr + k), bq = *(const float4*)(pr + k), t0 = *(const float4*)(type0 + k);
        v[j] = make_float4(a.x + bq.x + t0.x, a.y + bq.y + t0.y, a.z + bq.z + t0.z, a.w + bq.w + t0.w);
        s += (v[j].x + v[j].y) + (v[j].z + v[j].w);
      }
    }
    const float mean = mmr::wave_sum(s) / c;
    float ss = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (4 * (64 * j + lane) < c) {
        const float d0 = v[j].x - mean, d1 = v[j].y - mean, d2 = v[j].z - mean, d3 = v[j].w - mean;
        ss += (d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3);
      }
    const float rstd = rsqrtf(mmr::wave_sum(ss) / c + eps);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = 4 * (64 * j + lane);
      if (k < c) {
        const float4 gg = *(const float4*)(g + k), bb = *(const float4*)(b + k);
        uint2 o;
        o.x = mmr::pack2bf((v[j].x - mean) * rstd * gg.x + bb.x, (v[j].y - mean) * rstd * gg.y + bb.y);
        o.y = mmr::pack2bf((v[j].z - mean) * rstd * gg.z + bb.z, (v[j].w - mean) * rstd * gg.w + bb.w);
        *(uint2*)(y + tok * c + k) = o;
        if (q8) {  // k < c is wave-uniform here (c % 256 == 0)
          const float vb[4] = {__uint_as_float(o.x << 16), __uint_as_float(o.x & 0xFFFF0000u),
                               __uint_as_float(o.y << 16), __uint_as_float(o.y & 0xFFFF0000u)};
          float amax = fmaxf(fmaxf(fabsf(vb[0]), fabsf(vb[1])), fmaxf(fabsf(vb[2]), fabsf(vb[3])));
          amax = fmaxf(amax, __shfl_xor(amax, 1, 64));
          amax = fmaxf(amax, __shfl_xor(amax, 2, 64));
          amax = fmaxf(amax, __shfl_xor(amax, 4, 64));
          const int ex = mmr::q8_exp(amax);
          *(uint32_t*)(q8 + tok * c + k) = mmr::q8_pack4(vb, mmr::q8_inv(ex));
          if ((lane & 7) == 0) q8s[mmr::q8_soff(tok, k, c)] = (uint8_t)(ex + 127);
        }
      }
    }
    return;
  }
  float s = 0.f;
  for (int k = lane; k < c; k += 64) s += wr[k] + pr[k] + type0[k];
  const float mean = mmr::wave_sum(s) / c;
  float ss = 0.f;
  for (int k = lane; k < c; k += 64) {
    float v = wr[k] + pr[k] + type0[k] - mean;
    ss += v * v;
  }
  const float rstd = rsqrtf(mmr::wave_sum(ss) / c + eps);
  for (int k = lane; k < c; k += 64)
    y[tok * c + k] = f2bf((wr[k] + pr[k] + type0[k] - mean) * rstd * g[k] + b[k]);
}

// ------------------------------------------------------------------ Swin (shifted) window attention
// One wave per (image, window, head); 4 units per block.  Window of ws*ws = 49 tokens padded to
// 64, head_dim 32.  The cyclic shift + window partition are folded into the token gather (and
// the reverse shift into the scatter of the output): rolled coordinate (hr, wr) reads token
// ((hr+shift)%H, (wr+shift)%W).  S^T = K . Q^T (2x2 tiles of 32x32x16, 2 k-steps), + a dense
// additive bias (relative-position bias + shift-region mask -100 + padded keys -inf) prepared
// once per block by swin_attn_bias for the <= 4 window types (interior / last column / last row
// / corner), softmax over keys in registers, O^T = V^T . P^T with V^T staged per wave in LDS.
constexpr int SW_DH = 32;
#ifndef SWA_LATE_BIAS
#define SWA_LATE_BIAS 1
#endif

__device__ __forceinline__ int region_of(int rc, int H, int ws, int shift) {
  return rc < H - ws ? 0 : (rc < H - shift ? 1 : 2);
}

// bias[type][head][i][j] (64x64, f32): type = 2*(last window row) + (last window column)
__global__ __launch_bounds__(256) void swin_attn_bias(const float* __restrict__ table,
                                                      float* __restrict__ bias, int heads, int ws,
                                                      int H, int shift, int ntypes) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (int64_t)ntypes * heads * 64 * 64) return;
  const int j = (int)(idx % 64), i = (int)((idx / 64) % 64);
  const int hh = (int)((idx / 4096) % heads), type = (int)(idx / (4096 * (int64_t)heads));
  const int N = ws * ws;
  float v = 0.f;
  if (j >= N) {
    v = -FLT_MAX;
  } else if (i < N) {
    const int yi = i / ws, xi = i % ws, yj = j / ws, xj = j % ws;
    v = table[((yi - yj + ws - 1) * (2 * ws - 1) + (xi - xj + ws - 1)) * heads + hh];
    if (shift > 0) {
      const int nw = H / ws;
      const int wy = (type >> 1) ? nw - 1 : 0, wx = (type & 1) ? nw - 1 : 0;
      const int ri = region_of(wy * ws + yi, H, ws, shift) * 3 + region_of(wx * ws + xi, H, ws, shift);
      const int rj = region_of(wy * ws + yj, H, ws, shift) * 3 + region_of(wx * ws + xj, H, ws, shift);
      if (ri != rj) v += -100.0f;
    }
  }
  bias[idx] = v;
}

// Q8: the output is written as the proj GEMM's MX-fp8 activation operand instead of bf16 rows (a
// head's 32 dims are one 32-block: the lane pair (r, r + 32) holds them, one lane swap for the
// amax), bit-identical to mmr_quantize_mxfp8(out, kp); the K padding C..kp is written by the last
// head's waves (zero bytes, zero scale bytes).
// 4 waves per SIMD: without the bound hipcc kept the MFMA results in AGPRs and allocated 140-146
// registers (3 waves); with it 110 VGPRs, no AGPRs, no spills
template <bool Q8 = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void swin_window_attention(const uint16_t* __restrict__ qkv,
                                                             const float* __restrict__ bias,
                                                             uint16_t* __restrict__ out,
                                                             int64_t units, int H, int C,
                                                             int heads, int ws, int shift, int hpw,
                                                             uint8_t* __restrict__ q8 = nullptr,
                                                             uint8_t* __restrict__ q8s = nullptr, int kp = 0) {
  // round 3: every global load of a wave (Q / K fragments, V rows, the bias rows of both query
  // tiles) is issued up front from clamped token indices (padded lanes read a real token and are
  // masked by the bias / the store guard): the previous form's "token valid ? load : 0" gathers
  // compiled into branches with a vmcnt(0) each (7 serial memory round trips per wave).  V goes to
  // LDS row-major with 16-B writes and comes back as the V^T fragment by ds_read_b64_tr_b16 (was 32
  // 2-byte transposing writes per lane); no workgroup barrier (each wave owns its LDS slice).
  constexpr int VROW = 48;  // halfs per V row: tr-read rows land on disjoint banks
  __shared__ __attribute__((aligned(16))) uint16_t vs_all[4][64 * VROW];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t unit = (int64_t)blockIdx.x * 4 + wave;
  if (unit >= units) return;
  const int nwin1 = H / ws;
  // unit = (image, window, head group of hpw): with hpw = 2 a wave reads whole 128-B lines of Q / K / V (two heads x 32
  // dims; the second head's loads hit the lines the first head's brought in) and writes whole
  // output lines — with one head per wave the two halves of every line were fetched by waves of
  // different workgroups, i.e. usually by different XCDs (2x the HBM / MALL reads)
  const int nwin = nwin1 * nwin1, npair = (heads + hpw - 1) / hpw;
  const int hp = (int)(unit % npair);
  const int64_t bw = unit / npair;
  const int win = (int)(bw % nwin);
  const int64_t bi = bw / nwin;
  const int wy = win / nwin1, wx = win % nwin1;
  const int N = ws * ws;
  const int type = shift > 0 ? ((wy == nwin1 - 1) ? 2 : 0) + ((wx == nwin1 - 1) ? 1 : 0) : 0;
  uint16_t* vs = vs_all[wave];
  // window-local token of this lane (rolled coordinates; lanes >= N take token 0 of the window)
  int tl;
  {
    const int i = lane < N ? lane : 0;
    const int hr = wy * ws + i / ws, wr = wx * ws + i % ws;
    const int h0 = (hr + shift) % H, w0 = (wr + shift) % H;
    tl = (int)(bi * H * H + h0 * H + w0);
  }
  if constexpr (Q8) {
    // K padding C .. kp of this window's tokens: zero bytes, zero scale bytes, written up front by the
    // waves of the last head group (no registers held across the attention)
    if (kp > C && hpw * hp + hpw >= heads) {
      const int r = lane & 31, hf = lane >> 5;
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        const int qi = qt * 32 + r;
        const int tqi = __shfl(tl, qi, 64);
        if (qi < N) {
          uint8_t* qrow = q8 + (int64_t)tqi * kp;
          for (int off = C + 16 * hf; off < kp; off += 32) *(uint4*)(qrow + off) = make_uint4(0u, 0u, 0u, 0u);
          for (int bk = C / 32 + hf; bk < kp / 32; bk += 2) q8s[mmr::q8_soff(tqi, bk * 32, kp)] = 0;
        }
      }
    }
  }
#pragma unroll 1
  for (int h2 = 0; h2 < hpw; ++h2) {
    const int hh = hpw * hp + h2;
    if (hh >= heads) break;
    const float* bt = bias + ((int64_t)type * heads + hh) * 4096;
    asm volatile("" ::: "memory");  // the previous head's V reads stay before this head's V writes
    const int r = lane & 31, hf = lane >> 5;
    const uint16_t* hb = qkv + hh * SW_DH;
    const uint32_t rs = 3u * (uint32_t)C;  // element offsets fit 32 bits (launcher)
    bf16x8 qf[2][2], kf[2][2], vr[4];
    // bias rows of this lane's two queries, loaded straight into the S accumulators as bias / scale
    // (S = (q k^T + bias / scale) * scale: no separate 64-VGPR bias array live across the head)
    f32x16 sacc[2][2];  // [qt][kt], element 4 g4 + e = key kt 32 + 8 g4 + 4 hf + e
#pragma unroll
    for (int it = 0; it < 4; ++it)  // V rows: lane (key 16 it + lane / 4, 16-B chunk lane % 4)
      vr[it] = *(const bf16x8*)(hb + (uint32_t)__shfl(tl, 16 * it + (lane >> 2), 64) * rs + 2 * C + (lane & 3) * 8);
#pragma unroll
    for (int t2 = 0; t2 < 2; ++t2) {
      const uint16_t* row = hb + (uint32_t)__shfl(tl, t2 * 32 + r, 64) * rs;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        qf[t2][ks] = *(const bf16x8*)(row + ks * 16 + 8 * hf);
        kf[t2][ks] = *(const bf16x8*)(row + C + ks * 16 + 8 * hf);
      }
    }
    auto load_bias = [&](int qt) {
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const float4 bv = *(const float4*)(bt + (qt * 32 + r) * 64 + kt * 32 + 8 * g4 + 4 * hf);
          sacc[qt][kt][4 * g4] = bv.x;
          sacc[qt][kt][4 * g4 + 1] = bv.y;
          sacc[qt][kt][4 * g4 + 2] = bv.z;
          sacc[qt][kt][4 * g4 + 3] = bv.w;
        }
    };
    load_bias(0);
    if (!SWA_LATE_BIAS) load_bias(1);
    __builtin_amdgcn_sched_barrier(0);  // every load above in flight before the first use
#pragma unroll
    for (int it = 0; it < 4; ++it) *(bf16x8*)(vs + (16 * it + (lane >> 2)) * VROW + (lane & 3) * 8) = vr[it];
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's V rows are in LDS
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");

    constexpr float L2E = 1.4426950408889634f;
    const float scale = 0.17677669529663687f;  // 32^-0.5
    const float rscale = 5.656854249492381f;     // 32^0.5
    const int grp = lane >> 4, tq = (lane >> 2) & 3, tp = lane & 3;
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      const int qi = qt * 32 + r;  // this lane's query (local index)
      if (SWA_LATE_BIAS && qt == 1) load_bias(1);  // second query tile's bias after the first tile's S is free
      f32x16* s = sacc[qt];  // in place: the bias rows become this query tile's S
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        s[kt] *= rscale;  // bias / scale (-FLT_MAX padding -> -inf: exp2 -> 0)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
          s[kt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf[kt][ks], qf[qt][ks], s[kt], 0, 0, 0);
      }
      // row max / sum as 4 independent chains (SQ_WAIT_INST_ANY, dependency stalls, was 61 % of the
      // kernel's wave cycles with one 32-long chain each; stage 3 52.6 -> 50.1 us)
      float m4[4] = {-FLT_MAX, -FLT_MAX, -FLT_MAX, -FLT_MAX};
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int rg = 0; rg < 16; ++rg) {
          const float v = s[kt][rg] * scale;
          s[kt][rg] = v;
          m4[rg & 3] = fmaxf(m4[rg & 3], v);
        }
      float mloc = fmaxf(fmaxf(m4[0], m4[1]), fmaxf(m4[2], m4[3]));
      mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
      const float ml = mloc * L2E;
      float p4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int rg = 0; rg < 16; ++rg) {
          const float p = __builtin_amdgcn_exp2f(fmaf(s[kt][rg], L2E, -ml));
          s[kt][rg] = p;
          p4[rg & 3] += p;
        }
      float psum = (p4[0] + p4[1]) + (p4[2] + p4[3]);
      psum += __shfl_xor(psum, 32, 64);
      // O^T = V^T . P^T; the V^T fragment (lane: dim r, keys kbase..+3 and kbase+8..+11 in P^T's
      // register order) by two ds_read_b64_tr_b16 from the key-major V image
      f32x16 o = {0};
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int sidx = 0; sidx < 2; ++sidx) {
          const bf16x8 pf = __builtin_bit_cast(
              bf16x8, make_uint4(mmr::pack2bf(s[kt][8 * sidx], s[kt][8 * sidx + 1]), mmr::pack2bf(s[kt][8 * sidx + 2], s[kt][8 * sidx + 3]),
                                 mmr::pack2bf(s[kt][8 * sidx + 4], s[kt][8 * sidx + 5]), mmr::pack2bf(s[kt][8 * sidx + 6], s[kt][8 * sidx + 7])));
          const int r0 = kt * 32 + 16 * sidx + 4 * (grp >> 1);
          const uint16_t* va = vs + (r0 + tq) * VROW + (grp & 1) * 16 + 4 * tp;
          const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) bf16x4*)va);
          const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) bf16x4*)(va + 8 * VROW));
          const bf16x8 vf = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          o = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf, o, 0, 0, 0);
        }
      const int tqi = __shfl(tl, qi, 64);
      if constexpr (Q8) {
        const float inv = 1.0f / psum;
        // amax of the bf16 values the plain kernel stores = the bf16 rounding of max |o * inv| (RNE is
        // monotonic), and the values are re-rounded at the packing: no 16-register copy stays live
        float amax = 0.f;
#pragma unroll
        for (int e = 0; e < 16; ++e) amax = fmaxf(amax, fabsf(o[e] * inv));
        amax = bf2f(f2bf(amax));
        amax = fmaxf(amax, __shfl_xor(amax, 32, 64));
        const int ex = mmr::q8_exp(amax);
        const float qinv = mmr::q8_inv(ex);
        if (qi < N) {
          uint8_t* qrow = q8 + (int64_t)tqi * kp;
#pragma unroll
          for (int g4 = 0; g4 < 4; ++g4) {
            const float vb[4] = {bf2f(f2bf(o[4 * g4] * inv)), bf2f(f2bf(o[4 * g4 + 1] * inv)),
                                 bf2f(f2bf(o[4 * g4 + 2] * inv)), bf2f(f2bf(o[4 * g4 + 3] * inv))};
            *(uint32_t*)(qrow + hh * SW_DH + 8 * g4 + 4 * hf) = mmr::q8_pack4(vb, qinv);
          }
          if (hf == 0) q8s[mmr::q8_soff(tqi, hh * SW_DH, kp)] = (uint8_t)(ex + 127);
        }
      } else if (qi < N) {
        const float inv = 1.0f / psum;
        uint16_t* orow = out + (int64_t)tqi * C + hh * SW_DH;
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4)
          *(uint2*)(orow + 8 * g4 + 4 * hf) = make_uint2(mmr::pack2bf(o[4 * g4] * inv, o[4 * g4 + 1] * inv),
                                                         mmr::pack2bf(o[4 * g4 + 2] * inv, o[4 * g4 + 3] * inv));
      }
    }
  }
}

// ------------------------------------------------------------------ patch embed im2col (K padded to 64)
__global__ __launch_bounds__(256) void patch_im2col(const float* __restrict__ img,
                                                    uint16_t* __restrict__ cols, int64_t ntok,
                                                    int cin, int hw, int patch) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;  // (token, 8-chunk)
  const int kp = 64;
  if (idx >= ntok * (kp / 8)) return;
  const int64_t t = idx / 8;
  const int ch = (int)(idx % 8);
  const int g = hw / patch;
  const int64_t bi = t / (g * g);
  const int py = (int)((t / g) % g), px = (int)(t % g);
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = ch * 8 + j;  // k = c*16 + ky*4 + kx
    float val = 0.f;
    if (k < cin * patch * patch) {
      const int c = k / (patch * patch), ky = (k / patch) % patch, kx = k % patch;
      val = img[((bi * cin + c) * hw + (py * patch + ky)) * (int64_t)hw + px * patch + kx];
    }
    v[j] = val;
  }
  store8(cols + t * kp + ch * 8, v);
}

// Swin's patch 4 / 3 channels, fewer than 2^31 image elements: thread (token, 8-chunk) ch < 6 reads
// channel ch/2, kernel rows 2(ch%2), 2(ch%2)+1 as two float4 (k = c*16 + ky*4 + kx), ch 6-7 are the
// zero K padding; 32-bit index math (generic form with 64-bit divisions: 100 us, this one 40 us at 256 images).
__global__ __launch_bounds__(256) void patch_im2col_p4c3(const float* __restrict__ img,
                                                         uint16_t* __restrict__ cols, uint32_t ntok,
                                                         uint32_t hw) {
  const uint32_t idx = blockIdx.x * 256u + threadIdx.x;
  if (idx >= ntok * 8u) return;
  const uint32_t t = idx >> 3, ch = idx & 7u;
  const uint32_t g = hw >> 2, gg = g * g;
  const uint32_t bi = t / gg, r = t - bi * gg, py = r / g, px = r - py * g;
  float v[8];
  if (ch < 6) {
    const uint32_t c = ch >> 1, ky = (ch & 1u) * 2u;
    const float* p0 = img + ((bi * 3u + c) * hw + py * 4u + ky) * hw + px * 4u;
    const float4 a = *(const float4*)p0, b = *(const float4*)(p0 + hw);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = 0.f;
  }
  store8(cols + (size_t)t * 64 + ch * 8, v);
}

// ------------------------------------------------------------------ PatchMerging gather + LN(4c)
// Narrow merges (4c = 24 G: stage 1 -> 2 with G = 16, 2 -> 3 with G = 32): a group of G lanes per
// merged row, 3 16-B chunks per lane (chunk it of lane l: merged channels 8 (l + G it) .. +7, inside
// one source token since c % 8 == 0), 64 / G rows per wave.  The one-row-per-wave form below left
// 3/4 of the lanes on clamped duplicate loads at 4c = 384 (172 us for the 308 MB of stage 1 -> 2).
// q8 (both forms, a runtime pointer so y is the same code either way): also / instead (y NULL) emit the merged row as the reduction GEMM's MX-fp8
// operand (4c % 256 == 0, no K padding), bit-identical to mmr_quantize_mxfp8 of the bf16 row: a
// 32-block is 4 adjacent lanes' chunks in both lane maps.
template <int G>
__global__ __launch_bounds__(256) void patch_merge_ln_g(const uint16_t* __restrict__ x,
                                                        const float* __restrict__ g,
                                                        const float* __restrict__ b,
                                                        uint16_t* __restrict__ y, int64_t nout,
                                                        int hw, int c, float eps,
                                                        uint8_t* __restrict__ q8 = nullptr,
                                                        uint8_t* __restrict__ q8s = nullptr) {
  constexpr int C4 = 24 * G, RPW = 64 / G;
  const int lane = threadIdx.x & 63, lg = lane % G;
  const int64_t o0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW + lane / G;
  const int64_t o = o0 < nout ? o0 : nout - 1;  // clamped row: loads unconditional, store guarded
  const int h2 = hw / 2;
  const int64_t bi = o / (h2 * h2);
  const int i = (int)((o / h2) % h2), j = (int)(o % h2);
  bf16x8 xa[3];
  f32x4 ga[3][2], ba[3][2];
#pragma unroll
  for (int it = 0; it < 3; ++it) {
    const int k = 8 * (lg + G * it), p = k / c, off = k % c;
    const int yy = 2 * i + (p & 1), xx = 2 * j + (p >> 1);
    xa[it] = *(const bf16x8*)(x + ((bi * hw + yy) * hw + xx) * (int64_t)c + off);
    ga[it][0] = *(const f32x4*)(g + k);
    ga[it][1] = *(const f32x4*)(g + k + 4);
    ba[it][0] = *(const f32x4*)(b + k);
    ba[it][1] = *(const f32x4*)(b + k + 4);
  }
  float v[3][8];
  float s = 0.f;
#pragma unroll
  for (int it = 0; it < 3; ++it)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      v[it][e] = bf2f((uint16_t)xa[it][e]);
      s += v[it][e];
    }
#pragma unroll
  for (int m = 1; m < G; m <<= 1) s += __shfl_xor(s, m, 64);
  const float mean = s * (1.0f / C4);
  float ss = 0.f;
#pragma unroll
  for (int it = 0; it < 3; ++it)
#pragma unroll
    for (int e = 0; e < 8; ++e) ss += (v[it][e] - mean) * (v[it][e] - mean);
#pragma unroll
  for (int m = 1; m < G; m <<= 1) ss += __shfl_xor(ss, m, 64);
  const float rstd = rsqrtf(ss * (1.0f / C4) + eps);
#pragma unroll
  for (int it = 0; it < 3; ++it) {
    const f32x4 g0 = ga[it][0], g1 = ga[it][1], b0 = ba[it][0], b1 = ba[it][1];
    const float gg[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
    const float bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
    for (int e = 0; e < 8; ++e) v[it][e] = fmaf((v[it][e] - mean) * rstd, gg[e], bb[e]);  // explicit: same in both forms
    if (y && o0 < nout) store8(y + o0 * C4 + 8 * (lg + G * it), v[it]);
    if (q8) {  // wave-uniform
      float vb[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) vb[e] = bf2f(f2bf(v[it][e]));
      mmr::q8_chunk8(vb, o0, lg + G * it, C4, q8, q8s, o0 < nout);
    }
  }
}

__global__ __launch_bounds__(256) void patch_merge_ln(const uint16_t* __restrict__ x,
                                                      const float* __restrict__ g,
                                                      const float* __restrict__ b,
                                                      uint16_t* __restrict__ y, int64_t nout,
                                                      int hw, int c, float eps,
                                                      uint8_t* __restrict__ q8 = nullptr,
                                                      uint8_t* __restrict__ q8s = nullptr) {
  const int64_t o = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (o >= nout) return;
  const int h2 = hw / 2;
  const int64_t bi = o / (h2 * h2);
  const int i = (int)((o / h2) % h2), j = (int)(o % h2);
  const int c4 = 4 * c;
  // part p: (dy, dx) = (p&1, p>>1)  -> [x(2i,2j), x(2i+1,2j), x(2i,2j+1), x(2i+1,2j+1)]
  auto src = [&](int k) -> const uint16_t* {
    const int p = k / c, off = k % c;
    const int yy = 2 * i + (p & 1), xx = 2 * j + (p >> 1);
    return x + ((bi * hw + yy) * hw + xx) * (int64_t)c + off;
  };
  if (c4 <= 2048) {
    // the 4c-wide merged row in registers (<= 4 chunks of 8 per lane), every load issued at once:
    // one memory round trip instead of three passes that each wait on their loads
    // (loads unconditional — chunk clamped, value masked: a "load if k < 4c" branch makes hipcc
    // wait for each load before issuing the next)
    bf16x8 xa[4];
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int k = lane * 8 + 512 * it;
      xa[it] = *(const bf16x8*)src(k < c4 ? k : c4 - 8);
    }
    f32x4 ga[4][2], ba[4][2];
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int k = lane * 8 + 512 * it, kc = k < c4 ? k : c4 - 8;
      ga[it][0] = *(const f32x4*)(g + kc);
      ga[it][1] = *(const f32x4*)(g + kc + 4);
      ba[it][0] = *(const f32x4*)(b + kc);
      ba[it][1] = *(const f32x4*)(b + kc + 4);
    }
#pragma unroll
    for (int it = 0; it < 4; ++it) mmr::pin(xa[it]);
    float v[4][8];
    float s = 0.f;
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int k = lane * 8 + 512 * it;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        v[it][e] = bf2f((uint16_t)xa[it][e]);
        v[it][e] = k < c4 ? v[it][e] : 0.f;
        s += v[it][e];
      }
    }
    const float mean = mmr::wave_sum(s) / c4;
    float ss = 0.f;
#pragma unroll
    for (int it = 0; it < 4; ++it)
      if (lane * 8 + 512 * it < c4) {
#pragma unroll
        for (int e = 0; e < 8; ++e) ss += (v[it][e] - mean) * (v[it][e] - mean);
      }
    const float rstd = rsqrtf(mmr::wave_sum(ss) / c4 + eps);
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int k = lane * 8 + 512 * it;
      mmr::pin(ga[it][0]);
      mmr::pin(ga[it][1]);
      mmr::pin(ba[it][0]);
      mmr::pin(ba[it][1]);
      const f32x4 g0 = ga[it][0], g1 = ga[it][1], b0 = ba[it][0], b1 = ba[it][1];
      const float gg[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
      const float bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
      for (int e = 0; e < 8; ++e) v[it][e] = fmaf((v[it][e] - mean) * rstd, gg[e], bb[e]);
      if (y && k < c4) store8(y + o * c4 + k, v[it]);
      if (q8) {  // wave-uniform
        float vb[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) vb[e] = bf2f(f2bf(v[it][e]));
        mmr::q8_chunk8(vb, o, lane + 64 * it, c4, q8, q8s, k < c4);
      }
    }
    return;
  }
  if (q8) return;  // the launcher keeps q8 to 4c <= 2048
  float s = 0.f;
  for (int k = lane * 8; k < c4; k += 512) {
    float v[8];
    load8(src(k), v);
#pragma unroll
    for (int e = 0; e < 8; ++e) s += v[e];
  }
  const float mean = mmr::wave_sum(s) / c4;
  float ss = 0.f;
  for (int k = lane * 8; k < c4; k += 512) {
    float v[8];
    load8(src(k), v);
#pragma unroll
    for (int e = 0; e < 8; ++e) ss += (v[e] - mean) * (v[e] - mean);
  }
  const float rstd = rsqrtf(mmr::wave_sum(ss) / c4 + eps);
  for (int k = lane * 8; k < c4; k += 512) {
    float v[8];
    load8(src(k), v);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = (v[e] - mean) * rstd * g[k + e] + b[k + e];
    store8(y + o * c4 + k, v);
  }
}

// ------------------------------------------------------------------ Swin head: LN, LN(LN), means
constexpr int SH_MAXPL = 16;  // c <= 1024, c % 64 == 0
// 16 waves per image, tokens strided over the waves (4 waves: one token at a time per wave, 49 /
// 4 dependent load-reduce rounds: 103 -> 37 us at 256 x 49 x 768); per-wave partial sums reduced through
// one 64-KB LDS array in two rounds (acc1, then acc2).
constexpr int SH_WAVES = 16;
__global__ __launch_bounds__(64 * SH_WAVES) void swin_head(const uint16_t* __restrict__ x,
                                                 const float* __restrict__ g,
                                                 const float* __restrict__ b,
                                                 float* __restrict__ patches,
                                                 float* __restrict__ glob,
                                                 float* __restrict__ pool, int t, int c,
                                                 float eps) {
  __shared__ float part[SH_WAVES][1024];
  __shared__ float gs[1024], bs[1024];  // LN parameters (in registers they pushed the 128-VGPR budget into spills)
  const int bi = blockIdx.x;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int per = c / 64;
  float acc1[SH_MAXPL], acc2[SH_MAXPL];
  // every load unconditional (index clamped, value masked; a "load if e < per" branch makes hipcc wait
  // for each load before the next)
  for (int k = threadIdx.x; k < c; k += 64 * SH_WAVES) {
    gs[k] = g[k];
    bs[k] = b[k];
  }
#pragma unroll
  for (int e = 0; e < SH_MAXPL; ++e) acc1[e] = acc2[e] = 0.f;
  __syncthreads();
  for (int tk = wave; tk < t; tk += SH_WAVES) {
    const uint16_t* xr = x + ((int64_t)bi * t + tk) * c;
    float v[SH_MAXPL];
    float s = 0.f;
#pragma unroll
    for (int e = 0; e < SH_MAXPL; ++e) {
      const float xv = bf2f(xr[lane + 64 * (e < per ? e : per - 1)]);
      v[e] = e < per ? xv : 0.f;
      s += v[e];
    }
    float mean = mmr::wave_sum(s) / c, ss = 0.f;
#pragma unroll
    for (int e = 0; e < SH_MAXPL; ++e)
      if (e < per) ss += (v[e] - mean) * (v[e] - mean);
    float rstd = rsqrtf(mmr::wave_sum(ss) / c + eps);
    s = 0.f;
#pragma unroll
    for (int e = 0; e < SH_MAXPL; ++e)
      if (e < per) {
        v[e] = (v[e] - mean) * rstd * gs[lane + 64 * e] + bs[lane + 64 * e];  // once-normed token (forward_features output)
        acc1[e] += v[e];
        s += v[e];
      }
    mean = mmr::wave_sum(s) / c;
    ss = 0.f;
#pragma unroll
    for (int e = 0; e < SH_MAXPL; ++e)
      if (e < per) ss += (v[e] - mean) * (v[e] - mean);
    rstd = rsqrtf(mmr::wave_sum(ss) / c + eps);
#pragma unroll
    for (int e = 0; e < SH_MAXPL; ++e)
      if (e < per) {
        const int k = lane + 64 * e;
        const float p2 = (v[e] - mean) * rstd * gs[k] + bs[k];  // swin_norm applied again
        acc2[e] += p2;
        if (patches) patches[((int64_t)bi * t + tk) * c + k] = p2;
      }
  }
#pragma unroll
  for (int e = 0; e < SH_MAXPL; ++e)
    if (e < per) part[wave][lane + 64 * e] = acc1[e];
  __syncthreads();
  const int k = threadIdx.x;  // blockDim = 1024 >= c
  float s1 = 0.f, s2 = 0.f;
  if (k < c)
    for (int w = 0; w < SH_WAVES; ++w) s1 += part[w][k];  // fixed order: deterministic
  __syncthreads();
#pragma unroll
  for (int e = 0; e < SH_MAXPL; ++e)
    if (e < per) part[wave][lane + 64 * e] = acc2[e];
  __syncthreads();
  if (k < c) {
    for (int w = 0; w < SH_WAVES; ++w) s2 += part[w][k];
    const float gm = s1 / t;
    if (glob) glob[(int64_t)bi * c + k] = gm;
    if (pool) pool[(int64_t)bi * c + k] = (gm + s2) / (t + 1);
  }
}

// ------------------------------------------------------------------ unmasked token mean
__global__ __launch_bounds__(256) void mean_tokens(const uint16_t* __restrict__ x,
                                                   float* __restrict__ y, int l, int c) {
  const int bi = blockIdx.y;
  const int k = blockIdx.x * 256 + threadIdx.x;
  if (k >= c) return;
  const uint16_t* xr = x + (int64_t)bi * l * c + k;
  float s = 0.f;
  for (int t = 0; t < l; ++t) s += bf2f(xr[(int64_t)t * c]);
  y[(int64_t)bi * c + k] = s / l;
}

// ------------------------------------------------------------------ small f32 linear (heads)
// Y[b][o] = act(sum_i X[b][i] W[o][i] + bias[o]) in exact f32 (v_mfma_f32_32x32x2_f32) for the
// per-query vectors (a few hundred rows): pure latency, so one 32x32 output tile per 512-thread
// block with K split over the 8 waves, each wave issuing the loads of LF_CH 16-wide k-steps before
// their MFMAs (one memory round trip per chunk instead of one per step), partial tiles summed in
// LDS in a fixed order.  Operands straight to VGPRs as float4 with the k-permutation of knn_scores
// (lane half h owns k = kb+8h..kb+8h+7).  cin % 16 == 0, cout % 32 == 0.  Rows are strided (ldx,
// ldy; ldx % 4 == 0); optional residual R (ldr, may alias Y) added after the activation.
// Measured and dropped: 16x16 output tiles on v_mfma_f32_16x16x4_f32 (4x the workgroups, filling all
// 256 CUs at 256 x 768) — 25.7 vs 19.2 us average: twice the L2 operand traffic, same TA pattern.
constexpr int LF_WAVES = 8;
constexpr int LF_CH = 6;

__global__ __launch_bounds__(512) void linear_f32(const float* __restrict__ X,
                                                  const float* __restrict__ W,
                                                  const float* __restrict__ bias,
                                                  float* Y, int nb, int cin, int cout,
                                                  int act, int64_t ldx, int64_t ldy,
                                                  const float* R, int64_t ldr, int64_t bsx = 0,
                                                  int64_t bsw = 0, int64_t bsb = 0, int64_t bsr = 0,
                                                  int64_t bsy = 0) {
  __shared__ float part[LF_WAVES][1024];
  // batched form (blockIdx.y = problem index): independent problems at fixed element strides
  X += blockIdx.y * bsx;
  W += blockIdx.y * bsw;
  if (bias) bias += blockIdx.y * bsb;
  if (R) R += blockIdx.y * bsr;
  Y += blockIdx.y * bsy;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int tiles_o = cout / 32;
  const int tb = blockIdx.x / tiles_o, to = blockIdx.x % tiles_o;
  const int r = lane & 31, h = lane >> 5;
  const int b = tb * 32 + r;
  const bool bok = b < nb;
  const float* xa = X + (int64_t)(bok ? b : 0) * ldx + 8 * h;
  const float* wb = W + (int64_t)(to * 32 + r) * cin + 8 * h;
  const int nsteps = cin / 16;
  const int per = (nsteps + LF_WAVES - 1) / LF_WAVES;
  const int s0 = wave * per, s1 = min(nsteps, s0 + per);
  f32x16 acc = {0};
  for (int sc = s0; sc < s1; sc += LF_CH) {
    float4 a[LF_CH][2], w[LF_CH][2];
#pragma unroll
    for (int c = 0; c < LF_CH; ++c) {
      const int kb = (sc + c) * 16;
      if (sc + c < s1) {
        a[c][0] = *(const float4*)(xa + kb);
        a[c][1] = *(const float4*)(xa + kb + 4);
        w[c][0] = *(const float4*)(wb + kb);
        w[c][1] = *(const float4*)(wb + kb + 4);
      } else {
        a[c][0] = a[c][1] = w[c][0] = w[c][1] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
      if (!bok) a[c][0] = a[c][1] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int c = 0; c < LF_CH; ++c) {
      const float av[8] = {a[c][0].x, a[c][0].y, a[c][0].z, a[c][0].w, a[c][1].x, a[c][1].y, a[c][1].z, a[c][1].w};
      const float bv[8] = {w[c][0].x, w[c][0].y, w[c][0].z, w[c][0].w, w[c][1].x, w[c][1].y, w[c][1].z, w[c][1].w};
#pragma unroll
      for (int s8 = 0; s8 < 8; ++s8) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[s8], bv[s8], acc, 0, 0, 0);
    }
  }
#pragma unroll
  for (int rg = 0; rg < 16; ++rg) part[wave][lane * 16 + rg] = acc[rg];
  __syncthreads();
  for (int e = threadIdx.x; e < 1024; e += blockDim.x) {
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < LF_WAVES; ++w) v += part[w][e];
    const int ln = e >> 4, rg = e & 15;
    const int bb = tb * 32 + (rg & 3) + 8 * (rg >> 2) + 4 * (ln >> 5);
    const int o = to * 32 + (ln & 31);
    if (bb >= nb) continue;
    v += bias ? bias[o] : 0.f;
    if (act == 1) v = mmr::gelu_erf(v);
    if (R) v += R[(int64_t)bb * ldr + o];
    Y[(int64_t)bb * ldy + o] = v;
  }
}

void launch_linear_f32(const float* x, const float* w, const float* b, float* y, int nb, int cin, int cout,
                       int act, int64_t ldx, int64_t ldy, const float* r, int64_t ldr, hipStream_t st,
                       int nbatch = 1, int64_t bsx = 0, int64_t bsw = 0, int64_t bsb = 0, int64_t bsr = 0,
                       int64_t bsy = 0) {
  const int64_t tiles = mmr::ceil_div(nb, 32) * (cout / 32);
  linear_f32<<<dim3((unsigned)tiles, (unsigned)nbatch), dim3(64 * LF_WAVES), 0, st>>>(
      x, w, b, y, nb, cin, cout, act, ldx, ldy, r, ldr, bsx, bsw, bsb, bsr, bsy);
}

__global__ __launch_bounds__(256) void l2_normalize_rows(float* __restrict__ y, int nb, int d) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= nb) return;
  float* p = y + (int64_t)row * d;
  float s = 0.f;
  for (int k = lane; k < d; k += 64) s += p[k] * p[k];
  s = mmr::wave_sum(s);
  const float inv = s > 0.f ? rsqrtf(s) : 0.f;
  for (int k = lane; k < d; k += 64) p[k] *= inv;
}

}  // namespace

// ================================================================== C ABI
extern "C" {

static mmr_status layernorm_launch(const uint16_t* x, const uint16_t* r, const float* gamma,
                                   const float* beta, uint16_t* y, int64_t rows, int32_t c,
                                   float eps, void* stream, const char* who,
                                   const float* alpha = nullptr, uint8_t* q8 = nullptr,
                                   uint8_t* q8s = nullptr, int32_t kp = 0) {
  if (!kp) kp = c;
  MMR_REQUIRE(x && gamma && beta && (y || q8), "%s: NULL pointer", who);
  MMR_REQUIRE(!q8 || (q8s && rows % 256 == 0 && c % 32 == 0 && kp % 256 == 0 && kp >= c),
              "%s: the MX-fp8 output needs rows %% 256 == 0, c %% 32 == 0 and its padded K kp a multiple of 256 "
              ">= c (rows=%lld c=%d kp=%d)", who, (long long)rows, c, kp);
  MMR_REQUIRE(c > 0 && c % 8 == 0 && rows >= 0, "%s: c=%d must be a positive multiple of 8", who, c);
  MMR_REQUIRE(c <= 4096, "%s: c=%d > 4096", who, c);
  if (rows == 0) return MMR_OK;
  hipStream_t st = mmr::as_stream(stream);
  const int nch = c / 8;
  // lanes per row: the narrowest LPR that splits the row's 16-B chunks evenly into <= 3 per lane
  // (no idle lanes, the NC = 3 instantiation at 56 VGPRs = 8 waves/SIMD; measured 3-6 % faster
  // than <= 6 per lane on the BERT/Swin widths, tools/ln_bench.py); then <= 6; otherwise <= 2
  // chunks per lane for narrow rows
  int lpr = 0;
  for (int lim = 3; lim <= 6 && !lpr; lim += 3)
    for (int l = 8; l <= 64 && !lpr; l *= 2)
      if (nch % l == 0 && nch / l <= lim) lpr = l;
  if (!lpr) {
    lpr = 64;
    while (lpr > 8 && nch <= (lpr / 2) * 2) lpr /= 2;
  }
  const int cpl = (nch + lpr - 1) / lpr;                   // chunks per lane
  const int64_t rows_per_block = 4 * (64 / lpr);
  const dim3 grid((unsigned)mmr::ceil_div(rows, rows_per_block));
#define MMR_LN2(L, N)                                                                                          \
  (q8 ? (r ? layernorm_bf16<L, N, true, true><<<grid, 256, 0, st>>>(x, r, gamma, beta, y, rows, c, eps, alpha, q8,  \
                                                                    q8s, kp)                                        \
           : layernorm_bf16<L, N, false, true><<<grid, 256, 0, st>>>(x, r, gamma, beta, y, rows, c, eps, alpha, q8, \
                                                                     q8s, kp))                                        \
      : (r ? layernorm_bf16<L, N, true><<<grid, 256, 0, st>>>(x, r, gamma, beta, y, rows, c, eps, alpha)          \
           : layernorm_bf16<L, N, false><<<grid, 256, 0, st>>>(x, r, gamma, beta, y, rows, c, eps, alpha)))
#define MMR_LN(L) (cpl <= 3 ? MMR_LN2(L, 3) : (cpl <= 6 ? MMR_LN2(L, 6) : MMR_LN2(L, 8)))
  if (lpr == 8) MMR_LN(8);
  else if (lpr == 16) MMR_LN(16);
  else if (lpr == 32) MMR_LN(32);
  else MMR_LN(64);
#undef MMR_LN
#undef MMR_LN2
  MMR_LAUNCH_CHECK();
  return MMR_OK;
}

mmr_status mmr_layernorm_bf16(const uint16_t* x, const float* gamma, const float* beta,
                              uint16_t* y, int64_t rows, int32_t c, float eps, void* stream) {
  mmr::clear_error();
  return layernorm_launch(x, nullptr, gamma, beta, y, rows, c, eps, stream, "mmr_layernorm_bf16");
}

mmr_status mmr_add_layernorm_bf16(const uint16_t* x, const uint16_t* residual, const float* gamma,
                                  const float* beta, uint16_t* y, int64_t rows, int32_t c,
                                  float eps, void* stream) {
  mmr::clear_error();
  MMR_REQUIRE(residual, "mmr_add_layernorm_bf16: NULL residual");
  return layernorm_launch(x, residual, gamma, beta, y, rows, c, eps, stream, "mmr_add_layernorm_bf16");
}

mmr_status mmr_layernorm_bf16_q8(const uint16_t* x, const uint16_t* residual, const float* gamma,
                                 const float* beta, uint16_t* y, uint8_t* q8, uint8_t* q8_scales, int64_t rows,
                                 int32_t c, float eps, void* stream) {
  mmr::clear_error();
  MMR_REQUIRE(q8 && q8_scales, "mmr_layernorm_bf16_q8: NULL MX-fp8 output");
  return layernorm_launch(x, residual, gamma, beta, y, rows, c, eps, stream, "mmr_layernorm_bf16_q8", nullptr, q8,
                          q8_scales);
}

mmr_status mmr_layernorm_bf16_q8p(const uint16_t* x, const uint16_t* residual, const float* gamma,
                                  const float* beta, uint16_t* y, uint8_t* q8, uint8_t* q8_scales, int64_t rows,
                                  int32_t c, int32_t kp, float eps, void* stream) {
  mmr::clear_error();
  MMR_REQUIRE(q8 && q8_scales, "mmr_layernorm_bf16_q8p: NULL MX-fp8 output");
  return layernorm_launch(x, residual, gamma, beta, y, rows, c, eps, stream, "mmr_layernorm_bf16_q8p", nullptr, q8,
                          q8_scales, kp);
}

mmr_status mmr_scaled_add_layernorm_bf16(const uint16_t* x, const float* alpha, const uint16_t* residual,
                                         const float* gamma, const float* beta, uint16_t* y, int64_t rows,
                                         int32_t c, float eps, void* stream) {
  mmr::clear_error();
  return layernorm_launch(x, residual, gamma, beta, y, rows, c, eps, stream, "mmr_scaled_add_layernorm_bf16",
                          alpha);
}

mmr_status mmr_scaled_add_layernorm_bf16_q8(const uint16_t* x, const float* alpha, const uint16_t* residual,
                                            const float* gamma, const float* beta, uint16_t* y, uint8_t* q8,
                                            uint8_t* q8_scales, int64_t rows, int32_t c, float eps, void* stream) {
  mmr::clear_error();
  MMR_REQUIRE(q8 && q8_scales, "mmr_scaled_add_layernorm_bf16_q8: NULL MX-fp8 output");
  return layernorm_launch(x, residual, gamma, beta, y, rows, c, eps, stream, "mmr_scaled_add_layernorm_bf16_q8",
                          alpha, q8, q8_scales);
}

mmr_status mmr_bert_embed_q8(const int64_t* ids, const float* word, const float* pos, const float* type0,
                             const float* gamma, const float* beta, uint16_t* y, uint8_t* q8, uint8_t* q8_scales,
                             int32_t b, int32_t l, int32_t c, float eps, void* stream) {
  mmr::clear_error();
  MMR_REQUIRE(ids && word && pos && type0 && gamma && beta && y, "mmr_bert_embed: NULL pointer");
  MMR_REQUIRE(b >= 0 && l > 0 && c > 0, "mmr_bert_embed: bad shape");
  const int64_t ntok = (int64_t)b * l;
  MMR_REQUIRE(!q8 || (q8_scales && c % 256 == 0 && c <= 1024 && ntok % 256 == 0),
              "mmr_bert_embed_q8: needs c %% 256 == 0, c <= 1024 and b*l %% 256 == 0 (c=%d, b*l=%lld)", c,
              (long long)ntok);
  if (ntok == 0) return MMR_OK;
  bert_embed<<<dim3((unsigned)mmr::ceil_div(ntok, 4)), 256, 0, mmr::as_stream(stream)>>>(
      ids, word, pos, type0, gamma, beta, y, ntok, l, c, eps, q8, q8_scales);
  MMR_LAUNCH_CHECK();
  return MMR_OK;
}

mmr_status mmr_bert_embed(const int64_t* ids, const float* word, const float* pos,
                          const float* type0, const float* gamma, const float* beta, uint16_t* y,
                          int32_t b, int32_t l, int32_t c, float eps, void* stream) {
  return mmr_bert_embed_q8(ids, word, pos, type0, gamma, beta, y, nullptr, nullptr, b, l, c, eps, stream);
}

mmr_status mmr_swin_attn_bias(const float* relpos_table, float* bias, int32_t heads, int32_t ws,
                              int32_t hw, int32_t shift, void* stream) {
  mmr::clear_error();
  MMR_REQUIRE(relpos_table && bias, "mmr_swin_attn_bias: NULL pointer");
  MMR_REQUIRE(heads > 0 && ws > 0 && ws * ws <= 64 && hw % ws == 0 && shift >= 0 && shift < ws,
              "mmr_swin_attn_bias: heads=%d ws=%d hw=%d shift=%d", heads, ws, hw, shift);
  const int ntypes = shift > 0 ? 4 : 1;
  const int64_t n = (int64_t)ntypes * heads * 4096;
  swin_attn_bias<<<dim3((unsigned)mmr::ceil_div(n, 256)), 256, 0, mmr::as_stream(stream)>>>(
      relpos_table, bias, heads, ws, hw, shift, ntypes);
  MMR_LAUNCH_CHECK();
  return MMR_OK;
}

static mmr_status swin_window_attention_launch(const uint16_t* qkv, const float* bias, uint16_t* out, uint8_t* q8,
                                               uint8_t* q8s, int32_t b, int32_t hw, int32_t c, int32_t kp,
                                               int32_t heads, int32_t ws, int32_t shift, void* stream) {
  MMR_REQUIRE(qkv && bias && (out || (q8 && q8s)), "mmr_swin_window_attention: NULL pointer");
  MMR_REQUIRE(!q8 || ((int64_t)b * hw * hw % 256 == 0 && kp % 256 == 0 && kp >= c),
              "mmr_swin_window_attention_q8: rows %lld must be a multiple of 256 and kp=%d a multiple of 256 >= c=%d",
              (long long)b * hw * hw, kp, c);
  MMR_REQUIRE(heads > 0 && c == heads * SW_DH, "mmr_swin_window_attention: c=%d heads=%d (head_dim 32 only)", c, heads);
  MMR_REQUIRE(ws > 0 && ws * ws <= 64 && hw % ws == 0, "mmr_swin_window_attention: window %d / resolution %d", ws, hw);
  MMR_REQUIRE(shift >= 0 && shift < ws, "mmr_swin_window_attention: shift %d", shift);
  if (b == 0) return MMR_OK;
  MMR_REQUIRE((int64_t)b * hw * hw * 3 * c < ((int64_t)1 << 32), "mmr_swin_window_attention: %lld qkv elements (32-bit offsets)",
              (long long)b * hw * hw * 3 * c);
  // one head per wave: the head pairs (hpw = 2, a wave reading whole 128-B lines) serialise two load
  // round trips per wave, and the pair's halves of a line are read by adjacent waves of one workgroup
  // anyway (6 / 12 / 24 heads, 4 waves per workgroup): in the cfg2 step stage 2 131 -> 116 us, at
  // B = 2048 every stage 7 % faster with single heads (profiles/r05_swa_head_pairs_ab.txt)
  const int hpw = 1;
  const int64_t units = (int64_t)b * (hw / ws) * (hw / ws) * ((heads + hpw - 1) / hpw);
  if (q8)
    swin_window_attention<true><<<dim3((unsigned)mmr::ceil_div(units, 4)), 256, 0, mmr::as_stream(stream)>>>(
        qkv, bias, nullptr, units, hw, c, heads, ws, shift, hpw, q8, q8s, kp);
  else
    swin_window_attention<false><<<dim3((unsigned)mmr::ceil_div(units, 4)), 256, 0, mmr::as_stream(stream)>>>(
        qkv, bias, out, units, hw, c, heads, ws, shift, hpw);
  MMR_LAUNCH_CHECK();
  return MMR_OK;
}

mmr_status mmr_swin_window_attention(const uint16_t* qkv, const float* bias, uint16_t* out,
                                     int32_t b, int32_t hw, int32_t c, int32_t heads, int32_t ws,
                                     int32_t shift, void* stream) {
  mmr::clear_error();
  MMR_REQUIRE(out, "mmr_swin_window_attention: NULL output");
  return swin_window_attention_launch(qkv, bias, out, nullptr, nullptr, b, hw, c, c, heads, ws, shift, stream);
}

mmr_status mmr_swin_window_attention_q8(const uint16_t* qkv, const float* bias, uint8_t* q8, uint8_t* q8_scales,
                                        int32_t b, int32_t hw, int32_t c, int32_t kp, int32_t heads, int32_t ws,
                                        int32_t shift, void* stream) {
  mmr::clear_error();
  MMR_REQUIRE(q8 && q8_scales, "mmr_swin_window_attention_q8: NULL MX-fp8 output");
  return swin_window_attention_launch(qkv, bias, nullptr, q8, q8_scales, b, hw, c, kp, heads, ws, shift, stream);
}

mmr_status mmr_patch_im2col(const float* image, uint16_t* cols, int32_t b, int32_t cin,
                            int32_t hw, int32_t patch, void* stream) {
  mmr::clear_error();
  MMR_REQUIRE(image && cols, "mmr_patch_im2col: NULL pointer");
  MMR_REQUIRE(cin * patch * patch <= 64 && hw % patch == 0, "mmr_patch_im2col: cin*patch^2 must be <= 64");
  const int64_t ntok = (int64_t)b * (hw / patch) * (hw / patch);
  if (ntok == 0) return MMR_OK;
  if (patch == 4 && cin == 3 && hw % 4 == 0 && (int64_t)b * 3 * hw * hw < (int64_t(1) << 31) &&
      ((uintptr_t)image & 15u) == 0)
    patch_im2col_p4c3<<<dim3((unsigned)mmr::ceil_div(ntok * 8, 256)), 256, 0, mmr::as_stream(stream)>>>(
        image, cols, (uint32_t)ntok, (uint32_t)hw);
  else
    patch_im2col<<<dim3((unsigned)mmr::ceil_div(ntok * 8, 256)), 256, 0, mmr::as_stream(stream)>>>(
        image, cols, ntok, cin, hw, patch);
  MMR_LAUNCH_CHECK();
  return MMR_OK;
}

static mmr_status patch_merge_launch(const uint16_t* x, const float* gamma, const float* beta, uint16_t* y,
                                     uint8_t* q8, uint8_t* q8s, int32_t b, int32_t hw, int32_t c, float eps,
                                     void* stream) {
  MMR_REQUIRE(x && gamma && beta && (y || q8), "mmr_patch_merge_ln: NULL pointer");
  MMR_REQUIRE(hw % 2 == 0 && c % 8 == 0, "mmr_patch_merge_ln: hw=%d c=%d", hw, c);
  const int64_t nout = (int64_t)b * (hw / 2) * (hw / 2);
  MMR_REQUIRE(!q8 || (nout % 256 == 0 && (4 * c) % 256 == 0 && 4 * c <= 2048),
              "mmr_patch_merge_ln_q8: needs merged rows %% 256 == 0 and 4c %% 256 == 0, 4c <= 2048 (rows=%lld c=%d)",
              (long long)nout, c);
  if (nout == 0) return MMR_OK;
  hipStream_t st = mmr::as_stream(stream);
  if (4 * c == 24 * 16)
    patch_merge_ln_g<16><<<dim3((unsigned)mmr::ceil_div(nout, 16)), 256, 0, st>>>(x, gamma, beta, y, nout, hw, c, eps);
  else if (4 * c == 24 * 32)
    patch_merge_ln_g<32><<<dim3((unsigned)mmr::ceil_div(nout, 8)), 256, 0, st>>>(x, gamma, beta, y, nout, hw, c, eps,
                                                                                  q8, q8s);
  else
    patch_merge_ln<<<dim3((unsigned)mmr::ceil_div(nout, 4)), 256, 0, st>>>(x, gamma, beta, y, nout, hw, c, eps, q8,
                                                                            q8s);
  MMR_LAUNCH_CHECK();
  return MMR_OK;
}

mmr_status mmr_patch_merge_ln(const uint16_t* x, const float* gamma, const float* beta,
                              uint16_t* y, int32_t b, int32_t hw, int32_t c, float eps,
                              void* stream) {
  mmr::clear_error();
  MMR_REQUIRE(y, "mmr_patch_merge_ln: NULL output");
  return patch_merge_launch(x, gamma, beta, y, nullptr, nullptr, b, hw, c, eps, stream);
}

mmr_status mmr_patch_merge_ln_q8(const uint16_t* x, const float* gamma, const float* beta, uint16_t* y,
                                 uint8_t* q8, uint8_t* q8_scales, int32_t b, int32_t hw, int32_t c, float eps,
                                 void* stream) {
  mmr::clear_error();
  MMR_REQUIRE(q8 && q8_scales, "mmr_patch_merge_ln_q8: NULL MX-fp8 output");
  return patch_merge_launch(x, gamma, beta, y, q8, q8_scales, b, hw, c, eps, stream);
}

mmr_status mmr_swin_head(const uint16_t* x, const float* gamma, const float* beta, float* patches,
                         float* global, float* pool, int32_t b, int32_t t, int32_t c, float eps,
                         void* stream) {
  mmr::clear_error();
  MMR_REQUIRE(x && gamma && beta, "mmr_swin_head: NULL pointer");
  MMR_REQUIRE(c % 64 == 0 && c <= 64 * SH_MAXPL && t > 0, "mmr_swin_head: c=%d must be a multiple of 64 <= 1024", c);
  if (b == 0) return MMR_OK;
  swin_head<<<dim3((unsigned)b), 64 * SH_WAVES, 0, mmr::as_stream(stream)>>>(x, gamma, beta, patches, global,
                                                                   pool, t, c, eps);
  MMR_LAUNCH_CHECK();
  return MMR_OK;
}

mmr_status mmr_mean_tokens(const uint16_t* x, float* y, int32_t b, int32_t l, int32_t c,
                           void* stream) {
  mmr::clear_error();
  MMR_REQUIRE(x && y && l > 0 && c > 0, "mmr_mean_tokens: bad arguments");
  if (b == 0) return MMR_OK;
  mean_tokens<<<dim3((unsigned)mmr::ceil_div(c, 256), (unsigned)b), 256, 0, mmr::as_stream(stream)>>>(x, y, l, c);
  MMR_LAUNCH_CHECK();
  return MMR_OK;
}

mmr_status mmr_proj_head(const float* x, const float* wp, const float* bp, const float* w1,
                         const float* b1, const float* w2, const float* b2, float* y, int32_t b,
                         int32_t cin, int32_t d, int32_t l2norm, void* stream) {
  mmr::clear_error();
  MMR_REQUIRE(x && wp && y && b >= 0 && cin > 0 && d > 0, "mmr_proj_head: bad arguments");
  MMR_REQUIRE(cin % 16 == 0 && d % 32 == 0, "mmr_proj_head: cin=%d must be a multiple of 16, d=%d of 32", cin, d);
  MMR_REQUIRE((w1 == nullptr) == (w2 == nullptr), "mmr_proj_head: w1/w2 must both be set or both NULL");
  if (b == 0) return MMR_OK;
  hipStream_t st = mmr::as_stream(stream);
  const dim3 blk(256);
  auto lin = [&](const float* xi, const float* w, const float* bb, float* yo, int ci, int co, int act) {
    launch_linear_f32(xi, w, bb, yo, b, ci, co, act, ci, co, nullptr, 0, st);
  };
  if (w1 == nullptr) {
    lin(x, wp, bp, y, cin, d, 0);
    MMR_LAUNCH_CHECK();
  } else {
    float *t0 = nullptr, *t1 = nullptr;
    MMR_CHECK_HIP(hipMallocAsync((void**)&t0, sizeof(float) * (size_t)b * d, st));
    MMR_CHECK_HIP(hipMallocAsync((void**)&t1, sizeof(float) * (size_t)b * 2 * d, st));
    lin(x, wp, bp, t0, cin, d, 0);
    lin(t0, w1, b1, t1, d, 2 * d, 1);
    lin(t1, w2, b2, y, 2 * d, d, 0);
    MMR_LAUNCH_CHECK();
    MMR_CHECK_HIP(hipFreeAsync(t0, st));
    MMR_CHECK_HIP(hipFreeAsync(t1, st));
  }
  if (l2norm) {
    l2_normalize_rows<<<dim3((unsigned)mmr::ceil_div(b, 4)), blk, 0, st>>>(y, b, d);
    MMR_LAUNCH_CHECK();
  }
  return MMR_OK;
}

mmr_status mmr_linear_f32(const float* x, int64_t ldx, const float* w, const float* bias,
                          const float* residual, int64_t ldr, float* y, int64_t ldy, int32_t b,
                          int32_t cin, int32_t cout, int32_t act, void* stream) {
  mmr::clear_error();
  MMR_REQUIRE(x && w && y && b >= 0 && cin > 0 && cout > 0, "mmr_linear_f32: bad arguments");
  MMR_REQUIRE(cin % 16 == 0 && cout % 32 == 0, "mmr_linear_f32: cin=%d must be a multiple of 16, cout=%d of 32", cin, cout);
  MMR_REQUIRE(ldx >= cin && ldx % 4 == 0 && ldy >= cout && (!residual || ldr >= cout),
              "mmr_linear_f32: bad row strides");
  MMR_REQUIRE(((uintptr_t)x & 15u) == 0 && ((uintptr_t)w & 15u) == 0, "mmr_linear_f32: x / w must be 16-B aligned");
  MMR_REQUIRE(act == 0 || act == 1, "mmr_linear_f32: act=%d", act);
  if (b == 0) return MMR_OK;
  launch_linear_f32(x, w, bias, y, b, cin, cout, act, ldx, ldy, residual, ldr, mmr::as_stream(stream));
  MMR_LAUNCH_CHECK();
  return MMR_OK;
}

mmr_status mmr_linear_f32_batched(const float* x, int64_t ldx, int64_t bsx, const float* w, int64_t bsw,
                                  const float* bias, int64_t bsb, const float* residual, int64_t ldr,
                                  int64_t bsr, float* y, int64_t ldy, int64_t bsy, int32_t nbatch, int32_t b,
                                  int32_t cin, int32_t cout, int32_t act, void* stream) {
  mmr::clear_error();
  MMR_REQUIRE(x && w && y && b >= 0 && cin > 0 && cout > 0 && nbatch >= 1, "mmr_linear_f32_batched: bad arguments");
  MMR_REQUIRE(cin % 16 == 0 && cout % 32 == 0, "mmr_linear_f32_batched: cin=%d must be a multiple of 16, cout=%d of 32",
              cin, cout);
  MMR_REQUIRE(ldx >= cin && ldx % 4 == 0 && ldy >= cout && (!residual || ldr >= cout) && bsx % 4 == 0 && bsw % 4 == 0,
              "mmr_linear_f32_batched: bad strides");
  MMR_REQUIRE(((uintptr_t)x & 15u) == 0 && ((uintptr_t)w & 15u) == 0, "mmr_linear_f32_batched: x / w must be 16-B aligned");
  MMR_REQUIRE(act == 0 || act == 1, "mmr_linear_f32_batched: act=%d", act);
  if (b == 0) return MMR_OK;
  launch_linear_f32(x, w, bias, y, b, cin, cout, act, ldx, ldy, residual, ldr, mmr::as_stream(stream), nbatch, bsx,
                    bsw, bsb, bsr, bsy);
  MMR_LAUNCH_CHECK();
  return MMR_OK;
}

}  // extern "C"
