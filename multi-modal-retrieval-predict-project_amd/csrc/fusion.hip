// Multimodal fusion stack (model_type="multimodal"): the small-sequence attention core and the
// elementwise / row kernels around the GEMMs (gemm.hip) and f32 linears (tower.hip).
//
// Reference (semantics): CrossModalFusion.forward src/Model/fusion.py:390-471, PreFusionEnhancer
// fusion.py:20-35, MultiModalRetrievalModel.forward model.py:375-459, torch.nn.MultiheadAttention
// (batch_first, eval, no masks).  Host-side orchestration + weight folding: fusion.py in the package.
#include <float.h>
#include <math.h>

#include <algorithm>

#include "common.h"

namespace {

using mmr::bf2f;
using mmr::f2bf;

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// ------------------------------------------------------------------ small-sequence MHA core
// softmax(q k^T * scale) v per (batch, head): the fusion's short sequences (text L <= 512,
// 49 patches, 51-token fused sequence; no masks) and BERT self-attention (MASK: key-padding mask,
// HF BertSelfAttention).  Block = (batch*head, chunk of 128 queries), one 32-query tile per wave;
// keys stream through LDS in blocks of kbs (64 / 128) with an online softmax.  The swapped product
// S^T = K . Q^T on v_mfma_f32_32x32x16_bf16 puts the query on the lane, the softmax reductions
// stay in registers, and P^T feeds the P.V MFMA as its B operand with no data movement (V^T read
// in the matching key permutation).  head_dim is
// padded to DT*32 with zeros (dh % 8 == 0); ragged query/key counts are padded to 32 (padded keys
// -> -inf, padded queries never stored).  Operands are strided rows (q row (b*lq + i) at
// q + row*ldq + head*dh), so Q/K/V are read in place from packed projection outputs.  Optional f32
// mean over the lq query rows (mean_out (b, heads*dh)): the fusion only needs mean_L of several
// attention outputs (fusion.py:441,448, model.py:431), and mean_L(A) W^T + b == mean_L(A W^T + b),
// so those out-projections shrink to one row per batch.  With one query chunk (lq <= 128, every
// fusion call at L = 128) the mean is reduced in LDS and stored; with several chunks each adds its
// partial into the (pre-zeroed) output with a float atomic.
constexpr int MHA_KB = 128;
typedef __attribute__((address_space(3))) void* lds_ptr_t;

// occupancy targets (waves per SIMD; without them hipcc splits o into AGPRs and lands at 2 / 1):
// head_dim <= 32 -> 4, <= 96 -> 3 (BERT 64, fusion 96), else 2 (128 unmasked at 3: 168 VGPRs, no spill, but
// measured neutral to 4 % slower, profiles/r03_s5_attn_occupancy_ab.txt)
template <int DT, bool MASK>
__global__ __launch_bounds__(256, DT == 1 ? 4 : (DT <= 3 ? 3 : 2)) void mha_small(const uint16_t* __restrict__ q, int64_t ldq,
                                                 const uint16_t* __restrict__ k, int64_t ldk,
                                                 const uint16_t* __restrict__ v, int64_t ldv,
                                                 uint16_t* __restrict__ out, int64_t ldo,
                                                 float* __restrict__ mean_out,
                                                 const int64_t* __restrict__ kmask, int lq, int lk,
                                                 int heads, int dh, float scale, int kbs,
                                                 uint8_t* __restrict__ q8 = nullptr,
                                                 uint8_t* __restrict__ q8s = nullptr) {
  constexpr int DHP = DT * 32;
  constexpr int KS = DHP / 16;
  constexpr int KROW = DHP + 8;       // padded K row (elements): 16-B skew between consecutive keys
  // V row stride: (stride in 4-B banks) = 16 or 48 mod 64, so the 4 rows x 64 B of one half-wave's
  // transposed reads land on disjoint banks
  constexpr int VROW = DHP + ((DT & 1) ? 0 : 16);
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int unit = mmr::xcd_contiguous(blockIdx.x, gridDim.x);
  const int bi = unit / heads, hh = unit % heads;
  const int lkp = (lk + 31) & ~31;
  // LDS sized to the launch (mha_lds_bytes): kbs keys per staged block (64 / 128), one epilogue
  // area per wave — a 49-query / 51-key call then takes half the LDS of a 128 x 128 one, and with it
  // twice the workgroups per CU
  const int tid = threadIdx.x, nthr = blockDim.x, lane = tid & 63, wave = tid >> 6, nwv = nthr >> 6;
  uint16_t* Ks = (uint16_t*)smem;            // [kbs][KROW]
  uint16_t* Vs = Ks + kbs * KROW;            // [kbs][VROW], natural (key-major) layout
  // [waves][DHP] per-wave partial means, after the larger of the K/V image and the epilogue area
  const int kv_bytes = kbs * (KROW + VROW) * 2, red_bytes = nwv * DHP * 33 * 4;
  float* msum = (float*)(smem + (kv_bytes > red_bytes ? kv_bytes : red_bytes));
  float* madd = msum + nwv * DHP;  // [kbs] additive key mask of the current key block (kmask)
  const uint16_t* kbase = k + (int64_t)bi * lk * ldk + hh * dh;
  const uint16_t* vbase = v + (int64_t)bi * lk * ldv + hh * dh;

  const int r = lane & 31, hf = lane >> 5;
  const int q0 = blockIdx.y * 128 + wave * 32;
  const bool active = q0 < lq;               // wave-uniform
  const int qi = q0 + r;
  const bool qok = qi < lq;
  bf16x8 qf[KS];
  {
    const uint16_t* qrow = q + ((int64_t)bi * lq + (qok ? qi : 0)) * ldq + hh * dh;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int c8 = ks * 2 + hf;
      qf[ks] = (bf16x8){0, 0, 0, 0, 0, 0, 0, 0};
      if (qok && c8 * 8 < dh) qf[ks] = *(const bf16x8*)(qrow + c8 * 8);
    }
  }
  f32x16 o[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) o[dt] = (f32x16){0};
  float m_run = -FLT_MAX, l_run = 0.f;
  const float c2 = scale * 1.4426950408889634f;  // scale * log2(e)
  for (int k0 = 0; k0 < lkp; k0 += kbs) {
    const int kn = min(kbs, lkp - k0);      // keys staged this round (multiple of 32)
    __syncthreads();                          // previous key block consumed
    // HBM -> LDS by global_load_lds (16 B per lane, lane-linear per wave instruction): LDS slot j of
    // the padded image is filled from whichever global chunk belongs there, so every load of the
    // block is in flight at once with no VGPR staging.  Pad slots, chunks past dh and keys past lk
    // read a clamped in-bounds chunk: finite values that the zero Q columns / the -inf key mask /
    // the discarded O columns make irrelevant.
    {
      constexpr int KSL = KROW / 8, VSL = VROW / 8;
      const int nk = kn * KSL, nv = kn * VSL, nw64 = nthr;
      for (int b0 = wave * 64; b0 < nk; b0 += nw64) {
        const int slot = b0 + lane;
        if (slot < nk) {
          const int key = slot / KSL, ch = slot % KSL;
          const int ks = min(k0 + key, lk - 1), cs = (ch * 8 < dh) ? ch : 0;
          __builtin_amdgcn_global_load_lds((const void*)(kbase + (int64_t)ks * ldk + cs * 8),
                                           (lds_ptr_t)(Ks + b0 * 8), 16, 0, 0);
        }
      }
      for (int b0 = wave * 64; b0 < nv; b0 += nw64) {
        const int slot = b0 + lane;
        if (slot < nv) {
          const int key = slot / VSL, ch = slot % VSL;
          const int ks = min(k0 + key, lk - 1), cs = (ch * 8 < dh) ? ch : 0;
          __builtin_amdgcn_global_load_lds((const void*)(vbase + (int64_t)ks * ldv + cs * 8),
                                           (lds_ptr_t)(Vs + b0 * 8), 16, 0, 0);
        }
      }
    }
    if constexpr (MASK)
      for (int i = tid; i < kn; i += nthr) {
        const int key = k0 + i;
        madd[i] = (key < lk && kmask[(int64_t)bi * lk + key] != 0) ? 0.f : -FLT_MAX;
      }
    __syncthreads();
    if (!active) continue;
    for (int kb = 0; kb < kn; kb += 64) {
      const int nt = min(64, kn - kb) / 32;
      // with a key mask, 32-key tiles whose keys are all masked contribute exactly 0 (p = 2^-huge)
      // once any key has been seen: skipped (BERT reports are padded to L, ~40 % of the keys)
      bool live[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        live[t] = t < nt;
        if (MASK && live[t] && k0 + kb + t * 32 > 0)
          live[t] = __ballot(madd[kb + t * 32 + r] == 0.f) != 0;
      }
      f32x16 s[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        s[t] = (f32x16){0};
        if (live[t]) {
          const int key = kb + t * 32 + r;
#pragma unroll
          for (int ks = 0; ks < KS; ++ks) {
            const bf16x8 kf = *(const bf16x8*)(Ks + key * KROW + (ks * 2 + hf) * 8);
            s[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[ks], s[t], 0, 0, 0);
          }
        }
      }
      // softmax on raw scores with the scale folded into the exponent: p = 2^(s c - m c),
      // c = scale * log2(e) (one fma + v_exp per score); without a key mask, keys past lk are
      // masked only in the tile that holds them
      float mloc = -FLT_MAX;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        if (live[t]) {
          if constexpr (MASK) {
#pragma unroll
            for (int g = 0; g < 4; ++g) {
              const float4 mv = *(const float4*)(madd + kb + t * 32 + 8 * g + 4 * hf);
              s[t][4 * g] += mv.x;
              s[t][4 * g + 1] += mv.y;
              s[t][4 * g + 2] += mv.z;
              s[t][4 * g + 3] += mv.w;
            }
          } else if (k0 + kb + t * 32 + 32 > lk) {  // wave-uniform
#pragma unroll
            for (int rg = 0; rg < 16; ++rg) {
              const int key = k0 + kb + t * 32 + (rg & 3) + 8 * (rg >> 2) + 4 * hf;
              if (key >= lk) s[t][rg] = -FLT_MAX;
            }
          }
#pragma unroll
          for (int rg = 0; rg < 16; ++rg) mloc = fmaxf(mloc, s[t][rg]);
        }
      }
      mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
      const float m_new = fmaxf(m_run, mloc);
      const float mc = m_new * c2;
      const float alpha = __builtin_amdgcn_exp2f(fmaf(m_run, c2, -mc));  // 0 on the first block
      m_run = m_new;
      float psum = 0.f;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        if (live[t]) {
#pragma unroll
          for (int rg = 0; rg < 16; ++rg) {
            const float p = __builtin_amdgcn_exp2f(fmaf(s[t][rg], c2, -mc));
            s[t][rg] = p;
            psum += p;
          }
        }
      }
      l_run = l_run * alpha + psum;
      if (k0 + kb > 0) {  // O is still zero before the first key block: nothing to rescale
#pragma unroll
        for (int dt = 0; dt < DT; ++dt)
#pragma unroll
          for (int rg = 0; rg < 16; ++rg) o[dt][rg] *= alpha;
      }
      // O^T[d][q] += V^T[d][key] . P^T[key][q]; the V^T fragment (lane: d = its row, keys
      // kk..kk+3 and kk+8..kk+11 in P^T's register order) comes from the key-major V image by two
      // ds_read_b64_tr_b16: in each 16-lane group, lane 4q+p addresses row (key) r0+q, columns
      // c0+4p..+3, and lane i receives column c0+i of the 4 rows (cdna_hip_programming.md T10)
      const int grp = lane >> 4, tq = (lane >> 2) & 3, tp = lane & 3;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        if (live[t]) {
#pragma unroll
          for (int sidx = 0; sidx < 2; ++sidx) {
            uint32_t pw[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) pw[j] = mmr::pack2bf(s[t][8 * sidx + 2 * j], s[t][8 * sidx + 2 * j + 1]);
            const bf16x8 pf = __builtin_bit_cast(bf16x8, make_uint4(pw[0], pw[1], pw[2], pw[3]));
            const int r0 = kb + t * 32 + 16 * sidx + 4 * (grp >> 1);
#pragma unroll
            for (int dt = 0; dt < DT; ++dt) {
              const int c0 = dt * 32 + (grp & 1) * 16;
              const uint16_t* va = Vs + (r0 + tq) * VROW + c0 + 4 * tp;
              const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) bf16x4*)va);
              const bf16x4 hi =
                  __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) bf16x4*)(va + 8 * VROW));
              const bf16x8 vf = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
              o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf, o[dt], 0, 0, 0);
            }
          }
        }
      }
    }
  }
  // epilogue through LDS (the K/V image is free once every wave is past its last key block):
  //  - out: the wave's O tile is staged as bf16 [32 q][DHP + 4] and written back as contiguous 8-B
  //    chunks per query row (coalesced), instead of 4 scattered 8-B stores per MFMA tile;
  //  - mean: lane (q = r) writes its O^T column into red[d][q], then lane l sums rows d = l, l + 64,
  //    ... (no cross-lane shuffle chains).  Both use the wave's own region, one after the other.
  constexpr int RLD = 33, OROW = DHP + 4;
  float* red = (float*)smem + wave * DHP * RLD;
  __syncthreads();
  if (active) {
    const float inv = 1.0f / (l_run + __shfl_xor(l_run, 32, 64));
    if (out != nullptr || q8 != nullptr) {
      uint16_t* st = (uint16_t*)red;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const int d = dt * 32 + 8 * g4 + 4 * hf;
          uint2 w;
          w.x = mmr::pack2bf(o[dt][4 * g4] * inv, o[dt][4 * g4 + 1] * inv);
          w.y = mmr::pack2bf(o[dt][4 * g4 + 2] * inv, o[dt][4 * g4 + 3] * inv);
          *(uint2*)(st + r * OROW + d) = w;
        }
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's LDS writes landed
      __builtin_amdgcn_wave_barrier();
      const int nc4 = dh / 4;
      if (out != nullptr)
        for (int c = lane; c < 32 * nc4; c += 64) {
          const int row = c / nc4, ch = c % nc4;
          if (q0 + row < lq)
            *(bf16x4*)(out + ((int64_t)bi * lq + q0 + row) * ldo + hh * dh + ch * 4) =
                *(const bf16x4*)(st + row * OROW + ch * 4);
        }
      if (q8 != nullptr) {
        // the context as the O-proj GEMM's MX-fp8 operand (bit-identical to quantising the bf16
        // rows): lane = (query row, 32-channel block of this head), 32 values from the staged tile
        const int nb = dh / 32, c = heads * dh;
        for (int pr = lane; pr < 32 * nb; pr += 64) {
          const int row = pr / nb, blk = pr % nb;
          const int64_t grow = (int64_t)bi * lq + q0 + row;
          float v[32];
          float amax = 0.f;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const bf16x4 u = *(const bf16x4*)(st + row * OROW + blk * 32 + 4 * j);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              v[4 * j + e] = mmr::bf2f((uint16_t)u[e]);
              amax = fmaxf(amax, fabsf(v[4 * j + e]));
            }
          }
          const int ex = mmr::q8_exp(amax);
          const float iv = mmr::q8_inv(ex);
          uint32_t w[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) w[j] = mmr::q8_pack4(v + 4 * j, iv);
          if (q0 + row < lq) {
            uint8_t* dst = q8 + grow * c + hh * dh + blk * 32;
            *(uint4*)dst = make_uint4(w[0], w[1], w[2], w[3]);
            *(uint4*)(dst + 16) = make_uint4(w[4], w[5], w[6], w[7]);
            q8s[mmr::q8_soff(grow, hh * dh + blk * 32, c)] = (uint8_t)(ex + 127);
          }
        }
      }
      __builtin_amdgcn_s_waitcnt(0xC07F);
      __builtin_amdgcn_wave_barrier();
    }
    if (mean_out != nullptr) {
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int rg = 0; rg < 16; ++rg) {
          const int d = dt * 32 + (rg & 3) + 8 * (rg >> 2) + 4 * hf;
          red[d * RLD + r] = qok ? o[dt][rg] * inv : 0.f;
        }
      __builtin_amdgcn_s_waitcnt(0xC07F);
      __builtin_amdgcn_wave_barrier();
      for (int d = lane; d < DHP; d += 64) {
        float acc = 0.f;
#pragma unroll 8
        for (int j = 0; j < 32; ++j) acc += red[d * RLD + j];
        msum[wave * DHP + d] = acc;
      }
    }
  }
  if (mean_out != nullptr) {
    __syncthreads();
    const int nw = nthr >> 6;
    for (int d = tid; d < dh; d += nthr) {
      float s = 0.f;
      for (int w = 0; w < nw; ++w)  // fixed order: deterministic
        if (blockIdx.y * 128 + w * 32 < lq) s += msum[w * DHP + d];
      float* dst = mean_out + (int64_t)bi * heads * dh + hh * dh + d;
      if (gridDim.y == 1) *dst = s / (float)lq;
      else atomicAdd(dst, s / (float)lq);
    }
  }
}

// ------------------------------------------------------------------ x + positional table -> bf16
// y[b][t][c] = x[b][t][c] + pos[t][c] (PreFusionEnhancer.pos_embed fusion.py:32, PositionalEncoding
// model.py:99-107); x f32 or bf16, pos f32 [>= l][c], 8 channels per thread.
// Q8: also the row as the next GEMM's MX-fp8 activation operand (mmr::q8_chunk8; c % 256 == 0, so a
// row's chunks fill whole 4-lane groups and a group never straddles the grid's ragged end).
template <typename TX, bool Q8 = false>
__global__ __launch_bounds__(256) void add_pos_bf16(const TX* __restrict__ x, const float* __restrict__ pos,
                                                    uint16_t* __restrict__ y, int64_t rows, int l, int c,
                                                    uint8_t* __restrict__ q8 = nullptr,
                                                    uint8_t* __restrict__ q8s = nullptr) {
  const int nch = c / 8;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= rows * nch) return;
  int64_t row;
  int ch, t;
  if (rows * nch < (int64_t(1) << 31)) {  // 32-bit divisions (64-bit ones dominate this kernel)
    const uint32_t i32 = (uint32_t)i, r32 = i32 / (uint32_t)nch;
    row = r32;
    ch = (int)(i32 - r32 * (uint32_t)nch);
    t = (int)(r32 % (uint32_t)l);
  } else {
    row = i / nch;
    ch = (int)(i % nch);
    t = (int)(row % l);
  }
  float v[8];
  if constexpr (sizeof(TX) == 4) {
    const float4 a = *(const float4*)((const float*)x + row * c + ch * 8);
    const float4 b = *(const float4*)((const float*)x + row * c + ch * 8 + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  } else {
    const bf16x8 a = *(const bf16x8*)((const uint16_t*)x + row * c + ch * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = bf2f((uint16_t)a[j]);
  }
  const float4 p0 = *(const float4*)(pos + (int64_t)t * c + ch * 8);
  const float4 p1 = *(const float4*)(pos + (int64_t)t * c + ch * 8 + 4);
  v[0] += p0.x; v[1] += p0.y; v[2] += p0.z; v[3] += p0.w;
  v[4] += p1.x; v[5] += p1.y; v[6] += p1.z; v[7] += p1.w;
  *(uint4*)(y + row * c + ch * 8) = make_uint4(mmr::pack2bf(v[0], v[1]), mmr::pack2bf(v[2], v[3]),
                                               mmr::pack2bf(v[4], v[5]), mmr::pack2bf(v[6], v[7]));
  if constexpr (Q8) {
    float vb[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) vb[j] = mmr::bf2f(mmr::f2bf(v[j]));  // the stored bf16 value
    mmr::q8_chunk8(vb, row, ch, c, q8, q8s, true);
  }
}

// ------------------------------------------------------------------ scaled-residual LayerNorm
// y = LN(a*x + r) * g + b  (+ ps*post), one row per wave.  x/r/y bf16 or f32 (template), a and ps
// read from device scalars (learned nn.Parameter(1), no host sync) or 1 when NULL, r/post optional.
// Covers PreFusionEnhancer norm1(alpha*x + x2) (fusion.py:34), ln_img / ln_txt (fusion.py:443,449),
// norm1_i(joint) + alpha*fused and norm2_i (model.py:437-441).  Row kept in registers
// (c <= 1024), centred two-pass variance like torch.
template <typename TI, typename TO, int NI = 16>
__global__ __launch_bounds__(256) void ln_rows(const TI* __restrict__ x, int64_t ldx, const float* __restrict__ a,
                                               const TI* __restrict__ r, int64_t ldr,
                                               const float* __restrict__ g, const float* __restrict__ b,
                                               const float* __restrict__ post, int64_t ldp,
                                               const float* __restrict__ ps, TO* __restrict__ y, int64_t ldy,
                                               int64_t rows, int c, float eps, int groups, int64_t gdiv) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const int grp = (int)((row / gdiv) % groups);  // per-row parameter set (layers batched in one launch)
  g += (int64_t)grp * c;
  b += (int64_t)grp * c;
  if (a) a += grp;
  if (ps) ps += grp;
  auto ld = [](const TI* p, int64_t i) -> float {
    if constexpr (sizeof(TI) == 4) return ((const float*)p)[i];
    else return bf2f(((const uint16_t*)p)[i]);
  };
  const float av = a ? *a : 1.f;
  // all loads unconditional and issued before any use (index clamped, value masked): a "load if
  // ch < c" branch makes hipcc wait for each load before the next — 16-32 serial round trips
  float v[NI], rv[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int ch = lane + 64 * i;
    v[i] = ld(x, row * ldx + (ch < c ? ch : c - 1));
  }
  if (r) {
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int ch = lane + 64 * i;
      rv[i] = ld(r, row * ldr + (ch < c ? ch : c - 1));
    }
  } else {
#pragma unroll
    for (int i = 0; i < NI; ++i) rv[i] = 0.f;
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const float t = mmr::mul_rn(av, v[i]) + rv[i];  // product rounded, then the sum (torch's alpha * x + r)
    v[i] = lane + 64 * i < c ? t : 0.f;
    s += v[i];
  }
  const float mean = mmr::wave_sum(s) / c;
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < NI; ++i)
    if (lane + 64 * i < c) ss += (v[i] - mean) * (v[i] - mean);
  const float rstd = rsqrtf(mmr::wave_sum(ss) / c + eps);
  const float pv = ps ? *ps : 1.f;
  float gv[NI], bv[NI], pp[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int ch = lane + 64 * i, chc = ch < c ? ch : c - 1;
    gv[i] = g[chc];
    bv[i] = b[chc];
  }
  if (post) {
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int ch = lane + 64 * i;
      pp[i] = pv * post[row * ldp + (ch < c ? ch : c - 1)];
    }
  } else {
#pragma unroll
    for (int i = 0; i < NI; ++i) pp[i] = 0.f;
  }
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int ch = lane + 64 * i;
    const float t = (v[i] - mean) * rstd * gv[i] + bv[i] + pp[i];
    if (ch < c) {
      if constexpr (sizeof(TO) == 4) ((float*)y)[row * ldy + ch] = t;
      else ((uint16_t*)y)[row * ldy + ch] = f2bf(t);
    }
  }
}

// f32 rows with c % (64 VW) == 0 and VW-aligned rows (the x3 towers' LayerNorms, c = 384 ... 1024): the
// same arithmetic as ln_rows<float, float> with VW-wide loads / stores (lane owns channels
// VW lane + 64 VW i ...), so a row moves in c / (64 VW) instructions per operand instead of 16
template <int VW>
__global__ __launch_bounds__(256) void ln_rows_v(const float* __restrict__ x, int64_t ldx, const float* __restrict__ a,
                                                 const float* __restrict__ r, int64_t ldr, const float* __restrict__ g,
                                                 const float* __restrict__ b, const float* __restrict__ post, int64_t ldp,
                                                 const float* __restrict__ ps, float* __restrict__ y, int64_t ldy,
                                                 int64_t rows, int c, float eps, int groups, int64_t gdiv) {
  typedef float fv_t __attribute__((ext_vector_type(VW)));
  constexpr int NI = 1024 / (64 * VW);
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const int grp = (int)((row / gdiv) % groups);
  g += (int64_t)grp * c;
  b += (int64_t)grp * c;
  if (a) a += grp;
  if (ps) ps += grp;
  const int ni = c / (64 * VW);  // wave-uniform
  const float av = a ? *a : 1.f;
  auto ofs = [&](int i) { return VW * lane + 64 * VW * (i < ni ? i : ni - 1); };  // clamped: loads unconditional
  fv_t v[NI], rv[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) v[i] = *(const fv_t*)(x + row * ldx + ofs(i));
  if (r) {  // (the residual loads in one uniform branch, issued back to back)
#pragma unroll
    for (int i = 0; i < NI; ++i) rv[i] = *(const fv_t*)(r + row * ldr + ofs(i));
  } else {
#pragma unroll
    for (int i = 0; i < NI; ++i) rv[i] = (fv_t)0.f;
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    fv_t t = v[i];
#pragma unroll
    for (int e = 0; e < VW; ++e) t[e] = mmr::mul_rn(av, t[e]);  // product rounded, then the sum
    v[i] = i < ni ? t + rv[i] : (fv_t)0.f;
#pragma unroll
    for (int e = 0; e < VW; ++e) s += v[i][e];
  }
  const float mean = mmr::wave_sum(s) / c;
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < NI; ++i)
    if (i < ni)
#pragma unroll
      for (int e = 0; e < VW; ++e) ss += (v[i][e] - mean) * (v[i][e] - mean);
  const float rstd = rsqrtf(mmr::wave_sum(ss) / c + eps);
  const float pv = ps ? *ps : 1.f;
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    if (i >= ni) break;
    const fv_t gv = *(const fv_t*)(g + ofs(i)), bv = *(const fv_t*)(b + ofs(i));
    const fv_t pp = post ? pv * *(const fv_t*)(post + row * ldp + ofs(i)) : (fv_t)0.f;
    fv_t t;
#pragma unroll
    for (int e = 0; e < VW; ++e) t[e] = (v[i][e] - mean) * rstd * gv[e] + bv[e] + pp[e];
    *(fv_t*)(y + row * ldy + ofs(i)) = t;
  }
}

// f32 rows of c <= 64 LPR / ... short rows (the x3 Swin stages 1-2, c = 96 / 192): LPR lanes per row (64 / LPR
// rows per wave), PER channels per lane (lane j: channels j + LPR i), reductions over the row's lane
// group — one row per wave left 2/3 of a c = 96 wave idle and paid a full wave reduction per row
template <int LPR, int PER>
__global__ __launch_bounds__(256) void ln_rows_s(const float* __restrict__ x, int64_t ldx, const float* __restrict__ a,
                                                 const float* __restrict__ r, int64_t ldr, const float* __restrict__ g,
                                                 const float* __restrict__ b, const float* __restrict__ post, int64_t ldp,
                                                 const float* __restrict__ ps, float* __restrict__ y, int64_t ldy,
                                                 int64_t rows, int c, float eps, int groups, int64_t gdiv) {
  constexpr int RPW = 64 / LPR;
  const int lane = threadIdx.x & 63, j = lane % LPR;
  const int64_t row = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW + lane / LPR;
  const bool live = row < rows;
  const int64_t rw = live ? row : rows - 1;  // dead lanes compute a valid row and store nothing
  const int grp = (int)((rw / gdiv) % groups);
  g += (int64_t)grp * c;
  b += (int64_t)grp * c;
  const float av = a ? a[grp] : 1.f;
  const float pv = ps ? ps[grp] : 1.f;
  auto chc = [&](int i) { const int ch = j + LPR * i; return ch < c ? ch : c - 1; };
  float v[PER], rv[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) v[i] = x[rw * ldx + chc(i)];
  if (r) {
#pragma unroll
    for (int i = 0; i < PER; ++i) rv[i] = r[rw * ldr + chc(i)];
  } else {
#pragma unroll
    for (int i = 0; i < PER; ++i) rv[i] = 0.f;
  }
  auto gsum = [](float t) {
#pragma unroll
    for (int o = 1; o < LPR; o <<= 1) t += __shfl_xor(t, o, 64);
    return t;
  };
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    v[i] = j + LPR * i < c ? mmr::mul_rn(av, v[i]) + rv[i] : 0.f;  // product rounded, then the sum
    s += v[i];
  }
  const float mean = gsum(s) / c;
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i)
    if (j + LPR * i < c) ss += (v[i] - mean) * (v[i] - mean);
  const float rstd = rsqrtf(gsum(ss) / c + eps);
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int ch = j + LPR * i;
    const float pp = post ? pv * post[rw * ldp + chc(i)] : 0.f;
    const float t = (v[i] - mean) * rstd * g[chc(i)] + b[chc(i)] + pp;
    if (live && ch < c) y[rw * ldy + ch] = t;
  }
}

// f32 LayerNorm(x + residual) that also writes the x3 split GEMM's operand rows (the x3 towers' LN ->
// QKV / fc1 pairs): xs row = [hi | lo] bf16, 2 kp wide (kp = c rounded up to 128, zero columns c..kp),
// the split mmr_x3_split_rows would make of the f32 output, which is written too when y != NULL.
// 32 lanes per row, NCH = kp / 128 4-wide chunks per lane (lane j: columns 4 (j + 32 i) ..+3).
template <int NCH>
__global__ __launch_bounds__(256) void ln_rows_split(const float* __restrict__ x, int64_t ldx,
                                                     const float* __restrict__ alpha, const float* __restrict__ r,
                                                     int64_t ldr, const float* __restrict__ g, const float* __restrict__ b,
                                                     float* __restrict__ y, int64_t ldy, uint16_t* __restrict__ xs,
                                                     int64_t rows, int c, float eps) {
  constexpr int KP = 128 * NCH;
  const int lane = threadIdx.x & 63, j = lane & 31;
  const int64_t row = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 2 + (lane >> 5);
  const bool live = row < rows;
  const int64_t rw = live ? row : rows - 1;
  float4 v[NCH];
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int col = 4 * (j + 32 * i);
    v[i] = col < c ? *(const float4*)(x + rw * ldx + col) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  if (alpha) {  // LN(alpha x + r) (PreFusionEnhancer, fusion.py:33): the product rounded, then the sum
    const float av = *alpha;
#pragma unroll
    for (int i = 0; i < NCH; ++i)  // mmr::mul_rn: never contracted into the residual add below
      v[i] = make_float4(mmr::mul_rn(av, v[i].x), mmr::mul_rn(av, v[i].y), mmr::mul_rn(av, v[i].z), mmr::mul_rn(av, v[i].w));
  }
  if (r) {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int col = 4 * (j + 32 * i);
      if (col < c) {
        const float4 t = *(const float4*)(r + rw * ldr + col);
        v[i].x += t.x, v[i].y += t.y, v[i].z += t.z, v[i].w += t.w;
      }
    }
  }
  auto gsum = [](float t) {
#pragma unroll
    for (int o = 1; o < 32; o <<= 1) t += __shfl_xor(t, o, 64);
    return t;
  };
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NCH; ++i) s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
  const float mean = gsum(s) / c;
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    if (4 * (j + 32 * i) < c) {
      const float a0 = v[i].x - mean, a1 = v[i].y - mean, a2 = v[i].z - mean, a3 = v[i].w - mean;
      ss += (a0 * a0 + a1 * a1) + (a2 * a2 + a3 * a3);
    }
  }
  const float rstd = rsqrtf(gsum(ss) / c + eps);
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int col = 4 * (j + 32 * i);
    float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
    if (col < c) {
      const float4 gg = *(const float4*)(g + col), bb = *(const float4*)(b + col);
      t = make_float4((v[i].x - mean) * rstd * gg.x + bb.x, (v[i].y - mean) * rstd * gg.y + bb.y,
                      (v[i].z - mean) * rstd * gg.z + bb.z, (v[i].w - mean) * rstd * gg.w + bb.w);
      if (live && y) *(float4*)(y + rw * ldy + col) = t;
    }
    const uint32_t h0 = mmr::pack2bf(t.x, t.y), h1 = mmr::pack2bf(t.z, t.w);
    const uint32_t l0 = mmr::pack2bf(t.x - __uint_as_float(h0 << 16), t.y - __uint_as_float(h0 & 0xFFFF0000u));
    const uint32_t l1 = mmr::pack2bf(t.z - __uint_as_float(h1 << 16), t.w - __uint_as_float(h1 & 0xFFFF0000u));
    if (live) {
      uint16_t* o = xs + rw * 2 * KP + col;
      *(uint2*)o = make_uint2(h0, h1);
      *(uint2*)(o + KP) = make_uint2(l0, l1);
    }
  }
}

// ------------------------------------------------------------------ fused-sequence assembly
// seq[b] = [x1[b]; patches_fused[b][0..np); x2[b]] + pe[0..np+2)  -> bf16 (b, np+2, c)
// (fusion.py:451-468 cat, model.py:396-397 dropout(eval) + pos_encoder).
__global__ __launch_bounds__(256) void assemble_seq(const float* __restrict__ x1, const uint16_t* __restrict__ pf,
                                                    const float* __restrict__ x2, const float* __restrict__ pe,
                                                    uint16_t* __restrict__ seq, int nb, int np, int c) {
  const int ls = np + 2;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)nb * ls * c) return;
  const int ch = (int)(i % c);
  const int64_t row = i / c;
  const int t = (int)(row % ls);
  const int64_t bi = row / ls;
  float v;
  if (t == 0) v = x1[bi * c + ch];
  else if (t == ls - 1) v = x2[bi * c + ch];
  else v = bf2f(pf[(bi * np + t - 1) * c + ch]);
  seq[i] = f2bf(v + pe[(int64_t)t * c + ch]);
}

// Same, 8 channels per thread (c % 8 == 0, fewer than 2^31 chunks): 16-B bf16 loads / stores, 32-bit
// index math (the element-wise form spends its time in 64-bit divisions: 150 us at 1280 x 51 x 768).
// Q8: the sequence written only as the combiner QKV GEMM's MX-fp8 operand (mmr::q8_chunk8 of the
// bf16-rounded values: bit-identical to quantising the bf16 sequence; rows and c multiples of 256, so
// a 4-lane group never straddles a row or the grid's ragged end).
template <bool Q8 = false>
__global__ __launch_bounds__(256) void assemble_seq8(const float* __restrict__ x1, const uint16_t* __restrict__ pf,
                                                     const float* __restrict__ x2, const float* __restrict__ pe,
                                                     uint16_t* __restrict__ seq, int nb, int np, int c,
                                                     uint8_t* __restrict__ q8 = nullptr,
                                                     uint8_t* __restrict__ q8s = nullptr) {
  const uint32_t ls = (uint32_t)np + 2u, c8 = (uint32_t)c >> 3;
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= (uint32_t)nb * ls * c8) return;
  const uint32_t row = i / c8, ch = (i - row * c8) * 8u;
  const uint32_t bi = row / ls, t = row - bi * ls;
  float v[8];
  if (t == 0 || t == ls - 1) {
    const float4* src = (const float4*)((t == 0 ? x1 : x2) + (size_t)bi * c + ch);
    const float4 a = src[0], b = src[1];
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  } else {
    const uint4 u = *(const uint4*)(pf + ((size_t)bi * np + t - 1) * c + ch);
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[2 * e] = __uint_as_float(w[e] << 16);
      v[2 * e + 1] = __uint_as_float(w[e] & 0xFFFF0000u);
    }
  }
  const float4* pp = (const float4*)(pe + (size_t)t * c + ch);
  const float4 p0 = pp[0], p1 = pp[1];
  const float pv[8] = {p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, p1.z, p1.w};
  uint4 o;
  o.x = mmr::pack2bf(v[0] + pv[0], v[1] + pv[1]);
  o.y = mmr::pack2bf(v[2] + pv[2], v[3] + pv[3]);
  o.z = mmr::pack2bf(v[4] + pv[4], v[5] + pv[5]);
  o.w = mmr::pack2bf(v[6] + pv[6], v[7] + pv[7]);
  if constexpr (Q8) {
    const uint32_t w[4] = {o.x, o.y, o.z, o.w};
    float vb[8];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      vb[2 * e] = __uint_as_float(w[e] << 16);
      vb[2 * e + 1] = __uint_as_float(w[e] & 0xFFFF0000u);
    }
    mmr::q8_chunk8(vb, (int64_t)row, (int)(ch >> 3), c, q8, q8s, true);
  } else {
    *(uint4*)(seq + (size_t)row * c + ch) = o;
  }
}

// ------------------------------------------------------------------ strided bf16 -> f32 row gather
// y[b][:] = f32(x[b*ldx + :]) — e.g. the CLS row of each text sequence (fusion.py:447 txt_p[:, 0]).
__global__ __launch_bounds__(256) void rows_to_f32(const uint16_t* __restrict__ x, int64_t ldx,
                                                   float* __restrict__ y, int nb, int c) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)nb * c) return;
  y[i] = bf2f(x[(i / c) * ldx + (i % c)]);
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

mmr_status launch_mha(const char* who, const uint16_t* q, int64_t ldq, const uint16_t* k, int64_t ldk,
                      const uint16_t* v, int64_t ldv, uint16_t* out, int64_t ldo, float* mean_out,
                      const int64_t* kmask, int32_t b, int32_t lq, int32_t lk, int32_t heads, int32_t dh,
                      float scale, void* stream, uint8_t* q8 = nullptr, uint8_t* q8s = nullptr) {
  MMR_REQUIRE(q && k && v && (out || mean_out || q8), "%s: NULL pointer", who);
  MMR_REQUIRE(!q8 || (q8s && dh % 32 == 0 && ((int64_t)b * lq) % 256 == 0 && ((int64_t)heads * dh) % 256 == 0),
              "%s: the MX-fp8 output needs head_dim %% 32 == 0, b*lq %% 256 == 0 and heads*dh %% 256 == 0", who);
  MMR_REQUIRE(b >= 0 && lq > 0 && lk > 0 && heads > 0, "%s: bad shape b=%d lq=%d lk=%d heads=%d", who, b, lq, lk,
              heads);
  MMR_REQUIRE(dh > 0 && dh % 8 == 0 && dh <= 192, "%s: head_dim %d must be a multiple of 8 <= 192", who, dh);
  MMR_REQUIRE(ldq % 8 == 0 && ldk % 8 == 0 && ldv % 8 == 0 && (!out || ldo % 4 == 0),
              "%s: row strides must be multiples of 8 elements (16 B)", who);
  MMR_REQUIRE(ldq >= (int64_t)heads * dh && ldk >= (int64_t)heads * dh && ldv >= (int64_t)heads * dh &&
              (!out || ldo >= (int64_t)heads * dh), "%s: row stride below heads*dh", who);
  MMR_REQUIRE(aligned16(q) && aligned16(k) && aligned16(v) && (!out || ((uintptr_t)out & 7u) == 0),
              "%s: operands must be 16-B aligned", who);
  if (b == 0) return MMR_OK;
  const int dt = (dh + 31) / 32;
  const int nqt = (lq + 31) / 32, nchunk = (lq + 127) / 128, nwv = std::min(4, nqt);
  // key block: all keys when lk <= 64; 64 for a 1-2-wave block (its LDS, and with it the workgroups
  // per CU, is then set by the K/V image); else 128
  int kbs = (lk <= 64 || nwv <= 2) ? 64 : MHA_KB;
  kbs = std::min(kbs, (lk + 31) & ~31);
  const size_t kv_bytes = (size_t)kbs * (dt * 32 + 8) * 2 + (size_t)kbs * (dt * 32 + ((dt & 1) ? 0 : 16)) * 2;
  const size_t lds =
      std::max(kv_bytes, (size_t)nwv * dt * 32 * 33 * 4) + (size_t)nwv * dt * 32 * 4 + (size_t)kbs * 4;
  const dim3 grid((unsigned)((int64_t)b * heads), (unsigned)nchunk), blk(64 * nwv);
  hipStream_t st = mmr::as_stream(stream);
  if (mean_out && nchunk > 1)  // query chunks accumulate their partial means
    MMR_CHECK_HIP(hipMemsetAsync(mean_out, 0, sizeof(float) * (size_t)b * heads * dh, st));
#define MMR_MHA(D)                                                                                             \
  do {                                                                                                         \
    if (kmask)                                                                                                 \
      mha_small<D, true><<<grid, blk, lds, st>>>(q, ldq, k, ldk, v, ldv, out, ldo, mean_out, kmask, lq, lk,    \
                                                 heads, dh, scale, kbs, q8, q8s);                                   \
    else                                                                                                       \
      mha_small<D, false><<<grid, blk, lds, st>>>(q, ldq, k, ldk, v, ldv, out, ldo, mean_out, nullptr, lq, lk, \
                                                  heads, dh, scale, kbs, q8, q8s);                                  \
  } while (0)
  switch (dt) {
    case 1: MMR_MHA(1); break;
    case 2: MMR_MHA(2); break;
    case 3: MMR_MHA(3); break;
    case 4: MMR_MHA(4); break;
    case 5: MMR_MHA(5); break;
    default: MMR_MHA(6); break;
  }
#undef MMR_MHA
  MMR_LAUNCH_CHECK();
  return MMR_OK;
}

}  // namespace

// ================================================================== C ABI
extern "C" {

mmr_status mmr_mha(const uint16_t* q, int64_t ldq, const uint16_t* k, int64_t ldk, const uint16_t* v,
                   int64_t ldv, uint16_t* out, int64_t ldo, float* mean_out, int32_t b, int32_t lq,
                   int32_t lk, int32_t heads, int32_t dh, float scale, void* stream) {
  mmr::clear_error();
  return launch_mha("mmr_mha", q, ldq, k, ldk, v, ldv, out, ldo, mean_out, nullptr, b, lq, lk, heads, dh, scale,
                    stream);
}

// BERT self-attention (HF BertSelfAttention, eval) on the same kernel: Q / K / V are the column
// blocks of the fused QKV rows; key padding mask01 (0 -> masked; fully masked 32-key tiles skipped)
mmr_status mmr_bert_attention(const uint16_t* qkv, const int64_t* mask01, uint16_t* ctx, int32_t b, int32_t l,
                              int32_t h, int32_t dh, void* stream) {
  mmr::clear_error();
  MMR_REQUIRE(qkv && mask01 && ctx, "mmr_bert_attention: NULL pointer");
  MMR_REQUIRE(h > 0 && dh > 0, "mmr_bert_attention: bad shape h=%d dh=%d", h, dh);
  const int64_t C = (int64_t)h * dh;
  return launch_mha("mmr_bert_attention", qkv, 3 * C, qkv + C, 3 * C, qkv + 2 * C, 3 * C, ctx, C, nullptr, mask01,
                    b, l, l, h, dh, 1.0f / sqrtf((float)dh), stream);
}

// mmr_mha with the output as the next GEMM's MX-fp8 activation operand as well (or instead: out may
// be NULL): e4m3 [b*lq][heads*dh] + E8M0 scales in the layout-0 image, bit-identical to
// mmr_quantize_mxfp8 of the bf16 rows (the fusion head's enhancer / cross-attention out-projections
// on the fp8 path)
mmr_status mmr_mha_q8(const uint16_t* q, int64_t ldq, const uint16_t* k, int64_t ldk, const uint16_t* v, int64_t ldv,
                      uint16_t* out, int64_t ldo, float* mean_out, uint8_t* q8, uint8_t* q8_scales, int32_t b,
                      int32_t lq, int32_t lk, int32_t heads, int32_t dh, float scale, void* stream) {
  mmr::clear_error();
  MMR_REQUIRE(q8 && q8_scales, "mmr_mha_q8: NULL pointer");
  return launch_mha("mmr_mha_q8", q, ldq, k, ldk, v, ldv, out, ldo, mean_out, nullptr, b, lq, lk, heads, dh, scale,
                    stream, q8, q8_scales);
}

mmr_status mmr_bert_attention_q8(const uint16_t* qkv, const int64_t* mask01, uint16_t* ctx, uint8_t* q8,
                                 uint8_t* q8_scales, int32_t b, int32_t l, int32_t h, int32_t dh, void* stream) {
  mmr::clear_error();
  MMR_REQUIRE(qkv && mask01 && q8 && q8_scales, "mmr_bert_attention_q8: NULL pointer");
  MMR_REQUIRE(h > 0 && dh > 0, "mmr_bert_attention_q8: bad shape h=%d dh=%d", h, dh);
  const int64_t C = (int64_t)h * dh;
  return launch_mha("mmr_bert_attention_q8", qkv, 3 * C, qkv + C, 3 * C, qkv + 2 * C, 3 * C, ctx, C, nullptr, mask01,
                    b, l, l, h, dh, 1.0f / sqrtf((float)dh), stream, q8, q8_scales);
}

mmr_status mmr_add_pos_bf16(const void* x, int32_t x_is_f32, const float* pos, uint16_t* y, int64_t rows,
                            int32_t l, int32_t c, void* stream) {
  mmr::clear_error();
  MMR_REQUIRE(x && pos && y && l > 0 && c > 0 && c % 8 == 0 && rows >= 0, "mmr_add_pos_bf16: bad arguments");
  if (rows == 0) return MMR_OK;
  const dim3 grid((unsigned)mmr::ceil_div(rows * (c / 8), 256));
  hipStream_t st = mmr::as_stream(stream);
  if (x_is_f32) add_pos_bf16<float><<<grid, 256, 0, st>>>((const float*)x, pos, y, rows, l, c);
  else add_pos_bf16<uint16_t><<<grid, 256, 0, st>>>((const uint16_t*)x, pos, y, rows, l, c);
  MMR_LAUNCH_CHECK();
  return MMR_OK;
}

mmr_status mmr_add_pos_bf16_q8(const void* x, int32_t x_is_f32, const float* pos, uint16_t* y, uint8_t* q8,
                               uint8_t* q8_scales, int64_t rows, int32_t l, int32_t c, void* stream) {
  mmr::clear_error();
  MMR_REQUIRE(x && pos && y && q8 && q8_scales && l > 0 && rows >= 0, "mmr_add_pos_bf16_q8: bad arguments");
  MMR_REQUIRE(rows % 256 == 0 && c > 0 && c % 256 == 0,
              "mmr_add_pos_bf16_q8: the MX-fp8 output needs rows %% 256 == 0 and c %% 256 == 0 (rows=%lld c=%d)",
              (long long)rows, c);
  if (rows == 0) return MMR_OK;
  const dim3 grid((unsigned)mmr::ceil_div(rows * (c / 8), 256));
  hipStream_t st = mmr::as_stream(stream);
  if (x_is_f32) add_pos_bf16<float, true><<<grid, 256, 0, st>>>((const float*)x, pos, y, rows, l, c, q8, q8_scales);
  else add_pos_bf16<uint16_t, true><<<grid, 256, 0, st>>>((const uint16_t*)x, pos, y, rows, l, c, q8, q8_scales);
  MMR_LAUNCH_CHECK();
  return MMR_OK;
}

mmr_status mmr_ln_rows(const void* x, int64_t ldx, const float* alpha, const void* residual, int64_t ldr,
                       const float* gamma, const float* beta, const float* post, int64_t ldp,
                       const float* post_scale, void* y, int64_t ldy, int64_t rows, int32_t c, float eps,
                       int32_t io_bf16, int32_t groups, int64_t group_div, void* stream) {
  mmr::clear_error();
  MMR_REQUIRE(x && gamma && beta && y && rows >= 0 && c > 0 && c <= 1024 && groups >= 1 && group_div >= 1,
              "mmr_ln_rows: bad arguments (c <= 1024, groups >= 1, group_div >= 1)");
  if (rows == 0) return MMR_OK;
  const dim3 grid((unsigned)mmr::ceil_div(rows, 4));
  hipStream_t st = mmr::as_stream(stream);
  // the scalar forms load ceil(c / 64) channels per lane (NI), not 16: at c = 96 / 192 the clamped
  // duplicate loads of a fixed 16 were most of the instructions
  const int ni = (c + 63) / 64;
#define LNS(TI_, NI_)                                                                                            \
  ln_rows<TI_, TI_, NI_><<<grid, 256, 0, st>>>((const TI_*)x, ldx, alpha, (const TI_*)residual, ldr, gamma, beta, \
                                               post, ldp, post_scale, (TI_*)y, ldy, rows, c, eps, groups, group_div)
#define LNS_DISPATCH(TI_)                        \
  do {                                           \
    if (ni <= 2) LNS(TI_, 2);                    \
    else if (ni <= 3) LNS(TI_, 3);               \
    else if (ni <= 4) LNS(TI_, 4);               \
    else if (ni <= 6) LNS(TI_, 6);               \
    else if (ni <= 8) LNS(TI_, 8);               \
    else if (ni <= 12) LNS(TI_, 12);             \
    else LNS(TI_, 16);                           \
  } while (0)
  if (io_bf16)
    LNS_DISPATCH(uint16_t);
  else {
    auto al = [](const void* p, int64_t ld, int vw) {
      return p == nullptr || (((uintptr_t)p & (4 * vw - 1)) == 0 && ld % vw == 0);
    };
    auto ok = [&](int vw) {
      return c % (64 * vw) == 0 && al(x, ldx, vw) && al(residual, ldr, vw) && al(post, ldp, vw) && al(y, ldy, vw) &&
             al(gamma, 0, vw) && al(beta, 0, vw);
    };
#define LNV(VW_)                                                                                                  \
  ln_rows_v<VW_><<<grid, 256, 0, st>>>((const float*)x, ldx, alpha, (const float*)residual, ldr, gamma, beta, post, \
                                       ldp, post_scale, (float*)y, ldy, rows, c, eps, groups, group_div)
#define LNSM(LPR_, PER_)                                                                                          \
  ln_rows_s<LPR_, PER_><<<dim3((unsigned)mmr::ceil_div(rows, 4 * (64 / LPR_))), 256, 0, st>>>(                  \
      (const float*)x, ldx, alpha, (const float*)residual, ldr, gamma, beta, post, ldp, post_scale, (float*)y, ldy, \
      rows, c, eps, groups, group_div)
    if (ok(4)) LNV(4);
    else if (ok(2)) LNV(2);
    else if (c <= 128) LNSM(16, 8);
    else if (c <= 256) LNSM(32, 8);
    else LNS_DISPATCH(float);
#undef LNSM
#undef LNV
  }
#undef LNS_DISPATCH
#undef LNS
  MMR_LAUNCH_CHECK();
  return MMR_OK;
}

mmr_status mmr_ln_rows_split(const float* x, int64_t ldx, const float* alpha, const float* residual, int64_t ldr,
                             const float* gamma,
                             const float* beta, float* y, int64_t ldy, uint16_t* xs, int64_t rows, int32_t c, float eps,
                             void* stream) {
  mmr::clear_error();
  MMR_REQUIRE(x && gamma && beta && xs && rows >= 0 && c > 0 && c % 4 == 0 && c <= 1024,
              "mmr_ln_rows_split: bad arguments (c %% 4 == 0, c <= 1024; rows=%lld c=%d)", (long long)rows, c);
  auto al = [](const void* p, int64_t ld) { return p == nullptr || (((uintptr_t)p & 15) == 0 && ld % 4 == 0); };
  MMR_REQUIRE(al(x, ldx) && al(residual, ldr) && al(y, ldy) && al(gamma, 0) && al(beta, 0) && al(xs, 0),
              "mmr_ln_rows_split: rows / parameters must be 16-B aligned (row strides multiples of 4)");
  if (rows == 0) return MMR_OK;
  const int nch = (c + 127) / 128;
  const dim3 grid((unsigned)mmr::ceil_div(rows, 8));
  hipStream_t st = mmr::as_stream(stream);
#define LNSP(N_) \
  ln_rows_split<N_><<<grid, 256, 0, st>>>(x, ldx, alpha, residual, ldr, gamma, beta, y, ldy, xs, rows, c, eps)
  switch (nch) {
    case 1: LNSP(1); break;
    case 2: LNSP(2); break;
    case 3: LNSP(3); break;
    case 4: LNSP(4); break;
    case 5: LNSP(5); break;
    case 6: LNSP(6); break;
    case 7: LNSP(7); break;
    default: LNSP(8); break;
  }
#undef LNSP
  MMR_LAUNCH_CHECK();
  return MMR_OK;
}

mmr_status mmr_assemble_seq(const float* x1, const uint16_t* patches_fused, const float* x2, const float* pe,
                            uint16_t* seq, int32_t b, int32_t np, int32_t c, void* stream) {
  mmr::clear_error();
  MMR_REQUIRE(x1 && patches_fused && x2 && pe && seq && b >= 0 && np > 0 && c > 0, "mmr_assemble_seq: bad arguments");
  if (b == 0) return MMR_OK;
  const int64_t n = (int64_t)b * (np + 2) * c;
  const bool vec = c % 8 == 0 && n / 8 < (int64_t(1) << 31) && aligned16(x1) && aligned16(x2) && aligned16(pe) &&
                   aligned16(patches_fused) && aligned16(seq);
  if (vec)
    assemble_seq8<false><<<dim3((unsigned)mmr::ceil_div(n / 8, 256)), 256, 0, mmr::as_stream(stream)>>>(
        x1, patches_fused, x2, pe, seq, b, np, c);
  else
    assemble_seq<<<dim3((unsigned)mmr::ceil_div(n, 256)), 256, 0, mmr::as_stream(stream)>>>(x1, patches_fused, x2, pe,
                                                                                            seq, b, np, c);
  MMR_LAUNCH_CHECK();
  return MMR_OK;
}

mmr_status mmr_assemble_seq_q8(const float* x1, const uint16_t* patches_fused, const float* x2, const float* pe,
                               uint8_t* q8, uint8_t* q8_scales, int32_t b, int32_t np, int32_t c, void* stream) {
  mmr::clear_error();
  MMR_REQUIRE(x1 && patches_fused && x2 && pe && q8 && q8_scales && b >= 0 && np > 0 && c > 0,
              "mmr_assemble_seq_q8: bad arguments");
  const int64_t rows = (int64_t)b * (np + 2), n = rows * c;
  MMR_REQUIRE(rows % 256 == 0 && c % 256 == 0 && n / 8 < (int64_t(1) << 31),
              "mmr_assemble_seq_q8: needs b*(np+2) %% 256 == 0 and c %% 256 == 0 (rows=%lld c=%d)", (long long)rows, c);
  MMR_REQUIRE(aligned16(x1) && aligned16(x2) && aligned16(pe) && aligned16(patches_fused),
              "mmr_assemble_seq_q8: operands must be 16-B aligned");
  if (b == 0) return MMR_OK;
  assemble_seq8<true><<<dim3((unsigned)mmr::ceil_div(n / 8, 256)), 256, 0, mmr::as_stream(stream)>>>(
      x1, patches_fused, x2, pe, nullptr, b, np, c, q8, q8_scales);
  MMR_LAUNCH_CHECK();
  return MMR_OK;
}

mmr_status mmr_rows_to_f32(const uint16_t* x, int64_t ldx, float* y, int32_t b, int32_t c, void* stream) {
  mmr::clear_error();
  MMR_REQUIRE(x && y && b >= 0 && c > 0 && ldx >= c, "mmr_rows_to_f32: bad arguments");
  if (b == 0) return MMR_OK;
  rows_to_f32<<<dim3((unsigned)mmr::ceil_div((int64_t)b * c, 256)), 256, 0, mmr::as_stream(stream)>>>(x, ldx, y, b, c);
  MMR_LAUNCH_CHECK();
  return MMR_OK;
}

}  // extern "C"
