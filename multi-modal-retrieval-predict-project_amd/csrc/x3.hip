// fp32-faithful tower mode ("x3", Backbones(tower_dtype="x3")): the Swin / BERT towers and the
// multimodal head with f32 activations between kernels and every contraction (linears and both
// attention products) on bf16 MFMA with three-term splits: a = a_hi + a_lo (a_hi = bf16(a),
// a_lo = bf16(a - a_hi), |a - a_hi - a_lo| <= 2^-18 |a|), a.b ~= a_hi.b_hi + a_hi.b_lo + a_lo.b_hi
// summed in f32 (~2^-17 relative per product, f32 accumulation).  Everything else — LayerNorm,
// softmax, GELU, means — runs in f32 as torch does (the softmax's exp by mmr::exp_acc and the GELU's erf
// by Abramowitz-Stegun 7.1.26: a few f32 ulp, far below the products' 2^-17).  The reference runs these towers
// in fp32 (src/Model/fusion.py:198-199 timm forward_features, :322-325 BertModel, model.py:365-479
// heads); this mode exists so the end-to-end lists can be held to BASELINE.md §3's bar (identical
// top-K up to 1e-6 ties, scores within 1e-4, identical P@10) — the bf16 / MX-fp8 tower modes move
// embeddings by ~1e-3 and reorder near-ties.
//
// Kernels:
//   x3_gemm        Y = act(X W^T + bias) (+ R), X f32 split in registers while staged to LDS, W
//                  pre-split (hi / lo bf16 copies made once at load); 128 x 128 tiles, 4 waves of
//                  64 x 64, K-steps of 32 on v_mfma_f32_16x16x32_bf16 (3 per fragment pair),
//                  register-prefetched next K-step, XCD-contiguous tile order.
//   x3_attention   per (sequence or window, head): softmax(q k^T * scale + bias / mask) v, keys in
//                  LDS chunks of 64 (hi / lo K rows, hi / lo V^T), online softmax (running max and
//                  sum per query row, f32 exp), P re-split through a wave-private LDS tile; optional
//                  mean over the query rows (fixed-order reduction, deterministic).  Modes: strided
//                  rows (nn.MultiheadAttention, BERT with a key-padding mask) and Swin windows (the
//                  roll + window partition / reverse folded into the token index map, the dense
//                  rel-pos + shift-mask bias of mmr_swin_attn_bias).
//   small f32 kernels: patch im2col, PatchMerging gather + LN(4C), BERT embeddings + LN, add-pos,
//                  fused-sequence assembly, row means, row gather.
#include <float.h>

#include "common.h"

namespace {

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

// f32 x4 -> (hi, lo) bf16 x4 each, packed as two dwords
__device__ __forceinline__ void split4(const float4 v, uint2& hi, uint2& lo) {
  const uint32_t h0 = mmr::pack2bf(v.x, v.y), h1 = mmr::pack2bf(v.z, v.w);
  const float r0 = v.x - __uint_as_float(h0 << 16), r1 = v.y - __uint_as_float(h0 & 0xFFFF0000u);
  const float r2 = v.z - __uint_as_float(h1 << 16), r3 = v.w - __uint_as_float(h1 & 0xFFFF0000u);
  hi = make_uint2(h0, h1);
  lo = make_uint2(mmr::pack2bf(r0, r1), mmr::pack2bf(r2, r3));
}

__device__ __forceinline__ void split8(const float4 a, const float4 b, bf16x8& hi, bf16x8& lo) {
  uint2 h0, l0, h1, l1;
  split4(a, h0, l0);
  split4(b, h1, l1);
  hi = __builtin_bit_cast(bf16x8, make_uint4(h0.x, h0.y, h1.x, h1.y));
  lo = __builtin_bit_cast(bf16x8, make_uint4(l0.x, l0.y, l1.x, l1.y));
}

__device__ __forceinline__ f32x4 mfma3(const bf16x8 ah, const bf16x8 al, const bf16x8 bh, const bf16x8 bl, f32x4 acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, acc, 0, 0, 0);
}

// GELU (erf form, as torch) with erf by Abramowitz-Stegun 7.1.26 (|err| <= 1.5e-7, mmr::gelu_erf): 100x below
// the bf16x3 products' 2^-17, branch-free (ocml erff made the GEMM epilogues VALU-heavy)
__device__ __forceinline__ float gelu_exact(float x) { return mmr::gelu_erf(x); }

// ------------------------------------------------------------------ GEMM
constexpr int GX_BM = 128, GX_BN = 128, GX_BK = 32, GX_LD = 40;  // LDS row stride 80 B: conflict-free 16-B reads

template <int ACT, bool BIAS, bool RES>
__global__ __launch_bounds__(256, 2) void x3_gemm(const float* __restrict__ X, int64_t ldx,
                                                  const uint16_t* __restrict__ Wh, const uint16_t* __restrict__ Wl,
                                                  const float* __restrict__ bias, const float* R, int64_t ldr,
                                                  float* Y, int64_t ldy, int M, int N, int K, int tiles_n,
                                                  int ntiles) {
  __shared__ __attribute__((aligned(16))) uint16_t sAh[GX_BM * GX_LD], sAl[GX_BM * GX_LD];
  __shared__ __attribute__((aligned(16))) uint16_t sBh[GX_BN * GX_LD], sBl[GX_BN * GX_LD];
  const int tile = mmr::xcd_contiguous((int)blockIdx.x, ntiles);
  const int tm = tile / tiles_n, tn = tile % tiles_n;
  const int m0 = tm * GX_BM, n0 = tn * GX_BN;
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
  const int wm = wave >> 1, wn = wave & 1;
  const int r = lane & 15, g = lane >> 4;
  // staging: thread -> (row t / 2, 16 k from 16 (t % 2)); rows past M / N clamped (loaded, never stored)
  const int srow = t >> 1, sk = (t & 1) * 16;
  const int xr = m0 + srow < M ? m0 + srow : M - 1, wr = n0 + srow < N ? n0 + srow : N - 1;
  const float* xp = X + (int64_t)xr * ldx + sk;
  const uint16_t* whp = Wh + (int64_t)wr * K + sk;
  const uint16_t* wlp = Wl + (int64_t)wr * K + sk;
  float4 xv[4];
  uint4 wv[4];
  auto gload = [&](int k0) {
#pragma unroll
    for (int j = 0; j < 4; ++j) xv[j] = *(const float4*)(xp + k0 + 4 * j);
    wv[0] = *(const uint4*)(whp + k0);
    wv[1] = *(const uint4*)(whp + k0 + 8);
    wv[2] = *(const uint4*)(wlp + k0);
    wv[3] = *(const uint4*)(wlp + k0 + 8);
  };
  f32x4 acc[4][4];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[m][n] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const int nk = K / GX_BK;
  gload(0);
  for (int kt = 0; kt < nk; ++kt) {
    __syncthreads();  // every wave done reading the previous K-step
    {
      uint2 h[4], l[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) split4(xv[j], h[j], l[j]);
      uint16_t* ah = sAh + srow * GX_LD + sk;
      uint16_t* al = sAl + srow * GX_LD + sk;
      *(uint4*)ah = make_uint4(h[0].x, h[0].y, h[1].x, h[1].y);
      *(uint4*)(ah + 8) = make_uint4(h[2].x, h[2].y, h[3].x, h[3].y);
      *(uint4*)al = make_uint4(l[0].x, l[0].y, l[1].x, l[1].y);
      *(uint4*)(al + 8) = make_uint4(l[2].x, l[2].y, l[3].x, l[3].y);
      *(uint4*)(sBh + srow * GX_LD + sk) = wv[0];
      *(uint4*)(sBh + srow * GX_LD + sk + 8) = wv[1];
      *(uint4*)(sBl + srow * GX_LD + sk) = wv[2];
      *(uint4*)(sBl + srow * GX_LD + sk + 8) = wv[3];
    }
    __syncthreads();
    if (kt + 1 < nk) gload((kt + 1) * GX_BK);  // next K-step in flight under this one's MFMAs
    bf16x8 bh[4], bl[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const int row = wn * 64 + 16 * n + r;
      bh[n] = *(const bf16x8*)(sBh + row * GX_LD + 8 * g);
      bl[n] = *(const bf16x8*)(sBl + row * GX_LD + 8 * g);
    }
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int row = wm * 64 + 16 * m + r;
      const bf16x8 ah = *(const bf16x8*)(sAh + row * GX_LD + 8 * g);
      const bf16x8 al = *(const bf16x8*)(sAl + row * GX_LD + 8 * g);
#pragma unroll
      for (int n = 0; n < 4; ++n) acc[m][n] = mfma3(ah, al, bh[n], bl[n], acc[m][n]);
    }
  }
  // lane (r, g): rows 16 m + 4 g + i, column 16 n + r of the wave's 64 x 64 block
#pragma unroll
  for (int n = 0; n < 4; ++n) {
    const int col = n0 + wn * 64 + 16 * n + r;
    if (col >= N) continue;
    const float bv = BIAS ? bias[col] : 0.f;
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = m0 + wm * 64 + 16 * m + 4 * g + i;
        if (row >= M) continue;
        float v = acc[m][n][i];
        if (BIAS) v += bv;
        if (ACT == 1) v = gelu_exact(v);
        if (RES) v += R[(int64_t)row * ldr + col];
        Y[(int64_t)row * ldy + col] = v;
      }
  }
}

// ------------------------------------------------------------------ attention
struct AttnArgs {
  const float* q;
  int64_t ldq;
  const float* k;
  int64_t ldk;
  const float* v;
  int64_t ldv;
  float* out;
  int64_t ldo;
  float* mean_out;
  const int64_t* kmask;
  const float* bias;  // Swin: [types][heads][64][64]
  int lq, lk, heads, dh;
  float scale;
  int hw, ws, shift;  // Swin windows
  uint16_t* xs;       // non-NULL: the output as the x3 split GEMM's operand rows [hi | lo] (2 kp wide)
  int kp;             //   instead of out; columns heads*dh .. kp written zero by the last head
};

// ------------------------------------------------------------------ attention, round 5 (x3_mha)
// The bf16 core's structure (fusion.hip mha_small) on bf16x3 operands.  Block = (sequence or window,
// head); nwv = min(4, ceil(lq / 32)) waves, one 32-query tile per wave, the block walking its query
// chunks of 32 nwv rows (one chunk up to lq = 128; the mean then reduces in a fixed order inside the
// block).  S^T = K . Q^T on v_mfma_f32_32x32x16_bf16 as Kh.Qh + Kh.Ql + Kl.Qh puts the query on the
// lane: the softmax (f32, mmr::exp_acc, online over 64-key sub-blocks of kbs-key staged blocks) stays in
// registers, and P^T is split in registers into the B operands of O^T += V^T . P^T (Vh.Ph + Vh.Pl +
// Vl.Ph), V^T read from key-major hi / lo images by ds_read_b64_tr_b16 in P^T's key permutation.
// K / V f32 rows are split ONCE per block while staged (16-B LDS writes), Q once per wave in registers.
// (The round-4 kernel ran 16-query tiles on 16x16x32 MFMAs with P re-split through LDS by 2-byte stores
// and V^T written by 2-byte transposing stores: 0.06 of the bf16 MFMA peak; BERT 176 -> 119 us, Swin
// stage 1 552 -> 444 us, profiles/r05_x3_attn_ab.txt.)
// MODE 0: plain (nn.MultiheadAttention); 1: key-padding mask as HF's additive finfo.min (a row with
// every key masked -> HF's uniform softmax, the mean of V over the lk keys); 2: Swin windows (roll /
// partition folded into the token map, q pre-scaled as timm, rel-pos + shift-mask bias added).
template <int DT, int MODE, bool SINGLE>
__global__ __launch_bounds__(256, DT <= 2 ? 3 : 2) void x3_mha(const AttnArgs a, int kbs) {
  constexpr int DHP = DT * 32, KS = DHP / 16, KROW = DHP + 8, VROW = DHP + ((DT & 1) ? 0 : 16);
  constexpr int C8 = DHP / 8, OROW = DHP + 4;
  // 32-key tiles per online-softmax step: 2 at DT = 1 (Swin); 1 at DT >= 2, so the S / P registers fit 3
  // waves per SIMD at DT = 2 (an extra O rescale per 32 keys: one rounding, far below the products' 2^-17)
  constexpr int TPS = DT >= 2 ? 1 : 2;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, nthr = blockDim.x, lane = tid & 63, wave = tid >> 6, nwv = nthr >> 6;
  uint16_t* Kh = (uint16_t*)smem;  // [kbs][KROW]
  uint16_t* Kl = Kh + kbs * KROW;
  uint16_t* Vh = Kl + kbs * KROW;  // [kbs][VROW], key-major
  uint16_t* Vl = Vh + kbs * VROW;
  const int kv_bytes = kbs * (KROW + VROW) * 4, epi_bytes = nwv * 32 * OROW * 4;
  float* msum = (float*)(smem + (kv_bytes > epi_bytes ? kv_bytes : epi_bytes));  // [nwv][DHP]
  float* madd = msum + nwv * DHP;                                                  // [kbs] (MODE 1)
  int64_t* tokt = (int64_t*)(madd + kbs);  // [64] (MODE 2): the window's token rows (roll / partition map)
  const int unit = mmr::xcd_contiguous((int)blockIdx.x, (int)gridDim.x);
  const int head = unit % a.heads;
  const int64_t bb = unit / a.heads;
  const int lq = a.lq, lk = a.lk, dh = a.dh;
  int64_t sw_base = 0;
  int wy = 0, wx = 0, type = 0;
  if constexpr (MODE == 2) {
    const int nwin1 = a.hw / a.ws, nwin = nwin1 * nwin1;
    const int win = (int)(bb % nwin);
    sw_base = (bb / nwin) * (int64_t)a.hw * a.hw;
    wy = win / nwin1;
    wx = win % nwin1;
    type = a.shift > 0 ? ((wy == nwin1 - 1) ? 2 : 0) + ((wx == nwin1 - 1) ? 1 : 0) : 0;
  }
  // MODE 2: the token map (runtime divisions by ws / hw: ~40 VALU each) computed once per block into LDS
  if constexpr (MODE == 2) {
    for (int i = tid; i < 64; i += nthr) {
      const int ii = i < lq ? i : lq - 1;
      const int hr = wy * a.ws + ii / a.ws, wr = wx * a.ws + ii % a.ws;
      tokt[i] = sw_base + (int64_t)((hr + a.shift) % a.hw) * a.hw + (wr + a.shift) % a.hw;
    }
    __syncthreads();
  }
  auto qtok = [&](int i) -> int64_t {
    if constexpr (MODE == 2) return tokt[i];
    else return bb * lq + i;
  };
  auto ktok = [&](int j) -> int64_t {
    if constexpr (MODE == 2) return qtok(j);
    else return bb * lk + j;
  };
  const float* qb = a.q + head * dh;
  const float* kb = a.k + head * dh;
  const float* vb = a.v + head * dh;
  const int r = lane & 31, hf = lane >> 5;
  const int lkp = (lk + 31) & ~31;
  // MODE 1: a sequence with no unmasked key keeps every key tile (uniform softmax, as HF)
  bool anyv = true;
  if constexpr (MODE == 1) {
    int f = 0;
    for (int j = tid; j < lk; j += nthr) f |= a.kmask[bb * lk + j] != 0;
    anyv = __syncthreads_or(f) != 0;
  }
  if (a.mean_out)
    for (int d = lane; d < DHP; d += 64) msum[wave * DHP + d] = 0.f;

  // kn keys from k0 (kn % 32 == 0): f32 rows -> hi / lo images, 8 elements per chunk, 4 chunks per
  // thread in flight (keys past lk / columns past dh read a clamped in-bounds chunk; columns past dh
  // are zeroed, keys past lk are -inf in the scores)
  auto stage = [&](int k0, int kn) {
    // chunks in flight per thread: a block's staging is UB-deep rounds of HBM round trips (dh 96 at 128
    // threads: 12 chunks per thread, 6 rounds at UB = 2, 2 at 6); the registers come within each
    // instantiation's occupancy (fusion combiner 236 -> 218 us, profiles/r05_x3_attn_ub_ab.txt; 4 at dh 128,
    // whose 6 spilled once the first block's stage holds the raw Q rows)
    constexpr int UB = DT == 3 ? 6 : 4;
    const int nch = kn * C8, tot = 2 * nch;
    for (int e0 = tid; e0 < tot; e0 += UB * nthr) {
      float4 xa[UB], xb[UB];
#pragma unroll
      for (int u = 0; u < UB; ++u) {
        const int e = e0 + u * nthr < tot ? e0 + u * nthr : 0;
        const bool isv = e >= nch;
        const int e2 = isv ? e - nch : e;
        const int key = e2 / C8, d = (e2 % C8) * 8;
        const int j = k0 + key < lk ? k0 + key : lk - 1;
        const float* src = (isv ? vb + ktok(j) * a.ldv : kb + ktok(j) * a.ldk) + (d < dh ? d : 0);
        xa[u] = *(const float4*)src;
        xb[u] = *(const float4*)(src + 4);
      }
#pragma unroll
      for (int u = 0; u < UB; ++u) {
        const int e = e0 + u * nthr;
        if (e < tot) {
          const bool isv = e >= nch;
          const int e2 = isv ? e - nch : e;
          const int key = e2 / C8, d = (e2 % C8) * 8;
          if (d >= dh) xa[u] = xb[u] = make_float4(0.f, 0.f, 0.f, 0.f);
          bf16x8 h, l;
          split8(xa[u], xb[u], h, l);
          // integer offsets from the one LDS base, not a select between image pointers: at UB = 4 hipcc
          // kept {Kh, Vh} / {Kl, Vl} as generic pointer tables in scratch, and every image access of
          // the kernel became a flat op (the score loop's Kl reads then waited vmcnt(0))
          const int hoff = isv ? 2 * kbs * KROW + key * VROW + d : key * KROW + d;
          const int loff = hoff + (isv ? kbs * VROW : kbs * KROW);
          *(bf16x8*)(Kh + hoff) = h;
          *(bf16x8*)(Kh + loff) = l;
        }
      }
    }
    if constexpr (MODE == 1)
      for (int i = tid; i < kn; i += nthr) {
        const int key = k0 + i;
        madd[i] = key >= lk ? -INFINITY : (a.kmask[bb * lk + key] != 0 ? 0.f : -FLT_MAX);
      }
  };

  const int grp = lane >> 4, tq = (lane >> 2) & 3, tp = lane & 3;
  for (int qc = 0; qc < lq; qc += 32 * nwv) {
    const int q0 = qc + wave * 32;
    const bool active = q0 < lq;  // wave-uniform
    const int qi = q0 + r < lq ? q0 + r : lq - 1;
    // Q^T fragments: lane (query r, half hf) holds d = 16 ks + 8 hf .. + 7, split in registers.  The
    // raw rows are held until the first key block is staged, so the Q and K / V loads are in flight
    // together (split first, the Q load's round trip preceded the stage's): Swin stage 1 371 -> 353 us,
    // stage 2 204 -> 192, stage 3 110 -> 100 (profiles/r05_x3_attn_qlate_ab.txt); the first block's
    // stage is peeled out of the key loop, so the raw rows are dead before any compute
    bf16x8 qh[KS], ql[KS];
    {
      float4 qx[KS][2];
      const float* qrow = qb + qtok(qi) * a.ldq;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const int d = 16 * ks + 8 * hf;
        qx[ks][0] = *(const float4*)(qrow + (d < dh ? d : 0));
        qx[ks][1] = *(const float4*)(qrow + (d < dh ? d : 0) + 4);
      }
      __syncthreads();  // the previous query chunk's epilogue done with the LDS
      stage(0, min(kbs, lkp));
      __syncthreads();
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        float4 x0 = qx[ks][0], x1 = qx[ks][1];
        if (16 * ks + 8 * hf >= dh) x0 = x1 = make_float4(0.f, 0.f, 0.f, 0.f);
        if constexpr (MODE == 2) {  // timm scales q before q k^T
          x0 = make_float4(x0.x * a.scale, x0.y * a.scale, x0.z * a.scale, x0.w * a.scale);
          x1 = make_float4(x1.x * a.scale, x1.y * a.scale, x1.z * a.scale, x1.w * a.scale);
        }
        split8(x0, x1, qh[ks], ql[ks]);
      }
    }
    f32x16 o[DT];
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) o[dt] = (f32x16){0};
    float m_run = -INFINITY, l_run = 0.f;
    for (int k0 = 0; k0 < (SINGLE ? 1 : lkp); k0 += kbs) {  // SINGLE: one block, a loop hipcc removes
      const int kn = min(kbs, lkp - k0);
      if (k0 > 0) {
        __syncthreads();  // previous key block done with the LDS
        stage(k0, kn);
        __syncthreads();
      }
      if (!active) continue;
      for (int kb0 = 0; kb0 < kn; kb0 += 32 * TPS) {
        const int nt = min(32 * TPS, kn - kb0) / 32;
        bool live[TPS];
#pragma unroll
        for (int t = 0; t < TPS; ++t) {
          live[t] = t < nt;
          // fully masked 32-key tiles contribute exactly 0 once the row has an unmasked key
          if (MODE == 1 && live[t] && anyv) live[t] = __ballot(madd[kb0 + t * 32 + r] == 0.f) != 0;
        }
        f32x16 s[TPS];
#pragma unroll
        for (int t = 0; t < TPS; ++t) {
          s[t] = (f32x16){0};
          if (live[t]) {
            const int key = kb0 + t * 32 + r;
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
              const bf16x8 kh = *(const bf16x8*)(Kh + key * KROW + 16 * ks + 8 * hf);
              const bf16x8 kl = *(const bf16x8*)(Kl + key * KROW + 16 * ks + 8 * hf);
              s[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kh, qh[ks], s[t], 0, 0, 0);
              s[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kh, ql[ks], s[t], 0, 0, 0);
              s[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kl, qh[ks], s[t], 0, 0, 0);
            }
          }
        }
        // scores (lane: query r; register rg: key kb0 + 32 t + (rg & 3) + 8 (rg >> 2) + 4 hf)
        float mloc = -INFINITY;
#pragma unroll
        for (int t = 0; t < TPS; ++t) {
          if (!live[t]) continue;
#pragma unroll
          for (int g4 = 0; g4 < 4; ++g4) {
            const int kl0 = kb0 + t * 32 + 8 * g4 + 4 * hf;  // local key of register 4 g4
            float4 add = make_float4(0.f, 0.f, 0.f, 0.f);
            if constexpr (MODE == 1) add = *(const float4*)(madd + kl0);
            if constexpr (MODE == 2) {
              const int kc = k0 + kl0 < 64 ? k0 + kl0 : 60;
              add = *(const float4*)(a.bias + (((int64_t)type * a.heads + head) * 64 + (qi < 64 ? qi : 63)) * 64 + kc);
            }
            const float ad[4] = {add.x, add.y, add.z, add.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              float x = s[t][4 * g4 + e];
              if constexpr (MODE == 2) x += ad[e];
              else x = x * a.scale + ad[e];
              if (MODE != 1 && k0 + kl0 + e >= lk) x = -INFINITY;
              s[t][4 * g4 + e] = x;
              mloc = fmaxf(mloc, x);
            }
          }
        }
        mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
        const float m_new = fmaxf(m_run, mloc);
        const float alpha = m_run == -INFINITY ? 0.f : mmr::exp_acc(m_run - m_new);
        m_run = m_new;
        float psum = 0.f;
#pragma unroll
        for (int t = 0; t < TPS; ++t) {
          if (!live[t]) continue;
#pragma unroll
          for (int rg = 0; rg < 16; ++rg) {
            const float x = s[t][rg];
            const float p = (x == -INFINITY || m_new == -INFINITY) ? 0.f : mmr::exp_acc(x - m_new);
            s[t][rg] = p;
            psum += p;
          }
        }
        l_run = l_run * alpha + psum;
        if (k0 + kb0 > 0) {
#pragma unroll
          for (int dt = 0; dt < DT; ++dt) o[dt] *= alpha;
        }
        // O^T[d][q] += V^T[d][key] . P^T[key][q] (three products), P^T split in registers
#pragma unroll
        for (int t = 0; t < TPS; ++t) {
          if (!live[t]) continue;
#pragma unroll
          for (int sidx = 0; sidx < 2; ++sidx) {
            uint32_t ph[4], pl[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const float v0 = s[t][8 * sidx + 2 * j], v1 = s[t][8 * sidx + 2 * j + 1];
              ph[j] = mmr::pack2bf(v0, v1);
              pl[j] = mmr::pack2bf(v0 - __uint_as_float(ph[j] << 16), v1 - __uint_as_float(ph[j] & 0xFFFF0000u));
            }
            const bf16x8 pfh = __builtin_bit_cast(bf16x8, make_uint4(ph[0], ph[1], ph[2], ph[3]));
            const bf16x8 pfl = __builtin_bit_cast(bf16x8, make_uint4(pl[0], pl[1], pl[2], pl[3]));
            const int r0 = kb0 + t * 32 + 16 * sidx + 4 * (grp >> 1);
#pragma unroll
            for (int dt = 0; dt < DT; ++dt) {
              const int off = (r0 + tq) * VROW + dt * 32 + (grp & 1) * 16 + 4 * tp;
              const bf16x4 h0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(Vh + off));
              const bf16x4 h1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(Vh + off + 8 * VROW));
              const bf16x4 l0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(Vl + off));
              const bf16x4 l1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(Vl + off + 8 * VROW));
              const bf16x8 vfh = {h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
              const bf16x8 vfl = {l0[0], l0[1], l0[2], l0[3], l1[0], l1[1], l1[2], l1[3]};
              o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vfh, pfh, o[dt], 0, 0, 0);
              o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vfh, pfl, o[dt], 0, 0, 0);
              o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vfl, pfh, o[dt], 0, 0, 0);
            }
          }
        }
      }
    }
    // epilogue: the wave's O tile (f32, / l) staged [32 q][OROW] over the K / V image, then written as
    // row chunks (f32 rows and / or the split operand rows [hi | lo]) and summed for the mean
    __syncthreads();
    if (active) {
      float* st = (float*)smem + wave * 32 * OROW;
      const float inv = 1.0f / (l_run + __shfl_xor(l_run, 32, 64));
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4)
          *(float4*)(st + r * OROW + dt * 32 + 8 * g4 + 4 * hf) =
              make_float4(o[dt][4 * g4] * inv, o[dt][4 * g4 + 1] * inv, o[dt][4 * g4 + 2] * inv, o[dt][4 * g4 + 3] * inv);
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's LDS writes landed
      __builtin_amdgcn_wave_barrier();
      // lane -> (row lr + rpi j, 4-column chunk lc): the divisions once per lane, not per chunk
      const int nc4 = dh / 4, rpi = 64 / nc4, lr = lane / nc4, lc = lane - lr * nc4;
      if ((a.out != nullptr || a.xs != nullptr) && lr < rpi)
        for (int row = lr; row < 32; row += rpi) {
          const int ch = lc;
          if (q0 + row >= lq) break;
          const float4 v = *(const float4*)(st + row * OROW + 4 * ch);
          const int64_t tk = qtok(q0 + row);
          if (a.xs != nullptr) {
            uint2 h, l;
            split4(v, h, l);
            uint16_t* xr = a.xs + tk * 2 * a.kp + head * dh + 4 * ch;
            *(uint2*)xr = h;
            *(uint2*)(xr + a.kp) = l;
          } else {
            *(float4*)(a.out + tk * a.ldo + head * dh + 4 * ch) = v;
          }
        }
      if (a.xs != nullptr && head == a.heads - 1) {  // zero columns heads*dh .. kp of these rows
        const int z0 = a.heads * dh, nz4 = (a.kp - z0) / 4;
        for (int c = lane; c < 32 * nz4; c += 64) {
          const int row = c / nz4, ch = c - row * nz4;
          if (q0 + row >= lq) continue;
          uint16_t* xr = a.xs + qtok(q0 + row) * 2 * a.kp + z0 + 4 * ch;
          *(uint2*)xr = make_uint2(0u, 0u);
          *(uint2*)(xr + a.kp) = make_uint2(0u, 0u);
        }
      }
      if (a.mean_out != nullptr)
        for (int d = lane; d < DHP; d += 64) {
          float acc = msum[wave * DHP + d];
          for (int row = 0; row < 32; ++row)
            if (q0 + row < lq) acc += st[row * OROW + d];
          msum[wave * DHP + d] = acc;
        }
    }
  }
  if (a.mean_out != nullptr) {
    __syncthreads();
    for (int d = tid; d < dh; d += nthr) {
      float sm = 0.f;
      for (int w = 0; w < nwv; ++w) sm += msum[w * DHP + d];  // fixed order: deterministic
      a.mean_out[bb * (int64_t)a.heads * dh + head * dh + d] = sm / lq;
    }
  }
}

// ------------------------------------------------------------------ small f32 kernels
// im2col of the patch-embed conv: (b, cin, hw, hw) -> (b * g * g, kp) f32, k = c p^2 + ky p + kx,
// zero for k >= cin p^2
__global__ __launch_bounds__(256) void x3_im2col(const float* __restrict__ img, float* __restrict__ cols, int64_t ntok,
                                                 int cin, int hw, int patch, int kp) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= ntok * kp) return;
  const int64_t tk = idx / kp;
  const int k = (int)(idx % kp);
  const int gg = hw / patch;
  const int64_t bi = tk / (gg * gg);
  const int py = (int)((tk / gg) % gg), px = (int)(tk % gg);
  float val = 0.f;
  if (k < cin * patch * patch) {
    const int c = k / (patch * patch), ky = (k / patch) % patch, kx = k % patch;
    val = img[((bi * cin + c) * hw + (py * patch + ky)) * (int64_t)hw + px * patch + kx];
  }
  cols[idx] = val;
}

// One wave per merged row: gather [x(2i,2j), x(2i+1,2j), x(2i,2j+1), x(2i+1,2j+1)] (timm order),
// LayerNorm over 4c (two-pass, centred), f32 out.  4c <= 4096.
__global__ __launch_bounds__(256) void x3_patch_merge_ln(const float* __restrict__ x, const float* __restrict__ gm,
                                                         const float* __restrict__ bt, float* __restrict__ y,
                                                         int64_t nout, int hw, int c, float eps) {
  const int64_t o = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (o >= nout) return;
  const int h2 = hw / 2;
  const int64_t bi = o / (h2 * h2);
  const int i = (int)((o / h2) % h2), j = (int)(o % h2);
  const int c4 = 4 * c;
  float v[64];
  float s = 0.f;
#pragma unroll
  for (int e = 0; e < 64; ++e) {
    const int k = lane + 64 * e;
    v[e] = 0.f;
    if (k < c4) {
      const int p = k / c, off = k % c;
      const int yy = 2 * i + (p & 1), xx = 2 * j + (p >> 1);
      v[e] = x[((bi * hw + yy) * hw + xx) * (int64_t)c + off];
      s += v[e];
    }
  }
  const float mean = mmr::wave_sum(s) / c4;
  float ss = 0.f;
#pragma unroll
  for (int e = 0; e < 64; ++e)
    if (lane + 64 * e < c4) ss += (v[e] - mean) * (v[e] - mean);
  const float rstd = 1.0f / sqrtf(mmr::wave_sum(ss) / c4 + eps);
#pragma unroll
  for (int e = 0; e < 64; ++e) {
    const int k = lane + 64 * e;
    if (k < c4) y[o * c4 + k] = (v[e] - mean) * rstd * gm[k] + bt[k];
  }
}

// The same for c % 4 == 0, by 16-B chunks: lane takes chunks lane + 64 e (e < NCH) of the 4c-wide
// merged row (a chunk never straddles two source pixels); writes the f32 row to y and / or the x3
// split GEMM's [hi | lo] operand row to xs (2 kp wide, zero columns 4c..kp) — the reduction linear
// then skips its split pass.  (The scalar form above spent 64 unrolled element slots and an integer
// division per element on every lane: ~4x its bytes' time.)
template <int NCH>
__global__ __launch_bounds__(256) void x3_patch_merge_ln_v(const float* __restrict__ x, const float* __restrict__ gm,
                                                           const float* __restrict__ bt, float* __restrict__ y,
                                                           uint16_t* __restrict__ xs, int kp, int64_t nout, int hw,
                                                           int c, float eps) {
  const int64_t o = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (o >= nout) return;  // wave-uniform
  const int h2 = hw / 2;
  const int64_t bi = o / (h2 * h2);
  const int i = (int)((o / h2) % h2), j = (int)(o % h2);
  const int c4 = 4 * c;
  float4 v[NCH];
  float s = 0.f;
#pragma unroll
  for (int e = 0; e < NCH; ++e) {
    const int k = 4 * (lane + 64 * e);
    v[e] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (k < c4) {
      const int p = k / c, off = k - p * c;
      const int yy = 2 * i + (p & 1), xx = 2 * j + (p >> 1);
      v[e] = *(const float4*)(x + ((bi * hw + yy) * hw + xx) * (int64_t)c + off);
    }
    s += (v[e].x + v[e].y) + (v[e].z + v[e].w);
  }
  const float mean = mmr::wave_sum(s) / c4;
  float ss = 0.f;
#pragma unroll
  for (int e = 0; e < NCH; ++e)
    if (4 * (lane + 64 * e) < c4) {
      const float a0 = v[e].x - mean, a1 = v[e].y - mean, a2 = v[e].z - mean, a3 = v[e].w - mean;
      ss += (a0 * a0 + a1 * a1) + (a2 * a2 + a3 * a3);
    }
  const float rstd = 1.0f / sqrtf(mmr::wave_sum(ss) / c4 + eps);
#pragma unroll
  for (int e = 0; e < NCH; ++e) {
    const int k = 4 * (lane + 64 * e);
    float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
    if (k < c4) {
      const float4 g = *(const float4*)(gm + k), b = *(const float4*)(bt + k);
      t = make_float4((v[e].x - mean) * rstd * g.x + b.x, (v[e].y - mean) * rstd * g.y + b.y,
                      (v[e].z - mean) * rstd * g.z + b.z, (v[e].w - mean) * rstd * g.w + b.w);
      if (y) *(float4*)(y + o * c4 + k) = t;
    }
    if (xs && k < kp) {
      const uint32_t h0 = mmr::pack2bf(t.x, t.y), h1 = mmr::pack2bf(t.z, t.w);
      const uint32_t l0 = mmr::pack2bf(t.x - __uint_as_float(h0 << 16), t.y - __uint_as_float(h0 & 0xFFFF0000u));
      const uint32_t l1 = mmr::pack2bf(t.z - __uint_as_float(h1 << 16), t.w - __uint_as_float(h1 & 0xFFFF0000u));
      uint16_t* xo = xs + o * 2 * kp + k;
      *(uint2*)xo = make_uint2(h0, h1);
      *(uint2*)(xo + kp) = make_uint2(l0, l1);
    }
  }
}

// patch = 4 (Swin-T): one thread per 4 consecutive columns = one 16-B image row segment (kx 0..3)
__global__ __launch_bounds__(256) void x3_im2col_p4(const float* __restrict__ img, float* __restrict__ cols,
                                                    int64_t ntok, int cin, int hw, int kp) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int kq = kp / 4;
  if (idx >= ntok * kq) return;
  const int64_t tk = idx / kq;
  const int k = 4 * (int)(idx - tk * kq);
  const int gg = hw / 4;
  const int64_t bi = tk / (gg * gg);
  const int py = (int)((tk / gg) % gg), px = (int)(tk % gg);
  float4 val = make_float4(0.f, 0.f, 0.f, 0.f);
  if (k < cin * 16) {
    const int c = k / 16, ky = (k / 4) % 4;
    val = *(const float4*)(img + ((bi * cin + c) * hw + (py * 4 + ky)) * (int64_t)hw + px * 4);
  }
  *(float4*)(cols + tk * kp + k) = val;
}

// HF BertEmbeddings: LN(word[id] + pos[l] + type[0]) -> f32 (one wave per token, c <= 1024)
__global__ __launch_bounds__(256) void x3_bert_embed(const int64_t* __restrict__ ids, const float* __restrict__ word,
                                                     const float* __restrict__ pos, const float* __restrict__ type0,
                                                     const float* __restrict__ gm, const float* __restrict__ bt,
                                                     float* __restrict__ y, int64_t ntok, int l, int c, float eps) {
  const int64_t tk = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (tk >= ntok) return;
  const float* wr = word + ids[tk] * (int64_t)c;
  const float* pr = pos + (int64_t)(tk % l) * c;
  float v[16];
  float s = 0.f;
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int k = lane + 64 * e;
    v[e] = 0.f;
    if (k < c) {
      v[e] = (wr[k] + type0[k]) + pr[k];  // HF: inputs_embeds + token_type_embeddings, then + position
      s += v[e];
    }
  }
  const float mean = mmr::wave_sum(s) / c;
  float ss = 0.f;
#pragma unroll
  for (int e = 0; e < 16; ++e)
    if (lane + 64 * e < c) ss += (v[e] - mean) * (v[e] - mean);
  const float rstd = 1.0f / sqrtf(mmr::wave_sum(ss) / c + eps);
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int k = lane + 64 * e;
    if (k < c) y[tk * c + k] = (v[e] - mean) * rstd * gm[k] + bt[k];
  }
}

// y = x + pos[row % l] (f32)
__global__ __launch_bounds__(256) void x3_add_pos(const float* __restrict__ x, const float* __restrict__ pos,
                                                  float* __restrict__ y, int64_t rows, int l, int c) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= rows * c) return;
  const int64_t row = i / c;
  y[i] = x[i] + pos[(row % l) * c + i % c];
}

__global__ __launch_bounds__(256) void x3_add_pos4(const float* __restrict__ x, const float* __restrict__ pos,
                                                   float* __restrict__ y, int64_t rows, int l, int c) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;  // 4-float chunk
  const int c4 = c / 4;
  if (i >= rows * c4) return;
  const int64_t row = i / c4;
  const int col = 4 * (int)(i - row * c4);
  const float4 a = *(const float4*)(x + 4 * i), p = *(const float4*)(pos + (row % l) * c + col);
  *(float4*)(y + 4 * i) = make_float4(a.x + p.x, a.y + p.y, a.z + p.z, a.w + p.w);
}

// the same by 16-B chunks (c % 4 == 0)
__global__ __launch_bounds__(256) void x3_assemble_seq4(const float* __restrict__ x1, const float* __restrict__ pf,
                                                        const float* __restrict__ x2, const float* __restrict__ pe,
                                                        float* __restrict__ seq, int nb, int np, int c) {
  const int ls = np + 2, c4 = c / 4;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)nb * ls * c4) return;
  const int64_t row = i / c4;
  const int ch = 4 * (int)(i - row * c4);
  const int tt = (int)(row % ls);
  const int64_t bi = row / ls;
  const float* src = tt == 0 ? x1 + bi * c : tt == ls - 1 ? x2 + bi * c : pf + (bi * np + tt - 1) * c;
  const float4 v = *(const float4*)(src + ch), p = *(const float4*)(pe + (int64_t)tt * c + ch);
  *(float4*)(seq + 4 * i) = make_float4(v.x + p.x, v.y + p.y, v.z + p.z, v.w + p.w);
}

// The split-operand forms (round 5): the same sums written as the x3 split GEMM's [hi | lo] operand rows
// (2 kp wide, zero columns c..kp) — and, for add-pos, the f32 rows too when y != NULL (the enhancer's
// LayerNorm residual) — so the in-proj / combiner QKV GEMMs skip their split pass.  One thread per
// 4-column chunk of the kp-wide row.
__device__ __forceinline__ void store_split4(uint16_t* xr, int kp, const float4 v) {
  uint2 h, l;
  split4(v, h, l);
  *(uint2*)xr = h;
  *(uint2*)(xr + kp) = l;
}

__global__ __launch_bounds__(256) void x3_add_pos_split(const float* __restrict__ x, const float* __restrict__ pos,
                                                        float* __restrict__ y, uint16_t* __restrict__ xs, int64_t rows,
                                                        int l, int c, int kp) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int k4 = kp / 4;
  if (i >= rows * k4) return;
  const int64_t row = i / k4;
  const int col = 4 * (int)(i - row * k4);
  float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
  if (col < c) {
    const float4 a = *(const float4*)(x + row * c + col), p = *(const float4*)(pos + (row % l) * c + col);
    v = make_float4(a.x + p.x, a.y + p.y, a.z + p.z, a.w + p.w);
    if (y) *(float4*)(y + row * c + col) = v;
  }
  store_split4(xs + row * 2 * kp + col, kp, v);
}

__global__ __launch_bounds__(256) void x3_assemble_seq_split(const float* __restrict__ x1, const float* __restrict__ pf,
                                                             const float* __restrict__ x2, const float* __restrict__ pe,
                                                             uint16_t* __restrict__ xs, int nb, int np, int c, int kp) {
  const int ls = np + 2, k4 = kp / 4;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)nb * ls * k4) return;
  const int64_t row = i / k4;
  const int ch = 4 * (int)(i - row * k4);
  const int tt = (int)(row % ls);
  const int64_t bi = row / ls;
  float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
  if (ch < c) {
    const float* src = tt == 0 ? x1 + bi * c : tt == ls - 1 ? x2 + bi * c : pf + (bi * np + tt - 1) * c;
    const float4 a = *(const float4*)(src + ch), p = *(const float4*)(pe + (int64_t)tt * c + ch);
    v = make_float4(a.x + p.x, a.y + p.y, a.z + p.z, a.w + p.w);
  }
  store_split4(xs + row * 2 * kp + ch, kp, v);
}

// seq (b, np + 2, c) = [x1; pf; x2] + pe (f32)
__global__ __launch_bounds__(256) void x3_assemble_seq(const float* __restrict__ x1, const float* __restrict__ pf,
                                                       const float* __restrict__ x2, const float* __restrict__ pe,
                                                       float* __restrict__ seq, int nb, int np, int c) {
  const int ls = np + 2;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)nb * ls * c) return;
  const int ch = (int)(i % c);
  const int64_t row = i / c;
  const int tt = (int)(row % ls);
  const int64_t bi = row / ls;
  float v;
  if (tt == 0) v = x1[bi * c + ch];
  else if (tt == ls - 1) v = x2[bi * c + ch];
  else v = pf[(bi * np + tt - 1) * c + ch];
  seq[i] = v + pe[(int64_t)tt * c + ch];
}

// y[b][ch] = (extra[b][ch] + sum_t x[b][t][ch]) / (l + has_extra), summed in token order
__global__ __launch_bounds__(256) void x3_mean_rows(const float* __restrict__ x, const float* __restrict__ extra,
                                                    float* __restrict__ y, int l, int c) {
  const int bi = blockIdx.y;
  const int k = blockIdx.x * 256 + threadIdx.x;
  if (k >= c) return;
  const float* xr = x + (int64_t)bi * l * c + k;
  float s = 0.f;
  for (int tt = 0; tt < l; ++tt) s += xr[(int64_t)tt * c];
  if (extra) y[(int64_t)bi * c + k] = (extra[(int64_t)bi * c + k] + s) / (l + 1);
  else y[(int64_t)bi * c + k] = s / l;
}

// y[b][:] = x[b * ldx + 0..c)
__global__ __launch_bounds__(256) void x3_gather_rows(const float* __restrict__ x, int64_t ldx, float* __restrict__ y,
                                                      int nb, int c) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)nb * c) return;
  y[i] = x[(i / c) * ldx + (i % c)];
}

bool al16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

mmr_status launch_attention(const char* who, AttnArgs a, int64_t nbh, bool swin, void* stream) {
  MMR_REQUIRE(a.q && a.k && a.v && (a.out || a.mean_out || a.xs), "%s: NULL pointer", who);
  MMR_REQUIRE(a.lq > 0 && a.lk > 0 && a.heads > 0 && a.dh > 0 && a.dh % 8 == 0 && a.dh <= 128,
              "%s: bad shape lq=%d lk=%d heads=%d dh=%d (dh %% 8 == 0, <= 128)", who, a.lq, a.lk, a.heads, a.dh);
  MMR_REQUIRE(a.ldq % 4 == 0 && a.ldk % 4 == 0 && a.ldv % 4 == 0 && al16(a.q) && al16(a.k) && al16(a.v) &&
                  (((int64_t)a.heads * a.dh) <= a.ldq),
              "%s: rows must be 16-B aligned with strides >= heads*dh", who);
  if (nbh == 0) return MMR_OK;
  const int dt = (a.dh + 31) / 32;
  hipStream_t st = mmr::as_stream(stream);
  MMR_REQUIRE(!swin || dt == 1, "%s: Swin head_dim %d must be <= 32", who, a.dh);
  MMR_REQUIRE(!swin || (a.lq == a.lk && a.lk <= 64), "%s: Swin windows of <= 64 tokens (lq=%d lk=%d)", who, a.lq, a.lk);
  const int nwv = std::min(4, (a.lq + 31) / 32);
  const int lkp = (a.lk + 31) & ~31;
  const int kbs = dt <= 1 ? std::min(128, lkp) : std::min(64, lkp);  // dt 2: 39 KB -> 3 blocks per CU (3 waves / SIMD)
  const int dhp = 32 * dt, krow = dhp + 8, vrow = dhp + ((dt & 1) ? 0 : 16), orow = dhp + 4;
  const size_t kv = (size_t)kbs * (krow + vrow) * 4, epi = (size_t)nwv * 32 * orow * 4;
  const size_t lds = std::max(kv, epi) + (size_t)nwv * dhp * 4 + (size_t)kbs * 4 + (swin ? 64 * 8 : 0);
  const dim3 grid((unsigned)nbh), blk(64 * nwv);
  const int mode = swin ? 2 : (a.kmask ? 1 : 0);
#define XM(D_, M_) x3_mha<D_, M_, false><<<grid, blk, lds, st>>>(a, kbs)
  if (mode == 2) x3_mha<1, 2, true><<<grid, blk, lds, st>>>(a, kbs);  // lk <= 64 <= kbs (checked above)
  else if (mode == 1) {
    switch (dt) {
      case 1: XM(1, 1); break;
      case 2: XM(2, 1); break;
      case 3: XM(3, 1); break;
      default: XM(4, 1); break;
    }
  } else {
    switch (dt) {
      case 1: XM(1, 0); break;
      case 2: XM(2, 0); break;
      case 3: XM(3, 0); break;
      default: XM(4, 0); break;
    }
  }
#undef XM
  MMR_LAUNCH_CHECK();
  return MMR_OK;
}

mmr_status launch_patch_merge_v(const float* x, const float* g, const float* b, float* y, uint16_t* xs, int kp,
                                int64_t nout, int hw, int c, float eps, hipStream_t st) {
  const int nch = (int)mmr::ceil_div(std::max(4 * c, kp), 256);
  const dim3 grid((unsigned)mmr::ceil_div(nout, 4));
#define PMV(N_) x3_patch_merge_ln_v<N_><<<grid, 256, 0, st>>>(x, g, b, y, xs, kp, nout, hw, c, eps)
  if (nch <= 2) PMV(2);
  else if (nch <= 3) PMV(3);
  else if (nch <= 4) PMV(4);
  else if (nch <= 6) PMV(6);
  else if (nch <= 8) PMV(8);
  else if (nch <= 12) PMV(12);
  else PMV(16);
#undef PMV
  MMR_LAUNCH_CHECK();
  return MMR_OK;
}

}  // namespace

// ================================================================== C ABI
extern "C" {

mmr_status mmr_x3_linear(const float* x, int64_t ldx, const uint16_t* w_hi, const uint16_t* w_lo, const float* bias,
                         const float* residual, int64_t ldr, float* y, int64_t ldy, int64_t m, int32_t n, int32_t k,
                         int32_t act, void* stream) {
  mmr::clear_error();
  MMR_REQUIRE(x && w_hi && w_lo && y && m >= 0 && n > 0 && k > 0, "mmr_x3_linear: bad arguments");
  MMR_REQUIRE(k % 32 == 0 && ldx >= k && ldx % 4 == 0 && ldy >= n && (!residual || ldr >= n),
              "mmr_x3_linear: k=%d must be a multiple of 32 (ldx=%lld ldy=%lld)", k, (long long)ldx, (long long)ldy);
  MMR_REQUIRE(al16(x) && al16(w_hi) && al16(w_lo), "mmr_x3_linear: x / w must be 16-B aligned");
  MMR_REQUIRE(act == 0 || act == 1, "mmr_x3_linear: act=%d", act);
  MMR_REQUIRE(m < (int64_t(1) << 31), "mmr_x3_linear: m=%lld too large", (long long)m);
  if (m == 0) return MMR_OK;
  const int tiles_n = (int)mmr::ceil_div(n, GX_BN);
  const int64_t ntiles = mmr::ceil_div(m, GX_BM) * tiles_n;
  MMR_REQUIRE(ntiles < (int64_t(1) << 31), "mmr_x3_linear: too many tiles");
  const dim3 grid((unsigned)ntiles);
  hipStream_t st = mmr::as_stream(stream);
  const bool hb = bias != nullptr, hr = residual != nullptr;
#define X3G(A, B_, R_)                                                                                    \
  x3_gemm<A, B_, R_><<<grid, 256, 0, st>>>(x, ldx, w_hi, w_lo, bias, residual, ldr, y, ldy, (int)m, n, k, \
                                           tiles_n, (int)ntiles)
  if (act == 1) {
    if (hb && hr) X3G(1, true, true);
    else if (hb) X3G(1, true, false);
    else if (hr) X3G(1, false, true);
    else X3G(1, false, false);
  } else {
    if (hb && hr) X3G(0, true, true);
    else if (hb) X3G(0, true, false);
    else if (hr) X3G(0, false, true);
    else X3G(0, false, false);
  }
#undef X3G
  MMR_LAUNCH_CHECK();
  return MMR_OK;
}

mmr_status mmr_x3_attention(const float* q, int64_t ldq, const float* k, int64_t ldk, const float* v, int64_t ldv,
                            float* out, int64_t ldo, float* mean_out, const int64_t* mask01, int32_t b, int32_t lq,
                            int32_t lk, int32_t heads, int32_t dh, float scale, void* stream) {
  mmr::clear_error();
  MMR_REQUIRE(b >= 0, "mmr_x3_attention: b=%d", b);
  MMR_REQUIRE(!out || ldo >= (int64_t)heads * dh, "mmr_x3_attention: ldo below heads*dh");
  AttnArgs a{q, ldq, k, ldk, v, ldv, out, ldo, mean_out, mask01, nullptr, lq, lk, heads, dh, scale, 0, 1, 0};
  return launch_attention("mmr_x3_attention", a, (int64_t)b * heads, false, stream);
}

mmr_status mmr_x3_swin_window_attention(const float* qkv, const float* bias, float* out, int32_t b, int32_t hw,
                                        int32_t c, int32_t heads, int32_t ws, int32_t shift, void* stream) {
  mmr::clear_error();
  MMR_REQUIRE(qkv && bias && out && b >= 0 && hw > 0 && ws > 0 && hw % ws == 0 && ws * ws <= 64 && heads > 0 &&
                  c % heads == 0 && shift >= 0 && shift < ws,
              "mmr_x3_swin_window_attention: bad shape hw=%d ws=%d c=%d heads=%d shift=%d", hw, ws, c, heads, shift);
  const int dh = c / heads;
  const int64_t nwin = (int64_t)b * (hw / ws) * (hw / ws);
  AttnArgs a{qkv,     3 * (int64_t)c, qkv + c, 3 * (int64_t)c, qkv + 2 * c, 3 * (int64_t)c, out, c, nullptr, nullptr,
             bias,    ws * ws,        ws * ws, heads,          dh,          1.0f / sqrtf((float)dh), hw, ws, shift};
  return launch_attention("mmr_x3_swin_window_attention", a, nwin * heads, true, stream);
}

mmr_status mmr_x3_attention_xs(const float* q, int64_t ldq, const float* k, int64_t ldk, const float* v, int64_t ldv,
                               uint16_t* xs, float* mean_out, const int64_t* mask01, int32_t b, int32_t lq, int32_t lk,
                               int32_t heads, int32_t dh, float scale, void* stream) {
  mmr::clear_error();
  const int kp = mmr_x3_p8_kpad(heads * dh);
  MMR_REQUIRE(xs && b >= 0 && kp > 0, "mmr_x3_attention_xs: bad arguments (heads*dh=%d)", heads * dh);
  AttnArgs a{q, ldq, k, ldk, v, ldv, nullptr, 0, mean_out, mask01, nullptr, lq, lk, heads, dh, scale, 0, 1, 0, xs, kp};
  return launch_attention("mmr_x3_attention_xs", a, (int64_t)b * heads, false, stream);
}

mmr_status mmr_x3_swin_window_attention_xs(const float* qkv, const float* bias, uint16_t* xs, int32_t b, int32_t hw,
                                           int32_t c, int32_t heads, int32_t ws, int32_t shift, void* stream) {
  mmr::clear_error();
  const int kp = mmr_x3_p8_kpad(c);
  MMR_REQUIRE(qkv && bias && xs && kp > 0 && b >= 0 && hw > 0 && ws > 0 && hw % ws == 0 && ws * ws <= 64 && heads > 0 &&
                  c % heads == 0 && shift >= 0 && shift < ws,
              "mmr_x3_swin_window_attention_xs: bad shape hw=%d ws=%d c=%d heads=%d shift=%d", hw, ws, c, heads, shift);
  const int dh = c / heads;
  const int64_t nwin = (int64_t)b * (hw / ws) * (hw / ws);
  AttnArgs a{qkv,  3 * (int64_t)c, qkv + c, 3 * (int64_t)c, qkv + 2 * c, 3 * (int64_t)c, nullptr, 0,  nullptr, nullptr,
             bias, ws * ws,        ws * ws, heads,          dh,          1.0f / sqrtf((float)dh), hw, ws, shift, xs, kp};
  return launch_attention("mmr_x3_swin_window_attention_xs", a, nwin * heads, true, stream);
}

mmr_status mmr_x3_patch_im2col(const float* image, float* cols, int32_t b, int32_t cin, int32_t hw, int32_t patch,
                               int32_t kp, void* stream) {
  mmr::clear_error();
  MMR_REQUIRE(image && cols && b >= 0 && cin > 0 && patch > 0 && hw % patch == 0 && kp >= cin * patch * patch,
              "mmr_x3_patch_im2col: bad arguments");
  const int64_t ntok = (int64_t)b * (hw / patch) * (hw / patch);
  if (ntok == 0) return MMR_OK;
  if (patch == 4 && hw % 4 == 0 && kp % 4 == 0 && al16(image) && al16(cols))
    x3_im2col_p4<<<dim3((unsigned)mmr::ceil_div(ntok * (kp / 4), 256)), 256, 0, mmr::as_stream(stream)>>>(
        image, cols, ntok, cin, hw, kp);
  else
    x3_im2col<<<dim3((unsigned)mmr::ceil_div(ntok * kp, 256)), 256, 0, mmr::as_stream(stream)>>>(image, cols, ntok, cin,
                                                                                                hw, patch, kp);
  MMR_LAUNCH_CHECK();
  return MMR_OK;
}

mmr_status mmr_x3_patch_merge_ln(const float* x, const float* gamma, const float* beta, float* y, int32_t b,
                                 int32_t hw, int32_t c, float eps, void* stream) {
  mmr::clear_error();
  MMR_REQUIRE(x && gamma && beta && y && b >= 0 && hw % 2 == 0 && c > 0 && 4 * c <= 4096,
              "mmr_x3_patch_merge_ln: bad arguments (4c <= 4096)");
  const int64_t nout = (int64_t)b * (hw / 2) * (hw / 2);
  if (nout == 0) return MMR_OK;
  if (c % 4 == 0 && al16(x) && al16(gamma) && al16(beta) && al16(y))
    return launch_patch_merge_v(x, gamma, beta, y, nullptr, 0, nout, hw, c, eps, mmr::as_stream(stream));
  x3_patch_merge_ln<<<dim3((unsigned)mmr::ceil_div(nout, 4)), 256, 0, mmr::as_stream(stream)>>>(x, gamma, beta, y, nout,
                                                                                               hw, c, eps);
  MMR_LAUNCH_CHECK();
  return MMR_OK;
}

mmr_status mmr_x3_patch_merge_ln_xs(const float* x, const float* gamma, const float* beta, uint16_t* xs, int32_t b,
                                    int32_t hw, int32_t c, float eps, void* stream) {
  mmr::clear_error();
  const int kp = mmr_x3_p8_kpad(4 * c);
  MMR_REQUIRE(x && gamma && beta && xs && b >= 0 && hw % 2 == 0 && c > 0 && c % 4 == 0 && 4 * c <= 4096 && kp > 0 &&
                  al16(x) && al16(gamma) && al16(beta) && al16(xs),
              "mmr_x3_patch_merge_ln_xs: bad arguments (c %% 4 == 0, 4c <= 4096, 16-B aligned)");
  const int64_t nout = (int64_t)b * (hw / 2) * (hw / 2);
  if (nout == 0) return MMR_OK;
  return launch_patch_merge_v(x, gamma, beta, nullptr, xs, kp, nout, hw, c, eps, mmr::as_stream(stream));
}

mmr_status mmr_x3_bert_embed(const int64_t* ids, const float* word, const float* pos, const float* type0,
                             const float* gamma, const float* beta, float* y, int32_t b, int32_t l, int32_t c, float eps,
                             void* stream) {
  mmr::clear_error();
  MMR_REQUIRE(ids && word && pos && type0 && gamma && beta && y && b >= 0 && l > 0 && c > 0 && c <= 1024,
              "mmr_x3_bert_embed: bad arguments (c <= 1024)");
  const int64_t ntok = (int64_t)b * l;
  if (ntok == 0) return MMR_OK;
  x3_bert_embed<<<dim3((unsigned)mmr::ceil_div(ntok, 4)), 256, 0, mmr::as_stream(stream)>>>(ids, word, pos, type0, gamma,
                                                                                           beta, y, ntok, l, c, eps);
  MMR_LAUNCH_CHECK();
  return MMR_OK;
}

mmr_status mmr_x3_add_pos(const float* x, const float* pos, float* y, int64_t rows, int32_t l, int32_t c,
                          void* stream) {
  mmr::clear_error();
  MMR_REQUIRE(x && pos && y && rows >= 0 && l > 0 && c > 0, "mmr_x3_add_pos: bad arguments");
  if (rows == 0) return MMR_OK;
  if (c % 4 == 0 && al16(x) && al16(pos) && al16(y))
    x3_add_pos4<<<dim3((unsigned)mmr::ceil_div(rows * (c / 4), 256)), 256, 0, mmr::as_stream(stream)>>>(x, pos, y, rows,
                                                                                                       l, c);
  else
    x3_add_pos<<<dim3((unsigned)mmr::ceil_div(rows * c, 256)), 256, 0, mmr::as_stream(stream)>>>(x, pos, y, rows, l, c);
  MMR_LAUNCH_CHECK();
  return MMR_OK;
}

mmr_status mmr_x3_add_pos_split(const float* x, const float* pos, float* y, uint16_t* xs, int64_t rows, int32_t l,
                                int32_t c, void* stream) {
  mmr::clear_error();
  const int kp = mmr_x3_p8_kpad(c);
  MMR_REQUIRE(x && pos && xs && rows >= 0 && l > 0 && c > 0 && c % 4 == 0 && kp > 0 && al16(x) && al16(pos) &&
                  (!y || al16(y)) && al16(xs),
              "mmr_x3_add_pos_split: bad arguments (c %% 4 == 0, c <= 4096, 16-B aligned; c=%d)", c);
  if (rows == 0) return MMR_OK;
  x3_add_pos_split<<<dim3((unsigned)mmr::ceil_div(rows * (kp / 4), 256)), 256, 0, mmr::as_stream(stream)>>>(
      x, pos, y, xs, rows, l, c, kp);
  MMR_LAUNCH_CHECK();
  return MMR_OK;
}

mmr_status mmr_x3_assemble_seq_split(const float* x1, const float* patches_fused, const float* x2, const float* pe,
                                     uint16_t* xs, int32_t b, int32_t np, int32_t c, void* stream) {
  mmr::clear_error();
  const int kp = mmr_x3_p8_kpad(c);
  MMR_REQUIRE(x1 && patches_fused && x2 && pe && xs && b >= 0 && np > 0 && c > 0 && c % 4 == 0 && kp > 0 && al16(x1) &&
                  al16(patches_fused) && al16(x2) && al16(pe) && al16(xs),
              "mmr_x3_assemble_seq_split: bad arguments (c %% 4 == 0, c <= 4096, 16-B aligned; c=%d)", c);
  if (b == 0) return MMR_OK;
  const int64_t n4 = (int64_t)b * (np + 2) * (kp / 4);
  x3_assemble_seq_split<<<dim3((unsigned)mmr::ceil_div(n4, 256)), 256, 0, mmr::as_stream(stream)>>>(
      x1, patches_fused, x2, pe, xs, b, np, c, kp);
  MMR_LAUNCH_CHECK();
  return MMR_OK;
}

mmr_status mmr_x3_assemble_seq(const float* x1, const float* patches_fused, const float* x2, const float* pe,
                               float* seq, int32_t b, int32_t np, int32_t c, void* stream) {
  mmr::clear_error();
  MMR_REQUIRE(x1 && patches_fused && x2 && pe && seq && b >= 0 && np > 0 && c > 0, "mmr_x3_assemble_seq: bad arguments");
  if (b == 0) return MMR_OK;
  const int64_t n = (int64_t)b * (np + 2) * c;
  if (c % 4 == 0 && al16(x1) && al16(patches_fused) && al16(x2) && al16(pe) && al16(seq))
    x3_assemble_seq4<<<dim3((unsigned)mmr::ceil_div(n / 4, 256)), 256, 0, mmr::as_stream(stream)>>>(
        x1, patches_fused, x2, pe, seq, b, np, c);
  else
    x3_assemble_seq<<<dim3((unsigned)mmr::ceil_div(n, 256)), 256, 0, mmr::as_stream(stream)>>>(x1, patches_fused, x2, pe,
                                                                                               seq, b, np, c);
  MMR_LAUNCH_CHECK();
  return MMR_OK;
}

mmr_status mmr_x3_mean_rows(const float* x, const float* extra, float* y, int32_t b, int32_t l, int32_t c,
                            void* stream) {
  mmr::clear_error();
  MMR_REQUIRE(x && y && b >= 0 && l > 0 && c > 0, "mmr_x3_mean_rows: bad arguments");
  if (b == 0) return MMR_OK;
  x3_mean_rows<<<dim3((unsigned)mmr::ceil_div(c, 256), (unsigned)b), 256, 0, mmr::as_stream(stream)>>>(x, extra, y, l,
                                                                                                      c);
  MMR_LAUNCH_CHECK();
  return MMR_OK;
}

mmr_status mmr_x3_gather_rows(const float* x, int64_t ldx, float* y, int32_t b, int32_t c, void* stream) {
  mmr::clear_error();
  MMR_REQUIRE(x && y && b >= 0 && c > 0 && ldx >= c, "mmr_x3_gather_rows: bad arguments");
  if (b == 0) return MMR_OK;
  x3_gather_rows<<<dim3((unsigned)mmr::ceil_div((int64_t)b * c, 256)), 256, 0, mmr::as_stream(stream)>>>(x, ldx, y, b,
                                                                                                        c);
  MMR_LAUNCH_CHECK();
  return MMR_OK;
}

}  // extern "C"
