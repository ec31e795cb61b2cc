// Probe of v_mfma_scale_f32_16x16x128_f8f6f4 (e4m3 x e4m3) on gfx950: which per-lane k layout and
// which per-lane scale mapping reproduce a host GEMM on exact small-integer data.
// Hypotheses for lane l (r = l % 16, g = l / 16), byte j of its 32-byte fragment:
//   H1: k = 32 g + j            (each lane a contiguous 32-block; one E8M0 scale per lane = block g)
//   H2: k = 8 g + (j % 8) + 32 (j / 8)   (four 16x16x32-style chunks)
//   H3: k = 16 g + j (j < 16), 64 + 16 g + j - 16 (j >= 16)   (two 16-byte chunks; measured: this one)
// build: hipcc -x hip --offload-arch=gfx950 -O3 -std=c++17 tools/mfma_fp8_probe.hip -o tools/mfma_fp8_probe.bin
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// e4m3 (OCP) encode for small integers |v| <= 15 (exact)
static uint8_t e4m3(int v) {
  if (v == 0) return 0;
  const uint8_t s = v < 0 ? 0x80 : 0;
  int a = v < 0 ? -v : v;
  int e = 0;
  while ((1 << (e + 1)) <= a) ++e;           // a = 1.m * 2^e
  const int mant = ((a << 3) >> e) & 7;      // 3 mantissa bits (exact for |v| <= 15)
  return s | (uint8_t)(((e + 7) << 3) | mant);
}

__global__ void probe(const uint8_t* A, const uint8_t* B, const uint8_t* sa, const uint8_t* sb, float* C, int hyp,
                      int smode) {
  const int l = threadIdx.x, r = l % 16, g = l / 16;
  uint8_t fa[32], fb[32];
  for (int j = 0; j < 32; ++j) {
    const int k = hyp == 1 ? 32 * g + j : hyp == 2 ? 8 * g + (j % 8) + 32 * (j / 8) : (j < 16 ? 16 * g + j : 64 + 16 * g + j - 16);
    fa[j] = A[r * 128 + k];   // A[row r][k]
    fb[j] = B[r * 128 + k];   // B stored as [col][k]
  }
  i32x8 a, b;
  memcpy(&a, fa, 32);
  memcpy(&b, fb, 32);
  f32x4 c = {0.f, 0.f, 0.f, 0.f};
  // smode 0: unit scales; 1: lane's own (row r, block g) byte; 2: 4 blocks of row r packed in one dword
  int sA = 127, sB = 127;
  if (smode == 1) { sA = sa[r * 4 + g]; sB = sb[r * 4 + g]; }
  if (smode == 2) {
    sA = sa[r * 4] | (sa[r * 4 + 1] << 8) | (sa[r * 4 + 2] << 16) | (sa[r * 4 + 3] << 24);
    sB = sb[r * 4] | (sb[r * 4 + 1] << 8) | (sb[r * 4 + 2] << 16) | (sb[r * 4 + 3] << 24);
  }
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, sA, 0, sB);
  // C/D map of the 16x16 family: col = l & 15, row = 4 (l >> 4) + i
  for (int i = 0; i < 4; ++i) C[(4 * g + i) * 16 + r] = c[i];
}

int main() {
  int Ai[16 * 128], Bi[16 * 128];
  uint8_t A[16 * 128], B[16 * 128], sa[64], sb[64];
  unsigned s = 12345;
  auto rnd = [&] { s = s * 1103515245u + 12345u; return (int)((s >> 16) % 31) - 15; };
  for (int i = 0; i < 16 * 128; ++i) { Ai[i] = rnd(); Bi[i] = rnd(); A[i] = e4m3(Ai[i]); B[i] = e4m3(Bi[i]); }
  int ea[64], eb[64];
  for (int i = 0; i < 64; ++i) { ea[i] = (int)(s = s * 1103515245u + 12345u, (s >> 16) % 5) - 2; eb[i] = (int)(s = s * 1103515245u + 12345u, (s >> 16) % 5) - 2;
    sa[i] = (uint8_t)(127 + ea[i]); sb[i] = (uint8_t)(127 + eb[i]); }
  double ref[256], ref1[256];
  for (int m = 0; m < 16; ++m)
    for (int n = 0; n < 16; ++n) {
      double acc = 0, acc1 = 0;
      for (int k = 0; k < 128; ++k) {
        acc += (double)Ai[m * 128 + k] * Bi[n * 128 + k] * ldexp(1.0, ea[m * 4 + k / 32] + eb[n * 4 + k / 32]);
        acc1 += (double)Ai[m * 128 + k] * Bi[n * 128 + k];
      }
      ref[m * 16 + n] = acc;
      ref1[m * 16 + n] = acc1;
    }
  uint8_t *dA, *dB, *dsa, *dsb;
  float* dC;
  hipMalloc(&dA, sizeof A); hipMalloc(&dB, sizeof B); hipMalloc(&dsa, 64); hipMalloc(&dsb, 64); hipMalloc(&dC, 1024);
  hipMemcpy(dA, A, sizeof A, hipMemcpyHostToDevice); hipMemcpy(dB, B, sizeof B, hipMemcpyHostToDevice);
  hipMemcpy(dsa, sa, 64, hipMemcpyHostToDevice); hipMemcpy(dsb, sb, 64, hipMemcpyHostToDevice);
  for (int smode = 0; smode < 3; ++smode)
    for (int hyp = 1; hyp <= 3; ++hyp) {
      probe<<<1, 64>>>(dA, dB, dsa, dsb, dC, hyp, smode);
      float C[256];
      hipMemcpy(C, dC, 1024, hipMemcpyDeviceToHost);
      const double* R = smode == 0 ? ref1 : ref;
      int bad = 0;
      double maxd = 0;
      for (int i = 0; i < 256; ++i) { const double d = fabs(C[i] - R[i]); if (d > 1e-3 * (1 + fabs(R[i]))) ++bad; if (d > maxd) maxd = d; }
      printf("scales %d H%d: %d / 256 mismatches (max |diff| %.3g; C[0] %.3f ref %.3f)\n", smode, hyp, bad, maxd, C[0], R[0]);
    }
  return 0;
}
