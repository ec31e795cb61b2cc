// Scale-block probe for v_mfma_scale_f32_16x16x128_f8f6f4 (e4m3): A one-hot at (lane group g0,
// byte j0) of row 0, B all e4m3(1.0); A-scale of lane group g = 2^(g+1) for every row.  The output
// 2^(g+1) names the scale group that covers byte j0 of lane group g0.
// build: hipcc -x hip --offload-arch=gfx950 -O3 -std=c++17 tools/mfma_fp8_scale_probe.hip -o tools/mfma_fp8_scale_probe.bin
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void probe(float* C, int g0, int j0) {
  const int l = threadIdx.x, g = l >> 4, r = l & 15;
  unsigned char fa[32], fb[32];
  for (int j = 0; j < 32; ++j) { fa[j] = (g == g0 && r == 0 && j == j0) ? 0x38 : 0; fb[j] = 0x38; }
  i32x8 a, b;
  memcpy(&a, fa, 32);
  memcpy(&b, fb, 32);
  f32x4 c = {0.f, 0.f, 0.f, 0.f};
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, 128 + g, 0, 127);
  for (int i = 0; i < 4; ++i) C[(4 * g + i) * 16 + r] = c[i];
}

int main() {
  float* dC;
  if (hipMalloc(&dC, 1024) != hipSuccess) return 1;
  for (int g0 = 0; g0 < 4; ++g0) {
    printf("lane group %d bytes 0..31 -> scale group:", g0);
    for (int j0 = 0; j0 < 32; ++j0) {
      probe<<<1, 64>>>(dC, g0, j0);
      float C[256];
      if (hipMemcpy(C, dC, 1024, hipMemcpyDeviceToHost) != hipSuccess) return 1;
      int sg = -1;
      for (int s = 0; s < 4; ++s) if (C[0] == (float)(1 << (s + 1))) sg = s;
      printf(" %d", sg);
    }
    printf("\n");
  }
  return 0;
}
