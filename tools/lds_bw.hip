// Load-path micro-benchmark (MI355X): bytes/s into one CU's LDS by global_load_lds (LDS-DMA) vs into
// VGPRs by global_load_dwordx4, streaming a buffer far larger than the caches (HBM) or re-reading a
// small one (L2).  One workgroup of W waves per CU, each wave streaming its own contiguous range in
// 1-KB wave pieces with DEPTH pieces in flight.  Answers: what per-CU rate does each path reach?
// build: hipcc -x hip --offload-arch=gfx950 -O3 -std=c++17 tools/lds_bw.hip -o tools/lds_bw.bin
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int DEPTH>
__global__ void glds_stream(const char* __restrict__ src, int64_t bytes_per_wave, int64_t wrap, float* sink) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t gw = (int64_t)blockIdx.x * (blockDim.x >> 6) + wave;
  char* ring = lds + wave * DEPTH * 1024;
  const int64_t n = bytes_per_wave / 1024;
  for (int64_t i = 0; i < n; ++i) {
    const int64_t o = (gw * bytes_per_wave + i * 1024) & (wrap - 1);
    __builtin_amdgcn_global_load_lds((const void*)(src + o + lane * 16), (lds_ptr_t)(ring + (i % DEPTH) * 1024), 16, 0, 0);
    if (i >= DEPTH - 1) __builtin_amdgcn_s_waitcnt((DEPTH - 1) | (7 << 4) | (15 << 8));  // DEPTH-1 in flight (DEPTH <= 16)
  }
  __builtin_amdgcn_s_waitcnt(0 | (7 << 4) | (15 << 8));
  if (lane == 0 && gw == 0) sink[0] = (float)ring[0];
}

template <int DEPTH>
__global__ void vgpr_stream(const char* __restrict__ src, int64_t bytes_per_wave, int64_t wrap, float* sink) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t gw = (int64_t)blockIdx.x * (blockDim.x >> 6) + wave;
  const int64_t n = bytes_per_wave / 1024;
  u32x4 acc = {0, 0, 0, 0};
  for (int64_t i = 0; i < n; i += DEPTH) {
    u32x4 v[DEPTH];
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      const int64_t o = (gw * bytes_per_wave + (i + d) * 1024) & (wrap - 1);
      v[d] = __builtin_nontemporal_load((const u32x4*)(src + o + lane * 16));
    }
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      acc ^= v[d];
    }
  }
  if ((acc[0] ^ acc[1] ^ acc[2] ^ acc[3]) == 0x12345678u) sink[1] = 1.f;
}

template <class K>
float time_it(K launch, int reps) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  launch();
  hipEventRecord(a);
  for (int r = 0; r < reps; ++r) launch();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  return ms / reps;
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int64_t big = int64_t(1) << 30;  // 1 GiB: beyond L2 + MALL
  char* buf;
  float* sink;
  if (hipMalloc(&buf, big) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess) return 1;
  hipMemset(buf, 1, big);
  const int64_t per_cu = 2 << 20;  // bytes per CU per launch (512 MiB total at 256 CUs)
  for (int src = 0; src < 2; ++src) {
    const int64_t wrap = src == 0 ? big : int64_t(1) << 21;  // HBM stream, or a 2 MiB window re-read (L2)
    for (int w : {1, 2, 4, 8, 16}) {
      const int64_t bpw = per_cu / w;
      float g8 = time_it([&] { glds_stream<8><<<cus, 64 * w, w * 8 * 1024>>>(buf, bpw, wrap, sink); }, 5);
      float g16 = w * 16 <= 160 ? time_it([&] { glds_stream<16><<<cus, 64 * w, w * 16 * 1024>>>(buf, bpw, wrap, sink); }, 5) : 1e30f;
      float v8 = time_it([&] { vgpr_stream<8><<<cus, 64 * w>>>(buf, bpw, wrap, sink); }, 5);
      float v16 = time_it([&] { vgpr_stream<16><<<cus, 64 * w>>>(buf, bpw, wrap, sink); }, 5);
      auto gbs = [&](float ms) { return per_cu / (ms * 1e-3) / 1e9; };
      printf("%s waves/CU %2d | GB/s per CU: glds depth8 %6.1f  glds depth16 %6.1f | vgpr depth8 %6.1f  vgpr depth16 %6.1f"
             " | chip TB/s glds16 %.2f vgpr16 %.2f\n",
             src == 0 ? "HBM" : "L2 ", w, gbs(g8), gbs(g16), gbs(v8), gbs(v16),
             gbs(g16) * cus / 1e3, gbs(v16) * cus / 1e3);
    }
  }
  return 0;
}
