// Row-fragment load latency in isolation: each 256-thread workgroup loads its 256 bf16 rows of
// 128 features in the assign kernel's fragment pattern (lane (r, g): row r of a 16-row block,
// 16-B pieces 4q + g; P = 4 blocks per wave), waits, and records entry -> landed in real-time
// ticks (10 ns).  Compares with the landing time inside the assign kernel
// (scripts/assign_timeline.py) to separate the access pattern from in-kernel contention.
//   hipcc --offload-arch=gfx950 -O3 frag_load_latency.hip -o frag_load_latency
//   ./frag_load_latency <rows> <workgroups>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void frag_load(const unsigned short* X, long n, unsigned long long* ts,
                                                 float* sink) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  const long base = ((long)blockIdx.x * 256 + wid * 64) % (n - 64);
  u32x4 acc = {0u, 0u, 0u, 0u};
  u32x4 v[4][4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const unsigned short* rp = X + (base + p * 16 + r) * 128 + g * 8;
#pragma unroll
    for (int q = 0; q < 4; ++q) v[p][q] = *(const u32x4*)(rp + 32 * q);
  }
#pragma unroll
  for (int p = 0; p < 4; ++p)
#pragma unroll
    for (int q = 0; q < 4; ++q) acc ^= v[p][q];
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  if (acc.x == 0x12345678u) sink[threadIdx.x] = 1.f;   // (keeps the loads)
  if (lane == 0) ts[(long)blockIdx.x * 8 + wid * 2] = t0, ts[(long)blockIdx.x * 8 + wid * 2 + 1] = t1;
}

int main(int argc, char** argv) {
  const long n = argc > 1 ? atol(argv[1]) : 20000000;
  const int wgs = argc > 2 ? atoi(argv[2]) : 1024;
  unsigned short* X;
  unsigned long long* ts;
  float* sink;
  if (hipMalloc(&X, (size_t)n * 256) != hipSuccess || hipMalloc(&ts, (size_t)wgs * 64) != hipSuccess ||
      hipMalloc(&sink, 1024) != hipSuccess) {
    printf("alloc failed\n");
    return 1;
  }
  (void)hipMemset(X, 1, (size_t)n * 256);
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(frag_load, dim3(wgs), dim3(256), 0, 0, X, n, ts, sink);
    (void)hipDeviceSynchronize();
  }
  std::vector<unsigned long long> h((size_t)wgs * 8);
  (void)hipMemcpy(h.data(), ts, h.size() * 8, hipMemcpyDeviceToHost);
  std::vector<double> lat;
  for (int b = 0; b < wgs; ++b)
    for (int w = 0; w < 4; ++w) lat.push_back((h[b * 8 + w * 2 + 1] - h[b * 8 + w * 2]) * 0.01);
  std::sort(lat.begin(), lat.end());
  printf("{\"rows\": %ld, \"workgroups\": %d, \"landed_us\": {\"p10\": %.2f, \"median\": %.2f, \"p90\": %.2f, \"max\": %.2f}}\n",
         n, wgs, lat[lat.size() / 10], lat[lat.size() / 2], lat[lat.size() * 9 / 10], lat.back());
  return 0;
}
