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
                                                 float* sink, long shift) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  const long base = ((long)blockIdx.x * 256 + wid * 64 + shift) % (n - 64);
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

// Contention variant: workgroups b >= 256 (three per CU after the first 256, dispatched
// breadth-first) stream an L2-resident 256 KiB buffer into LDS by LDS-DMA (the assign
// kernel's centre ring traffic; stream = 0: they idle), workgroups b < 256 wait 20 us, then
// time their fragment loads.
__global__ __launch_bounds__(256) void frag_load_contended(const unsigned short* X, long n, const char* C,
                                                           unsigned long long* ts, float* sink, int stream,
                                                           int stream_us, long shift) {
  __shared__ __attribute__((aligned(16))) char ring[16384];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
  if (blockIdx.x >= 256) {
    const unsigned long long until = t_start + (unsigned long long)stream_us * 100ull;
    if (stream) {
      // a fixed trip count (the barrier inside needs every wave to take the same number of
      // trips; a time-based exit could differ between waves)
      const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc((void*)C, 0, 262144, 0x00020000);
      unsigned off = 0;
      for (int it = 0; it < stream_us * 2; ++it) {
        for (int i = 0; i < 4; ++i)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rc, (__attribute__((address_space(3))) void*)(ring + (wid * 4 + i) * 1024), 16,
                                                   (unsigned)lane * 16u, off + (unsigned)(wid * 4 + i) * 1024u, 0, 0);
        __builtin_amdgcn_s_waitcnt(0x0070 | (15 << 8));   // vmcnt(0)
        __syncthreads();
        off = (off + 16384u) & (262144u - 1u);
      }
    } else if (stream == 3) {   // LDS-DMA at full rate: 8 KiB per wave in flight, no barrier
      const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc((void*)C, 0, 262144, 0x00020000);
      unsigned off = 0;
      for (int it = 0; it < stream_us * 8; ++it) {
        for (int i = 0; i < 4; ++i)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rc, (__attribute__((address_space(3))) void*)(ring + (wid * 4 + i) * 1024), 16,
                                                   (unsigned)lane * 16u, off + (unsigned)(wid * 4 + i) * 1024u, 0, 0);
        __builtin_amdgcn_s_waitcnt((8 & 15) | (7 << 4) | (15 << 8));   // vmcnt(8): two batches in flight
        off = (off + 16384u) & (262144u - 1u);
      }
      __builtin_amdgcn_s_waitcnt((0) | (7 << 4) | (15 << 8));
    } else if (stream == 2) {   // matrix cores + LDS reads, as the assign's chunk loop (no barrier)
      typedef float f32x4 __attribute__((ext_vector_type(4)));
      typedef short short8 __attribute__((ext_vector_type(8)));
      f32x4 acc[4] = {};
      u32x4 a0 = {1u, 2u, 3u, (unsigned)lane};
      for (int it = 0; it < stream_us * 40; ++it) {
        const u32x4 bfr = *(const u32x4*)(ring + ((lane * 16 + it * 1024) & 16383));
#pragma unroll
        for (int p = 0; p < 4; ++p)
          acc[p] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(short8, a0), __builtin_bit_cast(short8, bfr),
                                                           acc[p], 0, 0, 0);
      }
      if (acc[0][0] + acc[1][1] + acc[2][2] + acc[3][3] == 1.2345f) sink[threadIdx.x] = 2.f;
    } else {   // (no barrier here: a per-wave time limit is safe)
      while (__builtin_amdgcn_s_memrealtime() < until) __builtin_amdgcn_s_sleep(8);
    }
    return;
  }
  while (__builtin_amdgcn_s_memrealtime() < t_start + 2000ull) __builtin_amdgcn_s_sleep(8);
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  const long base = ((long)blockIdx.x * 256 + wid * 64 + shift) % (n - 64);
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
  if (acc.x == 0x12345678u) sink[threadIdx.x] = 1.f;
  if (lane == 0) ts[(long)blockIdx.x * 8 + wid * 2] = t0, ts[(long)blockIdx.x * 8 + wid * 2 + 1] = t1;
}

static void report(const char* tag, std::vector<unsigned long long>& h, int wgs, long n) {
  std::vector<double> lat;
  for (int b = 0; b < wgs; ++b)
    for (int w = 0; w < 4; ++w) lat.push_back((h[b * 8 + w * 2 + 1] - h[b * 8 + w * 2]) * 0.01);
  std::sort(lat.begin(), lat.end());
  printf("{\"mode\": \"%s\", \"rows\": %ld, \"loader_workgroups\": %d, \"landed_us\": {\"p10\": %.2f, \"median\": %.2f, \"p90\": %.2f, \"max\": %.2f}}\n",
         tag, n, wgs, lat[lat.size() / 10], lat[lat.size() / 2], lat[lat.size() * 9 / 10], lat.back());
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
    hipLaunchKernelGGL(frag_load, dim3(wgs), dim3(256), 0, 0, X, n, ts, sink, (long)(rep + 1) * 3000000L);
    (void)hipDeviceSynchronize();
  }
  std::vector<unsigned long long> h((size_t)wgs * 8);
  (void)hipMemcpy(h.data(), ts, h.size() * 8, hipMemcpyDeviceToHost);
  if (argc > 3) {   // contention mode: 1024 workgroups, a quarter of them loaders
    char* C;
    (void)hipMalloc(&C, 262144);
    (void)hipMemset(C, 2, 262144);
    for (int stream = 0; stream < 4; ++stream) {
      for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(frag_load_contended, dim3(1024), dim3(256), 0, 0, X, n, C, ts, sink, stream, 60,
                           (long)(stream * 3 + rep + 1) * 1500000L);
        if (hipGetLastError() != hipSuccess) { printf("launch failed\n"); return 1; }
        (void)hipDeviceSynchronize();
      }
      (void)hipMemcpy(h.data(), ts, 256 * 64, hipMemcpyDeviceToHost);
      report(stream == 1 ? "loaders_with_centre_stream" : stream == 2 ? "loaders_with_mfma_neighbours"
             : stream == 3 ? "loaders_with_saturating_lds_dma" : "loaders_idle_neighbours", h, 256, n);
    }
    return 0;
  }
  std::vector<double> lat;
  for (int b = 0; b < wgs; ++b)
    for (int w = 0; w < 4; ++w) lat.push_back((h[b * 8 + w * 2 + 1] - h[b * 8 + w * 2]) * 0.01);
  std::sort(lat.begin(), lat.end());
  printf("{\"rows\": %ld, \"workgroups\": %d, \"landed_us\": {\"p10\": %.2f, \"median\": %.2f, \"p90\": %.2f, \"max\": %.2f}}\n",
         n, wgs, lat[lat.size() / 10], lat[lat.size() / 2], lat[lat.size() * 9 / 10], lat.back());
  return 0;
}
