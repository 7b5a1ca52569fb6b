// Microbenchmark: LDS accumulate throughput on gfx950 for the k-means M-step.
// Variants (all: 256 workgroups x 512 threads, 1 per CU, K=1024 x 33-float LDS rows):
//   0 ds_add_f32, random labels, 4 lanes/row x 8 cols (the update kernel's pattern)
//   1 ds_add_f32, conflict-free (lane -> own bank, label uniform per half-wave)
//   2 ds_add_u32, random labels (pattern 0)
//   3 ds_add_u64 (fixed point), random labels
//   4 non-atomic ds_read + add + ds_write, random labels (racy; throughput only)
//   5 ds_add_f32, 32 lanes per row (one row per half-wave: conflict-free by construction)
//   6 non-atomic RMW, 32 lanes per row
// Prints lane-ops per cycle per CU at an assumed 2.1 GHz.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__device__ __forceinline__ uint32_t hash(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352d; x ^= x >> 15; x *= 0x846ca68b; x ^= x >> 16; return x;
}

constexpr int K = 1024, LD = 33, NT = 512, ITERS = 4096;

template <int V>
__global__ __launch_bounds__(NT) void kern(float* out, int seed) {
  __shared__ __attribute__((aligned(16))) char smem[K * LD * 4];
  float* s = (float*)smem;
  uint32_t* su = (uint32_t*)smem;
  unsigned long long* s64 = (unsigned long long*)smem;
  for (int i = threadIdx.x; i < K * LD; i += NT) s[i] = 0.f;
  __syncthreads();
  const int tid = threadIdx.x;
  uint32_t st = hash(tid * 977 + blockIdx.x * 131 + seed);
  float acc = 0.f;
  for (int it = 0; it < ITERS; ++it) {
    st = hash(st + it);
    if (V == 0 || V == 2 || V == 3 || V == 4) {
      const int row = tid >> 2, lp = tid & 3;  // 4 lanes per row
      const uint32_t lab = hash(row * 7919 + it * 104729 + blockIdx.x) & (K - 1);
      const int base = lab * LD + lp * 8;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        if (V == 0) __hip_atomic_fetch_add(s + base + e, 1.0f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (V == 2) __hip_atomic_fetch_add(su + base + e, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (V == 3) __hip_atomic_fetch_add(s64 + (lab * LD + lp * 8 + e) / 2 * 1, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (V == 4) { float v = s[base + e]; s[base + e] = v + 1.0f; }
      }
    } else if (V == 1) {
      const int lane = tid & 63;
      const uint32_t lab = hash((tid >> 5) * 7919 + it * 104729 + blockIdx.x) & (K - 1);
#pragma unroll
      for (int e = 0; e < 8; ++e)
        __hip_atomic_fetch_add(s + lab * LD + (lane & 31), 1.0f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    } else if (V == 7) {
      double* sd = (double*)smem;
      const int row = tid >> 2, lp = tid & 3;
      const uint32_t lab = hash(row * 7919 + it * 104729 + blockIdx.x) & (K / 2 - 1);
#pragma unroll
      for (int e = 0; e < 8; ++e)
        __hip_atomic_fetch_add(sd + lab * LD + lp * 8 + e, 1.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    } else if (V == 5 || V == 6) {
      const int c = tid & 31;
      const uint32_t lab = hash((tid >> 5) * 7919 + it * 104729 + blockIdx.x) & (K - 1);
      const int base = lab * LD + c;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        if (V == 5) __hip_atomic_fetch_add(s + base, 1.0f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        else { float v = s[base]; s[base] = v + 1.0f; }
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 64; i += NT) acc += s[i * 97 % (K * LD)];
  if (threadIdx.x == 0) out[blockIdx.x] = acc;
}

template <int V>
double run(float* d, hipEvent_t a, hipEvent_t b) {
  hipLaunchKernelGGL(kern<V>, dim3(256), dim3(NT), 0, 0, d, 1);
  hipEventRecord(a);
  hipLaunchKernelGGL(kern<V>, dim3(256), dim3(NT), 0, 0, d, 2);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  const double ops = 256.0 * NT * ITERS * 8;
  const double per_cu_cycle = ops / 256.0 / (ms * 1e-3 * 2.1e9);
  printf("variant %d: %8.3f ms  %.3f lane-ops/cycle/CU  (%.1f cycles per wave-instruction)\n", V, ms,
         per_cu_cycle, 64.0 / per_cu_cycle);
  return ms;
}

int main() {
  float* d;
  hipMalloc(&d, 4096 * 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  run<0>(d, a, b); run<1>(d, a, b); run<2>(d, a, b); run<3>(d, a, b);
  run<4>(d, a, b); run<5>(d, a, b); run<6>(d, a, b); run<7>(d, a, b);
  hipFree(d);
  return 0;
}
