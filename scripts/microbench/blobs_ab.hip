// A/B harness for the blob generator (bf16 rows, the cfg5 batch): production
// (mikmeans/csrc/kpp.hip blobs_kernel) against copies of its vectorised path with
// R Philox rounds and the Box-Muller transform on or off, to see what the VALU time
// goes to.  One process, interleaved rounds, median of rounds x reps.
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I mikmeans/csrc \
//          scripts/microbench/blobs_ab.hip -o scripts/microbench/bin/blobs_ab
// run:   blobs_ab [N D n_centers rounds reps]
#include "../../mikmeans/csrc/kpp.hip"

#include <algorithm>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                             \
    }                                                                                      \
  } while (0)

namespace bx {
using mk::U4;
using mk::f32x4;
using mk::u32x4;

template <int R>
__device__ __forceinline__ U4 philox_r(U4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
    c = U4{(uint32_t)(p1 >> 32) ^ c.y ^ k0, (uint32_t)p1, (uint32_t)(p0 >> 32) ^ c.w ^ k1, (uint32_t)p0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// BM: 0 = none (uniforms as values), 1 = production transform
template <int TPR, int R, int BM>
__global__ __launch_bounds__(256) void blobs_x(uint16_t* X, int64_t i0, int64_t n, int D,
                                               const float* __restrict__ centers, int n_centers,
                                               float stddev, uint32_t k0, uint32_t k1, float* xn) {
  constexpr int EL = 8;
  const int G = D / EL;
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t il = e / TPR;
  const int t = (int)(e % TPR);
  const bool row_ok = il < n;
  const uint64_t gi = (uint64_t)(i0 + (row_ok ? il : 0));
  int cid = 0;
  if (t == 0) {
    const U4 rc = philox_r<R>(U4{(uint32_t)gi, (uint32_t)(gi >> 32), mk::TAG_CID, 0u}, k0, k1);
    cid = (int)__umulhi(rc.x, (uint32_t)n_centers);
  }
  cid = __shfl(cid, (int)(threadIdx.x & 63) & ~(TPR - 1), 64);
  float sq = 0.f;
  if (row_ok) {
    const float* mu = centers + (int64_t)cid * D;
    uint16_t* out = X + il * D;
    for (int g = t; g < G; g += TPR) {
      f32x4 m[2];
      m[0] = *(const f32x4*)(mu + EL * g);
      m[1] = *(const f32x4*)(mu + EL * g + 4);
      const U4 r = philox_r<R>(U4{(uint32_t)gi, (uint32_t)(gi >> 32), (uint32_t)g, mk::TAG_NRM}, k0, k1);
      float z[EL], f[EL];
      if constexpr (BM) {
        mk::box_muller<uint16_t>(r, z);
      } else {
        const uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          z[2 * j] = (float)(w[j] & 0xffffu) * (1.0f / 65536.0f);
          z[2 * j + 1] = (float)(w[j] >> 16) * (1.0f / 65536.0f);
        }
      }
#pragma unroll
      for (int j = 0; j < EL; ++j) f[j] = __builtin_fmaf(stddev, z[j], m[j / 4][j % 4]);
      uint32_t h[EL];
#pragma unroll
      for (int j = 0; j < EL; ++j) {
        const uint32_t u = __float_as_uint(f[j]);
        h[j] = (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
        const float q = __uint_as_float(h[j] << 16);
        sq = __builtin_fmaf(q, q, sq);
      }
      u32x4 wv;
#pragma unroll
      for (int j = 0; j < 4; ++j) wv[j] = h[2 * j] | (h[2 * j + 1] << 16);
      *(u32x4*)(out + EL * g) = wv;
    }
  }
#pragma unroll
  for (int o = 1; o < TPR; o <<= 1) sq += __shfl_xor(sq, o, 64);
  if (row_ok && t == 0) xn[il] = sq;
}

// XO: one Philox4x32-10 call per (row, lane chunk) seeds a xoshiro128++ state that
// yields the chunk's words (4 per 8-value group); chunk c holds groups c, c+8, ...
__device__ __forceinline__ uint32_t rotl32(uint32_t x, int k) { return (x << k) | (x >> (32 - k)); }
__device__ __forceinline__ uint32_t xo_next(uint32_t& s0, uint32_t& s1, uint32_t& s2, uint32_t& s3) {
  const uint32_t r = rotl32(s0 + s3, 7) + s0;
  const uint32_t t = s1 << 9;
  s2 ^= s0;
  s3 ^= s1;
  s1 ^= s2;
  s0 ^= s3;
  s2 ^= t;
  s3 = rotl32(s3, 11);
  return r;
}
template <int TPR>
__global__ __launch_bounds__(256) void blobs_xo(uint16_t* X, int64_t i0, int64_t n, int D,
                                                const float* __restrict__ centers, int n_centers,
                                                float stddev, uint32_t k0, uint32_t k1, float* xn) {
  constexpr int EL = 8;
  const int G = D / EL;
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t il = e / TPR;
  const int t = (int)(e % TPR);
  const bool row_ok = il < n;
  const uint64_t gi = (uint64_t)(i0 + (row_ok ? il : 0));
  int cid = 0;
  if (t == 0) {
    const U4 rc = philox_r<10>(U4{(uint32_t)gi, (uint32_t)(gi >> 32), mk::TAG_CID, 0u}, k0, k1);
    cid = (int)__umulhi(rc.x, (uint32_t)n_centers);
  }
  cid = __shfl(cid, (int)(threadIdx.x & 63) & ~(TPR - 1), 64);
  float sq = 0.f;
  if (row_ok) {
    const float* mu = centers + (int64_t)cid * D;
    uint16_t* out = X + il * D;
    const U4 sd = philox_r<10>(U4{(uint32_t)gi, (uint32_t)(gi >> 32), (uint32_t)t, 0x584Fu}, k0, k1);
    uint32_t s0 = sd.x, s1 = sd.y, s2 = sd.z, s3 = sd.w;
    for (int g = t; g < G; g += TPR) {
      f32x4 m[2];
      m[0] = *(const f32x4*)(mu + EL * g);
      m[1] = *(const f32x4*)(mu + EL * g + 4);
      U4 r;
      r.x = xo_next(s0, s1, s2, s3);
      r.y = xo_next(s0, s1, s2, s3);
      r.z = xo_next(s0, s1, s2, s3);
      r.w = xo_next(s0, s1, s2, s3);
      float z[EL], f[EL];
      mk::box_muller<uint16_t>(r, z);
#pragma unroll
      for (int j = 0; j < EL; ++j) f[j] = __builtin_fmaf(stddev, z[j], m[j / 4][j % 4]);
      uint32_t h[EL];
#pragma unroll
      for (int j = 0; j < EL; ++j) {
        const uint32_t u = __float_as_uint(f[j]);
        h[j] = (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
        const float q = __uint_as_float(h[j] << 16);
        sq = __builtin_fmaf(q, q, sq);
      }
      u32x4 wv;
#pragma unroll
      for (int j = 0; j < 4; ++j) wv[j] = h[2 * j] | (h[2 * j + 1] << 16);
      *(u32x4*)(out + EL * g) = wv;
    }
  }
#pragma unroll
  for (int o = 1; o < TPR; o <<= 1) sq += __shfl_xor(sq, o, 64);
  if (row_ok && t == 0) xn[il] = sq;
}
}  // namespace bx

struct Var { const char* name; int kind; };

int main(int argc, char** argv) {
  const int64_t N = argc > 1 ? atoll(argv[1]) : (1 << 24);
  const int D = argc > 2 ? atoi(argv[2]) : 256;
  const int NC = argc > 3 ? atoi(argv[3]) : 512;
  const int rounds = argc > 4 ? atoi(argv[4]) : 4;
  const int reps = argc > 5 ? atoi(argv[5]) : 5;
  uint16_t* X; float* xn; float* C;
  CK(hipMalloc(&X, N * D * 2));
  CK(hipMalloc(&xn, N * 4));
  CK(hipMalloc(&C, (size_t)NC * D * 4));
  CK(mk::launch_blob_centers(C, NC, D, 10.f, 7, 0));
  const uint32_t k0 = 7, k1 = 0;
  const unsigned nb = (unsigned)((N * 8 + 255) / 256);
  auto run = [&](int kind) {
    switch (kind) {
      case 0: return mk::launch_blobs(mk::DT_BF16, X, 0, N, D, D, C, NC, 1.f, 7, nullptr, xn, 0);
      case 1: hipLaunchKernelGGL((bx::blobs_x<8, 10, 1>), dim3(nb), dim3(256), 0, 0, X, 0, N, D, C, NC, 1.f, k0, k1, xn); break;
      case 2: hipLaunchKernelGGL((bx::blobs_x<8, 7, 1>), dim3(nb), dim3(256), 0, 0, X, 0, N, D, C, NC, 1.f, k0, k1, xn); break;
      case 3: hipLaunchKernelGGL((bx::blobs_x<8, 10, 0>), dim3(nb), dim3(256), 0, 0, X, 0, N, D, C, NC, 1.f, k0, k1, xn); break;
      case 4: hipLaunchKernelGGL((bx::blobs_x<8, 0, 1>), dim3(nb), dim3(256), 0, 0, X, 0, N, D, C, NC, 1.f, k0, k1, xn); break;
      case 5: hipLaunchKernelGGL((bx::blobs_x<8, 0, 0>), dim3(nb), dim3(256), 0, 0, X, 0, N, D, C, NC, 1.f, k0, k1, xn); break;
      case 6: hipLaunchKernelGGL((bx::blobs_xo<8>), dim3(nb), dim3(256), 0, 0, X, 0, N, D, C, NC, 1.f, k0, k1, xn); break;
      case 7: hipLaunchKernelGGL((bx::blobs_xo<4>), dim3((unsigned)((N * 4 + 255) / 256)), dim3(256), 0, 0, X, 0, N, D, C, NC, 1.f, k0, k1, xn); break;
      case 8: hipLaunchKernelGGL((bx::blobs_xo<2>), dim3((unsigned)((N * 2 + 255) / 256)), dim3(256), 0, 0, X, 0, N, D, C, NC, 1.f, k0, k1, xn); break;
    }
    return hipGetLastError();
  };
  std::vector<Var> vs = {{"prod", 0}, {"copy_r10", 1}, {"r7", 2}, {"r10_noBM", 3}, {"r0_BM", 4}, {"r0_noBM(store)", 5}, {"xo_tpr8", 6}, {"xo_tpr4", 7}, {"xo_tpr2", 8}};
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (auto& v : vs) CK(run(v.kind));
  CK(hipDeviceSynchronize());
  std::vector<std::vector<float>> ts(vs.size());
  for (int r = 0; r < rounds; ++r)
    for (size_t v = 0; v < vs.size(); ++v)
      for (int i = 0; i < reps; ++i) {
        CK(hipEventRecord(e0, 0));
        CK(run(vs[v].kind));
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ts[v].push_back(ms);
      }
  for (size_t v = 0; v < vs.size(); ++v) {
    auto t = ts[v];
    std::sort(t.begin(), t.end());
    const double med = t[t.size() / 2];
    printf("N=%lld D=%d %-16s median %.4f ms  min %.4f ms  %.0f GB/s written\n", (long long)N, D, vs[v].name, med, t[0],
           N * D * 2.0 / (med * 1e-3) / 1e9);
  }
  return 0;
}
