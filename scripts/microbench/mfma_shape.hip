// Microbenchmark: 16x16x32 vs 32x32x16 bf16 MFMA tiles in the assign kernel's data flow,
// on random vs all-zero operands, with the in-kernel clock (verdict r2 item 3).
//
// Each wave keeps 64 points x 128 features of X in registers (the assign kernel's point
// fragments) and sweeps 128 centres held in LDS, reading one 16-B centre fragment per lane
// per k-step (ds_read_b128 from a fragment-packed layout, 1 KB per tile and k-step, no bank
// conflicts), as assign16_kernel does:
//   S=16: v_mfma_f32_16x16x32_bf16, 4 point blocks of 16, tiles of 16 centres, 4 k-steps:
//         4 LDS fragments + 16 MFMAs (16 cyc) per tile  -> 8 tiles per sweep
//   S=32: v_mfma_f32_32x32x16_bf16, 2 point blocks of 32, tiles of 32 centres, 8 k-steps:
//         8 LDS fragments + 16 MFMAs (32 cyc) per tile  -> 4 tiles per sweep
// Both do the same FLOPs, the same LDS bytes and the same register footprint per sweep.
// EPI=1 adds a running min over every score (the argmin's v_min3 skeleton, equal VALU per
// score in both shapes).  A diagnostic build: s_memtime / s_memrealtime stamps at the start
// and end of each workgroup go to a buffer of their own; clock = dT/dR x 100 MHz (median WG).
//
// Build (the production flags): hipcc -O3 --offload-arch=gfx950 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form=1 \
//        mfma_shape.hip -o ../mbin/mfma_shape
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

#include "../../mikmeans/csrc/common.h"  // production key helpers: pack_key6, key6_mask, min3f

using namespace mk;

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                               \
    }                                                                         \
  } while (0)

constexpr int DMAX = 128, KC = 128, NT = 256;

__device__ __forceinline__ uint32_t hash(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352d; x ^= x >> 15; x *= 0x846ca68b; x ^= x >> 16; return x;
}

// bf16 values ~ uniform in [-4, 4) (zero = all-zero data)
__global__ void fill(uint16_t* p, int64_t n, int zero, uint32_t seed) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const float f = zero ? 0.f : ((hash((uint32_t)i * 2654435761u + seed) >> 8) * 0x1p-24f - 0.5f) * 8.f;
  p[i] = (uint16_t)(__float_as_uint(f) >> 16);
}

template <int S, int D, int EPI, int ORD = 0>
__global__ __launch_bounds__(NT) void kern(const uint16_t* __restrict__ X, const uint16_t* __restrict__ Cg,
                                           float* __restrict__ out, unsigned long long* __restrict__ stamps,
                                           int sweeps) {
  __shared__ __attribute__((aligned(16))) uint16_t cl[KC * D];
  for (int i = threadIdx.x; i < KC * D / 8; i += NT) ((u32x4*)cl)[i] = ((const u32x4*)Cg)[i];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t)blockIdx.x * (NT / 64) + (threadIdx.x >> 6);
  constexpr int NB = S == 16 ? 4 : 2;       // point blocks per wave
  constexpr int KW = S == 16 ? 32 : 16;     // k per MFMA
  constexpr int KS = D / KW;                // k-steps over D
  constexpr int ROWS = S;                   // rows per block / centres per tile
  constexpr int NTILE = KC / ROWS;
  short8 xf[NB][KS];
  const uint16_t* xw = X + (wave & 4095) * 64 * DMAX;
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int s = 0; s < KS; ++s)
      xf[b][s] = *(const short8*)(xw + (b * ROWS + lane % ROWS) * D + s * KW + (lane / ROWS) * 8);
  float m = 3.0e38f;
  float km = 3.0e38f;
  const unsigned kmask = key6_mask();
  uint32_t vb[NB], tb[NB];   // EPI=2: value-only running min per block + the tile that set it
#pragma unroll
  for (int b = 0; b < NB; ++b) { vb[b] = 0x7f7fffffu; tb[b] = 0u; }
  f32x4 p16[NB];
  f32x16 p32[NB];
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    p16[b] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 16; ++j) p32[b][j] = 0.f;
  }
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < sweeps; ++it) {
#pragma unroll 1
    for (int t = 0; t < NTILE; ++t) {
      if constexpr (S == 16) {
        f32x4 acc[NB];
#pragma unroll
        for (int b = 0; b < NB; ++b) acc[b] = EPI ? f32x4{0.f, 0.f, 0.f, 0.f} : p16[b];
        if constexpr (ORD) {   // point-block-major: each accumulator's k-steps back to back
          short8 cf[KS];
#pragma unroll
          for (int s = 0; s < KS; ++s) cf[s] = *(const short8*)(cl + ((t * KS + s) * 64 + lane) * 8);
#pragma unroll
          for (int b = 0; b < NB; ++b)
#pragma unroll
            for (int s = 0; s < KS; ++s) {
              acc[b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cf[s], xf[b][s], acc[b], 0, 0, 0);
              __builtin_amdgcn_sched_barrier(0);
            }
        } else {
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          const short8 cf = *(const short8*)(cl + ((t * KS + s) * 64 + lane) * 8);  // fragment-packed: 1 KB per (tile, k-step)
#pragma unroll
          for (int b = 0; b < NB; ++b) acc[b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cf, xf[b][s], acc[b], 0, 0, 0);
        }
        }
        if constexpr (EPI == 2) {
          // value-only argmin: 2 v_min3_u32 (non-negative scores order as their bits) fold
          // the tile's 4 scores into the running min, v_cmp + v_cndmask record the tile:
          // 4 VALU per 4 scores (the row inside the tile is recovered once at the end)
#pragma unroll
          for (int b = 0; b < NB; ++b) {
            const uint32_t u0 = __float_as_uint(acc[b][0]), u1 = __float_as_uint(acc[b][1]);
            const uint32_t u2 = __float_as_uint(acc[b][2]), u3 = __float_as_uint(acc[b][3]);
            const uint32_t nb = min(min(u0, u1), min(u2, min(u3, vb[b])));
            tb[b] = nb != vb[b] ? (uint32_t)t : tb[b];
            vb[b] = nb;
          }
        } else if constexpr (EPI == 1) {
#pragma unroll
          for (int b = 0; b < NB; ++b) {
            // production skeleton: 4 v_and_or_b32 key packs (indices in SGPRs) + 2 v_min3
            const unsigned tis = (unsigned)(t & 15) << 2;
            unsigned t0, t1, t2, t3;
            asm volatile("s_mov_b32 %0, %4\n\ts_or_b32 %1, %4, 1\n\ts_or_b32 %2, %4, 2\n\ts_or_b32 %3, %4, 3"
                         : "=s"(t0), "=s"(t1), "=s"(t2), "=s"(t3) : "s"(tis) : "scc");
            const float k0 = pack_key6(acc[b][0], kmask, t0), k1 = pack_key6(acc[b][1], kmask, t1);
            const float k2 = pack_key6(acc[b][2], kmask, t2), k3 = pack_key6(acc[b][3], kmask, t3);
            km = min3f(min3f(k0, k1, k2), k3, km);
          }
        } else {
#pragma unroll
          for (int b = 0; b < NB; ++b) p16[b] = acc[b];
        }
      } else {
        f32x16 acc[NB];
#pragma unroll
        for (int b = 0; b < NB; ++b)
#pragma unroll
          for (int j = 0; j < 16; ++j) acc[b][j] = EPI ? 0.f : p32[b][j];
        if constexpr (ORD) {
          short8 cf[KS];
#pragma unroll
          for (int s = 0; s < KS; ++s) cf[s] = *(const short8*)(cl + ((t * KS + s) * 64 + lane) * 8);
#pragma unroll
          for (int b = 0; b < NB; ++b)
#pragma unroll
            for (int s = 0; s < KS; ++s) {
              acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cf[s], xf[b][s], acc[b], 0, 0, 0);
              __builtin_amdgcn_sched_barrier(0);
            }
        } else {
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          const short8 cf = *(const short8*)(cl + ((t * KS + s) * 64 + lane) * 8);  // fragment-packed: 1 KB per (tile, k-step)
#pragma unroll
          for (int b = 0; b < NB; ++b) acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cf, xf[b][s], acc[b], 0, 0, 0);
        }
        }
        if constexpr (EPI != 0) {
#pragma unroll
          for (int b = 0; b < NB; ++b)
#pragma unroll
            for (int j = 0; j < 16; j += 4) {
              const unsigned tis = (unsigned)((t & 3) * 16 + j);
              unsigned t0, t1, t2, t3;
              asm volatile("s_mov_b32 %0, %4\n\ts_or_b32 %1, %4, 1\n\ts_or_b32 %2, %4, 2\n\ts_or_b32 %3, %4, 3"
                           : "=s"(t0), "=s"(t1), "=s"(t2), "=s"(t3) : "s"(tis) : "scc");
              const float k0 = pack_key6(acc[b][j], kmask, t0), k1 = pack_key6(acc[b][j + 1], kmask, t1);
              const float k2 = pack_key6(acc[b][j + 2], kmask, t2), k3 = pack_key6(acc[b][j + 3], kmask, t3);
              km = min3f(min3f(k0, k1, k2), k3, km);
            }
        } else {
#pragma unroll
          for (int b = 0; b < NB; ++b) p32[b] = acc[b];
        }
      }
    }
  }
  if constexpr (EPI == 2) {
#pragma unroll
    for (int b = 0; b < NB; ++b) km = fminf(km, __uint_as_float(vb[b] ^ tb[b]));
  }
  if constexpr (!EPI) {
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      if constexpr (S == 16) {
#pragma unroll
        for (int j = 0; j < 4; ++j) m = fminf(m, p16[b][j]);
      } else {
#pragma unroll
        for (int j = 0; j < 16; ++j) m = fminf(m, p32[b][j]);
      }
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  out[(int64_t)blockIdx.x * NT + threadIdx.x] = EPI ? km : m;
  if (threadIdx.x == 0) {
    unsigned long long* st = stamps + (int64_t)blockIdx.x * 2;
    st[0] = t1 - t0;
    st[1] = r1 - r0;
  }
}

template <int S, int D, int EPI, int ORD = 0>
int run(const char* name, const uint16_t* X, const uint16_t* C, float* out, unsigned long long* st, int grid,
        int sweeps, const char* data) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  // warm: >= 2 s of back-to-back launches (the clock settles under load)
  float warm = 0.f;
  while (warm < 2000.f) {
    CK(hipEventRecord(a));
    for (int i = 0; i < 20; ++i) hipLaunchKernelGGL((kern<S, D, EPI, ORD>), dim3(grid), dim3(NT), 0, 0, X, C, out, st, sweeps);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    warm += ms;
  }
  const int reps = 20;
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((kern<S, D, EPI, ORD>), dim3(grid), dim3(NT), 0, 0, X, C, out, st, sweeps);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  CK(hipGetLastError());
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  ms /= reps;
  std::vector<unsigned long long> h((size_t)grid * 2);
  CK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
  std::vector<double> clk(grid);
  for (int g = 0; g < grid; ++g) clk[g] = h[g * 2 + 1] ? (double)h[g * 2] / (double)h[g * 2 + 1] * 100.0 : 0.0;
  std::sort(clk.begin(), clk.end());
  const double flops = (double)grid * (NT / 64) * sweeps * 2.0 * 64 * KC * D;
  const double tf = flops / (ms * 1e-3) / 1e12;
  const double mhz = clk[grid / 2];
  // pipe utilisation at the measured clock: 1024 SIMDs x 1024 FLOP/cycle (bf16 dense)
  const double util = tf * 1e12 / (1024.0 * 1024.0 * mhz * 1e6);
  printf("%-10s ord=%d D=%-3d %-6s epi=%d  %8.3f ms  %7.1f TF/s  clock %6.0f MHz (p10 %4.0f p90 %4.0f)  MFMA util %5.1f %%\n",
         name, ORD, D, data, EPI, ms, tf, mhz, clk[grid / 10], clk[grid * 9 / 10], util * 100.0);
  fflush(stdout);
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return 0;
}

int main(int argc, char** argv) {
  const int grid = argc > 1 ? atoi(argv[1]) : 2048;
  const int sweeps = argc > 2 ? atoi(argv[2]) : 400;
  const int64_t nx = 4096LL * 64 * DMAX;
  uint16_t *X, *C;
  float* out;
  unsigned long long* st;
  CK(hipMalloc(&X, nx * 2));
  CK(hipMalloc(&C, (size_t)KC * DMAX * 2));
  CK(hipMalloc(&out, (size_t)grid * NT * 4));
  CK(hipMalloc(&st, (size_t)grid * 16));
  if (argc > 3 && atoi(argv[3]) == 1) {   // issue-order study: q-major vs point-block-major
    hipLaunchKernelGGL(fill, dim3((unsigned)((nx + 255) / 256)), dim3(256), 0, 0, X, nx, 0, 1u);
    hipLaunchKernelGGL(fill, dim3((KC * DMAX + 255) / 256), dim3(256), 0, 0, C, (int64_t)KC * DMAX, 0, 7u);
    CK(hipDeviceSynchronize());
    for (int round = 0; round < 2; ++round) {
      if (run<16, 128, true, 0>("16x16x32", X, C, out, st, grid, sweeps, "random")) return 1;
      if (run<16, 128, true, 1>("16x16x32", X, C, out, st, grid, sweeps, "random")) return 1;
      if (run<32, 128, true, 0>("32x32x16", X, C, out, st, grid, sweeps, "random")) return 1;
      if (run<32, 128, true, 1>("32x32x16", X, C, out, st, grid, sweeps, "random")) return 1;
      if (run<16, 128, false, 1>("16x16x32", X, C, out, st, grid, sweeps, "random")) return 1;
      if (run<32, 128, false, 1>("32x32x16", X, C, out, st, grid, sweeps, "random")) return 1;
    }
    return 0;
  }
  for (int zero = 0; zero < 2; ++zero) {
    const char* data = zero ? "zeros" : "random";
    hipLaunchKernelGGL(fill, dim3((unsigned)((nx + 255) / 256)), dim3(256), 0, 0, X, nx, zero, 1u);
    hipLaunchKernelGGL(fill, dim3((KC * DMAX + 255) / 256), dim3(256), 0, 0, C, (int64_t)KC * DMAX, zero, 7u);
    CK(hipDeviceSynchronize());
    // interleaved rounds: shape order alternates so drift does not favour one arm
    for (int round = 0; round < 2; ++round) {
      if (round == 0) {
        if (run<16, 128, false>("16x16x32", X, C, out, st, grid, sweeps, data)) return 1;
        if (run<32, 128, false>("32x32x16", X, C, out, st, grid, sweeps, data)) return 1;
        if (run<16, 128, true>("16x16x32", X, C, out, st, grid, sweeps, data)) return 1;
        if (run<32, 128, true>("32x32x16", X, C, out, st, grid, sweeps, data)) return 1;
        if (!zero && run<16, 64, true>("16x16x32", X, C, out, st, grid, 2 * sweeps, data)) return 1;
        if (!zero && run<32, 64, true>("32x32x16", X, C, out, st, grid, 2 * sweeps, data)) return 1;
        if (!zero && run<16, 64, 2>("16x16x32", X, C, out, st, grid, 2 * sweeps, data)) return 1;
        if (!zero && run<16, 128, 2>("16x16x32", X, C, out, st, grid, sweeps, data)) return 1;
      } else {
        if (!zero && run<16, 128, 2>("16x16x32", X, C, out, st, grid, sweeps, data)) return 1;
        if (!zero && run<16, 64, 2>("16x16x32", X, C, out, st, grid, 2 * sweeps, data)) return 1;
        if (!zero && run<32, 64, true>("32x32x16", X, C, out, st, grid, 2 * sweeps, data)) return 1;
        if (!zero && run<16, 64, true>("16x16x32", X, C, out, st, grid, 2 * sweeps, data)) return 1;
        if (run<32, 128, true>("32x32x16", X, C, out, st, grid, sweeps, data)) return 1;
        if (run<16, 128, true>("16x16x32", X, C, out, st, grid, sweeps, data)) return 1;
        if (run<32, 128, false>("32x32x16", X, C, out, st, grid, sweeps, data)) return 1;
        if (run<16, 128, false>("16x16x32", X, C, out, st, grid, sweeps, data)) return 1;
      }
    }
  }
  return 0;
}
