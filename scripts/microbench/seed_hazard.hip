// Standalone repro of the assign kernel's seed hazard (tests/test_isa_guard.py,
// profiles/r3_15_ppo_seed_race.md): an MFMA accumulator seed built by a packed-f32 VALU add
// (v_pk_add_f32, what the SLP vectorizer makes of four scalar adds of one offset) followed
// by v_mfma_f32_16x16x32_bf16 reading it as srcC.
//
// Two kernels compute the same thing -- per lane, acc = c + o (4 floats), then K MFMA
// chains on fixed fragments -- one with the seed added as a float2 vector (-> v_pk_add_f32
// straight into srcC), one with four scalar adds (v_add_f32; the production seed_add).
// The harness (1) prints the instructions between the seed write and the MFMA read of the
// packed kernel's code object (llvm-objdump), and (2) launches both ITERS times on random
// data with a fresh offset per launch and counts launches whose outputs differ bitwise.
// Results equal => the hazard did not fire in this micro pattern (the production kernel
// needed its full register / LDS pressure: 5 of 12 launches); the ISA listing shows the
// missing wait state either way.  Retire the workaround when a toolchain emits one.
//
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form=1 \
//        seed_hazard.hip -o bin/seed_hazard
// Dump:  /opt/rocm/llvm/bin/llvm-objdump -d --mcpu=gfx950 <unbundled code object>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <random>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef short short8 __attribute__((ext_vector_type(8)));

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

constexpr int NT = 256, P = 4, STEPS = 64;

template <bool PACKED>
__global__ __launch_bounds__(NT) void seeded_mfma(const short8* __restrict__ a, const short8* __restrict__ b,
                                                  const float* __restrict__ c, const float* __restrict__ off,
                                                  float* __restrict__ out) {
  const int tid = blockIdx.x * NT + threadIdx.x;
  short8 bf[P];
#pragma unroll
  for (int p = 0; p < P; ++p) bf[p] = b[tid * P + p];
  f32x4 best = {3e38f, 3e38f, 3e38f, 3e38f};
  for (int s = 0; s < STEPS; ++s) {
    const short8 af = a[(s * NT + threadIdx.x) % (STEPS * NT)];
    const f32x4 ci = *(const f32x4*)(c + 4 * ((s * 64 + (threadIdx.x & 63)) % 1024));
    const float4 o4 = *(const float4*)(off + 4 * ((tid >> 4) % 256));
    const float ov[4] = {o4.x, o4.y, o4.z, o4.w};
    f32x4 acc[P];
#pragma unroll
    for (int p = 0; p < P; ++p) {
      if constexpr (PACKED) {   // two float2 adds of a broadcast offset: v_pk_add_f32 -> srcC
        const f32x2 lo = f32x2{ci[0], ci[1]} + f32x2{ov[p], ov[p]};
        const f32x2 hi = f32x2{ci[2], ci[3]} + f32x2{ov[p], ov[p]};
        acc[p] = f32x4{lo[0], lo[1], hi[0], hi[1]};
      } else {                  // scalar v_add_f32 (the production seed_add)
        float a0 = ci[0], a1 = ci[1], a2 = ci[2], a3 = ci[3];
        asm volatile("" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3));
        a0 += ov[p]; a1 += ov[p]; a2 += ov[p]; a3 += ov[p];
        acc[p] = f32x4{a0, a1, a2, a3};
      }
    }
#pragma unroll
    for (int p = 0; p < P; ++p) acc[p] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bf[p], acc[p], 0, 0, 0);
#pragma unroll
    for (int p = 0; p < P; ++p)
#pragma unroll
      for (int e = 0; e < 4; ++e) best[e] = fminf(best[e], acc[p][e]);
  }
  *(f32x4*)(out + 4 * tid) = best;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 200;
  const int blocks = 4096;
  const size_t nthr = (size_t)blocks * NT;
  std::mt19937 rng(7);
  std::uniform_int_distribution<int> bits(0x3c00, 0x4100);   // bf16 values ~[0.0078, 8]
  std::uniform_real_distribution<float> u(0.f, 100.f);
  std::vector<short> ha(STEPS * NT * 8), hb(nthr * P * 8);
  for (auto& v : ha) v = (short)bits(rng);
  for (auto& v : hb) v = (short)bits(rng);
  std::vector<float> hc(4096), hoff(1024);
  for (auto& v : hc) v = u(rng);
  short8 *da, *db;
  float *dc, *doff, *o1, *o2;
  CK(hipMalloc(&da, ha.size() * 2));
  CK(hipMalloc(&db, hb.size() * 2));
  CK(hipMalloc(&dc, hc.size() * 4));
  CK(hipMalloc(&doff, hoff.size() * 4));
  CK(hipMalloc(&o1, nthr * 16));
  CK(hipMalloc(&o2, nthr * 16));
  CK(hipMemcpy(da, ha.data(), ha.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(db, hb.data(), hb.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dc, hc.data(), hc.size() * 4, hipMemcpyHostToDevice));
  std::vector<float> r1(nthr * 4), r2(nthr * 4);
  int bad = 0;
  long long badvals = 0;
  for (int it = 0; it < iters; ++it) {
    for (auto& v : hoff) v = u(rng);
    CK(hipMemcpy(doff, hoff.data(), hoff.size() * 4, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(seeded_mfma<true>, dim3(blocks), dim3(NT), 0, 0, da, db, dc, doff, o1);
    hipLaunchKernelGGL(seeded_mfma<false>, dim3(blocks), dim3(NT), 0, 0, da, db, dc, doff, o2);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(r1.data(), o1, nthr * 16, hipMemcpyDeviceToHost));
    CK(hipMemcpy(r2.data(), o2, nthr * 16, hipMemcpyDeviceToHost));
    long long d = 0;
    for (size_t i = 0; i < r1.size(); ++i) d += memcmp(&r1[i], &r2[i], 4) != 0;
    bad += d != 0;
    badvals += d;
  }
  printf("{\"launches\": %d, \"launches_differing\": %d, \"values_differing\": %lld}\n", iters, bad, badvals);
  return 0;
}
