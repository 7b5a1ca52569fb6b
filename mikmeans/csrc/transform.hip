// mikmeans — distances of every row to every centre (KMeans.transform) on the MFMA tiles.
//
// out[i, k] = sqrt(max(|x_i|^2 + |c_k|^2 - 2 x_i.c_k, 0)), written as f32 [N, K].  The same
// fragment-packed centres the assign kernel reads (csrc/kernels.h layout "16": -2c in the
// points' dtype, |c_q|^2 of the quantised centres in f32), so a fitted model's serving pack
// is reused and the distances are those the assign's argmin ranked: bf16 rows against
// bf16-quantised centres with f32 accumulation, f32 rows on the exact f32 MFMA.
//
// Each wave keeps P blocks of 16 rows in registers (as the assign) and walks the centre
// tiles straight from L2 (the pack is at most Kpad x 1024 x 4 B and every wave reads it in
// the same order).  Lane (r = l & 15, g = l >> 4) ends a tile with the 4 scores of row r
// against centres 16t + 4g + {0..3}: one 16-B store per lane and tile, so the [N, K] output
// -- the bound for any K >= 16 -- streams out as 64-B row segments.
#include "common.h"
#include "kernels.h"
#include "plan.h"

namespace mk {

template <typename T> struct TMfma;
template <> struct TMfma<uint16_t> {
  __device__ static __forceinline__ f32x4 run(const u32x4& a, const u32x4& b, const f32x4& c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(short8, a), __builtin_bit_cast(short8, b), c,
                                                   0, 0, 0);
  }
};
template <> struct TMfma<float> {
  __device__ static __forceinline__ f32x4 run(const u32x4& a, const u32x4& b, f32x4 c) {
#pragma unroll
    for (int e = 0; e < 4; ++e)
      c = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a[e]), __uint_as_float(b[e]), c, 0, 0, 0);
    return c;
  }
};

constexpr int TR_NW = 4;   // waves per workgroup

template <typename T, int DPAD, int P>
__global__ __launch_bounds__(TR_NW * 64) void transform_kernel(TransformArgs a) {
  constexpr int V = Elem<T>::V;
  constexpr int NQ = DPAD / 4 / V;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 15, g = lane >> 4;
  const int64_t pbase = ((int64_t)blockIdx.x * TR_NW + wid) * (P * 16);
  if (pbase >= a.N) return;   // (wave-uniform; no barrier below)
  u32x4 xr[P][NQ];
  float xn[P];
#pragma unroll
  for (int p = 0; p < P; ++p) {
    int64_t row = pbase + p * 16 + r;
    row = row < a.N ? row : a.N - 1;
    const T* rp = (const T*)a.X + row * a.ldx + g * V;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int col = (4 * q + g) * V;
      xr[p][q] = col < a.D ? *(const u32x4*)(rp + 4 * q * V) : u32x4{0u, 0u, 0u, 0u};
    }
    xn[p] = a.xn[row];
  }
  const T* pack = (const T*)a.pack;
  const int ntile = a.Kpad / 16;
  for (int t = 0; t < ntile; ++t) {
    const f32x4 ci = *(const f32x4*)(a.cn + t * 16 + 4 * g);
    f32x4 acc[P];
#pragma unroll
    for (int p = 0; p < P; ++p) acc[p] = ci;
    const T* tp = pack + ((int64_t)t * NQ * 64 + lane) * V;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const u32x4 aq = *(const u32x4*)(tp + (int64_t)q * 64 * V);
#pragma unroll
      for (int p = 0; p < P; ++p) acc[p] = TMfma<T>::run(aq, xr[p][q], acc[p]);
    }
    const int k0 = t * 16 + 4 * g;
#pragma unroll
    for (int p = 0; p < P; ++p) {
      const int64_t row = pbase + p * 16 + r;
      if (row >= a.N) continue;
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float d2 = fmaxf(xn[p] + acc[p][e], 0.f);
        v[e] = a.squared ? d2 : __builtin_sqrtf(d2);
      }
      float* o = a.out + row * a.ldo + k0;
      if (k0 + 3 < a.K && (a.ldo & 3) == 0) {
        *(float4*)o = make_float4(v[0], v[1], v[2], v[3]);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (k0 + e < a.K) o[e] = v[e];
      }
    }
  }
}

template <typename T, int DPAD>
static hipError_t launch_tr(const TransformArgs& a, hipStream_t s) {
  constexpr int NQ = DPAD / 4 / Elem<T>::V;
  // rows in registers: at most 32 16-B pieces per lane (128 VGPRs), at most 8 blocks
  constexpr int P = NQ >= 32 ? 1 : (32 / NQ > 8 ? 8 : 32 / NQ);
  const int64_t per_wg = (int64_t)TR_NW * P * 16;
  const int64_t nb = (a.N + per_wg - 1) / per_wg;
  hipLaunchKernelGGL((transform_kernel<T, DPAD, P>), dim3((unsigned)nb), dim3(TR_NW * 64), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_transform(int dtype, int dpad, const TransformArgs& a, hipStream_t s) {
  if (a.N <= 0 || a.K <= 0) return hipSuccess;
  if (a.Kpad % 16 || a.Kpad < a.K || a.D > dpad) return hipErrorInvalidValue;
  if (dtype == DT_BF16) {
    switch (dpad) {
      case 32: return launch_tr<uint16_t, 32>(a, s);
      case 64: return launch_tr<uint16_t, 64>(a, s);
      case 128: return launch_tr<uint16_t, 128>(a, s);
      case 256: return launch_tr<uint16_t, 256>(a, s);
      case 384: return launch_tr<uint16_t, 384>(a, s);
      case 512: return launch_tr<uint16_t, 512>(a, s);
      case 768: return launch_tr<uint16_t, 768>(a, s);
      case 1024: return launch_tr<uint16_t, 1024>(a, s);
    }
  } else {
    switch (dpad) {
      case 16: return launch_tr<float, 16>(a, s);
      case 32: return launch_tr<float, 32>(a, s);
      case 64: return launch_tr<float, 64>(a, s);
      case 128: return launch_tr<float, 128>(a, s);
      case 256: return launch_tr<float, 256>(a, s);
      case 384: return launch_tr<float, 384>(a, s);
      case 512: return launch_tr<float, 512>(a, s);
      case 768: return launch_tr<float, 768>(a, s);
      case 1024: return launch_tr<float, 1024>(a, s);
    }
  }
  return hipErrorInvalidValue;
}

}  // namespace mk
