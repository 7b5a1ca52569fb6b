// mikmeans — K2 variant: LDS-resident centroids, persistent workgroups (gfx950).
//
// assign16.hip streams the fragment-packed centroid tiles through a 2-slot LDS ring,
// which costs a workgroup barrier every 4 tiles and one L2->LDS copy of all K
// centroids per 256 points (~100 GB per Lloyd iteration at N=1e8, K=1024, bf16).
// Here a workgroup of 16 waves stages a whole K-range of tiles into LDS ONCE and
// then walks point tiles (1024 points each) with no barrier in its main loop: the
// MFMA + epilogue body of assign16 (16x16x32 bf16 / 16x16x4 f32, |c|^2 seeding the
// accumulators, segmented 6-bit packed-index keys + v_min3) runs back to back.
// The grid is persistent (one workgroup per CU) so the centroids cross L2->LDS once
// per CU per pass.
//
// When K does not fit (bf16 D=128: > 32 tiles = 512 centroids in ~130 KiB), the K
// range is split into passes: pass j keeps a per-point best (score, index) in a u64
// scratch array that pass j+1 reads and improves; the last pass writes labels, the
// squared distance, inertia and the changed count exactly like assign16.  X is read
// once per pass (the kernel stays MFMA-bound: 2 x 25.6 GB over ~20 ms at the headline).
#include "common.h"
#include "kernels.h"

namespace mk {

constexpr size_t RES_LDS_MAX = 160 * 1024;

template <typename T, int DPAD, int P>
struct ResCfg {
  static constexpr int NW = 16;                 // waves per workgroup (one workgroup per CU)
  static constexpr int V = Elem<T>::V;
  static constexpr int NQ = DPAD / 4 / V;       // 16-B pieces per lane per point
  static constexpr int TILE_BYTES = NQ * 1024;  // 16 centroids x DPAD
  static constexpr int PTS = NW * P * 16;       // points per workgroup step
  static_assert(NQ >= 1, "DPAD too small for the 16x16 layout");
};

template <typename T> struct MfmaR;
template <> struct MfmaR<uint16_t> {
  __device__ static __forceinline__ f32x4 run(const u32x4& a, const u32x4& b, const f32x4& c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(short8, a),
                                                   __builtin_bit_cast(short8, b), c, 0, 0, 0);
  }
};
template <> struct MfmaR<float> {
  __device__ static __forceinline__ f32x4 run(const u32x4& a, const u32x4& b, f32x4 c) {
#pragma unroll
    for (int e = 0; e < 4; ++e)
      c = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a[e]), __uint_as_float(b[e]), c, 0, 0, 0);
    return c;
  }
};

__device__ __forceinline__ unsigned long long pack_vk(float v, int k) {
  return ((unsigned long long)__float_as_uint(v) << 32) | (unsigned)k;
}

template <typename T, int DPAD, int P>
__global__ __launch_bounds__(1024, 4) void assign_res_kernel(AssignArgs a, int tile0, int ntl,
                                                             int first, int last,
                                                             unsigned long long* __restrict__ keys,
                                                             int64_t n_ptiles) {
  using C = ResCfg<T, DPAD, P>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 15, g = lane >> 4;
  const int cn_bytes = ((ntl * 64 + 1023) / 1024) * 1024;
  char* cn_lds = smem;
  char* tiles = smem + cn_bytes;

  // ---- stage this pass's tiles and |c|^2 once (LDS-DMA, 1 KiB per wave-instruction)
  {
    const char* gC = (const char*)a.Cpack + (int64_t)tile0 * C::TILE_BYTES;
    for (int pc = wid; pc < ntl * C::NQ; pc += C::NW)
      glds16(gC + (int64_t)pc * 1024 + lane * 16, (MK_LDS void*)(tiles + pc * 1024));
    const int64_t cn_len = (int64_t)((a.Kpad + 255) / 256) * 256 * 4;  // bytes (assign_cn_len)
    for (int pc = wid; pc < cn_bytes / 1024; pc += C::NW) {
      int64_t off = (int64_t)tile0 * 64 + (int64_t)pc * 1024 + lane * 16;
      if (off > cn_len - 16) off = cn_len - 16;  // tail piece: stay inside the array
      glds16((const char*)a.cn + off, (MK_LDS void*)(cn_lds + pc * 1024));
    }
    wait_vmcnt<0>();
    __syncthreads();
  }
  const unsigned kmask = key6_mask();
  float inert = 0.f;
  int changed = 0;

  for (int64_t pt = blockIdx.x; pt < n_ptiles; pt += gridDim.x) {
    const int64_t pbase = pt * C::PTS + (int64_t)wid * (P * 16);
    u32x4 xr[P][C::NQ];
#pragma unroll
    for (int p = 0; p < P; ++p) {
      int64_t row = pbase + p * 16 + r;
      row = row < a.N ? row : (a.N - 1);
      const T* rp = (const T*)a.X + row * a.ldx + g * (DPAD / 4);
#pragma unroll
      for (int q = 0; q < C::NQ; ++q) {
        const int col = g * (DPAD / 4) + q * C::V;
        if (col < a.D) xr[p][q] = *(const u32x4*)(rp + q * C::V);
        else xr[p][q] = u32x4{0u, 0u, 0u, 0u};
      }
    }
    float best[P], seg_best[P];
    int bg[P];
#pragma unroll
    for (int p = 0; p < P; ++p) { best[p] = 3.0e38f; seg_best[p] = 3.0e38f; bg[p] = 0; }

    for (int t = 0; t < ntl; ++t) {
      const f32x4 ci = *(const f32x4*)(cn_lds + (t * 16 + 4 * g) * 4);
      const char* tl = tiles + t * C::TILE_BYTES + lane * 16;
      u32x4 aw[C::NQ];
#pragma unroll
      for (int q = 0; q < C::NQ; ++q) aw[q] = *(const u32x4*)(tl + q * 1024);
      f32x4 acc[P];
#pragma unroll
      for (int q = 0; q < C::NQ; ++q) {
#pragma unroll
        for (int p = 0; p < P; ++p) acc[p] = MfmaR<T>::run(aw[q], xr[p][q], q == 0 ? ci : acc[p]);
      }
      // segmented 6-bit keys (as assign16.hip): 4 packs + 2 v_min3 per tile and block
      const unsigned tis = (unsigned)(t & 15) << 2;
      unsigned t0, t1, t2, t3;
      asm volatile("s_mov_b32 %0, %4\n\ts_or_b32 %1, %4, 1\n\ts_or_b32 %2, %4, 2\n\ts_or_b32 %3, %4, 3"
                   : "=s"(t0), "=s"(t1), "=s"(t2), "=s"(t3) : "s"(tis));
#pragma unroll
      for (int p = 0; p < P; ++p) {
        const float k0 = pack_key6(acc[p][0], kmask, t0), k1 = pack_key6(acc[p][1], kmask, t1);
        const float k2 = pack_key6(acc[p][2], kmask, t2), k3 = pack_key6(acc[p][3], kmask, t3);
        seg_best[p] = min3f(min3f(k0, k1, k2), k3, seg_best[p]);
      }
      if ((t & 15) == 15 || t == ntl - 1) {
#pragma unroll
        for (int p = 0; p < P; ++p) {
          const float sv = __uint_as_float(__float_as_uint(seg_best[p]) & ~63u);
          const float bv = __uint_as_float(__float_as_uint(best[p]) & ~63u);
          if (sv < bv) { best[p] = seg_best[p]; bg[p] = t >> 4; }
          seg_best[p] = 3.0e38f;
        }
      }
    }

#pragma unroll
    for (int p = 0; p < P; ++p) {
      const unsigned bits = __float_as_uint(best[p]);
      const int idx = (int)(bits & 63u);
      int k = (tile0 + bg[p] * 16 + (idx >> 2)) * 16 + 4 * g + (idx & 3);
      float v = __uint_as_float(bits & ~63u);
#pragma unroll
      for (int o = 16; o <= 32; o <<= 1) {
        const float vo = __shfl_xor(v, o, 64);
        const int ko = __shfl_xor(k, o, 64);
        if (vo < v || (vo == v && ko < k)) { v = vo; k = ko; }
      }
      if ((p & 3) == g) {
        const int64_t i = pbase + p * 16 + r;
        if (i < a.N) {
          if (!first) {  // earlier passes cover lower centroid indices: they win ties
            const unsigned long long pk = keys[i];
            const float pv = __uint_as_float((unsigned)(pk >> 32));
            if (!(v < pv)) { v = pv; k = (int)(unsigned)pk; }
          }
          if (last) {
            if (a.track_changed) changed += (a.labels[i] != k);
            a.labels[i] = k;
            if (a.xn) {
              const float d = fmaxf(a.xn[i] + v, 0.f);
              inert += d;
              if (a.mind) a.mind[i] = d;
            }
          } else {
            keys[i] = pack_vk(v, k);
          }
        }
      }
    }
  }

  if (last && a.slots) {
    double di = wave_sum((double)inert);
    int dc = wave_sum(changed);
    __syncthreads();  // the tiles are dead: reuse LDS for the cross-wave sums
    double* red = (double*)tiles;
    if (lane == 0) { red[2 * wid] = di; red[2 * wid + 1] = (double)dc; }
    __syncthreads();
    if (threadIdx.x == 0) {
      double si = 0, sc = 0;
      for (int w = 0; w < C::NW; ++w) { si += red[2 * w]; sc += red[2 * w + 1]; }
      double* slot = a.slots + (blockIdx.x % NSLOT) * SLOT_STRIDE;
      atomicAdd(slot + 0, si);
      atomicAdd(slot + 1, sc);
    }
  }
}

// Tiles per pass for this shape (0 if the variant does not apply).
static int res_tiles_per_pass(int tile_bytes) {
  return (int)((RES_LDS_MAX - 2048) / (size_t)(tile_bytes + 64));
}

int assign_res_passes(int dtype, int dpad, int Kpad) {
  const int V = dtype == DT_BF16 ? 8 : 4;
  const int nq = dpad / 4 / V;
  if (nq < 1) return 0;
  const int tpp = res_tiles_per_pass(nq * 1024);
  if (tpp < 1) return 0;
  const int kt = Kpad / 16;
  return (kt + tpp - 1) / tpp;
}

static int g_res_grid = 0;  // persistent workgroups (0 = one per CU)
void set_assign_res_grid(int g) { g_res_grid = g; }

template <typename T, int DPAD, int P>
static hipError_t launch_res_t(const AssignArgs& a, unsigned long long* keys, hipStream_t s) {
  using C = ResCfg<T, DPAD, P>;
  const int kt = a.Kpad / 16;
  const int tpp_max = res_tiles_per_pass(C::TILE_BYTES);
  const int passes = (kt + tpp_max - 1) / tpp_max;
  if (passes > 1 && keys == nullptr) return hipErrorInvalidValue;
  const int tpp = (kt + passes - 1) / passes;  // balanced passes
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)assign_res_kernel<T, DPAD, P>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)RES_LDS_MAX);
    attr = true;
  }
  const int64_t n_ptiles = (a.N + C::PTS - 1) / C::PTS;
  if (n_ptiles <= 0) return hipSuccess;
  static int n_cu = 0;
  if (!n_cu) {
    int dev = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev);
    if (n_cu <= 0) n_cu = 256;
  }
  const int grid = (int)(n_ptiles < (g_res_grid ? g_res_grid : n_cu) ? n_ptiles
                                                                     : (g_res_grid ? g_res_grid : n_cu));
  for (int j = 0; j < passes; ++j) {
    const int tile0 = j * tpp;
    const int ntl = (kt - tile0) < tpp ? (kt - tile0) : tpp;
    const int cn_bytes = ((ntl * 64 + 1023) / 1024) * 1024;
    const size_t lds = (size_t)cn_bytes + (size_t)ntl * C::TILE_BYTES;
    if (lds > RES_LDS_MAX) return hipErrorInvalidValue;
    hipLaunchKernelGGL((assign_res_kernel<T, DPAD, P>), dim3(grid), dim3(C::NW * 64), lds, s, a,
                       tile0, ntl, j == 0 ? 1 : 0, j == passes - 1 ? 1 : 0, keys, n_ptiles);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t launch_assign_res(int dtype, int dpad, const AssignArgs& a, unsigned long long* keys,
                             hipStream_t s) {
  if (dtype == DT_BF16) {
    switch (dpad) {
      case 32: return launch_res_t<uint16_t, 32, 4>(a, keys, s);
      case 64: return launch_res_t<uint16_t, 64, 4>(a, keys, s);
      case 128: return launch_res_t<uint16_t, 128, 4>(a, keys, s);
      case 256: return launch_res_t<uint16_t, 256, 2>(a, keys, s);
    }
  } else {
    switch (dpad) {
      case 16: return launch_res_t<float, 16, 4>(a, keys, s);
      case 32: return launch_res_t<float, 32, 4>(a, keys, s);
      case 64: return launch_res_t<float, 64, 4>(a, keys, s);
      case 128: return launch_res_t<float, 128, 2>(a, keys, s);
      case 256: return launch_res_t<float, 256, 1>(a, keys, s);
    }
  }
  return hipErrorInvalidValue;
}

}  // namespace mk
