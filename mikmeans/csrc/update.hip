// mikmeans — K3: Lloyd M-step scatter-add (per-cluster sums and counts) for gfx950.
//
// sums[k,:] += w_i x_i, counts[k] += w_i for k = labels[i].
//
// Why this shape (measured on MI355X, scripts/microbench/lds_atomics.hip):
//  * global float atomics run at ~1.3 TB/s of added bytes chip-wide, so a direct
//    scatter of N=1e8 x D=128 f32 adds (51 GB) would take ~40 ms per iteration;
//  * LDS ds_add_f32 costs ~169 cycles per wave-instruction whatever the bank
//    pattern, ds_add_f64 ~23, but the INTEGER ds_add_u64 only ~8.4.
// So every workgroup privatises a [K][SW] slice of the sums in LDS as 64-bit
// FIXED-POINT integers: each contribution is rounded to an int32 at scale
// 2^sum_exp (chosen per fit from max|x*w| so it cannot overflow) and added with
// ds_add_u64.  Integer addition is exact and associative: the M-step result is
// bitwise identical for any atomic order, and its error (<= 2^-31 max|x| per
// point, unbiased rounding) is far below an f32 accumulator's.
//
// D is split into column slices so the slice fits LDS; every workgroup streams
// its contiguous chunk of rows with 4..16-byte loads and flushes its slice once,
// with plain coalesced stores, into an int64 slab that launch_reduce sums in f64.
// Grid mapping is XCD-aware: blocks b and b+8 share an XCD on MI355X, so the
// n_slices workgroups that read the same rows (different column slices of the
// same lines) get block ids congruent mod 8 and meet in one 4 MB L2.
//
// Reference parity: the reference's "update step" is re-deriving the dashboard
// after humans move cards (app.mjs:481-496 snapshotMetrics counts); counts here
// are exactly those per-centroid counts.
#include <math.h>

#include "common.h"
#include "kernels.h"

namespace mk {

// One workgroup per CU (LDS-bound).  Measured (N=2e7, D=128, K=1024, bf16):
// 512 threads x 4 rows 1.56 ms, 1024 x 8 rows 1.69 ms -- the LDS atomics and
// their bank conflicts, not memory latency, bound this kernel.
constexpr int UPD_NT = 512;
constexpr int UPD_UNROLL = 8;
constexpr size_t UPD_LDS_MAX = 160 * 1024;

template <int BYTES> struct LoadT;
template <> struct LoadT<16> { typedef u32x4 type; };
template <> struct LoadT<8> { typedef uint2 type; };
template <> struct LoadT<4> { typedef uint32_t type; };

template <typename T, int BYTES>
__device__ __forceinline__ void unpack_any(const typename LoadT<BYTES>::type& w, float* o) {
  if constexpr (BYTES == 16) {
    unpack16(w, o, (T*)nullptr);
  } else {
    constexpr int NW = BYTES / 4;
    uint32_t d[NW];
    if constexpr (NW == 1) d[0] = w; else { d[0] = w.x; d[1] = w.y; }
#pragma unroll
    for (int i = 0; i < NW; ++i) {
      if constexpr (sizeof(T) == 2) { o[2 * i] = bf16lo(d[i]); o[2 * i + 1] = bf16hi(d[i]); }
      else o[i] = __uint_as_float(d[i]);
    }
  }
}

__device__ __forceinline__ long long to_fixed(float v, float scale) {
  return (long long)__float2int_rn(v * scale);
}

template <typename T, int SW, bool PAD>
__global__ __launch_bounds__(UPD_NT) void update_kernel(UpdateArgs a, int n_slices,
                                                        int64_t rows_per_chunk) {
  constexpr int ES = sizeof(T);
  constexpr int PB = (SW * ES >= 16) ? 16 : SW * ES;  // bytes per lane load
  constexpr int V = PB / ES;                           // elements per lane load
  constexpr int LPR = SW / V;                          // lanes per row
  constexpr int RPP = UPD_NT / LPR;                    // rows per pass
  constexpr int LD = PAD ? SW + 1 : SW;                // LDS row stride (int64 cells)
  typedef typename LoadT<PB>::type LT;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  long long* s = (long long*)smem;
  long long* cnt = s + (size_t)a.K * LD;

  const int b = blockIdx.x;
  const int j = b >> 3;
  const int slice = j % n_slices;
  const int chunk = (j / n_slices) * 8 + (b & 7);

  for (int e = threadIdx.x; e < a.K * (LD + 1); e += UPD_NT) s[e] = 0;
  __syncthreads();

  const float scale = ldexpf(1.f, a.sum_exp);
  const float cscale = ldexpf(1.f, a.cnt_exp);
  const int64_t row0 = (int64_t)chunk * rows_per_chunk;
  int64_t row1 = row0 + rows_per_chunk;
  if (row1 > a.N) row1 = a.N;
  const int lr = threadIdx.x / LPR, lp = threadIdx.x % LPR;
  const int col = slice * SW + lp * V;
  const bool colok = col < a.D;
  const bool counter = (slice == 0) && (lp == 0);

  for (int64_t base = row0; base < row1; base += (int64_t)RPP * UPD_UNROLL) {
    LT w[UPD_UNROLL];
    int lab[UPD_UNROLL];
    float wt[UPD_UNROLL];
#pragma unroll
    for (int u = 0; u < UPD_UNROLL; ++u) {
      const int64_t i = base + (int64_t)u * RPP + lr;
      const bool ok = i < row1;
      const int l = ok ? a.labels[i] : -1;
      lab[u] = ((unsigned)l < (unsigned)a.K) ? l : -1;  // never index LDS out of range
      wt[u] = (ok && a.weights) ? a.weights[i] : 1.f;
      if (ok && colok) w[u] = *(const LT*)((const T*)a.X + i * a.ldx + col);
      else w[u] = LT{};
    }
#pragma unroll
    for (int u = 0; u < UPD_UNROLL; ++u) {
      if (lab[u] < 0) continue;
      float f[V];
      unpack_any<T, PB>(w[u], f);
      long long* dst = s + lab[u] * LD + lp * V;
      const float sc = a.weights ? wt[u] * scale : scale;
#pragma unroll
      for (int e = 0; e < V; ++e)
        __hip_atomic_fetch_add(dst + e, to_fixed(f[e], sc), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
      if (counter)
        __hip_atomic_fetch_add(cnt + lab[u], a.weights ? to_fixed(wt[u], cscale) : 1ll,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  }
  __syncthreads();

  // flush this slice: slab[chunk][k][slice*SW + c]
  const int cols = (a.D - slice * SW) < SW ? (a.D - slice * SW) : SW;
  long long* slab = a.slab + (int64_t)chunk * a.K * a.D + slice * SW;
  for (int e = threadIdx.x; e < a.K * SW; e += UPD_NT) {
    const int k = e / SW, c = e % SW;
    if (c < cols) slab[(int64_t)k * a.D + c] = s[k * LD + c];
  }
  if (slice == 0)
    for (int k = threadIdx.x; k < a.K; k += UPD_NT) a.cnt_slab[(int64_t)chunk * a.K + k] = cnt[k];
}

// Fallback for K too large to privatise even 2 columns: direct int64 global atomics
// (same fixed-point arithmetic, so results match the LDS path bit for bit).
template <typename T>
__global__ __launch_bounds__(256) void update_global_kernel(UpdateArgs a) {
  const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (i >= a.N) return;
  const int k = a.labels[i];
  if ((unsigned)k >= (unsigned)a.K) return;
  const float wt = a.weights ? a.weights[i] : 1.f;
  const float sc = ldexpf(1.f, a.sum_exp) * wt;
  const T* xr = (const T*)a.X + i * a.ldx;
  for (int d = lane; d < a.D; d += 64)
    atomicAdd((unsigned long long*)(a.slab + (int64_t)k * a.D + d),
              (unsigned long long)to_fixed(Elem<T>::to_f32(xr[d]), sc));
  if (lane == 0)
    atomicAdd((unsigned long long*)(a.cnt_slab + k),
              (unsigned long long)(a.weights ? to_fixed(wt, ldexpf(1.f, a.cnt_exp)) : 1ll));
}

static int esize(int dtype) { return dtype == DT_BF16 ? 2 : 4; }

static size_t upd_lds(int K, int sw, bool pad) { return (size_t)K * ((pad ? sw + 1 : sw) + 1) * 8; }

// returns slice width; *pad says whether the padded LDS stride fits
// Cap on the slice width (0 = none).  A smaller slice shrinks the LDS footprint
// so an update workgroup can be co-resident with assign workgroups when the
// engine overlaps the two kernels on separate streams.
static int g_update_max_sw = 0;
void set_update_max_sw(int sw) { g_update_max_sw = sw; }

static int choose_sw(int dtype, int K, int D, bool* pad) {
  const int es = esize(dtype);
  if ((D * es) % 4) return 0;
  int dp = 1;
  while (dp < D) dp *= 2;
  for (int sw = 64; sw >= 2; sw /= 2) {
    if (sw > dp && sw > 2) continue;
    if (g_update_max_sw && sw > g_update_max_sw) continue;
    if (upd_lds(K, sw, true) <= UPD_LDS_MAX) { *pad = true; return sw; }
    if (upd_lds(K, sw, false) <= UPD_LDS_MAX) { *pad = false; return sw; }
  }
  return 0;
}

int update_slice_width(int dtype, int K, int D) {
  bool pad;
  return choose_sw(dtype, K, D, &pad);
}

int update_n_chunks(int dtype, int K, int D, int64_t N) {
  const int sw = update_slice_width(dtype, K, D);
  if (sw == 0) return 1;
  const int n_slices = (D + sw - 1) / sw;
  // LDS-bound: one resident workgroup per CU; aim for ~1-2 waves of the 256 CUs
  int nc = (256 + n_slices - 1) / n_slices;
  nc = ((nc + 7) / 8) * 8;
  const int64_t rows = (N + nc - 1) / nc;
  if (rows < 256) {  // tiny problems: fewer chunks
    nc = (int)((N + 255) / 256);
    nc = ((nc + 7) / 8) * 8;
    if (nc < 8) nc = 8;
  }
  return nc;
}

int fixed_exp(double maxabs) {
  if (!(maxabs > 0) || !isfinite(maxabs)) return 0;
  int e = 30 - (int)ceil(log2(maxabs));
  while (e > -1000 && ldexp(maxabs, e) > 1073741824.0) --e;  // guard rounding of log2
  return e;
}

template <typename T, int SW, bool PAD>
static hipError_t launch_sw(const UpdateArgs& a, hipStream_t s) {
  const int n_slices = (a.D + SW - 1) / SW;
  const int64_t rows_per_chunk = (a.N + a.n_chunks - 1) / a.n_chunks;
  const size_t lds = upd_lds(a.K, SW, PAD);
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)update_kernel<T, SW, PAD>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)UPD_LDS_MAX);
    attr = true;
  }
  hipLaunchKernelGGL((update_kernel<T, SW, PAD>), dim3(a.n_chunks * n_slices), dim3(UPD_NT), lds,
                     s, a, n_slices, rows_per_chunk);
  return hipGetLastError();
}

template <typename T, int SW>
static hipError_t launch_pad(const UpdateArgs& a, hipStream_t s, bool pad) {
  return pad ? launch_sw<T, SW, true>(a, s) : launch_sw<T, SW, false>(a, s);
}

template <typename T>
static hipError_t launch_update_t(const UpdateArgs& a, hipStream_t s, int sw, bool pad) {
  switch (sw) {
    case 64: return launch_pad<T, 64>(a, s, pad);
    case 32: return launch_pad<T, 32>(a, s, pad);
    case 16: return launch_pad<T, 16>(a, s, pad);
    case 8: return launch_pad<T, 8>(a, s, pad);
    case 4: return launch_pad<T, 4>(a, s, pad);
    case 2: return launch_pad<T, 2>(a, s, pad);
    case 0:
      // caller zeroed slab[K*D] + cnt_slab[K] (n_chunks == 1)
      hipLaunchKernelGGL((update_global_kernel<T>), dim3((unsigned)((a.N + 3) / 4)), dim3(256), 0,
                         s, a);
      return hipGetLastError();
  }
  return hipErrorInvalidValue;
}

hipError_t launch_update(int dtype, const UpdateArgs& a, hipStream_t s) {
  if (a.N <= 0) return hipSuccess;
  bool pad = true;
  const int sw = choose_sw(dtype, a.K, a.D, &pad);
  if (sw > 0 && a.n_chunks % 8) return hipErrorInvalidValue;
  return dtype == DT_BF16 ? launch_update_t<uint16_t>(a, s, sw, pad)
                          : launch_update_t<float>(a, s, sw, pad);
}

// ---------------------------------------------------------------------------
// launch_reduce: packed[e] = 2^-exp * sum_c slab[c][e] (f64), counts likewise,
// plus the assign kernel's inertia / changed slots (which it then re-zeroes).
__global__ __launch_bounds__(256) void reduce_kernel(const long long* __restrict__ slab,
                                                     const long long* __restrict__ cnt_slab,
                                                     int n_chunks, int K, int D, double inv_s,
                                                     double inv_c, double* slots, double* packed) {
  const int64_t KD = (int64_t)K * D;
  const int64_t total = KD + K;
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e < total) {
    double acc = 0.0;
    if (e < KD) {
      for (int c = 0; c < n_chunks; ++c) acc += (double)slab[(int64_t)c * KD + e];
      acc *= inv_s;
    } else {
      const int64_t k = e - KD;
      for (int c = 0; c < n_chunks; ++c) acc += (double)cnt_slab[(int64_t)c * K + k];
      acc *= inv_c;
    }
    packed[e] = acc;
  }
  if (blockIdx.x == gridDim.x - 1) {
    __shared__ double red[4][2];
    double si = 0, sc = 0;
    if (slots) {
      for (int i = threadIdx.x; i < NSLOT; i += 256) {
        si += slots[i * SLOT_STRIDE + 0];
        sc += slots[i * SLOT_STRIDE + 1];
        slots[i * SLOT_STRIDE + 0] = 0.0;
        slots[i * SLOT_STRIDE + 1] = 0.0;
      }
    }
    si = wave_sum(si);
    sc = wave_sum(sc);
    if ((threadIdx.x & 63) == 0) { red[threadIdx.x >> 6][0] = si; red[threadIdx.x >> 6][1] = sc; }
    __syncthreads();
    if (threadIdx.x == 0) {
      packed[total + 0] = red[0][0] + red[1][0] + red[2][0] + red[3][0];
      packed[total + 1] = red[0][1] + red[1][1] + red[2][1] + red[3][1];
    }
  }
}

hipError_t launch_reduce(const long long* slab, const long long* cnt_slab, int n_chunks, int K,
                         int D, int sum_exp, int cnt_exp, double* slots, double* packed,
                         hipStream_t s) {
  const int64_t total = (int64_t)K * D + K;
  const unsigned nb = (unsigned)((total + 255) / 256);
  hipLaunchKernelGGL(reduce_kernel, dim3(nb), dim3(256), 0, s, slab, cnt_slab, n_chunks, K, D,
                     ldexp(1.0, -sum_exp), ldexp(1.0, -cnt_exp), slots, packed);
  return hipGetLastError();
}

}  // namespace mk
