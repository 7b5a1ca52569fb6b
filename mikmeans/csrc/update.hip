// mikmeans — K3: Lloyd M-step scatter-add (per-cluster sums and counts) for gfx950.
//
// sums[k,:] += x_i, counts[k] += 1 for k = labels[i].  Float atomics to HBM run
// at ~1.3 TB/s of added bytes chip-wide (MI355X_MICROARCH.md, Global float
// atomics): at N=1e8, D=128 a direct scatter would be 51 GB of atomics per
// iteration.  Instead every workgroup privatises a [K][SW(+1)] f32 slice of the
// sums in LDS (D split into column slices so the slice fits ~150 KiB of LDS),
// streams its contiguous chunk of rows with 16-byte loads, accumulates with
// LDS atomics (ds_add_f32), and flushes its slice once, with plain coalesced
// stores, into a per-chunk slab.  launch_reduce then sums the slabs in f64.
// The padding column (index SW) of each LDS row carries the counts.
//
// Grid mapping is XCD-aware: blocks b and b+8 share an XCD on MI355X, so the
// n_slices workgroups that read the same rows (different column slices of the
// same 128-B lines) are given block ids congruent mod 8 and meet in one L2.
//
// Reference parity: the reference's "update step" is re-deriving the dashboard
// after humans move cards (app.mjs:481-496 snapshotMetrics counts); counts here
// are exactly those per-centroid counts.
#include "common.h"
#include "kernels.h"

namespace mk {

constexpr int UPD_NT = 512;
constexpr int UPD_UNROLL = 4;
constexpr size_t UPD_LDS_BUDGET = 150 * 1024;

template <typename T, int SW>
__global__ __launch_bounds__(UPD_NT) void update_kernel(UpdateArgs a, int n_slices,
                                                        int64_t rows_per_chunk) {
  constexpr int V = Elem<T>::V;
  constexpr int LPR = SW / V;           // lanes per row
  constexpr int RPP = UPD_NT / LPR;     // rows per pass
  constexpr int LD = SW + 1;            // LDS row stride (last column = count)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* s = (float*)smem;

  const int b = blockIdx.x;
  const int j = b >> 3;
  const int slice = j % n_slices;
  const int chunk = (j / n_slices) * 8 + (b & 7);

  for (int e = threadIdx.x; e < a.K * LD; e += UPD_NT) s[e] = 0.f;
  __syncthreads();

  const int64_t row0 = (int64_t)chunk * rows_per_chunk;
  int64_t row1 = row0 + rows_per_chunk;
  if (row1 > a.N) row1 = a.N;
  const int lr = threadIdx.x / LPR, lp = threadIdx.x % LPR;
  const int col = slice * SW + lp * V;
  const bool colok = col < a.D;
  const bool counter = (slice == 0) && (lp == 0);

  for (int64_t base = row0; base < row1; base += (int64_t)RPP * UPD_UNROLL) {
    u32x4 w[UPD_UNROLL];
    int lab[UPD_UNROLL];
    float wt[UPD_UNROLL];
#pragma unroll
    for (int u = 0; u < UPD_UNROLL; ++u) {
      const int64_t i = base + (int64_t)u * RPP + lr;
      const bool ok = i < row1;
      const int l = ok ? a.labels[i] : -1;
      lab[u] = ((unsigned)l < (unsigned)a.K) ? l : -1;  // never index LDS out of range
      wt[u] = (ok && a.weights) ? a.weights[i] : 1.f;
      if (ok && colok) w[u] = *(const u32x4*)((const T*)a.X + i * a.ldx + col);
      else w[u] = u32x4{0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int u = 0; u < UPD_UNROLL; ++u) {
      if (lab[u] < 0) continue;
      float f[V];
      unpack16(w[u], f, (T*)nullptr);
      float* dst = s + lab[u] * LD + lp * V;
#pragma unroll
      for (int e = 0; e < V; ++e)
        __hip_atomic_fetch_add(dst + e, f[e] * wt[u], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      if (counter)
        __hip_atomic_fetch_add(s + lab[u] * LD + SW, wt[u], __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  }
  __syncthreads();

  // flush this slice: slab[chunk][k][slice*SW + c]
  const int cols = (a.D - slice * SW) < SW ? (a.D - slice * SW) : SW;
  float* slab = a.slab + (int64_t)chunk * a.K * a.D + slice * SW;
  for (int e = threadIdx.x; e < a.K * SW; e += UPD_NT) {
    const int k = e / SW, c = e % SW;
    if (c < cols) slab[(int64_t)k * a.D + c] = s[k * LD + c];
  }
  if (slice == 0)
    for (int k = threadIdx.x; k < a.K; k += UPD_NT)
      a.cnt_slab[(int64_t)chunk * a.K + k] = s[k * LD + SW];
}

// Fallback for K too large to privatise even 8 columns: direct f32 atomics.
template <typename T>
__global__ __launch_bounds__(256) void update_global_kernel(UpdateArgs a) {
  const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (i >= a.N) return;
  const int k = a.labels[i];
  const float wt = a.weights ? a.weights[i] : 1.f;
  const T* xr = (const T*)a.X + i * a.ldx;
  for (int d = lane; d < a.D; d += 64)
    atomicAdd(a.slab + (int64_t)k * a.D + d, Elem<T>::to_f32(xr[d]) * wt);
  if (lane == 0) atomicAdd(a.cnt_slab + k, wt);
}

static int elem_v(int dtype) { return dtype == DT_BF16 ? 8 : 4; }

int update_slice_width(int dtype, int K, int D) {
  const int v = elem_v(dtype);
  if (D % v) return 0;
  int dp = v;
  while (dp < D) dp *= 2;  // slices never exceed the (pow2-padded) row
  for (int sw = 128; sw >= v; sw /= 2) {
    if (sw > dp) continue;
    if ((size_t)K * (sw + 1) * 4 <= UPD_LDS_BUDGET) return sw;
  }
  return 0;
}

int update_n_chunks(int dtype, int K, int D, int64_t N) {
  const int sw = update_slice_width(dtype, K, D);
  if (sw == 0) return 1;
  const int n_slices = (D + sw - 1) / sw;
  // one resident workgroup per CU (LDS-bound); aim for ~2 waves of the 256 CUs
  int nc = (512 + n_slices - 1) / n_slices;
  nc = ((nc + 7) / 8) * 8;
  // keep per-chunk row counts exact in f32 counts (< 2^24)
  while ((N + nc - 1) / nc >= (1 << 24)) nc += 8;
  int64_t rows = (N + nc - 1) / nc;
  if (rows < 64) {  // tiny problems: fewer chunks
    nc = (int)((N + 63) / 64);
    nc = ((nc + 7) / 8) * 8;
    if (nc < 8) nc = 8;
  }
  return nc;
}

template <typename T, int SW>
static hipError_t launch_sw(const UpdateArgs& a, hipStream_t s) {
  const int n_slices = (a.D + SW - 1) / SW;
  const int64_t rows_per_chunk = (a.N + a.n_chunks - 1) / a.n_chunks;
  const size_t lds = (size_t)a.K * (SW + 1) * 4;
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)update_kernel<T, SW>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  hipLaunchKernelGGL((update_kernel<T, SW>), dim3(a.n_chunks * n_slices), dim3(UPD_NT), lds, s, a,
                     n_slices, rows_per_chunk);
  return hipGetLastError();
}

template <typename T>
static hipError_t launch_update_t(const UpdateArgs& a, hipStream_t s, int sw) {
  switch (sw) {
    case 128: return launch_sw<T, 128>(a, s);
    case 64: return launch_sw<T, 64>(a, s);
    case 32: return launch_sw<T, 32>(a, s);
    case 16: return launch_sw<T, 16>(a, s);
    case 8: return launch_sw<T, 8>(a, s);
    case 4:
      if constexpr (Elem<T>::V <= 4) return launch_sw<T, 4>(a, s);
      break;
    case 0: {
      // caller zeroed slab[K*D] + cnt_slab[K] (n_chunks == 1)
      hipLaunchKernelGGL((update_global_kernel<T>), dim3((unsigned)((a.N + 3) / 4)), dim3(256), 0,
                         s, a);
      return hipGetLastError();
    }
  }
  return hipErrorInvalidValue;
}

hipError_t launch_update(int dtype, const UpdateArgs& a, hipStream_t s) {
  if (a.N <= 0) return hipSuccess;
  const int sw = update_slice_width(dtype, a.K, a.D);
  if (sw > 0 && a.n_chunks % 8) return hipErrorInvalidValue;
  return dtype == DT_BF16 ? launch_update_t<uint16_t>(a, s, sw) : launch_update_t<float>(a, s, sw);
}

// ---------------------------------------------------------------------------
// launch_reduce: packed[e] = sum_c slab[c][e] (f64), counts likewise, and the
// assign kernel's inertia / changed slots (which it then re-zeroes).
__global__ __launch_bounds__(256) void reduce_kernel(const float* __restrict__ slab,
                                                     const float* __restrict__ cnt_slab,
                                                     int n_chunks, int K, int D, double* slots,
                                                     double* packed) {
  const int64_t KD = (int64_t)K * D;
  const int64_t total = KD + K;
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e < total) {
    double acc = 0.0;
    if (e < KD) {
      for (int c = 0; c < n_chunks; ++c) acc += (double)slab[(int64_t)c * KD + e];
    } else {
      const int64_t k = e - KD;
      for (int c = 0; c < n_chunks; ++c) acc += (double)cnt_slab[(int64_t)c * K + k];
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

hipError_t launch_reduce(const float* slab, const float* cnt_slab, int n_chunks, int K, int D,
                         double* slots, double* packed, hipStream_t s) {
  const int64_t total = (int64_t)K * D + K;
  const unsigned nb = (unsigned)((total + 255) / 256);
  hipLaunchKernelGGL(reduce_kernel, dim3(nb), dim3(256), 0, s, slab, cnt_slab, n_chunks, K, D,
                     slots, packed);
  return hipGetLastError();
}

}  // namespace mk
