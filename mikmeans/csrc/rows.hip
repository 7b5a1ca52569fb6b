// mikmeans — row-level helper kernels for gfx950: the device mini-batch sampler, in-place
// row normalisation (cosine metric) and a weighted dot product (weighted inertia).
//
// sample_rows: batch row j of step s on rank r is source row
//   idx = floor(u * n),  u = (philox(j, s, r, TAG_SMP; seed) as a 64-bit word >> 11) * 2^-53
// (with replacement, clamped to n-1), a pure function of (seed, rank, step, j): the
// sampler's whole state is the step counter, so a resumed fit draws the rows the
// uninterrupted one would, and the host (NumPy, mikmeans/data/sampler.py) reproduces the
// indices for shards that live in host memory.  The kernel gathers the rows (16-B
// pieces, TPR lanes per row) and writes their squared norms (of the stored values) for
// the assign kernel's inertia -- one read of each sampled row and one write of the batch,
// the same bytes the blob generator writes for a streamed batch.
//
// Reference parity: the reference's "Shuffle unassigned" (app.mjs:159-166, Fisher-Yates
// over the cards) is its only random selection of points; mini-batch sampling is the
// numeric framework's use of it.
#include "common.h"
#include "kernels.h"

namespace mk {

constexpr uint32_t TAG_SMP = 0x53414D50u;  // "SAMP"

__device__ __forceinline__ int64_t sample_index(int64_t j, uint32_t step, uint32_t rank, int64_t n,
                                                uint32_t k0, uint32_t k1) {
  const U4 r = philox(U4{(uint32_t)j, step, rank, TAG_SMP}, k0, k1);
  const uint64_t w = ((uint64_t)r.y << 32) | r.x;
  const double u = (double)(w >> 11) * 0x1p-53;
  const int64_t i = (int64_t)(u * (double)n);
  return i < n ? i : n - 1;
}

template <typename T, int TPR>
__global__ __launch_bounds__(256) void sample_rows_kernel(const T* __restrict__ X, int64_t n, int64_t ldx,
                                                          int NP, T* __restrict__ out, int64_t ldo,
                                                          int64_t b, uint32_t k0, uint32_t k1,
                                                          uint32_t rank, uint32_t step, float* xn,
                                                          int64_t* idx_out) {
  constexpr int V = Elem<T>::V;
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t j = e / TPR;
  const int t = (int)(e % TPR);
  const bool ok = j < b;
  int64_t src = 0;
  if (t == 0 && ok) src = sample_index(j, step, rank, n, k0, k1);
  // broadcast within the row's lanes (TPR divides 64)
  const int leader = (int)(threadIdx.x & 63) & ~(TPR - 1);
  src = ((int64_t)__shfl((int)(uint32_t)src, leader, 64) & 0xffffffffll) |
        ((int64_t)__shfl((int)(src >> 32), leader, 64) << 32);
  float sq = 0.f;
  if (ok) {
    if (idx_out && t == 0) idx_out[j] = src;
    const T* rp = X + src * ldx;
    T* op = out + j * ldo;
    for (int p = t; p < NP; p += TPR) {
      const u32x4 w = *(const u32x4*)(rp + p * V);
      float f[V];
      unpack16(w, f, (T*)nullptr);
#pragma unroll
      for (int q = 0; q < V; ++q) sq = __builtin_fmaf(f[q], f[q], sq);
      *(u32x4*)(op + p * V) = w;
    }
  }
  if (xn) {
#pragma unroll
    for (int o = 1; o < TPR; o <<= 1) sq += __shfl_xor(sq, o, 64);
    if (ok && t == 0) xn[j] = sq;
  }
}

hipError_t launch_sample_rows(int dtype, const void* X, int64_t n, int64_t ldx, int D, void* out,
                              int64_t ldo, int64_t b, uint64_t seed, uint32_t rank, uint32_t step,
                              float* xn, int64_t* idx_out, hipStream_t s) {
  if (b <= 0) return hipSuccess;
  if (n <= 0) return hipErrorInvalidValue;
  const int V = dtype == DT_BF16 ? 8 : 4;
  if (D % V) return hipErrorInvalidValue;
  const int NP = D / V;
  int tpr = 1;
  while (tpr < NP && tpr < 16) tpr *= 2;
  const int64_t tot = b * tpr;
  const dim3 g((unsigned)((tot + 255) / 256)), blk(256);
  const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#define MK_SMP(TT, TP)                                                                           \
  hipLaunchKernelGGL((sample_rows_kernel<TT, TP>), g, blk, 0, s, (const TT*)X, n, ldx, NP, (TT*)out, \
                     ldo, b, k0, k1, rank, step, xn, idx_out)
#define MK_SMP_T(TT)                                                                             \
  switch (tpr) {                                                                                 \
    case 1: MK_SMP(TT, 1); break;                                                                \
    case 2: MK_SMP(TT, 2); break;                                                                \
    case 4: MK_SMP(TT, 4); break;                                                                \
    case 8: MK_SMP(TT, 8); break;                                                                \
    default: MK_SMP(TT, 16); break;                                                              \
  }
  if (dtype == DT_BF16) { MK_SMP_T(uint16_t) } else { MK_SMP_T(float) }
#undef MK_SMP_T
#undef MK_SMP
  return hipGetLastError();
}

__global__ __launch_bounds__(256) void sample_index_kernel(int64_t n, int64_t b, uint32_t k0, uint32_t k1,
                                                           uint32_t rank, uint32_t step, int64_t* idx) {
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j < b) idx[j] = sample_index(j, step, rank, n, k0, k1);
}

hipError_t launch_sample_index(int64_t n, int64_t b, uint64_t seed, uint32_t rank, uint32_t step, int64_t* idx,
                               hipStream_t s) {
  if (b <= 0) return hipSuccess;
  if (n <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(sample_index_kernel, dim3((unsigned)((b + 255) / 256)), dim3(256), 0, s, n, b,
                     (uint32_t)seed, (uint32_t)(seed >> 32), rank, step, idx);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// In-place unit rows: x <- x / max(|x|, 1e-30), f32 arithmetic (norm of the stored values,
// IEEE sqrt and division), rounded back to the storage type; xn (optional) receives the
// squared norm of the rounded row.  16 lanes per row.
template <typename T>
__global__ __launch_bounds__(256) void row_normalize_kernel(T* X, int64_t N, int NP, int64_t ldx, float* xn) {
  constexpr int V = Elem<T>::V;
  const int sub = threadIdx.x & 15;
  const int64_t i = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 4);
  const bool ok = i < N;
  T* row = X + (ok ? i : 0) * ldx;
  float s = 0.f;
  if (ok)
    for (int p = sub; p < NP; p += 16) {
      float f[V];
      unpack16(*(const u32x4*)(row + p * V), f, (T*)nullptr);
#pragma unroll
      for (int q = 0; q < V; ++q) s = __builtin_fmaf(f[q], f[q], s);
    }
  s = sum16_xor(s);
  const float nrm = fmaxf(sqrtf(s), 1e-30f);
  float s2 = 0.f;
  if (ok)
    for (int p = sub; p < NP; p += 16) {
      float f[V];
      unpack16(*(const u32x4*)(row + p * V), f, (T*)nullptr);
      T h[V];
#pragma unroll
      for (int q = 0; q < V; ++q) {
        h[q] = Elem<T>::from_f32(f[q] / nrm);
        const float r = Elem<T>::to_f32(h[q]);
        s2 = __builtin_fmaf(r, r, s2);
      }
      *(u32x4*)(row + p * V) = *(const u32x4*)h;
    }
  if (xn) {
    s2 = sum16_xor(s2);
    if (ok && sub == 0) xn[i] = s2;
  }
}

hipError_t launch_row_normalize(int dtype, void* X, int64_t N, int D, int64_t ldx, float* xn, hipStream_t s) {
  if (N <= 0) return hipSuccess;
  const int V = dtype == DT_BF16 ? 8 : 4;
  if (D % V) return hipErrorInvalidValue;
  const dim3 g((unsigned)((N + 15) / 16)), b(256);
  if (dtype == DT_BF16)
    hipLaunchKernelGGL(row_normalize_kernel<uint16_t>, g, b, 0, s, (uint16_t*)X, N, D / V, ldx, xn);
  else
    hipLaunchKernelGGL(row_normalize_kernel<float>, g, b, 0, s, (float*)X, N, D / V, ldx, xn);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// out[0] += sum_i a[i] * b[i] in f64 (weighted inertia: a = squared distances, b = weights).
// Deterministic: a fixed grid of WDOT_BLOCKS blocks writes per-block partials (each summed
// in a fixed order), and one block adds them in index order -- the same bits on every run,
// so a hipGraph replay reproduces the eager step exactly.
constexpr int WDOT_BLOCKS = 1024;

__global__ __launch_bounds__(256) void wdot_partial_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                           int64_t n, double* __restrict__ part) {
  double acc = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    acc += (double)a[i] * (double)b[i];
  acc = wave_sum(acc);
  __shared__ double red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ __launch_bounds__(256) void wdot_final_kernel(const double* __restrict__ part, int nb, double* out) {
  double acc = 0.0;
  for (int i = threadIdx.x; i < nb; i += 256) acc += part[i];
  acc = wave_sum(acc);
  __shared__ double red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) out[0] += (red[0] + red[1]) + (red[2] + red[3]);
}

int wdot_scratch_len() { return WDOT_BLOCKS; }

hipError_t launch_wdot(const float* a, const float* b, int64_t n, double* out, double* scratch, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  int64_t nb = (n + 255) / 256;
  if (nb > WDOT_BLOCKS) nb = WDOT_BLOCKS;
  hipLaunchKernelGGL(wdot_partial_kernel, dim3((unsigned)nb), dim3(256), 0, s, a, b, n, scratch);
  hipLaunchKernelGGL(wdot_final_kernel, dim3(1), dim3(256), 0, s, scratch, (int)nb, out);
  return hipGetLastError();
}

// ---- Hamerly bounds ----------------------------------------------------------------------
// ub / lb bound the distances of a row to its label's centre and to every other centre -- the
// QUANTISED centres the assign ranks (bf16 rounding of the f32 centres; the f32 centres
// themselves for f32 points), moved each step by the quantised centres' own shifts (finalize
// qshift), so the bounds carry no quantisation term.  The assign writes raw kernel distances
// (sqrt of its scores); the step after, while cand[i] still marks the row as freshly assigned,
// they are widened once by the scores' rounding slack (score_slack) -- sqrt(d^2 +- slack),
// which costs slack / 2d, not sqrt(slack).  Every later step only adds the shifts.
//
// Skipping a row must leave the label the FULL assign would give it (models/lloyd.py: the
// bounded E-step's iterates are bitwise the full E-step's), not merely the nearest centre: the
// full pass ranks rounded scores with 6-bit key truncation.  Its score for the label is at most
// u^2 + slack and every other score at least l^2 - slack, so the row is skipped only where the
// first is below the second -- the slack counted once more, on both sides (keys_keep_label).
//
// The slack of a score of row i (squared-distance units): its accumulation -- the seed
// |c|^2 + o_i and `nterms` exact bf16 (f32: rounded-once) products -- errs by at most
// 2 (nterms + 8) 2^-24 of the sum of the terms' magnitudes |c|^2 + o_i + 2|x||c| (recursive
// summation in any order, directed rounding allowed, plus the store's own roundings); the key
// truncation by 2^-17 of the key d^2 + o_i - |x_i|^2, counted twice.  o_i is the row's
// full-pass seed offset (AssignArgs::oseed; 0 for f32).
struct RowSlack {
  float acc, ex;   // accumulation term, |o_i - |x_i|^2|
  __device__ __forceinline__ float operator()(float d2) const { return acc + 1.52587890625e-05f * (d2 + ex); }
};

__device__ __forceinline__ RowSlack row_slack(float xn, float o, float cmax, float eacc) {
  return RowSlack{eacc * (cmax * cmax + o + 2.f * sqrtf(xn) * cmax), fabsf(o - xn)};
}

__device__ __forceinline__ float slack_eacc(int nterms) { return 2.f * (float)(nterms + 8) * 5.9604645e-08f; }

__device__ __forceinline__ bool keys_keep_label(float u, float l, const RowSlack& sl) {
  const float uu = u * u, ll = l * l;
  return l > 0.f && uu + sl(uu) < ll - sl(ll);   // (false for u = inf, NaN)
}

// One workgroup: the largest and second-largest centre shift, the largest's centre, and the
// largest |c|^2 (the slack's centre term) -> work[0..3].
__global__ __launch_bounds__(1024) void shift_top2_kernel(const float* __restrict__ shift2,
                                                         const float* __restrict__ cn, int K,
                                                         float* __restrict__ work) {
  float a1 = -1.f, a2 = -1.f, cm = 0.f;
  int i1 = -1;
  for (int k = threadIdx.x; k < K; k += 1024) {
    const float d = sqrtf(fmaxf(shift2[k], 0.f));
    if (d > a1) { a2 = a1; a1 = d; i1 = k; } else if (d > a2) { a2 = d; }
    cm = fmaxf(cm, cn[k]);
  }
  __shared__ float s1[1024], s2[1024], sc[1024];
  __shared__ int si[1024];
  s1[threadIdx.x] = a1; s2[threadIdx.x] = a2; si[threadIdx.x] = i1; sc[threadIdx.x] = cm;
  __syncthreads();
  for (int o = 512; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      const int j = threadIdx.x + o;
      const float b1 = s1[j], b2 = s2[j], x1 = s1[threadIdx.x], x2 = s2[threadIdx.x];
      const bool take = b1 > x1 || (b1 == x1 && si[j] >= 0 && (si[threadIdx.x] < 0 || si[j] < si[threadIdx.x]));
      s1[threadIdx.x] = take ? b1 : x1;
      s2[threadIdx.x] = fmaxf(fminf(x1, b1), fmaxf(x2, b2));
      si[threadIdx.x] = take ? si[j] : si[threadIdx.x];
      sc[threadIdx.x] = fmaxf(sc[threadIdx.x], sc[j]);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    work[0] = fmaxf(s1[0], 0.f);
    work[1] = fmaxf(s2[0], 0.f);
    work[2] = __int_as_float(si[0]);
    work[3] = sc[0];
  }
}

__global__ __launch_bounds__(256) void bounds_update_kernel(const int32_t* __restrict__ labels,
                                                           float* __restrict__ ub, float* __restrict__ lb,
                                                           const float* __restrict__ shift2,
                                                           const float* __restrict__ xn, int64_t n,
                                                           uint8_t* __restrict__ cand,
                                                           const float* __restrict__ work,
                                                           const float* __restrict__ oseed, int nterms) {
  const float d1 = work[0], d2 = work[1];
  const int a1 = __float_as_int(work[2]);
  // |c|max over the centres the last E-step ranked and the moved ones the pack now holds
  const float cmax = sqrtf(work[3]) + d1;
  const float eacc = slack_eacc(nterms);
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int a = labels[i];
    if (a < 0) { cand[i] = 1; continue; }       // unassigned: a full assign decides
    const RowSlack sl = row_slack(xn[i], oseed ? oseed[i] : 0.f, cmax, eacc);
    float u = ub[i], l = lb[i];
    if (cand[i]) {                               // raw kernel distances: widen them once
      const float uu = u * u, ll = l * l;
      u = sqrtf(uu + sl(uu));
      l = sqrtf(fmaxf(ll - sl(ll), 0.f));
    }
    u += sqrtf(fmaxf(shift2[a], 0.f));
    l -= (a == a1 ? d2 : d1);
    ub[i] = u;
    lb[i] = l;
    cand[i] = keys_keep_label(u, l, sl) ? 0 : 1;
  }
}

// ---- seed offsets of the full assign ------------------------------------------------------
// The full assign seeds a bf16 workgroup's scores with o = (1 + 2^-12) max |x|^2 over its block
// of block_rows rows, or each row's own (1 + 2^-12) |x|^2 where the block's max exceeds 4x its
// min (assign16.hip, the kernel's prologue: the same fmaxf / fminf folds from 0 / 3e38, the
// same fma).  The offset is part of every key, so near-ties resolve by it; a gathered assign
// seeded from this array (AssignArgs::oseed) ranks each row bitwise as the full pass does.
// One workgroup per block; a tail block's missing rows are the kernel's clamped copies of
// row n-1, which change neither extreme.
__global__ __launch_bounds__(256) void seed_offsets_kernel(const float* __restrict__ xn, int64_t n, int block_rows,
                                                          float* __restrict__ oseed) {
  const int64_t r0 = (int64_t)blockIdx.x * block_rows;
  const int64_t r1 = r0 + block_rows < n ? r0 + block_rows : n;
  float m = 0.f, mn = 3.0e38f;
  for (int64_t i = r0 + threadIdx.x; i < r1; i += 256) {
    m = fmaxf(m, xn[i]);
    mn = fminf(mn, xn[i]);
  }
  __shared__ float sm[256], sn[256];
  sm[threadIdx.x] = m;
  sn[threadIdx.x] = mn;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      sm[threadIdx.x] = fmaxf(sm[threadIdx.x], sm[threadIdx.x + o]);
      sn[threadIdx.x] = fminf(sn[threadIdx.x], sn[threadIdx.x + o]);
    }
    __syncthreads();
  }
  const float mx = sm[0];
  const bool ppo = mx > 4.f * sn[0];
  const float off = __builtin_fmaf(mx, 2.44140625e-04f, mx);   // * (1 + 2^-12)
  for (int64_t i = r0 + threadIdx.x; i < r1; i += 256)
    oseed[i] = ppo ? __builtin_fmaf(xn[i], 2.44140625e-04f, xn[i]) : off;
}

hipError_t launch_seed_offsets(const float* xn, int64_t n, int block_rows, float* oseed, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  if (block_rows <= 0) return hipErrorInvalidValue;
  const int64_t nb = (n + block_rows - 1) / block_rows;
  if (nb > 0x7fffffff) return hipErrorInvalidValue;
  hipLaunchKernelGGL(seed_offsets_kernel, dim3((unsigned)nb), dim3(256), 0, s, xn, n, block_rows, oseed);
  return hipGetLastError();
}

hipError_t launch_bounds_update(const int32_t* labels, float* ub, float* lb, const float* shift2, const float* cn,
                                int K, const float* xn, int64_t n, uint8_t* cand, float* work, const float* oseed,
                                int nterms, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  if (K < 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(shift_top2_kernel, dim3(1), dim3(1024), 0, s, shift2, cn, K, work);
  int64_t nb = (n + 255) / 256;
  if (nb > 8192) nb = 8192;
  hipLaunchKernelGGL(bounds_update_kernel, dim3((unsigned)nb), dim3(256), 0, s, labels, ub, lb, shift2, xn, n,
                     cand, work, oseed, nterms);
  return hipGetLastError();
}

// ---- Hamerly tightening ----------------------------------------------------------------
// A row whose moved bounds no longer prove its label first gets the exact distance to its
// label's (quantised) centre (Hamerly 2010's second test): ub drops to it, and a row whose tight ub
// passes the bounds test against lb (keys_keep_label) keeps its label without the assign.  A wave takes 4 rows per pass, 16
// lanes per row in 16-B pieces (one coalesced load per piece), |x - c|^2 summed directly
// (no |x|^2 + |c|^2 cancellation).  rows[0..*count): the compacted candidates.
template <typename T>
__global__ __launch_bounds__(256) void tighten_kernel(const T* __restrict__ X, int64_t ldx, int D,
                                                     const int32_t* __restrict__ labels,
                                                     const float* __restrict__ C, int64_t ldc,
                                                     const int64_t* __restrict__ rows,
                                                     const int64_t* __restrict__ count, float* __restrict__ ub,
                                                     const float* __restrict__ lb, uint8_t* __restrict__ cand,
                                                     const float* __restrict__ xn, const float* __restrict__ work,
                                                     const float* __restrict__ oseed, int nterms) {
  constexpr int V = Elem<T>::V;
  const int64_t m = count[0];
  // the slack terms of this step's bounds test (bounds_update_kernel)
  const float cmax = sqrtf(work[3]) + work[0];
  const float eacc = slack_eacc(nterms);
  const int lane = threadIdx.x & 63, grp = lane >> 4, gl = lane & 15;
  const int64_t wave = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  const int64_t nwave = ((int64_t)gridDim.x * 256) >> 6;
  const int pieces = (D + V - 1) / V;
  for (int64_t base = wave * 4; base < m; base += nwave * 4) {   // (wave-uniform loop)
    const int64_t j = base + grp;
    int64_t row = 0;
    int a = -1;
    if (j < m) {
      row = rows[j];
      a = labels[row];
    }
    float s = 0.f;
    if (a >= 0) {
      const T* xp = X + row * ldx;
      const float* cp = C + (int64_t)a * ldc;
      for (int p = gl; p < pieces; p += 16) {
        float f[V];
        unpack16(*(const u32x4*)(xp + p * V), f, (T*)nullptr);
#pragma unroll
        for (int q = 0; q < V; ++q) {
          const int col = p * V + q;
          if (col < D) {
            // (bf16 points: the bf16-rounded centre the assign ranks, as the bounds are)
            const float c = sizeof(T) == 2 ? round_bf16(cp[col]) : cp[col];
            const float d = f[q] - c;
            s = __builtin_fmaf(d, d, s);
          }
        }
      }
    }
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);   // (within the 16-lane group)
    if (gl == 0 && a >= 0) {
      const float u = __builtin_sqrtf(s) * (1.f + 1e-6f);   // (+ the f32 rounding of D terms)
      ub[row] = u;
      if (keys_keep_label(u, lb[row], row_slack(xn[row], oseed ? oseed[row] : 0.f, cmax, eacc))) cand[row] = 0;
    }
  }
}

hipError_t launch_tighten(int dtype, const void* X, int64_t ldx, int D, const int32_t* labels, const float* C,
                          int64_t ldc, const int64_t* rows, const int64_t* count, int64_t n_max, float* ub,
                          const float* lb, uint8_t* cand, const float* xn, const float* work, const float* oseed,
                          hipStream_t s) {
  if (n_max <= 0) return hipSuccess;
  int64_t nb = (n_max + 15) / 16;   // 16 rows per block and pass
  if (nb > 8192) nb = 8192;
  if (dtype == DT_BF16)
    hipLaunchKernelGGL(tighten_kernel<uint16_t>, dim3((unsigned)nb), dim3(256), 0, s, (const uint16_t*)X, ldx, D,
                       labels, C, ldc, rows, count, ub, lb, cand, xn, work, oseed, D);
  else
    hipLaunchKernelGGL(tighten_kernel<float>, dim3((unsigned)nb), dim3(256), 0, s, (const float*)X, ldx, D, labels,
                       C, ldc, rows, count, ub, lb, cand, xn, work, oseed, D);
  return hipGetLastError();
}

// ---- candidate compaction ----------------------------------------------------------------
// rows[0..count) = the indices i with cand[i] != 0, ascending; count stays on the device.
// Three launches, no atomics (so the order -- and with it each row's workgroup in the
// gathered assign that follows -- is the same every run): per-block counts of 4096 flags,
// one workgroup's exclusive scan of those counts, and a write pass whose threads place
// their 16 flags' rows after the block offset plus an in-block scan.
constexpr int CMP_T = 256, CMP_R = 16, CMP_ROWS = CMP_T * CMP_R;

__device__ __forceinline__ int flags16(const uint8_t* __restrict__ cand, int64_t base, int64_t n, unsigned& bits) {
  bits = 0u;
  if (base + CMP_R <= n) {
    const uint4 w = *(const uint4*)(cand + base);
    const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int b = 0; b < 4; ++b) bits |= ((ws[q] >> (8 * b)) & 0xffu) ? (1u << (4 * q + b)) : 0u;
  } else {
    for (int j = 0; j < CMP_R; ++j)
      if (base + j < n && cand[base + j]) bits |= 1u << j;
  }
  return __builtin_popcount(bits);
}

__global__ __launch_bounds__(CMP_T) void compact_count_kernel(const uint8_t* __restrict__ cand, int64_t n,
                                                           int64_t* __restrict__ bcnt) {
  unsigned bits;
  int c = flags16(cand, (int64_t)blockIdx.x * CMP_ROWS + threadIdx.x * CMP_R, n, bits);
  c = wave_sum(c);
  __shared__ int ws[CMP_T / 64];
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    int t = 0;
#pragma unroll
    for (int w = 0; w < CMP_T / 64; ++w) t += ws[w];
    bcnt[blockIdx.x] = t;
  }
}

// inclusive scan of one value per thread over a workgroup of T threads (T / 64 waves)
template <int T>
__device__ __forceinline__ int64_t block_incl_scan(int64_t v, int64_t* lds_waves) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int64_t u = __shfl_up(v, o, 64);
    if (lane >= o) v += u;
  }
  if (lane == 63) lds_waves[w] = v;
  __syncthreads();
  int64_t before = 0;
  for (int j = 0; j < w; ++j) before += lds_waves[j];
  __syncthreads();   // (lds_waves is reused by the caller's next scan)
  return v + before;
}

__global__ __launch_bounds__(1024) void compact_scan_kernel(int64_t* __restrict__ bcnt, int64_t nb,
                                                         int64_t* __restrict__ count) {
  __shared__ int64_t wsum[16];
  __shared__ int64_t tot;
  int64_t carry = 0;
  for (int64_t s0 = 0; s0 < nb; s0 += 1024) {
    const int64_t i = s0 + threadIdx.x;
    const int64_t v = i < nb ? bcnt[i] : 0;
    const int64_t incl = block_incl_scan<1024>(v, wsum);
    if (i < nb) bcnt[i] = carry + incl - v;   // exclusive offset
    if (threadIdx.x == 1023) tot = incl;      // this slice's total
    __syncthreads();
    carry += tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) count[0] = carry;
}

__global__ __launch_bounds__(CMP_T) void compact_write_kernel(const uint8_t* __restrict__ cand, int64_t n,
                                                           const int64_t* __restrict__ boff,
                                                           int64_t* __restrict__ rows) {
  __shared__ int64_t wsum[CMP_T / 64];
  const int64_t base = (int64_t)blockIdx.x * CMP_ROWS + threadIdx.x * CMP_R;
  unsigned bits;
  const int c = flags16(cand, base, n, bits);
  const int64_t incl = block_incl_scan<CMP_T>((int64_t)c, wsum);
  int64_t pos = boff[blockIdx.x] + incl - c;
  while (bits) {
    const int j = __builtin_ctz(bits);
    bits &= bits - 1u;
    rows[pos++] = base + j;
  }
}

int64_t compact_blocks(int64_t n) { return (n + CMP_ROWS - 1) / CMP_ROWS; }

hipError_t launch_compact(const uint8_t* cand, int64_t n, int64_t* rows, int64_t* count, int64_t* bscratch,
                          hipStream_t s) {
  const int64_t nb = compact_blocks(n);
  if (nb <= 0) {
    hipLaunchKernelGGL(compact_scan_kernel, dim3(1), dim3(1024), 0, s, bscratch, (int64_t)0, count);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(compact_count_kernel, dim3((unsigned)nb), dim3(CMP_T), 0, s, cand, n, bscratch);
  hipLaunchKernelGGL(compact_scan_kernel, dim3(1), dim3(1024), 0, s, bscratch, nb, count);
  hipLaunchKernelGGL(compact_write_kernel, dim3((unsigned)nb), dim3(CMP_T), 0, s, cand, n, bscratch, rows);
  return hipGetLastError();
}

// ---- k-means|| oversampling (models/init.py init_kmeans_parallel) ---------------------------
// Global row g is a candidate of round r when u_g < ell * d2_g / psi, u_g the 53-bit uniform
// of philox(g_lo, g_hi, r, TAG_KPAR; seed): a pure function of the global row, so the
// candidates do not depend on how rows are sharded.  psi (f64) stays on the device.  The
// NumPy mirror (data/sampler.py kpar_uniform) draws the same u.
constexpr uint32_t TAG_KPAR = 0x4B504152u;  // "KPAR"

__global__ __launch_bounds__(256) void kpar_select_kernel(const float* __restrict__ d2, int64_t n, int64_t start,
                                                        const double* __restrict__ psi, double ell, uint32_t k0,
                                                        uint32_t k1, uint32_t round, uint8_t* __restrict__ cand) {
  const double ps = psi[0];
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const uint64_t g = (uint64_t)(start + i);
    const U4 r = philox(U4{(uint32_t)g, (uint32_t)(g >> 32), round, TAG_KPAR}, k0, k1);
    const uint64_t w = ((uint64_t)r.y << 32) | r.x;
    const double u = (double)(w >> 11) * 0x1p-53;
    cand[i] = (ps > 0.0 && u < ell * (double)d2[i] / ps) ? 1 : 0;
  }
}

hipError_t launch_kpar_select(const float* d2, int64_t n, int64_t start, const double* psi, double ell,
                              uint64_t seed, uint32_t round, uint8_t* cand, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  int64_t nb = (n + 255) / 256;
  if (nb > 16384) nb = 16384;
  hipLaunchKernelGGL(kpar_select_kernel, dim3((unsigned)nb), dim3(256), 0, s, d2, n, start, psi, ell,
                     (uint32_t)seed, (uint32_t)(seed >> 32), round, cand);
  return hipGetLastError();
}

}  // namespace mk
