// mikmeans — K5/K6 k-means++ seeding and K8 on-device Gaussian blobs (gfx950).
//
// k-means++ (Arthur & Vassilvitskii 2007) is K-1 dependent passes.  Each pass:
//   K5 kpp_d2     d2[i] = min(d2[i], |x_i - c_new|^2) over fixed row blocks, plus an
//                 f64 partial sum per block (memory-bound streaming pass).
//   K6 kpp_sample one workgroup turns u*sum(d2) into an index with two
//                 prefix-sum searches (blocks, then rows) and copies the chosen
//                 row into C[k].  No host synchronisation anywhere, so all K-1
//                 steps are enqueued back to back (and capturable in a hipGraph).
// Multi-GPU: each rank's block sums are all-gathered and the
// rank-local target is computed on device; the owner contributes the row to an
// all-reduce (C4).
//
// K8 blobs: counter-based Philox4x32-10, so point i of a dataset is a pure
// function of (seed, i) -- every rank generates exactly its global row range and
// the dataset is identical for any world size.
#include <stdlib.h>

#include "common.h"
#include "kernels.h"

namespace mk {

constexpr int KPP_NT = 256;
// rows in flight per lane in the pruned pass: 6 (124 VGPRs, 4 waves/SIMD) beat 8 (166 VGPRs,
// 3 waves/SIMD) and 4 at cfg4: k-means++ seeding 0.95 -> 0.83 s (profiles/r1_18_kpp_unr_ab.json)
#ifndef MK_KPP_UNR_PRUNE
#define MK_KPP_UNR_PRUNE 6
#endif

// Pruned K5 (PRUNE): Elkan's triangle-inequality bound applied to D^2 seeding.
// owner[i] is the centre d2[i] was measured against and cc[j] = |c_new - c_j|^2.
// When cc[owner] >= KPP_PRUNE * d2[i], |x - c_new| >= |c_new - c_own| - |x - c_own|
// >= 1.0009 |x - c_own|: the new centre cannot lower d2[i], so row i is not read.
// The margin exceeds the f32 rounding of all three distances (relative <= D*2^-24
// for sums of squares), so d2, owner and the block sums are bit-identical to the
// unpruned pass; only the bytes read change.
constexpr float KPP_PRUNE = 4.004f;
constexpr int KPP_CC_LDS = 16384;  // centre-centre distances staged in LDS up to this k

// LPR lanes per row (each 16 B per pass over the row), UNR rows in flight per lane group.
// knew >= 0: the owner of every row whose d2 drops becomes knew (< 0: owner is read only,
// e.g. a greedy candidate evaluated into a scratch copy of d2).
template <typename T, int LPR, bool PRUNE>
__global__ __launch_bounds__(KPP_NT) void kpp_d2_kernel(const T* __restrict__ X, int64_t N, int D,
                                                        int64_t ldx, const float* __restrict__ c,
                                                        int first, float* __restrict__ d2,
                                                        double* __restrict__ block_sums,
                                                        int64_t rows_per_block, int32_t* __restrict__ owner,
                                                        const float* __restrict__ cc, int kcc, int knew) {
  constexpr int V = Elem<T>::V;
  constexpr int UNR = PRUNE ? MK_KPP_UNR_PRUNE : 4;
  constexpr int RPW = KPP_NT / LPR;  // rows per pass of the workgroup
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* cs = (float*)smem;
  for (int d = threadIdx.x; d < D; d += KPP_NT) cs[d] = c[d];
  // pruned pass: the k centre-centre distances live in LDS (one gather per row instead of a
  // dependent global load), unless there are too many of them
  // (ccs is addressed through the __shared__ array itself so the gathers below compile to
  // ds_read, not flat loads whose waits would also drain the in-flight row loads)
  const int cc_off = (D + 3) & ~3;
  const bool cc_lds = PRUNE && kcc <= KPP_CC_LDS;
  if constexpr (PRUNE) {
    if (cc_lds)
      for (int j = threadIdx.x; j < kcc; j += KPP_NT) ((float*)smem)[cc_off + j] = cc[j];
  }
  __syncthreads();
  const int sub = threadIdx.x % LPR;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  int64_t r1 = r0 + rows_per_block;
  if (r1 > N) r1 = N;
  double part = 0.0;
  // pruned pass: (d2, owner) of the next period are loaded while this one computes, so the
  // prune test costs no exposed global latency
  float old_n[UNR];
  int own_n[UNR];
  auto meta = [&](int64_t b) {
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int64_t i = b + (int64_t)u * RPW;
      old_n[u] = i < r1 ? d2[i] : 0.f;
      own_n[u] = i < r1 ? owner[i] : -1;
    }
  };
  if constexpr (PRUNE) meta(r0 + threadIdx.x / LPR);
  for (int64_t base = r0 + threadIdx.x / LPR; base < r1; base += (int64_t)RPW * UNR) {
    float acc[UNR], old[UNR], ccv[UNR];
    bool need[UNR];
    if constexpr (PRUNE) {
      // unconditional gathers (index clamped), all issued before the first compare: the
      // UNR reads share one wait instead of a branch + full wait each
      if (cc_lds) {
#pragma unroll
        for (int u = 0; u < UNR; ++u) ccv[u] = ((const float*)smem)[cc_off + (own_n[u] > 0 ? own_n[u] : 0)];
      } else {
#pragma unroll
        for (int u = 0; u < UNR; ++u) ccv[u] = cc[own_n[u] > 0 ? own_n[u] : 0];
      }
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      acc[u] = 0.f;
      if constexpr (PRUNE) {
        old[u] = old_n[u];
        need[u] = own_n[u] >= 0 && !(ccv[u] >= KPP_PRUNE * old[u]);
      } else {
        old[u] = 0.f;
        need[u] = base + (int64_t)u * RPW < r1;
      }
    }
    if constexpr (PRUNE) meta(base + (int64_t)RPW * UNR);
    for (int col = sub * V; col < D; col += LPR * V) {
      u32x4 w[UNR];
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const int64_t i = base + (int64_t)u * RPW;
        w[u] = need[u] ? *(const u32x4*)(X + i * ldx + col) : u32x4{0u, 0u, 0u, 0u};
      }
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        float f[V];
        unpack16(w[u], f, (T*)nullptr);
#pragma unroll
        for (int e = 0; e < V; ++e) { const float df = f[e] - cs[col + e]; acc[u] += df * df; }
      }
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
#pragma unroll
      for (int o = 1; o < LPR; o <<= 1) acc[u] += __shfl_xor(acc[u], o, 64);
      const int64_t i = base + (int64_t)u * RPW;
      if (sub == 0 && i < r1) {
        float v;
        if constexpr (PRUNE) {
          // == fminf(acc, old) of the unpruned pass (a NaN acc keeps old); stored on change only.
          // Rows are visited in the same order, so `part` sums the same values in the same order.
          v = old[u];
          if (need[u] && acc[u] < old[u]) {
            v = acc[u];
            d2[i] = v;
            if (knew >= 0) owner[i] = knew;
          }
        } else {
          v = first ? acc[u] : fminf(acc[u], d2[i]);
          d2[i] = v;
        }
        part += v;
      }
    }
  }
  part = wave_sum(part);
  __shared__ double red[KPP_NT / 64];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = part;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0;
    for (int w = 0; w < KPP_NT / 64; ++w) s += red[w];
    block_sums[blockIdx.x] = s;
  }
}

template <typename T, bool PRUNE>
static void launch_kpp_d2_t(const void* X, int64_t N, int D, int64_t ldx, const float* c, int first,
                            float* d2, double* block_sums, int64_t rows_per_block, int nblocks,
                            size_t lds, int32_t* owner, const float* cc, int kcc, int knew,
                            hipStream_t s) {
  const int pieces = (D * (int)sizeof(T) + 15) / 16;  // 16-byte pieces per row
  const T* Xt = (const T*)X;
#define MK_KPP_LAUNCH(L)                                                                         \
  hipLaunchKernelGGL((kpp_d2_kernel<T, L, PRUNE>), dim3(nblocks), dim3(KPP_NT), lds, s, Xt, N, D, \
                     ldx, c, first, d2, block_sums, rows_per_block, owner, cc, kcc, knew)
  if (pieces >= 16) MK_KPP_LAUNCH(16);
  else if (pieces >= 8) MK_KPP_LAUNCH(8);
  else if (pieces >= 4) MK_KPP_LAUNCH(4);
  else if (pieces >= 2) MK_KPP_LAUNCH(2);
  else MK_KPP_LAUNCH(1);
#undef MK_KPP_LAUNCH
}

hipError_t launch_kpp_d2(int dtype, const void* X, int64_t N, int D, int64_t ldx, const float* c,
                         int first, float* d2, double* block_sums, int64_t rows_per_block,
                         int nblocks, hipStream_t s, int32_t* owner, const float* cc, int kcc,
                         int knew) {
  const bool prune = owner != nullptr && cc != nullptr && !first;
  size_t lds = ((size_t)D * 4 + 15) / 16 * 16;
  if (prune && kcc <= KPP_CC_LDS) lds += (size_t)kcc * 4;
  if (dtype == DT_BF16) {
    if (prune)
      launch_kpp_d2_t<uint16_t, true>(X, N, D, ldx, c, 0, d2, block_sums, rows_per_block, nblocks, lds,
                                      owner, cc, kcc, knew, s);
    else
      launch_kpp_d2_t<uint16_t, false>(X, N, D, ldx, c, first, d2, block_sums, rows_per_block, nblocks,
                                       lds, nullptr, nullptr, 0, -1, s);
  } else {
    if (prune)
      launch_kpp_d2_t<float, true>(X, N, D, ldx, c, 0, d2, block_sums, rows_per_block, nblocks, lds,
                                   owner, cc, kcc, knew, s);
    else
      launch_kpp_d2_t<float, false>(X, N, D, ldx, c, first, d2, block_sums, rows_per_block, nblocks,
                                    lds, nullptr, nullptr, 0, -1, s);
  }
  return hipGetLastError();
}

// cc[j] = |cnew - C[j]|^2 for the k centres already chosen (one wave per centre): the
// centre-centre distances of the pruned K5 pass.
__global__ __launch_bounds__(256) void kpp_cc_kernel(const float* __restrict__ C, int64_t ldc, int k,
                                                     int D, const float* __restrict__ cnew,
                                                     float* __restrict__ cc) {
  const int j = blockIdx.x * 4 + (threadIdx.x >> 6);  // wave-uniform
  if (j >= k) return;
  const int lane = threadIdx.x & 63;
  float s = 0.f;
  for (int d = lane; d < D; d += 64) {
    const float df = cnew[d] - C[(int64_t)j * ldc + d];
    s += df * df;
  }
  s = wave_sum(s);
  if (lane == 0) cc[j] = s;
}

hipError_t launch_kpp_cc(const float* C, int64_t ldc, int k, int D, const float* cnew, float* cc,
                         hipStream_t s) {
  if (k <= 0) return hipSuccess;
  hipLaunchKernelGGL(kpp_cc_kernel, dim3((unsigned)((k + 3) / 4)), dim3(256), 0, s, C, ldc, k, D, cnew,
                     cc);
  return hipGetLastError();
}

// Block-wide inclusive scan (1024 threads) of one double per thread.
__device__ double block_scan_incl(double v, double* sh) {
  const int t = threadIdx.x;
  sh[t] = v;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    const double add = (t >= o) ? sh[t - o] : 0.0;
    __syncthreads();
    sh[t] += add;
    __syncthreads();
  }
  return sh[t];
}

// mode 0: *target_p is this rank's target (< 0: not the owner, write zeros).
// mode 1: *target_p is u in [0,1); target = u * (this rank's total potential) -- one rank.
// mode 2: *target_p is u; totals_all[world] are the gathered per-rank potentials: the
//         owner rank and its local target are derived here (no host round trip).
template <typename T>
__global__ __launch_bounds__(1024) void kpp_sample_kernel(const double* __restrict__ block_sums,
                                                          int nblocks, const float* __restrict__ d2,
                                                          int64_t N, int64_t rpb,
                                                          const double* __restrict__ target_p,
                                                          const T* __restrict__ X, int D,
                                                          int64_t ldx, float* __restrict__ crow,
                                                          int64_t* __restrict__ idx_out, int mode,
                                                          const double* __restrict__ totals_all,
                                                          int world, int rank) {
  __shared__ double sh[1024];
  __shared__ int64_t sel;
  __shared__ double base_sh;
  const int t = threadIdx.x;
  double target = *target_p;
  if (mode == 2) {
    double tot = 0.0, before = 0.0;
    int last = -1;
    for (int r = 0; r < world; ++r) {
      const double v = totals_all[r];
      tot += v;
      if (r < rank) before += v;
      if (v > 0.0) last = r;
    }
    const double tgt = target * tot;
    const double mine = totals_all[rank];
    double local = tgt - before;
    bool owner = local >= 0.0 && local < mine;
    if (tgt >= tot && last == rank) { owner = true; local = mine * (1.0 - 1e-12); }
    target = owner ? local : -1.0;
  }
  if (!(target >= 0.0)) {  // not the owner rank (or NaN): contribute zeros
    for (int d = t; d < D; d += 1024) crow[d] = 0.f;
    if (t == 0 && idx_out) *idx_out = -1;
    return;
  }
  // --- stage 1: which block
  const int per = (nblocks + 1023) / 1024;
  double segsum = 0.0;
  for (int b = t * per; b < (t + 1) * per && b < nblocks; ++b) segsum += block_sums[b];
  double incl = block_scan_incl(segsum, sh);
  const double total = sh[1023];
  if (mode == 1) target *= total;
  if (target >= total) target = total * (1.0 - 1e-12);
  if (t == 0) { sel = -1; base_sh = 0.0; }
  __syncthreads();
  {
    const double excl = incl - segsum;
    if (segsum > 0.0 && target >= excl && target < incl) {
      double run = excl;
      int64_t bsel = -1;
      for (int b = t * per; b < (t + 1) * per && b < nblocks; ++b) {
        const double bs = block_sums[b];
        if (bs > 0.0 && target < run + bs) { bsel = b; break; }
        run += bs;
      }
      if (bsel < 0) {  // rounding: last non-empty block of this segment
        for (int b = (t + 1) * per - 1; b >= t * per; --b)
          if (b < nblocks && block_sums[b] > 0.0) { bsel = b; break; }
        run = excl;
        for (int b = t * per; b < bsel; ++b) run += block_sums[b];
      }
      sel = bsel;
      base_sh = run;
    }
  }
  __syncthreads();
  int64_t b = sel;
  if (b < 0) {  // all-zero potential (duplicates): pick the last non-empty block, else row 0
    if (t == 0) {
      int64_t bb = -1;
      for (int i = nblocks - 1; i >= 0; --i) if (block_sums[i] > 0.0) { bb = i; break; }
      sel = bb;
      base_sh = 0.0;
      if (bb >= 0) for (int i = 0; i < bb; ++i) base_sh += block_sums[i];
    }
    __syncthreads();
    b = sel;
  }
  int64_t chosen = 0;
  if (b >= 0) {
    // --- stage 2: which row inside block b
    const double tb = target - base_sh;
    const int64_t r0 = b * rpb;
    int64_t r1 = r0 + rpb;
    if (r1 > N) r1 = N;
    const int64_t len = r1 - r0;
    const int64_t per2 = (len + 1023) / 1024;
    double s2 = 0.0;
    const int64_t a0 = r0 + t * per2;
    for (int64_t i = a0; i < a0 + per2 && i < r1; ++i) s2 += (double)d2[i];
    const double inc2 = block_scan_incl(s2, sh);
    __syncthreads();
    if (t == 0) sel = -1;
    __syncthreads();
    const double ex2 = inc2 - s2;
    if (s2 > 0.0 && tb >= ex2 && tb < inc2) {
      double run = ex2;
      int64_t isel = -1;
      for (int64_t i = a0; i < a0 + per2 && i < r1; ++i) {
        const double v = (double)d2[i];
        if (v > 0.0 && tb < run + v) { isel = i; break; }
        run += v;
      }
      if (isel < 0)
        for (int64_t i = (a0 + per2 < r1 ? a0 + per2 : r1) - 1; i >= a0; --i)
          if (d2[i] > 0.f) { isel = i; break; }
      sel = isel;
    }
    __syncthreads();
    if (sel < 0 && t == 0) {  // target beyond the block's float sum: last positive row
      for (int64_t i = r1 - 1; i >= r0; --i) if (d2[i] > 0.f) { sel = i; break; }
      if (sel < 0) sel = r0;
    }
    __syncthreads();
    chosen = sel;
  }
  const T* row = X + chosen * ldx;
  for (int d = t; d < D; d += 1024) crow[d] = Elem<T>::to_f32(row[d]);
  if (t == 0 && idx_out) *idx_out = chosen;
}

hipError_t launch_kpp_sample(int dtype, const double* block_sums, int nblocks, const float* d2,
                             int64_t N, int64_t rows_per_block, const double* target, const void* X,
                             int D, int64_t ldx, float* crow, int64_t* idx_out, int mode,
                             const double* totals_all, int world, int rank, hipStream_t s) {
  if (dtype == DT_BF16)
    hipLaunchKernelGGL(kpp_sample_kernel<uint16_t>, dim3(1), dim3(1024), 0, s, block_sums, nblocks,
                       d2, N, rows_per_block, target, (const uint16_t*)X, D, ldx, crow, idx_out,
                       mode, totals_all, world, rank);
  else
    hipLaunchKernelGGL(kpp_sample_kernel<float>, dim3(1), dim3(1024), 0, s, block_sums, nblocks,
                       d2, N, rows_per_block, target, (const float*)X, D, ldx, crow, idx_out,
                       mode, totals_all, world, rank);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Weighted k-means++ over a small candidate set (the k-means|| recluster, models/init.py):
// M candidates (Ct: f32, column-major [D][M], so a wave's candidate loads coalesce), weights
// w (f64), K draws u (f64).  Step k is two launches, with no host read in between:
//   wkpp_d2    d2[i] = min(d2[i], |c_i - c_j|^2) against the previous pick j (f64 sums of the
//              exact f64 differences), then p_i = w_i d2[i] scanned inside each 256-candidate
//              block (cum[i]: the block's inclusive prefix, part[b]: its total);
//   wkpp_pick  one workgroup: the block prefixes P_b (a chunked scan of part), the target
//              t = u[k] * total, the first block with P_b + part[b] > t and in it the first
//              candidate with P_b + cum[i] > t (torch.searchsorted(..., right=True) on the
//              cumulative weights; none: the last candidate) -> out[k] and state {j, k+1}.
// Every sum has a fixed order, so every rank draws the same centres from the same inputs.
// Step 0 (state j = -1) draws by weight alone; d2 starts at +inf.
constexpr int WK_NT = 256;

__device__ __forceinline__ double wave_incl_scan(double v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const double t = __shfl_up(v, o, 64);
    if (lane >= o) v += t;
  }
  return v;
}

// Inclusive scan over the 256 threads of a block (4 waves), fixed order; returns the thread's
// prefix and (all threads) the block total.
__device__ __forceinline__ double block_incl_scan(double v, double* red, double& total) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  v = wave_incl_scan(v, lane);
  if (lane == 63) red[wv] = v;
  __syncthreads();
  double off = 0.0;
  for (int q = 0; q < wv; ++q) off += red[q];
  total = red[0] + red[1] + red[2] + red[3];
  __syncthreads();   // (red is reused by the caller's next scan)
  return v + off;
}

__global__ __launch_bounds__(WK_NT) void wkpp_d2_kernel(const float* __restrict__ Ct, int64_t M, int D,
                                                       const double* __restrict__ w, double* __restrict__ d2,
                                                       double* __restrict__ cum, double* __restrict__ part,
                                                       const int64_t* __restrict__ state) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  double* red = (double*)smem;
  float* cj = (float*)(smem + 64);
  const int64_t j = state[0];
  if (j >= 0)
    for (int d = threadIdx.x; d < D; d += WK_NT) cj[d] = Ct[(int64_t)d * M + j];
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * WK_NT + threadIdx.x;
  double p = 0.0;
  if (i < M) {
    double dd = d2[i];
    if (j >= 0) {
      double s = 0.0;
      for (int d = 0; d < D; ++d) {
        const double t = (double)Ct[(int64_t)d * M + i] - (double)cj[d];
        s = __builtin_fma(t, t, s);
      }
      dd = s < dd ? s : dd;
      d2[i] = dd;
    }
    p = j >= 0 ? w[i] * dd : w[i];   // (step 0: by weight alone)
  }
  double total;
  const double c = block_incl_scan(p, red, total);
  if (i < M) cum[i] = c;
  if (threadIdx.x == 0) part[blockIdx.x] = total;
}

__global__ __launch_bounds__(WK_NT) void wkpp_pick_kernel(const float* __restrict__ Ct, int64_t M, int D,
                                                         const double* __restrict__ cum,
                                                         const double* __restrict__ part, int nb,
                                                         const double* __restrict__ u, int64_t* __restrict__ state,
                                                         float* __restrict__ out, int64_t ldo) {
  __shared__ double red[4];
  __shared__ double sh_carry, sh_pb;
  __shared__ int sh_b;
  __shared__ int64_t sh_j;
  const int64_t k = state[1];
  // P_b, the exclusive prefix of the block totals, chunk by chunk in a fixed order (an
  // inclusive scan of the totals shifted by one: no subtraction); with t >= 0, the first block
  // with P_b + part[b] > t is found in pass 2.  Pass 1 computes the grand total the same way.
  auto chunks = [&](double t, bool search) -> bool {
    double carry = 0.0;
    for (int b0 = 0; b0 < nb; b0 += WK_NT) {
      const int b = b0 + (int)threadIdx.x;
      const double prev = (b < nb && threadIdx.x > 0) ? part[b - 1] : 0.0;
      double tot;
      const double excl = block_incl_scan(prev, red, tot) + carry;
      const double own = b < nb ? part[b] : 0.0;
      const int last = b0 + WK_NT - 1 < nb ? b0 + WK_NT - 1 : nb - 1;
      if (b == last) sh_carry = excl + own;   // (one writer: the chunk's last block)
      if (search) {
        if (threadIdx.x == 0) sh_b = nb;
        __syncthreads();
        if (b < nb && excl + own > t) atomicMin(&sh_b, b);   // (LDS atomic)
        __syncthreads();
        const int f = sh_b;
        if (f < nb) {
          if (b == f) sh_pb = excl;
          __syncthreads();
          return true;
        }
      }
      __syncthreads();
      carry = sh_carry;
      __syncthreads();
    }
    if (threadIdx.x == 0) sh_pb = carry;
    __syncthreads();
    return false;
  };
  (void)chunks(0.0, false);
  const double t = u[k] * sh_pb;   // u * total
  __syncthreads();
  const bool hit = chunks(t, true);
  const int found = hit ? sh_b : nb;
  const double pb = sh_pb;
  // inside the block: the first candidate with P_b + cum[i] > t (its last candidate's cum is
  // the block total bitwise, so the block test guarantees a hit); no block: the last candidate
  if (threadIdx.x == 0) sh_j = hit ? (int64_t)found * WK_NT + WK_NT - 1 : M - 1;
  __syncthreads();
  if (hit) {
    const int64_t i = (int64_t)found * WK_NT + threadIdx.x;
    if (i < M && pb + cum[i] > t) atomicMin((unsigned long long*)&sh_j, (unsigned long long)i);
  }
  __syncthreads();
  const int64_t jj = sh_j < M ? sh_j : M - 1;
  for (int d = threadIdx.x; d < D; d += WK_NT) out[k * ldo + d] = Ct[(int64_t)d * M + jj];
  if (threadIdx.x == 0) {
    state[0] = jj;
    state[1] = k + 1;
  }
}

hipError_t launch_wkpp(const float* Ct, int64_t M, int D, const double* w, double* d2, double* cum, double* part,
                       const double* u, int64_t* state, float* out, int64_t ldo, int steps, hipStream_t s) {
  if (M <= 0 || steps <= 0) return M <= 0 && steps > 0 ? hipErrorInvalidValue : hipSuccess;
  const int64_t nb = (M + WK_NT - 1) / WK_NT;
  if (nb > (1 << 24)) return hipErrorInvalidValue;
  const size_t lds = 64 + (size_t)D * 4;
  if (lds > 64 * 1024) return hipErrorInvalidValue;
  for (int st = 0; st < steps; ++st) {
    hipLaunchKernelGGL(wkpp_d2_kernel, dim3((unsigned)nb), dim3(WK_NT), lds, s, Ct, M, D, w, d2, cum, part, state);
    hipLaunchKernelGGL(wkpp_pick_kernel, dim3(1), dim3(WK_NT), 0, s, Ct, M, D, cum, part, (int)nb, u, state, out,
                       ldo);
  }
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
constexpr uint32_t TAG_CID = 0xC1D0u, TAG_CTR = 0xCE27u, TAG_NRM = 0x4E52u;

__global__ void blob_centers_kernel(float* centers, int n_centers, int D, float box, uint32_t k0,
                                    uint32_t k1) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= (int64_t)n_centers * D) return;
  const int c = (int)(e / D), d = (int)(e % D);
  const U4 r = philox(U4{(uint32_t)c, (uint32_t)(d >> 2), TAG_CTR, 0u}, k0, k1);
  const uint32_t v = (d & 3) == 0 ? r.x : (d & 3) == 1 ? r.y : (d & 3) == 2 ? r.z : r.w;
  centers[e] = box * (2.f * u01(v) - 1.f);
}

hipError_t launch_blob_centers(float* centers, int n_centers, int D, float box, uint64_t seed,
                               hipStream_t s) {
  const int64_t tot = (int64_t)n_centers * D;
  hipLaunchKernelGGL(blob_centers_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s,
                     centers, n_centers, D, box, (uint32_t)seed, (uint32_t)(seed >> 32));
  return hipGetLastError();
}

// TPR threads per row (power of two); thread t generates the EL-element groups
// g = t, t + TPR, ... so each store instruction of the row's threads is contiguous.
// The row's blob id is drawn once (lane t == 0) and broadcast; the squared norm of
// the stored (rounded) values is reduced across the row's lanes when xn is given, so
// a streamed mini-batch needs no separate row-norm pass.
//
// Normals per Philox4x32-10 call: f32 rows take 4 (Box-Muller on 24-bit uniforms);
// bf16 rows (8 mantissa bits) take 8 from 16-bit uniforms -- radius from each word's
// low half, angle from its high half, tails truncated at sqrt(32 ln 2) = 4.7 sigma --
// which halves the Philox multiplies per value.  Box-Muller runs on the hardware
// transcendentals: v_log_f32 (log2), v_sqrt_f32, and v_sin_f32 / v_cos_f32, whose
// argument is in revolutions, so sin(2*pi*u) is one instruction.
template <typename T>
__device__ __forceinline__ void box_muller(const U4& r, float* z) {
  constexpr float M2LN2 = -1.38629436111989f;  // -2 ln 2
  if constexpr (sizeof(T) == 2) {
    const uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float u = (float)((w[j] & 0xffffu) + 1u) * (1.0f / 65536.0f);
      const float a = (float)(w[j] >> 16) * (1.0f / 65536.0f);
      const float rad = __builtin_amdgcn_sqrtf(M2LN2 * __builtin_amdgcn_logf(u));
      z[2 * j] = rad * __builtin_amdgcn_cosf(a);
      z[2 * j + 1] = rad * __builtin_amdgcn_sinf(a);
    }
  } else {
    const float rad0 = __builtin_amdgcn_sqrtf(M2LN2 * __builtin_amdgcn_logf(u01_open0(r.x)));
    const float rad1 = __builtin_amdgcn_sqrtf(M2LN2 * __builtin_amdgcn_logf(u01_open0(r.z)));
    const float a0 = u01(r.y), a1 = u01(r.w);
    z[0] = rad0 * __builtin_amdgcn_cosf(a0);
    z[1] = rad0 * __builtin_amdgcn_sinf(a0);
    z[2] = rad1 * __builtin_amdgcn_cosf(a1);
    z[3] = rad1 * __builtin_amdgcn_sinf(a1);
  }
}

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

// NORMS: the squared row norms of the stored values are fused in (xn != nullptr).
//
// A grid-stride loop over 64-row wave tiles (a few workgroups per CU instead of one short
// workgroup per 8 rows: the per-wave start-up and the dispatch of ~3M workgroups per 1e8 rows
// dominated the D=128 pass).  Each lane draws the blob id of ONE row of its wave's tile (one
// Philox per 64 rows instead of one per TPR-lane row group, and a coalesced label store); the
// tile's rows are then filled TPR lanes per row in 64/TPR sub-steps, the id shuffled from its
// owner lane.  Every value, label and fused norm is bitwise the one-row-per-lane-group form's.
template <typename T, int TPR, bool NORMS>
__global__ __launch_bounds__(256) void blobs_kernel(T* X, int64_t i0, int64_t n, int D, int64_t ldx,
                                                    const float* __restrict__ centers,
                                                    int n_centers, float stddev, uint32_t k0,
                                                    uint32_t k1, int32_t* y, float* xn, int vec) {
  constexpr int EL = sizeof(T) == 2 ? 8 : 4;  // values per Philox call (= 16-byte store)
  constexpr int RPS = 64 / TPR;               // rows per sub-step of a wave
  const int G = (D + EL - 1) / EL;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int t = lane % TPR, rs = lane / TPR;
  const int64_t tstride = (int64_t)gridDim.x * 256;
  for (int64_t w0 = (int64_t)blockIdx.x * 256 + wid * 64; w0 < n; w0 += tstride) {
    // this lane's row of the tile: its blob id (one Philox per lane)
    int cid_l = 0;
    {
      const int64_t ir = w0 + lane;
      const uint64_t gr = (uint64_t)(i0 + (ir < n ? ir : 0));
      const U4 rc = philox(U4{(uint32_t)gr, (uint32_t)(gr >> 32), TAG_CID, 0u}, k0, k1);
      cid_l = (int)__umulhi(rc.x, (uint32_t)n_centers);
      if (y && ir < n) y[ir] = cid_l;
    }
#pragma unroll 1
    for (int sub = 0; sub < TPR; ++sub) {
      const int64_t il = w0 + sub * RPS + rs;
      const bool row_ok = il < n;
      const uint64_t gi = (uint64_t)(i0 + (row_ok ? il : 0));
      const int cid = __shfl(cid_l, sub * RPS + rs, 64);
      float sq = 0.f;
      if (row_ok) {
        const float* mu = centers + (int64_t)cid * D;
        T* out = X + il * ldx;
        if (vec) {
          // Branch-free path (D % EL == 0, 16-byte aligned centres and rows): the group's
          // means are dwordx4 loads issued before the Philox rounds, so their L2 latency
          // hides under them (the general path waits on dependent dword loads).  Same bits.
          for (int g = t; g < G; g += TPR) {
            f32x4 m[EL / 4];
#pragma unroll
            for (int q = 0; q < EL / 4; ++q) m[q] = *(const f32x4*)(mu + EL * g + 4 * q);
            const U4 r = philox(U4{(uint32_t)gi, (uint32_t)(gi >> 32), (uint32_t)g, TAG_NRM}, k0, k1);
            float z[EL], f[EL];
            box_muller<T>(r, z);
#pragma unroll
            for (int j = 0; j < EL; ++j) f[j] = __builtin_fmaf(stddev, z[j], m[j / 4][j % 4]);
            if constexpr (sizeof(T) == 2) {
              // RNE to bf16 two values per v_cvt_pk_bf16_f32 (gfx950; values are finite by
              // construction, so the bits equal the integer rounding of the NumPy mirror)
              u32x4 w;
#pragma unroll
              for (int j = 0; j < 4; ++j) {
                w[j] = __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{f[2 * j], f[2 * j + 1]}, bf16x2));
                if constexpr (NORMS) {   // both squares of the stored pair in one v_dot2c_f32_bf16
                  const bf16x2 h = __builtin_bit_cast(bf16x2, w[j]);
                  sq = __builtin_amdgcn_fdot2_f32_bf16(h, h, sq, false);
                }
              }
              *(u32x4*)(out + EL * g) = w;
            } else {
              if constexpr (NORMS) {
#pragma unroll
                for (int j = 0; j < EL; ++j) sq = __builtin_fmaf(f[j], f[j], sq);
              }
              *(f32x4*)(out + EL * g) = f32x4{f[0], f[1], f[2], f[3]};
            }
          }
        } else {
          for (int g = t; g < G; g += TPR) {
            const U4 r = philox(U4{(uint32_t)gi, (uint32_t)(gi >> 32), (uint32_t)g, TAG_NRM}, k0, k1);
            float z[EL];
            box_muller<T>(r, z);
#pragma unroll
            for (int j = 0; j < EL; ++j) {
              const int d = EL * g + j;
              if (d < D) {
                const T v = Elem<T>::from_f32(__builtin_fmaf(stddev, z[j], mu[d]));
                const float f = Elem<T>::to_f32(v);
                sq = __builtin_fmaf(f, f, sq);
                out[d] = v;
              }
            }
          }
        }
      }
      if constexpr (NORMS) {
#pragma unroll
        for (int o = 1; o < TPR; o <<= 1) sq += __shfl_xor(sq, o, 64);
        if (row_ok && t == 0) xn[il] = sq;
      }
    }
  }
}

hipError_t launch_blobs(int dtype, void* X, int64_t i0, int64_t n, int D, int64_t ldx,
                        const float* centers, int n_centers, float stddev, uint64_t seed,
                        int32_t* y, float* xn, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const int el = dtype == DT_BF16 ? 8 : 4;  // values per group (see blobs_kernel)
  const int G = (D + el - 1) / el;
  const int es = dtype == DT_BF16 ? 2 : 4;
  const int vec = ((uintptr_t)X % 16 == 0 && (ldx * es) % 16 == 0 && D % el == 0 &&
                   (uintptr_t)centers % 16 == 0) ? 1 : 0;
  int tpr = 1;
  // Lanes per row: the row's blob-id Philox runs once per wave whatever the number of
  // active lanes, so fewer lanes per row (more rows per wave) amortise it over more
  // groups (8 lanes x 16 B still store whole 128-B lines; profiles/r1_18_blobs_tpr_ab.json:
  // 2.91 -> 2.69 ms per 16.8M x 256 bf16 batch).  Variant V_BLOBS_TPR (1..16) overrides the
  // cap for A/B runs.  The rows do not depend on it; the fused norms' f32 summation order does.
  const int tv = variant(V_BLOBS_TPR);
  const int tpr_cap = tv < 0 ? 8 : (tv >= 1 && tv <= 16 ? tv : 16);
  while (tpr < G && tpr * 2 <= tpr_cap) tpr *= 2;
  // 256 rows per workgroup step; at most 16 workgroups per CU's worth of grid (then strided)
  int64_t nb64 = (n + 255) / 256;
  if (nb64 > 4096) nb64 = 4096;
  const unsigned nb = (unsigned)nb64;
  const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#define MK_BLOBS(TT, TP)                                                                           \
  do {                                                                                             \
    if (xn)                                                                                        \
      hipLaunchKernelGGL((blobs_kernel<TT, TP, true>), dim3(nb), dim3(256), 0, s, (TT*)X, i0, n, D, \
                         ldx, centers, n_centers, stddev, k0, k1, y, xn, vec);                     \
    else                                                                                           \
      hipLaunchKernelGGL((blobs_kernel<TT, TP, false>), dim3(nb), dim3(256), 0, s, (TT*)X, i0, n,  \
                         D, ldx, centers, n_centers, stddev, k0, k1, y, xn, vec);                  \
  } while (0)
#define MK_BLOBS_T(TT)                                                                           \
  switch (tpr) {                                                                                 \
    case 1: MK_BLOBS(TT, 1); break;                                                              \
    case 2: MK_BLOBS(TT, 2); break;                                                              \
    case 4: MK_BLOBS(TT, 4); break;                                                              \
    case 8: MK_BLOBS(TT, 8); break;                                                              \
    default: MK_BLOBS(TT, 16); break;                                                            \
  }
  if (dtype == DT_BF16) { MK_BLOBS_T(uint16_t) } else { MK_BLOBS_T(float) }
#undef MK_BLOBS_T
#undef MK_BLOBS
  return hipGetLastError();
}

}  // namespace mk
