// mikmeans — K3: Lloyd M-step scatter-add (per-cluster sums and counts) for gfx950.
//
// sums[k,:] += w_i x_i, counts[k] += w_i for k = labels[i].
//
// Why this shape (measured on MI355X, scripts/microbench/lds_atomics.hip):
//  * global float atomics run at ~1.3 TB/s of added bytes chip-wide, so a direct
//    scatter of N=1e8 x D=128 f32 adds (51 GB) would take ~40 ms per iteration;
//  * LDS ds_add_f32 costs ~169 cycles per wave-instruction whatever the bank
//    pattern; integer LDS adds are ~20x faster and are bound by moving their
//    address + data dwords from VGPRs to the LDS (2 cycles per dword).
// So every workgroup privatises a [K][SW] slice of the sums in LDS as FIXED-POINT
// integers, TWO columns per 64-bit cell: a contribution q = rne(x * w * 2^e_col)
// (|q| <= 2^20, per-column exponent e_col from the global column max) is formed
// by ONE fma against the magic constant 1.5*2^23, whose result's bit pattern is
// 0x4B400000 + q; the bit patterns of two adjacent columns are added as one
// ds_add_u64 (3 dwords for 2 elements).  Modulo 2^64 the cell then holds
//   sum(q_a) + sum(q_b) * 2^32 + n * 0x4B400000 * (1 + 2^32)
// where n is the number of adds since the last flush (counted per label), and as
// long as |sum(q)| < 2^31 for both columns the two sums decode exactly.  Each
// label's add count is tracked; before any can reach 2^11 the workgroup flushes
// its slice (decode, add into its int64 slab rows, zero) and carries on.
// Integer addition is exact and associative: the M-step is bitwise identical for
// any atomic order, chunking or world size; the quantisation error per point is
// <= 2^-21 max|x_col|.
//
// D is split into column slices so a slice fits LDS; every workgroup streams its
// contiguous chunk of rows with 4..16-byte loads.  Grid mapping is XCD-aware:
// blocks b and b+8 share an XCD on MI355X, so the n_slices workgroups that read
// the same rows (different column slices of the same lines) get block ids
// congruent mod 8 and meet in one 4 MB L2.
//
// Reference parity: the reference's "update step" is re-deriving the dashboard
// after humans move cards (app.mjs:481-496 snapshotMetrics counts); counts here
// are exactly those per-centroid counts.
#include <math.h>

#include <cstdlib>

#include "common.h"
#include "kernels.h"
#include "plan.h"

namespace mk {

constexpr int UPD_NT = 512;                 // one LDS-filling workgroup per CU
using plan::UPD_LDS_MAX;
using plan::FX_BITS;                        // |q| <= 2^20 per contribution
constexpr int FX_LIM = (1 << (30 - FX_BITS)) * 2 - 1;  // adds per flush: 2047 * 2^20 < 2^31
constexpr float FX_MAGIC = 12582912.0f;     // 1.5 * 2^23, bits 0x4B400000
constexpr unsigned long long FX_MM = 0x4B4000004B400000ull;
constexpr int UPD_MAX_PERIOD = 1024;        // rows between flush checks
constexpr int UPD_NBUF = 3;                 // period buffers in the prefetch ring

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

// bits of (1.5*2^23 + rne(v * sc)); exact while |v * sc| <= 2^22.  CLAMP saturates
// out-of-range contributions at +-2^20 (streams whose scale came from an earlier
// batch), the bound FX_LIM's no-wrap guarantee assumes; the caller tracks the raw
// range (rlo, rhi) so a batch that clamped is reported instead of kept silently.
constexpr float FX_QMAX = 1048576.f;  // 2^FX_BITS
template <bool CLAMP>
__device__ __forceinline__ float fx_raw(float v, float sc) { return __builtin_fmaf(v, sc, FX_MAGIC); }
template <bool CLAMP>
__device__ __forceinline__ uint32_t fx_clamp(float r) {
  if constexpr (CLAMP) r = __builtin_amdgcn_fmed3f(r, FX_MAGIC - FX_QMAX, FX_MAGIC + FX_QMAX);
  return __float_as_uint(r);
}
template <bool CLAMP>
__device__ __forceinline__ uint32_t fx_bits(float v, float sc) { return fx_clamp<CLAMP>(fx_raw<CLAMP>(v, sc)); }
// Residual pass (wide-range columns): bits of 1.5*2^23 + rne((v*sc - rne(v*sc)) * sc2).
// v*sc - rne(v*sc) is exact in f32 (|.| <= 1/2), so the hi pass (col_exp) plus this lo
// pass (col_exp + 20) quantise x to 2^-41 of its column maximum instead of 2^-21.
__device__ __forceinline__ uint32_t fx_bits_resid(float v, float sc, float sc2) {
  const float hi = __builtin_fmaf(v, sc, FX_MAGIC) - FX_MAGIC;
  const float res = __builtin_fmaf(v, sc, -hi);
  return __float_as_uint(__builtin_fmaf(res, sc2, FX_MAGIC));
}

__device__ __forceinline__ long long fx_q(float v, float sc) {
  return (long long)(int)(fx_bits<true>(v, sc) - 0x4B400000u);
}

// LDS: cells [K+1][LDc] u64 (row K is a sink for rows outside the chunk, so the hot
// loop has no per-row branch) | add counts [K+1] u32 | flag | weighted counts [K+1] i64
// (weighted fits only).  With an odd stride (LDc = SW/2 + 1) rows start on scattered
// banks; where only LDc = SW/2 fits, the pair index is XOR-swizzled by label bits
// instead (swz), which scatters the banks of one instruction the same way.
// Within a label, lane lp's c-th pair (columns lp*V + 2c, +1) sits at index c*LPR + lp, so
// the lanes of one row hit consecutive cells in each ds_add_u64 (ds_write_b64 banking: 16
// contiguous lanes per LDS cycle, bank (a/4) mod 32); per-lane pairs (index lp*V/2 + c)
// put a row's lanes 8 or 16 dwords apart, 2-way conflicts inside every row.
struct UpdLayout {
  int K, LDc, np, ksh;
  bool swz;
  int lpr, npl;  // lanes per row, pairs per lane (lpr * npl == np)
  __device__ unsigned long long* cells(char* m) const { return (unsigned long long*)m; }
  __device__ unsigned* nadd(char* m) const { return (unsigned*)(cells(m) + (size_t)(K + 1) * LDc); }
  __device__ int* flag(char* m) const { return (int*)(nadd(m) + K + 1); }
  __device__ long long* wcnt(char* m) const {
    return (long long*)(((uintptr_t)(flag(m) + 2) + 7) & ~(uintptr_t)7);
  }
  __device__ int* nhot(char* m) const { return flag(m) + 1; }
  // list of labels being flushed (u16), after the weighted counts when present
  __device__ unsigned short* hot(char* m, bool weighted) const {
    return (unsigned short*)(wcnt(m) + (weighted ? K + 1 : 0));
  }
  // cell index of lane lp's pair c of label k
  __device__ int at(int k, int lp, int c) const {
    const int i = c * lpr + lp;
    return swz ? (i ^ ((k >> ksh) & (np - 1))) : i;
  }
  // cell index of column pair p of label k
  __device__ int pos(int k, int p) const { return at(k, p / npl, p % npl); }
};

// nadd[k]: adds since label k's last flush in bits 0..30; bit 31 = "k's slab row
// already holds a partial sum" (then a flush adds instead of storing).
constexpr unsigned NADD_MASK = 0x7fffffffu, NADD_WRITTEN = 0x80000000u;

// Mid-chunk flush of every label whose add count reached `thresh`: list them, then
// decode their cells with one (label, pair) per thread so the slab read-modify-writes
// of a label are contiguous across lanes.  Called by all threads after an LDS barrier.
// counts come from the signed 64-bit per-label counters (weighted or incremental
// M-step) instead of the add counts
__device__ __forceinline__ bool upd_wcounts(const UpdateArgs& a) { return a.weights || a.dlist; }

template <int SW>
__device__ void upd_flush_hot(const UpdateArgs& a, const UpdLayout& L, char* m, int slice, int chunk,
                              unsigned thresh) {
  constexpr int NP = SW / 2;
  const bool W = upd_wcounts(a);
  unsigned* nadd = L.nadd(m);
  unsigned short* hot = L.hot(m, W);
  if (threadIdx.x == 0) *L.nhot(m) = 0;
  __syncthreads();
  for (int k = threadIdx.x; k < a.K; k += blockDim.x)
    if ((nadd[k] & NADD_MASK) >= thresh) hot[atomicAdd(L.nhot(m), 1)] = (unsigned short)k;
  __syncthreads();
  const int nh = *L.nhot(m);
  const int cols = (a.D - slice * SW) < SW ? (a.D - slice * SW) : SW;
  unsigned long long* cells = L.cells(m);
  for (int e = threadIdx.x; e < nh * NP; e += blockDim.x) {
    const int k = hot[e / NP], p = e % NP;
    const unsigned na = nadd[k];
    const int q = k * L.LDc + L.pos(k, p);
    const unsigned long long T = cells[q] - (unsigned long long)(na & NADD_MASK) * FX_MM;
    cells[q] = 0;
    const int lo = (int)(uint32_t)T;
    const long long hi = (long long)(T - (unsigned long long)(long long)lo) >> 32;
    if (2 * p < cols) {
      long long* dst = a.slab + (int64_t)chunk * a.K * a.D + (int64_t)k * a.D + slice * SW + 2 * p;
      if (na & NADD_WRITTEN) { dst[0] += lo; dst[1] += hi; }
      else { dst[0] = lo; dst[1] = hi; }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nh; i += blockDim.x) {
    const int k = hot[i];
    const unsigned na = nadd[k];
    if (slice == 0) {
      const long long c = W ? L.wcnt(m)[k] : (long long)(na & NADD_MASK);
      long long* cd = a.cnt_slab + (int64_t)chunk * a.K + k;
      if (na & NADD_WRITTEN) *cd += c; else *cd = c;
    }
    if (W) L.wcnt(m)[k] = 0;
    nadd[k] = NADD_WRITTEN;
  }
  if (threadIdx.x == 0) *L.flag(m) = 0;
  __syncthreads();
}

// Final flush of every label, one (label, cell) per thread so the slab writes coalesce.
template <int SW>
__device__ void upd_flush_all(const UpdateArgs& a, const UpdLayout& L, char* m, int slice, int chunk) {
  constexpr int NP = SW / 2;
  unsigned long long* cells = L.cells(m);
  const unsigned* nadd = L.nadd(m);
  __syncthreads();
  long long* slab = a.slab + (int64_t)chunk * a.K * a.D + slice * SW;
  const int cols = (a.D - slice * SW) < SW ? (a.D - slice * SW) : SW;
  for (int e = threadIdx.x; e < a.K * NP; e += blockDim.x) {
    const int k = e / NP, p = e % NP;
    const unsigned na = nadd[k];
    const unsigned long long T = cells[k * L.LDc + L.pos(k, p)] - (unsigned long long)(na & NADD_MASK) * FX_MM;
    const int lo = (int)(uint32_t)T;
    const long long hi = (long long)(T - (unsigned long long)(long long)lo) >> 32;
    if (2 * p < cols) {
      long long* dst = slab + (int64_t)k * a.D + 2 * p;
      if (na & NADD_WRITTEN) { dst[0] += lo; dst[1] += hi; }
      else { dst[0] = lo; dst[1] = hi; }
    }
  }
  if (slice == 0) {
    for (int k = threadIdx.x; k < a.K; k += blockDim.x) {
      const unsigned na = nadd[k];
      const long long c = upd_wcounts(a) ? L.wcnt(m)[k] : (long long)(na & NADD_MASK);
      long long* dst = a.cnt_slab + (int64_t)chunk * a.K + k;
      if (na & NADD_WRITTEN) *dst += c; else *dst = c;
    }
  }
}

enum : int { UPD_CLAMP = 1, UPD_WEIGHTED = 2, UPD_SWZ = 4, UPD_DELTA = 8, UPD_RESID = 32, UPD_GATHER = 64,
             UPD_GSTAGE = 128 };

// Rows per period of the column-slice kernel (host and device agree on it: the gathered
// index staging sizes its LDS ring from it).
template <typename T, int SW, int NT, int PER>
constexpr int upd_period() {
  constexpr int PB = (SW * (int)sizeof(T) >= 16) ? 16 : SW * (int)sizeof(T);
  constexpr int V = PB / (int)sizeof(T);
  constexpr int RPP = NT / (SW / V);
  constexpr int UNR = (PER / RPP) < 8 ? (PER / RPP) : 8;
  return RPP * UNR;
}

constexpr int upd_ksh(int np) { return np >= 32 ? 0 : np == 16 ? 1 : np == 8 ? 2 : np == 4 ? 3 : np == 2 ? 4 : 5; }
using plan::upd_lds_bytes;

template <typename T, int SW, int MODE, int NT = UPD_NT, int NBF = UPD_NBUF, int PER = UPD_MAX_PERIOD>
__global__ __launch_bounds__(NT) void update_kernel(UpdateArgs a, int n_slices,
                                                        int64_t rows_per_chunk) {
  // (rows_per_chunk is recomputed from the list length in incremental mode)
  constexpr bool CLAMP = MODE & UPD_CLAMP;
  constexpr bool DELTA = MODE & UPD_DELTA;
  constexpr bool W = MODE & (UPD_WEIGHTED | UPD_DELTA);  // per-row signed weights
  constexpr bool SWZ = MODE & UPD_SWZ;
  constexpr bool RESID = MODE & UPD_RESID;               // lo pass of the wide-range columns
  constexpr bool GATHER = MODE & UPD_GATHER;             // logical row i is X row a.rows[i]
  // GSTAGE (gathered): the X rows of a period are staged in an LDS ring NBF periods ahead,
  // so no X load's address waits on an index load issued after older X loads (vmcnt retires
  // in order: the unstaged path drained the whole prefetch ring every period)
  constexpr bool GSTAGE = GATHER && (MODE & UPD_GSTAGE) && !DELTA;
  // FLAT (the staged builds): one straight-line load form for every period and unconditional
  // ring loads (labels clamped in accumulate), so the wait counter stays exact across the
  // period loop.  For plain passes the same form measured 3.5 % faster at D=256 bf16 but 29 %
  // slower for the f32 64-column kernel (profiles/r3_20_abu_*_flat*.log), so they keep theirs.
  constexpr bool FLAT = GSTAGE;
  constexpr int ES = sizeof(T);
  constexpr int PB = (SW * ES >= 16) ? 16 : SW * ES;  // bytes per lane load
  constexpr int V = PB / ES;                           // elements per lane load (even)
  constexpr int LPR = SW / V;                          // lanes per row
  constexpr int RPP = NT / LPR;                        // rows per pass
  constexpr int UNR = (PER / RPP) < 8 ? (PER / RPP) : 8;
  constexpr int PERIOD = RPP * UNR;
  constexpr unsigned THRESH = FX_LIM - PERIOD + 1;     // flush before any label passes FX_LIM
  constexpr int NP = SW / 2;
  constexpr int LDC = SWZ ? NP : NP + 1;                // unpadded + swizzle, or odd stride
  constexpr int KSH = upd_ksh(NP);
  static_assert(V % 2 == 0 && UNR >= 1 && FX_LIM >= PERIOD, "update tiling");
  static_assert(PERIOD == upd_period<T, SW, NT, PER>(), "host period");
  constexpr int GI = (PERIOD + NT - 1) / NT;            // GSTAGE: staged indices per thread
  typedef typename LoadT<PB>::type LT;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const UpdLayout L{a.K, LDC, NP, KSH, SWZ, LPR, V / 2};
  unsigned long long* cells = L.cells(smem);
  long long* wcnt = L.wcnt(smem);
  unsigned* nadd = L.nadd(smem);

  const int b = blockIdx.x;
  const int j = b >> 3;
  const int slice = j % n_slices;
  const int chunk = (j / n_slices) * 8 + (b & 7);
  if constexpr (RESID) {  // slices without a wide-range column have nothing to add
    bool any = false;
    for (int c = slice * SW; c < slice * SW + SW && c < a.D; ++c) any |= a.col_exp2[c] > -200;
    if (!any) return;
  }

  {
    unsigned long long* z = cells;
    const int nz = (int)((upd_lds_bytes(a.K, LDC, W) + 7) / 8);
    for (int e = threadIdx.x; e < nz; e += NT) z[e] = 0;
  }

  // Incremental mode: the rows are the 2*c entries of the changed-row list (c adds
  // to the new labels, then c subtractions from the old ones) unless it overflowed.
  int64_t nrows = a.N;
  int dc = 0;
  bool full = true;
  if constexpr (DELTA) {
    dc = *a.dcount;
    full = dc > a.dcap;
    if (!full) {
      nrows = 2 * (int64_t)dc;
      rows_per_chunk = (nrows + a.n_chunks - 1) / a.n_chunks;
    }
  }
  const int64_t row0 = (int64_t)chunk * rows_per_chunk;
  int64_t row1 = row0 + rows_per_chunk;
  if (row1 > nrows) row1 = nrows;
  const int lr = threadIdx.x / LPR, lp = threadIdx.x % LPR;
  const int col = slice * SW + lp * V;
  const bool colok = col < a.D;
  const bool all_cols = (a.D % SW) == 0;               // kernel-uniform
  const int colc = colok ? col : 0;
  const bool counter = lp == 0;
  const bool wcounter = W && counter && slice == 0;
  const float cscale = ldexpf(1.f, a.cnt_exp);
  float sc[V], sc2[V];
#pragma unroll
  for (int e = 0; e < V; ++e) {
    sc[e] = (col + e < a.D) ? ldexpf(1.f, a.col_exp[col + e]) : 0.f;
    // lo-pass scale 2^(col_exp2 - col_exp): 2^20 on wide columns, 0 elsewhere
    sc2[e] = (RESID && col + e < a.D && a.col_exp2[col + e] > -200)
                 ? ldexpf(1.f, a.col_exp2[col + e] - a.col_exp[col + e]) : 0.f;
  }
  float rlo = FX_MAGIC, rhi = FX_MAGIC;  // raw contribution range seen (CLAMP: clamp report)

  // Row mapping: in a period starting at `base`, lane (lr, lp) owns the UNR
  // consecutive rows base + lr*UNR + u, so runs of equal labels (sorted or
  // converged data) merge in registers before they reach the LDS, and the loads
  // of one lane are one address plus immediate offsets.
  const T* xrow = (const T*)a.X + (row0 + (int64_t)lr * UNR) * a.ldx + colc;
  const int* lrow = a.labels + row0 + lr * UNR;
  const float* wrow = a.weights ? a.weights + row0 + lr * UNR : nullptr;
  long long* gidx = (long long*)(smem + upd_lds_bytes(a.K, LDC, W));   // GSTAGE: [NBF][PERIOD]
  auto load = [&](int64_t base, LT* w_, int* lab_, float* wt_, int slot) {
    const long long* gs = gidx + slot * PERIOD + lr * UNR;
    const int64_t off = base - row0;
    if constexpr (FLAT) {
      // one straight-line form for every period (rows past the chunk clamp to its last row;
      // accumulate sends them to the sink): a branch between differently shaped load
      // sequences made the wait counter at the join fall back to vmcnt(0), draining the ring
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const int64_t i0 = base + (int64_t)lr * UNR + u;
        const int64_t i = i0 < row1 ? i0 : row1 - 1;
        lab_[u] = a.labels[i];
        if constexpr (W) wt_[u] = a.weights[i];
        if constexpr (GSTAGE) w_[u] = *(const LT*)((const T*)a.X + gs[u] * a.ldx + colc);
        else w_[u] = *(const LT*)((const T*)a.X + i * a.ldx + colc);
      }
    } else if (DELTA && !full) {                       // gather the listed rows
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const int64_t j0 = base + (int64_t)lr * UNR + u;
        const int64_t j = j0 < row1 ? j0 : row1 - 1;
        const bool neg = j >= dc;
        const int2 e = a.dlist[neg ? j - dc : j];
        const int l = neg ? e.y : a.labels[e.x];
        lab_[u] = (j0 < row1 && (unsigned)l < (unsigned)a.K) ? l : a.K;
        const float wv = a.weights ? a.weights[e.x] : 1.f;
        wt_[u] = neg ? -wv : wv;
        w_[u] = *(const LT*)((const T*)a.X + (int64_t)e.x * a.ldx + colc);
      }
    } else if (base + PERIOD <= row1) {                // whole period (all but the last)
      const T* p = xrow + off * a.ldx;
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const int l = lrow[off + u];
        lab_[u] = ((unsigned)l < (unsigned)a.K) ? l : a.K;
        if constexpr (DELTA) wt_[u] = wrow ? wrow[off + u] : 1.f;
        else if constexpr (W) wt_[u] = wrow[off + u];
        if constexpr (GSTAGE)
          w_[u] = *(const LT*)((const T*)a.X + gs[u] * a.ldx + colc);
        else if constexpr (GATHER)
          w_[u] = *(const LT*)((const T*)a.X + a.rows[base + (int64_t)lr * UNR + u] * a.ldx + colc);
        else
          w_[u] = *(const LT*)(p + u * a.ldx);
      }
    } else {                                           // clamp rows past the chunk -> sink row K
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const int64_t i0 = base + (int64_t)lr * UNR + u;
        const int64_t i = i0 < row1 ? i0 : row1 - 1;
        const int l = a.labels[i];
        lab_[u] = (i0 < row1 && (unsigned)l < (unsigned)a.K) ? l : a.K;
        if constexpr (DELTA) wt_[u] = a.weights ? a.weights[i] : 1.f;
        else if constexpr (W) wt_[u] = a.weights[i];
        if constexpr (GSTAGE) w_[u] = *(const LT*)((const T*)a.X + gs[u] * a.ldx + colc);   // staged rows[min(i0, row1-1)]
        else w_[u] = *(const LT*)((const T*)a.X + (GATHER ? a.rows[i] : i) * a.ldx + colc);
      }
    }
    // (staged builds: lanes past the last column read column 0 of the row and add
    // fma(x, 0, MAGIC) = +0 -- their scales are 0; zeroing the loaded registers here waited
    // for every load of the period right after issuing it.  The other builds keep the zeroing:
    // without it the f32 64-column kernel measured 2 % slower.)
    if constexpr (!FLAT) {
      if (!all_cols && !colok) {
#pragma unroll
        for (int u = 0; u < UNR; ++u) w_[u] = LT{};
      }
    }
  };

  // Accumulate one period; sets the flush flag when a label's add count nears FX_LIM.
  // (GSTAGE: load leaves the raw labels and accumulate sends rows past the chunk and
  // out-of-range labels -- unassigned rows -- to the sink row K; clamping them in load made
  // each period's labels wait for their load right after it was issued, draining the ring.
  // The other builds clamp in load, which measured 2 % faster for the f32 64-column kernel.)
  auto accumulate = [&](int64_t base, const LT* w_, const int* labr_, const float* wt_, auto&& pre_barrier) {
    int lab_[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      if constexpr (FLAT) {
        const bool in = base + (int64_t)lr * UNR + u < row1;
        lab_[u] = (in && (unsigned)labr_[u] < (unsigned)a.K) ? labr_[u] : a.K;
      } else {
        lab_[u] = labr_[u];
      }
    }
    unsigned seen = 0;
    unsigned long long acc[V / 2];
    int cur = lab_[0];
    unsigned run = 0;
    auto emit = [&]() {
      unsigned long long* dst = cells + cur * LDC;
#pragma unroll
      for (int c = 0; c < V / 2; ++c)
        __hip_atomic_fetch_add(dst + L.at(cur, lp, c), acc[c], __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
      if (counter) {
        const unsigned old = __hip_atomic_fetch_add(nadd + cur, run, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_WORKGROUP) & NADD_MASK;
        if (cur < a.K) seen = old + run > seen ? old + run : seen;  // the sink never flushes
      }
    };
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      float f[V];
      unpack_any<T, PB>(w_[u], f);
      unsigned long long v[V / 2];
#pragma unroll
      for (int e = 0; e < V; e += 2) {
        const float s0 = W ? sc[e] * wt_[u] : sc[e];
        const float s1 = W ? sc[e + 1] * wt_[u] : sc[e + 1];
        if constexpr (RESID)
          v[e / 2] = (unsigned long long)fx_bits_resid(f[e], s0, sc2[e]) |
                     ((unsigned long long)fx_bits_resid(f[e + 1], s1, sc2[e + 1]) << 32);
        else {
          const float r0 = fx_raw<CLAMP>(f[e], s0), r1 = fx_raw<CLAMP>(f[e + 1], s1);
          if constexpr (CLAMP) {
            rlo = fminf(fminf(rlo, r0), r1);
            rhi = fmaxf(fmaxf(rhi, r0), r1);
          }
          v[e / 2] = (unsigned long long)fx_clamp<CLAMP>(r0) | ((unsigned long long)fx_clamp<CLAMP>(r1) << 32);
        }
      }
      if constexpr (W)
        if (wcounter)  // weighted counts: one add per row (slice 0 only)
          __hip_atomic_fetch_add(wcnt + lab_[u], (long long)__float2int_rn(wt_[u] * cscale),
                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      if (u == 0) {
#pragma unroll
        for (int c = 0; c < V / 2; ++c) acc[c] = v[c];
        run = 1;
      } else {
        if (lab_[u] != cur) {  // label changes: emit the run so far
          emit();
          cur = lab_[u];
          run = 0;
#pragma unroll
          for (int c = 0; c < V / 2; ++c) acc[c] = 0;
        }
#pragma unroll
        for (int c = 0; c < V / 2; ++c) acc[c] += v[c];
        ++run;
      }
    }
    emit();
    if (seen >= THRESH) *L.flag(smem) = 1;
    pre_barrier();
    // LDS-only barrier: the prefetched global loads stay in flight
    wait_lgkm0();
    raw_barrier();
  };
  // GSTAGE: thread t < PERIOD stages rows[pbase + t] (clamped to the chunk's last row, as
  // the unstaged tail clamps); the load is issued before the step's X loads, the LDS store
  // happens before the step's closing barrier
  auto idx_load = [&](int64_t pbase, long long* v) {
#pragma unroll
    for (int q = 0; q < GI; ++q) {
      const int t = (int)threadIdx.x + q * NT;
      const int64_t i = pbase + t;
      v[q] = (GSTAGE && t < PERIOD && pbase < row1) ? a.rows[i < row1 ? i : row1 - 1] : 0;
    }
  };
  auto idx_store = [&](int slot, const long long* v) {
#pragma unroll
    for (int q = 0; q < GI; ++q) {
      const int t = (int)threadIdx.x + q * NT;
      // consumed on every lane: the index load's wait then sits here, not at the next
      // step's reuse of the register (which waited for every X load in flight)
      if constexpr (GSTAGE) asm volatile("" ::"v"(v[q]));
      if (GSTAGE && t < PERIOD) gidx[slot * PERIOD + t] = v[q];
    }
  };

  // NB-deep ring of period buffers: NB-1 periods of loads in flight while one accumulates
  constexpr int NB = NBF;
  LT wb[NB][UNR];
  int lb[NB][UNR];
  float tb[NB][UNR];
  if constexpr (GSTAGE) {   // the rows of periods 0..NB-1, slot j % NB for period j
    long long g[NB][GI];
#pragma unroll
    for (int q = 0; q < NB; ++q) idx_load(row0 + (int64_t)q * PERIOD, g[q]);
#pragma unroll
    for (int q = 0; q < NB; ++q) idx_store(q, g[q]);
    __syncthreads();
  }
#pragma unroll
  for (int s = 0; s < NB - 1; ++s)
    if (row0 + (int64_t)s * PERIOD < row1) load(row0 + (int64_t)s * PERIOD, wb[s], lb[s], tb[s], s);
  __syncthreads();
  for (int64_t base = row0; base < row1; base += (int64_t)NB * PERIOD) {
#pragma unroll
    for (int s = 0; s < NB; ++s) {
      const int64_t pb = base + (int64_t)s * PERIOD;
      if (pb < row1) {
        const int64_t nb = pb + (int64_t)(NB - 1) * PERIOD;
        const int ns = (s + NB - 1) % NB;  // static after unrolling
        if constexpr (FLAT) {
          // period j = s (mod NB): X of period j+NB-1 from slot ns; rows of period j+NB into
          // slot s (period j's, read NB-1 steps ago).  The X loads go out unconditionally
          // (past the chunk they clamp to its last row) so every step issues the same loads
          // and the staging store waits only for its own index load.
          long long gv[GI];
          idx_load(pb + (int64_t)NB * PERIOD, gv);   // (no-op unless GSTAGE)
          load(nb, wb[ns], lb[ns], tb[ns], ns);
          accumulate(pb, wb[s], lb[s], tb[s], [&] { idx_store(s, gv); });
        } else {
          if (nb < row1) load(nb, wb[ns], lb[ns], tb[ns], ns);
          accumulate(pb, wb[s], lb[s], tb[s], [] {});
        }
        if (*L.flag(smem)) upd_flush_hot<SW>(a, L, smem, slice, chunk, THRESH / 2);  // batch near-hot labels too
      }
    }
  }
  upd_flush_all<SW>(a, L, smem, slice, chunk);
  if constexpr (CLAMP) {
    if (a.clamp_count) {
      const unsigned long long any = __ballot(!(rlo >= FX_MAGIC - FX_QMAX && rhi <= FX_MAGIC + FX_QMAX));
      if (any && (threadIdx.x & 63) == __builtin_ctzll(any)) atomicAdd(a.clamp_count, 1);
    }
  }
}

// ---------------------------------------------------------------------------
// K-split M-step (plan::choose_ks): for plain full passes (unweighted, not incremental,
// not the residual pass) whenever the column-slice kernel above would need more than one
// slice.  KS workgroups share a row chunk; workgroup j owns labels [j*kq, j*kq + kn) in
// every column.  Each period of KS_NT rows:
//   1. every thread holds one row's label (loaded two periods ahead);
//   2. each wave compacts its rows whose label it owns into a wave-private LDS list
//      (ballot + mbcnt, no atomics);
//   3. the wave reads those rows WHOLE, LPR lanes x 16 B per row (RG = 64/LPR rows per
//      instruction: full 128-B lines, where the slice kernel reads 64-B pieces of 16 rows),
//      GM row groups of the NEXT period in flight while this period's groups accumulate;
//   4. the same fixed-point ds_add_u64 pairs as the slice kernel, so the sums are bitwise
//      identical (integer adds in any order); the per-period barrier and hot-label flush
//      bound every label's adds below FX_LIM.
// The slab layout ([n_chunks][K][D] int64 + [n_chunks][K] counts) and the reduce are
// shared with the slice kernel.
// Cell q of a label holds column pair p = (q % LPR) * NPL + q / LPR (see update_ks_kernel).
template <typename T, int LPR>
__device__ void ks_flush(const UpdateArgs& a, char* m, int kq, int kn, int ldc, int npair, int k0,
                         int chunk, unsigned thresh) {
  constexpr int NPL = 8 / (int)sizeof(T);           // cell pairs per lane
  unsigned long long* cells = (unsigned long long*)m;
  unsigned* nadd = (unsigned*)(cells + (size_t)kq * ldc);
  const int tot = kn * npair;
  for (int e = threadIdx.x; e < tot; e += blockDim.x) {
    const int kl = e / npair, p = e % npair;        // p-major: the slab writes coalesce
    const unsigned na = nadd[kl];
    if ((na & NADD_MASK) < thresh) continue;
    const int q = kl * ldc + (p % NPL) * LPR + p / NPL;
    const unsigned long long T_ = cells[q] - (unsigned long long)(na & NADD_MASK) * FX_MM;
    cells[q] = 0;
    const int lo = (int)(uint32_t)T_;
    const long long hi = (long long)(T_ - (unsigned long long)(long long)lo) >> 32;
    if (2 * p < a.D) {
      long long* dst = a.slab + (int64_t)chunk * a.K * a.D + (int64_t)(k0 + kl) * a.D + 2 * p;
      if (na & NADD_WRITTEN) { dst[0] += lo; if (2 * p + 1 < a.D) dst[1] += hi; }
      else { dst[0] = lo; if (2 * p + 1 < a.D) dst[1] = hi; }
    }
  }
  __syncthreads();
  for (int kl = threadIdx.x; kl < kn; kl += blockDim.x) {
    const unsigned na = nadd[kl];
    if ((na & NADD_MASK) < thresh) continue;
    long long* cd = a.cnt_slab + (int64_t)chunk * a.K + k0 + kl;
    if (na & NADD_WRITTEN) *cd += (long long)(na & NADD_MASK); else *cd = (long long)(na & NADD_MASK);
    nadd[kl] = NADD_WRITTEN;
  }
  __syncthreads();
}

template <typename T, int LPR, int GM, bool CLAMP, bool GATHER = false>
__global__ __launch_bounds__(plan::KS_NT) void update_ks_kernel(UpdateArgs a, int ks, int kq, int ldc,
                                                                int64_t rows_per_chunk) {
  constexpr int NT = plan::KS_NT;
  constexpr int V = 16 / (int)sizeof(T);
  constexpr int RG = 64 / LPR;                      // rows per wave-instruction
  constexpr int NPL = V / 2;                        // cell pairs per lane
  constexpr int NPAIR = LPR * NPL;
  constexpr unsigned THRESH = FX_LIM - NT + 1;      // a period adds <= NT rows to a label
  static_assert(LPR >= 1 && LPR <= 64 && (LPR & (LPR - 1)) == 0, "lanes per row");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  unsigned long long* cells = (unsigned long long*)smem;
  unsigned* nadd = (unsigned*)(cells + (size_t)kq * ldc);
  int* flag = (int*)(nadd + kq);
  unsigned* lists = (unsigned*)(flag + 4);          // [2 periods][NT/64 waves][64]
  // GATHER: the X row of every listed row, [2 periods][NT/64 waves][64], written by the
  // compaction from indices loaded with the labels two periods ahead, so no X load waits on
  // an index load issued after older X loads (vmcnt retires in order: it serialised the
  // row groups in flight)
  const size_t goff = ((size_t)((char*)(lists + 2 * (NT / 64) * 64) - smem) + 7) & ~(size_t)7;
  long long* glists = (long long*)(smem + goff);

  const int b = blockIdx.x, jb = b >> 3;
  const int ksi = jb % ks;
  const int chunk = (jb / ks) * 8 + (b & 7);
  const int k0 = ksi * kq;
  const int kn = a.K - k0 < kq ? a.K - k0 : kq;    // labels this workgroup owns
  if (kn <= 0 || chunk >= a.n_chunks) return;       // (uniform: before any barrier)
  for (int e = threadIdx.x; e < kq * ldc; e += NT) cells[e] = 0;
  for (int e = threadIdx.x; e < kq; e += NT) nadd[e] = 0;
  if (threadIdx.x == 0) *flag = 0;
  __syncthreads();

  const int64_t row0 = (int64_t)chunk * rows_per_chunk;
  int64_t row1 = row0 + rows_per_chunk;
  if (row1 > a.N) row1 = a.N;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int rr = lane / LPR, cc = lane % LPR;
  const int col = cc * V;
  const bool colok = col < a.D;
  float sc[V];
#pragma unroll
  for (int e = 0; e < V; ++e) sc[e] = (col + e < a.D) ? ldexpf(1.f, a.col_exp[col + e]) : 0.f;
  float rlo = FX_MAGIC, rhi = FX_MAGIC;
  unsigned seen = 0;
  const T* xcol = (const T*)a.X + (colok ? col : 0);
  const int64_t rsafe = row0 < row1 ? row0 : 0;    // a valid row for masked lanes

  auto label_at = [&](int64_t i) -> int { return i < row1 ? a.labels[i] : -1; };
  auto xrow_at = [&](int64_t i) -> long long { return GATHER ? (i < row1 ? a.rows[i] : a.rows[rsafe]) : 0; };
  // rows [base + wid*64, +64) of this wave: compact the owned ones into lst (and, gathered,
  // their X rows into gl), return the count
  auto compact = [&](int lab, long long xrow, unsigned* lst, long long* gl) -> int {
    const unsigned rel = (unsigned)(lab - k0);
    const bool m = rel < (unsigned)kn;
    const unsigned long long bal = __ballot(m);
    const int pos = (int)__builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32),
                                                   __builtin_amdgcn_mbcnt_lo((unsigned)bal, 0u));
    if (m) {
      lst[pos] = (unsigned)lane | (rel << 6);
      if constexpr (GATHER) gl[pos] = xrow;
    }
    return (int)__popcll(bal);
  };
  // one row group per instruction: entries [g0 + j*RG, +RG) of lst; label -1 = no row
  auto issue = [&](const unsigned* lst, const long long* gl, int cnt, int64_t wbase, int g0, u32x4* xb,
                   int* lb) {
#pragma unroll
    for (int j = 0; j < GM; ++j) {
      const int e = g0 + j * RG + rr;
      const bool v = e < cnt;
      const unsigned ent = lst[v ? e : 0];
      int64_t row;
      if constexpr (GATHER) row = v ? (int64_t)gl[e] : 0;   // (masked lanes: X row 0; gl[0] may be stale)
      else row = v ? wbase + (int64_t)(ent & 63u) : rsafe;
      xb[j] = *(const u32x4*)(xcol + row * a.ldx);
      lb[j] = v ? (int)(ent >> 6) : -1;
    }
  };
  auto accumulate = [&](const u32x4& w, int kl) {
    float f[V];
    unpack16(colok ? w : u32x4{0u, 0u, 0u, 0u}, f, (T*)nullptr);
    // lane cc's pair j sits in cell j*LPR + cc: the 16 lanes of one ds_add_u64 lane group
    // (ds_write_b64 banking: 16 contiguous lanes, bank (a/4) mod 32) cover 32 consecutive
    // dwords of one label, so every bank once.  Pairs stored per lane (cell cc*NPL + j) put
    // lanes 32 B apart: 4-way conflicts, ~12 extra LDS cycles per instruction at the
    // headline (profiles/r2_21_pmc_headline.md).
    unsigned long long* dst = cells + kl * ldc + cc;
#pragma unroll
    for (int e = 0; e < V; e += 2) {
      const float r0 = fx_raw<CLAMP>(f[e], sc[e]), r1 = fx_raw<CLAMP>(f[e + 1], sc[e + 1]);
      if constexpr (CLAMP) {
        rlo = fminf(fminf(rlo, r0), r1);
        rhi = fmaxf(fmaxf(rhi, r0), r1);
      }
      const unsigned long long v = (unsigned long long)fx_clamp<CLAMP>(r0) |
                                   ((unsigned long long)fx_clamp<CLAMP>(r1) << 32);
      __hip_atomic_fetch_add(dst + (e / 2) * LPR, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    if (cc == 0) {
      const unsigned old = __hip_atomic_fetch_add(nadd + kl, 1u, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_WORKGROUP) & NADD_MASK;
      seen = old + 1 > seen ? old + 1 : seen;
    }
  };

  unsigned* lbuf0 = lists + wid * 64;
  unsigned* lbuf1 = lists + (NT / 64) * 64 + wid * 64;
  long long* gbuf0 = glists + wid * 64;
  long long* gbuf1 = glists + (NT / 64) * 64 + wid * 64;
  // prologue: period 0 compacted and its first groups in flight, period 1's labels loaded
  int lab_next = label_at(row0 + NT + threadIdx.x);
  long long xr_next = xrow_at(row0 + NT + threadIdx.x);
  int cnt = compact(label_at(row0 + threadIdx.x), xrow_at(row0 + threadIdx.x), lbuf0, gbuf0);
  u32x4 xa[GM], xb[GM];
  int la[GM], lb[GM];
  int cnt_b = 0;
  issue(lbuf0, gbuf0, cnt, row0 + wid * 64, 0, xa, la);
  // One period: compact and issue the NEXT period's row groups into (xn, ln), then
  // accumulate this period's (xc, lc).  Called twice per loop trip with the two register
  // sets swapped (ping-pong, no copies): a rolled loop copied xb into xa at the latch, which
  // waited for every next-period load before the next labels were even read.
  auto period = [&](int64_t base, u32x4* xc, int* lc, int cc_, const unsigned* lcur, const long long* gcur,
                    u32x4* xn, int* ln, int& cn_, unsigned* lnxt, long long* gnxt) {
    const int lab_nn = label_at(base + 2 * NT + threadIdx.x);
    const long long xr_nn = xrow_at(base + 2 * NT + threadIdx.x);
    cn_ = compact(lab_next, xr_next, lnxt, gnxt);
    issue(lnxt, gnxt, cn_, base + NT + wid * 64, 0, xn, ln);
#pragma unroll
    for (int j = 0; j < GM; ++j)
      if (lc[j] >= 0) accumulate(xc[j], lc[j]);
    // rare: more owned rows than GM groups hold -- the rest synchronously
    for (int g0 = GM * RG; g0 < cc_; g0 += RG) {
      const int e = g0 + rr;
      if (e < cc_) {
        const unsigned ent = lcur[e];
        const int64_t row = GATHER ? (int64_t)gcur[e] : base + wid * 64 + (int64_t)(ent & 63u);
        const u32x4 w = *(const u32x4*)(xcol + row * a.ldx);
        accumulate(w, (int)(ent >> 6));
      }
    }
    if (seen >= THRESH) *flag = 1;
    __syncthreads();
    if (*flag) {
      ks_flush<T, LPR>(a, smem, kq, kn, ldc, NPAIR, k0, chunk, THRESH / 2);
      if (threadIdx.x == 0) *flag = 0;
      seen = 0;
      __syncthreads();
    }
    lab_next = lab_nn;
    xr_next = xr_nn;
  };
  for (int64_t base = row0; base < row1; base += 2 * NT) {
    period(base, xa, la, cnt, lbuf0, gbuf0, xb, lb, cnt_b, lbuf1, gbuf1);
    if (base + NT >= row1) break;   // (uniform)
    period(base + NT, xb, lb, cnt_b, lbuf1, gbuf1, xa, la, cnt, lbuf0, gbuf0);
  }
  __syncthreads();
  ks_flush<T, LPR>(a, smem, kq, kn, ldc, NPAIR, k0, chunk, 0u);
  if constexpr (CLAMP) {
    if (a.clamp_count) {
      const unsigned long long any = __ballot(!(rlo >= FX_MAGIC - FX_QMAX && rhi <= FX_MAGIC + FX_QMAX));
      if (any && lane == __builtin_ctzll(any)) atomicAdd(a.clamp_count, 1);
    }
  }
}

// Fallback for K too large to privatise even 2 columns: direct int64 global atomics
// (same fixed-point contributions, so results match the LDS path bit for bit).
template <typename T>
__global__ __launch_bounds__(256) void update_global_kernel(UpdateArgs a) {
  const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (i >= a.N) return;
  const int k = a.labels[i];
  if ((unsigned)k >= (unsigned)a.K) return;
  const float wt = a.weights ? a.weights[i] : 1.f;
  const T* xr = (const T*)a.X + (a.rows ? a.rows[i] : i) * a.ldx;
  for (int d = lane; d < a.D; d += 64)
    atomicAdd((unsigned long long*)(a.slab + (int64_t)k * a.D + d),
              (unsigned long long)fx_q(Elem<T>::to_f32(xr[d]), ldexpf(1.f, a.col_exp[d]) * wt));
  if (lane == 0)
    atomicAdd((unsigned long long*)(a.cnt_slab + k),
              (unsigned long long)(a.weights ? (long long)__float2int_rn(wt * ldexpf(1.f, a.cnt_exp))
                                             : 1ll));
}

static int esize(int dtype) { return dtype == DT_BF16 ? 2 : 4; }

// Cap on the slice width (0 = none).  A smaller slice shrinks the LDS footprint
// so an update workgroup can be co-resident with assign workgroups when the
// engine overlaps the two kernels on separate streams.
static int g_update_max_sw = 0;
void set_update_max_sw(int sw) { g_update_max_sw = sw; }

static int choose_sw(int dtype, int K, int D, bool weighted, int* ldc) {
  return plan::choose_sw(esize(dtype), K, D, weighted, g_update_max_sw, ldc);
}

int update_slice_width(int dtype, int K, int D, bool weighted) {
  int ldc;
  return choose_sw(dtype, K, D, weighted, &ldc);
}

static int esize(int dtype);

// The K-split kernel serves plain full passes where the slice kernel needs 2+ slices of
// under 128 B per row: N=1e8 D=128 K=1024 bf16 (64-B pieces) 5.20 -> 4.67 ms, N=1e7 D=64
// K=4096 (16-B pieces) 0.62 -> 0.44 ms; with 128-B or wider pieces (cfg5's 64 bf16
// columns, cfg2's 64 f32 columns) the slice kernel already reads whole lines and is as fast
// or faster (profiles/r2_05_update_study.md).
static bool use_ks(int dtype, int K, int D, bool weighted, plan::KsPlan* kp) {
  if (weighted) return false;
  const int sw = update_slice_width(dtype, K, D, false);
  // A/B override (0 = slice kernel, 1 = K-split); the memory planner assumes the default.
  // cfg5 (D=256 K=512, 128-B slices): K-split 6.58 vs slice 6.03 ms per resident step
  // (profiles/r3_09_update_ks_cfg5_ab.log), so the rule below stands.
  const int ov = variant(V_UPDATE_KS);
  if (ov >= 0) return ov != 0 && sw > 0 && sw < D && plan::choose_ks(esize(dtype), K, D, kp);
  return sw > 0 && sw < D && sw * esize(dtype) < 128 && plan::choose_ks(esize(dtype), K, D, kp);
}

int update_n_chunks(int dtype, int K, int D, int64_t N, bool weighted) {
  const int nc = plan::update_n_chunks(update_slice_width(dtype, K, D, weighted), D, N);
  plan::KsPlan kp;
  return use_ks(dtype, K, D, weighted, &kp) ? plan::update_n_chunks_ks(kp.ks, nc) : nc;
}

int fixed_exp(double maxabs) { return plan::fixed_exp(maxabs); }

template <typename T, int SW, int MODE, int NT, int NBF = UPD_NBUF, int PER = UPD_MAX_PERIOD>
static hipError_t launch_nt(const UpdateArgs& a, int ldc, hipStream_t s) {
  const int n_slices = (a.D + SW - 1) / SW;
  const int64_t rows_per_chunk = (a.N + a.n_chunks - 1) / a.n_chunks;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)update_kernel<T, SW, MODE, NT, NBF, PER>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)UPD_LDS_MAX);
    attr = true;
  }
  size_t lds = upd_lds_bytes(a.K, ldc, (MODE & (UPD_WEIGHTED | UPD_DELTA)) != 0);
  if constexpr ((MODE & UPD_GSTAGE) != 0) lds += (size_t)NBF * upd_period<T, SW, NT, PER>() * 8;
  hipLaunchKernelGGL((update_kernel<T, SW, MODE, NT, NBF, PER>), dim3(a.n_chunks * n_slices), dim3(NT), lds, s, a,
                     n_slices, rows_per_chunk);
  return hipGetLastError();
}

// 1024 threads (4 waves per SIMD, <= 128 VGPRs) where the period buffers fit without
// spilling; measured at N=1e8 D=128 K=1024 bf16: 5.67 ms vs 5.89 (512) vs 6.74 (256).
// 64-column slices (K <= ~600) take a 3-deep ring to stay under 128 VGPRs: 1.64 ms vs
// 1.95 at 512 threads for the cfg5 batch (N=16.8M D=256 K=512; profiles/r2_05_update_study.md).
// The clamped 64-column body (mini-batch without a value bound) takes a 2-deep ring:
// 1.79 ms vs 2.02 at 512 threads; a 3-deep one would spill 32 VGPRs.
// f32, 64-column slices, plain adds: 1024 threads with a 2-deep ring, 1.80 vs 2.02 ms at
// N=2e7 D=128 K=256 (0.121 vs 0.126 at cfg2's N=1e6; profiles/r2_05_update_study.md).
template <typename T, int SW, int MODE>
constexpr int upd_default_nt() {
  if constexpr (sizeof(T) == 4)
    return (SW == 64 && !(MODE & (UPD_WEIGHTED | UPD_DELTA | UPD_CLAMP | UPD_RESID))) ? 1024 : UPD_NT;
  return (SW <= 64 && !(MODE & (UPD_WEIGHTED | UPD_DELTA))) ? 1024 : UPD_NT;
}
template <typename T, int SW, int MODE>
constexpr int upd_ring_1024() {
  return sizeof(T) == 4 ? 2 : SW <= 32 ? 6 : (MODE & UPD_CLAMP) ? 2 : 3;
}

template <typename T, int SW, int MODE>
static hipError_t launch_sw(const UpdateArgs& a, int ldc, hipStream_t s) {
  constexpr int NT = upd_default_nt<T, SW, MODE>();
  // 1024 threads: 512-row periods, 6-deep ring (5 periods of loads in flight; 3-deep for
  // 64-column slices).  N=1e8 D=128 K=1024 bf16: 5.33-5.76 ms vs 5.96-6.34 for 3 x
  // 1024-row periods (same boxes).
  constexpr int ES = sizeof(T);
  constexpr int V = ((SW * ES >= 16) ? 16 : SW * ES) / ES;
  constexpr int RPP = NT / (SW / V);
  constexpr int PER = RPP > 512 ? RPP : 512;
  if constexpr ((MODE & UPD_GSTAGE) != 0) {   // the staged-index ring must fit beside the cells
    constexpr int NBF = NT == 1024 ? upd_ring_1024<T, SW, MODE>() : UPD_NBUF;
    constexpr int P = NT == 1024 ? upd_period<T, SW, NT, PER>() : upd_period<T, SW, NT, UPD_MAX_PERIOD>();
    if (upd_lds_bytes(a.K, ldc, false) + (size_t)NBF * P * 8 > UPD_LDS_MAX)
      return launch_sw<T, SW, (MODE & ~UPD_GSTAGE)>(a, ldc, s);
  }
  if constexpr (NT == 1024) return launch_nt<T, SW, MODE, 1024, upd_ring_1024<T, SW, MODE>(), PER>(a, ldc, s);
  else return launch_nt<T, SW, MODE, NT>(a, ldc, s);
}

template <typename T, int SW>
static hipError_t launch_clamp(const UpdateArgs& a, int ldc, hipStream_t s) {
  const int mode = (a.clamp ? UPD_CLAMP : 0) | (a.weights ? UPD_WEIGHTED : 0) |
                   (ldc == SW / 2 ? UPD_SWZ : 0);
  if (a.col_exp2) {  // residual (lo) pass of the wide-range columns: never clamped / incremental
    if (a.clamp || a.dlist || a.rows) return hipErrorInvalidValue;
    switch (mode) {
      case 0: return launch_sw<T, SW, UPD_RESID>(a, ldc, s);
      case 2: return launch_sw<T, SW, UPD_RESID | UPD_WEIGHTED>(a, ldc, s);
      case 4: return launch_sw<T, SW, UPD_RESID | UPD_SWZ>(a, ldc, s);
      default: return launch_sw<T, SW, UPD_RESID | UPD_WEIGHTED | UPD_SWZ>(a, ldc, s);
    }
  }
  if (a.rows) {  // gathered mini-batch rows: plain (bounded, unclamped) passes only
    if (a.clamp || a.dlist) return hipErrorInvalidValue;
    switch (mode) {
      case 0: return launch_sw<T, SW, UPD_GATHER | UPD_GSTAGE>(a, ldc, s);
      case 2: return launch_sw<T, SW, UPD_GATHER | UPD_WEIGHTED>(a, ldc, s);
      case 4: return launch_sw<T, SW, UPD_GATHER | UPD_SWZ | UPD_GSTAGE>(a, ldc, s);
      default: return launch_sw<T, SW, UPD_GATHER | UPD_WEIGHTED | UPD_SWZ>(a, ldc, s);
    }
  }
  if (a.dlist) {  // incremental M-step (Lloyd: never clamped; weights read at run time)
    if (a.clamp) return hipErrorInvalidValue;
    return (mode & UPD_SWZ) ? launch_sw<T, SW, UPD_DELTA | UPD_SWZ>(a, ldc, s)
                            : launch_sw<T, SW, UPD_DELTA>(a, ldc, s);
  }
  switch (mode) {
    case 0: return launch_sw<T, SW, 0>(a, ldc, s);
    case 1: return launch_sw<T, SW, 1>(a, ldc, s);
    case 2: return launch_sw<T, SW, 2>(a, ldc, s);
    case 3: return launch_sw<T, SW, 3>(a, ldc, s);
    case 4: return launch_sw<T, SW, 4>(a, ldc, s);
    case 5: return launch_sw<T, SW, 5>(a, ldc, s);
    case 6: return launch_sw<T, SW, 6>(a, ldc, s);
    default: return launch_sw<T, SW, 7>(a, ldc, s);
  }
}

template <typename T>
static hipError_t launch_update_t(const UpdateArgs& a, hipStream_t s, int sw, int ldc) {
  switch (sw) {
    case 64: return launch_clamp<T, 64>(a, ldc, s);
    case 32: return launch_clamp<T, 32>(a, ldc, s);
    case 16: return launch_clamp<T, 16>(a, ldc, s);
    case 8: return launch_clamp<T, 8>(a, ldc, s);
    case 4: return launch_clamp<T, 4>(a, ldc, s);
    case 2: return launch_clamp<T, 2>(a, ldc, s);
    case 0:
      // caller zeroed slab[K*D] + cnt_slab[K] (n_chunks == 1)
      hipLaunchKernelGGL((update_global_kernel<T>), dim3((unsigned)((a.N + 3) / 4)), dim3(256), 0,
                         s, a);
      return hipGetLastError();
  }
  return hipErrorInvalidValue;
}

template <typename T, int LPR, int GM, bool CLAMP, bool GATHER = false>
static hipError_t launch_ks_t(const UpdateArgs& a, const plan::KsPlan& kp, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)update_ks_kernel<T, LPR, GM, CLAMP, GATHER>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)UPD_LDS_MAX);
    attr = true;
  }
  const int64_t rows_per_chunk = (a.N + a.n_chunks - 1) / a.n_chunks;
  const size_t lds = plan::ks_lds_bytes(kp.kq, kp.ldc) + (GATHER ? plan::KS_GLIST_BYTES : 0);
  if (lds > UPD_LDS_MAX) return hipErrorInvalidValue;
  hipLaunchKernelGGL((update_ks_kernel<T, LPR, GM, CLAMP, GATHER>), dim3((unsigned)(a.n_chunks * kp.ks)),
                     dim3(plan::KS_NT), lds, s, a, kp.ks, kp.kq, kp.ldc, rows_per_chunk);
  return hipGetLastError();
}

template <typename T, int LPR>
static hipError_t launch_ks_l(const UpdateArgs& a, const plan::KsPlan& kp, hipStream_t s) {
  if (a.rows) {  // gathered mini-batch rows (bounded scales: never clamped)
    if (a.clamp) return hipErrorInvalidValue;
    if (kp.gm == 6) return launch_ks_t<T, LPR, 6, false, true>(a, kp, s);
    if (kp.gm == 3) return launch_ks_t<T, LPR, 3, false, true>(a, kp, s);
    return launch_ks_t<T, LPR, 2, false, true>(a, kp, s);
  }
  if (kp.gm == 6) return a.clamp ? launch_ks_t<T, LPR, 6, true>(a, kp, s) : launch_ks_t<T, LPR, 6, false>(a, kp, s);
  if (kp.gm == 3) return a.clamp ? launch_ks_t<T, LPR, 3, true>(a, kp, s) : launch_ks_t<T, LPR, 3, false>(a, kp, s);
  return a.clamp ? launch_ks_t<T, LPR, 2, true>(a, kp, s) : launch_ks_t<T, LPR, 2, false>(a, kp, s);
}

template <typename T>
static hipError_t launch_ks(const UpdateArgs& a, const plan::KsPlan& kp, hipStream_t s) {
  switch (kp.lpr) {
    case 8: return launch_ks_l<T, 8>(a, kp, s);
    case 16: return launch_ks_l<T, 16>(a, kp, s);
    case 32: return launch_ks_l<T, 32>(a, kp, s);
    case 64: return launch_ks_l<T, 64>(a, kp, s);
  }
  return hipErrorInvalidValue;
}

hipError_t launch_update(int dtype, const UpdateArgs& a, hipStream_t s) {
  if (a.N <= 0) return hipSuccess;
  plan::KsPlan kp;
  // (gathered batches stage their X rows in LDS too; where that does not fit, the slice
  // kernel takes the pass -- any chunk count that is a multiple of 8 serves it)
  if (!a.dlist && !a.col_exp2 && use_ks(dtype, a.K, a.D, a.weights != nullptr, &kp) &&
      (!a.rows || plan::ks_lds_bytes(kp.kq, kp.ldc) + plan::KS_GLIST_BYTES <= UPD_LDS_MAX)) {
    if (a.n_chunks % 8) return hipErrorInvalidValue;
    {   // A/B override of the row groups in flight (2, 3 or 6).  With the ping-pong periods the
        // plan's choice still wins: cfg4 2 > 3 > 6, headline 6 > 3 > 2 (profiles/r3_30_ks_gm_ab.log)
      const int gm = variant(V_UPDATE_KS_GM);
      if (gm == 2 || gm == 3 || gm == 6) kp.gm = gm;
    }
    return dtype == DT_BF16 ? launch_ks<uint16_t>(a, kp, s) : launch_ks<float>(a, kp, s);
  }
  int ldc = 0;
  const int sw = choose_sw(dtype, a.K, a.D, a.weights != nullptr || a.dlist != nullptr, &ldc);
  if (sw > 0 && a.n_chunks % 8) return hipErrorInvalidValue;
  if (a.dlist && sw == 0) return hipErrorInvalidValue;  // no incremental global fallback
  if (a.col_exp2 && sw == 0) return hipErrorInvalidValue;  // residual pass needs the LDS path
  return dtype == DT_BF16 ? launch_update_t<uint16_t>(a, s, sw, ldc)
                          : launch_update_t<float>(a, s, sw, ldc);
}

// ---------------------------------------------------------------------------
// The assign kernel's slots (common.h slot_add) -> out[0] = inertia, out[1] = changed rows,
// then re-zeroed.  Integer word totals, decoded in a fixed order: the same bits whatever
// order the assign's workgroups added in.  One 256-thread workgroup.
__device__ void slots_collect(double* slots, double* out) {
  __shared__ long long red[4][SLOT_STRIDE];
  long long w[SLOT_STRIDE];
#pragma unroll
  for (int j = 0; j < SLOT_STRIDE; ++j) w[j] = 0;
  if (slots) {
    unsigned long long* s = (unsigned long long*)slots;
    for (int i = threadIdx.x; i < NSLOT; i += 256) {
#pragma unroll
      for (int j = 0; j < SLOT_STRIDE; ++j) {
        w[j] += (long long)s[i * SLOT_STRIDE + j];
        s[i * SLOT_STRIDE + j] = 0ull;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < SLOT_STRIDE; ++j) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) w[j] += __shfl_xor(w[j], o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6][j] = w[j];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    long long W[SLOT_STRIDE];
#pragma unroll
    for (int j = 0; j < SLOT_STRIDE; ++j) W[j] = red[0][j] + red[1][j] + red[2][j] + red[3][j];
    out[0] = slot_decode(W);
    out[1] = (double)W[7];
  }
}

// ---------------------------------------------------------------------------
// launch_reduce: packed[k*D+d] = 2^-exp[d] * sum_c slab[c][k][d] (f64, exact: every
// partial is an integer below 2^53), counts likewise,
// plus the assign kernel's inertia / changed slots (which it then re-zeroes).
__global__ __launch_bounds__(256) void reduce_kernel(const long long* __restrict__ slab,
                                                     const long long* __restrict__ cnt_slab,
                                                     int n_chunks, int K, int D,
                                                     const int* __restrict__ col_exp,
                                                     double inv_c, double* slots, double* packed,
                                                     long long* tot, const int* dcount, int dcap) {
  const int64_t KD = (int64_t)K * D;
  const int64_t total = KD + K;
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e < total && tot) {  // incremental: running integer totals (exact, order-free)
    const long long* src = e < KD ? slab + e : cnt_slab + (e - KD);
    const int64_t stride = e < KD ? KD : K;
    long long acc = 0;
    for (int c = 0; c < n_chunks; ++c) acc += src[(int64_t)c * stride];
    const long long t = (*dcount > dcap) ? acc : tot[e] + acc;
    tot[e] = t;
    packed[e] = e < KD ? ldexp((double)t, -col_exp[e % D]) : (double)t * inv_c;
  } else if (e < total) {
    double acc = 0.0;
    if (e < KD) {
      for (int c = 0; c < n_chunks; ++c) acc += (double)slab[(int64_t)c * KD + e];
      acc = ldexp(acc, -col_exp[e % D]);
    } else {
      const int64_t k = e - KD;
      for (int c = 0; c < n_chunks; ++c) acc += (double)cnt_slab[(int64_t)c * K + k];
      acc *= inv_c;
    }
    packed[e] = acc;
  }
  // (the slots' own workgroup, one past the message's: it runs beside the others)
  if (blockIdx.x == gridDim.x - 1) slots_collect(slots, packed + total);
}

hipError_t launch_reduce(const long long* slab, const long long* cnt_slab, int n_chunks, int K,
                         int D, const int* col_exp, int cnt_exp, double* slots, double* packed,
                         hipStream_t s, long long* tot, const int* dcount, int dcap) {
  if (tot && !dcount) return hipErrorInvalidValue;
  const int64_t total = (int64_t)K * D + K;
  const unsigned nb = (unsigned)((total + 255) / 256) + 1;
  hipLaunchKernelGGL(reduce_kernel, dim3(nb), dim3(256), 0, s, slab, cnt_slab, n_chunks, K, D,
                     col_exp, ldexp(1.0, -cnt_exp), slots, packed, tot, dcount, dcap);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// launch_reduce_cols: out[k*nw + j] = 2^-exps[j] * sum_c slab[c][k][cols[j]] (f64, exact:
// integer partials below 2^53) -- the lo sums of the wide-range columns, appended to the
// all-reduce message and added onto the hi sums after it.
__global__ __launch_bounds__(256) void reduce_cols_kernel(const long long* __restrict__ slab, int n_chunks,
                                                          int K, int D, const int* __restrict__ cols,
                                                          const int* __restrict__ exps, int nw,
                                                          double* __restrict__ out) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= (int64_t)K * nw) return;
  const int k = (int)(e / nw), j = (int)(e % nw);
  const int64_t KD = (int64_t)K * D;
  const long long* src = slab + (int64_t)k * D + cols[j];
  long long acc = 0;
  for (int c = 0; c < n_chunks; ++c) acc += src[(int64_t)c * KD];
  out[e] = ldexp((double)acc, -exps[j]);
}

hipError_t launch_reduce_cols(const long long* slab, int n_chunks, int K, int D, const int* cols,
                              const int* exps, int nw, double* out, hipStream_t s) {
  const int64_t total = (int64_t)K * nw;
  if (total <= 0) return hipSuccess;
  hipLaunchKernelGGL(reduce_cols_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, slab,
                     n_chunks, K, D, cols, exps, nw, out);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// launch_label_delta: the changed-row list of the incremental M-step.  Each thread
// checks LD_R rows (coalesced, stride 256); a workgroup reserves its list range with
// one global atomic.  List order is not deterministic, but the M-step sums are
// integers, so the result is.
constexpr int LD_R = 16;

__global__ __launch_bounds__(256) void label_delta_kernel(const int32_t* __restrict__ labels,
                                                          int32_t* __restrict__ prev, int64_t N,
                                                          int2* __restrict__ list, int cap,
                                                          int* count) {
  __shared__ int wg_n, wg_base;
  if (threadIdx.x == 0) wg_n = 0;
  __syncthreads();
  const int64_t b0 = (int64_t)blockIdx.x * 256 * LD_R + threadIdx.x;
  int lab[LD_R], old[LD_R];
  unsigned m = 0;
#pragma unroll
  for (int t = 0; t < LD_R; ++t) {
    const int64_t i = b0 + t * 256;
    if (i < N) {
      lab[t] = labels[i];
      old[t] = prev[i];
      if (lab[t] != old[t]) m |= 1u << t;
    }
  }
  const int n = __popc(m);
  const int off = n ? atomicAdd(&wg_n, n) : 0;
  __syncthreads();
  if (threadIdx.x == 0) wg_base = wg_n ? atomicAdd(count, wg_n) : 0;
  __syncthreads();
  int pos = wg_base + off;
#pragma unroll
  for (int t = 0; t < LD_R; ++t) {
    if (m >> t & 1u) {
      const int64_t i = b0 + t * 256;
      prev[i] = lab[t];
      if (pos < cap) list[pos] = make_int2((int)i, old[t]);
      ++pos;
    }
  }
}

// The same over a candidate list rows[0..*rcount) (the bounded E-step re-assigned only those
// rows, so no other label can have changed): a pass over the candidates instead of all N.
// LDR_R candidates per thread and pass (coalesced, stride 256), all their loads in flight
// before any is used, and ONE global atomic per workgroup pass: with one candidate per thread
// the workgroups' reservations on the single list counter serialised (0.43 ms for 11M
// candidates at N=1e8, profiles/r6_29_rocprof_bounded.md).
constexpr int LDR_R = 8;

__global__ __launch_bounds__(256) void label_delta_rows_kernel(const int32_t* __restrict__ labels,
                                                               int32_t* __restrict__ prev,
                                                               const int64_t* __restrict__ rows,
                                                               const int64_t* __restrict__ rcount,
                                                               int2* __restrict__ list, int cap, int* count) {
  __shared__ int wg_n, wg_base;
  const int64_t m = rcount[0];
  const int64_t span = (int64_t)256 * LDR_R;
  for (int64_t base = (int64_t)blockIdx.x * span; base < m; base += (int64_t)gridDim.x * span) {  // block-uniform
    if (threadIdx.x == 0) wg_n = 0;
    __syncthreads();
    int64_t i[LDR_R];
#pragma unroll
    for (int t = 0; t < LDR_R; ++t) {
      const int64_t j = base + t * 256 + threadIdx.x;
      i[t] = j < m ? rows[j] : -1;
    }
    int lab[LDR_R], old[LDR_R];
    unsigned ch = 0;
#pragma unroll
    for (int t = 0; t < LDR_R; ++t) {
      lab[t] = i[t] >= 0 ? labels[i[t]] : 0;
      old[t] = i[t] >= 0 ? prev[i[t]] : 0;
    }
#pragma unroll
    for (int t = 0; t < LDR_R; ++t)
      if (i[t] >= 0 && lab[t] != old[t]) ch |= 1u << t;
    const int n = __popc(ch);
    const int off = n ? atomicAdd(&wg_n, n) : 0;
    __syncthreads();
    if (threadIdx.x == 0) wg_base = wg_n ? atomicAdd(count, wg_n) : 0;
    __syncthreads();
    int pos = wg_base + off;
#pragma unroll
    for (int t = 0; t < LDR_R; ++t) {
      if (ch >> t & 1u) {
        prev[i[t]] = lab[t];
        if (pos < cap) list[pos] = make_int2((int)i[t], old[t]);
        ++pos;
      }
    }
    __syncthreads();   // (wg_n / wg_base are rewritten by the next pass)
  }
}

hipError_t launch_label_delta_rows(const int32_t* labels, int32_t* prev, const int64_t* rows, const int64_t* rcount,
                                   int64_t n_max, int2* list, int cap, int* count, hipStream_t s) {
  hipError_t e = hipMemsetAsync(count, 0, sizeof(int), s);
  if (e != hipSuccess || n_max <= 0) return e;
  int64_t nb = (n_max + 256 * LDR_R - 1) / (256 * LDR_R);
  if (nb > 2048) nb = 2048;
  hipLaunchKernelGGL(label_delta_rows_kernel, dim3((unsigned)nb), dim3(256), 0, s, labels, prev, rows, rcount,
                     list, cap, count);
  return hipGetLastError();
}

hipError_t launch_label_delta(const int32_t* labels, int32_t* prev, int64_t N, int2* list, int cap,
                              int* count, hipStream_t s) {
  if (N >= (int64_t)1 << 31) return hipErrorInvalidValue;
  hipError_t e = hipMemsetAsync(count, 0, sizeof(int), s);
  if (e != hipSuccess || N <= 0) return e;
  const int64_t per = 256 * LD_R;
  hipLaunchKernelGGL(label_delta_kernel, dim3((unsigned)((N + per - 1) / per)), dim3(256), 0, s,
                     labels, prev, N, list, cap, count);
  return hipGetLastError();
}

}  // namespace mk
