// mikmeans — K2: nearest-centroid assignment on 16x16 MFMA tiles for gfx950
// (v_mfma_f32_16x16x32_bf16 / v_mfma_f32_16x16x4_f32).
//
// Pipeline: fragment-packed centroid chunks stream through an LDS ring fed by LDS-DMA
// (global_load_lds_dwordx4, no VGPR round trip); every wave keeps P blocks of 16
// points in registers and multiplies them against each 16-centroid tile:
//  * lane (r = l&15, g = l>>4) holds the B fragments of point p0+r, piece q covering
//    features [(4q+g)V, +V) (V = 16 B of elements), and the A fragments of centroid r
//    of the tile (the packed -2c), same features.  Interleaving the lane groups' pieces
//    makes each fragment load read 64 contiguous bytes per point (16 rows per wave
//    instruction); giving each lane group a contiguous quarter of the row instead made
//    every load touch 64 cache lines, and the loads cost a fixed ~27 % of the D=256
//    K=512 assign (profiles/r2_08_assign_clock_study.md);
//  * the accumulators are seeded with |c|^2 (+ the point offset below), so the output
//    D[row = 4g+reg][col = r] is the score of point r against centroid 16t+4g+reg and
//    each lane holds 4 scores of its point per tile; the 4 lane groups g merge once at
//    the end.
//
// Argmin epilogue.
//  * bf16: keys carry a 6-bit index in the low mantissa bits (tile-in-segment*4 + reg)
//    so one v_min3 tree yields (min, index): 1.5 VALU per score.  The workgroup adds
//    o = (1 + 2^-12) max |x|^2 over its 192-512 points to its LDS copy of |c|^2 once,
//    which makes every key |x-c|^2 + (o - |x|^2) > 0: among equal keys the lower index
//    then always wins (an OR of the index into a NEGATIVE float favours the higher one),
//    and the key resolution is 2^-17 of the squared distance plus the spread of |x|^2
//    inside the workgroup, not 2^-17 of |x|^2 (coarse for data far from the origin).
//    Where that spread is large (max |x|^2 > 4 min |x|^2: an outlier row, data around the
//    origin) the workgroup uses per-point offsets instead (they seed each tile's
//    accumulators, in a second instantiation of the chunk loop), so the resolution is never
//    worse than 2^-17 (|x-c|^2 + 3|x|^2).  Per-point offsets everywhere would make the keys
//    a function of the point alone, but cost 17 % at the headline shape (one process A/B,
//    round 2); workgroups are therefore aligned to the global ROW_ALIGN = 1536-row grid by
//    the callers (shard_range, streaming chunks), so near-tie resolution is the same on
//    any world size.
//  * bf16 D <= 64 with many centres (VARG): the keys' 1.5 VALU per score bound the body
//    (1-2 MFMAs per tile and block), so the main loop keeps only the running minimum value
//    (2 v_min3_u32 per tile and block: the positive scores order as their bits) and the
//    tile that lowered it (v_cmp + v_cndmask): 1.0 VALU per score.  After the loop the
//    winning tile's 4 candidate rows of every point are recomputed on the matrix cores,
//    bitwise the main loop's scores, and the first equal to the minimum is the label
//    (full fp32 resolution; 64/K extra matrix work, so K >= 2048 at D=64, >= 1024 at D=32).
//  * f32: an exact (value, index) compare per score (v_cmp + 2 v_cndmask).  The f32
//    MFMA is 16x slower per FLOP than bf16, so the epilogue is noise there and the
//    labels carry full fp32 score resolution; strict < in ascending index order keeps
//    the lowest index on exact ties.
//
// Layout "16" of the packed centroids (csrc/kernels.h):
//   element (k, d): t = k/16, r = k%16, q = d / (4V), g = (d / V) % 4
//   offset = ((t*NQ + q)*64 + r + 16*g)*V + d%V,  NQ = DPAD/(4V)
#include <cstdlib>
#include <type_traits>

#include "common.h"
#include "kernels.h"
#include "plan.h"

namespace mk {

using plan::chunk_tiles16;

// CT_: tiles per LDS chunk (0 = the 16 KiB default, which also fixes Kpad's
// granule); NBUF_: ring slots (prefetch depth NBUF-1).
template <typename T, int DPAD, int P_, int CT_ = 0, int NBUF_ = 2, int NW_ = 4>
struct Assign16Cfg {
  static constexpr int NW = NW_;                // waves per workgroup sharing the ring
  static constexpr int P = P_;                  // 16-point blocks per wave
  static constexpr int V = Elem<T>::V;
  static constexpr int NQ = DPAD / 4 / V;       // 16-B pieces per lane per point
  static constexpr int TILE_BYTES = NQ * 1024;  // 16 centroids x DPAD
  static constexpr int CT = CT_ ? CT_ : chunk_tiles16(sizeof(T), DPAD);
  static constexpr int CHUNK_BYTES = CT * TILE_BYTES;
  static constexpr int PIECES = CHUNK_BYTES / 1024;
  static constexpr int NPW = PIECES / NW;
  static constexpr int PTS = NW * P * 16;
  static constexpr int PP = (P + 3) / 4 * 4;    // per-point offset slots per lane (LDS, f32x4 reads)
  static constexpr int OPT_BYTES = 2 * NW * 16 * PP * 4;   // offsets + gathered |x|^2
  static constexpr int NBUF = NBUF_;
  static_assert(NBUF == 2 || NBUF == 3, "ring depth");
  static_assert(chunk_tiles16(sizeof(T), DPAD) % CT == 0 || CT % chunk_tiles16(sizeof(T), DPAD) == 0,
                "chunk and the Kpad granule must nest (a wider chunk runs only where Kpad is a multiple of it)");
  static_assert(NQ >= 1, "DPAD too small for the 16x16 layout");
  static_assert(PIECES % NW == 0, "chunk pieces must split evenly over waves");
};

template <typename T> struct Mfma16;
template <> struct Mfma16<uint16_t> {
  __device__ static __forceinline__ f32x4 run(const u32x4& a, const u32x4& b, const f32x4& c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(short8, a),
                                                   __builtin_bit_cast(short8, b), c, 0, 0, 0);
  }
};
template <> struct Mfma16<float> {
  __device__ static __forceinline__ f32x4 run(const u32x4& a, const u32x4& b, f32x4 c) {
#pragma unroll
    for (int e = 0; e < 4; ++e)
      c = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a[e]), __uint_as_float(b[e]), c, 0, 0, 0);
    return c;
  }
};

// Sum of squares of one lane's 16-byte piece.
__device__ __forceinline__ float sq16(const u32x4& w, uint16_t*) {
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float lo = bf16lo(w[i]), hi = bf16hi(w[i]);
    s = __builtin_fmaf(lo, lo, s);
    s = __builtin_fmaf(hi, hi, s);
  }
  return s;
}
__device__ __forceinline__ float sq16(const u32x4& w, float*) {
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) s = __builtin_fmaf(__uint_as_float(w[i]), __uint_as_float(w[i]), s);
  return s;
}

// OCC: minimum waves per SIMD the register allocation must allow (launch bounds).
// FULLD: D == DPAD, so no fragment piece needs a column check.  The per-piece check costs
// 7 % at D=256 K=512 even when every piece passes it (profiles/r2_08_assign_clock_study.md).
// VARG (bf16): value-only argmin in the main loop -- 2 v_min3_u32 fold a tile's 4 scores
// into the running minimum and v_cmp + v_cndmask record the tile that lowered it (1.0 VALU
// per score instead of the packed keys' 1.5); the row inside the winning tile is recovered
// once per point after the loop by recomputing the winning tile's candidates on the
// matrix cores (bitwise the main loop's scores), right after the chunk loop.
// (A persistent grid that carried the next block's fragments across the epilogue measured
// 13-15 % slower -- the second register set spills at 4 waves/SIMD -- and was removed,
// profiles/r4_04_persistent_grid_ab.md.)
template <typename T, int DPAD, int P, int CT_ = 0, int NBUF_ = 2, int OCC = 1, int NW_ = 4, bool FULLD = false,
          bool VARG = false, int PMAJ = 0, bool TOP2 = false, bool XV = false>
__global__ __launch_bounds__(NW_ * 64, OCC) void assign16_kernel(AssignArgs a) {
  using C = Assign16Cfg<T, DPAD, P, CT_, NBUF_, NW_>;
  constexpr bool F32 = sizeof(T) == 4;
  // exact (value, index) epilogue: f32, or bf16 scores where the full pass ranks by value (XV)
  constexpr bool EXACT = F32 || XV;
  // A fragments streamed one at a time (see the MFMA issue): rows of 384..1024 features
  constexpr bool WIDE = DPAD > 256;
  static_assert(!(VARG && F32), "value-only argmin is the bf16 epilogue");
  static_assert(!(TOP2 && VARG), "bounded E-step: keys / exact epilogues");
  static_assert(!XV || (TOP2 && !F32), "the bf16 exact epilogue stands in for VARG in the bounded E-step");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 15, g = lane >> 4;
  const int cn_bytes = ((a.Kpad * 4 + 1023) / 1024) * 1024;
  char* cn_lds = smem;
  char* bufs = smem + cn_bytes;
  // Centre split (small N): grid.y splits the chunk range; each split leaves its
  // (value, index) in a.split_keys and split_finish_kernel writes the labels.
  const int nch_all = a.Kpad / (16 * C::CT);
  const int cps = (nch_all + (int)gridDim.y - 1) / (int)gridDim.y;
  const int c0 = (int)blockIdx.y * cps;
  const int nch = c0 + cps < nch_all ? c0 + cps : nch_all;  // one past this split's last chunk
  const int ncl = nch - c0;                                    // chunks of this split
  // LDS-DMA through buffer descriptors: the per-lane part is one 32-bit voffset (lane*16)
  // and every chunk / piece offset is a scalar, so no 64-bit VGPR address stays live
  // across the main loop (the f32 and D=128 bf16 bodies are register-bound).
  const uint32_t loff = (uint32_t)lane * 16u;
  const __amdgpu_buffer_rsrc_t rC = make_rsrc(a.Cpack, (uint32_t)a.Kpad * DPAD * sizeof(T));
  const __amdgpu_buffer_rsrc_t rN = make_rsrc(a.cn, (uint32_t)a.Kpad * 4u);
  // Ring slots: chunk c sits in slot c % NBUF.
  auto issue_chunk = [&](int c, int slot) {  // c: chunk index within this split
    const uint32_t src = (uint32_t)(c0 + c) * C::CHUNK_BYTES;
    char* dst = bufs + slot * C::CHUNK_BYTES;
#pragma unroll
    for (int i = 0; i < C::NPW; ++i) {
      const int pc = wid + i * C::NW;
      blds16(rC, (MK_LDS void*)(dst + pc * 1024), loff, src + (uint32_t)pc * 1024u);
    }
  };

  // rows this launch assigns: N, or the device count of a compacted batch (wave-uniform;
  // a workgroup past it leaves before any barrier)
  const int64_t N = a.n_dev ? min(a.N, *a.n_dev) : a.N;
  if (a.n_dev && (int64_t)blockIdx.x * C::PTS >= N) return;
  const unsigned long long t_entry = a.timeline ? __builtin_amdgcn_s_memrealtime() : 0ull;
  const int64_t pbase = (int64_t)blockIdx.x * C::PTS + (int64_t)wid * (C::P * 16);
  u32x4 xr[C::P][C::NQ];
  float xnr[C::P];
  float osr[C::P];   // (a.oseed) the rows' full-pass seed offsets, at their X rows
  // The P blocks' fragment loads go out back to back: one memory round trip (two for a
  // gathered batch: the row indices first).  vmcnt retires in order, so a block whose
  // address waited on a load issued after the previous block's fragments (the row index,
  // or a row norm under a data-dependent branch) serialised the P round trips.
  auto row_of = [&](int p) -> int64_t {
    const int64_t row = pbase + p * 16 + r;
    return row < N ? row : (N - 1);
  };
  auto load_frags = [&](int p, int64_t src) {
    const T* rp = (const T*)a.X + src * a.ldx + g * C::V;
#pragma unroll
    for (int q = 0; q < C::NQ; ++q) {
      const int col = (4 * q + g) * C::V;
      if (FULLD || col < a.D) xr[p][q] = *(const u32x4*)(rp + 4 * q * C::V);
      else xr[p][q] = u32x4{0u, 0u, 0u, 0u};
    }
  };
  auto load_block = [&]() {   // fragments (+ caller norms) of the block at pbase
    if (a.rows) {   // gathered batch: logical row -> X row
      int64_t src[C::P];
#pragma unroll
      for (int p = 0; p < C::P; ++p) src[p] = a.rows[row_of(p)];
      __builtin_amdgcn_sched_barrier(0);   // all index loads in flight before the first use
#pragma unroll
      for (int p = 0; p < C::P; ++p) load_frags(p, src[p]);
      if (!F32 && a.xn && a.scatter) {   // (scattering: the caller's norms sit at the X rows)
#pragma unroll
        for (int p = 0; p < C::P; ++p) xnr[p] = a.xn[src[p]];
      }
      if (!F32 && a.oseed) {
#pragma unroll
        for (int p = 0; p < C::P; ++p) osr[p] = a.oseed[src[p]];
      }
    } else {
#pragma unroll
      for (int p = 0; p < C::P; ++p) load_frags(p, row_of(p));
      if (!F32 && a.oseed) {
#pragma unroll
        for (int p = 0; p < C::P; ++p) osr[p] = a.oseed[row_of(p)];
      }
    }
    if (!F32 && a.xn) {
      if (!(a.rows && a.scatter)) {
#pragma unroll
        for (int p = 0; p < C::P; ++p) xnr[p] = a.xn[row_of(p)];
      }
    } else {
#pragma unroll
      for (int p = 0; p < C::P; ++p) xnr[p] = 0.f;
    }
  };
  // Early prologue (one pass over plain full bf16 rows with caller norms): the |c|^2 DMA and
  // the norms go out first, then the fragments, the epilogue's reads and the first chunk, and
  // the seed-offset reduction waits for the norms alone -- its barrier runs while the fragments
  // are still in flight (the chunk loop's first wait retires them).  A/B switch V_ASSIGN_EARLY.
  constexpr int EJ = (C::P + 3) / 4;
  constexpr bool EARLY_OK = !F32 && FULLD && C::P * C::NQ + EJ + C::NPW < 64;   // (vmcnt range)
  const bool early = EARLY_OK && a.xn && !a.rows && !a.oseed && !a.split_keys && a.epi_prefetch &&
                     a.early_prologue;
  // early: lane (r, g) loads the norm of its epilogue rows only -- block p = 4j + g -- one
  // instruction per 4 blocks instead of one per block (the prologue's vector-memory issue is
  // what takes its time, profiles/r5_45_assign_prologue_study.md); lanes past the last block
  // repeat it (harmless to the max / min)
  float xg[EJ];
  if (early) {
    for (int pc = wid; pc < cn_bytes / 1024; pc += C::NW)
      blds16(rN, (MK_LDS void*)(cn_lds + pc * 1024), loff, (uint32_t)pc * 1024u);
#pragma unroll
    for (int j = 0; j < EJ; ++j) xg[j] = a.xn[row_of(4 * j + g < C::P ? 4 * j + g : C::P - 1)];
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int p = 0; p < C::P; ++p) load_frags(p, row_of(p));
    __builtin_amdgcn_sched_barrier(0);
  } else {
    load_block();
  }
  // (timeline) every row load issued: issue time vs landing time separates a full request
  // queue from memory latency
  const unsigned long long t_issued = a.timeline ? __builtin_amdgcn_s_memrealtime() : 0ull;
  // (one pass) the epilogue's per-row inputs, fetched with the fragments so their memory round
  // trip hides under the prologue's instead of opening the epilogue (~2 us of a workgroup's
  // ~50 us at D=128, scripts/assign_timeline.py): lane (r, g) stores the rows of the blocks
  // p = 4j + g, so it keeps their old label and caller norm -- two registers per 4 blocks
  int eold[EJ];
  float exn[EJ];
  const bool eread = !a.split_keys && a.epi_prefetch;
  if (eread) {
#pragma unroll
    for (int j = 0; j < EJ; ++j) {
      const int pg = 4 * j + g;
      const int64_t i = pbase + pg * 16 + r;
      const bool mine = pg < C::P && i < N;
      const int64_t oi = mine && a.scatter ? a.rows[i] : i;
      if (early) {   // (one load per j whatever the lane: the prologue's wait counts them)
        const int v = a.labels[i < N ? i : N - 1];
        eold[j] = mine && a.track_changed ? v : -2;
      } else {
        eold[j] = mine && a.track_changed ? a.labels[oi] : -2;
      }
      if (F32 || !a.xn) {
        exn[j] = mine && a.xn ? a.xn[oi] : 0.f;
      } else if (early) {   // (loaded per lane group above)
        exn[j] = xg[j];
      } else {   // (bf16: the prologue loaded them, xnr[p] = xn at block p's rows)
        float v = 0.f;
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (4 * j + q < C::P && q == g) v = xnr[4 * j + q];
        exn[j] = v;
      }
    }
  }
  // per-wave (inertia, changed) totals, in LDS after the offsets
  double* wacc = (double*)(bufs + C::NBUF * C::CHUNK_BYTES + 16 * C::NW + C::OPT_BYTES);
  {
    // |c|^2 and the first centre chunk by LDS-DMA, issued after the fragments so no wait for a
    // fragment address (the gathered row indices) also waits for them.
    __builtin_amdgcn_sched_barrier(0);
    if (!early)
      for (int p = wid; p < cn_bytes / 1024; p += C::NW)
        blds16(rN, (MK_LDS void*)(cn_lds + p * 1024), loff, (uint32_t)p * 1024u);
    issue_chunk(0, 0);
    unsigned long long t_frag = 0ull;
    if (early) {
      // the norms and |c|^2 landed; younger: the fragments, one label load per 4 blocks and
      // the first chunk (all issued unconditionally)
      if constexpr (EARLY_OK) wait_vmcnt<C::P * C::NQ + EJ + C::NPW>();
    } else {
      if (a.timeline) {   // (diagnostic: the fragments alone, the younger DMAs (<= 5 at Kpad <= 1024) may fly)
        wait_vmcnt<5>();
        t_frag = __builtin_amdgcn_s_memrealtime();
      }
      wait_vmcnt<0>();  // retire the fragments before the LDS-DMA loop (its vmcnt waits count chunks)
    }
    const unsigned long long t_landed = a.timeline ? __builtin_amdgcn_s_memrealtime() : 0ull;
    if (C::NBUF == 3 && ncl > 1) issue_chunk(1, 1);

    // bf16 seed offset (see the header): o = (1 + 2^-12) max |x|^2 over the workgroup's
    // points, from the caller's row norms when given (loaded with the fragments) or from
    // the fragments themselves, folded into this workgroup's LDS copy of |c|^2 once.
    // A workgroup whose max |x|^2 exceeds 4x its min (an outlier row, or data around the
    // origin) takes per-point offsets o_p = (1 + 2^-12) |x_p|^2 instead, parked in LDS and
    // added to each tile's seed (second chunk-loop instantiation): a shared offset would coarsen every
    // neighbour's keys to 2^-17 of the outlier's norm.  Either way a key resolves
    // 2^-17 (|x - c|^2 + 3 |x|^2) or better.
    float off = 0.f;
    bool ppo = false;
    float* opt = (float*)(bufs + C::NBUF * C::CHUNK_BYTES + 16 * C::NW);  // [NW][16][PP] offsets
    float* xnl = opt + C::NW * 16 * C::PP;                                 // [NW][16][PP] |x|^2
    if (!a.xn && (!F32 || a.slots)) {
#pragma unroll
      for (int p = 0; p < C::P; ++p) {
        float s = 0.f;
#pragma unroll
        for (int q = 0; q < C::NQ; ++q) s += sq16(xr[p][q], (T*)nullptr);
        s += __shfl_xor(s, 16, 64);
        s += __shfl_xor(s, 32, 64);
        xnr[p] = s;
      }
      if (a.slots && g == 0) {   // no caller norms: the epilogue's inertia reads them back
#pragma unroll
        for (int p = 0; p < C::P; ++p) xnl[(wid * 16 + r) * C::PP + p] = xnr[p];
      }
    }
    if constexpr (!F32) {
     if (a.oseed) {
      // the offsets the full pass gives these rows (launch_seed_offsets), per point: the scores
      // -- and so the labels and near-tie decisions -- are bitwise the full pass's, whichever
      // workgroup a gathered row lands in (the bounded E-step's exactness)
      ppo = true;
      if (g == 0) {
#pragma unroll
        for (int p = 0; p < C::P; ++p) opt[(wid * 16 + r) * C::PP + p] = osr[p];
      }
     } else {
      float m = 0.f, mn = 3.0e38f;
      if (early) {   // (one norm per lane and 4 blocks: reduce over the whole wave)
#pragma unroll
        for (int j = 0; j < EJ; ++j) { m = fmaxf(m, xg[j]); mn = fminf(mn, xg[j]); }
        m = fmaxf(m, __shfl_xor(m, 16, 64));
        mn = fminf(mn, __shfl_xor(mn, 16, 64));
        m = fmaxf(m, __shfl_xor(m, 32, 64));
        mn = fminf(mn, __shfl_xor(mn, 32, 64));
      } else {
#pragma unroll
        for (int p = 0; p < C::P; ++p) { m = fmaxf(m, xnr[p]); mn = fminf(mn, xnr[p]); }
      }
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        m = fmaxf(m, __shfl_xor(m, o, 64));
        mn = fminf(mn, __shfl_xor(mn, o, 64));
      }
      float* red = (float*)(bufs + C::NBUF * C::CHUNK_BYTES);
      if (lane == 0) { red[2 * wid] = m; red[2 * wid + 1] = mn; }
      // every wave's |c|^2 DMA has landed (its wait above); a raw barrier, so an early
      // prologue's fragments and first chunk stay in flight (__syncthreads drains vmcnt)
      wait_lgkm0();
      raw_barrier();
      float mnw = 3.0e38f;
#pragma unroll
      for (int w = 0; w < C::NW; ++w) { off = fmaxf(off, red[2 * w]); mnw = fminf(mnw, red[2 * w + 1]); }
      ppo = __builtin_amdgcn_readfirstlane((int)(off > 4.f * mnw)) != 0;
      if (!ppo) {
        off = __builtin_fmaf(off, 2.44140625e-04f, off);  // * (1 + 2^-12)
        off = __uint_as_float(__builtin_amdgcn_readfirstlane(__float_as_uint(off)));
        for (int k = threadIdx.x; k < a.Kpad; k += C::NW * 64) ((float*)cn_lds)[k] += off;
      } else {
        off = 0.f;
        if (early) {
#pragma unroll
          for (int j = 0; j < EJ; ++j)
            if (4 * j + g < C::P) opt[(wid * 16 + r) * C::PP + 4 * j + g] = __builtin_fmaf(xg[j], 2.44140625e-04f, xg[j]);
        } else if (g == 0) {
#pragma unroll
          for (int p = 0; p < C::P; ++p) opt[(wid * 16 + r) * C::PP + p] = __builtin_fmaf(xnr[p], 2.44140625e-04f, xnr[p]);
        }
      }
     }
      // (published by the main loop's first wait_lgkm0 + barrier)
    }

    float best[C::P], seg_best[C::P];
    int bg[C::P];
    uint32_t vb[C::P], tb[C::P];   // VARG: running minimum (bits of a positive float), its tile
    // TOP2 (bounded E-step): this lane's second-smallest score (keys: index bits included,
    // <= 2^-17 relative -- the bounds' slack covers it), merged over lanes later; the smallest
    // is the epilogue's own running minimum (min(best, seg_best)).  Keys: the segment's own
    // second-smallest m2s rides along seg_best (one v_med3 + one v_min per key, no per-tile
    // merge with the global pair) and joins m2 at the segment's end -- 12 VALU per tile and
    // block instead of 16 (the gathered bounded assign is VALU-bound).
    float m2[C::P], m2s[C::P];
#pragma unroll
    for (int p = 0; p < C::P; ++p) {
      best[p] = 3.0e38f; seg_best[p] = 3.0e38f; bg[p] = 0;
      vb[p] = 0x7f7fffffu; tb[p] = 0u;
      m2[p] = 3.0e38f; m2s[p] = 3.0e38f;
    }
    const int ngrp = nch * C::CT;   // one past the last tile (global tile numbering)
    const unsigned kmask = key6_mask();

    // The chunk loop, instantiated twice: per-point offsets (PPO, outlier workgroups) seed a
    // tile's accumulators with its points' offsets; the common instantiation has no such
    // code at all -- a per-tile branch cost 1-3 % (one-process A/B against round 2).
    auto chunk_loop = [&](auto ppo_tag) {
      constexpr bool PPO = decltype(ppo_tag)::value;
      for (int c = 0; c < ncl; ++c) {
        // chunk c landed; with 3 slots chunk c+1 may stay in flight across the barrier
        if (C::NBUF == 3 && c + 1 < ncl) wait_vmcnt<C::NPW>(); else wait_vmcnt<0>();
        wait_lgkm0();
        raw_barrier();  // RAW for chunk c, WAR for the slot refilled next (read at c-1)
        // (the next chunk's pieces all go out right after the barrier: spreading them one group
        // per tile after that tile's epilogue measured -2.5 % at D=128, -5 % at D=256 and far
        // slower at D=64, profiles/r3_28_ab_spread_dma.log)
        if (c + C::NBUF - 1 < ncl) issue_chunk(c + C::NBUF - 1, (c + C::NBUF - 1) % C::NBUF);
        const char* buf = bufs + (c % C::NBUF) * C::CHUNK_BYTES;
        // A fragments + |c|^2 of a tile from the LDS ring
        auto load_a = [&](int tl_i, u32x4* aw_, f32x4& ci_) {
          const int tile = (c0 + c) * C::CT + tl_i;
          ci_ = *(const f32x4*)(cn_lds + (tile * 16 + 4 * g) * 4);
          const char* tl = buf + tl_i * C::TILE_BYTES + lane * 16;
          if constexpr (!WIDE) {   // (wide rows read their A fragments one at a time, below)
    #pragma unroll
            for (int q = 0; q < C::NQ; ++q) aw_[q] = *(const u32x4*)(tl + q * 1024);
          }
        };
        // EARLY (bf16 D=64): the next tile's fragments are read right after this tile's
        // MFMAs are issued, so their LDS latency hides under the argmin epilogue (+2 % at D=64
        // in one-process A/B, profiles/r2_08_assign_clock_study.md; no gain at D=128)
        constexpr bool EARLY = !F32 && DPAD == 64;
        u32x4 awe[C::NQ];
        f32x4 cie;
        if constexpr (EARLY) load_a(0, awe, cie);
    #pragma unroll
        for (int tl_i = 0; tl_i < C::CT; ++tl_i) {
          const int tile = (c0 + c) * C::CT + tl_i;
          u32x4 aw[C::NQ];
          f32x4 ci;
          if constexpr (EARLY) {
    #pragma unroll
            for (int q = 0; q < C::NQ; ++q) aw[q] = awe[q];
            ci = cie;
          } else {
            load_a(tl_i, aw, ci);
          }
          f32x4 acc[C::P];
    #pragma unroll
          for (int p = 0; p < C::P; ++p) acc[p] = ci;
          if constexpr (PPO) {  // per-point offsets seed the accumulators (one LDS read per tile)
            // (added BEFORE the MFMAs: VALU writes the MFMA then reads as src C.  Adding them
            // to the MFMA results instead raced the matrix pipe: a v_pk_add_f32 read the
            // result registers early when the LDS read ahead of it returned fast, a rare,
            // nondeterministic wrong label, tests/test_gpu_kernels.py split-batch test)
            const float* o = opt + (wid * 16 + r) * C::PP;
    #pragma unroll
            for (int p4 = 0; p4 < C::P; p4 += 4) {
              const f32x4 ov = *(const f32x4*)(o + p4);
    #pragma unroll
              for (int j = 0; j < 4; ++j)
                if (p4 + j < C::P) seed_add(acc[p4 + j], ov[j]);
            }
          }
          // bf16: the wave issues its MFMAs at raised priority and drops back for the epilogue,
          // so a SIMD's arbiter feeds the matrix core before another wave's argmin VALU work
          // (profiles/r2_29_assign_setprio_ab.log, one process each: the harness copy -2.2 % at
          // D=128 K=1024 and -1.4 % at D=64 K=4096; this kernel against that copy +0.8 % at D=128,
          // +0.3 % at D=64, about +5 % at D=256 K=512)
          if constexpr (!F32) {
            __builtin_amdgcn_sched_barrier(0);
            __builtin_amdgcn_s_setprio(1);
            __builtin_amdgcn_sched_barrier(0);
          }
          // per-block argmin epilogue (bf16): packed 6-bit keys or the value-only running minimum
          unsigned t0 = 0, t1 = 0, t2 = 0, t3 = 0;
          if constexpr (!EXACT && !VARG) {
            // 6-bit keys over a segment of 16 tiles (tile-in-segment * 4 + reg): 4 key packs
            // + 2 v_min3 per tile and point block; the running best is merged with its
            // segment id once per segment.  The four indices as opaque SGPRs, so each key is
            // one v_and_or_b32.
            const unsigned tis = (unsigned)(tile & 15) << 2;
            asm volatile("s_mov_b32 %0, %4\n\ts_or_b32 %1, %4, 1\n\ts_or_b32 %2, %4, 2\n\ts_or_b32 %3, %4, 3"
                         : "=s"(t0), "=s"(t1), "=s"(t2), "=s"(t3) : "s"(tis) : "scc");  // s_or_b32 writes SCC
          }
          auto epi = [&](int p) {
            if constexpr (VARG) {
              // scores are positive (seed offset, see the header), so they order as their bits;
              // a tie with the running minimum keeps the earlier tile (the lower index)
              const uint32_t u0 = __float_as_uint(acc[p][0]), u1 = __float_as_uint(acc[p][1]);
              const uint32_t u2 = __float_as_uint(acc[p][2]), u3 = __float_as_uint(acc[p][3]);
              const uint32_t nb = min(min(u0, u1), min(u2, min(u3, vb[p])));
              tb[p] = nb != vb[p] ? (uint32_t)tile : tb[p];
              vb[p] = nb;
            } else {
              const f32x4& sv = acc[p];
              const float k0 = pack_key6(sv[0], kmask, t0), k1 = pack_key6(sv[1], kmask, t1);
              const float k2 = pack_key6(sv[2], kmask, t2), k3 = pack_key6(sv[3], kmask, t3);
              if constexpr (TOP2) {
                // the segment's sorted pair (seg_best, m2s): med3 of (smallest, second, new) is
                // the new second
                // (asm forms: no per-key canonicalisation, see common.h med3f)
                m2s[p] = med3f(seg_best[p], m2s[p], k0);
                seg_best[p] = min2f(seg_best[p], k0);
                m2s[p] = med3f(seg_best[p], m2s[p], k1);
                seg_best[p] = min2f(seg_best[p], k1);
                m2s[p] = med3f(seg_best[p], m2s[p], k2);
                seg_best[p] = min2f(seg_best[p], k2);
                m2s[p] = med3f(seg_best[p], m2s[p], k3);
                seg_best[p] = min2f(seg_best[p], k3);
              } else {
                seg_best[p] = min3f(min3f(k0, k1, k2), k3, seg_best[p]);
              }
            }
          };
          auto chain = [&](int p) {   // block p's NQ MFMAs back to back (srcC = the previous vDst)
    #pragma unroll
            for (int q = 0; q < C::NQ; ++q) {
              acc[p] = Mfma16<T>::run(aw[q], xr[p][q], acc[p]);
              __builtin_amdgcn_sched_barrier(0);
            }
          };
          if constexpr (WIDE) {
            // wide rows (DPAD > 256): one A fragment at a time, each against the P blocks --
            // all NQ of a tile would not fit in registers beside the rows.  The reads run WPF
            // fragments ahead of the MFMAs that use them, pinned in that order: left to the
            // scheduler, each read sat right before its P MFMAs behind an lgkmcnt(0), so one
            // wave per SIMD waited out every LDS round trip (bf16 D=512: 870 TF/s against
            // 1410 at D=256, profiles/r6_43_assign_sweep.log)
            const char* tl = buf + tl_i * C::TILE_BYTES + lane * 16;
            // (2 ahead where the rows leave room for 2 waves per SIMD under 256 VGPRs: bf16 D=384
            // at 4 ahead took 265 and ran 15 % slower at one wave, r6_44_ab_wide_d384_bf16.log;
            // 1 ahead for its bounded E-step, whose second-best keys spilled at 2)
            constexpr int WPF = C::NQ < 4 ? C::NQ : (C::P * C::NQ * 4 <= 192 ? (TOP2 && C::P == 4 ? 1 : 2) : 4);
            u32x4 aq[C::NQ];
#pragma unroll
            for (int q = 0; q < WPF; ++q) aq[q] = *(const u32x4*)(tl + q * 1024);
#pragma unroll
            for (int q = 0; q < C::NQ; ++q) {
              if (q + WPF < C::NQ) aq[q + WPF] = *(const u32x4*)(tl + (q + WPF) * 1024);
              __builtin_amdgcn_sched_barrier(0);
#pragma unroll
              for (int p = 0; p < C::P; ++p) acc[p] = Mfma16<T>::run(aq[q], xr[p][q], acc[p]);
              __builtin_amdgcn_sched_barrier(0);
            }
          } else if constexpr (PMAJ) {
            // point-block-major issue, pinned in this order
#pragma unroll
            for (int p = 0; p < C::P; ++p) chain(p);
          } else {
#pragma unroll
            for (int q = 0; q < C::NQ; ++q) {
#pragma unroll
              for (int p = 0; p < C::P; ++p) acc[p] = Mfma16<T>::run(aw[q], xr[p][q], acc[p]);
            }
          }
          if constexpr (!F32) {
            __builtin_amdgcn_sched_barrier(0);
            __builtin_amdgcn_s_setprio(0);
            __builtin_amdgcn_sched_barrier(0);
          }
          if constexpr (EARLY) {
            if (tl_i + 1 < C::CT) load_a(tl_i + 1, awe, cie);
            __builtin_amdgcn_sched_barrier(0);
          }
          if constexpr (EXACT) {
            // (tile*4 + reg) as wave-uniform values: the index select needs no VALU add
            const int u = tile * 4;
#pragma unroll
            for (int p = 0; p < C::P; ++p) {
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                if constexpr (TOP2) m2[p] = __builtin_amdgcn_fmed3f(best[p], m2[p], acc[p][e]);
                const bool lt = acc[p][e] < best[p];
                best[p] = lt ? acc[p][e] : best[p];
                bg[p] = lt ? u + e : bg[p];
              }
            }
          } else {
#pragma unroll
            for (int p = 0; p < C::P; ++p) epi(p);
          }
          if constexpr (!EXACT && !VARG) {
            if ((tile & 15) == 15 || tile == ngrp - 1) {
    #pragma unroll
              for (int p = 0; p < C::P; ++p) {
                if constexpr (TOP2) {   // the two sorted pairs -> the overall second-smallest key
                  m2[p] = min3f(m2[p], m2s[p], max2f(best[p], seg_best[p]));
                  m2s[p] = 3.0e38f;
                }
                // compare values only: on equal (truncated) values the earlier segment keeps
                // the lower centroid index (all keys are >= 0, see the header)
                const float sv = __uint_as_float(__float_as_uint(seg_best[p]) & ~63u);
                const float bv = __uint_as_float(__float_as_uint(best[p]) & ~63u);
                if (sv < bv) { best[p] = seg_best[p]; bg[p] = tile >> 4; }
                seg_best[p] = 3.0e38f;
              }
            }
          }
        }
      }
    };
    const unsigned long long t_loop = a.timeline ? __builtin_amdgcn_s_memrealtime() : 0ull;
    if (ppo) chunk_loop(std::true_type{});
    else chunk_loop(std::false_type{});
    if (a.timeline && threadIdx.x == 0 && blockIdx.y == 0) {
      unsigned long long* tl = a.timeline + (int64_t)blockIdx.x * 8;
      tl[0] = t_entry;
      tl[1] = t_loop;
      tl[2] = __builtin_amdgcn_s_memrealtime();
      tl[4] = (unsigned long long)__builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));    // HW_ID
      tl[5] = (unsigned long long)__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11));   // XCC_ID
      tl[6] = t_landed;   // fragments, |c|^2 and the first chunk landed (wave 0)
      tl[7] = early ? t_issued : t_frag;   // early prologue: the loads' issue completed; else
                                           // (Kpad <= 1024, 4 chunk pieces per wave) the fragments landed
    }

    // VARG: merge the 4 lane groups of each point on (value, tile, group) -- the centre index
    // 16 t + 4 g + e orders like that triple -- then recover e: for the points 4m..4m+3 the
    // 16 A rows carry the 4 candidates of each (row 4g'+e = candidate e of point 4m+g'), so
    // lane (r = 4m+g, g) receives its own point's 4 candidate scores, computed exactly as in
    // the main loop (same packed -2c, same seed from the LDS |c|^2 copy, same k-step order),
    // and takes the first that equals the minimum.  4 MFMA groups per point block: 64/K of
    // the main loop's matrix work.
    uint32_t kv[C::P];
    if constexpr (VARG) {
#pragma unroll
      for (int p = 0; p < C::P; ++p) {
        uint32_t v = vb[p], tg = tb[p] * 4u + (uint32_t)g;
#pragma unroll
        for (int o = 16; o <= 32; o <<= 1) {
          const uint32_t vo = (uint32_t)__shfl_xor((int)v, o, 64), to = (uint32_t)__shfl_xor((int)tg, o, 64);
          if (vo < v || (vo == v && to < tg)) { v = vo; tg = to; }
        }
        vb[p] = v;
        tb[p] = tg;
      }
      const T* pack = (const T*)a.Cpack;
      int efound[C::P];
#pragma unroll
      for (int p = 0; p < C::P; ++p) efound[p] = 0;
#pragma unroll
      for (int p = 0; p < C::P; ++p) {
        // MG candidate groups in flight at once (registers: MG * NQ fragments)
        constexpr int MG = C::NQ <= 2 ? 4 : 1;
#pragma unroll
        for (int m0 = 0; m0 < 4; m0 += MG) {
          u32x4 aw[MG][C::NQ];
          f32x4 acc[MG];
#pragma unroll
          for (int mi = 0; mi < MG; ++mi) {
            const int m = m0 + mi;
            const uint32_t tga = (uint32_t)__shfl((int)tb[p], 4 * m + (r >> 2), 64);
            const int ca = (int)(tga >> 2) * 16 + (int)(tga & 3u) * 4 + (r & 3);   // A row r's centre
            const T* src = pack + ((int64_t)(ca >> 4) * C::NQ * 64 + (ca & 15) + 16 * g) * C::V;
#pragma unroll
            for (int q = 0; q < C::NQ; ++q) aw[mi][q] = *(const u32x4*)(src + (int64_t)q * 64 * C::V);
            const uint32_t tgs = (uint32_t)__shfl((int)tb[p], 4 * m + g, 64);     // output rows' point
            acc[mi] = *(const f32x4*)(cn_lds + ((int)(tgs >> 2) * 16 + (int)(tgs & 3u) * 4) * 4);
            if (ppo) {
              seed_add(acc[mi], opt[(wid * 16 + r) * C::PP + p]);
            }
          }
#pragma unroll
          for (int mi = 0; mi < MG; ++mi) {
#pragma unroll
            for (int q = 0; q < C::NQ; ++q) acc[mi] = Mfma16<T>::run(aw[mi][q], xr[p][q], acc[mi]);
          }
#pragma unroll
          for (int mi = 0; mi < MG; ++mi) {
            if (r == 4 * (m0 + mi) + g) {
              int e = 3;
#pragma unroll
              for (int j = 2; j >= 0; --j) e = __float_as_uint(acc[mi][j]) == vb[p] ? j : e;
              efound[p] = e;
            }
          }
        }
      }
#pragma unroll
      for (int p = 0; p < C::P; ++p) {
        const int e = __shfl(efound[p], r + 16 * (r & 3), 64);
        kv[p] = (tb[p] >> 2) * 16u + (tb[p] & 3u) * 4u + (uint32_t)e;
      }
    }

    // The block's label epilogue.  Per point: the winning (score, centre) with the 4 lane
    // groups merged, then the label / distance stores and the inertia.
    auto merged = [&](int p, int& k, float& v) {
      if constexpr (VARG) {  // merged and recovered above
        k = (int)kv[p];
        v = __uint_as_float(vb[p]);
      } else {
        if constexpr (EXACT) {  // bg = tile * 4 + reg of the first strict minimum
          k = (bg[p] >> 2) * 16 + 4 * g + (bg[p] & 3);
          v = best[p];
        } else {               // bg = segment of 16 tiles, 6-bit key; undo the seed offset
          const unsigned bits = __float_as_uint(best[p]);
          const int idx = (int)(bits & 63u);
          k = (bg[p] * 16 + (idx >> 2)) * 16 + 4 * g + (idx & 3);
          v = __uint_as_float(bits & ~63u);
        }
#pragma unroll
        for (int o = 16; o <= 32; o <<= 1) {
          const float vo = __shfl_xor(v, o, 64);
          const int ko = __shfl_xor(k, o, 64);
          if (vo < v || (vo == v && ko < k)) { v = vo; k = ko; }
        }
      }
    };
    float inert = 0.f;
    int changed = 0;
    const int64_t pcur = pbase;
    // TOP2: the second-smallest score of the point, merged over its 4 lane groups like the
    // winner (two sorted pairs -> their two smallest); every lane takes part (shuffles)
    auto second = [&](int p) -> float {
      float a1 = EXACT ? best[p] : fminf(best[p], seg_best[p]), a2 = m2[p];
#pragma unroll
      for (int o = 16; o <= 32; o <<= 1) {
        const float b1 = __shfl_xor(a1, o, 64), b2 = __shfl_xor(a2, o, 64);
        const float n2 = fminf(fmaxf(a1, b1), fminf(a2, b2));
        a1 = fminf(a1, b1);
        a2 = n2;
      }
      return EXACT ? a2 : __uint_as_float(__float_as_uint(a2) & ~63u);
    };
    // ``oi``: where the row's outputs go (its row when a gathered batch scatters, else i);
    // ``old``: the row's previous label, ``xnv``: its caller norm (read by the caller of this
    // lambda, i < N, lanes with (p & 3) == g only); ``sec``: the second-smallest score (TOP2)
    auto store = [&](int p, int64_t oi, int k, float v, int old, float xnv, float sec) {
      const float offp = ppo ? opt[(wid * 16 + r) * C::PP + p] : off;   // the seed offset (0: f32)
      // inertia without caller norms: the prologue parked |x|^2 of the fragments in LDS
      const float xv = (a.slots && !a.xn) ? xnl[(wid * 16 + r) * C::PP + p] : xnv;
      if (a.split_keys) {
        // compare the (positive) keys across splits; split_finish undoes the offset
        // (parked in mind[], which the caller provides whenever xn is given)
        atomicMin(a.split_keys + oi, split_key(v, k));
        if (a.mind) a.mind[oi] = offp;
      } else {
        v -= offp;   // back to |c|^2 - 2 x.c
        if (a.track_changed) changed += (old != k);
        a.labels[oi] = k;
        if (a.xn || a.slots) {
          const float d = fmaxf(xv + v, 0.f);
          inert += d;
          if (a.mind) a.mind[oi] = d;
          if constexpr (TOP2) {   // Hamerly bounds: distances to the nearest and second nearest
            a.ub[oi] = __builtin_sqrtf(d);
            a.lb[oi] = __builtin_sqrtf(fmaxf(xv + (sec - offp), 0.f));
          }
        }
      }
    };
#pragma unroll
    for (int p = 0; p < C::P; ++p) {
      int k;
      float v;
      merged(p, k, v);
      float sec = 0.f;
      if constexpr (TOP2) sec = second(p);
      const int64_t i = pcur + p * 16 + r;
      if ((p & 3) == g && i < N) {
        const int64_t oi = a.scatter ? a.rows[i] : i;
        const bool rd = !a.split_keys;
        store(p, oi, k, v, eread ? eold[p >> 2] : (rd && a.track_changed ? a.labels[oi] : -2),
              eread ? exn[p >> 2] : (rd && a.xn ? a.xn[oi] : 0.f), sec);
      }
    }
    if (a.slots && !a.split_keys) {   // the wave's totals, in its LDS slot
      const double di = wave_sum((double)inert);
      const int dc = wave_sum(changed);
      if (lane == 0) {
        wacc[2 * wid] = di;
        wacc[2 * wid + 1] = (double)dc;
      }
    }
  }
  if (a.timeline && threadIdx.x == 0 && blockIdx.y == 0)
    a.timeline[(int64_t)blockIdx.x * 8 + 3] = __builtin_amdgcn_s_memrealtime();
  if (a.slots && !a.split_keys) {
    // the waves' LDS totals are published by a raw barrier: __syncthreads would first drain
    // vmcnt, i.e. wait for every label / distance store of the epilogue to be acknowledged
    wait_lgkm0();
    raw_barrier();
    if (threadIdx.x == 0) {
      double si = 0, sc = 0;
#pragma unroll
      for (int w = 0; w < C::NW; ++w) { si += wacc[2 * w]; sc += wacc[2 * w + 1]; }
      slot_add((unsigned long long*)(a.slots + (blockIdx.x % NSLOT) * SLOT_STRIDE), si, (long long)sc);
    }
  }
}

// Centre-split epilogue: labels, squared distances, inertia and changed count from the
// per-point minimum key the splits left; resets every key for the next call.
__global__ __launch_bounds__(256) void split_finish_kernel(AssignArgs a) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  float inert = 0.f;
  int changed = 0;
  if (i < a.N) {
    const unsigned long long key = a.split_keys[i];
    a.split_keys[i] = ~0ull;
    const int k = (int)(unsigned)key;
    const float v = split_value(key) - (a.mind ? a.mind[i] : 0.f);  // minus the parked seed offset
    if (a.track_changed) changed = a.labels[i] != k;
    a.labels[i] = k;
    if (a.xn) {
      const float d = fmaxf(a.xn[i] + v, 0.f);
      inert = d;
      if (a.mind) a.mind[i] = d;
    }
  }
  if (a.slots) {
    __shared__ double red[8];
    const double di = wave_sum((double)inert);
    const int dc = wave_sum(changed);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0) { red[2 * w] = di; red[2 * w + 1] = (double)dc; }
    __syncthreads();
    if (threadIdx.x == 0)
      slot_add((unsigned long long*)(a.slots + (blockIdx.x % NSLOT) * SLOT_STRIDE), red[0] + red[2] + red[4] + red[6],
               (long long)(red[1] + red[3] + red[5] + red[7]));
  }
}

// Splits of the centre range for N points: enough workgroups to fill the chip when the
// point blocks alone do not (a 1k-point batch is 4 workgroups streaming all of C).
static int assign16_splits(int64_t nblk, int nch) {
  if (nblk >= 1024 || nch <= 1) return 1;
  const int64_t want = (2048 + nblk - 1) / nblk;
  const int sp = (int)(want < nch ? want : nch);
  const int cps = (nch + sp - 1) / sp;
  return (nch + cps - 1) / cps;  // no empty split (the kernel's chunk range must be non-empty)
}

// Value-only argmin (VARG) where it pays: the D<=64 bf16 bodies are VALU-bound on the packed
// keys (2 MFMAs per tile and block at D=64, 1 at D=32, against 6 epilogue VALU), and the
// recovery pass costs 64/K of the matrix work, so it is taken for K >= 2048 at D=64 and
// K >= 1024 at D=32 (scripts/varg_ab.py, profiles/r3_08_varg_ab.log: cfg4 shape +8.2 %,
// D=64 K=2048 +8.5 %, K=1024 -3.7 %; D=32 K=1024 +5.6 %, K=512 -8.8 %).
// Variant V_ASSIGN_VARG = 0/1 forces it off / on (A/B, tests).

template <typename T, int DPAD, int P, int CT_, int NBUF_, int OCC, int NW_, bool VARG, int PMAJ, bool TOP2, bool XV>
static void set_lds_attr() {
  static bool done = false;
  if (done) return;
  (void)hipFuncSetAttribute((const void*)assign16_kernel<T, DPAD, P, CT_, NBUF_, OCC, NW_, false, VARG, PMAJ, TOP2, XV>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  (void)hipFuncSetAttribute((const void*)assign16_kernel<T, DPAD, P, CT_, NBUF_, OCC, NW_, true, VARG, PMAJ, TOP2, XV>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  done = true;
}

template <typename T, int DPAD, int P, int CT_, int NBUF_, int OCC, int NW_, bool VARG, int PMAJ, bool TOP2, bool XV>
static void launch16_kt(const AssignArgs& b, const dim3& grid, size_t lds, hipStream_t s) {
  set_lds_attr<T, DPAD, P, CT_, NBUF_, OCC, NW_, VARG, PMAJ, TOP2, XV>();
  if (b.D == DPAD)
    hipLaunchKernelGGL((assign16_kernel<T, DPAD, P, CT_, NBUF_, OCC, NW_, true, VARG, PMAJ, TOP2, XV>), grid,
                       dim3(NW_ * 64), lds, s, b);
  else
    hipLaunchKernelGGL((assign16_kernel<T, DPAD, P, CT_, NBUF_, OCC, NW_, false, VARG, PMAJ, TOP2, XV>), grid,
                       dim3(NW_ * 64), lds, s, b);
}

// The geometries that run the bounded E-step's TOP2 epilogue (launch16_d routes every call
// with bounds to them).  With a running (min, second) pair per point block the bf16
// defaults at D = 64 / 128 / 256 spilled 400-940 VGPRs and ran 5.7x slower
// (profiles/r4_05_hamerly_ab_top2_spills.log); the state is now the second minimum alone
// (profiles/r4_16_top2_register_study.md), and D = 256 keeps 3 blocks at 8 waves per ring.
template <typename T, int DPAD, int P, int OCC, int NW_>
constexpr bool top2_geom() {
  if (sizeof(T) == 4 || DPAD == 32 || DPAD > 256) return true;   // (the defaults hold it, 0 spills)
  if (DPAD == 64) return (P == 2 || P == 4) && OCC == 4 && NW_ == 4;
  if (DPAD == 128) return (P == 2 || P == 4) && OCC == 4 && NW_ == 4;
  if (DPAD == 256) return P == 3 && OCC == 2 && NW_ == 8;
  return false;
}

// With bounds (b.ub) the VARG flag says how the FULL pass of this shape ranks: by value (the
// value-only argmin) -> the TOP2 kernel takes the exact (value, index) epilogue (XV), else the
// packed keys; with the full pass's seed offsets (b.oseed) its labels are then the full pass's.
template <typename T, int DPAD, int P, int CT_, int NBUF_, int OCC, int NW_, bool VARG, int PMAJ>
static void launch16_kp(const AssignArgs& b, const dim3& grid, size_t lds, hipStream_t s) {
  if (b.ub) {
    if constexpr (top2_geom<T, DPAD, P, OCC, NW_>()) {
      if constexpr (VARG && sizeof(T) == 2)
        return launch16_kt<T, DPAD, P, CT_, NBUF_, OCC, NW_, false, PMAJ, true, true>(b, grid, lds, s);
      else
        return launch16_kt<T, DPAD, P, CT_, NBUF_, OCC, NW_, false, PMAJ, true, false>(b, grid, lds, s);
    }
    return;   // (unreachable: launch16_d sends bounds to a top2_geom geometry)
  }
  launch16_kt<T, DPAD, P, CT_, NBUF_, OCC, NW_, VARG, PMAJ, false, false>(b, grid, lds, s);
}

static unsigned long long* g_timeline = nullptr;
static int64_t g_timeline_cap = 0;
void set_assign_timeline(unsigned long long* buf, int64_t capacity) {
  g_timeline = buf;
  g_timeline_cap = buf ? capacity : 0;
}

template <typename T, int DPAD, int P, int CT_, int NBUF_, int OCC, int NW_, bool VARG>
static void launch16_k(const AssignArgs& b, const dim3& grid, size_t lds, hipStream_t s) {
  if constexpr (DPAD > 256) {   // streamed A fragments: one issue order
    return launch16_kp<T, DPAD, P, CT_, NBUF_, OCC, NW_, VARG, 0>(b, grid, lds, s);
  } else {
    const int e = variant(V_ASSIGN_PMAJ);
    const int pm = e >= 0 ? e : (sizeof(T) == 2 ? 1 : 0);
    if (pm != 0) return launch16_kp<T, DPAD, P, CT_, NBUF_, OCC, NW_, VARG, 1>(b, grid, lds, s);
    launch16_kp<T, DPAD, P, CT_, NBUF_, OCC, NW_, VARG, 0>(b, grid, lds, s);
  }
}

template <typename T, int DPAD, int P, int CT_ = 0, int NBUF_ = 2, int OCC = 1, int NW_ = 4>
static hipError_t launch16_t(const AssignArgs& a, hipStream_t s) {
  using C = Assign16Cfg<T, DPAD, P, CT_, NBUF_, NW_>;
  if (a.Kpad % (16 * C::CT) != 0) return hipErrorInvalidValue;
  const int cn_bytes = ((a.Kpad * 4 + 1023) / 1024) * 1024;
  // + min/max scratch + per-point offsets + per-wave slot totals
  const size_t lds = cn_bytes + C::NBUF * C::CHUNK_BYTES + 16 * C::NW + C::OPT_BYTES + 16 * C::NW;
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  const int64_t nblk = (a.N + C::PTS - 1) / C::PTS;
  if (nblk <= 0) return hipSuccess;
  // (bounded E-step: one-pass grid, keys or exact epilogue)
  const int splits = (a.split_keys && !a.ub && !a.n_dev) ? assign16_splits(nblk, a.Kpad / (16 * C::CT)) : 1;
  AssignArgs b = a;
  if ((a.ub != nullptr) != (a.lb != nullptr) || (a.scatter && !a.rows)) return hipErrorInvalidValue;
  if (splits == 1) b.split_keys = nullptr;
  const dim3 grid((unsigned)nblk, (unsigned)splits);
  if (g_timeline && nblk <= g_timeline_cap && splits == 1) b.timeline = g_timeline;
  b.epi_prefetch = variant(V_ASSIGN_EPI) != 0;
  b.early_prologue = variant(V_ASSIGN_EARLY) != 0;
  bool varg = false;
  constexpr bool VARG_OK = sizeof(T) == 2 && DPAD <= 64;   // D=128: -12 % at K=1024, -4 % at 2048 (r3_11)
  if constexpr (VARG_OK) {
    const int e = variant(V_ASSIGN_VARG);
    // (with bounds: whether the full pass would, see launch16_kp)
    varg = e >= 0 ? e != 0 : a.Kpad >= (DPAD == 64 ? 2048 : 1024);
  }
  if constexpr (VARG_OK) {
    if (varg) launch16_k<T, DPAD, P, CT_, NBUF_, OCC, NW_, true>(b, grid, lds, s);
    else launch16_k<T, DPAD, P, CT_, NBUF_, OCC, NW_, false>(b, grid, lds, s);
  } else {
    launch16_k<T, DPAD, P, CT_, NBUF_, OCC, NW_, false>(b, grid, lds, s);
  }
  if (splits > 1)
    hipLaunchKernelGGL(split_finish_kernel, dim3((unsigned)((a.N + 255) / 256)), dim3(256), 0, s, b);
  return hipGetLastError();
}

// Point blocks per wave of the default geometries (launch16_d / launch16_w, see there).
template <typename T, int DPAD>
constexpr int p_narrow() {
  return sizeof(T) == 2 ? (DPAD == 64 ? 8 : DPAD == 256 ? 3 : 4) : (DPAD / 4 / Elem<T>::V >= 8 ? 2 : 4);
}
template <typename T, int DPAD>
constexpr int p_wide() {
  return sizeof(T) == 2 ? (DPAD == 512 || DPAD == 1024 ? 3 : DPAD <= 512 ? 4 : 2) : (DPAD <= 512 ? 2 : 1);
}

// The workgroup's point count (NW*P*16) must divide parallel/shard.py ROW_ALIGN (1536).
template <typename T, int DPAD>
static hipError_t launch16_d(const AssignArgs& a, hipStream_t s) {
  constexpr int CT = chunk_tiles16(sizeof(T), DPAD);
  // 16 KiB chunks in a 2-slot ring.  A/B on MI355X (one process, interleaved rounds; round 1
  // profiles/r1_08_*, r1_16_*, r1_17_*, round 2 profiles/r2_04_assign_ab.md):
  //  * bf16 D=128: 4 point blocks per wave at <= 128 VGPRs (4 waves/SIMD) -- 3 / 5 / 6 / 8 blocks,
  //    2-3 waves/SIMD, 8/16 waves per ring, 4/8 KiB chunks x 3 slots and next-tile fragment
  //    loads under the MFMAs are all slower;
  //  * bf16 D=64: 8 point blocks at 3 waves/SIMD, -5 % against 4 blocks at 4; with the
  //    value-only argmin (K >= 2048) 4 blocks at 4 waves are 4-9 % slower and 12 blocks at
  //    2 waves 1-10 % slower (profiles/r3_10_assign_p64_ab.log);
  //  * bf16 D=256: 3 point blocks at 3 waves/SIMD, -4 % against 2 at 4; streamed A fragments
  //    (3, 4 or 6 blocks) and a 3-slot ring were slower too (r4_04, r5_67), and were removed;
  //  * f32: the register file sets 4 (D <= 64) or 2 blocks at one wave per SIMD minimum.
  constexpr int P = p_narrow<T, DPAD>();
  constexpr int OCC = sizeof(T) == 2 ? ((DPAD == 64 || DPAD == 256) ? 3 : 4) : 1;
  static_assert(1536 % (4 * P * 16) == 0, "workgroup points must tile the shard grid");
  if (a.ub) {   // bounded E-step (TOP2): the geometries of top2_geom
    // 4 point blocks per wave at D = 64 / 128 (the single-register TOP2 state: 0 / 14 spilled
    // VGPRs, the latter outside the MFMA loop); a 40-iteration bounded fit at N=2e7 D=128
    // K=1024 ran 6 % faster than with 2 blocks (profiles/r4_17_top2_geom_ab.md).  A/B switch
    // V_ASSIGN_TOP2_GEOM: 0 = 2 blocks
    const bool p4 = variant(V_ASSIGN_TOP2_GEOM) != 0;
    if constexpr (sizeof(T) == 2 && DPAD == 64) {
      if (p4) return launch16_t<T, DPAD, 4, CT, 2, 4>(a, s);
      return launch16_t<T, DPAD, 2, CT, 2, 4>(a, s);
    }
    if constexpr (sizeof(T) == 2 && DPAD == 128) {
      if (p4) return launch16_t<T, DPAD, 4, CT, 2, 4>(a, s);
      return launch16_t<T, DPAD, 2, CT, 2, 4>(a, s);
    }
    if constexpr (sizeof(T) == 2 && DPAD == 256) return launch16_t<T, DPAD, 3, CT, 2, 2, 8>(a, s);
  }
  if constexpr (sizeof(T) == 2 && DPAD == 256) {
    // A/B switch V_ASSIGN_GEOM = 1: 8 waves per ring (half the per-point centre stream and
    // per-workgroup start-up), 3 point blocks at 2 waves/SIMD -- the bounded E-step's geometry
    if (variant(V_ASSIGN_GEOM) == 1) return launch16_t<T, DPAD, 3, CT, 2, 2, 8>(a, s);
  }
  if constexpr (sizeof(T) == 2 && DPAD == 128) {
    // A/B switch V_ASSIGN_GEOM: 1 = 8 waves share a ring of 32 KiB chunks (a barrier
    // every 8 tiles instead of 4), 2 = 8 waves share the 16 KiB ring.  K=1024: -0.4 % / +0.1 %;
    // K=2048: +4.9 % / +4.4 % (profiles/r3_21_ab_geom128.log), near-tie labels move with
    // the workgroup's seed offset; the headline's K=1024 keeps 4 waves.
    // A K sweep keeps 4 waves as the default: 8-wave rings measured +5.0 % at K=2048 but
    // -5.3 % at 3072 and -5.5 % at 4096 (profiles/r3_33_ab_geom128_ksweep.log).
    const int gm = variant(V_ASSIGN_GEOM);
    if (gm == 1 && a.Kpad % (16 * 8) == 0) return launch16_t<T, DPAD, P, 8, 2, OCC, 8>(a, s);
    if (gm == 2) return launch16_t<T, DPAD, P, CT, 2, OCC, 8>(a, s);
  }
  return launch16_t<T, DPAD, P, CT, 2, OCC>(a, s);
}

int assign16_chunk_tiles(int dtype, int dpad) { return plan::assign16_chunk_tiles(dtype == DT_BF16 ? 2 : 4, dpad); }
int assign_kpad(int dtype, int dpad, int K) { return plan::assign_kpad(dtype == DT_BF16 ? 2 : 4, dpad, K); }
int assign_cn_len(int kpad) { return plan::assign_cn_len(kpad); }

// Wide rows (DPAD 384..1024, e.g. sentence-embedding widths): one centre tile per chunk
// (12-32 KiB), and as many point blocks as ~256 registers of rows hold -- bf16 4 blocks at
// 384 features, 2 at 768, f32 2 and 1 -- at one wave per SIMD, or two where the kernel
// stays under 256 VGPRs (D=384, D=768).  bf16 D=512 takes 3 blocks (192 registers of rows,
// 2 waves/SIMD): +18 % at K=1024 and 4096, +26 % at K=256 against 4 blocks at one wave
// (profiles/r6_45_ab_d512_*.log); bf16 D=1024 takes 3 blocks at one wave (~450 VGPRs): +1.3 %
// at K=1024, +1.9 % at 4096 against 2 (profiles/r6_53_ab_*.log).  The fragment layout, the
// seed offsets and the argmin epilogue are the narrow kernels'; only the MFMA issue reads
// the A fragments one at a time (WIDE in assign16_kernel).
template <typename T, int DPAD>
constexpr int C_wide_rows() {   // registers of rows per lane: P blocks x NQ 16-B pieces x 4
  return p_wide<T, DPAD>() * (DPAD / 4 / Elem<T>::V) * 4;
}
template <typename T, int DPAD>
static hipError_t launch16_w(const AssignArgs& a, hipStream_t s) {
  constexpr int CT = chunk_tiles16(sizeof(T), DPAD);
  static_assert(CT == 1, "wide rows: one tile per chunk");
  constexpr int P = p_wide<T, DPAD>();
  static_assert(1536 % (4 * P * 16) == 0, "workgroup points must tile the shard grid");
  // rows in <= 192 registers: hold the kernel to 2 waves/SIMD (the bounded E-step's D=384
  // build took 257 VGPRs without the bound)
  constexpr int OCC = C_wide_rows<T, DPAD>() <= 192 ? 2 : 1;
  return launch16_t<T, DPAD, P, CT, 2, OCC>(a, s);
}

// NW * P * 16 of the geometry launch16_d / launch16_w pick for a call without bounds (the A/B
// switch V_ASSIGN_GEOM included): the row block each bf16 seed offset is taken over.  The
// bounded E-step's exactness rests on this (tests/test_gpu_bounded.py, bitwise trajectories).
template <typename T, int DPAD>
static int block_rows_t(int kpad) {
  if constexpr (DPAD > 256) return 4 * p_wide<T, DPAD>() * 16;
  const int gm = variant(V_ASSIGN_GEOM);
  if constexpr (sizeof(T) == 2 && DPAD == 256) {
    if (gm == 1) return 8 * 3 * 16;
  }
  if constexpr (sizeof(T) == 2 && DPAD == 128) {
    if ((gm == 1 && kpad % (16 * 8) == 0) || gm == 2) return 8 * 4 * 16;
  }
  return 4 * p_narrow<T, DPAD>() * 16;
}

int assign16_block_rows(int dtype, int dpad, int kpad) {
  if (dtype == DT_BF16) {
    switch (dpad) {
      case 32: return block_rows_t<uint16_t, 32>(kpad);
      case 64: return block_rows_t<uint16_t, 64>(kpad);
      case 128: return block_rows_t<uint16_t, 128>(kpad);
      case 256: return block_rows_t<uint16_t, 256>(kpad);
      case 384: return block_rows_t<uint16_t, 384>(kpad);
      case 512: return block_rows_t<uint16_t, 512>(kpad);
      case 768: return block_rows_t<uint16_t, 768>(kpad);
      case 1024: return block_rows_t<uint16_t, 1024>(kpad);
    }
  } else {
    switch (dpad) {
      case 16: return block_rows_t<float, 16>(kpad);
      case 32: return block_rows_t<float, 32>(kpad);
      case 64: return block_rows_t<float, 64>(kpad);
      case 128: return block_rows_t<float, 128>(kpad);
      case 256: return block_rows_t<float, 256>(kpad);
      case 384: return block_rows_t<float, 384>(kpad);
      case 512: return block_rows_t<float, 512>(kpad);
      case 768: return block_rows_t<float, 768>(kpad);
      case 1024: return block_rows_t<float, 1024>(kpad);
    }
  }
  return 0;
}

hipError_t launch_assign16(int dtype, int dpad, const AssignArgs& a, hipStream_t s) {
  if (dtype == DT_BF16) {
    switch (dpad) {
      case 32: return launch16_d<uint16_t, 32>(a, s);
      case 64: return launch16_d<uint16_t, 64>(a, s);
      case 128: return launch16_d<uint16_t, 128>(a, s);
      case 256: return launch16_d<uint16_t, 256>(a, s);
      case 384: return launch16_w<uint16_t, 384>(a, s);
      case 512: return launch16_w<uint16_t, 512>(a, s);
      case 768: return launch16_w<uint16_t, 768>(a, s);
      case 1024: return launch16_w<uint16_t, 1024>(a, s);
    }
  } else {
    switch (dpad) {
      case 16: return launch16_d<float, 16>(a, s);
      case 32: return launch16_d<float, 32>(a, s);
      case 64: return launch16_d<float, 64>(a, s);
      case 128: return launch16_d<float, 128>(a, s);
      case 256: return launch16_d<float, 256>(a, s);
      case 384: return launch16_w<float, 384>(a, s);
      case 512: return launch16_w<float, 512>(a, s);
      case 768: return launch16_w<float, 768>(a, s);
      case 1024: return launch16_w<float, 1024>(a, s);
    }
  }
  return hipErrorInvalidValue;
}

}  // namespace mk
