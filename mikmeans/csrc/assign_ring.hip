// mikmeans -- K2 with ONE centre ring per CU (bf16, plain full passes with row norms).
//
// assign16.hip runs four independent 4-wave workgroups per CU, each streaming all K centres
// through its own LDS ring: the L2 -> LDS centre stream is 4x the X bytes at the headline
// shape and one barrier per chunk paces every workgroup (profiles/r5_45_assign_prologue_study.md).
// Here one persistent 16-wave workgroup per CU shares a single deep ring, and no barrier
// paces it.  The ring is an endless stream of positions q = 0, 1, 2, ...; position q holds
// centre chunk q mod NCH in slot q mod NS.  Every wave follows a STATIC schedule: wave w
// consumes positions s0_w + k PERIOD + [0, NCH) for its k-th row block (one sweep over all
// NCH chunks, in rotated order), then spends SKIP positions on its epilogue and the next
// block's prologue, so the waves' start-up and finish are spread over the period and the
// ring never waits for a wave that is loading rows (PERIOD = NCH + SKIP; the starts s0_w are
// spread over one period).  Hand-off, all in LDS:
//  * ready[slot] = the position whose chunk has landed there (published by the wave that
//    issued its LDS-DMA, after that wave's own vmcnt wait);
//  * cnt[q mod 2NS] counts the touches of position q: one per consuming wave after its reads,
//    plus one token from the publisher.  need(q) -- how many waves consume q -- follows from
//    the schedule, so the wave whose add makes the count need(q) + 1 completes q: it takes the
//    count back down and issues the refill of slot q mod NS with position q + NS.  An add for
//    position q can only come after q + NS - ... completed (the refill chain), so a counter never
//    mixes two generations.
// Every spin is bounded (a fault word is set and the kernel drains instead of hanging).
//
// The scores, keys and labels are assign16's bit for bit: the same fragment layout, MFMA
// order, per-256-row seed offsets (here computed by each wave from the caller's norms of its
// row group) and per-point offsets for outlier groups; the rotated sweep merges its 16-tile
// segments on (truncated value, segment, index), the order the sequential sweep implies.
// A/B switch V_ASSIGN_RING (default off).
#include <type_traits>

#include "common.h"
#include "kernels.h"
#include "plan.h"

namespace mk {

static int* g_ring_fault = nullptr;

template <int DPAD, int P_, int NW_, int NS_, int SKIP_>
struct RingCfg {
  static constexpr int NW = NW_, P = P_, NS = NS_, SKIP = SKIP_;
  static constexpr int V = 8;                              // bf16 per 16-B piece
  static constexpr int NQ = DPAD / 4 / V;
  static constexpr int TILE_BYTES = NQ * 1024;
  static constexpr int CT = plan::chunk_tiles16(2, DPAD);
  static constexpr int CHUNK_BYTES = CT * TILE_BYTES;      // 16 KiB
  static constexpr int PIECES = CHUNK_BYTES / 1024;        // LDS-DMA wave-instructions per chunk
  static constexpr int ROWS = P * 16;                      // rows per wave block
  static constexpr int PP = (P + 3) / 4 * 4;
  // control words: cnt[2NS] | ready[NS] | s0[NW] | nb[NW] | need tables (steady [PERIOD],
  // start [PERIOD], end [3 PERIOD])
  static constexpr int CTRL_BYTES = 2048;
  static constexpr int OPT_BYTES = NW * 16 * PP * 4;       // per-point offsets (outlier groups)
  static constexpr int WS0 = 3 * NS, WNB = WS0 + NW, TAB = WNB + NW;
  static constexpr int PERIOD_MAX = (CTRL_BYTES / 4 - TAB) / 5;
  static_assert(256 % ROWS == 0, "a seed-offset group is whole wave blocks");
};

constexpr unsigned RING_SPIN_LIMIT = 1u << 22;   // polls (s_sleep 1 apart) before giving up

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const MK_LDS void*)p;
}
// LDS word ops by 32-bit LDS address, as inline asm: the compiler then inserts no vmcnt drain
// of the wave's in-flight LDS-DMA in front of them (it does before LDS atomics it emits itself).
// The atomics and the store run on lane 0 alone (a wave-wide ds_add would add 64 times); the
// results are broadcast with readfirstlane.
__device__ __forceinline__ uint32_t ring_add_rtn_at(uint32_t addr, uint32_t v) {
  uint32_t r = 0;
  if ((threadIdx.x & 63) == 0)
    asm volatile("ds_add_rtn_u32 %0, %1, %2\n\ts_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(addr), "v"(v) : "memory");
  return __builtin_amdgcn_readfirstlane(r);
}
__device__ __forceinline__ void ring_sub_at(uint32_t addr, uint32_t v) {
  if ((threadIdx.x & 63) == 0) asm volatile("ds_sub_u32 %0, %1" ::"v"(addr), "v"(v) : "memory");
}
__device__ __forceinline__ uint32_t ring_load_at(uint32_t addr) {
  uint32_t r;
  asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(addr) : "memory");
  return __builtin_amdgcn_readfirstlane(r);
}
__device__ __forceinline__ void ring_store_at(uint32_t addr, uint32_t v) {
  if ((threadIdx.x & 63) == 0) asm volatile("ds_write_b32 %0, %1" ::"v"(addr), "v"(v) : "memory");
}

// The static schedule: wave w starts at s0_w = w PERIOD / NW and processes nb_w row blocks
// (positions fit 32 bits).  need(q), the waves consuming position q, is tabulated at start:
// the start [0, s0max), the steady state (every wave inside its schedule: a function of
// q mod PERIOD) and the end [qfull, qmax] (the waves' last sweeps; <= 3 periods, since the
// waves' block counts differ by at most one).
__device__ __forceinline__ uint32_t ring_need_count(const int* s0, const int* nb, int nw, int period, int nch, int q) {
  uint32_t n = 0;
  for (int w = 0; w < nw; ++w) {
    const int d = q - s0[w];
    if (d >= 0 && d < nb[w] * period && (d % period) < nch) ++n;
  }
  return n;
}

template <int DPAD, int P, int NW, int NS, int SKIP>
__global__ __launch_bounds__(NW * 64, 4) void assign_ring_kernel(AssignArgs a, int* fault) {
  using C = RingCfg<DPAD, P, NW, NS, SKIP>;
  static_assert((NS & (NS - 1)) == 0, "ring slots: a power of two");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 15, g = lane >> 4;
  const int cn_bytes = ((a.Kpad * 4 + 1023) / 1024) * 1024;
  char* cn_lds = smem;
  char* ring = smem + cn_bytes;
  uint32_t* ctrl = (uint32_t*)(ring + C::NS * C::CHUNK_BYTES);
  // control words by 32-bit LDS address (inline-asm operands)
  const uint32_t a_cnt = lds_addr(ctrl), a_ready = a_cnt + 4 * 2 * C::NS;
  int* ws0 = (int*)(ctrl + C::WS0);   // [NW] schedule starts
  int* wnb = (int*)(ctrl + C::WNB);   // [NW] row blocks per wave
  float* opt = (float*)((char*)ctrl + C::CTRL_BYTES) + wid * 16 * C::PP;   // this wave's [16][PP]

  const int64_t N = a.N;
  const int nch = a.Kpad / (16 * C::CT);
  const int ngrp = nch * C::CT;   // tiles
  const int period = nch + C::SKIP;
  const int64_t nblk = (N + C::ROWS - 1) / C::ROWS;
  const int64_t G = (int64_t)gridDim.x * C::NW;
  const int64_t gbase = (int64_t)blockIdx.x * C::NW;
  uint32_t* tab = ctrl + C::TAB;         // steady [period]
  uint32_t* tab_s = tab + period;        // start [period]
  uint32_t* tab_e = tab + 2 * period;    // end [3 period]

  // ---- start: |c|^2, the control words and the schedule's need tables; two barriers
  for (int i = threadIdx.x; i < cn_bytes / 4; i += C::NW * 64)
    ((float*)cn_lds)[i] = i < a.Kpad ? a.cn[i] : 0.f;
  if (threadIdx.x < 2 * C::NS) ctrl[threadIdx.x] = 0u;
  if (threadIdx.x < C::NS) ctrl[2 * C::NS + threadIdx.x] = 0xffffffffu;
  if (threadIdx.x < C::NW) {
    const int64_t gw = gbase + threadIdx.x;
    ws0[threadIdx.x] = ((int)threadIdx.x * period) / C::NW;
    wnb[threadIdx.x] = gw < nblk ? (int)((nblk - gw + G - 1) / G) : 0;
  }
  __syncthreads();
  const int s0max = ws0[C::NW - 1];
  int qmax = -1, qfull = 0x7fffffff;
  for (int w = 0; w < C::NW; ++w) {
    const int s0w = ws0[w], nbw = wnb[w];
    if (nbw > 0) qmax = max(qmax, s0w + (nbw - 1) * period + nch - 1);   // last position consumed
    qfull = min(qfull, nbw > 0 ? s0w + (nbw - 1) * period : s0max);
  }
  qfull = __builtin_amdgcn_readfirstlane(max(qfull, s0max));
  qmax = __builtin_amdgcn_readfirstlane(qmax);
  if ((int)threadIdx.x < period) {
    tab[threadIdx.x] = ring_need_count(ws0, wnb, C::NW, period, nch,
                                       s0max + ((int)threadIdx.x - s0max % period + period) % period);
    tab_s[threadIdx.x] = ring_need_count(ws0, wnb, C::NW, period, nch, (int)threadIdx.x);
  }
  if ((int)threadIdx.x < 3 * period)
    tab_e[threadIdx.x] = ring_need_count(ws0, wnb, C::NW, period, nch, qfull + (int)threadIdx.x);
  if (threadIdx.x == 0 && qmax - qfull >= 3 * period) atomicOr(fault, 2);   // (the end table's bound)
  __syncthreads();

  // consumers of position q at phase ph = q mod period
  auto need = [&](int q, int ph) -> uint32_t {
    if (q < s0max) return tab_s[q];
    if (q < qfull) return tab[ph];
    return tab_e[q - qfull];
  };
  const uint32_t loff = (uint32_t)lane * 16u;
  const __amdgpu_buffer_rsrc_t rC = make_rsrc(a.Cpack, (uint32_t)a.Kpad * DPAD * 2u);
  auto issue = [&](int q) {   // position q's chunk into its slot (this wave's LDS-DMAs)
    const uint32_t src = (uint32_t)(q % nch) * C::CHUNK_BYTES;
    char* dst = ring + (q & (C::NS - 1)) * C::CHUNK_BYTES;
#pragma unroll
    for (int i = 0; i < C::PIECES; ++i)
      blds16(rC, (MK_LDS void*)(dst + i * 1024), loff, src + (uint32_t)i * 1024u);
  };
  // publish q (its DMA has landed: the caller waited vmcnt) and add the token; while that
  // completes a position nobody consumes, refill and publish synchronously (rare)
  auto publish = [&](int q) {
    for (;;) {
      ring_store_at(a_ready + 4 * (q & (C::NS - 1)), (uint32_t)q);
      const uint32_t nd = need(q, q % period);
      const uint32_t ca = a_cnt + 4 * (q & (2 * C::NS - 1));
      if (ring_add_rtn_at(ca, 1u) != nd) return;   // consumers still to come
      ring_sub_at(ca, nd + 1u);
      if (q + C::NS > qmax) return;
      q += C::NS;
      issue(q);
      wait_vmcnt<0>();
    }
  };
  int pending = -1;   // a refill this wave issued and has not published yet
  bool faulted = false;
  // (a.timeline: per-wave cycle counters -- total, ready spins, prologues, epilogues, touch /
  // publish work inside sweeps, blocks, sleeping polls, start-up)
  const bool tl_on = a.timeline != nullptr;
  unsigned long long tl[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const unsigned long long t_entry = tl_on ? __builtin_amdgcn_s_memtime() : 0ull;
  if (wid < C::NS && wid <= qmax) {   // the first NS positions
    issue(wid);
    wait_vmcnt<0>();
    publish(wid);
  }

  if (tl_on) tl[7] = __builtin_amdgcn_s_memtime() - t_entry;
  const unsigned kmask = key6_mask();
  const float* xn = a.xn;
  const int nb = wnb[wid];
  const int s0 = ws0[wid];
  for (int k = 0; k < nb && !faulted; ++k) {
    const int64_t blk = gbase + wid + (int64_t)k * G;
    const int64_t pbase = blk * C::ROWS;
    const unsigned long long t_pro = tl_on ? __builtin_amdgcn_s_memtime() : 0ull;
    // ---- prologue: the group's norms (seed offset), the rows' fragments, the epilogue's reads
    const int64_t grp = pbase & ~(int64_t)255;
    float m = 0.f, mn = 3.0e38f;
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int64_t i = grp + lane + 64 * jj;
      const float v = xn[i < N ? i : N - 1];
      m = fmaxf(m, v);
      mn = fminf(mn, v);
    }
    u32x4 xr[C::P][C::NQ];
#pragma unroll
    for (int p = 0; p < C::P; ++p) {
      const int64_t row = min(pbase + p * 16 + r, N - 1);
      const uint16_t* rp = (const uint16_t*)a.X + row * a.ldx + g * C::V;
#pragma unroll
      for (int qq = 0; qq < C::NQ; ++qq) xr[p][qq] = *(const u32x4*)(rp + 4 * qq * C::V);
    }
    constexpr int EJ = (C::P + 3) / 4;
    int eold[EJ];
    float exn[EJ];
#pragma unroll
    for (int jj = 0; jj < EJ; ++jj) {
      const int pg = 4 * jj + g;
      const int64_t i = pbase + pg * 16 + r;
      const bool mine = pg < C::P && i < N;
      const int64_t ic = i < N ? i : N - 1;
      eold[jj] = mine && a.track_changed ? a.labels[ic] : -2;
      exn[jj] = mine ? xn[ic] : 0.f;
    }
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      m = fmaxf(m, __shfl_xor(m, o, 64));
      mn = fminf(mn, __shfl_xor(mn, o, 64));
    }
    const bool ppo = __builtin_amdgcn_readfirstlane((int)(m > 4.f * mn)) != 0;
    float off = 0.f;
    if (!ppo) {
      off = __builtin_fmaf(m, 2.44140625e-04f, m);   // * (1 + 2^-12), as assign16
      off = __uint_as_float(__builtin_amdgcn_readfirstlane(__float_as_uint(off)));
    } else if (g == 0) {
      // per-point offsets o_p = (1 + 2^-12) |x_p|^2 of this wave's rows (lane r, block p)
#pragma unroll
      for (int p = 0; p < C::P; ++p) {
        const int64_t row = min(pbase + p * 16 + r, N - 1);
        const float v = xn[row];
        opt[r * C::PP + p] = __builtin_fmaf(v, 2.44140625e-04f, v);
      }
    }
    wait_vmcnt<0>();   // fragments, norms, labels (and any refill still pending: published here)
    wait_lgkm0();
    if (pending >= 0) {
      publish(pending);
      pending = -1;
    }

    if (tl_on) { tl[2] += __builtin_amdgcn_s_memtime() - t_pro; tl[5] += 1; }
    // ---- the sweep: positions q0 .. q0 + nch - 1, chunk c = q mod nch, phase ph = q mod period
    int q = s0 + k * period;
    int c = q % nch;
    int ph = s0;   // (s0 < period)
    float best[C::P], seg_best[C::P];
    int bg[C::P];
#pragma unroll
    for (int p = 0; p < C::P; ++p) { best[p] = 3.0e38f; seg_best[p] = 3.0e38f; bg[p] = 0x7fffffff; }
    auto merge_seg = [&](int seg) {
#pragma unroll
      for (int p = 0; p < C::P; ++p) {
        // (truncated value, segment, index) order, branch-free: the sequential sweep's winner
        const uint32_t sb = __float_as_uint(seg_best[p]), bb = __float_as_uint(best[p]);
        const uint32_t sv = sb & ~63u, bv = bb & ~63u;
        const bool take = (sv < bv) | ((sv == bv) & ((seg < bg[p]) | ((seg == bg[p]) & (sb < bb))));
        best[p] = take ? seg_best[p] : best[p];
        bg[p] = take ? seg : bg[p];
        seg_best[p] = 3.0e38f;
      }
    };
    auto chunk_loop = [&](auto ppo_tag) {
      constexpr bool PPO = decltype(ppo_tag)::value;
      for (int j = 0; j < nch; ++j) {
        // wait for position q
        {
          unsigned spins = 0;
          const unsigned long long t_w = tl_on ? __builtin_amdgcn_s_memtime() : 0ull;
          while (ring_load_at(a_ready + 4 * (q & (C::NS - 1))) != (uint32_t)q) {
            __builtin_amdgcn_s_sleep(1);
            if (++spins > RING_SPIN_LIMIT) { faulted = true; break; }
          }
          if (tl_on) { tl[1] += __builtin_amdgcn_s_memtime() - t_w; tl[6] += spins; }
          if (faulted) break;
        }
        const char* buf = ring + (q & (C::NS - 1)) * C::CHUNK_BYTES;
#pragma unroll
        for (int tl_i = 0; tl_i < C::CT; ++tl_i) {
          const int tile = c * C::CT + tl_i;
          f32x4 ci = *(const f32x4*)(cn_lds + (tile * 16 + 4 * g) * 4);
          const char* tl = buf + tl_i * C::TILE_BYTES + lane * 16;
          u32x4 aw[C::NQ];
#pragma unroll
          for (int qq = 0; qq < C::NQ; ++qq) aw[qq] = *(const u32x4*)(tl + qq * 1024);
          f32x4 acc[C::P];
          if constexpr (PPO) {
#pragma unroll
            for (int p = 0; p < C::P; ++p) acc[p] = ci;
            const float* o = opt + r * C::PP;
#pragma unroll
            for (int p4 = 0; p4 < C::P; p4 += 4) {
              const f32x4 ov = *(const f32x4*)(o + p4);
#pragma unroll
              for (int jj = 0; jj < 4; ++jj)
                if (p4 + jj < C::P) seed_add(acc[p4 + jj], ov[jj]);
            }
          } else {
            seed_add(ci, off);   // |c|^2 + o: assign16's LDS copy of |c|^2 + o, the same f32 adds
#pragma unroll
            for (int p = 0; p < C::P; ++p) acc[p] = ci;
          }
          unsigned t0, t1, t2, t3;
          const unsigned tis = __builtin_amdgcn_readfirstlane((unsigned)(tile & 15) << 2);
          asm volatile("s_mov_b32 %0, %4\n\ts_or_b32 %1, %4, 1\n\ts_or_b32 %2, %4, 2\n\ts_or_b32 %3, %4, 3"
                       : "=s"(t0), "=s"(t1), "=s"(t2), "=s"(t3) : "s"(tis) : "scc");
          __builtin_amdgcn_sched_barrier(0);
          __builtin_amdgcn_s_setprio(1);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int p = 0; p < C::P; ++p) {
#pragma unroll
            for (int qq = 0; qq < C::NQ; ++qq) {
              acc[p] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(short8, aw[qq]),
                                                              __builtin_bit_cast(short8, xr[p][qq]), acc[p], 0, 0, 0);
              __builtin_amdgcn_sched_barrier(0);
            }
          }
          __builtin_amdgcn_sched_barrier(0);
          __builtin_amdgcn_s_setprio(0);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int p = 0; p < C::P; ++p) {
            const f32x4& sv = acc[p];
            const float k0 = pack_key6(sv[0], kmask, t0), k1 = pack_key6(sv[1], kmask, t1);
            const float k2 = pack_key6(sv[2], kmask, t2), k3 = pack_key6(sv[3], kmask, t3);
            seg_best[p] = min3f(min3f(k0, k1, k2), k3, seg_best[p]);
          }
          // a segment ends at its 16th tile, at the stream's last tile, or where the sweep ends
          if ((tile & 15) == 15 || tile == ngrp - 1 || (j == nch - 1 && tl_i == C::CT - 1)) merge_seg(tile >> 4);
        }
        // done with position q: the deferred publish of this wave's last refill (issued a
        // chunk ago: landed), then the touch; the wave that completes q refills its slot
        const unsigned long long t_t = tl_on ? __builtin_amdgcn_s_memtime() : 0ull;
        if (pending >= 0) {
          wait_vmcnt<0>();
          publish(pending);
          pending = -1;
        }
        {
          const uint32_t nd = need(q, ph);
          const uint32_t ca = a_cnt + 4 * (q & (2 * C::NS - 1));
          if (ring_add_rtn_at(ca, 1u) == nd) {   // (the token and the other touches are in)
            ring_sub_at(ca, nd + 1u);
            if (q + C::NS <= qmax) {
              issue(q + C::NS);
              pending = q + C::NS;
            }
          }
        }
        if (tl_on) tl[4] += __builtin_amdgcn_s_memtime() - t_t;
        ++q;
        c = c + 1 == nch ? 0 : c + 1;
        ph = ph + 1 == period ? 0 : ph + 1;
      }
    };
    if (ppo) chunk_loop(std::true_type{});
    else chunk_loop(std::false_type{});
    if (faulted) {
      if (lane == 0) atomicOr(fault, 1);
      break;
    }
    if (pending >= 0) {   // (a refill from the sweep's last touch: NS positions ahead, publish now)
      wait_vmcnt<0>();
      publish(pending);
      pending = -1;
    }

    // ---- epilogue: the 4 lane groups of each point merged on (value, centre), then stores
    const unsigned long long t_epi = tl_on ? __builtin_amdgcn_s_memtime() : 0ull;
    float inert = 0.f;
    int changed = 0;
#pragma unroll
    for (int p = 0; p < C::P; ++p) {
      const unsigned bits = __float_as_uint(best[p]);
      const int idx = (int)(bits & 63u);
      int kk = (bg[p] * 16 + (idx >> 2)) * 16 + 4 * g + (idx & 3);
      float v = __uint_as_float(bits & ~63u);
#pragma unroll
      for (int o = 16; o <= 32; o <<= 1) {
        const float vo = __shfl_xor(v, o, 64);
        const int ko = __shfl_xor(kk, o, 64);
        if (vo < v || (vo == v && ko < kk)) { v = vo; kk = ko; }
      }
      const int64_t i = pbase + p * 16 + r;
      if ((p & 3) == g && i < N) {
        const float offp = ppo ? opt[r * C::PP + p] : off;
        v -= offp;
        if (a.track_changed) changed += (eold[p >> 2] != kk);
        a.labels[i] = kk;
        const float d = fmaxf(exn[p >> 2] + v, 0.f);
        inert += d;
        if (a.mind) a.mind[i] = d;
      }
    }
    if (a.slots) {
      const double di = wave_sum((double)inert);
      const int dc = wave_sum(changed);
      if (lane == 0) slot_add((unsigned long long*)(a.slots + ((blk >> 2) % NSLOT) * SLOT_STRIDE), di, (long long)dc);
    }
    if (tl_on) tl[3] += __builtin_amdgcn_s_memtime() - t_epi;
  }
  // every DMA this wave issued lands before the workgroup's LDS is released; a refill issued at
  // the last sweep's end is published, so no consumer waits on it
  wait_vmcnt<0>();
  if (pending >= 0 && !faulted) publish(pending);
  wait_vmcnt<0>();
  if (tl_on && lane == 0) {
    tl[0] = __builtin_amdgcn_s_memtime() - t_entry;
    unsigned long long* o = a.timeline + ((int64_t)blockIdx.x * C::NW + wid) * 8;
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = tl[i];
  }
}

template <int DPAD, int P, int NW, int NS, int SKIP>
static hipError_t launch_ring_t(const AssignArgs& a, hipStream_t s) {
  using C = RingCfg<DPAD, P, NW, NS, SKIP>;
  static int* fault = nullptr;
  if (!fault) {
    if (hipMalloc(&fault, sizeof(int)) != hipSuccess) return hipErrorOutOfMemory;
    (void)hipMemsetAsync(fault, 0, sizeof(int), s);
  }
  const int cn_bytes = ((a.Kpad * 4 + 1023) / 1024) * 1024;
  const size_t lds = cn_bytes + (size_t)C::NS * C::CHUNK_BYTES + C::CTRL_BYTES + C::OPT_BYTES;
  if (lds > 160 * 1024 || a.Kpad % (16 * C::CT) != 0 || a.Kpad / (16 * C::CT) + SKIP > C::PERIOD_MAX)
    return hipErrorInvalidValue;   // (period bound: PERIOD_MAX)
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)assign_ring_kernel<DPAD, P, NW, NS, SKIP>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  static int cus = [] {
    int dev = 0, n = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    return n;
  }();
  const int64_t nblk = (a.N + C::ROWS - 1) / C::ROWS;
  const int64_t wgs = (nblk + C::NW - 1) / C::NW;
  const unsigned grid = (unsigned)(wgs < cus ? wgs : cus);
  AssignArgs b = a;
  int64_t cap = 0;
  unsigned long long* tlb = assign_timeline_buffer(&cap);
  b.timeline = (tlb && cap >= (int64_t)grid * NW) ? tlb : nullptr;   // (per wave, see the kernel)
  hipLaunchKernelGGL((assign_ring_kernel<DPAD, P, NW, NS, SKIP>), dim3(grid), dim3(NW * 64), lds, s, b, fault);
  g_ring_fault = fault;
  return hipGetLastError();
}

bool assign_ring_takes(int dtype, int dpad, const AssignArgs& a) {
  return dtype == DT_BF16 && dpad == 128 && a.D == 128 && a.xn && !a.rows && !a.split_keys && !a.ub && !a.oseed &&
         !a.n_dev && !a.scatter && a.N >= 256;
}

hipError_t launch_assign_ring(int dpad, const AssignArgs& a, hipStream_t s) {
  (void)dpad;
  // (A/B: the switch's value picks the skip window -- positions a wave spends on its
  // epilogue and next prologue between sweeps)
  switch (variant(V_ASSIGN_RING)) {
    case 2: return launch_ring_t<128, 4, 16, 8, 10>(a, s);
    case 3: return launch_ring_t<128, 4, 16, 8, 14>(a, s);
    default: return launch_ring_t<128, 4, 16, 8, 6>(a, s);
  }
}

int assign_ring_fault() {
  int h = 0;
  if (g_ring_fault) (void)hipMemcpy(&h, g_ring_fault, sizeof(int), hipMemcpyDeviceToHost);
  return h;
}

}  // namespace mk
