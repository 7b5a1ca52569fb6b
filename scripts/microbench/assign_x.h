// Experimental assign variants for scripts/microbench/assign_ab.hip (bf16 only, no
// centre split, xn given).  Same arithmetic as mk::assign16_kernel, so labels must match
// bit for bit; only the schedule differs.
//   MODE bit 0: skew -- the argmin epilogue of tile j runs after the MFMAs of tile j+1
//               are issued (two accumulator sets), so VALU overlaps the matrix pipe
//               inside one wave instead of waiting for the MFMA results.
//   MODE bit 1: sched_group_barrier interleave (1 MFMA : 2 VALU) of that overlap.
//   MODE bit 2: A fragments of tile j+1 read from LDS while tile j's MFMAs run.
#pragma once
#include "../../mikmeans/csrc/common.h"
#include "../../mikmeans/csrc/kernels.h"

namespace mkx {
using namespace mk;

template <int DPAD, int P, int OCC, int MODE, int NW = 4, int NBUF = 2>
__global__ __launch_bounds__(NW * 64, OCC) void assign_x_kernel(AssignArgs a) {
  constexpr int V = 8;
  constexpr int NQ = DPAD / 4 / V;
  constexpr int TILE_BYTES = NQ * 1024;
  constexpr int CT = plan::chunk_tiles16(2, DPAD);
  constexpr int CHUNK_BYTES = CT * TILE_BYTES;
  constexpr int PIECES = CHUNK_BYTES / 1024;
  constexpr int NPW = PIECES / NW;
  constexpr int PTS = NW * P * 16;
  constexpr bool SKEW = MODE & 1, SGB = MODE & 2, PF = MODE & 4;
  constexpr bool STAMP = MODE & 8;   // per-workgroup (s_memtime, s_memrealtime) at start/end
  constexpr bool NOEPI = MODE & 16;
  constexpr bool EARLY = MODE & 32;
  constexpr bool PRIO = MODE & (1024 | 2048 | 4096);  // raised s_setprio while this wave issues its MFMAs
  constexpr int PRIO_LV = (MODE & 2048) ? 3 : 1;       // 2048: level 3 instead of 1
  constexpr bool PRIO_LD = MODE & 4096;                // 4096: raised already for the tile's LDS reads
  // exact fp32 (value, index) compare, gated per tile: a tile's keyed update runs only for
  // point blocks where some lane's tile minimum is <= its threshold, seeded with the score
  // to the previous label's centre (VALU dot product + rounding margin)
  constexpr bool GATE = MODE & 64;
  constexpr bool NOWAIT = MODE & 512;  // ablation: ring refills issued but never waited for (racy)
  constexpr bool NORING = MODE & 256;  // ablation: no ring refills after the first two chunks (stale C)
  constexpr bool DUMP = MODE & 128;  // debug: mind[i] = seed (unfudged) + |x|^2  // next tile's fragments read into the same registers before the epilogue  // ablation: no argmin epilogue (accumulators kept live)
  unsigned long long t_beg = 0, r_beg = 0;
  if constexpr (STAMP) { t_beg = __builtin_amdgcn_s_memtime(); r_beg = __builtin_amdgcn_s_memrealtime(); }
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 15, g = lane >> 4;
  const int cn_bytes = ((a.Kpad * 4 + 1023) / 1024) * 1024;
  char* cn_lds = smem;
  char* bufs = smem + cn_bytes;
  const int nch = a.Kpad / (16 * CT);
  const uint32_t loff = (uint32_t)lane * 16u;
  const __amdgpu_buffer_rsrc_t rC = make_rsrc(a.Cpack, (uint32_t)a.Kpad * DPAD * 2);
  const __amdgpu_buffer_rsrc_t rN = make_rsrc(a.cn, (uint32_t)a.Kpad * 4u);
  for (int p = wid; p < cn_bytes / 1024; p += NW)
    blds16(rN, (MK_LDS void*)(cn_lds + p * 1024), loff, (uint32_t)p * 1024u);
  auto issue_chunk = [&](int c) {
    const uint32_t src = (uint32_t)c * CHUNK_BYTES;
    char* dst = bufs + (c % NBUF) * CHUNK_BYTES;
#pragma unroll
    for (int i = 0; i < NPW; ++i) {
      const int pc = wid + i * NW;
      blds16(rC, (MK_LDS void*)(dst + pc * 1024), loff, src + (uint32_t)pc * 1024u);
    }
  };
#pragma unroll
  for (int c = 0; c < NBUF - 1; ++c)
    if (c < a.Kpad / (16 * CT)) issue_chunk(c);

  const int64_t pbase = (int64_t)blockIdx.x * PTS + (int64_t)wid * (P * 16);
  u32x4 xr[P][NQ];
  float xnr[P];
#pragma unroll
  for (int p = 0; p < P; ++p) {
    int64_t row = pbase + p * 16 + r;
    row = row < a.N ? row : (a.N - 1);
    xnr[p] = a.xn[row];
    const uint16_t* rp = (const uint16_t*)a.X + row * a.ldx + g * (DPAD / 4);
#pragma unroll
    for (int q = 0; q < NQ; ++q) xr[p][q] = *(const u32x4*)(rp + q * V);
  }
  wait_vmcnt<0>();

  float off = 0.f;
  {
    float m = 0.f;
#pragma unroll
    for (int p = 0; p < P; ++p) m = fmaxf(m, xnr[p]);
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    float* red = (float*)(bufs + NBUF * CHUNK_BYTES);
    if (lane == 0) red[wid] = m;
    __syncthreads();
#pragma unroll
    for (int w = 0; w < NW; ++w) off = fmaxf(off, red[w]);
    off = __builtin_fmaf(off, 2.44140625e-04f, off);
    off = __uint_as_float(__builtin_amdgcn_readfirstlane(__float_as_uint(off)));
    for (int k = threadIdx.x; k < a.Kpad; k += NW * 64) ((float*)cn_lds)[k] += off;
  }

  float thr[P], seedv[P];
  if constexpr (GATE) {
    typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
    const char* cp = (const char*)a.Cpack;
#pragma unroll
    for (int p = 0; p < P; ++p) {
      int64_t row = pbase + p * 16 + r;
      row = row < a.N ? row : (a.N - 1);
      const int lab = a.labels[row];
      const bool ok = (unsigned)lab < (unsigned)a.Kpad;
      const int kk = ok ? lab : 0;
      float dot = 0.f;
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const u32x4 w = *(const u32x4*)(cp + ((size_t)((kk >> 4) * NQ + q) * 64 + (kk & 15) + 16 * g) * 16);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          dot = __builtin_fmaf(bf16lo(xr[p][q][e]), bf16lo(w[e]), dot);
          dot = __builtin_fmaf(bf16hi(xr[p][q][e]), bf16hi(w[e]), dot);
        }
      }
      dot += __shfl_xor(dot, 16, 64);
      dot += __shfl_xor(dot, 32, 64);
      const float cnk = a.cn[kk];
      // |mfma - valu| <= 2 gamma_{D+1} (|c|^2 + 2 sum|x_i c_i|) <= 2^-12 (|x|^2 + 2|c|^2) for D <= 256
      const float seed = (cnk + off) + dot + 2.44140625e-04f * (xnr[p] + 2.f * cnk) + 1e-30f;
      thr[p] = ok ? seed : 3.0e38f;
      seedv[p] = cnk + dot;
    }
  }
  float best[P], seg_best[P];
  int bg[P];
#pragma unroll
  for (int p = 0; p < P; ++p) { best[p] = 3.0e38f; seg_best[p] = 3.0e38f; bg[p] = 0; }
  const int ngrp = nch * CT;
  const unsigned kmask = key6_mask();

  // epilogue of one tile's accumulators
  auto epilogue = [&](const f32x4* acc, int tile) {
    const unsigned tis = (unsigned)(tile & 15) << 2;
    unsigned t0, t1, t2, t3;
    asm volatile("s_mov_b32 %0, %4\n\ts_or_b32 %1, %4, 1\n\ts_or_b32 %2, %4, 2\n\ts_or_b32 %3, %4, 3"
                 : "=s"(t0), "=s"(t1), "=s"(t2), "=s"(t3) : "s"(tis));
#pragma unroll
    for (int p = 0; p < P; ++p) {
      const f32x4& sv = acc[p];
      const float k0 = pack_key6(sv[0], kmask, t0), k1 = pack_key6(sv[1], kmask, t1);
      const float k2 = pack_key6(sv[2], kmask, t2), k3 = pack_key6(sv[3], kmask, t3);
      seg_best[p] = min3f(min3f(k0, k1, k2), k3, seg_best[p]);
    }
    if ((tile & 15) == 15 || tile == ngrp - 1) {
#pragma unroll
      for (int p = 0; p < P; ++p) {
        const float sv = __uint_as_float(__float_as_uint(seg_best[p]) & ~63u);
        const float bv = __uint_as_float(__float_as_uint(best[p]) & ~63u);
        if (sv < bv) { best[p] = seg_best[p]; bg[p] = tile >> 4; }
        seg_best[p] = 3.0e38f;
      }
    }
  };

  f32x4 accp[P];
#pragma unroll
  for (int p = 0; p < P; ++p) accp[p] = f32x4{3.0e38f, 3.0e38f, 3.0e38f, 3.0e38f};
  int tprev = -1;

  for (int c = 0; c < nch; ++c) {
    if constexpr (NOWAIT) { if (c < 1) wait_vmcnt<0>(); }
    else if constexpr (NBUF > 2) { if (c + NBUF - 2 < nch) wait_vmcnt<(NBUF - 2) * NPW>(); else wait_vmcnt<0>(); }
    else wait_vmcnt<0>();
    wait_lgkm0();
    raw_barrier();
    if (c + NBUF - 1 < nch && (!NORING || c + 1 < 2)) issue_chunk(c + NBUF - 1);
    const char* buf = bufs + (c % NBUF) * CHUNK_BYTES;
    u32x4 awn[NQ];
    f32x4 cin;
    auto load_a = [&](int tl_i, u32x4* aw_, f32x4& ci_) {
      const int tile = c * CT + tl_i;
      ci_ = *(const f32x4*)(cn_lds + (tile * 16 + 4 * g) * 4);
      const char* tl = buf + tl_i * TILE_BYTES + lane * 16;
#pragma unroll
      for (int q = 0; q < NQ; ++q) aw_[q] = *(const u32x4*)(tl + q * 1024);
    };
    if constexpr (PF) load_a(0, awn, cin);
    u32x4 awe[NQ];
    f32x4 cie;
    if constexpr (EARLY) load_a(0, awe, cie);
#pragma unroll
    for (int tl_i = 0; tl_i < CT; ++tl_i) {
      const int tile = c * CT + tl_i;
      u32x4 aw[NQ];
      f32x4 ci;
      if constexpr (PF) {
#pragma unroll
        for (int q = 0; q < NQ; ++q) aw[q] = awn[q];
        ci = cin;
        if (tl_i + 1 < CT) load_a(tl_i + 1, awn, cin);
      } else if constexpr (EARLY) {
#pragma unroll
        for (int q = 0; q < NQ; ++q) aw[q] = awe[q];
        ci = cie;
      } else {
        if constexpr (PRIO_LD) {
          __builtin_amdgcn_sched_barrier(0);
          __builtin_amdgcn_s_setprio(1);
          __builtin_amdgcn_sched_barrier(0);
        }
        load_a(tl_i, aw, ci);
      }
      f32x4 acc[P];
#pragma unroll
      for (int p = 0; p < P; ++p) acc[p] = ci;
      if constexpr (PRIO && !PRIO_LD) {
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(PRIO_LV);
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
#pragma unroll
        for (int p = 0; p < P; ++p) acc[p] = Mfma16<uint16_t>::run(aw[q], xr[p][q], acc[p]);
      }
      if constexpr (PRIO) {
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
      }
      if constexpr (SKEW) {
        epilogue(accp, tprev);
        if constexpr (SGB) {
          // interleave: the tile's NQ*P MFMAs with the previous tile's 6P VALU
#pragma unroll
          for (int i = 0; i < NQ * P; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
            __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);  // VALU
          }
        }
#pragma unroll
        for (int p = 0; p < P; ++p) accp[p] = acc[p];
        tprev = tile;
      } else if constexpr (GATE) {
        unsigned long long open[P];
#pragma unroll
        for (int p = 0; p < P; ++p) {
          // keys are > 0 (seed offset), so the float order is the unsigned order of the bits
          const unsigned b0 = __float_as_uint(acc[p][0]), b1 = __float_as_uint(acc[p][1]);
          const unsigned b2 = __float_as_uint(acc[p][2]), b3 = __float_as_uint(acc[p][3]);
          const unsigned m = __builtin_elementwise_min(__builtin_elementwise_min(b0, b1), __builtin_elementwise_min(b2, b3));
          open[p] = __builtin_amdgcn_ballot_w64(m <= __float_as_uint(thr[p]));
        }
        const int u = tile * 4;
#pragma unroll
        for (int p = 0; p < P; ++p) {
          if (open[p]) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const bool lt = acc[p][e] < best[p];
              best[p] = lt ? acc[p][e] : best[p];
              bg[p] = lt ? u + e : bg[p];
            }
            thr[p] = __uint_as_float(__builtin_elementwise_min(__float_as_uint(thr[p]), __float_as_uint(best[p])));
          }
        }
      } else if constexpr (EARLY) {
        if (tl_i + 1 < CT) load_a(tl_i + 1, awe, cie);
        __builtin_amdgcn_sched_barrier(0);
        epilogue(acc, tile);
      } else if constexpr (NOEPI) {
#pragma unroll
        for (int p = 0; p < P; ++p) asm volatile("" :: "v"(acc[p]));
      } else {
        epilogue(acc, tile);
      }
    }
  }
  if constexpr (SKEW) epilogue(accp, tprev);

  float inert = 0.f;
#pragma unroll
  for (int p = 0; p < P; ++p) {
    int k;
    float v;
    if constexpr (GATE) {
      k = (bg[p] >> 2) * 16 + 4 * g + (bg[p] & 3);
      v = best[p];
    } else {
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
    if ((p & 3) == g) {
      const int64_t i = pbase + p * 16 + r;
      if (i < a.N) {
        v -= off;
        a.labels[i] = k;
        const float d = fmaxf(a.xn[i] + v, 0.f);
        inert += d;
        if (a.mind) a.mind[i] = d;
        if constexpr (DUMP) a.mind[i] = seedv[p] + a.xn[i];
      }
    }
  }
  (void)inert;
  if constexpr (STAMP) {
    const unsigned long long t_end = __builtin_amdgcn_s_memtime(), r_end = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0 && a.split_keys) {
      unsigned long long* st = a.split_keys + (size_t)blockIdx.x * 2;
      st[0] = t_end - t_beg;
      st[1] = r_end - r_beg;
    }
  }
}

template <int DPAD, int P, int OCC, int MODE, int NW = 4, int NBUF = 2>
static hipError_t launch_x(const AssignArgs& a, hipStream_t s) {
  constexpr int CT = plan::chunk_tiles16(2, DPAD);
  constexpr int CHUNK_BYTES = CT * (DPAD / 32) * 1024;
  const int cn_bytes = ((a.Kpad * 4 + 1023) / 1024) * 1024;
  const size_t lds = cn_bytes + NBUF * CHUNK_BYTES + 16 * NW;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)assign_x_kernel<DPAD, P, OCC, MODE, NW, NBUF>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  const int64_t nblk = (a.N + NW * P * 16 - 1) / (NW * P * 16);
  hipLaunchKernelGGL((assign_x_kernel<DPAD, P, OCC, MODE, NW, NBUF>), dim3((unsigned)nblk), dim3(NW * 64), lds, s, a);
  return hipGetLastError();
}

template <typename VS>
static void add_variants(int D, VS& vs) {
  if (D == 64) {
    vs.push_back({"x64_p8o3_m0", launch_x<64, 8, 3, 0>});
    vs.push_back({"x64_p8o3_prio", launch_x<64, 8, 3, 1024>});
    vs.push_back({"x64_p8o3_prio_ld", launch_x<64, 8, 3, 4096>});
    vs.push_back({"x64_p8o3_early_prio", launch_x<64, 8, 3, 1024 | 32>});
  }
  if (D == 128) {
    vs.push_back({"x_p4o4_m0", launch_x<128, 4, 4, 0>});
    vs.push_back({"x_p4o4_st", launch_x<128, 4, 4, 8>});
    vs.push_back({"x_p4o4_prio", launch_x<128, 4, 4, 1024>});
    vs.push_back({"x_p4o4_prio3", launch_x<128, 4, 4, 2048>});
    vs.push_back({"x_p4o4_prio_ld", launch_x<128, 4, 4, 4096>});

  }
  if (D == 256) {
    vs.push_back({"x256_p3o3_m0", launch_x<256, 3, 3, 0>});
    vs.push_back({"x256_p3o3_early", launch_x<256, 3, 3, 32>});
    vs.push_back({"x256_p3o3_prio", launch_x<256, 3, 3, 1024>});
    vs.push_back({"x256_p3o3_prio_ld", launch_x<256, 3, 3, 4096>});
  }
}

}  // namespace mkx
