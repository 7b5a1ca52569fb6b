// The production assign16_kernel as of HEAD, compiled in its own namespace: the
// baseline for A/B against the working-tree kernel.
#pragma once
namespace mkc {
using namespace mk;
// OCC: minimum waves per SIMD the register allocation must allow (launch bounds).
// FULLD: D == DPAD, so no fragment piece needs a column check.  The per-piece check costs
// 7 % at D=256 K=512 even when every piece passes it (profiles/r2_08_assign_clock_study.md).
template <typename T, int DPAD, int P, int CT_ = 0, int NBUF_ = 2, int OCC = 1, int NW_ = 4, bool FULLD = false>
__global__ __launch_bounds__(NW_ * 64, OCC) void old_kernel(AssignArgs a) {
  using C = mk::Assign16Cfg<T, DPAD, P, CT_, NBUF_, NW_>;
  constexpr bool EXACT = sizeof(T) == 4;  // f32: exact (value, index) epilogue
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
  for (int p = wid; p < cn_bytes / 1024; p += C::NW)
    blds16(rN, (MK_LDS void*)(cn_lds + p * 1024), loff, (uint32_t)p * 1024u);
  auto issue_chunk = [&](int c) {  // c: chunk index within this split (ring slot c % NBUF)
    const uint32_t src = (uint32_t)(c0 + c) * C::CHUNK_BYTES;
    char* dst = bufs + (c % C::NBUF) * C::CHUNK_BYTES;
#pragma unroll
    for (int i = 0; i < C::NPW; ++i) {
      const int pc = wid + i * C::NW;
      blds16(rC, (MK_LDS void*)(dst + pc * 1024), loff, src + (uint32_t)pc * 1024u);
    }
  };
  issue_chunk(0);

  const int64_t pbase = (int64_t)blockIdx.x * C::PTS + (int64_t)wid * (C::P * 16);
  u32x4 xr[C::P][C::NQ];
  float xnr[C::P];
#pragma unroll
  for (int p = 0; p < C::P; ++p) {
    int64_t row = pbase + p * 16 + r;
    row = row < a.N ? row : (a.N - 1);
    xnr[p] = (!EXACT && a.xn) ? a.xn[row] : 0.f;
    const T* rp = (const T*)a.X + row * a.ldx + g * (DPAD / 4);
#pragma unroll
    for (int q = 0; q < C::NQ; ++q) {
      const int col = g * (DPAD / 4) + q * C::V;
      if (FULLD || col < a.D) xr[p][q] = *(const u32x4*)(rp + q * C::V);
      else xr[p][q] = u32x4{0u, 0u, 0u, 0u};
    }
  }
  wait_vmcnt<0>();  // retire the fragments before the LDS-DMA loop (its vmcnt waits count chunks)
  if (C::NBUF == 3 && ncl > 1) issue_chunk(1);

  // bf16 seed offset (see the header): o = (1 + 2^-12) max |x|^2 over the workgroup's
  // points, from the caller's row norms when given (loaded with the fragments) or from
  // the fragments themselves, folded into this workgroup's LDS copy of |c|^2 once.
  float off = 0.f;
  if constexpr (!EXACT) {
    float m = 0.f;
    if (a.xn) {
#pragma unroll
      for (int p = 0; p < C::P; ++p) m = fmaxf(m, xnr[p]);
    } else {
#pragma unroll
      for (int p = 0; p < C::P; ++p) {
        float s = 0.f;
#pragma unroll
        for (int q = 0; q < C::NQ; ++q) s += sq16(xr[p][q], (T*)nullptr);
        s += __shfl_xor(s, 16, 64);
        s += __shfl_xor(s, 32, 64);
        m = fmaxf(m, s);
      }
    }
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    float* red = (float*)(bufs + C::NBUF * C::CHUNK_BYTES);
    if (lane == 0) red[wid] = m;
    __syncthreads();  // (every wave's cn / chunk-0 DMA has landed: vmcnt(0) above)
#pragma unroll
    for (int w = 0; w < C::NW; ++w) off = fmaxf(off, red[w]);
    off = __builtin_fmaf(off, 2.44140625e-04f, off);  // * (1 + 2^-12)
    off = __uint_as_float(__builtin_amdgcn_readfirstlane(__float_as_uint(off)));
    for (int k = threadIdx.x; k < a.Kpad; k += C::NW * 64) ((float*)cn_lds)[k] += off;
    // (published by the main loop's first wait_lgkm0 + barrier)
  }

  float best[C::P], seg_best[C::P];
  int bg[C::P];
#pragma unroll
  for (int p = 0; p < C::P; ++p) { best[p] = 3.0e38f; seg_best[p] = 3.0e38f; bg[p] = 0; }
  const int ngrp = nch * C::CT;   // one past the last tile (global tile numbering)
  const unsigned kmask = key6_mask();

  for (int c = 0; c < ncl; ++c) {
    // chunk c landed; with 3 slots chunk c+1 may stay in flight across the barrier
    if (C::NBUF == 3 && c + 1 < ncl) wait_vmcnt<C::NPW>(); else wait_vmcnt<0>();
    wait_lgkm0();
    raw_barrier();  // RAW for chunk c, WAR for the slot refilled next (read at c-1)
    if (c + C::NBUF - 1 < ncl) issue_chunk(c + C::NBUF - 1);
    const char* buf = bufs + (c % C::NBUF) * C::CHUNK_BYTES;
    // A fragments + |c|^2 of a tile from the LDS ring
    auto load_a = [&](int tl_i, u32x4* aw_, f32x4& ci_) {
      const int tile = (c0 + c) * C::CT + tl_i;
      ci_ = *(const f32x4*)(cn_lds + (tile * 16 + 4 * g) * 4);
      const char* tl = buf + tl_i * C::TILE_BYTES + lane * 16;
#pragma unroll
      for (int q = 0; q < C::NQ; ++q) aw_[q] = *(const u32x4*)(tl + q * 1024);
    };
#pragma unroll
    for (int tl_i = 0; tl_i < C::CT; ++tl_i) {
      const int tile = (c0 + c) * C::CT + tl_i;
      u32x4 aw[C::NQ];
      f32x4 ci;
      load_a(tl_i, aw, ci);
      f32x4 acc[C::P];
#pragma unroll
      for (int p = 0; p < C::P; ++p) acc[p] = ci;
#pragma unroll
      for (int q = 0; q < C::NQ; ++q) {
#pragma unroll
        for (int p = 0; p < C::P; ++p) acc[p] = mk::Mfma16<T>::run(aw[q], xr[p][q], acc[p]);
      }
      if constexpr (EXACT) {
        // (tile*4 + reg) as wave-uniform values: the index select needs no VALU add
        const int u = tile * 4;
#pragma unroll
        for (int p = 0; p < C::P; ++p) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const bool lt = acc[p][e] < best[p];
            best[p] = lt ? acc[p][e] : best[p];
            bg[p] = lt ? u + e : bg[p];
          }
        }
      } else {
        // 6-bit keys over a segment of 16 tiles (tile-in-segment * 4 + reg): 4 key packs
        // + 2 v_min3 per tile and point block; the running best is merged with its
        // segment id once per segment.  The four indices as opaque SGPRs, so each key is
        // one v_and_or_b32.
        const unsigned tis = (unsigned)(tile & 15) << 2;
        unsigned t0, t1, t2, t3;
        asm volatile("s_mov_b32 %0, %4\n\ts_or_b32 %1, %4, 1\n\ts_or_b32 %2, %4, 2\n\ts_or_b32 %3, %4, 3"
                     : "=s"(t0), "=s"(t1), "=s"(t2), "=s"(t3) : "s"(tis));
#pragma unroll
        for (int p = 0; p < C::P; ++p) {
          const f32x4& sv = acc[p];
          const float k0 = pack_key6(sv[0], kmask, t0), k1 = pack_key6(sv[1], kmask, t1);
          const float k2 = pack_key6(sv[2], kmask, t2), k3 = pack_key6(sv[3], kmask, t3);
          seg_best[p] = min3f(min3f(k0, k1, k2), k3, seg_best[p]);
        }
        if ((tile & 15) == 15 || tile == ngrp - 1) {
#pragma unroll
          for (int p = 0; p < C::P; ++p) {
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

  float inert = 0.f;
  int changed = 0;
#pragma unroll
  for (int p = 0; p < C::P; ++p) {
    int k;
    float v;
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
    // this point's seed offset (0 for f32)
    const float offp = off;
    if ((p & 3) == g) {
      const int64_t i = pbase + p * 16 + r;
      if (a.split_keys) {
        // compare the (positive) keys across splits; split_finish undoes the offset
        // (parked in mind[], which the caller provides whenever xn is given)
        if (i < a.N) {
          atomicMin(a.split_keys + i, split_key(v, k));
          if (a.mind) a.mind[i] = offp;
        }
      } else if (i < a.N) {
        v -= offp;   // back to |c|^2 - 2 x.c
        if (a.track_changed) changed += (a.labels[i] != k);
        a.labels[i] = k;
        if (a.xn) {
          const float d = fmaxf(a.xn[i] + v, 0.f);
          inert += d;
          if (a.mind) a.mind[i] = d;
        }
      }
    }
  }
  if (a.slots && !a.split_keys) {
    double di = wave_sum((double)inert);
    int dc = wave_sum(changed);
    double* red = (double*)(bufs + C::NBUF * C::CHUNK_BYTES);
    if (lane == 0) { red[2 * wid] = di; red[2 * wid + 1] = (double)dc; }
    __syncthreads();
    if (threadIdx.x == 0) {
      double si = 0, sc = 0;
#pragma unroll
      for (int w = 0; w < C::NW; ++w) { si += red[2 * w]; sc += red[2 * w + 1]; }
      double* slot = a.slots + (blockIdx.x % NSLOT) * SLOT_STRIDE;
      atomicAdd(slot + 0, si);
      atomicAdd(slot + 1, sc);
    }
  }
}


template <int DPAD, int P, int CT, int OCC>
static hipError_t launch_old(const AssignArgs& a, hipStream_t s) {
  using C = mk::Assign16Cfg<uint16_t, DPAD, P, CT, 2, 4>;
  const int cn_bytes = ((a.Kpad * 4 + 1023) / 1024) * 1024;
  const size_t lds = cn_bytes + C::NBUF * C::CHUNK_BYTES + 16 * C::NW;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)old_kernel<uint16_t, DPAD, P, CT, 2, OCC, 4, true>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  const int64_t nblk = (a.N + C::PTS - 1) / C::PTS;
  AssignArgs b = a; b.split_keys = nullptr;
  hipLaunchKernelGGL((old_kernel<uint16_t, DPAD, P, CT, 2, OCC, 4, true>), dim3((unsigned)nblk, 1), dim3(256), lds, s, b);
  return hipGetLastError();
}
}  // namespace mkc
