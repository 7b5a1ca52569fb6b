// mikmeans — K2 variant: assignment on 16x16 MFMA tiles (v_mfma_f32_16x16x32_bf16 /
// v_mfma_f32_16x16x4_f32) for gfx950.
//
// Same algorithm and pipeline as assign.hip (fragment-packed centroid chunks in a
// 3-slot LDS ring fed by LDS-DMA, |c|^2 seeding the accumulators, packed-index
// v_min3 argmin), re-tiled for the 16x16 matrix-core shape:
//  * lane (r = l&15, g = l>>4) holds the B fragment of point p0+r, feature
//    quarter g: x[p0+r][g*DPAD/4 .. +DPAD/4) (contiguous), and the A fragment of
//    centroid r of the tile, same quarter;
//  * output D[row = 4g+reg][col = r]: each lane holds 4 centroid scores of its
//    point per tile; GT consecutive tiles are reduced together (4-bit index =
//    tile-in-group * 4 + reg), the 4 lane groups g merge once at the end.
// On MI355X the chip holds a higher clock on the 16x16 shape under load
// (MI355X_MICROARCH.md, DVFS give-back item 7), which is why this variant exists;
// scripts/ab_kernels.py picks the faster one per shape.
//
// Layout "16" of the packed centroids (csrc/kernels.h describes layout "32"):
//   element (k, d): t = k/16, r = k%16, g = d / (DPAD/4), e = d % (DPAD/4)
//   offset = ((t*NQ + e/V)*64 + r + 16*g)*V + e%V,  NQ = DPAD/(4V)
#include "common.h"
#include "kernels.h"

namespace mk {

constexpr int chunk_tiles16(int esize, int dpad) {
  return (16 * dpad * esize) >= 16384 ? 1 : 16384 / (16 * dpad * esize);
}

// CT_: tiles per LDS chunk (0 = the 16 KiB default, which also fixes Kpad's
// granule); NBUF_: ring slots (prefetch depth NBUF-1).
template <typename T, int DPAD, int P_, int GT_, int CT_ = 0, int NBUF_ = 3, int NW_ = 4>
struct Assign16Cfg {
  static constexpr int NW = NW_;                // waves per workgroup sharing the ring
  static constexpr int P = P_;                  // 16-point blocks per wave
  static constexpr int GT = GT_;                // tiles reduced per epilogue
  static constexpr int V = Elem<T>::V;
  static constexpr int NQ = DPAD / 4 / V;       // 16-B pieces per lane per point
  static constexpr int TILE_BYTES = NQ * 1024;  // 16 centroids x DPAD
  static constexpr int CT = CT_ ? CT_ : chunk_tiles16(sizeof(T), DPAD);
  static constexpr int CHUNK_BYTES = CT * TILE_BYTES;
  static constexpr int PIECES = CHUNK_BYTES / 1024;
  static constexpr int NPW = PIECES / NW;
  static constexpr int PTS = NW * P * 16;
  static constexpr int NBUF = NBUF_;
  static_assert(NBUF == 2 || NBUF == 3, "ring depth");
  static_assert(chunk_tiles16(sizeof(T), DPAD) % CT == 0, "chunk must divide the Kpad granule");
  static_assert(NQ >= 1, "DPAD too small for the 16x16 layout");
  static_assert(CT % GT == 0, "tile group must divide the chunk");
  static_assert(GT * 4 <= 16, "4-bit packed index");
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

// DBG bit flags (diagnostic builds for A/B; 4, 16 and 32 are pipeline options; 16 = at
// least 4 waves per SIMD, i.e. <= 128 VGPRs; 32 = at least 3, <= 168): 1 = epilogue replaced by
// one add per tile (MFMA + LDS pipeline alone), 2 = no ring refills / waits (MFMA +
// epilogue alone on whatever the LDS holds).
template <typename T, int DPAD, int P, int GT, int CT_ = 0, int NBUF_ = 3, int DBG = 0, int NW_ = 4>
__global__ __launch_bounds__(NW_ * 64, (DBG & 16) ? 4 : ((DBG & 32) ? 3 : 1)) void assign16_kernel(AssignArgs a) {
  using C = Assign16Cfg<T, DPAD, P, GT, CT_, NBUF_, NW_>;
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
  const char* gC = (const char*)a.Cpack + (int64_t)c0 * C::CHUNK_BYTES;

  for (int p = wid; p < cn_bytes / 1024; p += C::NW)
    glds16((const char*)a.cn + p * 1024 + lane * 16, (MK_LDS void*)(cn_lds + p * 1024));
  auto issue_chunk = [&](int c) {  // c: chunk index within this split (ring slot c % NBUF)
    const char* src = gC + (int64_t)c * C::CHUNK_BYTES + lane * 16;
    char* dst = bufs + (c % C::NBUF) * C::CHUNK_BYTES;
#pragma unroll
    for (int i = 0; i < C::NPW; ++i) {
      const int pc = wid + i * C::NW;
      glds16(src + pc * 1024, (MK_LDS void*)(dst + pc * 1024));
    }
  };
  issue_chunk(0);

  const int64_t pbase = (int64_t)blockIdx.x * C::PTS + (int64_t)wid * (C::P * 16);
  u32x4 xr[C::P][C::NQ];
#pragma unroll
  for (int p = 0; p < C::P; ++p) {
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
  wait_vmcnt<0>();  // see assign.hip: retire the fragments before the LDS-DMA loop
  if (C::NBUF == 3 && ncl > 1) issue_chunk(1);

  float best[C::P], seg_best[C::P];
  int bg[C::P];
#pragma unroll
  for (int p = 0; p < C::P; ++p) { best[p] = 3.0e38f; seg_best[p] = 3.0e38f; bg[p] = 0; }
  const int last_grp = nch * (C::CT / GT) - 1;
  const unsigned kmask = key6_mask();

  float dbg_sink = 0.f;
  if constexpr ((DBG & 2) != 0) { wait_vmcnt<0>(); raw_barrier(); }
  for (int c = 0; c < ncl; ++c) {
    if constexpr ((DBG & 2) == 0) {
      // chunk c landed; with 3 slots chunk c+1 may stay in flight across the barrier
      if (C::NBUF == 3 && c + 1 < ncl) wait_vmcnt<C::NPW>(); else wait_vmcnt<0>();
      wait_lgkm0();
      raw_barrier();  // RAW for chunk c, WAR for the slot refilled next (read at c-1)
      if (c + C::NBUF - 1 < ncl) issue_chunk(c + C::NBUF - 1);
    }
    const char* buf = bufs + (c % C::NBUF) * C::CHUNK_BYTES;
    // DBG & 64 / 128: LLVM's MFMA/DS interleaving strategies for the chunk body (A/B)
    if constexpr ((DBG & 64) != 0) __builtin_amdgcn_iglp_opt(0);
    if constexpr ((DBG & 128) != 0) __builtin_amdgcn_iglp_opt(1);
    // A fragments + |c|^2 of one tile from the LDS ring
    auto load_tile = [&](int tl_i, u32x4* aw_, f32x4& ci_) {
      const int tile = (c0 + c) * C::CT + tl_i;
      ci_ = *(const f32x4*)(cn_lds + (tile * 16 + 4 * g) * 4);
      const char* tl = buf + tl_i * C::TILE_BYTES + lane * 16;
#pragma unroll
      for (int q = 0; q < C::NQ; ++q) aw_[q] = *(const u32x4*)(tl + q * 1024);
    };
    // DBG & 4: prefetch the next tile's fragments before this tile's MFMAs (GT == 1)
    u32x4 awn[C::NQ];
    f32x4 cin;
    if constexpr ((DBG & 4) != 0 && GT == 1) load_tile(0, awn, cin);
#pragma unroll
    for (int tg = 0; tg < C::CT / GT; ++tg) {
      f32x4 acc[C::P][GT];
#pragma unroll
      for (int t = 0; t < GT; ++t) {
        const int tl_i = tg * GT + t;
        u32x4 aw[C::NQ];
        f32x4 ci;
        if constexpr ((DBG & 4) != 0 && GT == 1) {
#pragma unroll
          for (int q = 0; q < C::NQ; ++q) aw[q] = awn[q];
          ci = cin;
          if (tl_i + 1 < C::CT) load_tile(tl_i + 1, awn, cin);
        } else {
          load_tile(tl_i, aw, ci);
        }
#pragma unroll
        for (int q = 0; q < C::NQ; ++q) {
#pragma unroll
          for (int p = 0; p < C::P; ++p)
            acc[p][t] = Mfma16<T>::run(aw[q], xr[p][q], q == 0 ? ci : acc[p][t]);
        }
      }
      const int grp = (c0 + c) * (C::CT / GT) + tg;
      if constexpr ((DBG & 1) != 0) {
#pragma unroll
        for (int p = 0; p < C::P; ++p) dbg_sink += acc[p][0][0];
        continue;
      }
      if constexpr (GT == 1) {
        // 6-bit keys over a segment of 16 tiles (tile-in-segment * 4 + reg): 4 key
        // packs + 2 v_min3 per tile and point block; the running best is merged
        // with its segment id once per segment.
        // the four indices as opaque SGPRs, so each key is one v_and_or_b32
        const unsigned tis = (unsigned)(grp & 15) << 2;
        unsigned t0, t1, t2, t3;
        asm volatile("s_mov_b32 %0, %4\n\ts_or_b32 %1, %4, 1\n\ts_or_b32 %2, %4, 2\n\ts_or_b32 %3, %4, 3"
                     : "=s"(t0), "=s"(t1), "=s"(t2), "=s"(t3) : "s"(tis));
#pragma unroll
        for (int p = 0; p < C::P; ++p) {
          const f32x4& sv = acc[p][0];
          const float k0 = pack_key6(sv[0], kmask, t0), k1 = pack_key6(sv[1], kmask, t1);
          const float k2 = pack_key6(sv[2], kmask, t2), k3 = pack_key6(sv[3], kmask, t3);
          if constexpr ((DBG & 8) != 0) {
            seg_best[p] = min3f_v(min3f_v(k0, k1, k2), k3, seg_best[p]);
          } else {
            seg_best[p] = min3f(min3f(k0, k1, k2), k3, seg_best[p]);
          }
        }
        if ((grp & 15) == 15 || grp == last_grp) {
#pragma unroll
          for (int p = 0; p < C::P; ++p) {
            // compare values only: on equal (truncated) values the earlier segment keeps
            // the lower centroid index
            const float sv = __uint_as_float(__float_as_uint(seg_best[p]) & ~63u);
            const float bv = __uint_as_float(__float_as_uint(best[p]) & ~63u);
            if (sv < bv) { best[p] = seg_best[p]; bg[p] = grp >> 4; }
            seg_best[p] = 3.0e38f;
          }
        }
        continue;
      }
#pragma unroll
      for (int p = 0; p < C::P; ++p) {
        float m;
        if constexpr (GT == 2) {
          const f32x4& s0 = acc[p][0];
          const f32x4& s1 = acc[p][1];
          const float m0 = min3f(pack_key(s0[0], 0), pack_key(s0[1], 1), pack_key(s0[2], 2));
          const float m1 = min3f(pack_key(s0[3], 3), pack_key(s1[0], 4), pack_key(s1[1], 5));
          m = min3f(min3f(m0, m1, pack_key(s1[2], 6)), pack_key(s1[3], 7), pack_key(s1[3], 7));
        } else {
          float k[16];
#pragma unroll
          for (int t = 0; t < GT; ++t)
#pragma unroll
            for (int e = 0; e < 4; ++e) k[4 * t + e] = pack_key(acc[p][t][e], 4 * t + e);
          const float m0 = min3f(k[0], k[1], k[2]), m1 = min3f(k[3], k[4], k[5]);
          const float m2 = min3f(k[6], k[7], k[8]), m3 = min3f(k[9], k[10], k[11]);
          const float m4 = min3f(k[12], k[13], k[14]);
          m = min3f(min3f(m0, m1, m2), min3f(m3, m4, k[15]), min3f(m3, m4, k[15]));
        }
        if (m < best[p]) { best[p] = m; bg[p] = grp; }
      }
    }
  }

  if constexpr ((DBG & 1) != 0) best[0] = fminf(best[0], dbg_sink);
  float inert = 0.f;
  int changed = 0;
#pragma unroll
  for (int p = 0; p < C::P; ++p) {
    const unsigned bits = __float_as_uint(best[p]);
    int k;
    float v;
    if constexpr (GT == 1) {  // bg = segment of 16 tiles, 6-bit key
      const int idx = (int)(bits & 63u);
      k = (bg[p] * 16 + (idx >> 2)) * 16 + 4 * g + (idx & 3);
      v = __uint_as_float(bits & ~63u);
    } else {
      const int idx = (int)(bits & 15u);
      k = (bg[p] * GT + (idx >> 2)) * 16 + 4 * g + (idx & 3);
      v = __uint_as_float(bits & ~15u);
    }
#pragma unroll
    for (int o = 16; o <= 32; o <<= 1) {
      const float vo = __shfl_xor(v, o, 64);
      const int ko = __shfl_xor(k, o, 64);
      if (vo < v || (vo == v && ko < k)) { v = vo; k = ko; }
    }
    if ((p & 3) == g) {
      const int64_t i = pbase + p * 16 + r;
      if (a.split_keys) {
        if (i < a.N) atomicMin(a.split_keys + i, split_key(v, k));
      } else if (i < a.N) {
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
    const float v = split_value(key);
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
    if (threadIdx.x == 0) {
      double* slot = a.slots + (blockIdx.x % NSLOT) * SLOT_STRIDE;
      atomicAdd(slot + 0, red[0] + red[2] + red[4] + red[6]);
      atomicAdd(slot + 1, red[1] + red[3] + red[5] + red[7]);
    }
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

template <typename T, int DPAD, int P, int GT, int CT_ = 0, int NBUF_ = 3, int DBG = 0, int NW_ = 4>
static hipError_t launch16_t(const AssignArgs& a, hipStream_t s) {
  using C = Assign16Cfg<T, DPAD, P, GT, CT_, NBUF_, NW_>;
  if (a.Kpad % (16 * C::CT) != 0) return hipErrorInvalidValue;
  const int cn_bytes = ((a.Kpad * 4 + 1023) / 1024) * 1024;
  const size_t lds = cn_bytes + C::NBUF * C::CHUNK_BYTES + 16 * C::NW;
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)assign16_kernel<T, DPAD, P, GT, CT_, NBUF_, DBG, NW_>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  const int64_t nblk = (a.N + C::PTS - 1) / C::PTS;
  if (nblk <= 0) return hipSuccess;
  const int splits = a.split_keys ? assign16_splits(nblk, a.Kpad / (16 * C::CT)) : 1;
  AssignArgs b = a;
  if (splits == 1) b.split_keys = nullptr;
  hipLaunchKernelGGL((assign16_kernel<T, DPAD, P, GT, CT_, NBUF_, DBG, NW_>),
                     dim3((unsigned)nblk, (unsigned)splits), dim3(C::NW * 64), lds, s, b);
  if (splits > 1)
    hipLaunchKernelGGL(split_finish_kernel, dim3((unsigned)((a.N + 255) / 256)), dim3(256), 0, s, b);
  return hipGetLastError();
}

static int g_assign16_gt = 0;
static int g_assign16_cfg = 0;  // tuned-shape pipeline variant (A/B), 0 = default
void set_assign16_gt(int gt) { g_assign16_gt = gt; }
void set_assign16_cfg(int v) { g_assign16_cfg = v; }

template <typename T, int DPAD>
static hipError_t launch16_d(const AssignArgs& a, hipStream_t s) {
  constexpr int CT = chunk_tiles16(sizeof(T), DPAD);
  constexpr int NQ = DPAD / 4 / Elem<T>::V;
  constexpr int P = NQ >= 8 ? 2 : 4;  // keep the point fragments within ~64-128 VGPRs
#ifdef MK_AB_VARIANTS
  // Diagnostic / A-B builds only (MIKMEANS_AB=1 python -m mikmeans._build): every
  // variant below was measured against the default (profiles/r1_08_*, r1_16_*, r1_17_*).
  if constexpr (sizeof(T) == 2 && DPAD == 128) {
    // pipeline variants of the headline shape (occupancy vs barrier frequency):
    //   1: GT1, 16 KiB chunks, 2 slots (36 KiB LDS at K=1024 -> 4 WGs/CU at <=128 VGPRs)
    //   2: GT1,  8 KiB chunks, 3 slots (28 KiB)     3: GT2, 16 KiB chunks, 2 slots
    //   4: GT2,  8 KiB chunks, 3 slots
    switch (g_assign16_cfg) {
      case 1: return launch16_t<T, DPAD, P, 1, 4, 2>(a, s);
      case 2: return launch16_t<T, DPAD, P, 1, 2, 3>(a, s);
      case 3: return launch16_t<T, DPAD, P, 2, 4, 2>(a, s);
      case 4: return launch16_t<T, DPAD, P, 2, 2, 3>(a, s);
      case 10: return launch16_t<T, DPAD, P, 1, 2, 3, 1>(a, s);   // diagnostics of the default
      case 11: return launch16_t<T, DPAD, P, 1, 2, 3, 2>(a, s);
      case 12: return launch16_t<T, DPAD, 8, 1, 2, 3>(a, s);      // 8 point-blocks per wave
      case 13: return launch16_t<T, DPAD, 2, 1, 2, 3>(a, s);      // 2 point-blocks per wave
      case 14: return launch16_t<T, DPAD, P, 1, 2, 3, 8>(a, s);   // volatile min3 (sched barrier)
      case 15: return launch16_t<T, DPAD, P, 1, 4, 2, 8>(a, s);
      case 16: return launch16_t<T, DPAD, P, 1, 4, 2>(a, s);
      case 17: return launch16_t<T, DPAD, P, 1, 4, 3>(a, s);
      case 18: return launch16_t<T, DPAD, P, 1, 1, 3>(a, s);
      case 19: return launch16_t<T, DPAD, P, 1, 1, 2>(a, s);
      case 20: return launch16_t<T, DPAD, P, 1, 4, 3, 8>(a, s);
      case 23: return launch16_t<T, DPAD, P, 1, 4, 2, 3>(a, s);   // no epilogue, no ring
      case 24: return launch16_t<T, DPAD, P, 1, 4, 2, 4>(a, s);   // A prefetch
      case 25: return launch16_t<T, DPAD, P, 1, 4, 2, 5>(a, s);   // A prefetch, no epilogue
      case 26: return launch16_t<T, DPAD, P, 1, 4, 2, 1>(a, s);   // no epilogue
      case 27: return launch16_t<T, DPAD, P, 1, 4, 2, 2>(a, s);   // no ring
      case 29: return launch16_t<T, DPAD, P, 1, 4, 2, 16>(a, s);  // <= 128 VGPRs (4 waves/SIMD)
      case 30: return launch16_t<T, DPAD, P, 1, 2, 3, 16>(a, s);
      case 31: return launch16_t<T, DPAD, P, 1, 4, 3, 16>(a, s);
      case 32: return launch16_t<T, DPAD, P, 1, 4, 2, 16, 8>(a, s);  // 8 waves share the ring
      case 33: return launch16_t<T, DPAD, P, 1, 4, 3, 16, 8>(a, s);
      case 34: return launch16_t<T, DPAD, P, 1, 2, 3, 16, 8>(a, s);
      case 35: return launch16_t<T, DPAD, P, 1, 2, 2, 16, 2>(a, s);  // 2 waves per ring
      case 40: return launch16_t<T, DPAD, P, 1, 4, 2, 16, 16>(a, s);  // 16 waves share the ring
      case 41: return launch16_t<T, DPAD, P, 1, 4, 3, 16, 16>(a, s);
      case 50: return launch16_t<T, DPAD, 6, 1, 4, 2, 32>(a, s);  // 6 point blocks, 3 waves/SIMD
      case 51: return launch16_t<T, DPAD, 5, 1, 4, 2, 32>(a, s);
      case 52: return launch16_t<T, DPAD, 6, 1, 4, 3, 32>(a, s);
      case 53: return launch16_t<T, DPAD, 6, 1, 2, 3, 32>(a, s);
      case 36: return launch16_t<T, DPAD, P, 1, 2, 3, 16, 2>(a, s);
      case 37: return launch16_t<T, DPAD, P, 1, 1, 3, 16, 4>(a, s);  // 4 KiB chunks
      case 38: return launch16_t<T, DPAD, P, 1, 4, 2, 16 | 64>(a, s);   // iglp_opt(0)
      case 39: return launch16_t<T, DPAD, P, 1, 4, 2, 16 | 128>(a, s);  // iglp_opt(1)
      case 21: return launch16_t<T, DPAD, 2, 1, 4, 2>(a, s);
      case 22: return launch16_t<T, DPAD, 8, 1, 4, 2>(a, s);
      case 63: return launch16_t<T, DPAD, P, 1, 4, 2, 4 | 32>(a, s);  // A prefetch at 3 waves/SIMD
      case 64: return launch16_t<T, DPAD, P, 1, 4, 3, 4 | 32>(a, s);
      case 65: return launch16_t<T, DPAD, 5, 1, 4, 2, 4 | 32>(a, s);
      case 66: return launch16_t<T, DPAD, 3, 1, 4, 2, 4 | 16>(a, s);  // P=3 + prefetch at 4 waves/SIMD
      case 67: return launch16_t<T, DPAD, P, 1, 2, 3, 4 | 32>(a, s);
      default: break;
    }
  }
  if constexpr (sizeof(T) == 2 && DPAD == 256) {  // cfg5 shape (P=2 default, 8 KiB tiles)
    switch (g_assign16_cfg) {
      case 70: return launch16_t<T, DPAD, 3, 1, 2, 2, 32>(a, s);  // 3 point blocks, 3 waves/SIMD
      case 71: return launch16_t<T, DPAD, 4, 1, 2, 2>(a, s);      // 4 point blocks, 2 waves/SIMD
      case 72: return launch16_t<T, DPAD, 3, 1, 1, 3, 32>(a, s);
      case 73: return launch16_t<T, DPAD, 2, 1, 1, 3, 16>(a, s);
      case 74: return launch16_t<T, DPAD, 4, 1, 1, 3>(a, s);
      default: break;
    }
  }
#else
  if (g_assign16_cfg != 0) return hipErrorNotSupported;  // variant knob needs an A/B build
#endif
  // gt knob: 0/1 = the GT1 default below, 2/4 = GT2/GT4.  GT1 is the fastest on every
  // BASELINE shape when timed on the bench's own data and centres (scripts/ab_shapes.py,
  // profiles/r1_16_assign_shapes.md); on random centres GT2 can look faster.
  if (g_assign16_gt <= 1) {
    // Default: 1-tile epilogue with segmented 6-bit keys (1.5 VALU per score), 16 KiB
    // chunks in a 2-slot ring.  A/B on MI355X at N=2e7 D=128 K=1024 bf16 (scripts/
    // ab_kernels.py, one process, interleaved rounds): 1279-1317 TF/s vs 1218-1265 for
    // 4/8 KiB chunks with 3 slots, 1099 / 1250 for 2 / 8 point blocks per wave.
    // bf16: at most 128 VGPRs (4 waves per SIMD; <= 5 spilled registers): +2.5 % at the
    // headline shape (1339 vs 1306 TF/s).  f32 would spill heavily under that bound.
    constexpr int WB = sizeof(T) == 2 ? 16 : 0;
    return launch16_t<T, DPAD, P, 1, CT, 2, WB>(a, s);
  }
  const int want = g_assign16_gt;  // >= 2
  if (want >= 4 && CT % 4 == 0) return launch16_t<T, DPAD, P, (CT % 4 == 0 ? 4 : 1)>(a, s);
  if (want >= 2 && CT % 2 == 0) return launch16_t<T, DPAD, P, (CT % 2 == 0 ? 2 : 1)>(a, s);
  return launch16_t<T, DPAD, P, 1>(a, s);
}

int assign16_chunk_tiles(int dtype, int dpad) {
  const bool ok = dtype == DT_BF16 ? (dpad == 32 || dpad == 64 || dpad == 128 || dpad == 256)
                                   : (dpad == 16 || dpad == 32 || dpad == 64 || dpad == 128 || dpad == 256);
  return ok ? chunk_tiles16(dtype == DT_BF16 ? 2 : 4, dpad) : 0;
}

hipError_t launch_assign16(int dtype, int dpad, const AssignArgs& a, hipStream_t s) {
  if (dtype == DT_BF16) {
    switch (dpad) {
      case 32: return launch16_d<uint16_t, 32>(a, s);
      case 64: return launch16_d<uint16_t, 64>(a, s);
      case 128: return launch16_d<uint16_t, 128>(a, s);
      case 256: return launch16_d<uint16_t, 256>(a, s);
    }
  } else {
    switch (dpad) {
      case 16: return launch16_d<float, 16>(a, s);
      case 32: return launch16_d<float, 32>(a, s);
      case 64: return launch16_d<float, 64>(a, s);
      case 128: return launch16_d<float, 128>(a, s);
      case 256: return launch16_d<float, 256>(a, s);
    }
  }
  return hipErrorInvalidValue;
}

}  // namespace mk
