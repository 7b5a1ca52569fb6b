// mikmeans — host-side launch planning shared by the kernels and the sanitizer harness.
//
// Everything that turns (K, D, N, dtype) into launch geometry and buffer sizes lives
// here as plain C++ (no HIP types), so tests/native/plan_fuzz.cpp can build it with
// g++ -fsanitize=address,undefined and sweep it on the CPU: the
// M-step's LDS footprint and slice width, its chunk count, the fixed-point exponent
// and the assign kernel's padded K.
#pragma once
#include <math.h>
#include <stddef.h>
#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define MK_HD __host__ __device__
#else
#define MK_HD
#endif

namespace mk {
namespace plan {

constexpr size_t UPD_LDS_MAX = 160 * 1024;  // one LDS-filling M-step workgroup per CU
constexpr int FX_BITS = 20;                 // |q| <= 2^20 per fixed-point contribution

// M-step LDS: cells [K+1][ldc] u64 | add counts [K+1] u32 | flag, nhot | weighted counts
// [K+1] i64 (weighted / incremental) | hot-label list [K+1] u16.
MK_HD inline size_t upd_lds_bytes(int K, int ldc, bool weighted) {
  size_t b = (size_t)(K + 1) * (size_t)ldc * 8 + (size_t)(K + 1) * 4 + 8;
  b = (b + 7) & ~(size_t)7;
  b += weighted ? (size_t)(K + 1) * 8 : 0;
  return b + ((size_t)(K + 1) * 2 + 7) / 8 * 8;
}

// Columns per M-step workgroup (0 = global-atomic fallback) and the LDS cell stride:
// the widest power-of-two slice <= 64 (and <= max_sw when nonzero) that fits, odd
// stride preferred (sw/2 + 1), else unpadded (sw/2, XOR-swizzled in the kernel).
inline int choose_sw(int esize, int K, int D, bool weighted, int max_sw, int* ldc) {
  if (K < 1 || D < 1 || (D * esize) % 4 || D % 2) return 0;
  int dp = 2;
  while (dp < D) dp *= 2;
  for (int sw = 64; sw >= 2; sw /= 2) {
    if (sw > dp) continue;
    if (max_sw && sw > max_sw) continue;
    if (upd_lds_bytes(K, sw / 2 + 1, weighted) <= UPD_LDS_MAX) { *ldc = sw / 2 + 1; return sw; }
    if (upd_lds_bytes(K, sw / 2, weighted) <= UPD_LDS_MAX) { *ldc = sw / 2; return sw; }
  }
  return 0;
}

// Row chunks of the M-step (a multiple of 8: blocks b and b+8 share an XCD): one wave of
// the 256 CUs over (chunk, slice) workgroups, fewer for tiny N.
inline int update_n_chunks(int sw, int D, int64_t N) {
  if (sw == 0) return 1;
  const int n_slices = (D + sw - 1) / sw;
  int nc = (256 + n_slices - 1) / n_slices;
  nc = ((nc + 7) / 8) * 8;
  const int64_t rows = (N + nc - 1) / nc;
  if (rows < 256) {
    const int64_t c = (N + 255) / 256;
    nc = (int)((c + 7) / 8 * 8);
    if (nc < 8) nc = 8;
  }
  return nc;
}

// Largest e with maxabs * 2^e <= 2^FX_BITS, kept in [-126, 126] (2^e a normal float);
// 0 for a zero, negative or non-finite bound.
inline int fixed_exp(double maxabs) {
  if (!(maxabs > 0) || !isfinite(maxabs)) return 0;
  const double l = ceil(log2(maxabs));
  if (l > 200) return -126;
  if (l < -200) return 126;
  int e = FX_BITS - (int)l;
  while (e > -1000 && ldexp(maxabs, e) > ldexp(1.0, FX_BITS)) --e;  // guard rounding of log2
  if (e > 126) e = 126;
  if (e < -126) e = -126;
  return e;
}

// K-split M-step (plain full passes: unweighted, not incremental, not the residual pass).
// KS workgroups share a row chunk; workgroup j owns labels [j*kq, (j+1)*kq) and every
// column, and takes whole rows (LPR lanes x 16 B), so each wave-instruction reads full
// 128-B lines instead of the column-slice kernel's 64-B row pieces.
struct KsPlan {
  int ks;   // workgroups per row chunk (power of two)
  int kq;   // labels per workgroup
  int lpr;  // lanes per row (power of two <= 64): 16-B pieces of a (column-padded) row
  int ldc;  // u64 cells per label (2 columns each, + 1 for an odd bank stride)
  int gm;   // row groups of loads kept in flight per wave and period
};
constexpr int KS_NT = 1024;                         // threads per workgroup
constexpr size_t KS_LIST_BYTES = 2 * (KS_NT / 64) * 64 * 4;  // per-wave match lists, 2 periods
constexpr size_t KS_GLIST_BYTES = 2 * (KS_NT / 64) * 64 * 8 + 8;  // gathered batches: their X rows (+ 8-B alignment)
MK_HD inline size_t ks_lds_bytes(int kq, int ldc) {
  return (size_t)kq * (size_t)ldc * 8 + (size_t)kq * 4 + 16 + KS_LIST_BYTES;
}
inline bool choose_ks(int esize, int K, int D, KsPlan* p) {
  if (K < 2 || D < 2 || D % 2 || (D * esize) % 4) return false;
  const int v = 16 / esize;
  int lpr = 1;
  while (lpr * v < D) lpr *= 2;
  if (lpr > 64 || lpr < 8) return false;            // rows past 1 KiB, or rows of 64 B or less
  const int ldc = lpr * v / 2 + 1;
  // prefer ~4 row groups of matches per wave and period (LPR / KS of them on average)
  int ks = lpr / 4 > 1 ? lpr / 4 : 1;
  while (ks > K) ks /= 2;                            // no workgroup without labels
  for (;;) {
    const int kq = (K + ks - 1) / ks;
    if (ks_lds_bytes(kq, ldc) <= UPD_LDS_MAX) {
      if (ks < 2) return false;                      // one workgroup would scan every row alone
      p->ks = ks; p->kq = kq; p->lpr = lpr; p->ldc = ldc;
      // row groups in flight: the owned rows of a wave's 64 (mean m = 64/ks) plus 2.5
      // standard deviations, in groups of 64/lpr rows; too few sends rows to the
      // synchronous overflow path, too many issues masked loads (headline 6, cfg4 2:
      // profiles/r2_05_update_study.md)
      const double m = 64.0 / ks;
      const int g = (int)ceil((m + 2.5 * sqrt(m)) / (64.0 / lpr));
      // (g = 4 takes 3 groups: 3 beat 6 at D=64 K=2048 by 11 %, D=128 K=2048 by 4 % and
      // D=384 / 512 K=4096 by 13 %; 6 stays ahead from g = 5, profiles/r6_55_*, r6_56_*, r6_57_*)
      p->gm = g <= 2 ? 2 : g <= 4 ? 3 : 6;
      return true;
    }
    if (ks >= 64) return false;
    ks *= 2;
  }
}
// Row chunks for the K-split grid: at least the column-slice kernel's count for the same
// shape (so both kernels fill the chip with one slab layout), a multiple of 8.
inline int update_n_chunks_ks(int ks, int nc_slice) {
  int nc = (256 + ks - 1) / ks;
  nc = ((nc + 7) / 8) * 8;
  return nc > nc_slice ? nc : nc_slice;
}

// Assign kernel: centroid tiles (16 centroids) per 16 KiB LDS chunk (one tile per chunk for
// rows of 16 KiB tiles and wider), 0 = unsupported width.  Padded widths: powers of two up
// to 256, then 384, 512, 768, 1024 (the wide-row kernels).
constexpr int chunk_tiles16(int esize, int dpad) {
  return (16 * dpad * esize) >= 16384 ? 1 : 16384 / (16 * dpad * esize);
}
inline int assign_dpad(int esize, int D) {
  int d = 4 * (16 / esize);
  while (d < D && d < 256) d *= 2;
  if (D <= d) return d;
  for (int w : {384, 512, 768, 1024})
    if (D <= w) return w;
  return 0;
}
inline int assign16_chunk_tiles(int esize, int dpad) {
  const bool ok = dpad >= 4 * (16 / esize) && assign_dpad(esize, dpad) == dpad;
  return ok ? chunk_tiles16(esize, dpad) : 0;
}
// K rounded up to a whole chunk (0 = unsupported width or K out of range).
inline int assign_kpad(int esize, int dpad, int K) {
  const int ct = assign16_chunk_tiles(esize, dpad);
  if (ct <= 0 || K < 1 || K > (1 << 24)) return 0;
  const int m = 16 * ct;
  return ((K + m - 1) / m) * m;
}
inline int assign_cn_len(int kpad) { return ((kpad + 255) / 256) * 256; }

}  // namespace plan
}  // namespace mk
