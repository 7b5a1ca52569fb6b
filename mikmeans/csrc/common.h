// mikmeans — shared device helpers for the CDNA4 (gfx950 / MI355X) kernels.
//
// Everything here is written for 64-lane wavefronts, the 32x32 MFMA C/D layout
// (col = lane&31, row = (reg&3) + 8*(reg>>2) + 4*(lane>>5)) and LDS-DMA
// (`global_load_lds_dwordx4`).  No CUDA shims, no dual paths.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mk {

typedef short short8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int WAVE = 64;
// Score given to padded (non-existent) centroids: finite so that the packed
// argmin key stays a valid float, large enough never to win.
constexpr float PAD_SCORE = 1.0e30f;

#define MK_LDS __attribute__((address_space(3)))

// ---------------------------------------------------------------------------
// bf16 <-> f32 (raw uint16 storage; RNE rounding, NaN stays NaN)
__device__ __forceinline__ float bf16_to_f32(uint16_t h) {
  return __uint_as_float(((uint32_t)h) << 16);
}
__device__ __forceinline__ float bf16lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bf16hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }
__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);  // quiet NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
__device__ __forceinline__ float round_bf16(float f) { return bf16_to_f32(f32_to_bf16(f)); }

// ---------------------------------------------------------------------------
// Element traits: storage type, elements per 16-byte piece.
template <typename T> struct Elem;
template <> struct Elem<uint16_t> {  // bf16
  static constexpr int V = 8;
  __device__ static float to_f32(uint16_t v) { return bf16_to_f32(v); }
  __device__ static uint16_t from_f32(float f) { return f32_to_bf16(f); }
};
template <> struct Elem<float> {
  static constexpr int V = 4;
  __device__ static float to_f32(float v) { return v; }
  __device__ static float from_f32(float f) { return f; }
};

// Unpack a 16-byte piece into f32 values.
__device__ __forceinline__ void unpack16(const u32x4& w, float* o, uint16_t*) {
#pragma unroll
  for (int i = 0; i < 4; ++i) { o[2 * i] = bf16lo(w[i]); o[2 * i + 1] = bf16hi(w[i]); }
}
__device__ __forceinline__ void unpack16(const u32x4& w, float* o, float*) {
#pragma unroll
  for (int i = 0; i < 4; ++i) o[i] = __uint_as_float(w[i]);
}

// ---------------------------------------------------------------------------
// LDS-DMA: each lane copies 16 B from its own global address to
// lds_base + lane*16 (lds_base must be wave-uniform).
__device__ __forceinline__ void glds16(const void* gsrc, MK_LDS void* lds_base) {
  __builtin_amdgcn_global_load_lds(gsrc, lds_base, 16, 0, 0);
}

// Buffer-descriptor LDS-DMA: 16 B per lane from rsrc + voff + soff to lds_base + lane*16.
// The descriptor is built from wave-uniform values (readfirstlane'd, so the compiler can
// prove it and never wraps the load in a waterfall loop); voff is the only VGPR operand.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
  const uint64_t b = (uint64_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
  const uint32_t n = __builtin_amdgcn_readfirstlane(bytes);
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0, n, 0x00020000);
}
__device__ __forceinline__ void blds16(__amdgpu_buffer_rsrc_t r, MK_LDS void* lds_base, uint32_t voff,
                                       uint32_t soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, lds_base, 16, voff, soff, 0, 0);
}

// s_waitcnt with only vmcnt constrained (gfx9 encoding: vmcnt[3:0] | vmcnt_hi[15:14],
// expcnt[6:4]=7, lgkmcnt[11:8]=15).
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}
__device__ __forceinline__ void wait_lgkm0() { __builtin_amdgcn_s_waitcnt(0xC07F); }

// Raw workgroup barrier that does NOT drain outstanding LDS-DMA (unlike
// __syncthreads, whose fence emits vmcnt(0)).  The asm statement is a compiler
// memory barrier so LDS reads are not hoisted above it.
__device__ __forceinline__ void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// An MFMA seed plus a per-point offset, as four scalar v_add_f32.  Never a packed
// v_pk_add_f32: seeds built that way (op_sel broadcasts of the offset) intermittently
// reached the next MFMA wrong on gfx950 -- one point block of a per-point-offset
// workgroup got labels from a corrupted seed in 5 of 12 launches
// (scripts/debug/keys_d32_repro.py, profiles/r3_15_ppo_seed_race.md).  Files that use it are
// built with -fno-slp-vectorize (mikmeans/_build.py), so these stay scalar.
__device__ __forceinline__ void seed_add(f32x4& acc, float o) {
  float a0 = acc[0], a1 = acc[1], a2 = acc[2], a3 = acc[3];
  a0 += o; a1 += o; a2 += o; a3 += o;
  acc = f32x4{a0, a1, a2, a3};
}

// Volatile form: also a scheduling barrier, which keeps MFMA groups contiguous.
__device__ __forceinline__ float min3f_v(float a, float b, float c) {
  float d;
  asm volatile("v_min3_f32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}
// v_min3_f32 without the canonicalisation hipcc inserts around fminf.  Not
// volatile: a pure instruction the scheduler may interleave with the MFMAs.
__device__ __forceinline__ float min3f(float a, float b, float c) {
  float d;
  asm("v_min3_f32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}

// v_med3_f32 / v_min_f32 the same way (the TOP2 epilogue's per-key pair update: with fminf /
// the builtin med3 hipcc canonicalised every key first, one v_max_f32 per key).
__device__ __forceinline__ float med3f(float a, float b, float c) {
  float d;
  asm("v_med3_f32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}
__device__ __forceinline__ float min2f(float a, float b) {
  float d;
  asm("v_min_f32 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b));
  return d;
}
__device__ __forceinline__ float max2f(float a, float b) {
  float d;
  asm("v_max_f32 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b));
  return d;
}

// (score, centre) as one u64 whose unsigned order is (score, then lower index): the
// float's bits mapped to an order-preserving u32 in the high word.
__device__ __forceinline__ unsigned long long split_key(float v, int k) {
  const unsigned b = __float_as_uint(v);
  const unsigned o = (b & 0x80000000u) ? ~b : (b | 0x80000000u);
  return ((unsigned long long)o << 32) | (unsigned)k;
}
__device__ __forceinline__ float split_value(unsigned long long key) {
  const unsigned o = (unsigned)(key >> 32);
  return __uint_as_float((o & 0x80000000u) ? (o & 0x7fffffffu) : ~o);
}

// ---------------------------------------------------------------------------
// Unsigned minimum over lanes l and l ^ 16 / l ^ 32 with the gfx950 lane swaps (one VALU op
// each, no LDS traffic and no address arithmetic, unlike a ds_bpermute shuffle): swapping a
// value with itself leaves each lane holding itself in one result and its partner in the other.
__device__ __forceinline__ uint32_t lane_min_x16(uint32_t x) {
  const auto p = __builtin_amdgcn_permlane16_swap(x, x, false, false);
  return min((uint32_t)p[0], (uint32_t)p[1]);
}
__device__ __forceinline__ uint32_t lane_min_x32(uint32_t x) {
  const auto p = __builtin_amdgcn_permlane32_swap(x, x, false, false);
  return min((uint32_t)p[0], (uint32_t)p[1]);
}

// ---------------------------------------------------------------------------
// The canonical row-norm butterfly: v += v[lane ^ o] for o = 1, 2, 4, 8 inside each aligned
// group of 16 lanes (only the steps o < lim), as DPP lane moves (one v_add_f32_dpp per step,
// no ds_bpermute and no address VALU).  xor 1 / 2 are quad permutes; for o = 4 / 8 the partner
// quad / half-row is reached by a mirror instead, which reads the same values: after the
// steps before it every lane of a quad (half-row) holds the same partial sum, and a + b == b + a
// in IEEE arithmetic, so the sums are bitwise the xor butterfly's.
template <int CTRL>
__device__ __forceinline__ float dpp_f32(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float sum16_xor(float v, int lim = 16) {
  if (lim > 1) v += dpp_f32<0xB1>(v);    // quad_perm [1,0,3,2]: lane ^ 1
  if (lim > 2) v += dpp_f32<0x4E>(v);    // quad_perm [2,3,0,1]: lane ^ 2
  if (lim > 4) v += dpp_f32<0x141>(v);   // row_half_mirror: the other quad of the half-row
  if (lim > 8) v += dpp_f32<0x140>(v);   // row_mirror: the other half of the row
  return v;
}

// ---------------------------------------------------------------------------
// 64-lane reductions
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// ---------------------------------------------------------------------------
// Order-free inertia / changed-count slots.  A slot is 8 u64 words: words 0..6 hold
// signed 32-bit "digits" of a fixed-point sum at scale 2^-64 (word j weighs 2^(32 j - 64),
// range up to 2^160), word 7 an integer count.  Every addend is truncated to a multiple of
// 2^-64 by its own value alone and added with integer atomics, so the totals -- and the
// f64 decoded from them in a fixed order -- are bitwise the same whatever order the
// workgroups finish in (f64 atomicAdd made the logged inertia vary in its low bits from
// launch to launch).  A non-finite or >= 2^149 addend marks word 6 with 2^61 (inf).
constexpr unsigned long long SLOT_OVF = 1ull << 61;
__device__ __forceinline__ void slot_add(unsigned long long* w, double v, long long cnt) {
  if (cnt) atomicAdd(w + 7, (unsigned long long)cnt);
  if (v == 0.0) return;
  const unsigned long long bits = (unsigned long long)__double_as_longlong(v);
  const bool neg = bits >> 63;
  const int ex = (int)((bits >> 52) & 0x7ff);
  if (ex == 0x7ff) { atomicAdd(w + 6, SLOT_OVF); return; }
  unsigned long long m = (bits & ((1ull << 52) - 1)) | (ex ? (1ull << 52) : 0ull);
  int s = (ex ? ex : 1) - 1075 + 64;          // v = m * 2^(s - 64)
  if (s < 0) { m = -s >= 64 ? 0ull : m >> -s; s = 0; }
  const int j0 = s >> 5, o = s & 31;
  if (j0 > 4) { atomicAdd(w + 6, SLOT_OVF); return; }
  const unsigned long long lo = m << o, hi = o ? (m >> (64 - o)) : 0ull;
  const unsigned long long d[3] = {lo & 0xffffffffull, lo >> 32, hi};
#pragma unroll
  for (int i = 0; i < 3; ++i)
    if (d[i]) atomicAdd(w + j0 + i, neg ? (unsigned long long)(-(long long)d[i]) : d[i]);
}
// The value of summed digit words W[0..6] (each the int64 total over slots), fixed order.
__device__ __forceinline__ double slot_decode(const long long* W) {
  if (W[6] >= (long long)(SLOT_OVF >> 1)) return __builtin_inf();
  double v = 0.0;
#pragma unroll
  for (int j = 6; j >= 0; --j) v += __builtin_ldexp((double)W[j], 32 * j - 64);
  return v;
}

// argmin key: a score with a 4-bit index in its low mantissa bits (relative
// resolution 2^-19), so one v_min3_f32 tree yields (min score, index).
__device__ __forceinline__ float pack_key(float s, int r) {
  return __uint_as_float((__float_as_uint(s) & ~15u) | (unsigned)r);
}
// 6-bit variant (relative resolution 2^-17): one key space spans 64 candidates.
// `mask` must be ~63u held in a VGPR (see key6_mask): -64 is no inline constant and a
// gfx9 VOP3 takes no literal, so with the index in an SGPR this is ONE v_and_or_b32.
// Plain C++ (not inline asm): the first reader of an MFMA result must be an
// instruction the compiler's hazard recognizer sees, or it reads the register early.
__device__ __forceinline__ float pack_key6(float s, unsigned mask, unsigned r) {
  return __uint_as_float((__float_as_uint(s) & mask) | r);
}
__device__ __forceinline__ unsigned key6_mask() {
  unsigned m;
  asm volatile("v_mov_b32 %0, 0xffffffc0" : "=v"(m));  // opaque VGPR constant
  return m;
}

// ---------------------------------------------------------------------------
// Philox4x32-10 (Salmon et al., SC'11): the counter-based generator of the synthetic
// blobs (kpp.hip) and the mini-batch row sampler (rows.hip); NumPy mirror in
// mikmeans/data/blobs.py.
struct U4 { uint32_t x, y, z, w; };
// a ^ b ^ k in one VALU instruction: gfx950's three-input v_bitop3_b32 with the XOR3 truth
// table 0x96 (the compiler emits two v_xor_b32 for the round's key mix; the round keys are
// wave-uniform, so k is the SGPR operand).  Plain VALU asm.
__device__ __forceinline__ uint32_t xor3_sk(uint32_t a, uint32_t b, uint32_t k) {
  uint32_t r;
  asm("v_bitop3_b32 %0, %3, %1, %2 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "s"(k));
  return r;
}
__device__ __forceinline__ U4 philox(U4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    // one 32x32->64 product per word: a single v_mad_u64_u32 (quarter rate) instead of a
    // v_mul_lo_u32 + v_mul_hi_u32 pair
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
    const uint32_t lo0 = (uint32_t)p0, hi0 = (uint32_t)(p0 >> 32);
    const uint32_t lo1 = (uint32_t)p1, hi1 = (uint32_t)(p1 >> 32);
    c = U4{xor3_sk(hi1, c.y, k0), lo1, xor3_sk(hi0, c.w, k1), lo0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}
__device__ __forceinline__ float u01_open0(uint32_t v) { return ((v >> 8) + 1) * (1.0f / 16777216.0f); }
__device__ __forceinline__ float u01(uint32_t v) { return (v >> 8) * (1.0f / 16777216.0f); }

// Row index of accumulator register `reg` for lane half `h` in the 32x32 MFMA C/D map.
__device__ __forceinline__ int mfma32_row(int reg, int h) { return (reg & 3) + 8 * (reg >> 2) + 4 * h; }

}  // namespace mk
