// mikmeans — K4 finalize (new centroids, shift, re-pack for the next E-step)
// and K1 row squared norms, for gfx950.
//
// finalize runs once per iteration on the all-reduced f64 message
// [K*D sums | K counts | inertia | changed]: C_new = sums / counts (empty or
// frozen centres keep their position -- the frozen mask is the reference's
// "locked" centroid, app.mjs:128 / :360), shift_k = |C_new - C_old|^2, and it
// writes the fragment-packed -2*C (bf16 or f32) plus |C_q|^2 that the assign
// kernel streams (layout in kernels.h).  One workgroup per 32-centroid tile.
#include "common.h"
#include "kernels.h"

namespace mk {

// Packed layout (kernels.h): 16-centroid tiles; piece q of lane r+16g holds features
// [(4q+g)V, (4q+g+1)V).
template <typename T>
__device__ __forceinline__ void store_pack(void* pack, int dpad, int k, int d, float v) {
  constexpr int V = Elem<T>::V;
  const int nq = dpad / (4 * V);
  const int t = k >> 4, r = k & 15;
  const int g = (d / V) & 3, q = d / (4 * V);
  const int64_t off = ((int64_t)(t * nq + q) * 64 + r + 16 * g) * V + d % V;
  ((T*)pack)[off] = Elem<T>::from_f32(v);
}

template <typename T>
__global__ __launch_bounds__(256) void finalize_kernel(FinalizeArgs a) {
  const int kk = threadIdx.x >> 3, part = threadIdx.x & 7;
  const int k = blockIdx.x * 32 + kk;
  const int64_t KD = (int64_t)a.K * a.D;
  float shift = 0.f, cn = 0.f, cnt = 0.f, qs = 0.f;
  if (k < a.K) {
    double c = 0.0;
    bool upd = false;
    double scale = 0.0, keep = 1.0;
    if (a.mode != FIN_PACK_ONLY) {
      c = a.packed[KD + k];
      cnt = (float)c;
      const bool frozen = a.frozen && a.frozen[k];
      if (a.mode == FIN_LLOYD) {
        upd = (c > 0.0) && !frozen;
        scale = upd ? 1.0 / c : 0.0;
        keep = 0.0;
      } else {  // FIN_MINIBATCH: running weighted mean (Sculley 2010, batch form)
        upd = (c > 0.0) && !frozen;
        if (upd) {
          const double v_old = a.mb_counts[k];
          const double v_new = v_old + c;
          scale = 1.0 / v_new;
          keep = v_old / v_new;
        }
      }
    }
    for (int d = part; d < a.D; d += 8) {
      const float old = a.Cold[(int64_t)k * a.D + d];
      float nv = old;
      if (upd) nv = (float)(keep * (double)old + scale * a.packed[(int64_t)k * a.D + d]);
      if (a.Cnew) a.Cnew[(int64_t)k * a.D + d] = nv;
      const float diff = nv - old;
      shift += diff * diff;
      const float q = (a.dtype == DT_BF16) ? round_bf16(nv) : nv;
      cn += q * q;
      const float dq = q - ((a.dtype == DT_BF16) ? round_bf16(old) : old);
      qs += dq * dq;
      if (a.dtype == DT_BF16) store_pack<uint16_t>(a.pack, a.dpad, k, d, -2.f * q);
      else store_pack<float>(a.pack, a.dpad, k, d, -2.f * q);
    }
    for (int d = a.D + part; d < a.dpad; d += 8) {
      if (a.dtype == DT_BF16) store_pack<uint16_t>(a.pack, a.dpad, k, d, 0.f);
      else store_pack<float>(a.pack, a.dpad, k, d, 0.f);
    }
    if (a.mode == FIN_MINIBATCH && upd && part == 0) a.mb_counts[k] += c;
  } else if (k < a.Kpad) {
    for (int d = part; d < a.dpad; d += 8) {
      if (a.dtype == DT_BF16) store_pack<uint16_t>(a.pack, a.dpad, k, d, 0.f);
      else store_pack<float>(a.pack, a.dpad, k, d, 0.f);
    }
  }
  // reduce over the 8 threads of a centroid
#pragma unroll
  for (int o = 1; o < 8; o <<= 1) {
    shift += __shfl_xor(shift, o, 64);
    cn += __shfl_xor(cn, o, 64);
    qs += __shfl_xor(qs, o, 64);
  }
  if (part == 0 && k < a.Kpad) {
    a.cn[k] = (k < a.K) ? cn : PAD_SCORE;
    if (k < a.K) {
      if (a.shift) a.shift[k] = shift;
      if (a.qshift) a.qshift[k] = qs;
      if (a.counts_out) a.counts_out[k] = cnt;
    }
  }
}

hipError_t launch_finalize(const FinalizeArgs& a, hipStream_t s) {
  const unsigned nb = (unsigned)((a.Kpad + 31) / 32);
  if (a.dtype == DT_BF16) hipLaunchKernelGGL(finalize_kernel<uint16_t>, dim3(nb), dim3(256), 0, s, a);
  else hipLaunchKernelGGL(finalize_kernel<float>, dim3(nb), dim3(256), 0, s, a);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// K1: xn[i] = sum_d x[i,d]^2 (f32).  16 lanes per row, 16-B loads.  The order is canonical --
// lane s chains fmas over the elements of pieces s, s+16, s+32, ... in turn, then a 16-lane
// butterfly (1, 2, 4, 8; common.h sum16_xor) -- and shared with every other producer of row norms (the fused
// column-statistics pass below, csrc/rows.hip sample_rows), so all of them give the same bits.
template <typename T>
__global__ __launch_bounds__(256) void row_sqnorm_kernel(const T* __restrict__ X, int64_t N, int D,
                                                         int64_t ldx, float* __restrict__ out) {
  constexpr int V = Elem<T>::V;
  const int sub = threadIdx.x & 15;
  const int64_t stride = (int64_t)gridDim.x * 16;
  for (int64_t i = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 4); i < N; i += stride) {
    const T* row = X + i * ldx;
    float acc = 0.f;
    if ((D % V) == 0) {
      for (int c = sub * V; c < D; c += 16 * V) {
        const u32x4 w = *(const u32x4*)(row + c);
        float f[V];
        unpack16(w, f, (T*)nullptr);
#pragma unroll
        for (int e = 0; e < V; ++e) acc = __builtin_fmaf(f[e], f[e], acc);
      }
    } else {
      for (int c = sub; c < D; c += 16) { const float f = Elem<T>::to_f32(row[c]); acc = __builtin_fmaf(f, f, acc); }
    }
    acc = sum16_xor(acc);
    if (sub == 0) out[i] = acc;
  }
}

hipError_t launch_row_sqnorm(int dtype, const void* X, int64_t N, int D, int64_t ldx, float* out,
                             hipStream_t s) {
  if (N <= 0) return hipSuccess;
  int64_t nb = (N + 15) / 16;
  if (nb > 8192) nb = 8192;
  if (dtype == DT_BF16)
    hipLaunchKernelGGL(row_sqnorm_kernel<uint16_t>, dim3((unsigned)nb), dim3(256), 0, s,
                       (const uint16_t*)X, N, D, ldx, out);
  else
    hipLaunchKernelGGL(row_sqnorm_kernel<float>, dim3((unsigned)nb), dim3(256), 0, s,
                       (const float*)X, N, D, ldx, out);
  return hipGetLastError();
}

// Packed 16-bit helpers, written out (left to itself the compiler turns min(y, 1) per half into
// a compare + select per half, six instructions for one).
__device__ __forceinline__ uint32_t pk_min_u16(uint32_t a, uint32_t b) {
  uint32_t d;
  asm("v_pk_min_u16 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b));
  return d;
}
__device__ __forceinline__ uint32_t pk_max_u16(uint32_t a, uint32_t b) {
  uint32_t d;
  asm("v_pk_max_u16 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b));
  return d;
}
__device__ __forceinline__ uint32_t pk_add_u16(uint32_t a, uint32_t b) {
  uint32_t d;
  asm("v_pk_add_u16 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b));
  return d;
}
__device__ __forceinline__ uint32_t pk_sub_sat_u16(uint32_t a, uint32_t b) {   // max(a - b, 0)
  uint32_t d;
  asm("v_pk_sub_u16 %0, %1, %2 clamp" : "=v"(d) : "v"(a), "v"(b));
  return d;
}
__device__ __forceinline__ uint32_t pk_mad_u16(uint32_t a, uint32_t b, uint32_t c) {   // a * b + c
  uint32_t d;
  asm("v_pk_mad_u16 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}
__device__ __forceinline__ uint32_t pk_shr_u16(uint32_t a, uint32_t s) {   // a >> s per half
  uint32_t d;
  asm("v_pk_lshrrev_b16 %0, %1, %2" : "=v"(d) : "v"(s), "v"(a));
  return d;
}

// The lowest-bit keys of two bf16 values at once (y = both values' |bits|, 15 bits a half):
// key = max(E, 1) + min(ctz(m), 7) per half, the high half offset by 16, and 0x4000 added to
// a half that is zero, inf or NaN -- lowbit_exp(x) = key - 134 for the others (E the biased
// exponent, m the 7 mantissa bits; a subnormal's E is 0 and its exponent that of E = 1).
__device__ __forceinline__ uint32_t lowbit_keys_bf16x2(uint32_t y) {
  const uint32_t e2 = pk_max_u16(pk_shr_u16(y, 0x00070007u), 0x00010001u);
  const uint32_t g2 = (y & 0x007f007fu) | 0x00800080u;   // bit 7 stands in for the hidden bit
  const uint32_t clo = __builtin_ctz(g2);                // min(ctz(m_lo), 7)
  const uint32_t chi = __builtin_ctz(g2 & 0xffff0000u);  // 16 + min(ctz(m_hi), 7)
  const uint32_t k2 = e2 + clo + (chi << 16);
  // invalid halves: y - 1 >= 0x7f7f (y = 0 wraps to 0xffff)
  const uint32_t inv = pk_min_u16(pk_sub_sat_u16(pk_add_u16(y, 0xffffffffu), 0x7f7e7f7eu), 0x00010001u);
  return pk_mad_u16(inv, 0x40004000u, k2);
}
// Per-column max |x| (the fixed-point M-step's column scales, csrc/update.hip).  L lanes
// per row (power of two >= the row's 16-byte pieces, <= 64), 256/L rows per pass, four
// independent row loads in flight per lane; |x| compared as bit patterns (non-negative
// floats order like unsigned integers, and a NaN's pattern exceeds +inf's, so NaN
// propagates like torch.aminmax).  One global atomicMax per (block, column).  STATS: also,
// per column, the sums of |x|, x and x^2 (f64 per lane; every block writes its partial sums
// to its own row of fpart [COLSTAT_BLOCKS][3][D], which colstat_reduce_kernel then sums in a
// fixed order -- no f64 atomics, so the statistics are bitwise the same on every launch:
// fstats = [sum |x| | sum x | sum x^2], the last two give the tol scale's variance without
// an f32 copy of X), the count of nonzero values and the exponent of the lowest set bit over
// all nonzero finite values (x is an integer multiple of 2^lowbit; integer atomics, order-free).
// From these the engine flags wide-range columns for the residual M-step pass: a column whose
// values all sit on the hi pass's grid (lowbit >= -col_exp: one-hot, small integers, coarse
// bf16) never needs it, and otherwise the max is compared with the mean of the NONZERO |x|
// (sparse columns stay single-pass).  NORMS (the launch covers whole rows, <= 64 pieces): also
// every row's |x|^2 in row_sqnorm_kernel's canonical order -- the fit's setup reads X once.
constexpr int COLSTAT_BLOCKS = 8192;   // the partials' row cap (colstat_cap sizes a launch)

// Branch-free (it runs once per element of the pass; the branchy form cost ~20 VALU + SALU
// exec-mask instructions per element and made the statistics pass VALU-bound): with y = |f|'s
// bits, ctz(y | 2^23) is the mantissa's trailing-zero count capped at 23 (the hidden bit), and
// max(e, 1) covers subnormals (-149 + ctz(m) = max(0, 1) + ctz(m) - 150).  Zero, inf and NaN
// (y - 1 >= 0x7f7fffff unsigned) give "no constraint".
__device__ __forceinline__ int lowbit_exp(float f) {
  const uint32_t y = __float_as_uint(f) & 0x7fffffffu;
  const int v = (int)(__builtin_ctz(y | 0x800000u) + max(y >> 23, 1u)) - 150;
  return y - 1u < 0x7f7fffffu ? v : 1 << 30;
}

// One launch covers up to 64 16-B pieces of a row (a column block: X, out, fpart, nnz and
// lowbit point at its first column; fpart rows are fstride columns apart).
// LT: the lanes per row when fixed at compile time (16: a 128-column bf16 row, whose fused row
// norms then run without the runtime lane-count branches), 0 = runtime L.
template <typename T, bool STATS, bool NORMS, int LT = 0>
__global__ __launch_bounds__(256) void col_absmax_kernel(const T* __restrict__ X, int64_t N, int NP,
                                                         int L_, int64_t ldx, uint32_t* __restrict__ out,
                                                         double* __restrict__ fpart, int64_t fstride,
                                                         unsigned long long* __restrict__ nnz,
                                                         int* __restrict__ lowbit, float* __restrict__ xn) {
  constexpr int V = Elem<T>::V;
  const int L = LT ? LT : L_;
  const int p = threadIdx.x & (L - 1);
  const int R = 256 / L;
  const int64_t step = (int64_t)gridDim.x * R;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t m[V];
  double q[V], sx[V], sxx[V];   // f64 per lane: chunked / sharded passes agree to ~1e-16
  uint32_t nz[V];
  int lb[V];
#pragma unroll
  for (int e = 0; e < V; ++e) { m[e] = 0u; q[e] = 0.0; sx[e] = 0.0; sxx[e] = 0.0; nz[e] = 0u; lb[e] = 1 << 30; }
  auto take = [&](const u32x4& w, int64_t row) {
    float f[V];
    unpack16(w, f, (T*)nullptr);
#pragma unroll
    for (int e = 0; e < V; ++e) {
      m[e] = max(m[e], __float_as_uint(f[e]) & 0x7fffffffu);
      if constexpr (STATS) {
        const double d = (double)f[e];
        q[e] += fabs(d);
        sx[e] += d;
        sxx[e] = __builtin_fma(d, d, sxx[e]);
        nz[e] += f[e] != 0.f;
        lb[e] = min(lb[e], lowbit_exp(f[e]));
      }
    }
    if constexpr (NORMS) {
      // the row's |x|^2 as row_sqnorm_kernel chains it: lane s < 16 takes its own piece, then
      // pieces s+16, s+32, s+48 (from the lanes holding them), then the 16-lane butterfly
      float acc = 0.f;
#pragma unroll
      for (int e = 0; e < V; ++e) acc = __builtin_fmaf(f[e], f[e], acc);
      for (int g = 16; g < L; g += 16) {   // (L > 16: every lane of the row group runs it)
        const int src = (lane & ~(L - 1)) + ((p + g) & (L - 1));
#pragma unroll
        for (int e = 0; e < V; ++e) {
          const float o = __shfl(f[e], src, 64);
          if (p + g < NP) acc = __builtin_fmaf(o, o, acc);
        }
      }
      acc = sum16_xor(acc, L);
      if (p == 0) xn[row] = acc;
    }
  };
  // bf16 statistics, VALU-lean (the per-element form above made the pass VALU-bound: 6.9 ms
  // against 4.6 ms for the max alone at N=1e8 D=128, profiles/r6_10_hbm_ceiling.log).  Same
  // results bit for bit: the max, the nonzero count and the lowest-bit exponent run on packed
  // 16-bit halves, two values per instruction (|x|'s bf16 bits order like its f32 bits;
  // lowbit_keys_bf16x2); the f64 sums and the row norms keep their per-row order.
  [[maybe_unused]] uint32_t mp[4], nzp[4], kp[4];
  [[maybe_unused]] int pend = 0;
  [[maybe_unused]] auto flush_nz = [&]() {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      nz[2 * j] += nzp[j] & 0xffffu;
      nz[2 * j + 1] += nzp[j] >> 16;
      nzp[j] = 0u;
    }
    pend = 0;
  };
  constexpr bool LEAN = STATS && sizeof(T) == 2;
  if constexpr (LEAN) {
#pragma unroll
    for (int j = 0; j < 4; ++j) { mp[j] = 0u; nzp[j] = 0u; kp[j] = 0xffffffffu; }
  }
  // cnt rows' pieces (rows row0, row0 + step, ...)
  [[maybe_unused]] auto take_lean = [&](const u32x4* w, auto cnt_c, int64_t row0) {
    constexpr int cnt = decltype(cnt_c)::value;
#pragma unroll
    for (int u = 0; u < cnt; ++u) {
      float f[V];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t x = w[u][j];
        const uint32_t y = x & 0x7fff7fffu;
        mp[j] = pk_max_u16(mp[j], y);
        nzp[j] = pk_add_u16(nzp[j], pk_min_u16(y, 0x00010001u));
        kp[j] = pk_min_u16(kp[j], lowbit_keys_bf16x2(y));
        f[2 * j] = __uint_as_float(x << 16);
        f[2 * j + 1] = __uint_as_float(x & 0xffff0000u);
      }
#pragma unroll
      for (int e = 0; e < V; ++e) {
        const double d = (double)f[e];
        q[e] += fabs(d);
        sx[e] += d;
        sxx[e] = __builtin_fma(d, d, sxx[e]);
      }
      if constexpr (NORMS) {
        float acc = 0.f;
#pragma unroll
        for (int e = 0; e < V; ++e) acc = __builtin_fmaf(f[e], f[e], acc);
        for (int g = 16; g < L; g += 16) {
          const int src = (lane & ~(L - 1)) + ((p + g) & (L - 1));
#pragma unroll
          for (int e = 0; e < V; ++e) {
            const float o = __shfl(f[e], src, 64);
            if (p + g < NP) acc = __builtin_fmaf(o, o, acc);
          }
        }
        acc = sum16_xor(acc, L);
        if (p == 0) xn[row0 + u * step] = acc;
      }
    }
    pend += cnt;
    if (pend > 65535 - 4) flush_nz();   // (16-bit counts)
  };
  // (NORMS: a row group's lanes all run the loop -- lanes past the row's pieces take zeros --
  // so the shuffles above see every lane of the group)
  if (NORMS || p < NP) {
    int64_t i = (int64_t)blockIdx.x * R + threadIdx.x / L;
    const T* base = X + (int64_t)p * V;
    auto load = [&](int64_t row) -> u32x4 {
      return p < NP ? *(const u32x4*)(base + row * ldx) : u32x4{0u, 0u, 0u, 0u};
    };
    for (; i + 3 * step < N; i += 4 * step) {
      u32x4 w[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) w[u] = load(i + u * step);
      if constexpr (LEAN) {
        take_lean(w, std::integral_constant<int, 4>{}, i);
      } else {
#pragma unroll
        for (int u = 0; u < 4; ++u) take(w[u], i + u * step);
      }
    }
    for (; i < N; i += step) {
      const u32x4 w1 = load(i);
      if constexpr (LEAN) take_lean(&w1, std::integral_constant<int, 1>{}, i);
      else take(w1, i);
    }
  }
  if constexpr (LEAN) {
    flush_nz();
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      m[2 * j] = mp[j] << 16;
      m[2 * j + 1] = mp[j] & 0xffff0000u;
      const int klo = (int)(kp[j] & 0xffffu), khi = (int)(kp[j] >> 16);
      lb[2 * j] = klo >= 0x4000 ? 1 << 30 : klo - 134;
      lb[2 * j + 1] = khi >= 0x4000 ? 1 << 30 : khi - 16 - 134;
    }
  }
  for (int o = L; o < 64; o <<= 1)
#pragma unroll
    for (int e = 0; e < V; ++e) {
      m[e] = max(m[e], (uint32_t)__shfl_xor((int)m[e], o, 64));
      if constexpr (STATS) {
        q[e] += __shfl_xor(q[e], o, 64);
        sx[e] += __shfl_xor(sx[e], o, 64);
        sxx[e] += __shfl_xor(sxx[e], o, 64);
        nz[e] += (uint32_t)__shfl_xor((int)nz[e], o, 64);
        lb[e] = min(lb[e], __shfl_xor(lb[e], o, 64));
      }
    }
  __shared__ uint32_t red[4][64 * V];
  if (lane < L && p < NP)
#pragma unroll
    for (int e = 0; e < V; ++e) red[wv][lane * V + e] = m[e];
  __syncthreads();
  for (int j = threadIdx.x; j < NP * V; j += 256) {
    const uint32_t v = max(max(red[0][j], red[1][j]), max(red[2][j], red[3][j]));
    if (v) atomicMax(out + j, v);
  }
  if constexpr (STATS) {
    __shared__ double rd[4][64 * 8];
    double* mine = fpart + (int64_t)blockIdx.x * 3 * fstride;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      __syncthreads();
      if (lane < L && p < NP)
#pragma unroll
        for (int e = 0; e < V; ++e) rd[wv][lane * V + e] = k == 0 ? q[e] : k == 1 ? sx[e] : sxx[e];
      __syncthreads();
      for (int j = threadIdx.x; j < NP * V; j += 256)
        mine[(int64_t)k * fstride + j] = (rd[0][j] + rd[1][j]) + (rd[2][j] + rd[3][j]);
    }
    __syncthreads();
    if (lane < L && p < NP)
#pragma unroll
      for (int e = 0; e < V; ++e) red[wv][lane * V + e] = nz[e];
    __syncthreads();
    for (int j = threadIdx.x; j < NP * V; j += 256) {
      const unsigned long long c = (unsigned long long)red[0][j] + red[1][j] + red[2][j] + red[3][j];
      if (c) atomicAdd(nnz + j, c);
    }
    __syncthreads();
    int* ri = (int*)&red[0][0];
    if (lane < L && p < NP)
#pragma unroll
      for (int e = 0; e < V; ++e) ri[wv * 64 * V + lane * V + e] = lb[e];
    __syncthreads();
    for (int j = threadIdx.x; j < NP * V; j += 256) {
      const int v = min(min(ri[j], ri[64 * V + j]), min(ri[128 * V + j], ri[192 * V + j]));
      if (v < (1 << 30)) atomicMin(lowbit + j, v);
    }
  }
}

// fstats[j] = sum over the first `rows` rows of fpart[.][j] (j < n = 3 D; the launched blocks), in
// one fixed order: each of 256 threads sums its 8 consecutive row slots (rows past `rows` count as
// zero), then a fixed LDS tree.  One workgroup per j.
__global__ __launch_bounds__(256) void colstat_reduce_kernel(const double* __restrict__ fpart, int64_t n,
                                                            int rows, double* __restrict__ fstats) {
  constexpr int PER = COLSTAT_BLOCKS / 256;
  const int64_t j = blockIdx.x;
  double v = 0.0;
#pragma unroll
  for (int r = 0; r < PER; ++r) {
    const int row = (int)threadIdx.x * PER + r;
    if (row < rows) v += fpart[(int64_t)row * n + j];
  }
  __shared__ double t[256];
  t[threadIdx.x] = v;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) t[threadIdx.x] += t[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) fstats[j] = t[0];
}

int colstat_blocks() { return COLSTAT_BLOCKS; }

// The launch's block cap for D columns: as many blocks as keep the f64 partials within 32 MiB,
// between 2048 and COLSTAT_BLOCKS (8192 at D <= 128) -- more, shorter-lived blocks run the
// pass faster: 7.24 / 6.99 / 6.89 ms at 2048 / 4096 / 8192 blocks, N=1e8 D=128
// (profiles/r6_05_setup_blocks_d128.log); or the A/B switch V_COLSTAT_BLOCKS (1..8192).
static int colstat_cap(int D) {
  const int v = variant(V_COLSTAT_BLOCKS);
  if (v > 0 && v <= COLSTAT_BLOCKS) return v;
  const int64_t fit = (int64_t)(32 << 20) / ((int64_t)24 * (D > 0 ? D : 1));
  return (int)(fit < 2048 ? 2048 : fit > COLSTAT_BLOCKS ? COLSTAT_BLOCKS : fit);
}

// Blocks of the widest launch launch_col_absmax makes for N rows of D columns: the rows of
// fpart it writes (the caller's allocation; ADVICE r5: sized to N, not to COLSTAT_BLOCKS).
int colstat_rows(int dtype, int64_t N, int D) {
  const int V = dtype == DT_BF16 ? 8 : 4;
  const int NPT = D / V;
  int64_t rows = 0;
  for (int p0 = 0; p0 < NPT; p0 += 64) {
    const int NP = NPT - p0 < 64 ? NPT - p0 : 64;
    int L = 1;
    while (L < NP) L *= 2;
    int64_t nb = (N + 256 / L - 1) / (256 / L);
    if (nb > colstat_cap(D)) nb = colstat_cap(D);
    rows = nb > rows ? nb : rows;
  }
  return (int)rows;
}

hipError_t launch_col_absmax(int dtype, const void* X, int64_t N, int D, int64_t ldx, uint32_t* out,
                             hipStream_t s, double* fstats, unsigned long long* nnz, int* lowbit, double* fpart,
                             float* xn) {
  const int V = dtype == DT_BF16 ? 8 : 4;
  const int NPT = D / V;
  if (N <= 0 || D % V || NPT < 1) return N <= 0 ? hipSuccess : hipErrorInvalidValue;
  if ((fstats != nullptr) != (nnz != nullptr) || (fstats != nullptr) != (lowbit != nullptr) ||
      (fstats != nullptr) != (fpart != nullptr))
    return hipErrorInvalidValue;  // the statistics come together
  if (xn && NPT > 64) return hipErrorInvalidValue;   // (row norms: one launch must cover the row)
  // wide rows: one launch per block of 64 pieces (512 bf16 / 256 f32 columns)
  for (int p0 = 0; p0 < NPT; p0 += 64) {
    const int NP = NPT - p0 < 64 ? NPT - p0 : 64;
    const int64_t c0 = (int64_t)p0 * V;
    int L = 1;
    while (L < NP) L *= 2;
    const int R = 256 / L;
    int64_t nb = (N + R - 1) / R;
    // each block streams its rows with 4 loads in flight per lane (colstat_cap: one resident
    // round of longer-lived blocks, 768, measured 7.6 % slower than 2048,
    // profiles/r6_04_ab_colstats_d128.log)
    if (nb > colstat_cap(D)) nb = colstat_cap(D);
    const dim3 g((unsigned)nb), b(256);
    double* fp = fpart ? fpart + c0 : nullptr;
    unsigned long long* nz = nnz ? nnz + c0 : nullptr;
    int* lb = lowbit ? lowbit + c0 : nullptr;
#define MK_COLSTAT(TT, ST, NR, LT)                                                                              \
  hipLaunchKernelGGL((col_absmax_kernel<TT, ST, NR, LT>), g, b, 0, s, (const TT*)X + c0, N, NP, L, ldx, out + c0, \
                     fp, (int64_t)D, nz, lb, xn)
    if (dtype == DT_BF16) {
      if (fstats) {
        if (xn && L == 16) MK_COLSTAT(uint16_t, true, true, 16);
        else if (xn) MK_COLSTAT(uint16_t, true, true, 0);
        else MK_COLSTAT(uint16_t, true, false, 0);
      } else {
        if (xn) MK_COLSTAT(uint16_t, false, true, 0); else MK_COLSTAT(uint16_t, false, false, 0);
      }
    } else {
      if (fstats) { if (xn) MK_COLSTAT(float, true, true, 0); else MK_COLSTAT(float, true, false, 0); }
      else { if (xn) MK_COLSTAT(float, false, true, 0); else MK_COLSTAT(float, false, false, 0); }
    }
#undef MK_COLSTAT
  }
  if (fstats)
    hipLaunchKernelGGL(colstat_reduce_kernel, dim3((unsigned)(3 * D)), dim3(256), 0, s, fpart, (int64_t)3 * D,
                       colstat_rows(dtype, N, D), fstats);
  return hipGetLastError();
}

}  // namespace mk
