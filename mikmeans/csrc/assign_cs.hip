// mikmeans — K2, centre-stationary form: nearest-centroid assignment for bf16 rows of 128 or
// 256 features with up to 1024 / 512 centres (gfx950, v_mfma_f32_16x16x32_bf16).
//
// The streaming kernel (assign16.hip) keeps a few point blocks in registers and streams every
// centre tile through an LDS ring, once per 192-256-point workgroup: each workgroup pays a
// prologue (its rows' loads, the first centre chunks, the seed offset) and the ring's
// barriers.  Here the roles are swapped.  One workgroup of 16 waves per CU holds ALL the
// centres in registers for its whole life -- wave w the A fragments of tiles [wT, wT+T) -- and
// the points stream through a 3-slot LDS ring of 64-point super-blocks, fetched by LDS-DMA
// two super-blocks ahead.  Every wave multiplies every super-block against its own centres;
// each wave parks its per-point winners (truncated score | local index) in LDS, and one wave
// (the finisher) merges the 16 waves' winners and writes a super-block's labels / distances /
// changed count while the others compute the next one: one barrier per 64 points, no
// per-workgroup prologue.  (No LDS atomics: the compiler drains every in-flight LDS-DMA before
// one, which would serialise the ring.)
//
// Numerics are the streaming kernel's: the seed offset o = (1 + 2^-12) max |x|^2 over the
// block of rows (here the 64-row super-block; per-point offsets where max > 4 min), each
// score seeded fl(|c|^2 + o) and accumulated over the K-steps in the same order, 6-bit
// truncated keys, and the winner is the lexicographic minimum (truncated score, centre
// index) -- the same rule as the streaming kernel's segment merge.  The seed-offset block
// differs (64 rows), so assign16_block_rows reports 64 while this kernel is selected.
//
// Layout of a super-block in the ring: for 16-point block j and 16-B piece q, 1 KiB where
// lane l = r + 16g holds point 16j + r's features [(4q+g)8, +8) -- the B fragments, read
// with one conflict-free ds_read_b128 per lane (the centroid pack's layout, kernels.h).
//
// Measured (profiles/r5_24_ab_d*_cs_v2.log, r5_25_pmc_cs256_v2.md): slower than the streaming
// kernel -- 4.55 vs 3.83 ms at D=256 K=512, 5.44 vs 3.93 ms at D=128 K=1024 -- so it stays an
// opt-in A/B switch.  Each 16-point block is merged across its 4 lane groups and parked per
// wave, a cost the streaming kernel pays once per segment of 16 tiles but this one once per
// T = 2 / 4 tiles (1.9 non-MFMA VALU per MFMA against 1.3), and its B-fragment + seed reads per
// MFMA exceed the streaming kernel's A-fragment reads shared by 3-4 point blocks.
#include <type_traits>

#include "common.h"
#include "kernels.h"

namespace mk {

template <int DPAD>
struct CsCfg {
  static constexpr int NW = 16;                    // waves (one workgroup per CU)
  static constexpr int NQ = DPAD / 32;             // K-steps of 32 bf16
  static constexpr int T = DPAD == 128 ? 4 : 2;    // centre tiles per wave (64 A VGPRs)
  static constexpr int KCS = NW * T * 16;          // centres held
  static constexpr int SB = 4;                     // 16-point blocks per super-block
  static constexpr int SPTS = SB * 16;             // points per super-block
  static constexpr int SLOT = SB * NQ * 1024;      // ring slot bytes
  static constexpr int NB = 3;                     // ring slots (two super-blocks in flight)
  static constexpr int NXB = 8;                    // |x|^2 ring (fetched a step ahead of the rows,
                                                   // read by the finisher a step behind)
  static constexpr int NDMA = SB * NQ;             // 1-KiB DMA instructions per super-block
  static constexpr int FIN = NW - 1;               // the finisher wave (no DMA duty)
  static constexpr int NDW = NW - 1;               // waves sharing the DMA
  // row DMA instructions of wave w per super-block (fragments d = w, w + NDW, ...)
  static constexpr __device__ int dma_x(int w) {
    int c = 0;
    for (int d = w; d < NDMA; d += NDW) ++c;
    return c;
  }
};

template <int N>
__device__ __forceinline__ void wait_vm_n(int n) {   // s_waitcnt vmcnt(n), n < N runtime-uniform
  if constexpr (N > 0) {
    if (n == N) { wait_vmcnt<N>(); return; }
    wait_vm_n<N - 1>(n);
  } else {
    wait_vmcnt<0>();
  }
}

__device__ __forceinline__ float wave_max_f(float v) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float wave_min_f(float v) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) v = fminf(v, __shfl_xor(v, o, 64));
  return v;
}

template <int DPAD>
__global__ __launch_bounds__(1024, 1) void assign_cs_kernel(AssignArgs a) {
  using C = CsCfg<DPAD>;
  constexpr int NQ = C::NQ, T = C::T;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* ring = smem;                                                     // [NB][SLOT]
  float* xnr = (float*)(smem + C::NB * C::SLOT);                         // [NXB][SPTS]
  uint32_t* mrg = (uint32_t*)(xnr + C::NXB * C::SPTS);                   // [2][NW][SPTS] wave winners
  f32x4* sdl = (f32x4*)(mrg + 2 * C::NW * C::SPTS);                      // [NW][T][64] seeds
  float* offl = (float*)(sdl + C::NW * T * 64);                          // [4] super-block offsets
  float* cnl = offl + 4;                                                 // [Kpad]
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 15, g = lane >> 4;
  const int64_t N = a.N;
  const int64_t nsb = (N + C::SPTS - 1) / C::SPTS;
  const int64_t cnt = blockIdx.x < nsb ? (nsb - 1 - blockIdx.x) / gridDim.x + 1 : 0;
  if (cnt == 0) return;   // (workgroup-uniform)
  const int ntiles = a.Kpad / 16;
  const int tw = min(max(ntiles - wid * T, 0), T);   // this wave's tiles (wave-uniform)
  const size_t rowb = (size_t)a.ldx * 2;             // bytes per X row

  // centres: A fragments into registers for the kernel's life (tiles past Kpad: zeros, seeded
  // with PAD_SCORE below, so they never win and the MFMA loop needs no per-tile guard)
  const uint16_t* pack = (const uint16_t*)a.Cpack;
  u32x4 af[T][NQ];
#pragma unroll
  for (int t = 0; t < T; ++t) {
    const int tg = wid * T + t;
#pragma unroll
    for (int q = 0; q < NQ; ++q)
      af[t][q] = t < tw ? *(const u32x4*)(pack + ((int64_t)(tg * NQ + q) * 64 + lane) * 8) : u32x4{0u, 0u, 0u, 0u};
  }
  for (int k = threadIdx.x; k < a.Kpad; k += 1024) cnl[k] = a.cn[k];

  // LDS-DMA of the i-th super-block's rows into ring slot i % NB (rows past N read as zeros:
  // buffer bounds), and -- one step further ahead -- of its row norms into |x|^2 slot i % NXB
  auto sb_rows = [&](int64_t i, int64_t& r0) {   // (rows of the i-th super-block; <= 0 past the end)
    r0 = (blockIdx.x + i * gridDim.x) * (int64_t)C::SPTS;
    return N - r0 < C::SPTS ? N - r0 : (int64_t)C::SPTS;
  };
  auto issue_x = [&](int64_t i) {
    int64_t r0;
    const int64_t nv = sb_rows(i, r0);
    const __amdgpu_buffer_rsrc_t rx = make_rsrc((const char*)a.X + (size_t)r0 * rowb, (uint32_t)(nv * rowb));
    char* slot = ring + (int)(i % C::NB) * C::SLOT;
#pragma unroll
    for (int c = 0; c < (C::NDMA + C::NDW - 1) / C::NDW; ++c) {
      const int d = wid + c * C::NDW;
      if (d < C::NDMA) {
        const int j = d / NQ, q = d % NQ;
        // (pieces past D read as zeros -- an offset past the buffer -- as assign16 zeroes them)
        const uint32_t voff = (4 * q + g) * 8 < a.D ? (uint32_t)((16 * j + r) * rowb) + (uint32_t)((4 * q + g) * 16)
                                                    : 0x80000000u;
        blds16(rx, (MK_LDS void*)(slot + d * 1024), voff, 0u);
      }
    }
  };
  auto issue_xn = [&](int64_t i) {   // (wave NDW-1; past the last super-block: an empty buffer)
    int64_t r0;
    const int64_t nv = sb_rows(i, r0);
    const __amdgpu_buffer_rsrc_t rn = make_rsrc(nv > 0 ? a.xn + r0 : a.xn, (uint32_t)(nv > 0 ? nv * 4 : 0));
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rn, (MK_LDS void*)(xnr + (int)(i % C::NXB) * C::SPTS), 4,
                                             (uint32_t)lane * 4u, 0u, 0, 0);
  };
  constexpr int XNW = C::NDW - 1;   // the wave that fetches the row norms
  if (wid != C::FIN) {
    issue_x(0);
    if (cnt > 1) issue_x(1);
    if (wid == XNW) { issue_xn(0); issue_xn(1); issue_xn(2); }
  }
  __syncthreads();   // (cn and the centre fragments' loads: vmcnt(0) drains the DMA too)

  const unsigned kmask = key6_mask();
  const int nwt = (ntiles + T - 1) / T;   // waves holding centres
  // finisher state: the current super-block's old labels (loaded a step before they are used;
  // the compiler's counted vmcnt waits cover them)
  int oldl = -2;
  double inert = 0.0;
  int changed = 0;
  const bool want_mind = a.mind != nullptr;

  // (finisher) the i-th super-block's seed offset from its row norms, into LDS slot i % 4 for
  // every wave: the shared offset, or -1 for per-point offsets (max > 4 min)
  auto offsets = [&](int64_t i) {
    int64_t r0;
    const int64_t nv = sb_rows(i, r0);
    if (nv <= 0) return;
    const float xs = xnr[(int)(i % C::NXB) * C::SPTS + (lane < nv ? lane : (int)nv - 1)];   // (assign16 clamps)
    const float m = wave_max_f(fmaxf(0.f, xs)), mn = wave_min_f(fminf(3.0e38f, xs));
    if (lane == 0) offl[(int)(i & 3)] = m > 4.f * mn ? -1.f : __builtin_fmaf(m, 2.44140625e-04f, m);
  };

  auto finish = [&](int64_t i, int old) {   // (finisher) super-block i's outputs
    int64_t r0;
    const int64_t nv = sb_rows(i, r0);
    const float xs = xnr[(int)(i % C::NXB) * C::SPTS + lane];
    const float off = offl[(int)(i & 3)];
    // the 16 waves' winners of each point: lexicographic (truncated score, wave, local index) --
    // the waves' centre ranges ascend, so that is (score, centre index)
    const uint32_t* ms = mrg + (int)(i & 1) * C::NW * C::SPTS + lane;
    uint32_t best = ms[0];
    int bw = 0;
    for (int w = 1; w < nwt; ++w) {
      const uint32_t kw = ms[w * C::SPTS];
      if ((kw & ~63u) < (best & ~63u)) { best = kw; bw = w; }
    }
    if (lane < nv) {
      const float offp = off < 0.f ? __builtin_fmaf(xs, 2.44140625e-04f, xs) : off;
      const int k = bw * T * 16 + (int)(best & 63u);
      const float v = __uint_as_float(best & ~63u) - offp;
      const float d = fmaxf(xs + v, 0.f);
      if (a.track_changed) changed += (old != k);
      a.labels[r0 + lane] = k;
      if (want_mind) a.mind[r0 + lane] = d;
      inert += (double)d;
    }
  };

  // one 16-point block against this wave's T tiles: seeds from LDS (+ the point's own offset
  // under PPO), NQ K-steps, the lane's 6-bit key minimum, then the 4 lane groups' via two
  // shuffles; the winner (truncated score | local index 16t + 4g + reg) parked for the finisher
  auto block = [&](auto ppo_tag, const char* slot, const float* xb, const f32x4* sdw, uint32_t* ms, int j) {
    constexpr bool PPO = decltype(ppo_tag)::value;
    const char* blk = slot + j * NQ * 1024 + lane * 16;
    f32x4 acc[T];
#pragma unroll
    for (int t = 0; t < T; ++t) acc[t] = sdw[t * 64];
    if constexpr (PPO) {
      const float xv = xb[16 * j + r];
      const float op = __builtin_fmaf(xv, 2.44140625e-04f, xv);
#pragma unroll
      for (int t = 0; t < T; ++t) seed_add(acc[t], op);
    }
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
    __builtin_amdgcn_sched_barrier(0);
    u32x4 b0 = *(const u32x4*)blk;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      u32x4 b1;
      if (q + 1 < NQ) b1 = *(const u32x4*)(blk + (q + 1) * 1024);
#pragma unroll
      for (int t = 0; t < T; ++t)
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(short8, af[t][q]),
                                                         __builtin_bit_cast(short8, b0), acc[t], 0, 0, 0);
      if (q + 1 < NQ) b0 = b1;
    }
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    // keys: truncated score | (16 t + reg) -- wave-uniform index bits (lane group g added after
    // the lane's minimum, bits 2-3), so each key is one v_and_or_b32
    float kb = 3.0e38f;
#pragma unroll
    for (int t = 0; t < T; ++t) {
      const float k0 = pack_key6(acc[t][0], kmask, (unsigned)(16 * t + 0));
      const float k1 = pack_key6(acc[t][1], kmask, (unsigned)(16 * t + 1));
      const float k2 = pack_key6(acc[t][2], kmask, (unsigned)(16 * t + 2));
      const float k3 = pack_key6(acc[t][3], kmask, (unsigned)(16 * t + 3));
      kb = min3f(min3f(k0, k1, k2), k3, kb);
    }
    uint32_t kbits = __float_as_uint(kb) | ((uint32_t)g << 2);     // local index 16t + 4g + reg
    kbits = lane_min_x32(lane_min_x16(kbits));                      // (positive floats: integer order)
    if (g == 0) ms[16 * j + r] = kbits;
  };

  if (wid == C::FIN) offsets(0);
  for (int64_t i = 0; i < cnt; ++i) {
    // super-block i landed: each DMA wave waits for its own instructions of i (those issued a
    // step ago may stay in flight), then the barrier publishes them, the merge slots and offsets
    if (wid != C::FIN) {
      const int ahead = (i + 1 < cnt ? C::dma_x(wid) : 0) + (wid == XNW ? 1 : 0);
      wait_vm_n<3>(ahead);
    }
    wait_lgkm0();
    raw_barrier();
    if (wid != C::FIN) {
      if (i + 2 < cnt) issue_x(i + 2);   // (slot (i+2) % NB was last read at step i-1)
      if (wid == XNW) issue_xn(i + 3);   // (slot (i+3) % NXB: none of i-1 .. i+2)
    } else {
      // the finisher: old labels of super-block i for the next step, super-block i-1's outputs,
      // super-block i+1's offsets (its norms landed with this step's wait)
      int64_t r0;
      const int64_t nv = sb_rows(i, r0);
      const int prev_old = oldl;
      oldl = lane < nv ? a.labels[r0 + lane] : -2;
      if (i > 0) finish(i - 1, prev_old);
      if (i + 1 < cnt) offsets(i + 1);
    }
    if (tw > 0) {
      const char* slot = ring + (int)(i % C::NB) * C::SLOT;
      uint32_t* ms = mrg + (int)(i & 1) * C::NW * C::SPTS + wid * C::SPTS;
      const float* xb = xnr + (int)(i % C::NXB) * C::SPTS;
      const float off = offl[(int)(i & 3)];
      // this wave's seeds per tile in LDS (not registers: the centre fragments fill those):
      // fl(|c|^2 + o) with the shared offset, |c|^2 for per-point offsets, PAD past Kpad
      f32x4* sdw = sdl + wid * T * 64 + lane;
#pragma unroll
      for (int t = 0; t < T; ++t) {
        f32x4 c = f32x4{PAD_SCORE, PAD_SCORE, PAD_SCORE, PAD_SCORE};
        if (t < tw) {
          c = *(const f32x4*)(cnl + (wid * T + t) * 16 + 4 * g);
          if (off >= 0.f) seed_add(c, off);
        }
        sdw[t * 64] = c;
      }
      if (off >= 0.f) {
#pragma unroll
        for (int j = 0; j < C::SB; ++j) block(std::false_type{}, slot, xb, sdw, ms, j);
      } else {
#pragma unroll
        for (int j = 0; j < C::SB; ++j) block(std::true_type{}, slot, xb, sdw, ms, j);
      }
    }
  }
  // the last super-block: every wave's merges, then the finisher's outputs and the totals
  wait_lgkm0();
  raw_barrier();
  if (wid == C::FIN) {
    finish(cnt - 1, oldl);
    if (a.slots) {
      const double di = wave_sum(inert);
      const int dc = wave_sum(changed);
      if (lane == 0) {
        double* sl = a.slots + (blockIdx.x % NSLOT) * SLOT_STRIDE;
        atomicAdd(sl + 0, di);
        atomicAdd(sl + 1, (double)dc);
      }
    }
  }
}

template <int DPAD>
static hipError_t launch_cs_t(const AssignArgs& a, hipStream_t s) {
  using C = CsCfg<DPAD>;
  const size_t lds = (size_t)C::NB * C::SLOT + C::NXB * C::SPTS * 4 + 2 * C::NW * C::SPTS * 4 + C::NW * C::T * 64 * 16 +
                     16 + (size_t)a.Kpad * 4;
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)assign_cs_kernel<DPAD>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    attr = true;
  }
  static int cus = [] {
    int dev = 0, n = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    return n;
  }();
  const int64_t nsb = (a.N + C::SPTS - 1) / C::SPTS;
  if (nsb <= 0) return hipSuccess;
  const unsigned grid = (unsigned)(nsb < cus ? nsb : cus);
  hipLaunchKernelGGL(assign_cs_kernel<DPAD>, dim3(grid), dim3(1024), lds, s, a);
  return hipGetLastError();
}

// Whether the centre-stationary kernel takes a call (bf16, 128 / 256 features, the centres
// fit in registers, a plain full pass with row norms); variant V_ASSIGN_CS = 1 selects it.
bool assign_cs_eligible(int dtype, int dpad, int kpad) {
  if (dtype != DT_BF16) return false;
  if (dpad == 128) return kpad <= CsCfg<128>::KCS;
  if (dpad == 256) return kpad <= CsCfg<256>::KCS;
  return false;
}

bool assign_cs_takes(int dtype, int dpad, const AssignArgs& a) {
  // (a split_keys scratch is only an offer: the streaming launcher splits small batches)
  return assign_cs_eligible(dtype, dpad, a.Kpad) && a.Kpad % 16 == 0 && a.xn && a.labels && !a.rows && !a.ub &&
         !a.n_dev && !a.oseed && !a.scatter;
}

hipError_t launch_assign_cs(int dpad, const AssignArgs& a, hipStream_t s) {
  if (!assign_cs_takes(DT_BF16, dpad, a)) return hipErrorInvalidValue;
  if (dpad == 128) return launch_cs_t<128>(a, s);
  if (dpad == 256) return launch_cs_t<256>(a, s);
  return hipErrorInvalidValue;
}

}  // namespace mk
