// A/B harness for the assign (E-step) kernel: the production assign16_kernel against
// experimental variants, on bf16 blob data, one process, interleaved rounds.
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form=1 \
//          -I mikmeans/csrc scripts/microbench/assign_ab.hip -o build/assign_ab
// run:   build/assign_ab N D K [rounds reps]
// Prints one line per variant: median / min ms, TF/s, label mismatches vs production.
#include "../../mikmeans/csrc/assign16.hip"

#include <algorithm>
#include <string.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#include "assign_x.h"
#include "assign_copy.h"

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                             \
    }                                                                                      \
  } while (0)

__device__ __forceinline__ uint32_t hsh(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16; return x;
}
__device__ __forceinline__ float unif(uint32_t h) { return (h >> 8) * (1.0f / 16777216.0f); }

// x[i][d] = centre[i % NB][d] + (sum of 4 uniforms - 2) * 1.7  (blob-like, bf16)
__global__ void gen_kernel(uint16_t* X, int64_t N, int D, int NB, int64_t i0) {
  const int64_t i = i0 + blockIdx.x;
  const int b = (int)(hsh((uint32_t)i * 2654435761u) % (uint32_t)NB);
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    const float c = (unif(hsh(b * 7919u + d * 104729u + 17u)) - 0.5f) * 20.f;
    uint32_t h = hsh(hsh((uint32_t)i ^ 0x9e3779b9u) + (uint32_t)d * 0x85ebca6bu);
    float n = unif(h) + unif(hsh(h + 1)) + unif(hsh(h + 2)) + unif(hsh(h + 3)) - 2.f;
    X[(int64_t)blockIdx.x * D + d] = mk::f32_to_bf16(c + 1.7f * n);
  }
}
__global__ void sqnorm_kernel(const uint16_t* X, int64_t N, int D, float* xn) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  float s = 0.f;
  for (int d = 0; d < D; ++d) { const float v = mk::bf16_to_f32(X[i * D + d]); s = fmaf(v, v, s); }
  xn[i] = s;
}

static float bf2f(uint16_t h) { uint32_t u = (uint32_t)h << 16; float f; memcpy(&f, &u, 4); return f; }
static uint16_t f2bf(float f) {
  uint32_t u; memcpy(&u, &f, 4); u += 0x7fffu + ((u >> 16) & 1u); return (uint16_t)(u >> 16);
}

typedef hipError_t (*LaunchFn)(const mk::AssignArgs&, hipStream_t);
struct Variant { const char* name; LaunchFn fn; };

static void* g_pack2 = nullptr;  // centres in the production layout (old copies read the old one)
static hipError_t v_prod128(const mk::AssignArgs& a, hipStream_t s) {
  mk::AssignArgs b = a; b.Cpack = g_pack2;
  return mk::launch_assign16(mk::DT_BF16, 128, b, s);
}
static double* g_slots = nullptr;
// the Lloyd engine's call: previous labels read (changed count), inertia/changed slots
static hipError_t v_prod128_lloyd(const mk::AssignArgs& a, hipStream_t s) {
  mk::AssignArgs b = a; b.Cpack = g_pack2; b.track_changed = 1; b.slots = g_slots;
  return mk::launch_assign16(mk::DT_BF16, 128, b, s);
}
static hipError_t v_prod128_lloyd_nomind(const mk::AssignArgs& a, hipStream_t s) {
  mk::AssignArgs b = a; b.Cpack = g_pack2; b.track_changed = 1; b.slots = g_slots; b.mind = nullptr;
  return mk::launch_assign16(mk::DT_BF16, 128, b, s);
}
static hipError_t v_prod128_nomind(const mk::AssignArgs& a, hipStream_t s) {
  mk::AssignArgs b = a; b.Cpack = g_pack2; b.mind = nullptr;
  return mk::launch_assign16(mk::DT_BF16, 128, b, s);
}
static hipError_t v_prod64(const mk::AssignArgs& a, hipStream_t s) {
  mk::AssignArgs b = a; b.Cpack = g_pack2;
  return mk::launch_assign16(mk::DT_BF16, 64, b, s);
}
static hipError_t v_prod256(const mk::AssignArgs& a, hipStream_t s) {
  mk::AssignArgs b = a; b.Cpack = g_pack2;
  return mk::launch_assign16(mk::DT_BF16, 256, b, s);
}

int main(int argc, char** argv) {
  const int64_t N = argc > 1 ? atoll(argv[1]) : 20000000;
  const int D = argc > 2 ? atoi(argv[2]) : 128;
  const int K = argc > 3 ? atoi(argv[3]) : 1024;
  const int rounds = argc > 4 ? atoi(argv[4]) : 5;
  const int reps = argc > 5 ? atoi(argv[5]) : 10;
  const int zero = argc > 6 ? atoi(argv[6]) : 0;  // 1: all-zero X (DVFS probe)
  if (N % 1536 != 0 || K % 64 != 0 || (D != 64 && D != 128 && D != 256)) {
    fprintf(stderr, "need N %% 1536 == 0, K %% 64 == 0, D in {64,128,256}\n");
    return 2;
  }
  const int Kpad = mk::assign_kpad(mk::DT_BF16, D, K);
  uint16_t* X; float* xn; int32_t* labels; int32_t* ref; float* mind; uint16_t* pack; float* cn;
  CK(hipMalloc(&X, N * D * 2));
  CK(hipMalloc(&xn, N * 4));
  CK(hipMalloc(&labels, N * 4));
  CK(hipMalloc(&ref, N * 4));
  CK(hipMalloc(&mind, N * 4));
  const int cnl = mk::assign_cn_len(Kpad);
  CK(hipMalloc(&pack, (size_t)Kpad * D * 2));
  CK(hipMalloc(&cn, cnl * 4));
  for (int64_t i0 = 0; i0 < N; i0 += (1 << 24)) {  // (grid <= 2^32 threads)
    const int64_t n = std::min<int64_t>(1 << 24, N - i0);
    gen_kernel<<<dim3((unsigned)n), 64>>>(X + i0 * D, n, D, 4096, i0);
  }
  if (zero) CK(hipMemset(X, 0, N * D * 2));
  sqnorm_kernel<<<dim3((unsigned)((N + 255) / 256)), 256>>>(X, N, D, xn);
  CK(hipDeviceSynchronize());
  {
    std::vector<float> hx(N);
    CK(hipMemcpy(hx.data(), xn, N * 4, hipMemcpyDeviceToHost));
    double s = 0; int64_t z = 0; float mn = 3e38f, mx = 0;
    for (int64_t i = 0; i < N; ++i) { s += hx[i]; z += hx[i] == 0; mn = std::min(mn, hx[i]); mx = std::max(mx, hx[i]); }
    printf("data: mean |x|^2 %.3f min %.3f max %.3f zero rows %lld (tail mean %.3f)\n", s / N, mn, mx, (long long)z,
           (double)hx[N - 1] + hx[N / 2]);
  }
  // centres: K pseudo-random rows of X
  std::vector<uint16_t> C((size_t)K * D), row(D);
  for (int k = 0; k < K; ++k) {
    const int64_t i = (int64_t)((1103515245ull * (k + 1) + 12345ull) % (uint64_t)N);
    CK(hipMemcpy(row.data(), X + i * D, D * 2, hipMemcpyDeviceToHost));
    for (int d = 0; d < D; ++d) C[(size_t)k * D + d] = row[d];
  }
  // layout 16: offset = ((t*NQ + e/V)*64 + r + 16*g)*V + e%V, value -2c; cn = |c|^2 (f32)
  const int V = 8, NQ = D / 4 / V;
  std::vector<uint16_t> hp((size_t)Kpad * D, 0), hp2((size_t)Kpad * D, 0);
  std::vector<float> hcn(cnl, mk::PAD_SCORE);
  for (int k = 0; k < K; ++k) {
    double s = 0;
    for (int d = 0; d < D; ++d) {
      const float c = bf2f(C[(size_t)k * D + d]);
      s += (double)c * c;
      const int t = k / 16, r = k % 16, g = d / (D / 4), e = d % (D / 4);
      const size_t off = ((size_t)(t * NQ + e / V) * 64 + r + 16 * g) * V + e % V;
      hp[off] = f2bf(-2.f * c);
      // production layout: piece q of lane group g holds features [(4q+g)V, +V)
      const int q2 = d / (4 * V), g2 = (d / V) & 3;
      hp2[((size_t)(t * NQ + q2) * 64 + r + 16 * g2) * V + d % V] = f2bf(-2.f * c);
    }
    hcn[k] = (float)s;
  }
  CK(hipMemcpy(pack, hp.data(), hp.size() * 2, hipMemcpyHostToDevice));
  CK(hipMalloc(&g_pack2, (size_t)Kpad * D * 2));
  CK(hipMemcpy(g_pack2, hp2.data(), hp2.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(cn, hcn.data(), cnl * 4, hipMemcpyHostToDevice));

  mk::AssignArgs a{};
  a.X = X; a.N = N; a.D = D; a.ldx = D; a.Cpack = pack; a.cn = cn; a.Kpad = Kpad;
  a.xn = xn; a.labels = labels; a.mind = mind; a.slots = nullptr; a.track_changed = 0;

  std::vector<Variant> vs;
  CK(hipMalloc(&g_slots, mk::NSLOT * mk::SLOT_STRIDE * 8));
  CK(hipMemset(g_slots, 0, mk::NSLOT * mk::SLOT_STRIDE * 8));
  if (D == 128) {
    vs.push_back({"prod", v_prod128});
  }
  if (D == 64) vs.push_back({"prod", v_prod64});
  if (D == 256) vs.push_back({"prod", v_prod256});
  mkx::add_variants(D, vs);
  if (D == 64) vs.push_back({"old_head", mkc::launch_old<64, 8, 8, 3>});
  if (D == 256) vs.push_back({"old_head", mkc::launch_old<256, 3, 2, 3>});
  if (D == 128) vs.push_back({"old_head", mkc::launch_old<128, 4, 4, 4>});
  vs.push_back({"prod_again", vs[0].fn});

  // reference labels
  mk::AssignArgs ar = a; ar.labels = ref;
  CK(vs[0].fn(ar, 0));
  CK(hipDeviceSynchronize());
  std::vector<int32_t> href(N), hl(N);
  CK(hipMemcpy(href.data(), ref, N * 4, hipMemcpyDeviceToHost));
  std::vector<float> mref(N), ml(N);
  CK(hipMemcpy(mref.data(), mind, N * 4, hipMemcpyDeviceToHost));
  std::vector<std::vector<float>> times(vs.size());
  std::vector<long> mism(vs.size(), 0);
  for (size_t v = 0; v < vs.size(); ++v) {
    if (strstr(vs[v].name, "gate")) CK(hipMemcpy(labels, ref, N * 4, hipMemcpyDeviceToDevice));
    else CK(hipMemset(labels, 0xff, N * 4));
    CK(vs[v].fn(a, 0));
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(hl.data(), labels, N * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(ml.data(), mind, N * 4, hipMemcpyDeviceToHost));
    int shown = 0;
    int64_t huge = 0;
    for (int64_t i = 0; i < N; ++i) {
      huge += ml[i] > 1e29f;
      if (hl[i] != href[i]) {
        ++mism[v];
        if (shown < 4 && strstr(vs[v].name, "gate")) {
          printf("  %s row %lld: label %d (d %.4f) vs prod %d (d %.4f)\n", vs[v].name, (long long)i, hl[i], ml[i],
                 href[i], mref[i]);
          ++shown;
        }
      }
    }
    if (huge) printf("  %s: %lld rows with d > 1e29\n", vs[v].name, (long long)huge);
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int r = 0; r < rounds; ++r)
    for (size_t v = 0; v < vs.size(); ++v)
      for (int i = 0; i < reps; ++i) {
        CK(hipEventRecord(e0, 0));
        CK(vs[v].fn(a, 0));
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        times[v].push_back(ms);
      }
  unsigned long long* stamps;
  const int64_t nblk_max = N / 64 + 1;
  CK(hipMalloc(&stamps, nblk_max * 16));
  for (size_t v = 0; v < vs.size(); ++v) {
    if (!strstr(vs[v].name, "_st")) continue;
    CK(hipMemset(stamps, 0, nblk_max * 16));
    // warm the clock up, then one stamped launch
    for (int i = 0; i < 20; ++i) CK(vs[v].fn(a, 0));
    mk::AssignArgs as = a; as.split_keys = stamps;
    CK(vs[v].fn(as, 0));
    CK(hipDeviceSynchronize());
    std::vector<unsigned long long> hs(nblk_max * 2);
    CK(hipMemcpy(hs.data(), stamps, nblk_max * 16, hipMemcpyDeviceToHost));
    std::vector<double> clk;
    for (int64_t b = 0; b < nblk_max; ++b)
      if (hs[2 * b + 1] > 0) clk.push_back((double)hs[2 * b] / (double)hs[2 * b + 1] * 100.0);
    std::sort(clk.begin(), clk.end());
    if (!clk.empty())
      printf("%-16s in-kernel clock: median %.0f MHz (p10 %.0f, p90 %.0f) over %zu workgroups\n", vs[v].name,
             clk[clk.size() / 2], clk[clk.size() / 10], clk[clk.size() * 9 / 10], clk.size());
  }
  for (size_t v = 0; v < vs.size(); ++v) {
    auto t = times[v];
    std::sort(t.begin(), t.end());
    const double med = t[t.size() / 2];
    printf("N=%lld D=%d K=%d %-14s median %.4f ms  min %.4f ms  %.1f TF/s  mismatches %ld\n", (long long)N, D, K,
           vs[v].name, med, t[0], 2.0 * N * K * D / (med * 1e-3) / 1e12, mism[v]);
  }
  fflush(stdout);
  return 0;
}
