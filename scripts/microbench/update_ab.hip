// A/B harness for the M-step scatter-add (update_kernel): production against an
// experimental copy (update_x.hip: MODE bit 256 drops the per-period barrier and flush
// check, bit 512 drops the LDS adds), plus variants of the copy's NT / ring depth /
// period, on bf16 blob-like data with random labels (one process, interleaved rounds).
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I mikmeans/csrc \
//          scripts/microbench/update_ab.hip -o scripts/microbench/bin/update_ab
// run:   update_ab N D K [rounds reps]
#include "../../mikmeans/csrc/update.hip"
#include "update_x.hip"

#include <algorithm>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

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
template <typename T>
__global__ void gen_kernel(T* X, int32_t* lab, int64_t i0, int D, int K) {
  const int64_t i = i0 + blockIdx.x;
  const uint32_t b = hsh((uint32_t)i * 2654435761u);
  if (threadIdx.x == 0) lab[blockIdx.x] = (int32_t)(b % (uint32_t)K);
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    const float c = (unif(hsh((b % 4096u) * 7919u + d * 104729u + 17u)) - 0.5f) * 20.f;
    const uint32_t h = hsh(hsh((uint32_t)i ^ 0x9e3779b9u) + (uint32_t)d * 0x85ebca6bu);
    const float n = unif(h) + unif(hsh(h + 1)) + unif(hsh(h + 2)) + unif(hsh(h + 3)) - 2.f;
    if constexpr (sizeof(T) == 2) X[(int64_t)blockIdx.x * D + d] = mk::f32_to_bf16(c + 1.7f * n);
    else X[(int64_t)blockIdx.x * D + d] = c + 1.7f * n;
  }
}

typedef hipError_t (*Fn)(const mk::UpdateArgs&, int, hipStream_t);
struct Var { const char* name; Fn fn; };

static int g_dt = mk::DT_BF16;
static hipError_t prod(const mk::UpdateArgs& a, int, hipStream_t s) { return mk::launch_update(g_dt, a, s); }
template <int MODE, int NT, int NBF, int PER, int SW = 32, typename T = uint16_t>
static hipError_t xv(const mk::UpdateArgs& a, int ldc, hipStream_t s) {
  return mku::launch_nt<T, SW, MODE, NT, NBF, PER>(a, ldc, s);
}

static int g_K = 0, g_D = 0;
template <int LPR, int GM, int KS>
static hipError_t ksv(const mk::UpdateArgs& a, int, hipStream_t s) {
  mk::plan::KsPlan kp{};
  kp.ks = KS; kp.kq = (a.K + KS - 1) / KS; kp.lpr = LPR; kp.ldc = LPR * 8 / 2 + 1; kp.gm = GM;
  if (mk::plan::ks_lds_bytes(kp.kq, kp.ldc) > mk::plan::UPD_LDS_MAX) return hipErrorInvalidValue;
  mk::UpdateArgs b = a;
  b.n_chunks = ((256 / KS + 7) / 8) * 8 > a.n_chunks ? ((256 / KS + 7) / 8) * 8 : a.n_chunks;
  return mku::launch_ks_t<uint16_t, LPR, GM, false>(b, kp, s);
}

// the production K-split kernel (pair x lanes cell layout) at other row-group depths
template <int LPR, int GM, int KS>
static hipError_t ksn(const mk::UpdateArgs& a, int, hipStream_t s) {
  mk::plan::KsPlan kp{};
  kp.ks = KS; kp.kq = (a.K + KS - 1) / KS; kp.lpr = LPR; kp.ldc = LPR * 8 / 2 + 1; kp.gm = GM;
  if (mk::plan::ks_lds_bytes(kp.kq, kp.ldc) > mk::plan::UPD_LDS_MAX) return hipErrorInvalidValue;
  mk::UpdateArgs b = a;
  b.n_chunks = ((256 / KS + 7) / 8) * 8 > a.n_chunks ? ((256 / KS + 7) / 8) * 8 : a.n_chunks;
  return mk::launch_ks_t<uint16_t, LPR, GM, false>(b, kp, s);
}

int main(int argc, char** argv) {
  const int64_t N = argc > 1 ? atoll(argv[1]) : 100000000;
  const int D = argc > 2 ? atoi(argv[2]) : 128;
  const int K = argc > 3 ? atoi(argv[3]) : 1024;
  const int rounds = argc > 4 ? atoi(argv[4]) : 4;
  const int reps = argc > 5 ? atoi(argv[5]) : 5;
  const bool f32 = argc > 6 && atoi(argv[6]) == 1;
  g_dt = f32 ? mk::DT_F32 : mk::DT_BF16;
  const int es = f32 ? 4 : 2;
  int ldc = 0;
  const int sw = mk::plan::choose_sw(es, K, D, false, 0, &ldc);
  printf("slice width %d, n_chunks from production %d\n", sw, mk::update_n_chunks(g_dt, K, D, N));
  const int nc = mk::update_n_chunks(g_dt, K, D, N);
  void* X; int32_t* lab; long long *slab, *cnt; int* cexp;
  CK(hipMalloc(&X, N * D * es));
  CK(hipMalloc(&lab, N * 4));
  CK(hipMalloc(&slab, (size_t)nc * K * D * 8));
  CK(hipMalloc(&cnt, (size_t)nc * K * 8));
  CK(hipMalloc(&cexp, D * 4));
  for (int64_t i0 = 0; i0 < N; i0 += (1 << 24)) {
    const int64_t n = std::min<int64_t>(1 << 24, N - i0);
    if (f32) gen_kernel<float><<<dim3((unsigned)n), 64>>>((float*)X + i0 * D, lab + i0, i0, D, K);
    else gen_kernel<uint16_t><<<dim3((unsigned)n), 64>>>((uint16_t*)X + i0 * D, lab + i0, i0, D, K);
  }
  std::vector<int> he(D, mk::plan::fixed_exp(16.0));
  CK(hipMemcpy(cexp, he.data(), D * 4, hipMemcpyHostToDevice));
  CK(hipDeviceSynchronize());
  mk::UpdateArgs a{};
  a.X = X; a.N = N; a.D = D; a.ldx = D; a.labels = lab; a.K = K; a.n_chunks = nc;
  a.slab = slab; a.cnt_slab = cnt; a.weights = nullptr; a.col_exp = cexp; a.cnt_exp = 0; a.clamp = 0;

  std::vector<Var> vs;
  vs.push_back({"prod", prod});
  // the column-slice kernel as production had it before the K-split kernel
  if (!f32 && sw == 32) vs.push_back({"slice_old", xv<0, 1024, 6, 512, 32>});
  if (!f32 && D == 128 && K == 1024) {
    vs.push_back({"ks4_gm6", ksv<16, 6, 4>});
    vs.push_back({"ks4_gm8", ksv<16, 8, 4>});
    vs.push_back({"ks4_gm4", ksv<16, 4, 4>});
    vs.push_back({"ks8_gm3", ksv<16, 3, 8>});
    vs.push_back({"ks8_gm6", ksv<16, 6, 8>});
    vs.push_back({"new_gm4", ksn<16, 4, 4>});
    vs.push_back({"new_gm6", ksn<16, 6, 4>});
    vs.push_back({"new_gm8", ksn<16, 8, 4>});
    vs.push_back({"new_gm10", ksn<16, 10, 4>});
  }
  if (!f32 && D == 64 && K == 4096) {
    vs.push_back({"ks8_gm3", ksv<8, 3, 8>});
    vs.push_back({"ks8_gm2", ksv<8, 2, 8>});
    vs.push_back({"ks16_gm2", ksv<8, 2, 16>});
    vs.push_back({"new_ks8_gm2", ksn<8, 2, 8>});
    vs.push_back({"new_ks8_gm3", ksn<8, 3, 8>});
    vs.push_back({"new_ks8_gm4", ksn<8, 4, 8>});
  }
  if (!f32 && sw == 64) vs.push_back({"slice_old", xv<0, 1024, 3, 512, 64>});
  if (!f32 && sw == 8) vs.push_back({"slice_old", xv<4, 1024, 6, 1024, 8>});
  if (f32 && sw == 64) vs.push_back({"slice_old", xv<0, 1024, 2, 512, 64, float>});
  // reference: column sums over all chunks
  auto totals = [&](std::vector<long long>& t) {
    std::vector<long long> h((size_t)nc * K * D);
    CK(hipMemcpy(h.data(), slab, h.size() * 8, hipMemcpyDeviceToHost));
    t.assign((size_t)K * D, 0);
    for (int c = 0; c < nc; ++c)
      for (size_t e = 0; e < (size_t)K * D; ++e) t[e] += h[(size_t)c * K * D + e];
  };
  std::vector<long long> ref, got;
  CK(vs[0].fn(a, ldc, 0));
  CK(hipDeviceSynchronize());
  totals(ref);
  for (size_t v = 1; v < vs.size(); ++v) {
    if (strstr(vs[v].name, "nolds")) continue;
    CK(vs[v].fn(a, ldc, 0));
    CK(hipDeviceSynchronize());
    totals(got);
    size_t bad = 0;
    for (size_t e = 0; e < ref.size(); ++e) bad += got[e] != ref[e];
    printf("%-16s sums differing from production: %zu of %zu\n", vs[v].name, bad, ref.size());
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<std::vector<float>> times(vs.size());
  for (int r = 0; r < rounds; ++r)
    for (size_t v = 0; v < vs.size(); ++v)
      for (int i = 0; i < reps; ++i) {
        CK(hipEventRecord(e0, 0));
        CK(vs[v].fn(a, ldc, 0));
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        times[v].push_back(ms);
      }
  for (size_t v = 0; v < vs.size(); ++v) {
    auto t = times[v];
    std::sort(t.begin(), t.end());
    const double med = t[t.size() / 2];
    printf("%s N=%lld D=%d K=%d %-16s median %.4f ms  min %.4f ms  %.0f GB/s\n", f32 ? "f32" : "bf16", (long long)N, D, K, vs[v].name, med,
           t[0], N * D * (double)es / (med * 1e-3) / 1e9);
  }
  fflush(stdout);
  return 0;
}
