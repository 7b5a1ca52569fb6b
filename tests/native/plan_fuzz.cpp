// Host sanitizer harness for the launch planning of csrc/plan.h (built by
// tests/test_native_host.py with -fsanitize=address,undefined).  Sweeps K in [1, 2^20],
// D in [1, 256] and N over 1 .. 2^34, and checks every invariant the kernels rely on;
// prints "ok <cases>" or the first violation.
#include <stdio.h>
#include <stdlib.h>

#include <random>
#include <vector>

#include "plan.h"

using namespace mk::plan;

static int fail(const char* what, long long a, long long b, long long c) {
  printf("FAIL %s %lld %lld %lld\n", what, a, b, c);
  return 1;
}

int main() {
  std::mt19937_64 rng(12345);
  long long cases = 0;
  std::vector<int> Ks;
  for (int k = 1; k <= 4096; ++k) Ks.push_back(k);
  for (int k = 4097; k <= (1 << 20); k += 1 + (int)(rng() % 997)) Ks.push_back(k);
  Ks.push_back(1 << 20);
  for (int K : Ks) {
    for (int D = 1; D <= 256; D += (K > 4096 ? 7 : 1)) {
      for (int es : {2, 4}) {
        for (int w = 0; w < 2; ++w) {
          for (int max_sw : {0, 8, 16}) {
            int ldc = -1;
            const int sw = choose_sw(es, K, D, w, max_sw, &ldc);
            ++cases;
            if (sw == 0) continue;
            if (sw < 2 || sw > 64 || (sw & (sw - 1))) return fail("sw pow2", K, D, sw);
            if (max_sw && sw > max_sw) return fail("sw cap", K, D, sw);
            if (ldc != sw / 2 && ldc != sw / 2 + 1) return fail("ldc", K, sw, ldc);
            if (upd_lds_bytes(K, ldc, w) > UPD_LDS_MAX) return fail("lds", K, sw, ldc);
            if ((D * es) % 4 || D % 2) return fail("odd D accepted", K, D, es);
            for (long long N : {1LL, 255LL, 256LL, 4097LL, 1000000LL, 100000000LL, 1LL << 34}) {
              const int nc = update_n_chunks(sw, D, N);
              if (nc < 8 || nc % 8) return fail("n_chunks", N, D, nc);
              const long long rpc = (N + nc - 1) / nc;
              if (rpc * nc < N) return fail("chunk cover", N, nc, rpc);
              const long long slab = (long long)nc * K * (long long)D;   // int64 slab entries
              if (slab <= 0) return fail("slab size", nc, K, D);
            }
          }
        }
      }
      for (int es : {2, 4}) {   // K-split M-step plan
        KsPlan kp{};
        ++cases;
        if (!choose_ks(es, K, D, &kp)) continue;
        const int v = 16 / es;
        if (kp.ks < 2 || kp.ks > 64 || (kp.ks & (kp.ks - 1))) return fail("ks pow2", K, D, kp.ks);
        if ((long long)kp.kq * kp.ks < K || (long long)kp.kq * (kp.ks / 2) >= K) return fail("kq cover", K, kp.ks, kp.kq);
        if (kp.lpr < 8 || kp.lpr > 64 || (kp.lpr & (kp.lpr - 1))) return fail("lpr", D, es, kp.lpr);
        if (kp.lpr * v < D || (kp.lpr / 2) * v >= D) return fail("lpr cover", D, es, kp.lpr);
        if (kp.ldc != kp.lpr * v / 2 + 1 || kp.ldc % 2 == 0) return fail("ks ldc", D, es, kp.ldc);
        if (ks_lds_bytes(kp.kq, kp.ldc) > UPD_LDS_MAX) return fail("ks lds", K, D, kp.kq);
        if (kp.gm != 2 && kp.gm != 3 && kp.gm != 6) return fail("ks gm", K, D, kp.gm);
        for (int ncs : {8, 32, 64, 128}) {
          const int nc = update_n_chunks_ks(kp.ks, ncs);
          if (nc % 8 || nc < ncs || (long long)nc * kp.ks < 256) return fail("ks n_chunks", kp.ks, ncs, nc);
        }
      }
      for (int es : {2, 4}) {
        for (int dpad : {8, 16, 32, 64, 128, 256, 512}) {
          const int kp = assign_kpad(es, dpad, K);
          const int ct = assign16_chunk_tiles(es, dpad);
          ++cases;
          if (ct == 0) { if (kp != 0) return fail("kpad unsupported", es, dpad, kp); continue; }
          if (kp < K || kp % (16 * ct) || kp - K >= 16 * ct) return fail("kpad", K, dpad, kp);
          const long long cn = assign_cn_len(kp);
          if (cn < kp || cn % 256) return fail("cn_len", kp, cn, 0);
          if ((long long)kp * dpad * es <= 0) return fail("pack bytes", kp, dpad, es);
          if (16 * dpad * es * ct > 16384 && ct > 1) return fail("chunk bytes", dpad, es, ct);
        }
      }
    }
  }
  std::uniform_real_distribution<double> u(-1100.0, 1100.0);
  for (int i = 0; i < 200000; ++i) {
    double m = (i % 3 == 0) ? ldexp(1.0, (int)(rng() % 300) - 150) : exp2(u(rng));
    if (i % 7 == 0) m = nextafter(m, 0.0);
    if (!isfinite(m) || m == 0.0) continue;  // non-finite / zero bounds: exponent 0 by definition (edge list below)
    const int e = fixed_exp(m);
    ++cases;
    if (e < -126 || e > 126) return fail("exp range", i, e, 0);
    const double q = ldexp(m, e);
    if (e > -126 && q > ldexp(1.0, FX_BITS)) return fail("exp too big", i, e, 0);
    if (e < 126 && isfinite(q) && q > 0 && ldexp(m, e + 1) <= ldexp(1.0, FX_BITS)) return fail("exp not max", i, e, 0);
  }
  for (double m : std::initializer_list<double>{0.0, -1.0, HUGE_VAL, -HUGE_VAL, (double)NAN, 5e-324, 1.7976931348623157e308}) {
    const int e = fixed_exp(m);
    if (e < -126 || e > 126) return fail("exp edge", 0, e, 0);
  }
  printf("ok %lld\n", cases);
  return 0;
}
