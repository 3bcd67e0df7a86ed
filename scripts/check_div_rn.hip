// Host check of div_rn (cwq_refmath.h) against IEEE float division: every positive and
// negative float dividend for a set of divisors (the fitters' counts and variance-like
// values), then random pairs over the whole guarded range and near-midpoint pairs.
//   hipcc -O2 -std=c++17 scripts/check_div_rn.hip -o /tmp/check_div_rn -lpthread
#include <atomic>
#include <random>
#include <stdio.h>
#include <thread>
#include <vector>
#include "../rag-cobweb_amd/csrc/cwq_refmath.h"

static bool same(float x, float y) { return __builtin_bit_cast(uint32_t, x) == __builtin_bit_cast(uint32_t, y); }

int main(int argc, char** argv) {
  const int T = 8;
  const long long nrand = argc > 1 ? atoll(argv[1]) : 400000000LL;
  std::atomic<long long> bad{0}, checked{0};
  const float divs[] = {1.f, 2.f, 3.f, 7.f, 10.f, 13.f, 255.f, 1000.f, 65537.f, 16777215.f, 0.0585498f,
                        0.3f, 1.7320508f, 123.456f, 3.0e-5f, 8.5e7f, 0x1.fffffep+3f, 0x1.000002p+0f};
  auto run = [&](auto body) {
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t) th.emplace_back(body, t);
    for (auto& x : th) x.join();
  };
  // every dividend (both signs, all finite bit patterns) for each divisor
  for (float b : divs) {
    const float y = cwq::div_recip(b);
    run([&, b, y](int t) {
      long long nb = 0, nc = 0;
      for (uint32_t u = (uint32_t)t; u < 0x7f800000u; u += T)
        for (int sg = 0; sg < 2; ++sg) {
          const float a = __builtin_bit_cast(float, u | (sg ? 0x80000000u : 0u));
          ++nc;
          if (!same(cwq::div_rn(a, b, y), a / b)) {
            if (nb < 5) fprintf(stderr, "mismatch %a / %a: %a vs %a\n", a, b, cwq::div_rn(a, b, y), a / b);
            ++nb;
          }
        }
      bad += nb;
      checked += nc;
    });
  }
  // random (a, b) over [2^-70, 2^70] magnitudes, random signs; and a near a midpoint of b's
  // quotients: a = fl(b * m) for a midpoint m between two adjacent floats
  run([&](int t) {
    std::mt19937_64 g(1234 + t);
    long long nb = 0, nc = 0;
    for (long long i = t; i < nrand; i += T) {
      const uint32_t eb = 127 - 70 + (uint32_t)(g() % 141), ea = 127 - 70 + (uint32_t)(g() % 141);
      const float b = __builtin_bit_cast(float, (eb << 23) | (uint32_t)(g() & 0x7fffffu));
      float a;
      if (i & 1) {
        a = __builtin_bit_cast(float, (ea << 23) | (uint32_t)(g() & 0x7fffffu) | ((uint32_t)(g() & 1) << 31));
      } else {
        const float q = __builtin_bit_cast(float, ((127u - 20 + (uint32_t)(g() % 41)) << 23) | (uint32_t)(g() & 0x7fffffu));
        const double m = ((double)q + (double)nextafterf(q, INFINITY)) * 0.5;
        a = (float)((double)b * m);
      }
      const float y = cwq::div_recip(b);
      ++nc;
      if (!same(cwq::div_rn(a, b, y), a / b)) {
        if (nb < 5) fprintf(stderr, "mismatch %a / %a: %a vs %a\n", a, b, cwq::div_rn(a, b, y), a / b);
        ++nb;
      }
    }
    bad += nb;
    checked += nc;
  });
  printf("div_rn vs IEEE division: %lld pairs, %lld mismatches\n", (long long)checked, (long long)bad);
  return bad ? 1 : 0;
}
