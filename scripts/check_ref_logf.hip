// Exhaustive host check of ref_logf (cwq_refmath.h) against the double log rounded once, on
// every positive float bit pattern.  hipcc -O2 scripts/check_ref_logf.hip -o /tmp/check_ref_logf
#include <thread>
#include <vector>
#include <atomic>
#include <stdio.h>
#include "../rag-cobweb_amd/csrc/cwq_refmath.h"

int main() {
  const int T = 8;
  std::atomic<long long> bad{0};
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t)
    th.emplace_back([&, t] {
      long long b = 0;
      for (uint32_t u = (uint32_t)t; u < 0x7f800000u; u += T) {
        const float v = __builtin_bit_cast(float, u);
        const float a = cwq::ref_logf(v), r = (float)log((double)v);
        if (__builtin_bit_cast(uint32_t, a) != __builtin_bit_cast(uint32_t, r)) {
          if (b < 5) fprintf(stderr, "mismatch v=%a: %a vs %a\n", v, a, r);
          ++b;
        }
      }
      bad += b;
    });
  for (auto& x : th) x.join();
  printf("ref_logf vs (float)log((double)v) over all positive floats: %lld mismatches\n", (long long)bad);
  return bad ? 1 : 0;
}
