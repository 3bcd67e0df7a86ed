// libcwq: the reference's float32 arithmetic for the category-utility KL of ifit
// (CobwebTorchTree.compute_score, CobwebTorchTree.py:344-356: torch.log, .sum() on CPU
// tensors), shared by the host-driven fitter (cwq_fit.hip) and the device-resident loop
// (cwq_fitdev.hip).  Not part of the public interface.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

namespace cwq {

// The KL terms' float32 divisions.  FIT_PROBE_DIV (a timing-only variant build, never the
// product: scripts/build_variant.py) swaps them for the hardware reciprocal to bound what
// faster division could save.
#ifdef FIT_PROBE_DIV
#define CWQ_KDIV(a, b) ((a) * __builtin_amdgcn_rcpf(b))
#else
#define CWQ_KDIV(a, b) ((a) / (b))
#endif

// a / b rounded to nearest, from y = div_recip(b) (computed once per divisor): q = fl(a y),
// then two Markstein corrections q <- fl(q + r y) with r = a - b q (exact by fma).  One
// correction leaves q within (1/2 + 2^-23) ulp of a/b; with y = RN(1/b) the second returns
// RN(a/b): |fl-free q + r y - a/b| <= |a/b - q| |1 - b y| < (1/2 + 2^-23) u B 2^-48 (u the ulp of
// a/b, B the divisor's 24-bit integer significand), while a/b is never a midpoint and any
// midpoint is at least u / (2B) away (|a - b m| is a nonzero multiple of b's and m's joint
// grain), and (1 + 2^-22) B^2 < 2^48 for B <= 2^24 - 2.  So: a divisor with an all-ones
// significand (B = 2^24 - 1), or outside [2^-60, 2^60], gets y = NaN and every quotient by it
// the IEEE division; so does a dividend outside [2^-60, 2^60] (0 excepted: 0 / b = 0 with
// a's sign, which the sequence keeps).  Checked against IEEE division on host
// (scripts/check_div_rn.hip: every dividend for a set of divisors, random and near-midpoint
// pairs; tests/test_div_rn.py).
__host__ __device__ __forceinline__ float div_recip(float b) {
  const uint32_t u = __builtin_bit_cast(uint32_t, b) & 0x7fffffffu;
  const bool ok = (u & 0x007fffffu) != 0x007fffffu && u - 0x21800000u < 0x5d800000u - 0x21800000u;
  return ok ? 1.0f / b : __builtin_nanf("");
}
__host__ __device__ __forceinline__ float div_rn(float a, float b, float y) {
#pragma clang fp contract(off)
  const uint32_t ua = __builtin_bit_cast(uint32_t, a) & 0x7fffffffu;
  const bool ok = y == y && (ua == 0u || ua - 0x21800000u < 0x5d800000u - 0x21800000u);
  float q = a * y;
  float r = fmaf(b, q, -a);   // -(a - b q), exact
  q = fmaf(-r, y, q);
  r = fmaf(b, q, -a);
  q = fmaf(-r, y, q);
#ifdef __HIP_DEVICE_COMPILE__
  // the IEEE division only in a wave that has a lane outside the range (never on the data
  // the fitters see): a uniform branch, so the division's code is not run for every term
  if (__builtin_expect(__builtin_amdgcn_ballot_w64(!ok) != 0, 0))
    if (!ok) q = a / b;
#else
  if (!ok) q = a / b;
#endif
  return q;
}

// log: torch's float32 log (Sleef, 1-ulp) is the correctly rounded value for 99.96% of
// inputs; a log computed to a few double ulps and rounded once is that value.  The library's
// fp64 log was most of a clustered ifit's insert time, so: a 128-entry table on the top 7
// mantissa bits (c_i = float(1/centre_i), L_i = -ln c_i in double, less ln 2 for the upper
// half whose exponent counts one more; scripts/gen_logtab.py), r = m c_i - 1 exact in double
// (|r| <= 2^-7; the buckets either side of 1 have c = 1, 1/2 and L = 0, so r = v - 1 there),
// log(1 + r) to degree 7 (truncation < 2^-59).  Equal to (float)log((double)v)
// on every positive float (scripts/check_ref_logf.hip, exhaustive); 0, denormals, inf and NaN
// take the library log.
static constexpr float kRefLogC[128] = {
    0x1.0000000000000p+0f, 0x1.fa11ca0000000p-1f, 0x1.f6310a0000000p-1f, 0x1.f25f640000000p-1f,
    0x1.ee9c800000000p-1f, 0x1.eae8080000000p-1f, 0x1.e741aa0000000p-1f, 0x1.e3a9180000000p-1f,
    0x1.e01e020000000p-1f, 0x1.dca01e0000000p-1f, 0x1.d92f220000000p-1f, 0x1.d5cac80000000p-1f,
    0x1.d272ca0000000p-1f, 0x1.cf26e60000000p-1f, 0x1.cbe6da0000000p-1f, 0x1.c8b2660000000p-1f,
    0x1.c5894e0000000p-1f, 0x1.c26b540000000p-1f, 0x1.bf583e0000000p-1f, 0x1.bc4fd60000000p-1f,
    0x1.b951e20000000p-1f, 0x1.b65e2e0000000p-1f, 0x1.b374840000000p-1f, 0x1.b094b40000000p-1f,
    0x1.adbe880000000p-1f, 0x1.aaf1d20000000p-1f, 0x1.a82e660000000p-1f, 0x1.a574100000000p-1f,
    0x1.a2c2a80000000p-1f, 0x1.a01a020000000p-1f, 0x1.9d79f20000000p-1f, 0x1.9ae24e0000000p-1f,
    0x1.9852f00000000p-1f, 0x1.95cbb00000000p-1f, 0x1.934c680000000p-1f, 0x1.90d4f20000000p-1f,
    0x1.8e65280000000p-1f, 0x1.8bfce80000000p-1f, 0x1.899c100000000p-1f, 0x1.87427c0000000p-1f,
    0x1.84f00c0000000p-1f, 0x1.82a4a00000000p-1f, 0x1.8060180000000p-1f, 0x1.7e22560000000p-1f,
    0x1.7beb3a0000000p-1f, 0x1.79baa60000000p-1f, 0x1.7790820000000p-1f, 0x1.756cac0000000p-1f,
    0x1.734f0c0000000p-1f, 0x1.7137860000000p-1f, 0x1.6f26020000000p-1f, 0x1.6d1a620000000p-1f,
    0x1.6b14900000000p-1f, 0x1.6914740000000p-1f, 0x1.6719f40000000p-1f, 0x1.6524f80000000p-1f,
    0x1.63356c0000000p-1f, 0x1.614b360000000p-1f, 0x1.5f66440000000p-1f, 0x1.5d867c0000000p-1f,
    0x1.5babcc0000000p-1f, 0x1.59d6200000000p-1f, 0x1.5805600000000p-1f, 0x1.56397c0000000p-1f,
    0x1.54725e0000000p-1f, 0x1.52aff60000000p-1f, 0x1.50f22e0000000p-1f, 0x1.4f38f60000000p-1f,
    0x1.4d843c0000000p-1f, 0x1.4bd3ee0000000p-1f, 0x1.4a27fa0000000p-1f, 0x1.4880520000000p-1f,
    0x1.46dce40000000p-1f, 0x1.453d9e0000000p-1f, 0x1.43a2740000000p-1f, 0x1.420b520000000p-1f,
    0x1.40782e0000000p-1f, 0x1.3ee8f40000000p-1f, 0x1.3d5d9a0000000p-1f, 0x1.3bd60e0000000p-1f,
    0x1.3a52440000000p-1f, 0x1.38d22e0000000p-1f, 0x1.3755be0000000p-1f, 0x1.35dce60000000p-1f,
    0x1.34679a0000000p-1f, 0x1.32f5ce0000000p-1f, 0x1.3187760000000p-1f, 0x1.301c820000000p-1f,
    0x1.2eb4ea0000000p-1f, 0x1.2d50a00000000p-1f, 0x1.2bef980000000p-1f, 0x1.2a91ca0000000p-1f,
    0x1.2937260000000p-1f, 0x1.27dfa40000000p-1f, 0x1.268b380000000p-1f, 0x1.2539d80000000p-1f,
    0x1.23eb7a0000000p-1f, 0x1.22a0120000000p-1f, 0x1.2157980000000p-1f, 0x1.2012020000000p-1f,
    0x1.1ecf440000000p-1f, 0x1.1d8f560000000p-1f, 0x1.1c52300000000p-1f, 0x1.1b17c60000000p-1f,
    0x1.19e0120000000p-1f, 0x1.18ab080000000p-1f, 0x1.1778a20000000p-1f, 0x1.1648d60000000p-1f,
    0x1.151b9a0000000p-1f, 0x1.13f0e80000000p-1f, 0x1.12c8b80000000p-1f, 0x1.11a3020000000p-1f,
    0x1.107fbc0000000p-1f, 0x1.0f5ee00000000p-1f, 0x1.0e40660000000p-1f, 0x1.0d24460000000p-1f,
    0x1.0c0a780000000p-1f, 0x1.0af2f80000000p-1f, 0x1.09ddba0000000p-1f, 0x1.08cabc0000000p-1f,
    0x1.07b9f20000000p-1f, 0x1.06ab5a0000000p-1f, 0x1.059eea0000000p-1f, 0x1.04949c0000000p-1f,
    0x1.038c6c0000000p-1f, 0x1.0286500000000p-1f, 0x1.0182440000000p-1f, 0x1.0000000000000p-1f};
static constexpr double kRefLogL[128] = {
    0x0.0p+0, 0x1.7dc49e7810addp-7, 0x1.3cea5df46a5c8p-6, 0x1.b9fc0afaf91a1p-6,
    0x1.1b0d90923d990p-5, 0x1.58a5b57c8e4dcp-5, 0x1.95c836cc8e3f4p-5, 0x1.d276b22db0b5dp-5,
    0x1.075982498e472p-4, 0x1.253f6120a1419p-4, 0x1.42edcd9a646f2p-4, 0x1.60658ad3750c4p-4,
    0x1.7da76907b12cfp-4, 0x1.9ab42252033afp-4, 0x1.b78c7d2b0edb1p-4, 0x1.d4313a96cb361p-4,
    0x1.f0a30391162cap-4, 0x1.06714f3ca5972p-3, 0x1.14785c6e742bep-3, 0x1.2266f328a5acep-3,
    0x1.303d74c647fddp-3, 0x1.3dfc2c26cc62bp-3, 0x1.4ba37269a55f0p-3, 0x1.5933896982097p-3,
    0x1.66acd4072ad51p-3, 0x1.740f93fc037bap-3, 0x1.815c059c357ffp-3, 0x1.8e92902886d46p-3,
    0x1.9bb36547dfb89p-3, 0x1.a8becdf082f1cp-3, 0x1.b5b51740fb5abp-3, 0x1.c2968890c18cbp-3,
    0x1.cf6359209c5eep-3, 0x1.dc1bcdcabec8bp-3, 0x1.e8c0250aa5a60p-3, 0x1.f550a0ecb7b4bp-3,
    0x1.00e6c38ad501ep-2, 0x1.071b860cd590dp-2, 0x1.0d46b3d9ab750p-2, 0x1.13686fa13a8b1p-2,
    0x1.1980d34542370p-2, 0x1.1f8ffa248a2f3p-2, 0x1.2596011df763ap-2, 0x1.2b93013789d31p-2,
    0x1.31871a4144190p-2, 0x1.37726827fd863p-2, 0x1.3d54f7e81f71cp-2, 0x1.432ef2f84e814p-2,
    0x1.490068ec009d2p-2, 0x1.4ec9758200275p-2, 0x1.548a2aa6dd268p-2, 0x1.5a42ac334cfe4p-2,
    0x1.5ff308ea793dbp-2, 0x1.659b56383e1f4p-2, 0x1.6b3bb05b59444p-2, 0x1.70d42f1789238p-2,
    0x1.7664dfcb9dbd2p-2, 0x1.7bede21f7afc4p-2, 0x1.816f3fb20d49fp-2, 0x1.86e91a5b30ba1p-2,
    0x1.8c5b7dad8b48dp-2, 0x1.91c67bf45a84dp-2, 0x1.972a345135159p-2, 0x1.9c86af25c0865p-2,
    -0x1.23ec584deba46p-2, -0x1.1e9e183c899eep-2, -0x1.1956d385bc2fap-2, -0x1.14167e6767782p-2,
    -0x1.0edd064378081p-2, -0x1.09aa57a26c6d4p-2, -0x1.047e5e31e83aap-2, -0x1.feb22276a07ccp-3,
    -0x1.f474b5c4df214p-3, -0x1.ea4448d84aaf3p-3, -0x1.e020d27235a90p-3, -0x1.d60a15710350ep-3,
    -0x1.cc001295b3c2fp-3, -0x1.c20289a17f9b3p-3, -0x1.b81178d3823b1p-3, -0x1.ae2ca9be72bcdp-3,
    -0x1.a4540b3e6aafcp-3, -0x1.9a877e06baa1ep-3, -0x1.90c6e177cbcb7p-3, -0x1.8712139d0e994p-3,
    -0x1.7d68fe72f5ab3p-3, -0x1.73cb8adcfd12dp-3, -0x1.6a39a0a3bd37bp-3, -0x1.60b30b8309461p-3,
    -0x1.5737cbb818cddp-3, -0x1.4dc7b817bc1c7p-3, -0x1.4462b3bc9b3b6p-3, -0x1.3b08bc0d7f28ap-3,
    -0x1.31b996aba4f81p-3, -0x1.28753ef11ab9ap-3, -0x1.1f3b93bf25d3fp-3, -0x1.160c80c4b27b0p-3,
    -0x1.0ce7f0c4cc27dp-3, -0x1.03cdbf7d1ec0cp-3, -0x1.f57bc799005dbp-4, -0x1.e3708b530482ep-4,
    -0x1.d1797ba21935fp-4, -0x1.bf9680f9fc9fcp-4, -0x1.adc78265aea86p-4, -0x1.9c0c2ba4d252ep-4,
    -0x1.8a647d391dc19p-4, -0x1.78d01f23d82cep-4, -0x1.674f0ee365a66p-4, -0x1.55e10e20e0324p-4,
    -0x1.4485dc8dbdfa6p-4, -0x1.333d734183f00p-4, -0x1.2207ac8785473p-4, -0x1.10e4612cae81fp-4,
    -0x1.ffa694dab92fdp-5, -0x1.dda8b7c67ee35p-5, -0x1.bbced3a68f3bdp-5, -0x1.9a188df73de25p-5,
    -0x1.7885892357793p-5, -0x1.5715df403ce3fp-5, -0x1.35c8b2ca13042p-5, -0x1.149e5680059fap-5,
    -0x1.e72bccc13cd9fp-6, -0x1.a55f624c5c427p-6, -0x1.63d615c690bd6p-6, -0x1.228f827ea2d0ep-6,
    -0x1.c3177b4c75deep-7, -0x1.4192bb96832bfp-7, -0x1.8121bb458686fp-8, 0x0.0p+0};

// ref_logf with the tables given (the device fitter keeps copies in LDS: a lane-indexed
// table read from global memory is a vector-memory round trip per log)
__host__ __device__ __forceinline__ float ref_logf_tab(float v, const float* __restrict__ tabC,
                                                       const double* __restrict__ tabL) {
#if defined(FIT_PROBE_LOG) && defined(__HIP_DEVICE_COMPILE__)
  return __logf(v);   // timing-only variant build (see CWQ_KDIV)
#endif
  const uint32_t u = __builtin_bit_cast(uint32_t, v);
  if (u - 0x00800000u >= 0x7f000000u) return (float)log((double)v);   // not a positive normal
  const int i = (int)((u >> 16) & 127);
  const int e = (int)(u >> 23) - 127 + (i >> 6);
  const double m = (double)__builtin_bit_cast(float, (u & 0x007fffffu) | 0x3f800000u);
  const double r = fma(m, (double)tabC[i], -1.0);
  double p = 1.0 / 7.0;
  p = fma(p, r, -1.0 / 6.0);
  p = fma(p, r, 1.0 / 5.0);
  p = fma(p, r, -1.0 / 4.0);
  p = fma(p, r, 1.0 / 3.0);
  p = fma(p, r, -0.5);
  p = fma(p, r * r, r);   // r + r^2 (-1/2 + r (1/3 - ...))
  const double ed = (double)e;
  const double y = fma(ed, 0x1.62e42fefa39efp-1, tabL[i] + fma(ed, 0x1.abc9e3b39803fp-56, p));
  return (float)y;
}
__host__ __device__ __forceinline__ float ref_logf(float v) { return ref_logf_tab(v, kRefLogC, kRefLogL); }

// torch's CPU float32 sum of a contiguous vector, bit for bit (ATen's cascade sum as this
// build runs it -- 8-wide vectors: 4 vector accumulators, cascade levels of 16 rows, the
// accumulators added in order, then the scalar tail from 0 and the 8 vector lanes in order;
// checked against torch.sum on 8..4096 elements, scripts/torch_sum_order.py), for two term
// sequences at once.  One wave calls it; lane L < 32 is vector-lane (L & 7) of accumulator
// (L >> 3).  term(d, a, b) forms element d's two terms.  The sums come back on every lane.
constexpr int kSumPf = 8;   // rows of terms formed ahead of their adds (register budget of the fit loop)

template <typename Term>
__device__ __forceinline__ void torch_sum2(int D, int lane, Term term, float& Sa, float& Sb) {
#pragma clang fp contract(off)
  if (D < 8) {   // the scalar path: 4 accumulators, the tail into the first, then in order
    float a[4] = {0.f, 0.f, 0.f, 0.f}, b[4] = {0.f, 0.f, 0.f, 0.f};
    const int nr = D >> 2;
    for (int r = 0; r < nr; ++r)
      for (int k = 0; k < 4; ++k) {
        float ta, tb;
        term(r * 4 + k, ta, tb);
        a[k] = a[k] + ta;
        b[k] = b[k] + tb;
      }
    for (int d = nr * 4; d < D; ++d) {
      float ta, tb;
      term(d, ta, tb);
      a[0] = a[0] + ta;
      b[0] = b[0] + tb;
    }
    for (int k = 1; k < 4; ++k) {
      a[0] = a[0] + a[k];
      b[0] = b[0] + b[k];
    }
    Sa = a[0];
    Sb = b[0];
    return;
  }
  const int vec_size = D >> 3, size_ilp = vec_size >> 2;
  int cl = 0;   // ceil(log2(size_ilp))
  while ((1 << cl) < size_ilp) ++cl;
  const int lp = cl / 4 > 4 ? cl / 4 : 4;
  const int step = 1 << lp, mask = step - 1;
  const bool act = lane < 32;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f, b0 = 0.f, b1 = 0.f, b2 = 0.f, b3 = 0.f;
  int i = 0;
  if (size_ilp <= 32) {   // D < 1056: kSumPf rows' terms first, their loads in flight together
#pragma unroll
    for (int c = 0; c < (32 + kSumPf - 1) / kSumPf; ++c) {
      float ta[kSumPf], tb[kSumPf];
#pragma unroll
      for (int r = 0; r < kSumPf; ++r) {
        ta[r] = 0.f;
        tb[r] = 0.f;
        if (kSumPf * c + r < size_ilp && act) term((kSumPf * c + r) * 32 + lane, ta[r], tb[r]);
      }
#pragma unroll
      for (int r = 0; r < kSumPf; ++r) {
        const int row = kSumPf * c + r;
        if (row < size_ilp) {
          a0 = a0 + ta[r];
          b0 = b0 + tb[r];
        }
        if (((row + 1) & 15) == 0 && row + 1 <= (size_ilp & ~15)) {   // a whole step: level 1 takes level 0 (never a carry further)
          a1 = a1 + a0;
          a0 = 0.f;
          b1 = b1 + b0;
          b0 = 0.f;
        }
      }
    }
    i = size_ilp;
  }
  while (i + step <= size_ilp) {
    for (int j = 0; j < step; ++j, ++i)
      if (act) {
        float ta, tb;
        term(i * 32 + lane, ta, tb);
        a0 = a0 + ta;
        b0 = b0 + tb;
      }
    a1 = a1 + a0;
    a0 = 0.f;
    b1 = b1 + b0;
    b0 = 0.f;
    if ((i & (mask << lp)) != 0) continue;
    a2 = a2 + a1;
    a1 = 0.f;
    b2 = b2 + b1;
    b1 = 0.f;
    if ((i & (mask << (2 * lp))) != 0) continue;
    a3 = a3 + a2;
    a2 = 0.f;
    b3 = b3 + b2;
    b2 = 0.f;
  }
  for (; i < size_ilp; ++i)
    if (act) {
      float ta, tb;
      term(i * 32 + lane, ta, tb);
      a0 = a0 + ta;
      b0 = b0 + tb;
    }
  a0 = a0 + a1;
  a0 = a0 + a2;
  a0 = a0 + a3;
  b0 = b0 + b1;
  b0 = b0 + b2;
  b0 = b0 + b3;
  if (lane < 8)   // the vectors past the last whole accumulator row go to accumulator 0
    for (int v = size_ilp * 4; v < vec_size; ++v) {
      float ta, tb;
      term(v * 8 + lane, ta, tb);
      a0 = a0 + ta;
      b0 = b0 + tb;
    }
  {
    const int l = lane & 7;
    const float pa1 = __shfl(a0, l + 8, 64), pa2 = __shfl(a0, l + 16, 64), pa3 = __shfl(a0, l + 24, 64);
    const float pb1 = __shfl(b0, l + 8, 64), pb2 = __shfl(b0, l + 16, 64), pb3 = __shfl(b0, l + 24, 64);
    a0 = a0 + pa1;
    a0 = a0 + pa2;
    a0 = a0 + pa3;
    b0 = b0 + pb1;
    b0 = b0 + pb2;
    b0 = b0 + pb3;
  }
  float fa = 0.f, fb = 0.f;   // the scalar tail first, from zero, then the lanes in order
  for (int d = vec_size * 8; d < D; ++d) {
    float ta, tb;
    term(d, ta, tb);
    fa = fa + ta;
    fb = fb + tb;
  }
  for (int l = 0; l < 8; ++l) {
    fa = fa + __shfl(a0, l, 64);
    fb = fb + __shfl(b0, l, 64);
  }
  Sa = fa;
  Sb = fb;
}

// Two independent torch-order sums pairs in one wave: lanes 0-31 sum sequence 0, lanes 32-63
// sequence 1 (the same accumulation pattern per half, so no lane divergence).
// term(d, h, a, b) forms element d's two terms of sequence h = lane >> 5.  Returns the
// half's two sums on each of its lanes.
template <typename Term>
__device__ __forceinline__ void torch_sum2_halves(int D, int lane, Term term, float& Sa, float& Sb) {
#pragma clang fp contract(off)
  const int h = lane >> 5, hl = lane & 31, base = h << 5;
  if (D < 8) {   // the scalar path (torch_sum2's), every lane of a half the same
    torch_sum2(D, lane, [&](int d, float& a, float& b) { term(d, h, a, b); }, Sa, Sb);
    return;
  }
  const int vec_size = D >> 3, size_ilp = vec_size >> 2;
  int cl = 0;
  while ((1 << cl) < size_ilp) ++cl;
  const int lp = cl / 4 > 4 ? cl / 4 : 4;
  const int step = 1 << lp, mask = step - 1;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f, b0 = 0.f, b1 = 0.f, b2 = 0.f, b3 = 0.f;
  int i = 0;
  if (size_ilp <= 32) {   // D < 1056: kSumPf rows' terms first, their loads in flight together
#pragma unroll
    for (int c = 0; c < (32 + kSumPf - 1) / kSumPf; ++c) {
      float ta[kSumPf], tb[kSumPf];
#pragma unroll
      for (int r = 0; r < kSumPf; ++r) {
        ta[r] = 0.f;
        tb[r] = 0.f;
        if (kSumPf * c + r < size_ilp) term((kSumPf * c + r) * 32 + hl, h, ta[r], tb[r]);
      }
#pragma unroll
      for (int r = 0; r < kSumPf; ++r) {
        const int row = kSumPf * c + r;
        if (row < size_ilp) {
          a0 = a0 + ta[r];
          b0 = b0 + tb[r];
        }
        if (((row + 1) & 15) == 0 && row + 1 <= (size_ilp & ~15)) {   // a whole step: level 1 takes level 0 (never a carry further)
          a1 = a1 + a0;
          a0 = 0.f;
          b1 = b1 + b0;
          b0 = 0.f;
        }
      }
    }
    i = size_ilp;
  }
  while (i + step <= size_ilp) {
    for (int j = 0; j < step; ++j, ++i) {
      float ta, tb;
      term(i * 32 + hl, h, ta, tb);
      a0 = a0 + ta;
      b0 = b0 + tb;
    }
    a1 = a1 + a0;
    a0 = 0.f;
    b1 = b1 + b0;
    b0 = 0.f;
    if ((i & (mask << lp)) != 0) continue;
    a2 = a2 + a1;
    a1 = 0.f;
    b2 = b2 + b1;
    b1 = 0.f;
    if ((i & (mask << (2 * lp))) != 0) continue;
    a3 = a3 + a2;
    a2 = 0.f;
    b3 = b3 + b2;
    b2 = 0.f;
  }
  for (; i < size_ilp; ++i) {
    float ta, tb;
    term(i * 32 + hl, h, ta, tb);
    a0 = a0 + ta;
    b0 = b0 + tb;
  }
  a0 = a0 + a1;
  a0 = a0 + a2;
  a0 = a0 + a3;
  b0 = b0 + b1;
  b0 = b0 + b2;
  b0 = b0 + b3;
  for (int v = size_ilp * 4; v < vec_size; ++v) {   // every lane computes, accumulator 0 keeps
    float ta, tb;
    term(v * 8 + (hl & 7), h, ta, tb);
    if (hl < 8) {
      a0 = a0 + ta;
      b0 = b0 + tb;
    }
  }
  {
    const int l = hl & 7;
    const float pa1 = __shfl(a0, base + l + 8, 64), pa2 = __shfl(a0, base + l + 16, 64),
                pa3 = __shfl(a0, base + l + 24, 64);
    const float pb1 = __shfl(b0, base + l + 8, 64), pb2 = __shfl(b0, base + l + 16, 64),
                pb3 = __shfl(b0, base + l + 24, 64);
    a0 = a0 + pa1;
    a0 = a0 + pa2;
    a0 = a0 + pa3;
    b0 = b0 + pb1;
    b0 = b0 + pb2;
    b0 = b0 + pb3;
  }
  float fa = 0.f, fb = 0.f;
  for (int d = vec_size * 8; d < D; ++d) {
    float ta, tb;
    term(d, h, ta, tb);
    fa = fa + ta;
    fb = fb + tb;
  }
  for (int l = 0; l < 8; ++l) {
    fa = fa + __shfl(a0, base + l, 64);
    fb = fb + __shfl(b0, base + l, 64);
  }
  Sa = fa;
  Sb = fb;
}

}  // namespace cwq
