// libcwq: the reference's float32 arithmetic for the category-utility KL of ifit
// (CobwebTorchTree.compute_score, CobwebTorchTree.py:344-356: torch.log, .sum() on CPU
// tensors), shared by the host-driven fitter (cwq_fit.hip) and the device-resident loop
// (cwq_fitdev.hip).  Not part of the public interface.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>

namespace cwq {

// log: torch's float32 log (Sleef, 1-ulp) is the correctly rounded value for 99.96% of
// inputs; the fp64 log rounded once is that value.
__device__ __forceinline__ float ref_logf(float v) { return (float)log((double)v); }

// torch's CPU float32 sum of a contiguous vector, bit for bit (ATen's cascade sum as this
// build runs it -- 8-wide vectors: 4 vector accumulators, cascade levels of 16 rows, the
// accumulators added in order, then the scalar tail from 0 and the 8 vector lanes in order;
// checked against torch.sum on 8..4096 elements, scripts/torch_sum_order.py), for two term
// sequences at once.  One wave calls it; lane L < 32 is vector-lane (L & 7) of accumulator
// (L >> 3).  term(d, a, b) forms element d's two terms.  The sums come back on every lane.
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
// half's two sums on each of its lanes.  D >= 8.
template <typename Term>
__device__ __forceinline__ void torch_sum2_halves(int D, int lane, Term term, float& Sa, float& Sb) {
#pragma clang fp contract(off)
  const int h = lane >> 5, hl = lane & 31, base = h << 5;
  const int vec_size = D >> 3, size_ilp = vec_size >> 2;
  int cl = 0;
  while ((1 << cl) < size_ilp) ++cl;
  const int lp = cl / 4 > 4 ? cl / 4 : 4;
  const int step = 1 << lp, mask = step - 1;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f, b0 = 0.f, b1 = 0.f, b2 = 0.f, b3 = 0.f;
  int i = 0;
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
