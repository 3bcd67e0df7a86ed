// libcwq: group-centred filter rows for clustered (real-structure) trees.
//
// The bf16-MFMA filters bound x'.mu' for root-centred query and row (x' = x - c0,
// mu' = mu - c0); the error bound grows with |x'| |mu'|.  On a clustered corpus every row
// sits far from the root mean (|mu'| ~ the cluster spread between clusters) while the keys
// that decide the top-k differ by the spread WITHIN a cluster, so the bound admits most of
// a cluster (C2-shaped ifit tree, 100k x 768: ~1,160 candidates and ~1,000 exact reranks
// per query).  Rows in a group g (the subtree of a depth-1 internal node, mean c_g) are
// therefore stored centred at c_g instead: M = fl(mu - c_g), d = c_g - c0 (exact in fp64),
//   S = |x - mu|^2 = |x'|^2 + |M + d|^2 - 2 x'.M - 2 x'.d      (x' = fl(x - c0) as before)
// so the kernels keep their arithmetic -- n2 = |x'|^2 + rn2 with rn2 = |M + d|^2, the dot
// x'.M on the matrix cores, whose bound now scales with |M| (the within-group spread) --
// and the per-(query, group) term -2 x'.d moves into the parent-prefix table the filters
// already read: P'[q][p] = P[q][p] + (hs_p / invL_p) * sh[q][g(p)], sh = -2 x'.d in fp64,
// rounded outward into [P'lo, P'hi] (categorize: P'c = hs_c * sh with invL = 1, the
// bottleneck min taken from BF separately).  The exact rerank keeps the exact P and the
// uncentred fp32 rows, so results stay the exact scan's bit for bit.  The rounding of M
// adds 2^-23 |M| to the rows' beta / delta (cwq_api.hip build_filter); its row-only cross
// term 2^-23 |M| |M + d| stays within eps_n * rn2 for groups whose rows all have
// |M| <= 2 |M + d| (plan_groups).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "cwq_internal.h"

namespace cwq {

// Rows of `mean` by node id into a dense [n][D] array (group centres).
__global__ void gather_rows_f32_kernel(const float* __restrict__ mean, int D, const int64_t* __restrict__ nodes,
                                       int64_t n, float* out) {
  const int64_t r = blockIdx.x;
  if (r >= n) return;
  for (int d = threadIdx.x; d < D; d += blockDim.x) out[r * D + d] = mean[nodes[r] * (int64_t)D + d];
}

hipError_t launch_gather_rows_f32(const float* mean, int D, const int64_t* nodes, int64_t n, float* out,
                                  hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(gather_rows_f32_kernel, dim3((unsigned)n), dim3(256), 0, s, mean, D, nodes, n, out);
  return hipGetLastError();
}

// Per row (one wave): |fl(mu - c0)|^2 and |fl(mu - c_g)|^2 (g = grp[r], -1: none) in fp64.
__global__ void group_norms_kernel(const float* __restrict__ mean, int D, const int64_t* __restrict__ nodes, int64_t n,
                                   const float* __restrict__ c0, const float* __restrict__ cent,
                                   const int* __restrict__ grp, double* root2, double* grp2) {
  const int lane = threadIdx.x & 63;
  const int64_t r = blockIdx.x * (int64_t)(blockDim.x / 64) + (threadIdx.x >> 6);
  if (r >= n) return;
  const int g = grp[r];
  double a = 0.0, b = 0.0;
  for (int d = lane; d < D; d += 64) {
    const float v = mean[nodes[r] * (int64_t)D + d];
    const float u0 = v - c0[d];
    a += (double)u0 * (double)u0;
    if (g >= 0) {
      const float ug = v - cent[(int64_t)g * D + d];
      b += (double)ug * (double)ug;
    }
  }
  for (int off = 32; off > 0; off >>= 1) {
    a += __shfl_xor(a, off, 64);
    b += __shfl_xor(b, off, 64);
  }
  if (lane == 0) {
    root2[r] = a;
    grp2[r] = g >= 0 ? b : a;
  }
}

hipError_t launch_group_norms(const float* mean, int D, const int64_t* nodes, int64_t n, const float* c0,
                              const float* cent, const int* grp, double* root2, double* grp2, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(group_norms_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, s, mean, D, nodes, n, c0, cent,
                     grp, root2, grp2);
  return hipGetLastError();
}

// The tree-adaptive cut (cwq_api.hip plan_groups): per isotropic row (one wave), |fl(mu_r -
// c0)|^2 (out[r][0]) and |fl(mu_r - mu_a)|^2 for each internal ancestor a of the row at depth
// 1..maxd (out[r][depth(a)]; -1: no ancestor at that depth), in fp64 -- the squared norms of
// the row centred at the root or at a, as rows_prep would store it.  rpar: the row's parent
// (internal id); a row is below every ancestor of its parent.
__global__ void group_anc_dist_kernel(const float* __restrict__ mean, int D, const int64_t* __restrict__ rows,
                                      int64_t n, const float* __restrict__ c0, const int* __restrict__ rpar,
                                      const int* __restrict__ par_int, const int* __restrict__ idep,
                                      const int64_t* __restrict__ int_nodes, int maxd, double* out) {
  const int lane = threadIdx.x & 63;
  const int64_t r = blockIdx.x * (int64_t)(blockDim.x / 64) + (threadIdx.x >> 6);
  if (r >= n) return;
  const int W = maxd + 1;   // [0]: the root centre c0, [d]: the ancestor at depth d
  if (lane == 0)
    for (int j = 1; j < W; ++j) out[r * W + j] = -1.0;
  const float* mr = mean + rows[r] * (int64_t)D;
  double s0 = 0.0;
  for (int d = lane; d < D; d += 64) {
    const float u = mr[d] - c0[d];
    s0 += (double)u * (double)u;
  }
  for (int off = 32; off > 0; off >>= 1) s0 += __shfl_xor(s0, off, 64);
  if (lane == 0) out[r * W] = s0;
  for (int a = rpar[r]; a > 0; a = par_int[a]) {
    const int da = idep[a];
    if (da > maxd) continue;
    const float* ma = mean + int_nodes[a] * (int64_t)D;
    double s = 0.0;
    for (int d = lane; d < D; d += 64) {
      const float u = mr[d] - ma[d];
      s += (double)u * (double)u;
    }
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    if (lane == 0) out[r * W + da] = s;
  }
}

hipError_t launch_group_anc_dist(const float* mean, int D, const int64_t* rows, int64_t n, const float* c0,
                                 const int* rpar, const int* par_int, const int* idep, const int64_t* int_nodes,
                                 int maxd, double* out, hipStream_t s) {
  if (n <= 0 || maxd <= 0) return hipSuccess;
  hipLaunchKernelGGL(group_anc_dist_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, s, mean, D, rows, n, c0,
                     rpar, par_int, idep, int_nodes, maxd, out);
  return hipGetLastError();
}

// sh[q][g] = -2 x'.d_g in fp64 (x' = fl(x - c0) exactly as query_prep forms it; d_g = c_g - c0
// in fp64, exact).  One wave per (query, group).  she[q][g] bounds the fp64 evaluation error
// of sh: products rounded once, ceil(D/64) sequential adds per lane, 6 butterfly levels, so
// |err| <= gamma_{D/64+8} * 2 sum |x'_i d_i| -- relative to the sum of |terms|, not to |sh|,
// which cancellation can make much smaller (a query nearly orthogonal to d_g).
// dist2 (optional, group pruning): |x - c_g|^2 in fp64 -- each difference of two floats is
// exact in fp64 and each square of it too (<= 50 significant bits), so the only error is
// the fp64 summation's, <= gamma_{D/64+7} dist2 (relative; cwq_prune.hip takes 2^-40).
__global__ void group_shift_kernel(const float* __restrict__ q, int64_t nq, int D, const float* __restrict__ c0,
                                   const float* __restrict__ cent, int G, double* sh, double* she, double* dist2) {
  const int lane = threadIdx.x & 63;
  const int64_t w = blockIdx.x * (int64_t)(blockDim.x / 64) + (threadIdx.x >> 6);
  if (w >= nq * (int64_t)G) return;
  const int64_t qi = w / G;
  const int g = (int)(w % G);
  double a = 0.0, ab = 0.0, e2 = 0.0;
  for (int d = lane; d < D; d += 64) {
    const float x = q[qi * D + d];
    const float xc = x - c0[d];
    const float cg = cent[(int64_t)g * D + d];
    const double dd = (double)cg - (double)c0[d];
    const double t = (double)xc * dd;
    a += t;
    ab += fabs(t);
    const double u = (double)x - (double)cg;
    e2 += u * u;
  }
  for (int off = 32; off > 0; off >>= 1) {
    a += __shfl_xor(a, off, 64);
    ab += __shfl_xor(ab, off, 64);
    e2 += __shfl_xor(e2, off, 64);
  }
  if (lane == 0) {
    sh[qi * G + g] = -2.0 * a;
    she[qi * G + g] = 2.0 * ab * ((double)(D / 64 + 8) * 0x1.02p-53);
    if (dist2) dist2[qi * G + g] = e2;
  }
}

hipError_t launch_group_shift(const float* q, int nq, int D, const float* c0, const float* cent, int G, double* sh,
                              double* dist2, hipStream_t s) {
  if (nq <= 0 || G <= 0) return hipSuccess;
  const int64_t nw = (int64_t)nq * G;
  hipLaunchKernelGGL(group_shift_kernel, dim3((unsigned)((nw + 3) / 4)), dim3(256), 0, s, q, (int64_t)nq, D, c0, cent,
                     G, sh, sh + nw, dist2);
  return hipGetLastError();
}

// Outward-rounded fp32 interval of t (fp64), widened by e.
__device__ __forceinline__ void out_round(double t, double e, float& lo, float& hi) {
  lo = __double2float_rd(t - e);
  hi = __double2float_ru(t + e);
}

// The filters' prefix tables for group-centred rows: per (query, internal node p),
// Fast [P'lo, P'hi] = P + F[p] * sh[q][grp[p]] (F = hs / invL of p's rows) and, when
// Pclo is set, categorize [P'c lo, hi] = Fc[p] * sh (zero for nodes without a group).
__global__ void group_pprime_kernel(const float* __restrict__ P, int64_t ldP, int nq, int NI,
                                    const int* __restrict__ grp, const double* __restrict__ F,
                                    const double* __restrict__ Fc, const double* __restrict__ sh,
                                    const double* __restrict__ she, int G, float* Plo, float* Phi, float* Pclo,
                                    float* Pchi) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= (int64_t)nq * NI) return;
  const int64_t qi = i / NI;
  const int p = (int)(i % NI);
  const int g = grp[p];
  const size_t o = (size_t)qi * ldP + p;
  const float pv = P[o];
  if (g < 0) {
    Plo[o] = pv;
    Phi[o] = pv;
    if (Pclo) {
      Pclo[o] = 0.f;
      Pchi[o] = 0.f;
    }
    return;
  }
  const double s = sh[qi * G + g], se = she[qi * G + g];
  const double a = F[p] * s;
  const double t = (double)pv + a;
  float lo, hi;
  out_round(t, fabs(F[p]) * se + (fabs((double)pv) + fabs(a)) * 0x1p-50, lo, hi);
  Plo[o] = lo;
  Phi[o] = hi;
  if (Pclo) {
    const double c = Fc[p] * s;
    out_round(c, fabs(Fc[p]) * se + fabs(c) * 0x1p-50, lo, hi);
    Pclo[o] = lo;
    Pchi[o] = hi;
  }
}

hipError_t launch_group_prefixes(const float* q, int nq, int D, const float* c0, const float* cent, int G,
                                 const float* P, int64_t ldP, int NI, const int* grp, const double* F, const double* Fc,
                                 double* sh, float* Plo, float* Phi, float* Pclo, float* Pchi, hipStream_t s) {
  if (nq <= 0 || NI <= 0 || G <= 0) return hipSuccess;
  const int64_t nw = (int64_t)nq * G;
  double* she = sh + nw;   // sh holds 2 nq G doubles: the shifts, then their error bounds
  hipLaunchKernelGGL(group_shift_kernel, dim3((unsigned)((nw + 3) / 4)), dim3(256), 0, s, q, (int64_t)nq, D, c0, cent,
                     G, sh, she, nullptr);
  const int64_t n = (int64_t)nq * NI;
  hipLaunchKernelGGL(group_pprime_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, P, ldP, nq, NI, grp, F,
                     Fc, sh, she, G, Plo, Phi, Pclo, Pchi);
  return hipGetLastError();
}

// Internal prefixes for a few queries in one launch: one thread per (query, node) forms
// the node's P, BF, LPF from the root down its path -- the ancestor t levels above found
// by walking parents (depth^2 parent loads, no local array) -- with prefix_level_kernel's
// arithmetic in the same order (P = fmaf(w, lp', P) per level, BF = fminf chain), so the
// values are the per-level launches' bit for bit; then (G > 0) the group-centred prefix
// tables from the shifts group_shift_kernel wrote.  At one query per call on C2's
// depth-9 ifit tree this replaces one launch per level plus one (a workgroup per query
// walking the levels measured 293 us: each level a chain of dependent loads).
__global__ void internal_chain_kernel(const IntFinishArgs f) {
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (t >= (int64_t)f.nq * f.NI) return;
  const int qi = (int)(t / f.NI);
  const int i = (int)(t % f.NI);
  const size_t ro = (size_t)qi * f.ldS;
  int d = 0;
  for (int a = i; f.par_int[a] >= 0; a = f.par_int[a]) ++d;
  float P = 0.f, B = 0.f, lpf = 0.f;
  for (int l = d; l >= 0; --l) {   // the ancestor l levels above i, root first
    int a = i;
    for (int u = 0; u < l; ++u) a = f.par_int[a];
    const float sv = f.S[ro + a];
    const float ld = f.logdet_int[a];
    const float lp = -0.5f * (ld + sv);
    lpf = -0.5f * (ld + f.dfull + sv);
    if (l == d) {
      P = f.w_int[a] * lp;
      B = lpf;
    } else {
      P = fmaf(f.w_int[a], lp, P);
      B = fminf(B, lpf);
    }
  }
  const size_t o = ro + i;
  f.P[o] = P;
  if (f.BF) f.BF[o] = B;
  if (f.LPF) f.LPF[o] = lpf;
  if (f.G <= 0) return;
  const int g = f.grp[i];
  if (g < 0) {
    f.Plo[o] = P;
    f.Phi[o] = P;
    if (f.Pclo) {
      f.Pclo[o] = 0.f;
      f.Pchi[o] = 0.f;
    }
    return;
  }
  const double sv = f.sh[(size_t)qi * f.G + g];
  const double se = f.sh[(size_t)f.nq * f.G + (size_t)qi * f.G + g];   // its error bound (group_shift_kernel)
  const double a = f.F[i] * sv;
  const double tt = (double)P + a;
  float lo, hi;
  out_round(tt, fabs(f.F[i]) * se + (fabs((double)P) + fabs(a)) * 0x1p-50, lo, hi);
  f.Plo[o] = lo;
  f.Phi[o] = hi;
  if (f.Pclo) {
    const double c = f.Fc[i] * sv;
    out_round(c, fabs(f.Fc[i]) * se + fabs(c) * 0x1p-50, lo, hi);
    f.Pclo[o] = lo;
    f.Pchi[o] = hi;
  }
}

hipError_t launch_internal_finish(const IntFinishArgs& f, hipStream_t s) {
  if (f.nq <= 0 || f.NI <= 0) return hipSuccess;
  if (f.ldS < f.NI || (f.G > 0 && (!f.q || !f.sh || !f.Plo || !f.Phi))) return hipErrorInvalidValue;
  if (f.G > 0) {   // the shifts first (one wave per (query, group))
    const int64_t nw = (int64_t)f.nq * f.G;
    hipLaunchKernelGGL(group_shift_kernel, dim3((unsigned)((nw + 3) / 4)), dim3(256), 0, s, f.q, (int64_t)f.nq, f.D,
                       f.c0, f.cent, f.G, f.sh, f.sh + nw, nullptr);
  }
  const int64_t n = (int64_t)f.nq * f.NI;
  hipLaunchKernelGGL(internal_chain_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, f);
  return hipGetLastError();
}

}  // namespace cwq
