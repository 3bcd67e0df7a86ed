// libcwq: group pruning of the Fast query on clustered (group-centred) trees.
//
// On a Cobweb tree of a clustered corpus every depth-1 node g heads one cluster, and a
// query's top-k lies in one or a few of them; yet the exact internal pass computes every
// internal node's lp' for every query (C2's ifit tree: 35,506 nodes x 1,000 queries, 1.93
// of a 3.59 ms batch).  Here a certified bound prunes whole groups:
//
//   every member a of g (internal node or leaf row below g) has its mean within r_g of the
//   centre c_g, weights w_{a,d} in [wmin_g, wmax_g] and logdet >= ldmin_g, so for a query x
//     S_a = sum_d w_{a,d} (x_d - mu_{a,d})^2 >= wmin_g (|x - c_g| - r_g)_+^2
//     lp'(a) = -(logdet_a + S_a)/2 <= UB_g(x)
//   and, with every level weight >= 0, the Fast key of a usable row n of g
//     key(n) = invL_n P(root) + invL_n sum_{a in path, a != root} w_a lp'(a) + cw_n lp'(n)
//            <= invL_n P(root) + C_n UB_g(x)                  (C_n = invL_n sum w_a + cw_n)
//   so KUB[q][g] = max over the group's (invL, C) ranges, plus margins for the fp32
//   evaluation of the exact keys (every bound below is on the fp32 values the exact pass and
//   the rerank compute, not on real arithmetic).
//
// First (before the filter's threshold exists): for each query only its best group g* =
// argmax_g KUB gets the exact internal pass (the scan's arithmetic, bit for bit) and exact
// prefixes; every other (query, node) gets the sentinel prefix kPruneSent in the filters'
// tables, so its rows are never candidates and their lower bounds never raise a threshold.
// The seed threshold T[q] (the K-th largest exact key over up to 64 rows of g*, <= tau_K)
// then decides stage B: the groups with KUB[q][g] >= T[q] get the exact pass too.  Every
// group left has KUB < T <= tau_K: none of its rows can be in the top-K, so the result is the
// exact scan's bit for bit.  Launches: head (bounds, root, g*), g*'s pass, seed, stage B.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <algorithm>
#include <map>
#include <mutex>

#include "cwq_internal.h"

namespace cwq {

// Per member (one wave each; grp[r] < 0: not in a group): fp64 {wmin, wmax, |mu - c_g|^2,
// |mu|^2}.  Weights as the exact pass uses them: iv[r] > 0 for isotropic rows (S = iv *
// sum (x - mu)^2), else A^2 with A = 1 / sqrtf(v) (gather_T_kernel's A).
__global__ void prune_member_kernel(const float* __restrict__ mean, const VarSrc var, int D,
                                    const int64_t* __restrict__ nodes, const float* __restrict__ iv,
                                    const int* __restrict__ grp, const float* __restrict__ cent, int64_t n,
                                    double4* out) {
  const int lane = threadIdx.x & 63;
  const int64_t r = blockIdx.x * (int64_t)(blockDim.x / 64) + (threadIdx.x >> 6);
  if (r >= n) return;
  const int g = grp[r];
  if (g < 0) {
    if (lane == 0) out[r] = make_double4(0.0, 0.0, 0.0, 0.0);
    return;
  }
  const int64_t nd = nodes[r];
  const float ivr = iv ? iv[r] : 0.f;
  double wmn = INFINITY, wmx = 0.0, d2 = 0.0, m2 = 0.0;
  for (int d = lane; d < D; d += 64) {
    double w;
    if (ivr > 0.f) {
      w = (double)ivr;
    } else {
      const float A = 1.0f / sqrtf(var.at(nd, d, D));
      w = (double)A * (double)A;
    }
    wmn = fmin(wmn, w);
    wmx = fmax(wmx, w);
    const float mu = mean[nd * (int64_t)D + d];
    const double u = (double)mu - (double)cent[(int64_t)g * D + d];
    d2 += u * u;
    m2 += (double)mu * (double)mu;
  }
  for (int off = 32; off > 0; off >>= 1) {
    wmn = fmin(wmn, __shfl_xor(wmn, off, 64));
    wmx = fmax(wmx, __shfl_xor(wmx, off, 64));
    d2 += __shfl_xor(d2, off, 64);
    m2 += __shfl_xor(m2, off, 64);
  }
  if (lane == 0) out[r] = make_double4(wmn, wmx, d2, m2);
}

hipError_t launch_prune_members(const float* mean, const VarSrc& var, int D, const int64_t* nodes, const float* iv,
                                const int* grp, const float* cent, int64_t n, double4* out, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(prune_member_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, s, mean, var, D, nodes, iv, grp,
                     cent, n, out);
  return hipGetLastError();
}

// P, and the filters' tables [Plo, Phi] of node i (internal_chain_kernel's tail: the
// group-centred rows' shifted prefix, outward-rounded).
__device__ __forceinline__ void prune_write_tables(const PruneArgs& a, int q, int i, float P) {
  const size_t o = (size_t)q * a.ldS + i;
  a.P[o] = P;
  const int g = a.grp[i];
  if (g < 0) {
    a.Plo[o] = P;
    a.Phi[o] = P;
    return;
  }
  const size_t gi = (size_t)q * a.G + g;
  const double sv = a.sh[gi];
  const double se = a.sh[(size_t)a.nq * a.G + gi];
  const double ad = a.F[i] * sv;
  const double tt = (double)P + ad;
  const double e = fabs(a.F[i]) * se + (fabs((double)P) + fabs(ad)) * 0x1p-50;
  a.Plo[o] = __double2float_rd(tt - e);
  a.Phi[o] = __double2float_ru(tt + e);
}

// The prefixes and tables of group g's internal nodes for query q, level by level down the
// group's BFS-ordered list: P(i) = fmaf(w_i, lp'(i), P(parent)) with the parent's P from LDS
// (s_P[position - gi_ptr[g]]; the centre's parent's P, a top node's, from P) -- internal_chain_kernel's
// top-down chain, the same values, without walking every node's chain from the root.  nt threads; the raw
// sums S of the group's nodes must be complete and visible.
__device__ __forceinline__ void prune_group_prefixes(const PruneArgs& a, int q, int g, float* s_P, int nt) {
  const int b0 = a.gi_ptr[g], b1 = a.gi_ptr[g + 1];
  const float Pt = a.P[(size_t)q * a.ldS + a.top_nodes[a.grp_tpos[g]]];   // the centre's parent (head kernel)
  for (int L = a.gmindep; L <= a.gmaxdep; ++L) {
    for (int j = b0 + (int)threadIdx.x; j < b1; j += nt) {
      if (a.gi_dep[j] != L) continue;
      const int node = a.gi_nodes[j], pp = a.gi_ppos[j];
      const float lp = -0.5f * (a.logdet_int[node] + a.S[(size_t)q * a.ldS + node]);
      const float P = fmaf(a.w_int[node], lp, pp < 0 ? Pt : s_P[pp - b0]);
      s_P[j - b0] = P;
      prune_write_tables(a, q, node, P);
    }
    __syncthreads();
  }
}

// The bound terms of one (query, group) pair, by one wave: the group shift -2 x'.d_g and its
// error bound (as group_shift_kernel), |x - c_g|^2, and the terms of KUB that do not depend
// on the root's prefix P0: kpart[0] = max(Cmin UB, Cmax UB), kpart[1] = Cmax mag (the margin's).
//   every member a of g: S_a >= wmin (|x - c_g| - r_g)_+^2 in real arithmetic; the fp32 S
//   >= (1 - 2^-16) (sqrt(wmin) dlo - 2^-23 sqrt(wmax) mmax)_+^2 (t = x A - B with B = fl(mu
//   A), the partial sums' relative error < 64 * 2^-24); lp'_fp32 = fl(-0.5 fl(logdet + S))
//   <= -logdet/2 + 2^-22 |logdet| - (1/2 - 2^-22) S_fp32 = UB; |lp'| <= mag.
// xs / c0s: the query and the root centre (prune_terms_kernel: global, L2-resident).
__device__ __forceinline__ void prune_group_terms(const PruneArgs& a, const float* xs, const float* c0s, int64_t qi, int g,
                                                  int lane) {
  double d1 = 0.0, ab = 0.0, e2 = 0.0;
#pragma unroll 4
  for (int d = lane; d < a.D; d += 64) {
    const float x = xs[d];
    const float xc = x - c0s[d];
    const float cg = a.cent[(int64_t)g * a.D + d];
    const double dd = (double)cg - (double)c0s[d];
    const double t = (double)xc * dd;
    d1 += t;
    ab += fabs(t);
    const double u = (double)x - (double)cg;
    e2 += u * u;
  }
  for (int off = 32; off > 0; off >>= 1) {
    d1 += __shfl_xor(d1, off, 64);
    ab += __shfl_xor(ab, off, 64);
    e2 += __shfl_xor(e2, off, 64);
  }
  if (lane != 0) return;
  const size_t o = (size_t)qi * a.G + g;
  a.sh[o] = -2.0 * d1;
  a.sh[(size_t)a.nq * a.G + o] = 2.0 * ab * ((double)(a.D / 64 + 8) * 0x1.02p-53);
  const GroupBound b = a.gb[g];
  double kp = -INFINITY, m2 = 0.0, kp0 = -INFINITY;
  if (b.valid) {
    // e2: exact differences, squares and fp64 sums: relative error < 2^-40
    const double dist_lo = sqrt(e2 * (1.0 - 0x1p-40)) * (1.0 - 0x1p-50);
    const double dist_hi = sqrt(e2 * (1.0 + 0x1p-40)) * (1.0 + 0x1p-50);
    const double dlo = fmax(0.0, dist_lo - b.r);
    const double sv = sqrt(b.wmin) * dlo - 0x1p-23 * sqrt(b.wmax) * b.mmax;
    const double SLB = sv > 0.0 ? (1.0 - 0x1p-16) * sv * sv : 0.0;
    const double UB = -0.5 * b.ldmin + 0x1p-22 * b.ldabs - (0.5 - 0x1p-22) * SLB;
    const double shv = sqrt(b.wmax) * (dist_hi + b.r) + 0x1p-23 * sqrt(b.wmax) * b.mmax;
    const double mag = 0.5 * (b.ldabs + (1.0 + 0x1p-16) * shv * shv) * (1.0 + 0x1p-20);
    kp = fmax(b.Cmin * UB, b.Cmax * UB);
    m2 = b.Cmax * mag;
    // the same bound at the centre itself (r_g = 0): not a bound of the group, a point
    // estimate that ranks the groups for g* (a loose broad group has the largest KUB yet is
    // rarely where the top-K lies)
    const double s0 = sqrt(b.wmin) * dist_lo;
    kp0 = fmax(b.Cmin, b.Cmax) * (-0.5 * b.ldmin - 0.5 * s0 * s0);
  }
  a.kpart[o] = kp;
  a.kpart[(size_t)a.nq * a.G + o] = m2;
  a.kpart[(size_t)2 * a.nq * a.G + o] = kp0;
}

// S of cnt nodes of a group's list from position c0, for query q (its slices in s_x): every
// (node, 16-dim slice) partial in parallel -- exact_aniso_S's fma chain -- and one thread per
// node adding them in slice order (the scan kernel's raw sums bit for bit).  NT threads.
template <int NT>
__device__ __forceinline__ void prune_nodes_S(const PruneArgs& a, int q, int c0, int cnt, const float* s_x,
                                              float* s_part) {
  const int tid = threadIdx.x;
  const int NV16 = a.DP / 16, LDP = NV16 + 1;
  for (int it = tid; it < cnt * NV16; it += NT) {
    const int e = it / NV16, v = it - e * NV16;
    const int node = a.gi_nodes[c0 + e];
    const float* __restrict__ ar = a.Ar + (size_t)node * a.DP + v * 16;
    const float* __restrict__ br = a.Br + (size_t)node * a.DP + v * 16;
    float4 a4[4], b4[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      a4[j] = *reinterpret_cast<const float4*>(ar + j * 4);
      b4[j] = *reinterpret_cast<const float4*>(br + j * 4);
    }
    float part;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const float4 ta = a4[j >> 2], tb = b4[j >> 2];
      const float aj = (j & 3) == 0 ? ta.x : (j & 3) == 1 ? ta.y : (j & 3) == 2 ? ta.z : ta.w;
      const float bj = (j & 3) == 0 ? tb.x : (j & 3) == 1 ? tb.y : (j & 3) == 2 ? tb.z : tb.w;
      const float tt = fmaf(s_x[v * 16 + j], aj, -bj);
      part = (j == 0) ? tt * tt : fmaf(tt, tt, part);
    }
    s_part[e * LDP + v] = part;
  }
  __syncthreads();
  if (tid < cnt) {
    const float acc = sum_in_order(s_part + tid * LDP, NV16);
    a.S[(size_t)q * a.ldS + a.gi_nodes[c0 + tid]] = acc;
  }
  __syncthreads();
}

// The query's padded slices into LDS.
__device__ __forceinline__ void prune_load_query(const PruneArgs& a, int q, float* s_x, int nt) {
  const int NV16 = a.DP / 16;
  const float* xq = a.X + ((size_t)(q / kXQ) * NV16 * kXQ + (q % kXQ)) * 16;
  for (int d = threadIdx.x; d < a.DP; d += nt) s_x[d] = xq[(size_t)(d >> 4) * kXQ * 16 + (d & 15)];
}

// The exact internal pass of one (query, group) pair by one workgroup (stage B): the nodes'
// raw sums in chunks of kPrChunk, then their prefixes and tables.
constexpr int kPrThreads = 512, kPrChunk = 128;
__device__ void prune_pair(const PruneArgs& a, int q, int g, float* s_x, float* s_part) {
  prune_load_query(a, q, s_x, kPrThreads);
  __syncthreads();
  const int b0 = a.gi_ptr[g], b1 = a.gi_ptr[g + 1];
  for (int c0 = b0; c0 < b1; c0 += kPrChunk) prune_nodes_S<kPrThreads>(a, q, c0, min(kPrChunk, b1 - c0), s_x, s_part);
  // the raw sums complete and visible before the chain walks read them back
  __threadfence();
  __syncthreads();
  prune_group_prefixes(a, q, g, s_part + kPrChunk * (a.DP / 16 + 1), kPrThreads);   // ends with a barrier
}

// s_x [DP], s_part [kPrChunk][DP/16 + 1], then the group prefixes [gnodes_max]
size_t prune_pair_lds(int DP, int gmax) {
  return ((size_t)DP + (size_t)kPrChunk * (DP / 16 + 1) + (size_t)gmax) * 4;
}

// Every (query, group) pair's bound terms, one wave each over the whole chip
// (prune_group_terms: the group shift, |x - c_g|^2, the Pt-free part of KUB) -- before the
// head, so a call of one query spreads its G waves over many CUs.
__global__ void prune_terms_kernel(const PruneArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t w = blockIdx.x * (int64_t)(blockDim.x / 64) + (threadIdx.x >> 6);
  if (w >= (int64_t)a.nq * a.G) return;
  const int q = (int)(w / a.G), g = (int)(w % a.G);
  prune_group_terms(a, a.q + (int64_t)q * a.D, a.c0, q, g, lane);
}

// Head, one workgroup per query: the top nodes' raw sums (every (node, 16-dim slice) partial
// in parallel, one thread per node adding them in slice order: the scan's sums bit for bit)
// and their prefixes level by level (internal_chain_kernel's chain: the root's w lp', then
// fmaf(w, lp', P(parent))) with their tables; from the bound terms (prune_terms_kernel) KUB[q][g] = max(iLmin Pt, iLmax Pt) + kpart + 2^-16 (iLmax |Pt| + Cmax
// mag), Pt = P(t_g) the exact prefix of the centre's parent (the rest of the key's fp32 chain:
// <= 64 fmaf steps and the final fmaf, < 2^-17 of its terms), rounded up; g* = the group
// whose centre point scores best among those with >= K seed rows (any group will do for the
// threshold: its K rows' exact keys are <= tau_K; a good one prunes the most).  Block 0 zeroes the pair and claim counters (and the call's total on its
// first pruned chunk).
constexpr int kHdThreads = 512, kHdChunk = 32;
__global__ __launch_bounds__(kHdThreads) void prune_head_kernel(const PruneArgs a) {
  __shared__ float s_x[2048];                // the query's padded slices (DP <= 2048)
  __shared__ float s_tp[kHdChunk * 129];     // partials of a chunk of top nodes [kHdChunk][NV16 + 1]
  __shared__ float s_St[kPruneMaxTop], s_Pt[kPruneMaxTop];   // the top nodes' raw sums and prefixes
  __shared__ double s_best[kHdThreads / 64];
  __shared__ int s_bg[kHdThreads / 64], s_bt[kHdThreads / 64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int q = blockIdx.x;
  const int NV16 = a.DP / 16, LDP = NV16 + 1;
  if (q == 0 && tid < 6 && (tid != 4 || a.zero_total)) a.ctr[tid] = 0;
  prune_load_query(a, q, s_x, kHdThreads);
  __syncthreads();
  for (int c0 = 0; c0 < a.n_top; c0 += kHdChunk) {
    const int cnt = min(kHdChunk, a.n_top - c0);
    for (int it = tid; it < cnt * NV16; it += kHdThreads) {
      const int e = it / NV16, v = it - e * NV16;
      const int node = a.top_nodes[c0 + e];
      const float* __restrict__ ar = a.Ar + (size_t)node * a.DP + v * 16;
      const float* __restrict__ br = a.Br + (size_t)node * a.DP + v * 16;
      float4 a4[4], b4[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        a4[j] = *reinterpret_cast<const float4*>(ar + j * 4);
        b4[j] = *reinterpret_cast<const float4*>(br + j * 4);
      }
      float part;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const float4 ta = a4[j >> 2], tb = b4[j >> 2];
        const float aj = (j & 3) == 0 ? ta.x : (j & 3) == 1 ? ta.y : (j & 3) == 2 ? ta.z : ta.w;
        const float bj = (j & 3) == 0 ? tb.x : (j & 3) == 1 ? tb.y : (j & 3) == 2 ? tb.z : tb.w;
        const float tt = fmaf(s_x[v * 16 + j], aj, -bj);
        part = (j == 0) ? tt * tt : fmaf(tt, tt, part);
      }
      s_tp[e * LDP + v] = part;
    }
    __syncthreads();
    if (tid < cnt) {
      const float acc = sum_in_order(s_tp + tid * LDP, NV16);
      a.S[(size_t)q * a.ldS + a.top_nodes[c0 + tid]] = acc;
      s_St[c0 + tid] = acc;
    }
    __syncthreads();
  }
  for (int L = 0; L <= a.top_maxdep; ++L) {   // BFS list: a level's parents are finished first
    for (int j = tid; j < a.n_top; j += kHdThreads) {
      if (a.top_dep[j] != L) continue;
      const int node = a.top_nodes[j], pp = a.top_ppos[j];
      const float lp = -0.5f * (a.logdet_int[node] + s_St[j]);
      const float P = pp < 0 ? a.w_int[node] * lp : fmaf(a.w_int[node], lp, s_Pt[pp]);
      s_Pt[j] = P;
      prune_write_tables(a, q, node, P);
    }
    __syncthreads();
  }
  // g*: the group whose centre scores best (kpart[2], the bound at the centre point) among
  // the groups with >= K sample rows (the seed threshold needs K of them); none of those: the
  // best KUB.  Order: (tier, score, smaller g).
  double best = -INFINITY;
  int bt = -1, bg = 0x7fffffff;
  auto better = [](int t1, double s1, int g1, int t2, double s2, int g2) {
    return t1 != t2 ? t1 > t2 : (s1 != s2 ? s1 > s2 : g1 < g2);
  };
  for (int g = tid; g < a.G; g += kHdThreads) {
    const GroupBound b = a.gb[g];
    const size_t o = (size_t)q * a.G + g;
    double kub = -INFINITY;
    if (b.valid) {
      const double Pt = (double)s_Pt[a.grp_tpos[g]];
      const double pt = fmax(b.iLmin * Pt, b.iLmax * Pt);
      kub = pt + a.kpart[o] + 0x1p-16 * (b.iLmax * fabs(Pt) + a.kpart[(size_t)a.nq * a.G + o]);
      const int tier = a.gs_ptr[g + 1] - a.gs_ptr[g] >= a.K ? 1 : 0;
      const double sc = tier ? pt + a.kpart[(size_t)2 * a.nq * a.G + o] : kub;
      if (better(tier, sc, g, bt, best, bg)) {
        bt = tier;
        best = sc;
        bg = g;
      }
    }
    a.kub[o] = b.valid ? __double2float_ru(kub) : -INFINITY;
  }
  for (int off = 32; off > 0; off >>= 1) {
    const double ob = __shfl_xor(best, off, 64);
    const int ot = __shfl_xor(bt, off, 64);
    const int og = __shfl_xor(bg, off, 64);
    if (better(ot, ob, og, bt, best, bg)) {
      best = ob;
      bt = ot;
      bg = og;
    }
  }
  if (lane == 0) {
    s_best[wave] = best;
    s_bt[wave] = bt;
    s_bg[wave] = bg;
  }
  __syncthreads();
  if (tid == 0) {
    for (int w = 1; w < kHdThreads / 64; ++w)
      if (better(s_bt[w], s_best[w], s_bg[w], bt, best, bg)) {
        best = s_best[w];
        bt = s_bt[w];
        bg = s_bg[w];
      }
    a.gstar[q] = bg == 0x7fffffff ? -1 : bg;
  }
}

// g*'s exact pass: kGsNodes of its nodes per workgroup, nb workgroups per query (the
// workgroups past g*'s list leave at once) -- the per-call path's one query then reads its
// best group's ~100s of node rows with a few dozen CUs instead of one.
constexpr int kGsNodes = 16, kGsThreads = 256;
__global__ __launch_bounds__(kGsThreads) void prune_gstar_kernel(const PruneArgs a, int nb) {
  extern __shared__ float s_dyn[];
  float* s_x = s_dyn;
  float* s_part = s_dyn + a.DP;
  const int q = blockIdx.x / nb, blk = blockIdx.x - q * nb;
  const int g = a.gstar[q];
  if (g < 0) return;
  const int c0 = a.gi_ptr[g] + blk * kGsNodes, b1 = a.gi_ptr[g + 1];
  if (c0 >= b1) return;
  prune_load_query(a, q, s_x, kGsThreads);
  __syncthreads();
  prune_nodes_S<kGsThreads>(a, q, c0, min(kGsNodes, b1 - c0), s_x, s_part);
}

// g*'s exact pass for a batch: one workgroup per (group, kGgNodes of its nodes) serving every
// query whose g* is that group -- the nodes' A / B rows staged in LDS once and reused by the
// group's queries (a 1,000-query C2 chunk: ~10 queries per group; per query the same
// arithmetic as prune_nodes_S, bit for bit).  The group's queries are found by a scan of g*
// (windows of kGgWin queries; their order does not matter: each query's sums are its own).
constexpr int kGgNodes = 8, kGgThreads = 256, kGgWin = 1024;
// Off by default: measured slower (C2 batch, 1,000 queries: 1,163 us against 309 us for the
// per-query pass, profiles/r05_c2_batch_grouped_rocprof_kernel_stats.csv -- each workgroup
// walks its group's queries one after another, a load round trip and three barriers per
// query); CWQ_PRUNE_GROUPED_MIN = n takes it for chunks of >= n queries (A/B).
constexpr int kGgMinQ = 0x7fffffff;
__global__ __launch_bounds__(kGgThreads) void prune_gstar_grouped_kernel(const PruneArgs a, int nb) {
  extern __shared__ float s_dyn[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int NV16 = a.DP / 16, LDP = NV16 + 1;
  float* s_a = s_dyn;                           // [kGgNodes][DP]
  float* s_b = s_a + (size_t)kGgNodes * a.DP;   // [kGgNodes][DP]
  float* s_x = s_b + (size_t)kGgNodes * a.DP;   // [DP]
  float* s_part = s_x + a.DP;                   // [kGgNodes][LDP]
  int* s_q = reinterpret_cast<int*>(s_part + kGgNodes * LDP);   // [kGgWin]
  __shared__ int s_n;
  const int g = blockIdx.x / nb, blk = blockIdx.x - g * nb;
  const int c0 = a.gi_ptr[g] + blk * kGgNodes, b1 = a.gi_ptr[g + 1];
  if (c0 >= b1) return;
  const int cnt = min(kGgNodes, b1 - c0);
  bool staged = false;
  for (int w0 = 0; w0 < a.nq; w0 += kGgWin) {
    if (tid == 0) s_n = 0;
    __syncthreads();
    for (int q = w0 + tid; q < min(a.nq, w0 + kGgWin); q += kGgThreads) {
      const bool m = a.gstar[q] == g;
      const uint64_t bm = __ballot(m);
      int base = 0;
      if (lane == 0 && bm) base = atomicAdd(&s_n, __popcll(bm));
      base = __shfl(base, 0, 64);
      if (m) s_q[base + __popcll(bm & ((1ull << lane) - 1))] = q;
    }
    __syncthreads();
    const int n = s_n;
    if (n == 0) continue;   // uniform
    if (!staged) {
      for (int it = tid; it < cnt * a.DP; it += kGgThreads) {
        const int e = it / a.DP, d = it - e * a.DP;
        const size_t o = (size_t)a.gi_nodes[c0 + e] * a.DP + d;
        s_a[it] = a.Ar[o];
        s_b[it] = a.Br[o];
      }
      staged = true;
    }
    for (int i = 0; i < n; ++i) {
      const int q = s_q[i];
      prune_load_query(a, q, s_x, kGgThreads);
      __syncthreads();
      for (int it = tid; it < cnt * NV16; it += kGgThreads) {
        const int e = it / NV16, v = it - e * NV16;
        const float* ar = s_a + (size_t)e * a.DP + v * 16;
        const float* br = s_b + (size_t)e * a.DP + v * 16;
        float part;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          const float tt = fmaf(s_x[v * 16 + j], ar[j], -br[j]);
          part = (j == 0) ? tt * tt : fmaf(tt, tt, part);
        }
        s_part[e * LDP + v] = part;
      }
      __syncthreads();
      if (tid < cnt) {
        const float acc = sum_in_order(s_part + tid * LDP, NV16);
        a.S[(size_t)q * a.ldS + a.gi_nodes[c0 + tid]] = acc;
      }
      __syncthreads();   // s_x and s_part reused by the next query
    }
  }
}

// Seed threshold and stage-B pairs, one workgroup per query (blocks >= nq: the sentinel fill
// of every (query, node) outside the root and g*).  The exact keys of up to 64 sample rows of
// g* (their parents' prefixes: written first, from prune_gstar_kernel's raw sums): every (row, slice) partial in parallel, summed
// in slice order and finished by iso_key_tail -- the rerank's keys bit for bit -- so T = the
// K-th largest over distinct rows is <= tau_K (fewer than K rows: -inf).  Then the groups
// g != g* with KUB >= T go to the pair list.
constexpr int kSeedThreads = 256;
__global__ __launch_bounds__(kSeedThreads) void prune_seed_kernel(const PruneArgs a) {
  const int tid = threadIdx.x;
  if ((int)blockIdx.x >= a.nq) {   // sentinel fill
    const int64_t t = ((int64_t)blockIdx.x - a.nq) * kSeedThreads + tid;
    if (t >= (int64_t)a.nq * a.NI) return;
    const int q = (int)(t / a.NI), i = (int)(t % a.NI);
    const int g = a.gint[i];
    if (g < 0 || g == a.gstar[q]) return;   // top nodes (the head's) and g*'s
    const size_t o = (size_t)q * a.ldS + i;
    a.Plo[o] = kPruneSent;
    a.Phi[o] = kPruneSent;
    if (a.fillP) a.P[o] = kPruneSent;
    return;
  }
  extern __shared__ float s_part[];   // [64][NV16 + 1]
  __shared__ float s_T;
  const int q = blockIdx.x, lane = tid & 63, wave = tid >> 6;
  const int NV16 = a.DP / 16, LDP = NV16 + 1;
  const int g = a.gstar[q];
  // g*'s prefixes and tables (its raw sums: prune_gstar_kernel), read back below by the
  // sample rows whose parents they are
  if (g >= 0) prune_group_prefixes(a, q, g, s_part + 64 * LDP, kSeedThreads);   // ends with a barrier
  __threadfence();   // the P stores, read back below by other waves
  __syncthreads();
  const int n = g >= 0 ? min(64, a.gs_ptr[g + 1] - a.gs_ptr[g]) : 0;
  const float* xq = a.X + ((size_t)(q / kXQ) * NV16 * kXQ + (q % kXQ)) * 16;
  for (int it = tid; it < n * NV16; it += kSeedThreads) {
    const int e = it / NV16, v = it - e * NV16;
    const int rr = a.gs_rows[a.gs_ptr[g] + e];
    const float* __restrict__ mr = a.Mf + (size_t)rr * a.DP + v * 16;
    float4 m4[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) m4[j] = *reinterpret_cast<const float4*>(mr + j * 4);
    float part;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const float4 t4 = m4[j >> 2];
      const float mj = (j & 3) == 0 ? t4.x : (j & 3) == 1 ? t4.y : (j & 3) == 2 ? t4.z : t4.w;
      const float t = xq[(size_t)v * kXQ * 16 + j] - mj;
      part = (j == 0) ? t * t : fmaf(t, t, part);
    }
    s_part[e * LDP + v] = part;
  }
  __syncthreads();
  if (wave == 0) {
    float key = -__builtin_inff();
    int rid = 0x7fffffff;
    if (lane < n) {
      const int rr = a.gs_rows[a.gs_ptr[g] + lane];
      const float acc = sum_in_order(s_part + lane * LDP, NV16);
      const int p = a.row_par[rr];
      const float pp = p >= 0 ? a.P[(size_t)q * a.ldS + p] : 0.f;
      float lp;
      key = iso_key_tail(acc, a.meta[rr], pp, lp, 0, 0.f);
      if (!(key == key)) key = -__builtin_inff();
      rid = rr;
    }
    float dummy = 0.f;
    wave_sort64<false>(key, rid, dummy, lane);
    const float tk = __shfl(key, a.K - 1, 64);
    if (lane == 0) {
      const float T = n >= a.K ? tk : -__builtin_inff();
      s_T = T;
      a.Tseed[q] = T;
      if (a.T0) a.T0[(size_t)q * a.ldT0] = T;
    }
  }
  __syncthreads();
  const float T = s_T;
  for (int gg = tid; gg < a.G; gg += kSeedThreads) {
    if (gg == g || !a.gb[gg].valid) continue;
    if (a.kub[(size_t)q * a.G + gg] >= T || !(T == T)) {
      const int j = atomicAdd(&a.ctr[0], 1);
      a.pairs[j] = make_int2(q, gg);
      atomicAdd(&a.ctr[4], 1);   // the call's total (diagnostics)
    }
  }
}

// Group g kept for query q: g*, or a valid group whose KUB reaches the seed threshold (the
// seed kernel's pair test).
__device__ __forceinline__ bool prune_kept(const PruneArgs& a, int q, int g) {
  if (g == a.gstar[q]) return true;
  if (!a.gb[g].valid) return false;
  const float T = a.Tseed[q];
  return a.kub[(size_t)q * a.G + g] >= T || !(T == T);
}

// Stage B: persistent workgroups claim the pairs; every workgroup leaves when the claim
// counter passes the pair count.  First (blk_grp set) the live list of 16-row blocks for the
// filter pass: one thread per block, appended in any order (the candidate lists' order does
// not reach the results: the rerank orders by key and row).
__global__ __launch_bounds__(kPrThreads) void prune_stage_b_kernel(const PruneArgs a) {
  extern __shared__ float s_dyn[];
  float* s_x = s_dyn;
  float* s_part = s_dyn + a.DP;
  __shared__ int s_p;
  if (a.blk_grp) {
    const int lane = threadIdx.x & 63;
    for (int64_t b0 = (int64_t)blockIdx.x * kPrThreads; b0 < a.nblk; b0 += (int64_t)gridDim.x * kPrThreads) {
      const int64_t b = b0 + threadIdx.x;
      bool keep = false;
      if (b < a.nblk) {
        const int g = a.blk_grp[b];
        keep = g < 0;
        for (int q = 0; q < a.nq && !keep; ++q) keep = prune_kept(a, q, g);
      }
      const uint64_t m = __ballot(keep);
      int base = 0;
      if (lane == 0 && m) base = atomicAdd(&a.ctr[5], __popcll(m));
      base = __shfl(base, 0, 64);
      if (keep) a.live[base + __popcll(m & ((1ull << lane) - 1))] = (int)b;
    }
  }
  const int npairs = a.ctr[0];
  for (;;) {
    if (threadIdx.x == 0) s_p = atomicAdd(&a.ctr[3], 1);
    __syncthreads();
    const int p = s_p;
    __syncthreads();
    if (p >= npairs) break;
    const int2 pr = a.pairs[p];
    prune_pair(a, pr.x, pr.y, s_x, s_part);
  }
}

// A kernel's dynamic-LDS limit raised to `bytes` when that passes the 64 KiB default (and
// what was set before for that kernel on the current device): the attribute is only ever set
// to a size the launch requests, which with the kernel's static LDS stays within the 160 KiB
// of a CU.  One process-wide table under a mutex: calls on different index handles (each
// serialised by its own mutex only) may launch the same kernels concurrently.
hipError_t ensure_dyn_lds(const void* fn, size_t bytes) {
  if (bytes <= (size_t)64 * 1024) return hipSuccess;
  int dev = 0;
  if (hipError_t e = hipGetDevice(&dev)) return e;
  static std::mutex mu;
  static std::map<std::pair<const void*, int>, size_t> cur;
  std::lock_guard<std::mutex> lk(mu);
  size_t& c = cur[{fn, dev}];
  if (bytes <= c) return hipSuccess;
  const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
  if (e == hipSuccess) c = bytes;
  else (void)hipGetLastError();   // not left as the runtime's sticky error for the next caller
  return e;
}

// The seed and stage-B kernels' dynamic LDS for a largest group of gmax internal nodes
// (build_prune keeps pruning off when it passes kPruneLdsCap).
size_t prune_lds_max(int DP, int gmax) {
  const size_t seed = ((size_t)64 * (DP / 16 + 1) + (size_t)gmax) * 4;
  return std::max(seed, prune_pair_lds(DP, gmax));
}

// The whole pruned internal pass of a chunk: head, g*'s pass, seed (+ fill), stage B.
// ctr[0..3] zeroed by the head, and ctr[4] (the call's stage-B pair total) on its first
// pruned chunk.
hipError_t launch_prune(const PruneArgs& a0, int cus, bool first, hipStream_t s) {
  if (a0.nq <= 0) return hipSuccess;
  if (a0.DP % 16 || a0.DP / 16 > 128 || a0.gnodes_max < 1 || a0.n_top < 1 || a0.n_top > kPruneMaxTop ||
      prune_lds_max(a0.DP, a0.gnodes_max) > kPruneLdsCap)
    return hipErrorInvalidValue;
  PruneArgs a = a0;
  a.zero_total = first ? 1 : 0;
  const int64_t npg = (int64_t)a.nq * a.G;
  hipLaunchKernelGGL(prune_terms_kernel, dim3((unsigned)((npg + 3) / 4)), dim3(256), 0, s, a);
  hipLaunchKernelGGL(prune_head_kernel, dim3((unsigned)a.nq), dim3(kHdThreads), 0, s, a);
  int gmin = kGgMinQ;
  if (const char* e = getenv("CWQ_PRUNE_GROUPED_MIN")) gmin = atoi(e) > 0 ? atoi(e) : kGgMinQ;
  if (a.nq >= gmin) {   // a batch: per (group, node chunk), the group's queries together
    const int nbg = (a.gnodes_max + kGgNodes - 1) / kGgNodes;
    const size_t lds = ((size_t)(2 * kGgNodes + 1) * a.DP + (size_t)kGgNodes * (a.DP / 16 + 1) + kGgWin) * 4;
    if (hipError_t e = ensure_dyn_lds(reinterpret_cast<const void*>(&prune_gstar_grouped_kernel), lds)) return e;
    hipLaunchKernelGGL(prune_gstar_grouped_kernel, dim3((unsigned)((int64_t)a.G * nbg)), dim3(kGgThreads), lds, s, a,
                       nbg);
  } else {   // a few queries: per (query, node chunk)
    const int nb = (a.gnodes_max + kGsNodes - 1) / kGsNodes;
    hipLaunchKernelGGL(prune_gstar_kernel, dim3((unsigned)((int64_t)a.nq * nb)), dim3(kGsThreads),
                       ((size_t)a.DP + (size_t)kGsNodes * (a.DP / 16 + 1)) * 4, s, a, nb);
  }
  // the group-prefix LDS of a large group can pass the 64 KiB default
  const size_t lds_seed = ((size_t)64 * (a.DP / 16 + 1) + (size_t)a.gnodes_max) * 4;
  const size_t lds_b = prune_pair_lds(a.DP, a.gnodes_max);
  if (hipError_t e = ensure_dyn_lds(reinterpret_cast<const void*>(&prune_seed_kernel), lds_seed)) return e;
  if (hipError_t e = ensure_dyn_lds(reinterpret_cast<const void*>(&prune_stage_b_kernel), lds_b)) return e;
  const int64_t nfill = ((int64_t)a.nq * a.NI + kSeedThreads - 1) / kSeedThreads;
  hipLaunchKernelGGL(prune_seed_kernel, dim3((unsigned)(a.nq + nfill)), dim3(kSeedThreads), lds_seed, s, a);
  const int64_t nw = (int64_t)a.nq * a.G;
  const int wgs = (int)std::max<int64_t>(1, std::min<int64_t>(nw, cus));
  hipLaunchKernelGGL(prune_stage_b_kernel, dim3((unsigned)wgs), dim3(kPrThreads), lds_b, s, a);
  return hipGetLastError();
}

// T[q * ldT] = max(T, Tfloor[q]) (both lower bounds of tau_K; the filter's sample / probe
// threshold sees only the groups pruning kept, the seed only the best group's sample rows).
__global__ void raise_threshold_kernel(float* T, int64_t ldT, const float* __restrict__ Tfloor, int nq) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q < nq) T[(size_t)q * ldT] = fmaxf(T[(size_t)q * ldT], Tfloor[q]);
}

hipError_t launch_raise_threshold(float* T, int64_t ldT, const float* Tfloor, int nq, hipStream_t s) {
  if (nq <= 0) return hipSuccess;
  hipLaunchKernelGGL(raise_threshold_kernel, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, s, T, ldT, Tfloor, nq);
  return hipGetLastError();
}

}  // namespace cwq
