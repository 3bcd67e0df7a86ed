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
// Stage A (before the filter's threshold exists): for each query only its best group g* =
// argmax_g KUB gets the exact internal pass (prune_scan_kernel: the scan's arithmetic, bit
// for bit) and exact prefixes; every other (query, node) gets the sentinel prefix kPruneSent
// in the filters' tables, so its rows are never candidates and their lower bounds never
// raise a threshold.  The filter's first threshold T[q] (the sample / probe pass: the K-th
// largest lower bound over distinct rows, <= tau_K) then decides stage B: the groups with
// KUB[q][g] >= T[q] get the exact pass too.  Every group left has KUB < T <= tau_K: none of
// its rows can be in the top-K, so the result is the exact scan's bit for bit.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <algorithm>

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

// The root's exact prefix, as internal_chain_kernel / prefix_level_kernel form it.
__device__ __forceinline__ float prune_root_prefix(const PruneArgs& a, int q) {
  const float lp = -0.5f * (a.logdet_int[0] + a.S[(size_t)q * a.ldS]);
  return a.w_int[0] * lp;
}

// KUB[q][g] for every group and g*(q) = argmax (ties: the smaller g).  One wave per query.
__global__ void prune_bound_kernel(const PruneArgs a) {
  const int lane = threadIdx.x & 63;
  const int q = blockIdx.x * (int)(blockDim.x / 64) + (int)(threadIdx.x >> 6);
  if (q >= a.nq) return;
  const double P0 = (double)prune_root_prefix(a, q);
  double best = -INFINITY;
  int bg = 0x7fffffff;
  for (int g = lane; g < a.G; g += 64) {
    const GroupBound b = a.gb[g];
    double kub = -INFINITY;
    if (b.valid) {
      const double e2 = a.dist2[(size_t)q * a.G + g];
      const double dist_lo = sqrt(e2 * (1.0 - 0x1p-40)) * (1.0 - 0x1p-50);
      const double dist_hi = sqrt(e2 * (1.0 + 0x1p-40)) * (1.0 + 0x1p-50);
      const double dlo = fmax(0.0, dist_lo - b.r);
      // S_fp32 >= (1 - 2^-16) (sqrt(wmin) dlo - 2^-23 sqrt(wmax) mmax)_+^2: the t = x A - B
      // rounding (B = fl(mu A)) and the fp32 sums' relative error (< 64 * 2^-24)
      const double sv = sqrt(b.wmin) * dlo - 0x1p-23 * sqrt(b.wmax) * b.mmax;
      const double SLB = sv > 0.0 ? (1.0 - 0x1p-16) * sv * sv : 0.0;
      // lp'_fp32 = fl(-0.5 fl(logdet + S)) <= -logdet/2 + 2^-22 |logdet| - (1/2 - 2^-22) S_fp32
      const double UB = -0.5 * b.ldmin + 0x1p-22 * b.ldabs - (0.5 - 0x1p-22) * SLB;
      // |lp'| of any member, for the rounding margin of the keys' fp32 chains
      const double shv = sqrt(b.wmax) * (dist_hi + b.r) + 0x1p-23 * sqrt(b.wmax) * b.mmax;
      const double mag = 0.5 * (b.ldabs + (1.0 + 0x1p-16) * shv * shv) * (1.0 + 0x1p-20);
      kub = fmax(b.iLmin * P0, b.iLmax * P0) + fmax(b.Cmin * UB, b.Cmax * UB);
      // the exact key's fp32 chain (<= 64 fmaf steps + the final fmaf): < 2^-17 of its terms
      kub += 0x1p-16 * (b.iLmax * fabs(P0) + b.Cmax * mag);
    }
    a.kub[(size_t)q * a.G + g] = b.valid ? __double2float_ru(kub) : -INFINITY;
    if (b.valid && (kub > best || (kub == best && g < bg))) {
      best = kub;
      bg = g;
    }
  }
  for (int off = 32; off > 0; off >>= 1) {
    const double ob = __shfl_xor(best, off, 64);
    const int og = __shfl_xor(bg, off, 64);
    if (ob > best || (ob == best && og < bg)) {
      best = ob;
      bg = og;
    }
  }
  if (lane == 0) a.gstar[q] = bg == 0x7fffffff ? -1 : bg;
}

// Exact prefix of internal node i for query q from the raw sums S (the node's ancestors all
// computed): internal_chain_kernel's arithmetic, top-down, bit for bit.
__device__ __forceinline__ float prune_chain_prefix(const PruneArgs& a, int q, int i) {
  const size_t ro = (size_t)q * a.ldS;
  int d = 0;
  for (int j = i; a.par_int[j] >= 0 && d < kMaxChain; j = a.par_int[j]) ++d;
  float P = 0.f;
  for (int l = d; l >= 0; --l) {
    int j = i;
    for (int u = 0; u < l; ++u) j = a.par_int[j];
    const float lp = -0.5f * (a.logdet_int[j] + a.S[ro + j]);
    P = (l == d) ? a.w_int[j] * lp : fmaf(a.w_int[j], lp, P);
  }
  return P;
}

// P, and the filters' tables [Plo, Phi] of node i (internal_chain_kernel's tail: the
// group-centred rows' shifted prefix, outward-rounded).
__device__ __forceinline__ void prune_write_prefix(const PruneArgs& a, int q, int i) {
  const size_t o = (size_t)q * a.ldS + i;
  const float P = prune_chain_prefix(a, q, i);
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

// Stage A tables over every (query, node): the root and the nodes of g*(q) exact, the rest
// the sentinel.
__global__ void prune_prefix_all_kernel(const PruneArgs a) {
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (t >= (int64_t)a.nq * a.NI) return;
  const int q = (int)(t / a.NI);
  const int i = (int)(t % a.NI);
  const int g = a.gint[i];
  if (i == 0 || (g >= 0 && g == a.gstar[q])) {
    prune_write_prefix(a, q, i);
    return;
  }
  const size_t o = (size_t)q * a.ldS + i;
  a.Plo[o] = kPruneSent;
  a.Phi[o] = kPruneSent;
  if (a.fillP) a.P[o] = kPruneSent;
}

// Stage B pair list: (q, g) with g != g*(q) and KUB[q][g] >= T[q] (T = -inf or NaN: every
// valid group).
__global__ void prune_pairs_kernel(const PruneArgs a, const float* __restrict__ T, int64_t ldT) {
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (t >= (int64_t)a.nq * a.G) return;
  const int q = (int)(t / a.G);
  const int g = (int)(t % a.G);
  if (g == a.gstar[q] || !a.gb[g].valid) return;
  const float Tq = T[(size_t)q * ldT];
  if (a.kub[t] >= Tq || !(Tq == Tq)) {
    const int j = atomicAdd(&a.ctr[0], 1);
    a.pairs[j] = make_int2(q, g);
    atomicAdd(&a.ctr[4], 1);   // the call's total (diagnostics)
  }
}

// The exact internal pass of (query, group) pairs: persistent workgroups claim (pair, chunk
// of 64 of the group's nodes) tasks from a counter (stage A: pair p = (p, g*(p)); B: the
// list), stage the query's slices in LDS, form every (node, 16-dim slice) partial of the
// chunk in parallel -- exact_aniso_S's fma chain -- and one thread per node adds its
// partials in slice order: the scan kernel's raw sums bit for bit.  A one-query call spreads
// a group's chunks over as many workgroups.  Every workgroup leaves when the counter passes
// the task count.
constexpr int kPrThreads = 256, kPrChunk = 64;
__global__ __launch_bounds__(kPrThreads) void prune_scan_kernel(const PruneArgs a, int stage_b, int* claim) {
  extern __shared__ float s_dyn[];
  const int NV16 = a.DP / 16, LDP = NV16 + 1;
  float* s_x = s_dyn;                  // [DP] the query's slices
  float* s_part = s_dyn + a.DP;        // [kPrChunk][LDP]
  __shared__ int s_t;
  const int tid = threadIdx.x;
  const int mc = a.max_chunks;
  const int64_t ntask = (int64_t)(stage_b ? a.ctr[0] : a.nq) * mc;
  for (;;) {
    if (tid == 0) s_t = atomicAdd(claim, 1);
    __syncthreads();
    const int t = s_t;
    __syncthreads();
    if (t >= ntask) break;
    const int p = t / mc, ch = t - p * mc;
    int q, g;
    if (stage_b) {
      const int2 pr = a.pairs[p];
      q = pr.x;
      g = pr.y;
    } else {
      q = p;
      g = a.gstar[p];
    }
    if (g < 0) continue;
    const int c0 = a.gi_ptr[g] + ch * kPrChunk, b1 = a.gi_ptr[g + 1];
    if (c0 >= b1) continue;   // uniform over the workgroup
    const int cnt = min(kPrChunk, b1 - c0);
    const float* xq = a.X + ((size_t)(q / kXQ) * NV16 * kXQ + (q % kXQ)) * 16;
    for (int d = tid; d < a.DP; d += kPrThreads) {
      const int v = d >> 4, j = d & 15;
      s_x[d] = xq[(size_t)v * kXQ * 16 + j];
    }
    __syncthreads();
    for (int it = tid; it < cnt * NV16; it += kPrThreads) {
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
      float acc = 0.f;
      for (int v = 0; v < NV16; ++v) acc += s_part[tid * LDP + v];
      a.S[(size_t)q * a.ldS + a.gi_nodes[c0 + tid]] = acc;
    }
    __syncthreads();
  }
}

// Stage B prefixes: persistent workgroups over the pair list, threads over the group's nodes.
__global__ __launch_bounds__(256) void prune_prefix_pairs_kernel(const PruneArgs a, int* claim) {
  __shared__ int s_p;
  const int npairs = a.ctr[0];
  for (;;) {
    if (threadIdx.x == 0) s_p = atomicAdd(claim, 1);
    __syncthreads();
    const int p = s_p;
    __syncthreads();
    if (p >= npairs) break;
    const int2 pr = a.pairs[p];
    const int b0 = a.gi_ptr[pr.y], b1 = a.gi_ptr[pr.y + 1];
    for (int j = b0 + threadIdx.x; j < b1; j += blockDim.x) prune_write_prefix(a, pr.x, a.gi_nodes[j]);
  }
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

size_t prune_scan_lds(int DP) { return ((size_t)DP + (size_t)kPrChunk * (DP / 16 + 1)) * 4; }

// Stage A: bounds and g* (the caller has written the root's raw sums S[q][0] and the group
// shifts and distances), the exact pass of g*, the tables.  ctr[0..3] zeroed here, and
// ctr[4] (the call's stage-B pair total) on the call's first pruned chunk.
hipError_t launch_prune_stage_a(const PruneArgs& a, int cus, hipStream_t s, bool first) {
  if (a.nq <= 0) return hipSuccess;
  if (hipError_t e = hipMemsetAsync(a.ctr, 0, (first ? 5 : 4) * sizeof(int), s)) return e;
  hipLaunchKernelGGL(prune_bound_kernel, dim3((unsigned)((a.nq + 3) / 4)), dim3(256), 0, s, a);
  const int wgs = (int)std::max<int64_t>(1, std::min<int64_t>((int64_t)a.nq * a.max_chunks, (int64_t)cus * 4));
  hipLaunchKernelGGL(prune_scan_kernel, dim3((unsigned)wgs), dim3(kPrThreads), prune_scan_lds(a.DP), s, a, 0, a.ctr + 1);
  const int64_t n = (int64_t)a.nq * a.NI;
  hipLaunchKernelGGL(prune_prefix_all_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a);
  return hipGetLastError();
}

// Stage B, after the first threshold T[q * ldT] (<= tau_K) is on the device.
hipError_t launch_prune_stage_b(const PruneArgs& a, const float* T, int64_t ldT, int cus, hipStream_t s) {
  if (a.nq <= 0 || a.G <= 0) return hipSuccess;
  const int64_t n = (int64_t)a.nq * a.G;
  hipLaunchKernelGGL(prune_pairs_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a, T, ldT);
  const int wgs = std::max(1, (int)std::min<int64_t>(n * a.max_chunks, (int64_t)cus * 4));
  hipLaunchKernelGGL(prune_scan_kernel, dim3((unsigned)wgs), dim3(kPrThreads), prune_scan_lds(a.DP), s, a, 1, a.ctr + 2);
  const int wgp = std::max(1, (int)std::min<int64_t>(n, (int64_t)cus * 4));
  hipLaunchKernelGGL(prune_prefix_pairs_kernel, dim3((unsigned)wgp), dim3(256), 0, s, a, a.ctr + 3);
  return hipGetLastError();
}

}  // namespace cwq
