// libcwq: incremental fit (ifit) support -- the category-utility scoring of the
// add path on the GPU.
//
// Node statistics live in a device pool (count[cap], mean[cap][D], meanSq[cap][D]).
// The host walks the tree and selects operations exactly as CobwebTorchTree.cobweb
// (CobwebTorchTree.py:143-233) does; every D-length arithmetic runs here:
//   * cwq_fit_kl: one wave per job computes compute_score = KL(cand || ref)
//     (CobwebTorchTree.py:344-364) for cand in {node, node+x, new(x), merge(a,b)+x}
//     and ref in {P, P+x} -- all the per-child terms of two_best_children /
//     pu_for_insert / pu_for_new_child / pu_for_merge / pu_for_split
//     (CobwebTorchNode.py:374-650) in one launch per tree level;
//   * cwq_fit_node_op: increment_counts / update_counts_from_node / zero /
//     is_exact_match (CobwebTorchNode.py:57-85, 652-666).
// The element-wise fp32 op sequence follows the reference exactly (FMA
// contraction off); the two D-sums are accumulated in fp64 and rounded once.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "../../include/cobweb_query.h"
#include "cwq_refmath.h"

namespace cwq {

struct Stats {
  const float* count;
  const float* mean;
  const float* meanSq;
};

// candidate / reference distribution of element d (fp32, reference op order)
__device__ __forceinline__ void insert_mv(float c, float m, float m2, float x, float pv, float& mo, float& vo) {
#pragma clang fp contract(off)
  const float cnt = c + 1.0f;
  const float delta = x - m;
  const float mm = m + delta / cnt;
  const float mm2 = m2 + delta * (x - mm);
  mo = mm;
  vo = mm2 / cnt + pv;
}

__global__ void fit_kl_kernel(Stats st, int D, const float* __restrict__ x, float pv, int p_slot,
                              const int* __restrict__ jobs, int n_jobs, float* out) {
#pragma clang fp contract(off)
  const int lane = threadIdx.x & 63;
  const int job = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (job >= n_jobs) return;
  const int type = jobs[4 * job], n1 = jobs[4 * job + 1], n2 = jobs[4 * job + 2], rtype = jobs[4 * job + 3];
  const float cP = st.count[p_slot];
  const float c1 = n1 >= 0 ? st.count[n1] : 0.f;
  const float c2 = n2 >= 0 ? st.count[n2] : 0.f;
  float sa, sb;
  torch_sum2(D, lane, [&](int d, float& a, float& b) {
#pragma clang fp contract(off)
    const float xd = x[d];
    // reference P or P+x
    float mu2, v2;
    const float mP = st.mean[(size_t)p_slot * D + d], m2P = st.meanSq[(size_t)p_slot * D + d];
    if (rtype == 1) {
      insert_mv(cP, mP, m2P, xd, pv, mu2, v2);
    } else {
      mu2 = mP;
      v2 = m2P / cP + pv;
    }
    float mu1, v1;
    if (type == 0) {
      mu1 = st.mean[(size_t)n1 * D + d];
      v1 = st.meanSq[(size_t)n1 * D + d] / c1 + pv;
    } else if (type == 1) {
      insert_mv(c1, st.mean[(size_t)n1 * D + d], st.meanSq[(size_t)n1 * D + d], xd, pv, mu1, v1);
    } else if (type == 2) {
      mu1 = xd;
      v1 = 0.f + pv;
    } else {   // mean_var_merge(n1, n2, x), CobwebTorchNode.py:224-239
      const float ma = st.mean[(size_t)n1 * D + d], mb = st.mean[(size_t)n2 * D + d];
      const float sa2 = st.meanSq[(size_t)n1 * D + d], sb2 = st.meanSq[(size_t)n2 * D + d];
      const float delta = mb - ma;
      const float tot = c1 + c2;
      float m2 = (sa2 + sb2) + (delta * delta) * ((c1 * c2) / tot);
      float m = (c1 * ma + c2 * mb) / tot;
      const float cnt = tot + 1.0f;
      const float dl = xd - m;
      m = m + dl / cnt;
      m2 = m2 + dl * (xd - m);
      mu1 = m;
      v1 = m2 / cnt + pv;
    }
    a = ref_logf(v2) - ref_logf(v1);
    const float df = mu1 - mu2;
    b = (v1 + df * df) / v2;
  }, sa, sb);
  if (lane == 0) {
    float score = sa;
    score = score + sb;
    score = score - (float)D;
    score = score / 2.0f;
    out[job] = score;
  }
}

// op 0: increment_counts(dst, x)      op 1: update_counts_from_node(dst, src)
// op 2: zero(dst)                      op 3: is_exact_match(dst, x) -> *flag
__global__ void fit_node_op_kernel(int op, float* count, float* mean, float* meanSq, int D, int dst, int src,
                                   const float* __restrict__ x, int* flag) {
#pragma clang fp contract(off)
  __shared__ int all_ok;
  const float cd = count[dst];
  const float cs = src >= 0 ? count[src] : 0.f;
  if (threadIdx.x == 0) all_ok = 1;
  __syncthreads();
  int ok = 1;
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    const size_t o = (size_t)dst * D + d;
    if (op == 0) {
      const float cnt = cd + 1.0f;
      const float delta = x[d] - mean[o];
      const float m = mean[o] + delta / cnt;
      meanSq[o] = meanSq[o] + delta * (x[d] - m);
      mean[o] = m;
    } else if (op == 1) {
      const size_t os = (size_t)src * D + d;
      const float delta = mean[os] - mean[o];
      const float tot = cd + cs;
      meanSq[o] = (meanSq[o] + meanSq[os]) + (delta * delta) * ((cd * cs) / tot);
      mean[o] = (cd * mean[o] + cs * mean[os]) / tot;
    } else if (op == 2) {
      mean[o] = 0.f;
      meanSq[o] = 0.f;
    } else {
      const float sd = sqrtf(meanSq[o] / cd);
      if (!(fabsf(sd) <= 1e-8f)) ok = 0;
      if (!(fabsf(x[d] - mean[o]) <= 1e-8f + 1e-5f * fabsf(mean[o]))) ok = 0;
    }
  }
  if (op == 3 && !ok) atomicAnd(&all_ok, 0);
  __syncthreads();
  if (threadIdx.x == 0) {
    if (op == 0) count[dst] = cd + 1.0f;
    if (op == 1) count[dst] = cd + cs;
    if (op == 2) count[dst] = 0.f;
    if (op == 3) *flag = all_ok;
  }
}

}  // namespace cwq

extern "C" int cwq_fit_kl(const float* count, const float* mean, const float* meanSq, int32_t dim, const float* x,
                          float prior_var, int32_t p_slot, const int32_t* jobs, int32_t n_jobs, float* out,
                          void* stream) {
  if (!count || !mean || !meanSq || !x || !jobs || !out || dim <= 0 || n_jobs < 0 || p_slot < 0) return CWQ_ERR_ARG;
  if (n_jobs == 0) return CWQ_OK;
  cwq::Stats st{count, mean, meanSq};
  hipLaunchKernelGGL(cwq::fit_kl_kernel, dim3((n_jobs + 3) / 4), dim3(256), 0, (hipStream_t)stream, st, dim, x,
                     prior_var, p_slot, jobs, n_jobs, out);
  return hipGetLastError() == hipSuccess ? CWQ_OK : CWQ_ERR_HIP;
}

extern "C" int cwq_fit_node_op(int32_t op, float* count, float* mean, float* meanSq, int32_t dim, int32_t dst,
                               int32_t src, const float* x, int32_t* flag, void* stream) {
  if (op < 0 || op > 3 || !count || !mean || !meanSq || dim <= 0 || dst < 0) return CWQ_ERR_ARG;
  if ((op == 0 || op == 3) && !x) return CWQ_ERR_ARG;
  if (op == 1 && src < 0) return CWQ_ERR_ARG;
  if (op == 3 && !flag) return CWQ_ERR_ARG;
  hipLaunchKernelGGL(cwq::fit_node_op_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, op, count, mean, meanSq, dim,
                     dst, src, x, flag);
  return hipGetLastError() == hipSuccess ? CWQ_OK : CWQ_ERR_HIP;
}
