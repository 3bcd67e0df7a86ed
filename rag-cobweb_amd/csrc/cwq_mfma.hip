// libcwq: bf16-MFMA candidate filter + exact fp32 rerank for isotropic rows
// ("Cobweb Fast", A6).  Results are EXACT (identical keys to the fp32 scan):
//
//   1. approx_gemm: S~ = |x|^2 + |mu|^2 - 2 x.mu with x.mu on v_mfma_f32_32x32x16_bf16
//      (bf16 operands, fp32 accumulate); writes an UPPER BOUND of every key,
//        u = key~ + e(q, r),   e = 0.5*cw*iv*(2*eta*|x||mu| + ...)    (see bound_slack)
//      since |x.mu - (x.mu)~| <= eta * sum_d |x_d mu_d| <= eta |x| |mu| (Cauchy-Schwarz),
//      eta = 2*2^-8 + 2^-16 + D*2^-24 (bf16 rounding of both operands + fp32 sums);
//   2. select: per query the K' = 64 rows with the largest u;
//   3. rerank: exact fp32 keys of those rows, op for op the scan kernel's (so the
//      keys are bit-identical), top-k, and the certificate u_(K') < tau_k: every row
//      outside the set has key <= u <= u_(K') < tau_k.  Queries without the
//      certificate are flagged and re-run by the exact scan.
//
// CDNA4 mapping of the GEMM: 256-thread workgroups, 128 queries x 128 rows per
// workgroup, 2x2 waves each owning 64x64 = 2x2 tiles of 32x32 (four 16-register
// accumulators), K staged 32 deep through LDS (double buffer, 80-B padded rows:
// conflict-free ds_read_b128 fragment reads), queries fastest in the grid so the
// co-running workgroups share each row tile in L2.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <algorithm>

#include "cwq_internal.h"

namespace cwq {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16v __attribute__((ext_vector_type(16)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define CWQ_INF __builtin_inff()

__device__ __forceinline__ float rl_f2(float v, int lane) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}

// ---------------------------------------------------------------------------
// Row / query preparation: row-major fp32 copy (rerank), bf16 copy (GEMM), norms.
// The GEMM operands are centred on c (the root mean): |x-mu|^2 is unchanged while
// the bf16 error, ~|x-c||mu-c| instead of |x||mu|, tracks the spread of the data
// rather than its offset.  (The fp32 rounding of the centring is covered by eta_n.)
// ---------------------------------------------------------------------------
__global__ void rows_prep_kernel(const float* __restrict__ mean, int D, const int64_t* __restrict__ nodes, int64_t n,
                                 const float* __restrict__ c, int DP, int64_t ld, float* Mf, __bf16* Mb, float* n2,
                                 float* n1) {
  const int lane = threadIdx.x & 63;
  const int64_t r = blockIdx.x * (int64_t)kWavesPerWG + (threadIdx.x >> 6);
  if (r >= ld) return;
  double s = 0.0;
  for (int d = lane; d < DP; d += kWave) {
    const float v = (r < n && d < D) ? mean[nodes[r] * (int64_t)D + d] : 0.f;
    const float vc = (r < n && d < D) ? v - c[d] : 0.f;
    Mf[r * DP + d] = v;
    Mb[r * DP + d] = (__bf16)vc;
    s += (double)vc * (double)vc;
  }
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  if (lane == 0) {
    n2[r] = (float)s;
    n1[r] = (float)sqrt(s);
  }
}

hipError_t launch_rows_prep(const float* mean, int D, const int64_t* nodes, int64_t n, const float* c, int DP,
                            int64_t ld, float* Mf, void* Mb, float* n2, float* n1, hipStream_t s) {
  if (ld <= 0) return hipSuccess;
  hipLaunchKernelGGL(rows_prep_kernel, dim3((unsigned)((ld + 3) / 4)), dim3(256), 0, s, mean, D, nodes, n, c, DP, ld,
                     Mf, (__bf16*)Mb, n2, n1);
  return hipGetLastError();
}

__global__ void query_prep_kernel(const float* __restrict__ q, int64_t nq, int D, const float* __restrict__ c, int DP,
                                  int64_t nq_pad, __bf16* Xb, float* n2, float* n1) {
  const int lane = threadIdx.x & 63;
  const int64_t r = blockIdx.x * (int64_t)kWavesPerWG + (threadIdx.x >> 6);
  if (r >= nq_pad) return;
  double s = 0.0;
  for (int d = lane; d < DP; d += kWave) {
    const float v = (r < nq && d < D) ? q[r * D + d] - c[d] : 0.f;
    Xb[r * DP + d] = (__bf16)v;
    s += (double)v * (double)v;
  }
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  if (lane == 0) {
    n2[r] = (float)s;
    n1[r] = (float)sqrt(s);
  }
}

hipError_t launch_query_prep(const float* q, int64_t nq, int D, const float* c, int DP, int64_t nq_pad, void* Xb,
                             float* n2, float* n1, hipStream_t s) {
  hipLaunchKernelGGL(query_prep_kernel, dim3((unsigned)((nq_pad + 3) / 4)), dim3(256), 0, s, q, nq, D, c, DP, nq_pad,
                     (__bf16*)Xb, n2, n1);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// 1. approximate-key GEMM (bf16 MFMA) -> upper bounds u[q][r]
// ---------------------------------------------------------------------------
constexpr int GB = 128;        // queries and rows per workgroup tile
constexpr int GK = 32;         // K depth per LDS stage
constexpr int GLD = GK + 8;    // padded LDS row (80 B): conflict-free ds_read_b128


// u[q][r] = key~(q, r) + e(q, r) >= key(q, r)   (q local to the launch's query block)
__global__ __launch_bounds__(256) void approx_gemm_kernel(const __bf16* __restrict__ Xb, const __bf16* __restrict__ Mb,
                                                          float* __restrict__ u, const GemmArgs a) {
  __shared__ __attribute__((aligned(16))) __bf16 Xs[2][GB][GLD];
  __shared__ __attribute__((aligned(16))) __bf16 Ms[2][GB][GLD];
  __shared__ float sxn2[GB], sxn1[GB];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wq = wave >> 1, wr = wave & 1;
  const int qt = blockIdx.x % a.n_qt;
  const int rt = blockIdx.x / a.n_qt;
  const int q0 = qt * GB, r0 = rt * GB;
  if (tid < GB) {
    const int q = min(q0 + tid, a.nq - 1);
    sxn2[tid] = a.xn2[q];
    sxn1[tid] = a.xn1[q];
  }

  // staging: thread -> (tile row, 16-element half); operands are padded to whole tiles
  const int srow = tid >> 1, shalf = (tid & 1) * 16;
  const __bf16* xg = Xb + (size_t)(q0 + srow) * a.DP + shalf;
  const __bf16* mg = Mb + (size_t)(r0 + srow) * a.DP + shalf;
  typedef int v4i __attribute__((ext_vector_type(4)));
  v4i xr0, xr1, mr0, mr1;
  auto gload = [&](int k0) {
    xr0 = *reinterpret_cast<const v4i*>(xg + k0);
    xr1 = *reinterpret_cast<const v4i*>(xg + k0 + 8);
    mr0 = *reinterpret_cast<const v4i*>(mg + k0);
    mr1 = *reinterpret_cast<const v4i*>(mg + k0 + 8);
  };
  auto swrite = [&](int b) {
    *reinterpret_cast<v4i*>(&Xs[b][srow][shalf]) = xr0;
    *reinterpret_cast<v4i*>(&Xs[b][srow][shalf + 8]) = xr1;
    *reinterpret_cast<v4i*>(&Ms[b][srow][shalf]) = mr0;
    *reinterpret_cast<v4i*>(&Ms[b][srow][shalf + 8]) = mr1;
  };

  f32x16v acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  const int nk = a.DP / GK;
  gload(0);
  swrite(0);
  __syncthreads();
  const int fr = lane & 31, fk = (lane >> 5) * 8;
  for (int kt = 0; kt < nk; ++kt) {
    const int b = kt & 1;
    if (kt + 1 < nk) gload((kt + 1) * GK);
#pragma unroll
    for (int kk = 0; kk < GK / 16; ++kk) {
      bf16x8 af[2], bfr[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        af[t] = *reinterpret_cast<const bf16x8*>(&Xs[b][wq * 64 + t * 32 + fr][kk * 16 + fk]);
        bfr[t] = *reinterpret_cast<const bf16x8*>(&Ms[b][wr * 64 + t * 32 + fr][kk * 16 + fk]);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) swrite(b ^ 1);
    __syncthreads();
  }

  // ---- epilogue: C[i = query][j = row]; lane: row j = lane&31, query i = (e&3) + 8(e>>2) + 4(lane>>5)
  //   key~ = P[q][par]*invL + cw*(-0.5*(logdet + iv*S~)),  S~ = |x|^2 + |mu|^2 - 2 x.mu~
  //   e    = ci*(2 eta |x||mu| + eta_n(|x|^2+|mu|^2))                    (dot-product + norm rounding)
  //        + slack*(|P invL| + 0.5 cw |logdet| + 3 ci (|x|^2+|mu|^2))   (fp32 evaluation of both keys)
  //   with ci = 0.5*cw*iv and |S| <= 2(|x|^2+|mu|^2).
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int r = r0 + wr * 64 + j * 32 + (lane & 31);
    const bool vrow = r < a.nrows;
    RowMeta md{0.f, 0.f, 0.f, 0.f};
    int p = -1, fl = 0;
    float rn2 = 0.f, rn1 = 0.f;
    if (vrow) {
      md = a.meta[r];
      p = a.par[r];
      fl = a.flags[r];
      rn2 = a.rn2[r];
      rn1 = a.rn1[r];
    }
    const bool usable = vrow && (fl & FLAG_HAS_SENT);
    const float ci = 0.5f * md.cw * md.iv;
    const float c1 = 2.0f * a.eta * ci * rn1;
    const float c2 = ci * (a.eta_n + 3.0f * a.slack);
    const float c0 = a.slack * 0.5f * md.cw * fabsf(md.logdet);
    const float hl = -0.5f * md.cw * md.logdet;     // cw * (-0.5 logdet)
    const float hs = -0.5f * md.cw * md.iv;         // cw * (-0.5 iv)
    const float* Pp = a.P + (p >= 0 ? p : 0);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int ql = wq * 64 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
        const int q = q0 + ql;
        if (!vrow || q >= a.nq) continue;
        const float xn2 = sxn2[ql], xn1 = sxn1[ql];
        const float n2 = xn2 + rn2;
        const float S = fmaf(-2.0f, acc[i][j][e], n2);
        const float pi = p >= 0 ? Pp[(size_t)q * a.ldP] * md.invL : 0.f;
        const float key = pi + fmaf(hs, S, hl);
        const float err = fmaf(c1, xn1, fmaf(c2, n2, fmaf(a.slack, fabsf(pi), c0)));
        u[(size_t)q * a.ldu + r] = usable ? key + err : -CWQ_INF;
      }
    }
  }
}

hipError_t launch_approx_gemm(const void* Xb, const void* Mb, float* u, const GemmArgs& a, int n_rt, hipStream_t s) {
  dim3 grid((unsigned)(a.n_qt * n_rt)), block(256);
  hipLaunchKernelGGL(approx_gemm_kernel, grid, block, 0, s, (const __bf16*)Xb, (const __bf16*)Mb, u, a);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// list helpers (64-lane lists, order: key desc, row asc)
// ---------------------------------------------------------------------------
__device__ __forceinline__ void list64_insert(float& lk, int& lr, int lane, float ck, int cr, int K) {
  const bool prec = lk > ck || (lk == ck && lr < cr);
  const int pos = __popcll(__ballot(prec));
  if (pos < K) {
    const float sk = __int_as_float(__shfl_up(__float_as_int(lk), 1, 64));
    const int sr = __shfl_up(lr, 1, 64);
    if (lane == pos) {
      lk = ck;
      lr = cr;
    } else if (lane > pos) {
      lk = sk;
      lr = sr;
    }
  }
}

__device__ __forceinline__ void list64_offer(float& lk, int& lr, int lane, float key, int row, int K) {
  const float tk = rl_f2(lk, K - 1);
  const int tr = __builtin_amdgcn_readlane(lr, K - 1);
  const bool c = key != -CWQ_INF && (key > tk || (key == tk && row < tr));
  uint64_t mask = __ballot(c);
  while (mask) {
    const int j = __builtin_ctzll(mask);
    mask &= mask - 1;
    list64_insert(lk, lr, lane, rl_f2(key, j), __builtin_amdgcn_readlane(row, j), K);
  }
}

// ---------------------------------------------------------------------------
// 2. select: top-K' rows by u per query (workgroup per query, 4 wave lists merged)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void select_kernel(const float* __restrict__ u, int64_t ldu, int nrows, int Kp,
                                                     float* cu, int* crow) {
  __shared__ float sk[4][64];
  __shared__ int sr[4][64];
  const int q = blockIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const float* uq = u + (size_t)q * ldu;
  float lk = -CWQ_INF;
  int lr = 0x7fffffff;
  // each wave owns a contiguous range of whole 1024-row steps (16 values per lane per step;
  // the u buffer carries >= 1024 floats of tail slack, masked here)
  constexpr int STEP = 1024;
  const int per = (int)(((int64_t)nrows + 4 * STEP - 1) / (4 * STEP)) * STEP;
  const int r_lo = wave * per, r_hi = min(nrows, r_lo + per);
  for (int r0 = r_lo; r0 < r_hi; r0 += STEP) {
    float4 v4[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) v4[t] = *reinterpret_cast<const float4*>(uq + r0 + t * 256 + lane * 4);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const float vv[4] = {v4[t].x, v4[t].y, v4[t].z, v4[t].w};
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int r = r0 + t * 256 + lane * 4 + c;
        list64_offer(lk, lr, lane, r < r_hi ? vv[c] : -CWQ_INF, r, Kp);
      }
    }
  }
  sk[wave][lane] = lk;
  sr[wave][lane] = lr;
  __syncthreads();
  if (wave == 0) {
    for (int w = 1; w < 4; ++w) list64_offer(lk, lr, lane, sk[w][lane], sr[w][lane], Kp);
    cu[(size_t)q * 64 + lane] = lk;
    crow[(size_t)q * 64 + lane] = lr;
  }
}

hipError_t launch_select(const float* u, int64_t ldu, int nq, int nrows, int Kp, float* cu, int* crow, hipStream_t s) {
  hipLaunchKernelGGL(select_kernel, dim3((unsigned)nq), dim3(256), 0, s, u, ldu, nrows, Kp, cu, crow);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// 3. rerank: exact keys of the K' candidates (bit-identical to the scan kernel's
//    ISO arithmetic), exact top-K and the certificate.  One wave per query.
//    X is the scan's interleaved query layout [q/16][v][q%16][16].
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void rerank_kernel(const float* __restrict__ X, const float* __restrict__ Mf,
                                                     int DP, int nq, int Kp, int K, const float* __restrict__ cu,
                                                     const int* __restrict__ crow, const RowMeta* __restrict__ meta,
                                                     const int* __restrict__ par, const float* __restrict__ P,
                                                     int64_t ldP, int seg_base, float* pkey, float* paux, int* prow,
                                                     int64_t lstride, int* ok_flag) {
  const int lane = threadIdx.x & 63;
  const int q = blockIdx.x * kWavesPerWG + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  if (q >= nq) return;
  const int row = crow[(size_t)q * 64 + lane];
  const float uc = cu[(size_t)q * 64 + lane];
  const bool valid = lane < Kp && uc != -CWQ_INF && row != 0x7fffffff;
  const int rr = valid ? row : 0;
  const float* __restrict__ mr = Mf + (size_t)rr * DP;
  const int NV16 = DP / 16;
  const f32x16* __restrict__ xg = reinterpret_cast<const f32x16*>(X) + (size_t)(q / kXQ) * NV16 * kXQ + (q % kXQ);
  float acc = 0.f;
  for (int v = 0; v < NV16; ++v) {
    const f32x16 xa = xg[(size_t)v * kXQ];
    float m[16];
#pragma unroll
    for (int j = 0; j < 16; j += 4) {
      const float4 t4 = *reinterpret_cast<const float4*>(mr + v * 16 + j);
      m[j] = t4.x;
      m[j + 1] = t4.y;
      m[j + 2] = t4.z;
      m[j + 3] = t4.w;
    }
    float part;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const float t = xa[j] - m[j];
      part = (j == 0) ? t * t : fmaf(t, t, part);
    }
    acc += part;
  }
  const RowMeta md = meta[rr];
  const int p = par[rr];
  const float S = md.iv * acc;
  const float lp = -0.5f * (md.logdet + 0.f + S);
  const float pp = p >= 0 ? P[(size_t)q * ldP + p] : 0.f;
  float key = fmaf(pp, md.invL, md.cw * lp);
  if (!valid) key = -CWQ_INF;
  // exact top-K among the candidates
  float lk = -CWQ_INF, la = 0.f;
  int lr = 0x7fffffff;
  const int rid = seg_base + rr;
  {
    const bool c = key != -CWQ_INF;
    uint64_t mask = __ballot(c);
    while (mask) {
      const int j = __builtin_ctzll(mask);
      mask &= mask - 1;
      const float ck = rl_f2(key, j), ca = rl_f2(lp, j);
      const int cr = __builtin_amdgcn_readlane(rid, j);
      const bool prec = lk > ck || (lk == ck && lr < cr);
      const int pos = __popcll(__ballot(prec));
      if (pos < K) {
        const float sk = __int_as_float(__shfl_up(__float_as_int(lk), 1, 64));
        const float sa = __int_as_float(__shfl_up(__float_as_int(la), 1, 64));
        const int sr = __shfl_up(lr, 1, 64);
        if (lane == pos) {
          lk = ck;
          la = ca;
          lr = cr;
        } else if (lane > pos) {
          lk = sk;
          la = sa;
          lr = sr;
        }
      }
    }
  }
  // certificate: rows outside the candidate set have u <= u_(K') < tau_K
  const float tau = rl_f2(lk, K - 1);
  const float ulast = rl_f2(uc, Kp - 1);
  const bool complete = ulast == -CWQ_INF;   // fewer than K' usable rows: all are candidates
  const bool ok = complete || ulast < tau;
  if (lane < K) {
    const size_t o = (size_t)q * lstride + lane;
    pkey[o] = lk;
    paux[o] = la;
    prow[o] = lr;
  }
  if (lane == 0) ok_flag[q] = ok ? 1 : 0;
}

hipError_t launch_rerank(const float* X, const float* Mf, int DP, int nq, int Kp, int K, const float* cu,
                         const int* crow, const RowMeta* meta, const int* par, const float* P, int64_t ldP,
                         int seg_base, float* pkey, float* paux, int* prow, int64_t lstride, int* ok_flag,
                         hipStream_t s) {
  hipLaunchKernelGGL(rerank_kernel, dim3((unsigned)((nq + 3) / 4)), dim3(256), 0, s, X, Mf, DP, nq, Kp, K, cu, crow,
                     meta, par, P, ldP, seg_base, pkey, paux, prow, lstride, ok_flag);
  return hipGetLastError();
}

}  // namespace cwq
