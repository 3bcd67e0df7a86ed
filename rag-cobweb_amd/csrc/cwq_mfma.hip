// libcwq: bf16-MFMA candidate filter + exact fp32 rerank for isotropic rows
// ("Cobweb Fast", A6; CobwebWrapper.py:210-265).  Results are EXACT: the final
// keys are the scan kernel's fp32 arithmetic, op for op.
//
// Key of an isotropic row r for query x:
//   key = pi + hl + hs * S,   S = |x - mu|^2 = |x'|^2 + |mu'|^2 - 2 x'.mu'
//   (x' = x - c, mu' = mu - c, c = root mean; pi = P[q][parent] / L; hs = -cw*iv/2 < 0,
//   hl = -cw*logdet/2).  The bf16 MFMA computes x_hi.mu_hi (x_hi = bf16(x'),
//   x_lo = x' - x_hi exactly, same for mu); since
//     x'.mu' - x_hi.mu_hi = x_hi.mu_lo + x_lo.mu_hi + x_lo.mu_lo,
//   |error| <= a*b + c*d + c*b  (a=|x_hi|, c=|x_lo|, d=|mu_hi|, b=|mu_lo|, Cauchy-Schwarz),
//   plus fp32 accumulation gamma*a*d.  That gives rigorous bounds l <= key_fp32 <= u.
//
// Pipeline per query chunk:
//   1. sample pass: fgemm over a strided sample of S rows, dense lower bounds l;
//      T[q] = k-th largest l  (<= the true k-th key: those k rows have key >= l);
//   2. filter pass: fgemm over all rows; each (q, r) with u >= T[q] is a candidate
//      (every true top-k row has u >= key >= tau_k >= T).  The epilogue does NOT
//      materialise u: the accumulator starts at R_r - Qv_q so that acc >= 0 is a
//      conservative pretest of u >= T (2 VALU/element, no stores); survivors get the
//      rigorous u/l and go to a per-tile record list (LDS, then one coalesced flush);
//   3. bucket: records -> per-query candidate lists;
//   4. final (one wave per query): T2 = k-th largest l among the candidates
//      (<= tau_k), exact fp32 keys of the candidates with u >= T2, exact top-k.
//   Queries whose lists overflow (or have no usable threshold) are flagged and re-run
//   by the exact scan, so the result never depends on the filter's statistics.
//
// CDNA4 mapping of fgemm: persistent, one 512-thread workgroup per CU,
// 256 queries x 256 rows per tile, 8 waves as 2 (queries) x 4 (rows), each 128 x 64 =
// 8 x 4 v_mfma_f32_16x16x32_bf16 accumulators; K staged 32 deep by global_load_lds (16 B
// per lane) into a 4-buffer LDS ring (128 KiB: three stages in flight while one is
// consumed), XOR-swizzled 16-B chunks (conflict-free ds_read_b128); ping-pong wave
// groups (waves 0-3 / 4-7 one barrier interval apart: one wave per SIMD issues its MFMA
// cluster while its partner stages and reads the next stage).  Tiles are split over the
// 8 XCDs by query group so each XCD keeps its query panel in L2 while all XCDs stream
// the same row panels; within an XCD, tiles are claimed from a per-XCD counter.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <algorithm>

#include "cwq_internal.h"

namespace cwq {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void glb_void;

#define CWQ_INF __builtin_inff()

// |v| rounded up a little (norms are used as bounds)
__device__ __forceinline__ float up(double v) { return (float)(v * (1.0 + 0x1p-20)); }

// ---------------------------------------------------------------------------
// Row / query preparation
// ---------------------------------------------------------------------------
// Rows: fp32 row-major copy (exact rerank, DP wide), bf16 hi part of the centred row
// (DPB wide, zero padded), |mu'|^2, |mu_lo|, |mu_hi|.  One wave per row.  Group-centred
// rows (cwq_group.hip; grp[r] >= 0): centred at cent[g] instead of c, n2 = |M + d|^2
// (d = cent[g] - c in fp64) and nm = |M|.
__global__ void rows_prep_kernel(const float* __restrict__ mean, int D, const int64_t* __restrict__ nodes, int64_t n,
                                 const float* __restrict__ c, int DP, int DPB, int64_t ld, float* Mf, __bf16* Mb,
                                 float* n2, float* nlo, float* nhi, const float* __restrict__ cent,
                                 const int* __restrict__ grp, float* nm) {
  const int lane = threadIdx.x & 63;
  const int64_t r = blockIdx.x * (int64_t)kWavesPerWG + (threadIdx.x >> 6);
  if (r >= ld) return;
  const int g = (grp && r < n) ? grp[r] : -1;
  const float* cc = g >= 0 ? cent + (int64_t)g * D : c;
  double s = 0.0, slo = 0.0, shi = 0.0, sm = 0.0;
  const int W = DP > DPB ? DP : DPB;
  for (int d = lane; d < W; d += kWave) {
    const bool ok = r < n && d < D;
    const float v = ok ? mean[nodes[r] * (int64_t)D + d] : 0.f;
    const float vc = ok ? v - cc[d] : 0.f;
    const __bf16 h = (__bf16)vc;
    const float hf = (float)h;
    const float lo = vc - hf;   // exact
    if (d < DP) Mf[r * DP + d] = v;
    if (d < DPB) Mb[r * DPB + d] = h;
    const double vs = g >= 0 && ok ? (double)vc + ((double)cc[d] - (double)c[d]) : (double)vc;
    s += vs * vs;
    sm += (double)vc * (double)vc;
    slo += (double)lo * (double)lo;
    shi += (double)hf * (double)hf;
  }
  for (int off = 32; off > 0; off >>= 1) {
    s += __shfl_xor(s, off, 64);
    sm += __shfl_xor(sm, off, 64);
    slo += __shfl_xor(slo, off, 64);
    shi += __shfl_xor(shi, off, 64);
  }
  if (lane == 0) {
    n2[r] = (float)s;
    nlo[r] = up(sqrt(slo));
    nhi[r] = up(sqrt(shi));
    if (nm) nm[r] = up(sqrt(sm));
  }
}

hipError_t launch_rows_prep(const float* mean, int D, const int64_t* nodes, int64_t n, const float* c, int DP,
                            int DPB, int64_t ld, float* Mf, void* Mb, float* n2, float* nlo, float* nhi,
                            hipStream_t s, const float* cent, const int* grp, float* nm) {
  if (ld <= 0) return hipSuccess;
  hipLaunchKernelGGL(rows_prep_kernel, dim3((unsigned)((ld + 3) / 4)), dim3(256), 0, s, mean, D, nodes, n, c, DP, DPB,
                     ld, Mf, (__bf16*)Mb, n2, nlo, nhi, cent, grp, nm);
  return hipGetLastError();
}

// Copy the sample rows (bf16) into a compact operand: Sb[j] = Mb[srow[j]] (zero if srow < 0).
__global__ void gather_bf16_rows_kernel(const __bf16* __restrict__ Mb, int DPB, const int* __restrict__ srow,
                                        int64_t n, __bf16* Sb) {
  const int64_t j = blockIdx.x;
  const int r = srow[j];
  typedef int v4i __attribute__((ext_vector_type(4)));
  const v4i* src = reinterpret_cast<const v4i*>(Mb + (size_t)(r < 0 ? 0 : r) * DPB);
  v4i* dst = reinterpret_cast<v4i*>(Sb + (size_t)j * DPB);
  for (int i = threadIdx.x; i < DPB / 8; i += blockDim.x) dst[i] = r < 0 ? v4i{0, 0, 0, 0} : src[i];
}

hipError_t launch_gather_bf16_rows(const void* Mb, int DPB, const int* srow, int64_t n, void* Sb, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(gather_bf16_rows_kernel, dim3((unsigned)n), dim3(64), 0, s, (const __bf16*)Mb, DPB, srow, n,
                     (__bf16*)Sb);
  return hipGetLastError();
}

// int8 split of one centred row or query (one wave; cwq_internal.h launch_rows_i8):
// s = max|v| / 127, q = rint(v / s) clamped to +-127, hi = s q, lo = v - hi.  hi and lo are
// formed in fp64, where both are exact (a 24-bit by 8-bit product; a difference within 31
// bits), so the split is exact whatever s rounds to; the norms are rounded up by the callers.
template <class F>
__device__ __forceinline__ void i8_split_wave(F val, int DPB, int8_t* dst, double& sv, double& shi, double& slo,
                                              float& sc) {
  const int lane = threadIdx.x & 63;
  float m = 0.f;
  for (int d = lane; d < DPB; d += kWave) m = fmaxf(m, fabsf(val(d)));
  for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off, 64));
  const float s = m / 127.f;
  sv = shi = slo = 0.0;
  for (int d = lane; d < DPB; d += kWave) {
    const float v = val(d);
    const int qv = s > 0.f ? max(-127, min(127, (int)rintf(v / s))) : 0;
    dst[d] = (int8_t)qv;
    const double hi = (double)s * (double)qv;
    const double lo = (double)v - hi;
    sv += (double)v * (double)v;
    shi += hi * hi;
    slo += lo * lo;
  }
  for (int off = 32; off > 0; off >>= 1) {
    sv += __shfl_xor(sv, off, 64);
    shi += __shfl_xor(shi, off, 64);
    slo += __shfl_xor(slo, off, 64);
  }
  sc = s;
}

// Rows (launch_rows_i8): the centred row as rows_prep forms it (Mf - c in fp32), one wave
// per row; unusable rows (par < -1) get zeros and scale 0.
__global__ void rows_i8_kernel(const float* __restrict__ Mf, int DP, int D, const float* __restrict__ c, int DPB,
                               int64_t ld, const RowF* __restrict__ rf, int8_t* Mq, RowF* rf8) {
  const int lane = threadIdx.x & 63;
  const int64_t r = blockIdx.x * (int64_t)kWavesPerWG + (threadIdx.x >> 6);
  if (r >= ld) return;
  RowF f = rf[r];
  const bool ok = f.par >= -1;
  double sv, shi, slo;
  float sc;
  i8_split_wave([&](int d) { return (ok && d < D) ? Mf[r * DP + d] - c[d] : 0.f; }, DPB, Mq + r * DPB, sv, shi, slo,
                sc);
  if (lane == 0) {
    if (ok) {
      const double bh = sqrt(shi), bl = sqrt(slo);
      f.beta = up(bl);
      f.delta = up(bh + bl);
      f.R0 = sc;
    } else {
      f.R0 = 0.f;
    }
    rf8[r] = f;
  }
}

hipError_t launch_rows_i8(const float* Mf, int DP, int D, const float* c, int DPB, int64_t ld, const RowF* rf,
                          void* Mq, RowF* rf8, hipStream_t s) {
  if (ld <= 0) return hipSuccess;
  if (DPB % 64) return hipErrorInvalidValue;
  hipLaunchKernelGGL(rows_i8_kernel, dim3((unsigned)((ld + 3) / 4)), dim3(256), 0, s, Mf, DP, D, c, DPB, ld, rf,
                     (int8_t*)Mq, rf8);
  return hipGetLastError();
}

// Queries for the int8 pass, as query_prep_kernel forms the centred query.
__global__ void query_prep_i8_kernel(const float* __restrict__ q, int64_t nq, int D, const float* __restrict__ c,
                                     int DPB, int64_t nq16, int8_t* Xq, float4* qinfo8) {
  const int lane = threadIdx.x & 63;
  const int64_t r = blockIdx.x * (int64_t)kWavesPerWG + (threadIdx.x >> 6);
  if (r >= nq16) return;
  double sv, shi, slo;
  float sc;
  i8_split_wave([&](int d) { return (r < nq && d < D) ? q[r * D + d] - c[d] : 0.f; }, DPB, Xq + r * DPB, sv, shi, slo,
                sc);
  if (lane == 0) qinfo8[r] = make_float4((float)sv, up(sqrt(shi)), up(sqrt(slo)), sc);
}

hipError_t launch_query_prep_i8(const float* q, int64_t nq, int D, const float* c, int DPB, int64_t nq16, void* Xq,
                                float4* qinfo8, hipStream_t s) {
  if (DPB % 64) return hipErrorInvalidValue;
  hipLaunchKernelGGL(query_prep_i8_kernel, dim3((unsigned)((nq16 + 3) / 4)), dim3(256), 0, s, q, nq, D, c, DPB, nq16,
                     (int8_t*)Xq, qinfo8);
  return hipGetLastError();
}

// Queries: bf16 hi part of the centred query, and {|x'|^2, |x_hi|, |x_lo|}.
__global__ void query_prep_kernel(const float* __restrict__ q, int64_t nq, int D, const float* __restrict__ c,
                                  int DPB, int64_t nq_pad, __bf16* Xb, float4* qinfo, int* zero, int nzero) {
  const int lane = threadIdx.x & 63;
  const int64_t r = blockIdx.x * (int64_t)kWavesPerWG + (threadIdx.x >> 6);
  if (blockIdx.x == 0)   // the call's counters (a memset launch less per call)
    for (int i = threadIdx.x; i < nzero; i += blockDim.x) zero[i] = 0;
  if (r >= nq_pad) return;
  double s = 0.0, slo = 0.0, shi = 0.0;
  for (int d = lane; d < DPB; d += kWave) {
    const float v = (r < nq && d < D) ? q[r * D + d] - c[d] : 0.f;
    const __bf16 h = (__bf16)v;
    const float hf = (float)h;
    const float lo = v - hf;
    Xb[r * DPB + d] = h;
    s += (double)v * (double)v;
    slo += (double)lo * (double)lo;
    shi += (double)hf * (double)hf;
  }
  for (int off = 32; off > 0; off >>= 1) {
    s += __shfl_xor(s, off, 64);
    slo += __shfl_xor(slo, off, 64);
    shi += __shfl_xor(shi, off, 64);
  }
  if (lane == 0) qinfo[r] = make_float4((float)s, up(sqrt(shi)), up(sqrt(slo)), 0.f);
}

hipError_t launch_query_prep(const float* q, int64_t nq, int D, const float* c, int DPB, int64_t nq_pad, void* Xb,
                             float4* qinfo, hipStream_t s, int* zero, int nzero) {
  if (nzero < 0 || (nzero > 0 && !zero)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(query_prep_kernel, dim3((unsigned)((nq_pad + 3) / 4)), dim3(256), 0, s, q, nq, D, c, DPB, nq_pad,
                     (__bf16*)Xb, qinfo, zero, nzero);
  return hipGetLastError();
}

// Small-batch query prep (the per-call stream path, nq <= kStreamMaxQ, flat trees and
// trees with few internal nodes): one launch does the work of pad_queries_kernel,
// query_prep_kernel, the exact internal pass (int_small_kernel + one
// prefix_level_kernel per level) and the candidate-counter clear.  One 256-thread
// workgroup per padded query row.  The arithmetic is the same as those kernels':
// query_prep's sums run in wave 0 with its loop and shuffle order; an internal node's
// raw sum is its 16-dim fma partials (t = fmaf(x, A, -B), dimension order), computed
// here one slice per thread, then added in slice order by one thread (acc += part);
// the prefixes are prefix_level_kernel's fmaf chain, level by level.
__global__ __launch_bounds__(256) void sb_prep_kernel(const SbPrepArgs a) {
  extern __shared__ float s_sb[];   // [DQ] query row, [DQ] centre, [NI][NV16] partials, [NI] prefixes
  const int tid = threadIdx.x, lane = tid & 63;
  const int64_t r = blockIdx.x;
  const bool valid = r < a.nq;
  const int NV16 = a.DP / 16;
  const int DQ = a.DP > a.DPB ? a.DP : a.DPB;
  float* xq = s_sb;   // the query row, zero padded: every phase below reads it from LDS
  float* cq = s_sb + DQ;   // the centre, staged with the row (a global load inside the bf16
                           // prep loop below was one dependent round trip per iteration)
  for (int d = tid; d < DQ; d += 256) {
    xq[d] = (valid && d < a.D) ? a.q[r * a.D + d] : 0.f;
    cq[d] = d < a.D ? a.c[d] : 0.f;
  }
  __syncthreads();
  // pad_queries_kernel: the scan's interleaved layout [r/kXQ][v][r%kXQ][16]
  for (int d = tid; d < a.DP; d += 256) {
    const int64_t o = (((r / kXQ) * NV16 + d / 16) * kXQ + (r % kXQ)) * 16 + (d % 16);
    a.X[o] = xq[d];
  }
  if (r < a.nq16 && tid < 64) {   // query_prep_kernel (wave 0)
    double sv = 0.0, slo = 0.0, shi = 0.0;
    for (int d = lane; d < a.DPB; d += kWave) {
      const float v = (valid && d < a.D) ? xq[d] - cq[d] : 0.f;
      const __bf16 h = (__bf16)v;
      const float hf = (float)h;
      const float lo = v - hf;
      reinterpret_cast<__bf16*>(a.Xb)[r * a.DPB + d] = h;
      sv += (double)v * (double)v;
      slo += (double)lo * (double)lo;
      shi += (double)hf * (double)hf;
    }
    for (int off = 32; off > 0; off >>= 1) {
      sv += __shfl_xor(sv, off, 64);
      slo += __shfl_xor(slo, off, 64);
      shi += __shfl_xor(shi, off, 64);
    }
    if (lane == 0) a.qinfo[r] = make_float4((float)sv, up(sqrt(shi)), up(sqrt(slo)), 0.f);
  }
  if (r < a.nq16 && a.Xq && tid >= 64 && tid < 128) {   // query_prep_i8_kernel (wave 1)
    double sv, shi, slo;
    float sc;
    i8_split_wave([&](int d) { return (valid && d < a.D) ? xq[d] - cq[d] : 0.f; }, a.DPB,
                  reinterpret_cast<int8_t*>(a.Xq) + r * a.DPB, sv, shi, slo, sc);
    if (lane == 0) a.qinfo8[r] = make_float4((float)sv, up(sqrt(shi)), up(sqrt(slo)), sc);
  }
  if (!valid) return;
  if (tid < 5) a.qcnt[(size_t)tid * a.nq + r] = 0;
  if (r == 0 && tid == 5) a.qcnt[(size_t)5 * a.nq] = 0;   // the probe's fused-select counter
  if (a.NI == 0) return;
  // internal nodes: partials of (node n, slice v), straight from the caller's query
  float* part = s_sb + 2 * DQ;
  for (int t = tid; t < a.NI * NV16; t += 256) {
    const int n = t / NV16, v = t - n * NV16;
    float pp;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int d = v * 16 + j;
      const float x = xq[d];
      const float tt = fmaf(x, a.A[(size_t)d * a.ld + n], -a.B[(size_t)d * a.ld + n]);
      pp = (j == 0) ? tt * tt : fmaf(tt, tt, pp);
    }
    part[t] = pp;
  }
  __syncthreads();
  float* Pl = part + a.NI * NV16;
  for (int lv = 0; lv < a.nlev; ++lv) {
    for (int i = a.lv0[lv] + tid; i < a.lv0[lv + 1]; i += 256) {
      const float acc = sum_in_order(part + i * NV16, NV16);
      const float lp = -0.5f * (a.logdet_int[i] + acc);
      const int p = a.par_int[i];
      const float P = p >= 0 ? fmaf(a.w_int[i], lp, Pl[p]) : a.w_int[i] * lp;
      Pl[i] = P;
      a.P[(size_t)r * a.ldP + i] = P;
    }
    __syncthreads();
  }
}

hipError_t launch_sb_prep(const SbPrepArgs& a, hipStream_t s) {
  const size_t lds = ((size_t)2 * std::max(a.DP, a.DPB) + (size_t)a.NI * (a.DP / 16) + a.NI) * 4;
  if (a.nq <= 0 || a.nq_pad < a.nq16 || a.nq16 < a.nq || a.DP % 16 || a.NI > kSbMaxNI || a.nlev > kSbMaxNI ||
      lds > 65536)
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(sb_prep_kernel, dim3((unsigned)a.nq_pad), dim3(256), lds, s, a);
  return hipGetLastError();
}

// One prefix_level_kernel step on intervals: parent prefix in [pl, ph], lp' in [lo, hi]
// -> [lo, hi] <- bounds of fmaf(w, lp', P_parent) as the exact pass computes it.  fp32:
// each fmaf here and the exact one round by <= 2^-24 of (|P_parent| + |w lp'|), the
// margin subtraction by 2^-24 of the result; m = 2^-21 of the magnitudes covers all three.
__device__ __forceinline__ void prefix_step(float pl, float ph, float w, float& lo, float& hi) {
  const float a = w >= 0.f ? lo : hi, b = w >= 0.f ? hi : lo;   // w * [a, b] is ordered
  const float m = 0x1p-21f * (fmaxf(fabsf(pl), fabsf(ph)) + fabsf(w) * fmaxf(fabsf(lo), fabsf(hi)));
  lo = fmaf(w, a, pl) - m;
  hi = fmaf(w, b, ph) + m;
}

// Internal-node bound operands (launch_int_prep, cwq_internal.h).  One wave per node.
__global__ void int_prep_kernel(const float* __restrict__ mean, const VarSrc var, int D,
                                const int64_t* __restrict__ nodes, int64_t n, const float* __restrict__ c,
                                const float* __restrict__ logdet, const int* __restrict__ par_int,
                                const float* __restrict__ w_int, int DP, int DPB2, int64_t ld, __bf16* Mb2, RowF* rf,
                                float* Ar, float* Br, float gamma) {
  const int lane = threadIdx.x & 63;
  const int64_t r = blockIdx.x * (int64_t)kWavesPerWG + (threadIdx.x >> 6);
  if (r >= ld) return;
  double shi = 0.0, slo = 0.0, cn = 0.0, mn = 0.0;
  float wmax = 0.f;
  for (int k = lane; k < DPB2; k += kWave) {   // b' = [-w/2 (DP wide), mu' w (DP wide), 0 pad]
    const int d = k < DP ? k : k - DP;
    const bool ok = r < n && k < 2 * DP && d < D;
    float v = 0.f;
    if (ok) {
      const int64_t o = nodes[r] * (int64_t)D + d;
      const float A = 1.0f / sqrtf(var.at(nodes[r], d, D));   // as gather_T_kernel (the exact scan's A)
      const float w = A * A;
      const float mu = mean[o];
      const float mc = mu - c[d];
      if (k < DP) {
        v = -0.5f * w;
        const double am = fabs((double)mu) + fabs((double)c[d]);
        cn += (double)mc * (double)mc * (double)w;
        mn += (double)w * am * am;
        wmax = fmaxf(wmax, w);
        Ar[r * DP + d] = A;
        Br[r * DP + d] = mu * A;
      } else {
        v = mc * w;
      }
    } else if (r < n && k < DP) {
      Ar[r * DP + k] = 0.f;   // padding dims, as int_A / int_B
      Br[r * DP + k] = 0.f;
    }
    const __bf16 h = (__bf16)v;
    const float hf = (float)h;
    const float lo = v - hf;
    if (Mb2) Mb2[r * DPB2 + k] = h;
    shi += (double)hf * (double)hf;
    slo += (double)lo * (double)lo;
  }
  for (int off = 32; off > 0; off >>= 1) {
    shi += __shfl_xor(shi, off, 64);
    slo += __shfl_xor(slo, off, 64);
    cn += __shfl_xor(cn, off, 64);
    mn += __shfl_xor(mn, off, 64);
    wmax = fmaxf(wmax, __shfl_xor(wmax, off, 64));
  }
  if (lane == 0) {
    RowF f;
    if (r < n) {
      const double bh = sqrt(shi) * (1.0 + 0x1p-20), bl = sqrt(slo) * (1.0 + 0x1p-20);
      f.R0 = up(mn);
      f.beta = up(bl + (double)gamma * bh);
      f.delta = up(bh + bl);
      f.rn2 = (float)cn;
      f.hs = wmax;
      f.hl = logdet[r];
      f.invL = w_int[r];
      f.par = par_int[r];
    } else {
      f = RowF{0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, -2};
    }
    if (rf) rf[r] = f;
  }
}

hipError_t launch_int_prep(const float* mean, const VarSrc& var, int D, const int64_t* nodes, int64_t n,
                           const float* c, const float* logdet, const int* par_int, const float* w_int, int DP, int DPB2,
                           int64_t ld, void* Mb2, RowF* rf, float* Ar, float* Br, float gamma, hipStream_t s) {
  if (ld <= 0) return hipSuccess;
  hipLaunchKernelGGL(int_prep_kernel, dim3((unsigned)((ld + 3) / 4)), dim3(256), 0, s, mean, var, D, nodes, n, c,
                     logdet, par_int, w_int, DP, DPB2, ld, (__bf16*)Mb2, rf, Ar, Br, gamma);
  return hipGetLastError();
}

// Path-sum operands (launch_int_path_prep, cwq_internal.h).  The Fast filter needs the path
// prefix P(n) = P(root) + sum_a w_a lp'(a) of leaf parents n only (a: the path's non-root
// nodes), and with int_prep's split lp'(a) = -0.5 (logdet_a + c_a) + a.b'_a that sum is one
// linear form in the query vector a = [x'^2, x']:
//   P(n) - P(root) = K0 + a.Bsum,  K0 = -0.5 sum w_a (logdet_a + c_a),  Bsum = sum w_a b'_a,
// so one GEMM row per leaf parent replaces a row per internal node and the level-by-level
// prefix passes.  Bsum is accumulated in fp64 from int_prep's fp32 b' values and rounded
// once.  The bound must hold for the exact pass's fp32 chain P_i = fmaf(w_i, lp'_fp32(i),
// P_{i-1}); its distance to the real sum is bounded per node a, as int_bounds does, by
// 2^-12 (wmax_a qx + M_a + |logdet_a| + c_a) (the fp32 S evaluation, lp' roundings; |S_a|
// <= 2 wmax_a |x'|^2 + 2 c_a), plus one rounding of <= 2^-24 |P_i| per chain step with
// |P_i| <= |P(root)| + sum_a (|logdet_a| + c_a + M_a + 1.01 wmax_a qx) |w_a|.  Hence, with
// Z3 = sum |w_a| wmax_a, Z0 = sum |w_a| (M_a + |logdet_a| + c_a), depth = path length:
//   Zq = cz Z3, Zc = cz Z0 + 2^-23 |K0|, cz = 1.02 (2^-12 + depth 2^-24), cr = depth 2^-24 + 2^-22
// (the 1.02 also covers Bsum's fp32 rounding, <= 2^-24 sum |w_a| (wmax_a qx + c_a)).
// One wave per row.
__global__ void int_path_prep_kernel(const float* __restrict__ mean, const VarSrc var, int D,
                                     const int64_t* __restrict__ nodes, const int* __restrict__ rows, int64_t n,
                                     const float* __restrict__ c, const float* __restrict__ logdet,
                                     const int* __restrict__ par_int, const float* __restrict__ w_int, int DP, int DPB2,
                                     int64_t ld, __bf16* Mb2, RowF* rf, float gamma) {
  const int lane = threadIdx.x & 63;
  const int64_t r = blockIdx.x * (int64_t)kWavesPerWG + (threadIdx.x >> 6);
  if (r >= ld) return;
  const int i = r < n ? rows[r] : -1;
  // per-node scalar terms, node by node up the path (the root excluded)
  double K0 = 0.0, Z0 = 0.0, Z3 = 0.0;
  int depth = 0;
  for (int a = i; a >= 0 && par_int[a] >= 0; a = par_int[a]) {
    ++depth;
    const int64_t nd = nodes[a];
    double cn = 0.0, mn = 0.0;
    float wmax = 0.f;
    for (int d = lane; d < D; d += kWave) {
      const float A = 1.0f / sqrtf(var.at(nd, d, D));   // as int_prep
      const float w = A * A;
      const float mu = mean[nd * (int64_t)D + d];
      const float mc = mu - c[d];
      const double am = fabs((double)mu) + fabs((double)c[d]);
      cn += (double)mc * (double)mc * (double)w;
      mn += (double)w * am * am;
      wmax = fmaxf(wmax, w);
    }
    for (int off = 32; off > 0; off >>= 1) {
      cn += __shfl_xor(cn, off, 64);
      mn += __shfl_xor(mn, off, 64);
      wmax = fmaxf(wmax, __shfl_xor(wmax, off, 64));
    }
    const double wa = (double)w_int[a], ld_a = (double)logdet[a];
    K0 += -0.5 * wa * (ld_a + cn);
    Z0 += fabs(wa) * (mn + fabs(ld_a) + cn);
    Z3 += fabs(wa) * (double)wmax;
  }
  // Bsum, bf16 hi parts and the split norms
  double shi = 0.0, slo = 0.0;
  for (int k = lane; k < DPB2; k += kWave) {
    const int d = k < DP ? k : k - DP;
    double acc = 0.0;
    if (k < 2 * DP && d < D)
      for (int a = i; a >= 0 && par_int[a] >= 0; a = par_int[a]) {
        const int64_t nd = nodes[a];
        const float A = 1.0f / sqrtf(var.at(nd, d, D));
        const float w = A * A;
        const float v = k < DP ? -0.5f * w : (mean[nd * (int64_t)D + d] - c[d]) * w;   // int_prep's b'
        acc += (double)w_int[a] * (double)v;
      }
    const float v = (float)acc;
    const __bf16 h = (__bf16)v;
    const float hf = (float)h;
    const float lo = v - hf;
    Mb2[r * DPB2 + k] = h;
    shi += (double)hf * (double)hf;
    slo += (double)lo * (double)lo;
  }
  for (int off = 32; off > 0; off >>= 1) {
    shi += __shfl_xor(shi, off, 64);
    slo += __shfl_xor(slo, off, 64);
  }
  if (lane == 0) {
    RowF f = RowF{0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, -2};
    if (i >= 0) {
      f.par = par_int[i];   // -1: the root (exact row)
      if (f.par >= 0) {
        const double bh = sqrt(shi) * (1.0 + 0x1p-20), bl = sqrt(slo) * (1.0 + 0x1p-20);
        const double cz = 1.02 * (0x1p-12 + depth * 0x1p-24);
        f.beta = up(bl + (double)gamma * bh);
        f.delta = up(bh + bl);
        f.rn2 = (float)K0;
        f.hs = up(cz * Z3);
        f.R0 = up(cz * Z0 + 0x1p-23 * fabs(K0));
        f.hl = up(depth * 0x1p-24 + 0x1p-22);
      }
    }
    rf[r] = f;
  }
}

hipError_t launch_int_path_prep(const float* mean, const VarSrc& var, int D, const int64_t* nodes, const int* rows,
                                int64_t n, const float* c, const float* logdet, const int* par_int,
                                const float* w_int, int DP, int DPB2, int64_t ld, void* Mb2, RowF* rf, float gamma,
                                hipStream_t s) {
  if (ld <= 0) return hipSuccess;
  hipLaunchKernelGGL(int_path_prep_kernel, dim3((unsigned)((ld + 3) / 4)), dim3(256), 0, s, mean, var, D, nodes, rows,
                     n, c, logdet, par_int, w_int, DP, DPB2, ld, (__bf16*)Mb2, rf, gamma);
  return hipGetLastError();
}

// Queries for the internal bounds: a = [x'^2 (DP wide), x' (DP wide), 0 pad].
__global__ void query_prep2_kernel(const float* __restrict__ q, int64_t nq, int D, const float* __restrict__ c,
                                   int DP, int DPB2, int64_t nq_pad, __bf16* Xb2, float4* qinfo) {
  const int lane = threadIdx.x & 63;
  const int64_t r = blockIdx.x * (int64_t)kWavesPerWG + (threadIdx.x >> 6);
  if (r >= nq_pad) return;
  double shi = 0.0, slo = 0.0, sx = 0.0;
  for (int k = lane; k < DPB2; k += kWave) {
    const int d = k < DP ? k : k - DP;
    float v = 0.f;
    if (r < nq && k < 2 * DP && d < D) {
      const float x = q[r * D + d];
      const float xc = x - c[d];
      v = k < DP ? xc * xc : xc;
      if (k < DP) sx += (double)x * (double)x + (double)xc * (double)xc;
    }
    const __bf16 h = (__bf16)v;
    const float hf = (float)h;
    const float lo = v - hf;
    Xb2[r * DPB2 + k] = h;
    shi += (double)hf * (double)hf;
    slo += (double)lo * (double)lo;
  }
  for (int off = 32; off > 0; off >>= 1) {
    shi += __shfl_xor(shi, off, 64);
    slo += __shfl_xor(slo, off, 64);
    sx += __shfl_xor(sx, off, 64);
  }
  if (lane == 0) qinfo[r] = make_float4(up(sx), up(sqrt(shi)), up(sqrt(slo)), 0.f);
}

hipError_t launch_query_prep2(const float* q, int64_t nq, int D, const float* c, int DP, int DPB2, int64_t nq_pad,
                              void* Xb2, float4* qinfo, hipStream_t s) {
  hipLaunchKernelGGL(query_prep2_kernel, dim3((unsigned)((nq_pad + 3) / 4)), dim3(256), 0, s, q, nq, D, c, DP, DPB2,
                     nq_pad, (__bf16*)Xb2, qinfo);
  return hipGetLastError();
}

// Prefix bounds of one tree level (prefix_level_kernel's recurrence P = fmaf(w, lp,
// P[parent]) on intervals): lp' bounds in (Plo, Phi) become prefix bounds, in fp64 and
// widened by 2^-22 of the magnitudes for the exact fp32 fmaf's rounding.  Root level:
// exact, from Sroot (same arithmetic as prefix_level_kernel).
__global__ void prefix_bounds_kernel(float* Plo, float* Phi, int64_t ldP, int nq, int i0, int i1,
                                     const int* __restrict__ par_int, const float* __restrict__ w_int,
                                     const float* __restrict__ logdet_int, const float* __restrict__ Sroot) {
  const int n = i1 - i0;
  const int64_t total = (int64_t)n * nq;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int q = (int)(t / n);
    const int i = i0 + (int)(t % n);
    const size_t o = (size_t)q * ldP + i;
    const int p = par_int[i];
    const float w = w_int[i];
    if (p < 0) {   // the root: exact
      const float lp = -0.5f * (logdet_int[i] + Sroot[q]);
      const float P = w * lp;
      Plo[o] = P;
      Phi[o] = P;
      continue;
    }
    const size_t op = (size_t)q * ldP + p;
    float lo = Plo[o], hi = Phi[o];
    prefix_step(Plo[op], Phi[op], w, lo, hi);
    Plo[o] = lo;
    Phi[o] = hi;
  }
}

hipError_t launch_prefix_bounds(float* Plo, float* Phi, int64_t ldP, int nq, int i0, int i1, const int* par_int,
                                const float* w_int, const float* logdet_int, const float* Sroot, hipStream_t s) {
  const int64_t total = (int64_t)(i1 - i0) * nq;
  if (total <= 0) return hipSuccess;
  dim3 grid((unsigned)std::min<int64_t>((total + 255) / 256, 8192));
  hipLaunchKernelGGL(prefix_bounds_kernel, grid, dim3(256), 0, s, Plo, Phi, ldP, nq, i0, i1, par_int, w_int,
                     logdet_int, Sroot);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// fgemm: bf16-MFMA bounds over (query tile x row tile), persistent
// ---------------------------------------------------------------------------
constexpr int FT = kFgTile;       // 256 queries and rows per tile
constexpr int FK = 32;            // K per LDS stage
constexpr int FNBUF = 4;          // LDS stage ring: 3 stages in flight while one is consumed
constexpr int FSTAGE = 2 * FT * FK * 2;   // bytes of one stage (A + B images) = 32 KiB
constexpr int OFF_QV = FNBUF * FSTAGE;    // float  [FT]   pretest query terms
constexpr int OFF_QI = OFF_QV + FT * 4;   // float4 [FT]   {|x'|^2, a, c, T}
constexpr int OFF_PI = OFF_QI + FT * 16;  // float  [FT]   pi of the tile's parent (upper bound)
constexpr int OFF_PL = OFF_PI + FT * 4;   // float  [FT]   its lower bound (= pi when exact)
constexpr int OFF_REC = OFF_PL + FT * 4;  // int4   [kFgCap] record staging
constexpr int OFF_CNT = OFF_REC + kFgCap * 16;   // int[16]: count, chunk, fill, flush scratch, claim
constexpr int FLDS = OFF_CNT + 64;


// Internal node i, query x (mode 2): lp'(i) = -0.5 (logdet_i + S), S = sum_d w_d (x_d - mu_d)^2
// (w = A^2, A = 1/sqrtf(var): the exact scan's sum_d (x_d A_d - B_d)^2).  With x' = x - c,
// mu' = mu - c, a = [x'^2, x'], b' = [-w/2, mu' w]:  S = c_n - 2 a.b',  c_n = sum w mu'^2.
// The MFMA gives a_hi.b'_hi; as for the leaves (header), |a.b' - a_hi.b'_hi| <= |a_hi||b_lo|
// + |a_lo||b_hi| + |a_lo||b_lo| + gamma |a_hi||b_hi| (+ 2^-23 |dot| for the last rounding).
// The fp32 evaluation of the exact S (scan order, stored A/B = fl(1/sqrt v), fl(mu A), the
// query/mean centring and the fp32 squares) differs from that real value by far less than
// 2^-12 (wmax (sum x^2 + sum x'^2) + M_n), M_n = sum w (|mu| + |c|)^2, which is added as
// slack; lp' then gets 2^-20 (|logdet| + S) for its own two roundings.  Returns bounds
// lo <= lp'_fp32 <= hi.  RowF fields: beta = |b_lo| + gamma|b_hi|, delta = |b_hi| + |b_lo|,
// rn2 = c_n, hs = wmax, hl = logdet, R0 = M_n.  qinfo: {sum x^2 + sum x'^2, |a_hi|, |a_lo|}.
__device__ __forceinline__ void int_bounds(float dot, float4 qi, const RowF& f, float gamma, float& lo, float& hi) {
  (void)gamma;   // inside f.beta
  const float S0 = fmaf(-2.f, dot, f.rn2);
  const float E = 2.f * (fmaf(qi.y, f.beta, qi.z * f.delta) + 0x1p-23f * fabsf(dot)) + 0x1p-20f * fabsf(f.rn2) +
                  0x1p-12f * fmaf(f.hs, qi.x, f.R0);
  const float Eu = E * (1.f + 0x1p-20f);   // the fp32 evaluation of E itself
  const float Shi = (S0 + Eu) * (1.f + 0x1p-22f);
  const float Slo = fmaxf(0.f, (S0 - Eu) * (1.f - 0x1p-22f));
  const float m = 0x1p-20f * (fabsf(f.hl) + Shi);
  hi = -0.5f * (f.hl + Slo) + m;
  lo = -0.5f * (f.hl + Shi) - m;
}

// XCD-local tile i -> (query tile, row tile).  order 0/2: query tiles fastest (the
// XCD's query panels stay in L2 while row panels stream past, each read by every
// query tile of the group at about the same time); order 1: row tiles fastest.
__device__ __forceinline__ void fg_decode(const FgArgs& a, int xcd, int i, int& qt, int& rt) {
  const int qg = xcd % a.qgroups, rg = xcd / a.qgroups;
  const int nqt_g = (a.n_qt + a.qgroups - 1) / a.qgroups;
  const int nrt_g = (a.n_rt + a.rgroups - 1) / a.rgroups;
  const int q_lo = qg * nqt_g, r_lo = rg * nrt_g;
  const int nq_l = max(1, min(nqt_g, a.n_qt - q_lo));
  const int nr_l = max(1, min(nrt_g, a.n_rt - r_lo));
  if (a.order == 1) {
    qt = q_lo + i / nr_l;
    rt = a.rt_off + r_lo + i % nr_l;
  } else {
    qt = q_lo + i % nq_l;
    rt = a.rt_off + r_lo + i / nq_l;
  }
}

__device__ __forceinline__ int fg_count(const FgArgs& a, int xcd) {
  const int qg = xcd % a.qgroups, rg = xcd / a.qgroups;
  const int nqt_g = (a.n_qt + a.qgroups - 1) / a.qgroups;
  const int nrt_g = (a.n_rt + a.rgroups - 1) / a.rgroups;
  const int nq_l = max(0, min(nqt_g, a.n_qt - qg * nqt_g));
  const int nr_l = max(0, min(nrt_g, a.n_rt - rg * nrt_g));
  return nq_l * nr_l;
}

#ifndef FG_STAMP
#define FG_STAMP 0   // diagnostic builds: s_memtime stamps of the ping-pong loop (FgArgs::stamp)
#endif
#ifndef FG_LEAN
#define FG_LEAN 1   // filter tiles without records skip the flush's second barrier and the per-tile third one
#endif
#define FG_CSLOT (FG_LEAN && MODE == 0 && (tile_no & 1) ? 9 : 0)
// 16-B chunk position of logical chunk 0 in row r of a stage image (a permutation of the
// row's 4 chunks, XORed with the chunk index), chosen so that the ds_read_b128 fragment
// reads of a wave are bank-conflict free: for 16x16x32 lane l reads row l&15, chunk
// l>>4 -> f = (4 - ((r>>2)&3))&3.
__device__ __forceinline__ int fg_swz(int r) { return (4 - ((r >> 2) & 3)) & 3; }

// one K stage (32 deep) of both operands into an LDS stage buffer: 4 glds per wave.
// Image: [256 rows][64 B] per operand; 16-B chunk c of row r sits at position
// c ^ ((r >> 2) & 3) (conflict-free ds_read_b128 fragment reads); the LDS side of a
// glds is lane-linear, so the permutation is applied to the global source address.
// ipart 0/1: the half of the stage (one A and one B glds per wave); -1: both.
// Addressing: wave-uniform 64-bit tile bases (SGPR, global_load_lds saddr form) plus a
// per-lane 32-bit byte offset fixed for the kernel (row within the 16-row piece, swizzled
// chunk), so issuing a piece costs no 64-bit VALU math; the LDS destination (M0) is
// computed on the scalar unit from the wave-uniform wave index.
__device__ __forceinline__ void fg_stage(const __bf16* __restrict__ Xb, const __bf16* __restrict__ Mb, int DPB, int q0,
                                         int r0, int k0, char* sb, int wave, const uint32_t* loff, int ipart = -1) {
  const char* gA = reinterpret_cast<const char*>(Xb) + ((size_t)q0 * DPB + k0) * 2;
  const char* gB = reinterpret_cast<const char*>(Mb) + ((size_t)r0 * DPB + k0) * 2;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    if (ipart >= 0 && i != ipart) continue;
    __builtin_amdgcn_global_load_lds((glb_void*)(gA + loff[i]), (lds_void*)(sb + (wave * 32 + i * 16) * 64), 16, 0, 0);
    __builtin_amdgcn_global_load_lds((glb_void*)(gB + loff[i]), (lds_void*)(sb + FT * 64 + (wave * 32 + i * 16) * 64), 16,
                                     0, 0);
  }
}

// A tile's TileF (wave-uniform) through the constant address space: scalar loads,
// counted by lgkmcnt, so they never wait behind the LDS-DMA on the vector counter.
__device__ __forceinline__ TileF fg_tile_const(const TileF* p, int i) {
  static_assert(sizeof(TileF) == 32, "TileF is 8 dwords");
  typedef const __attribute__((address_space(4))) int* cip;
  const cip src = (cip)(uintptr_t)(p + i);
  TileF t;
  int* d = reinterpret_cast<int*>(&t);
#pragma unroll
  for (int k = 0; k < 8; ++k) d[k] = src[k];
  return t;
}

// MODE 0: filter pass (records), MODE 1: threshold-sample pass (dense lower bounds);
// separate instantiations so profiles tell them apart and each drops the other's code.
// ALLUNI: every row tile of the launch is uniform (flat trees): the per-element generic
// bound path is compiled out.
template <int MODE, bool ALLUNI>
__global__ __launch_bounds__(512) void fgemm_kernel(const __bf16* __restrict__ Xb, const __bf16* __restrict__ Mb,
                                                    const FgArgs a) {
  __shared__ __attribute__((aligned(16))) char smem[FLDS];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wq = wave & 1, wr = wave >> 1;
  const int xcd = blockIdx.x & 7;
  const int lw = blockIdx.x >> 3;
  const int nw_x = ((int)gridDim.x - xcd + 7) >> 3;
  const int ntl = fg_count(a, xcd);
  const bool dyn = a.order == 2;   // tiles claimed from a per-XCD counter (contiguous in-flight window)
  if (!dyn && lw >= ntl) return;
  const int nk = a.DPB / FK;
  float* s_qv = reinterpret_cast<float*>(smem + OFF_QV);
  float4* s_qi = reinterpret_cast<float4*>(smem + OFF_QI);
  float* s_pi = reinterpret_cast<float*>(smem + OFF_PI);
  float* s_pl = reinterpret_cast<float*>(smem + OFF_PL);
  const float* Pu = a.Phi ? a.Phi : a.P;   // upper bounds of the parent prefixes
  // bounds [lo, hi] of internal node p's prefix for query q: the path-sum dots (a.pb) or
  // the P / Phi matrices (equal when exact)
  auto pboth = [&](int64_t q, int p, float& lo, float& hi) {
    if (a.pb.dot) {
      pathb_bounds(a.pb, q, p, lo, hi);
    } else {
      lo = a.P[pidx(a.ldP, a.pT, q, p)];
      hi = Pu[pidx(a.ldP, a.pT, q, p)];
    }
  };
  int4* s_rec = reinterpret_cast<int4*>(smem + OFF_REC);
  int* s_cnt = reinterpret_cast<int*>(smem + OFF_CNT);
  // per-lane source offsets of the two 16-row pieces a wave stages per operand
  uint32_t loff[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = wave * 32 + i * 16 + (lane >> 2);
    loff[i] = (uint32_t)((row * a.DPB + (((lane & 3) ^ fg_swz(row)) * 8)) * 2);
  }
  // fragment read offsets (bytes) within an operand image; the swizzle term is the
  // same for every 32-row block, so one per-lane value per k-substep
  const int r16 = lane & 15, c16 = lane >> 4;
  const int foff16 = r16 * 64 + ((c16 ^ fg_swz(r16)) << 4);

  // stage ring: stages are numbered over this workgroup's whole tile sequence, so the
  // next tile's first stages are in flight during the current tile's last steps
  int i = lw;
  if (dyn) {
    if (tid == 0) s_cnt[8] = atomicAdd(&a.tctr[xcd], 1);
    __syncthreads();
    i = __builtin_amdgcn_readfirstlane(s_cnt[8]);
    if (i >= ntl) return;
  }
  int next_i = dyn ? ntl : i + nw_x;   // dynamic: claimed one tile ahead
  int ic_i = i, ic_k = 0, ic_qt, ic_rt, issued = 0, gs = 0;
  fg_decode(a, xcd, ic_i, ic_qt, ic_rt);
  // the next tile is resolved lazily: its first stage is issued during the current
  // tile's K loop, after the setup that claimed it
  auto issue_next = [&]() {
    if (ic_i == -2) {
      ic_i = next_i;
      if (ic_i < ntl) fg_decode(a, xcd, ic_i, ic_qt, ic_rt);
    }
    if (ic_i >= ntl) return;
    if (!(a.dbg & 1)) fg_stage(Xb, Mb, a.DPB, ic_qt * FT, ic_rt * FT, ic_k * FK, smem + (issued & (FNBUF - 1)) * FSTAGE, wave, loff);
    ++issued;
    if (++ic_k == nk) {
      ic_k = 0;
      ic_i = -2;
    }
  };
  issue_next();
  issue_next();
  issue_next();
  int qt, rt;
  int tile_no = 0;   // tiles done by this workgroup (diagnostics)
  (void)tile_no;
  fg_decode(a, xcd, i, qt, rt);
  if (tid == 0) {
    s_cnt[0] = 0;    // records of the current tile (FG_LEAN: even tiles; odd tiles count in [9])
    s_cnt[9] = 0;
    s_cnt[1] = -1;   // owned chunk
    s_cnt[2] = 0;    // its fill
  }
  f32x4 acc[8][4];
#if FG_STAMP
  // diagnostic: per-tile timestamps of wave 0 of workgroups 0..63, tiles 0..15: [wg][tile][4]
  // (setup start, setup barrier passed, K loop done, epilogue done) after the stage stamps
  unsigned long long* tsp = (a.stamp && blockIdx.x < 64 && tid == 0) ? a.stamp + 16384 + (size_t)blockIdx.x * 64 : nullptr;
#define FG_TS(k)                                                                  \
  do {                                                                            \
    if (tsp && tile_no < 16) tsp[tile_no * 4 + (k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define FG_TS(k) \
  do {           \
  } while (0)
#endif
  for (;;) {
    FG_TS(0);
    const int q0 = qt * FT, r0 = rt * FT;
    // ---- tile setup: per-query terms in LDS, per-row terms in registers ----
    TileF tf;
    if (MODE == 0) tf = fg_tile_const(a.tf, rt);
    else tf.uniform = 0;
    const bool uni = ALLUNI || tf.uniform != 0;
    const bool multi = !ALLUNI && tf.uniform == 2;   // per-row parent prefix for survivors
    // all setup loads are issued before any of them is used, so the tile pays one
    // memory round trip (per-query terms, then per-row terms below)
    int claimv = 0;   // the tile after this one (when not claimed ahead): in flight with the loads
    if (dyn && tid == 0) {
      int z;   // opaque zero: a divergent address keeps the atomic optimizer from waiting on the spot
      asm volatile("v_mov_b32 %0, 0" : "=v"(z));
      claimv = atomicAdd(a.tctr + xcd + z, 1);
    }
    const int qs = q0 + tid;
    float4 qi = make_float4(0.f, 0.f, 0.f, 0.f);
    float Tq = CWQ_INF, Pq = 0.f, Pql = 0.f;
    if (tid < FT) {
      qi = a.qinfo[qs];
      if (qs < a.nq && MODE == 0) Tq = a.T[(size_t)qs * a.ldT];
      if (uni && tf.par >= 0 && qs < a.nq) {
        if (a.pb.dot) {
          pathb_bounds(a.pb, qs, tf.par, Pql, Pq);
        } else {
          Pq = Pu[pidx(a.ldP, a.pT, qs, tf.par)];
          Pql = a.P[pidx(a.ldP, a.pT, qs, tf.par)];
        }
      }
    }
    float R0[4];
#pragma unroll
    for (int jb = 0; jb < 4; ++jb) {
      const int r = r0 + wr * 64 + jb * 16 + r16;
      R0[jb] = (uni && r < a.nrows) ? a.rf[r].R0 : 0.f;
    }
    if (tid < FT) {
      const float T = Tq;
      qi.w = T;
      s_qi[tid] = qi;
      // pretest query term for a parent prefix pi (smaller = more permissive)
      auto qv_of = [&](float pi) {
        const float tpg = (T - pi) / tf.g;
        float v = qi.x * (0.5f - 0.5f * a.eps_n) - 1.5f * a.slack * qi.x + tpg - a.slack * fabsf(pi) / tf.g -
                  qi.y * tf.beta_max - qi.z * tf.delta_max;
        v -= 4.f * a.gamma * (fabsf(v) + qi.x + fabsf(tpg) + fabsf(pi) / tf.g);
        return v == v ? v : CWQ_INF;
      };
      float pi = 0.f, qv = CWQ_INF;
      if (uni) {
        pi = Pq * tf.invL;
        if (qs < a.nq && T > -CWQ_INF) {   // T = +inf / NaN / -inf: never a candidate here
          qv = qv_of(pi);
          if (multi) {
            // several parents: a lower bound of qv_of over the tile's parent-prefix range
            // [lo, hi] (each term of qv_of bounded separately; the margin term uses the
            // range's largest magnitudes), from one precomputed load
            const float2 pm = a.pmm[(size_t)rt * a.ldq + qs];
            const float A = qi.x * (0.5f - 0.5f * a.eps_n) - 1.5f * a.slack * qi.x - qi.y * tf.beta_max -
                            qi.z * tf.delta_max;
            const float M = fmaxf(fabsf(pm.x), fabsf(pm.y));
            const float v1L = A + (T - pm.y) / tf.g - a.slack * M / tf.g;
            const float v1U = A + (T - pm.x) / tf.g;
            const float tpm = fmaxf(fabsf(T - pm.x), fabsf(T - pm.y)) / tf.g;
            const float v = v1L - 4.f * a.gamma * (fmaxf(fabsf(v1L), fabsf(v1U)) + qi.x + tpm + M / tf.g);
            qv = v == v ? fminf(qv, v) : CWQ_INF;
          }
        }
      }
      s_pi[tid] = pi;
      s_pl[tid] = uni ? Pql * tf.invL : 0.f;
      if (MODE == 2) s_pl[tid] = qs < a.nq ? a.root_w * (-0.5f * (a.root_ld + a.Sroot[qs])) : 0.f;   // exact root P
      s_qv[tid] = qv;
    }
    if (dyn && tid == 0) s_cnt[8] = claimv;   // the tile after this one
    __syncthreads();   // stage 0 landed, setup visible
    FG_TS(1);
    if (dyn) next_i = __builtin_amdgcn_readfirstlane(s_cnt[8]);   // uniform: scalar tile loads
    // FG_LEAN: the previous tile's record counter (every thread read it before this
    // barrier) is cleared for the tile after this one
    if (FG_LEAN && MODE == 0 && tid == 0 && tile_no > 0) s_cnt[(tile_no & 1) ? 0 : 9] = 0;
    // ---- accumulator init: R_r - Qv_q on uniform tiles, 0 otherwise ----
    // 16x16x32 layout: acc[ib][jb][j] = C[query wq*128 + ib*16 + 4*c16 + j][row wr*64 + jb*16 + r16]
#pragma unroll
    for (int ib = 0; ib < 8; ++ib) {
      const float4 qv4 = uni ? *reinterpret_cast<const float4*>(s_qv + wq * 128 + ib * 16 + 4 * c16)
                             : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) {
        acc[ib][jb][0] = R0[jb] - qv4.x;
        acc[ib][jb][1] = R0[jb] - qv4.y;
        acc[ib][jb][2] = R0[jb] - qv4.z;
        acc[ib][jb][3] = R0[jb] - qv4.w;
      }
    }
    // ---- K loop: one 32-deep v_mfma_f32_16x16x32_bf16 substep per stage ----
    bf16x8 xa1[8], xb0[4];
    // Ping-pong: waves 0-3 and 4-7 (one of each per SIMD) run one barrier interval apart,
    // so in every interval one wave per SIMD issues its 32-MFMA cluster while its partner
    // works through its memory section:
    //   group 0:     M(s) B C(s) B | M(s+1) B C(s+1) B ...
    //   group 1:   B M(s) B C(s) | B M(s+1) B C(s+1) ...
    // M(s): issue stage s+3's LDS-DMA, read all 12 fragments of stage s, wait (own vmcnt)
    // for stage s+1;  C(s): the stage's 32 MFMAs.  Group 1 starts with one extra barrier
    // and skips the last one, so both groups pass the same barriers and group 1's last
    // cluster overlaps group 0's epilogue.  RAW: both groups' waits for stage s+1 precede
    // the barrier before its first read (group 0's M(s+1)).  WAR: the DMA into stage s-1's
    // slot is issued in M(s), after the barrier that follows group 1's last read of it
    // (its M(s-1) ends with lgkmcnt(0)).
    const int grp = wave >> 2;
    auto sbar = [&]() {
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    };
    if (grp) sbar();
#if FG_STAMP
    // diagnostic: per-stage timestamps of waves 0 and 4 (one SIMD) of workgroups 0..15,
    // tiles 4 and 5 of each: [wg][tile-4][wave/4][stage][6]
    const bool stp = a.stamp && blockIdx.x < 16 && (wave & 3) == 0 && lane == 0 && tile_no >= 4 && tile_no < 6;
    unsigned long long* sp =
        stp ? a.stamp + ((((size_t)blockIdx.x * 2 + (tile_no - 4)) * 2 + (wave >> 2)) * 32) * 6 : nullptr;
#define FG_ST(k)                                                               \
  do {                                                                         \
    if (stp && t < 32) sp[t * 6 + (k)] = __builtin_amdgcn_s_memtime();         \
  } while (0)
#else
#define FG_ST(k) \
  do {           \
  } while (0)
#endif
    for (int t = 0; t < nk; ++t) {
      FG_ST(0);
      const char* sb = smem + (gs & (FNBUF - 1)) * FSTAGE;
      issue_next();
      if (!(a.dbg & 128)) {
        const char* sA = sb + wq * 128 * 64 + foff16;
        const char* sB = sb + FT * 64 + wr * 64 * 64 + foff16;
#pragma unroll
        for (int ib = 0; ib < 8; ++ib) xa1[ib] = *reinterpret_cast<const bf16x8*>(sA + ib * 1024);
#pragma unroll
        for (int jb = 0; jb < 4; ++jb) xb0[jb] = *reinterpret_cast<const bf16x8*>(sB + jb * 1024);
      }
      ++gs;
      const int n_out = issued - gs - 1;
      if (a.dbg & 256) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      else if (n_out >= 2) asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)" ::: "memory");
      else if (n_out == 1) asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      FG_ST(1);
      sbar();
      FG_ST(2);
#pragma unroll
      for (int ib = 0; ib < 8; ++ib)
#pragma unroll
        for (int jb = 0; jb < 4; ++jb)
          acc[ib][jb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xa1[ib], xb0[jb], acc[ib][jb], 0, 0, 0);
      FG_ST(3);
      if (t + 1 < nk || grp == 0) sbar();
      FG_ST(4);
    }
#undef FG_ST
    FG_TS(2);
    // ---- epilogue ----
    // The stage buffer just consumed is free until the next tile's first K step
    // re-issues it: 4 KiB per wave of it hold one 32x32 block for the scalar paths.
    float* wsc = reinterpret_cast<float*>(smem + ((gs - 1) & (FNBUF - 1)) * FSTAGE) + wave * 1024;
    // blocks: jb (16 rows) x half (query blocks 0-3 / 4-7): 16 values per lane
    bool anyb[4][2];
    if (a.dbg & 2) goto flush;
    if (MODE == 2 && a.pT) {
      // path sums, node-major [node][ldlb]: the dot of each (node, query) -- readers turn
      // it into bounds with path_bounds (PathB) -- and the root's exact prefix in its line.
      // Lane (r16, c16) of MFMA block (ib, jb) holds queries 4 c16 .. 4 c16 + 3 of one row
      // -- 16 contiguous bytes of that node's line -- so the values go straight from the
      // accumulators to float4 stores (a store instruction covers 16 rows x 64 B)
      int par[4], rid[4];
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) {
        const int r = r0 + wr * 64 + jb * 16 + r16;
        par[jb] = r < a.nrows ? a.rf[r].par : -2;
        rid[jb] = r < a.nrows ? a.row_id[r] : -1;
      }
#pragma unroll
      for (int ib = 0; ib < 8; ++ib) {
        const int ql = wq * 128 + ib * 16 + 4 * c16;
        const int q = q0 + ql;
        if (q >= a.ldlb) continue;   // query padding beyond the lines (ldlb: a multiple of 4)
#pragma unroll
        for (int jb = 0; jb < 4; ++jb) {
          if (par[jb] < -1 || rid[jb] < 0) continue;
          const size_t o = (size_t)rid[jb] * a.ldlb + q;
          const float4 v = par[jb] < 0 ? *reinterpret_cast<const float4*>(s_pl + ql)   // the root: its exact prefix
                                       : make_float4(acc[ib][jb][0], acc[ib][jb][1], acc[ib][jb][2], acc[ib][jb][3]);
          *reinterpret_cast<float4*>(a.lb + o) = v;
        }
      }
      goto flush;
    }
    if (MODE == 2) {
      // internal-node bounds, dense: per 16-query block ib, the wave's 16 x 64 block goes
      // through LDS so that each store covers 64 consecutive rows of one query (256 B)
      const int rl = r0 + wr * 64 + lane;   // this lane's row in the store phase
      const RowF f = rl < a.nrows ? a.rf[rl] : RowF{0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, -2};
      const int rid = a.row_id ? (rl < a.nrows ? a.row_id[rl] : -1) : rl;   // internal node id
      // ib unrolled: a dynamically indexed acc[ib] would be copied to scratch memory
#pragma unroll
      for (int ib = 0; ib < 8; ++ib) {
        // acc[ib][jb][j] = C[query wq*128 + ib*16 + 4*c16 + j][row wr*64 + jb*16 + r16]
#pragma unroll
        for (int jb = 0; jb < 4; ++jb)
#pragma unroll
          for (int j = 0; j < 4; ++j) wsc[(4 * c16 + j) * 64 + jb * 16 + r16] = acc[ib][jb][j];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll 4
        for (int e = 0; e < 16; ++e) {
          const int ql = wq * 128 + ib * 16 + e;
          const int q = q0 + ql;
          if (f.par >= -1 && q < a.nq) {
            const float d0 = wsc[e * 64 + lane];
            float lo, hi;
            if (f.par < 0) {   // the root: its exact prefix
              lo = hi = s_pl[ql];
            } else if (a.path_sum) {   // the path prefix itself
              path_bounds(d0, s_qi[ql], f, s_pl[ql], lo, hi);
            } else {
              int_bounds(d0, s_qi[ql], f, a.gamma, lo, hi);
              if (f.par == 0) prefix_step(s_pl[ql], s_pl[ql], f.invL, lo, hi);   // depth 1: fused
            }
            a.lb[(size_t)q * a.ldlb + rid] = lo;
            a.lb_hi[(size_t)q * a.ldlb + rid] = hi;
          }
        }
        __builtin_amdgcn_wave_barrier();   // reads of this block done before the next dump
      }
      goto flush;
    }
    if (MODE == 1 && a.lbg == 4 && !a.pb.dot) {   // (path-sum bounds: one value per row, below)
      // sample pass: lower bounds reduced to row groups of 4 -- rows r16 + 16 jb of this
      // wave's 64-row block, all in one lane -- before the store.  The K-th largest group
      // maximum is still <= the K-th largest row lower bound (distinct groups are
      // distinct rows), and the bounds array and its select shrink 4x.  Per row only the
      // approximate-key terms stay in registers; the chosen row's RowF is re-read (an L1
      // hit).  The path-sum bounds' reads (PathB) take the per-row form below: inlined 32
      // times here they spilled registers.
      int rrow[4];
      float pa[4], pb[4];
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) {
        const int r = r0 + wr * 64 + jb * 16 + r16;
        const int rr = a.rowmap ? a.rowmap[r] : (r < a.nrows ? r : -1);
        const RowF f = rr >= 0 ? a.rf[rr] : RowF{-CWQ_INF, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, -2};
        rrow[jb] = f.par >= -1 ? rr : -1;
        pa[jb] = fmaf(f.hs, f.rn2, f.hl);   // approximate key = pa + pb * dot (no pi, no error)
        pb[jb] = -2.f * f.hs;
      }
      const int g = (r0 + wr * 64) / 4 + r16;
#pragma unroll
      for (int ib = 0; ib < 8; ++ib)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int ql = wq * 128 + ib * 16 + 4 * c16 + j;
          const int q = q0 + ql;
          // rigorous bound of ONE row per group: the one with the largest approximate key
          // (any row's lower bound is a valid group value)
          int best = -1;
          float bk = -CWQ_INF;
#pragma unroll
          for (int jb = 0; jb < 4; ++jb) {
            const float pk = fmaf(pb[jb], acc[ib][jb][j], pa[jb]);
            if (rrow[jb] >= 0 && (best < 0 || pk > bk)) {
              bk = pk;
              best = jb;
            }
          }
          float m = -CWQ_INF;
          if (best >= 0) {
            int rb = rrow[0];
            float d0 = acc[ib][0][j];
#pragma unroll
            for (int jb = 1; jb < 4; ++jb)
              if (best == jb) {
                rb = rrow[jb];
                d0 = acc[ib][jb][j];
              }
            const RowF fb = a.rf[rb];
            const float4 qi = s_qi[ql];
            float pi = 0.f;
            if (fb.par >= 0 && q < a.nq) pi = a.P[pidx(a.ldP, a.pT, q, fb.par)] * fb.invL;   // exact or lower bounds
            float u;
            fg_bounds(d0, 0x1p-23f * fabsf(d0), qi, fb, pi, a.eps_n, a.slack, u, m);
            if (a.cat && fb.par >= 0 && q < a.nq) m = fminf(m, (a.BFt ? a.BFt : a.P)[pidx(a.ldP, a.pT, q, fb.par)]);
          }
          a.lb[(size_t)q * a.ldlb + g] = m;
        }
      goto flush;
    }
    if (MODE == 0 && uni) {
      bool any = false;
#pragma unroll
      for (int jb = 0; jb < 4; ++jb)
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
          float m = -CWQ_INF;
#pragma unroll
          for (int ib = hf * 4; ib < hf * 4 + 4; ++ib)
            m = __builtin_fmaxf(m, __builtin_fmaxf(__builtin_fmaxf(acc[ib][jb][0], acc[ib][jb][1]),
                                                   __builtin_fmaxf(acc[ib][jb][2], acc[ib][jb][3])));
          anyb[jb][hf] = __ballot(m >= 0.f) != 0;
          any = any || anyb[jb][hf];
        }
      if (!any) goto flush;
    } else {
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) anyb[jb][0] = anyb[jb][1] = true;
    }
#pragma unroll
    for (int jb = 0; jb < 4; ++jb) {
      if (!anyb[jb][0] && !anyb[jb][1]) continue;
      const int r = r0 + wr * 64 + jb * 16 + r16;
      const int rr = a.rowmap ? a.rowmap[r] : (r < a.nrows ? r : -1);
      const RowF f = rr >= 0 ? a.rf[rr] : RowF{-CWQ_INF, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, -2};
      const bool usable = f.par >= -1;
      // the row's parent's path-sum RowF, once per row (not per survivor)
      const RowF fpar = (MODE == 0 && a.pb.dot && f.par > 0) ? a.pb.nrf[f.par]
                                                           : RowF{0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, -1};
      auto pboth_row = [&](int64_t q, float& lo, float& hi) {
        if (a.pb.dot) pathb_bounds_f(a.pb, q, f.par, fpar, lo, hi);
        else pboth(q, f.par, lo, hi);
      };
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        if (!anyb[jb][hf]) continue;
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
          for (int j = 0; j < 4; ++j) wsc[(k * 4 + j) * 64 + lane] = acc[hf * 4 + k][jb][j];
#pragma unroll 1
        for (int e = 0; e < 16; ++e) {
          const float d0 = wsc[e * 64 + lane];
          const int ql = wq * 128 + (hf * 4 + (e >> 2)) * 16 + 4 * c16 + (e & 3);
          const int q = q0 + ql;
            if (MODE == 2) {
              if (usable && q < a.nq && r < a.nrows) {
                float lo, hi;
                if (f.par < 0) {   // the root: its exact prefix
                  lo = hi = s_pl[ql];
                } else {
                  int_bounds(d0, s_qi[ql], f, a.gamma, lo, hi);
                  if (f.par == 0) prefix_step(s_pl[ql], s_pl[ql], f.invL, lo, hi);   // depth 1: fused
                }
                a.lb[(size_t)q * a.ldlb + r] = lo;
                a.lb_hi[(size_t)q * a.ldlb + r] = hi;
              }
            } else if (MODE == 1) {
              float lo = -CWQ_INF;
              if (usable) {
                const float4 qi = s_qi[ql];
                float pi = 0.f;
                if (f.par >= 0 && q < a.nq) {
                  float plo_, phi_;
                  pboth(q, f.par, plo_, phi_);
                  pi = plo_ * f.invL;
                }
                float u;
                fg_bounds(d0, 0x1p-23f * fabsf(d0), qi, f, pi, a.eps_n, a.slack, u, lo);
                if (a.cat && f.par >= 0 && q < a.nq) lo = fminf(lo, (a.BFt ? a.BFt : a.P)[pidx(a.ldP, a.pT, q, f.par)]);
              }
              a.lb[(size_t)q * a.ldlb + r] = lo;
            } else if (usable && q < a.nq && (!uni || d0 >= 0.f)) {
              const float4 qi = s_qi[ql];
              float d, ex, pi, pl;
              if (uni) {
                const float init = f.R0 - s_qv[ql];
                d = d0 - init;
                ex = a.gamma * fabsf(init) + 0x1p-23f * (fabsf(d0) + fabsf(init));
                if (!ALLUNI && multi) {
                  float plo_, phi_;
                  pboth_row(q, plo_, phi_);
                  pi = phi_ * f.invL;
                  pl = plo_ * f.invL;
                } else {
                  pi = s_pi[ql];
                  pl = s_pl[ql];
                }
              } else {
                d = d0;
                ex = 0x1p-23f * fabsf(d0);
                float plo_ = 0.f, phi_ = 0.f;
                if (f.par >= 0) pboth_row(q, plo_, phi_);
                pi = phi_ * f.invL;
                pl = plo_ * f.invL;
              }
              float u, lo;
              fg_bounds2(d, ex, qi, f, pi, pl, a.eps_n, a.slack, u, lo);
              if (a.cat && f.par >= 0) {   // categorize key min(BF[parent], lp)
                const float bp = (a.BFt ? a.BFt : a.P)[pidx(a.ldP, a.pT, q, f.par)];
                u = fminf(u, bp);
                lo = fminf(lo, bp);
              }
              if (u >= qi.w) {
                const int4 rv = make_int4(q, r, __float_as_int(u), __float_as_int(lo));
                const int slot = atomicAdd(&s_cnt[FG_CSLOT], 1);
                if (slot < kFgCap) {
                  s_rec[slot] = rv;
                } else {   // dense tile (small or clustered data): straight to the direct region
                  const int gs = atomicAdd(&a.gctr[1], 1);
                  if (gs < a.dir_cap) a.rec_dir[gs] = rv;
                  else a.qover[q] = 1;
                }
              }
            }
          }
        }
    }
  flush:
    if (MODE == 0) {
      // records -> global append buffer, in chunks of kFgChunk slots owned by this
      // workgroup (one atomic per chunk, not per tile).  This barrier also ends every
      // epilogue LDS read of the tile (wsc, s_qi/s_qv/s_pi), so the next setup may
      // rewrite them; a tile without records skips the rest (uniform: all read cnt here).
      __syncthreads();
      const int cnt = s_cnt[FG_CSLOT];
      const int n = min(cnt, kFgCap);
      if (FG_LEAN && n == 0) goto next_tile;
      if (tid == 0) {
        int chunk = s_cnt[1], fill = s_cnt[2];
        int n1 = chunk >= 0 ? min(n, kFgChunk - fill) : 0;
        int base1 = chunk * kFgChunk + fill, base2 = 0, lost = 0;
        fill += n1;
        if (n > n1) {
          if (chunk >= 0) a.chunk_fill[chunk] = fill;
          const int c2 = atomicAdd(a.gctr, 1);
          if ((int64_t)(c2 + 1) * kFgChunk > a.rec_cap) {   // buffer full: records lost
            lost = 1;
            chunk = -1;
            fill = 0;
            s_cnt[5] = n1;   // write only the first part
          } else {
            chunk = c2;
            fill = n - n1;
            base2 = c2 * kFgChunk;
            s_cnt[5] = n;
          }
        } else {
          s_cnt[5] = n;
        }
        s_cnt[1] = chunk;
        s_cnt[2] = fill;
        s_cnt[3] = base1;
        s_cnt[4] = n1;
        s_cnt[6] = base2;
        s_cnt[7] = lost;
      }
      __syncthreads();
      const int nw = s_cnt[5], n1 = s_cnt[4];
      if (tid < nw) a.rec[tid < n1 ? s_cnt[3] + tid : s_cnt[6] + (tid - n1)] = s_rec[tid];
      if (s_cnt[7] && tid < FT && q0 + tid < a.nq) a.qover[q0 + tid] = 1;   // re-run this tile's queries exactly
    }
  next_tile:
    i = next_i;
    FG_TS(3);
    ++tile_no;
    if (i >= ntl) break;
    if (!dyn) next_i = i + nw_x;
    fg_decode(a, xcd, i, qt, rt);
    if (MODE != 0 || !FG_LEAN) {
      __syncthreads();   // epilogue LDS reads done before the next setup rewrites them
      if (tid == 0) s_cnt[0] = 0;
    }
  }
  if (MODE == 0 && tid == 0 && s_cnt[1] >= 0) a.chunk_fill[s_cnt[1]] = s_cnt[2];
}

// Padded bf16 operand width: whole stages (an even number of them), at least the ring's
// prefetch depth.
int fgemm_dpb(int D) {
  const int g = 2 * FK;
  const int r = (D + g - 1) / g * g;
  const int lo = 4 * FK;
  return r > lo ? r : lo;
}

hipError_t launch_fgemm(const void* Xb, const void* Mb, const FgArgs& a, int n_wg, hipStream_t s) {
  if (a.DPB != fgemm_dpb(a.DPB) || a.n_qt <= 0 || a.n_rt <= 0) return hipErrorInvalidValue;
  if (a.qgroups * a.rgroups != 8) return hipErrorInvalidValue;
  n_wg = std::max(8, n_wg / 8 * 8);
  if (a.mode == 1)
    hipLaunchKernelGGL((fgemm_kernel<1, false>), dim3((unsigned)n_wg), dim3(512), 0, s, (const __bf16*)Xb,
                       (const __bf16*)Mb, a);
  else if (a.mode == 2)
    hipLaunchKernelGGL((fgemm_kernel<2, false>), dim3((unsigned)n_wg), dim3(512), 0, s, (const __bf16*)Xb,
                       (const __bf16*)Mb, a);
  else if (a.all_uniform)
    hipLaunchKernelGGL((fgemm_kernel<0, true>), dim3((unsigned)n_wg), dim3(512), 0, s, (const __bf16*)Xb,
                       (const __bf16*)Mb, a);
  else
    hipLaunchKernelGGL((fgemm_kernel<0, false>), dim3((unsigned)n_wg), dim3(512), 0, s, (const __bf16*)Xb,
                       (const __bf16*)Mb, a);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// bucket: appended records -> per-query candidate lists
// ---------------------------------------------------------------------------
// one record into its query's candidate list
__device__ __forceinline__ void bucket_one(const int4 r, int capq, int* qcnt, int* qover, int* crow, float* cu,
                                           float* cl) {
  const int q = r.x;
  const int slot = atomicAdd(&qcnt[q], 1);
  if (slot < capq) {
    const size_t o = (size_t)q * capq + slot;
    crow[o] = r.y;
    cu[o] = __int_as_float(r.z);
    cl[o] = __int_as_float(r.w);
  } else {
    qover[q] = 1;
  }
}

// grid-stride over the claimed chunks only (gctr[0] of them) and the direct region: the
// grid no longer scales with the buffer capacity (30k mostly idle workgroups at C3)
__global__ __launch_bounds__(256) void bucket_kernel(const int4* __restrict__ rec, const int* __restrict__ gctr,
                                                     const int* __restrict__ chunk_fill, int64_t rec_cap,
                                                     const int4* __restrict__ rec_dir, int dir_cap, int capq,
                                                     int* qcnt, int* qover, int* crow, float* cu, float* cl) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t g0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t n_rec = min((int64_t)gctr[0] * kFgChunk, rec_cap);
  for (int64_t g = g0; g < n_rec; g += stride)
    if ((int)(g % kFgChunk) < chunk_fill[g / kFgChunk]) bucket_one(rec[g], capq, qcnt, qover, crow, cu, cl);
  const int n_dir = min(gctr[1], dir_cap);
  for (int64_t d = g0; d < n_dir; d += stride) bucket_one(rec_dir[d], capq, qcnt, qover, crow, cu, cl);
}

hipError_t launch_bucket(const int4* rec, const int* gctr, const int* chunk_fill, int64_t rec_cap, const int4* rec_dir,
                         int dir_cap, int capq, int* qcnt, int* qover, int* crow, float* cu, float* cl, hipStream_t s) {
  const int64_t n = rec_cap + dir_cap;
  const unsigned grid = (unsigned)std::min<int64_t>((n + 255) / 256, 2048);
  hipLaunchKernelGGL(bucket_kernel, dim3(grid), dim3(256), 0, s, rec, gctr, chunk_fill, rec_cap, rec_dir, dir_cap,
                     capq, qcnt, qover, crow, cu, cl);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// select: top-Kp values per query of a dense [nq][ld] array (the sample bounds; the
// values are first reduced to maxima of up to 16 per lane)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void select_kernel(const float* __restrict__ u, int64_t ldu, int nq, int nrows,
                                                     int Kp, float* cu, int* crow) {
  const int lane = threadIdx.x & 63;
  const int q = blockIdx.x * kWavesPerWG + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  if (q >= nq) return;
  float lk;
  int lr;
  select_wave(u + (size_t)q * ldu, nrows, Kp, lane, lk, lr);
  cu[(size_t)q * 64 + lane] = lk;
  crow[(size_t)q * 64 + lane] = lr;
}

hipError_t launch_select(const float* u, int64_t ldu, int nq, int nrows, int Kp, float* cu, int* crow, hipStream_t s) {
  hipLaunchKernelGGL(select_kernel, dim3((unsigned)((nq + kWavesPerWG - 1) / kWavesPerWG)), dim3(256), 0, s, u, ldu,
                     nq, nrows, Kp, cu, crow);
  return hipGetLastError();
}

// Multi-parent row tiles: per (tile, query) the range of the parents' prefixes x invL, so
// the fgemm tile setup bounds its pretest term with one load instead of walking the
// tile's parents.  Thread = query; tiles along blockIdx.y.
// One workgroup per (32 queries, run of 4 tiles): the run's parents are a contiguous range
// (BFS order); the block copies that range of its queries' prefix rows (P and its upper
// bound Phi) into LDS with coalesced loads, then thread (query, tile) takes min/max over
// the tile's parents from LDS.  Earlier forms: thread per query reading its own row
// (lanes ldP floats apart: 5.1 ms at G = 100k, 10k queries), wave per query with
// cross-lane reductions (slower still: the shuffles).
constexpr int kPrQ = 32, kPrTiles = 4, kPrSpan = 128;   // span: parents per run staged in LDS
__global__ __launch_bounds__(256) void tile_prange_kernel(const float* __restrict__ P, const float* __restrict__ Phi,
                                                          int64_t ldP, int nq, const TileF* __restrict__ tf, int n_rt,
                                                          float2* __restrict__ pmm, int64_t ldq) {
  __shared__ float s_lo[kPrQ][kPrSpan + 1], s_hi[kPrQ][kPrSpan + 1];
  const int tid = threadIdx.x;
  const int runs = (n_rt + kPrTiles - 1) / kPrTiles;
  const int q0 = (blockIdx.x / runs) * kPrQ;
  const int t0 = (blockIdx.x % runs) * kPrTiles, t1 = min(t0 + kPrTiles, n_rt);
  int pa = 0x7fffffff, pb = -1;
  for (int t = t0; t < t1; ++t) {
    const TileF T = tf[t];
    if (T.uniform == 2) {
      pa = min(pa, T.par);
      pb = max(pb, T.par_hi);
    }
  }
  if (pb < 0) return;   // no multi-parent tile in the run (uniform over the block)
  const int ql = tid % kPrQ, t = t0 + tid / kPrQ;
  const int q = q0 + ql;
  bool act = t < t1 && q < nq;
  TileF T{};
  if (act) {
    T = tf[t];
    act = T.uniform == 2;
  }
  float mn = CWQ_INF, mx = -CWQ_INF;
  // the run's parent range through LDS in windows of kPrSpan parents (coalesced rows)
  for (int w0 = pa; w0 <= pb; w0 += kPrSpan) {
    const int span = min(kPrSpan, pb - w0 + 1);
    __syncthreads();   // the previous window is consumed
    for (int i = tid; i < kPrQ * span; i += 256) {
      const int qq = i / span, p = w0 + (i - qq * span);
      if (q0 + qq < nq) {
        s_lo[qq][p - w0] = P[(size_t)(q0 + qq) * ldP + p];
        s_hi[qq][p - w0] = Phi[(size_t)(q0 + qq) * ldP + p];
      }
    }
    __syncthreads();
    if (act) {
      const int p0 = max(T.par, w0), p1 = min(T.par_hi, w0 + span - 1);
      for (int p = p0; p <= p1; ++p) {
        // a pruned parent (cwq_prune.hip: sentinel prefix) holds no candidate: it must not
        // widen the range the other parents' rows are pretested with
        if (s_hi[ql][p - w0] <= kPruneCut) continue;
        const float a = s_lo[ql][p - w0] * T.invL, b = s_hi[ql][p - w0] * T.invL;
        mn = fminf(mn, fminf(a, b));
        mx = fmaxf(mx, fmaxf(a, b));
      }
    }
  }
  if (act) pmm[(size_t)t * ldq + q] = make_float2(mn, mx);
}

// Node-major prefixes (pidx pT): thread = query, one tile per blockIdx.y; the tile's parents
// are read one line at a time, each read coalesced over the block's 256 queries.
__global__ __launch_bounds__(256) void tile_prange_t_kernel(const float* __restrict__ P, const float* __restrict__ Phi,
                                                            int64_t ldP, int nq, const TileF* __restrict__ tf,
                                                            int t0, float2* __restrict__ pmm, int64_t ldq) {
  const int t = t0 + blockIdx.y;
  const TileF T = tf[t];
  if (T.uniform != 2) return;
  const int q = blockIdx.x * 256 + threadIdx.x;
  if (q >= nq) return;
  float mn0 = CWQ_INF, mx0 = -CWQ_INF, mn1 = CWQ_INF, mx1 = -CWQ_INF;
  int p = T.par;
  for (; p + 1 <= T.par_hi; p += 2) {   // two lines in flight per step
    const float a0 = P[(size_t)p * ldP + q], b0 = Phi[(size_t)p * ldP + q];
    const float a1 = P[(size_t)(p + 1) * ldP + q], b1 = Phi[(size_t)(p + 1) * ldP + q];
    mn0 = fminf(mn0, fminf(a0 * T.invL, b0 * T.invL));
    mx0 = fmaxf(mx0, fmaxf(a0 * T.invL, b0 * T.invL));
    mn1 = fminf(mn1, fminf(a1 * T.invL, b1 * T.invL));
    mx1 = fmaxf(mx1, fmaxf(a1 * T.invL, b1 * T.invL));
  }
  if (p <= T.par_hi) {
    const float a0 = P[(size_t)p * ldP + q], b0 = Phi[(size_t)p * ldP + q];
    mn0 = fminf(mn0, fminf(a0 * T.invL, b0 * T.invL));
    mx0 = fmaxf(mx0, fmaxf(a0 * T.invL, b0 * T.invL));
  }
  pmm[(size_t)t * ldq + q] = make_float2(fminf(mn0, mn1), fmaxf(mx0, mx1));
}

// Path-sum dots (PathB): thread = query, one tile per blockIdx.y; each parent's dot line
// read coalesced over the block's queries (eight in flight), turned into [lo, hi] by
// path_bounds with the parent's RowF (staged in LDS once per block); parents without an
// operand row (no isotropic leaf row below them) are not parents of the tile's rows and are
// skipped.
__global__ __launch_bounds__(256) void tile_prange_pb_kernel(const PathB pb, int nq, const TileF* __restrict__ tf,
                                                             int t0, float2* __restrict__ pmm, int64_t ldq) {
  __shared__ RowF s_f[kFgMaxTileParents];   // the tile's parents' RowF, staged once per block
  const int t = t0 + blockIdx.y;
  const TileF T = tf[t];
  if (T.uniform != 2) return;   // uniform over the block
  const int np = min(T.par_hi - T.par + 1, kFgMaxTileParents);
  for (int i = threadIdx.x; i < np; i += blockDim.x) s_f[i] = pb.nrf[T.par + i];
  __syncthreads();
  const int q = blockIdx.x * 256 + threadIdx.x;
  if (q >= nq) return;
  const float4 qi = pb.qi2[q];
  const float proot = pb.dot[q];
  float mn = CWQ_INF, mx = -CWQ_INF;
  // eight dot lines in flight per step (independent loads, then the bounds)
  for (int i0 = 0; i0 < np; i0 += 8) {
    float d8[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) d8[u] = i0 + u < np ? pb.dot[(size_t)(T.par + i0 + u) * pb.ld + q] : 0.f;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = i0 + u, p = T.par + i;
      if (i >= np) break;
      const RowF f = s_f[i];
      if (f.par < -1 && p != 0) continue;   // no operand row: not a parent of the tile's rows
      float lo, hi;
      if (p == 0) lo = hi = d8[u];
      else path_bounds(d8[u], qi, f, proot, lo, hi);
      mn = fminf(mn, fminf(lo * T.invL, hi * T.invL));
      mx = fmaxf(mx, fmaxf(lo * T.invL, hi * T.invL));
    }
  }
  pmm[(size_t)t * ldq + q] = make_float2(mn, mx);
}

// Diagnostic (cwq_prefix_bounds): the path-sum dots as [lo, hi] matrices [nq][NI].
__global__ void pathb_expand_kernel(const PathB pb, int nq, int NI, float* lo, float* hi) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)nq * NI) return;
  const int q = (int)(i / NI), p = (int)(i % NI);
  float l, h;
  pathb_bounds(pb, q, p, l, h);
  lo[i] = l;
  hi[i] = h;
}

hipError_t launch_pathb_expand(const PathB& pb, int nq, int NI, float* lo, float* hi, hipStream_t s) {
  const int64_t n = (int64_t)nq * NI;
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(pathb_expand_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, pb, nq, NI, lo, hi);
  return hipGetLastError();
}

hipError_t launch_tile_prange(const float* P, const float* Phi, int64_t ldP, int pT, int nq, const TileF* tf,
                              int n_rt, float2* pmm, int64_t ldq, hipStream_t s, const PathB* pb) {
  static_assert(kPrQ * kPrTiles <= 256, "one thread per (query, tile)");
  if (pb && pb->dot) {
    if (nq <= 0 || n_rt <= 0) return hipSuccess;
    for (int t0 = 0; t0 < n_rt; t0 += 65535) {   // grid y limit
      hipLaunchKernelGGL(tile_prange_pb_kernel, dim3((unsigned)((nq + 255) / 256), (unsigned)std::min(65535, n_rt - t0)),
                         dim3(256), 0, s, *pb, nq, tf, t0, pmm, ldq);
      if (hipError_t e = hipGetLastError()) return e;
    }
    return hipSuccess;
  }
  if (pT) {
    if (nq <= 0 || n_rt <= 0) return hipSuccess;
    for (int t0 = 0; t0 < n_rt; t0 += 65535) {   // grid y limit
      hipLaunchKernelGGL(tile_prange_t_kernel, dim3((unsigned)((nq + 255) / 256), (unsigned)std::min(65535, n_rt - t0)),
                         dim3(256), 0, s, P, Phi ? Phi : P, ldP, nq, tf, t0, pmm, ldq);
      if (hipError_t e = hipGetLastError()) return e;
    }
    return hipSuccess;
  }
  const int64_t blocks = (int64_t)((nq + kPrQ - 1) / kPrQ) * ((n_rt + kPrTiles - 1) / kPrTiles);
  if (blocks <= 0) return hipSuccess;
  hipLaunchKernelGGL(tile_prange_kernel, dim3((unsigned)blocks), dim3(256), 0, s, P, Phi ? Phi : P, ldP, nq, tf, n_rt,
                     pmm, ldq);
  return hipGetLastError();
}


// ---------------------------------------------------------------------------
// tighten: between filter phases, T[q] = max(T[q], K-th largest lower bound among the
// candidates found so far) -- still <= tau_K (they are K distinct rows).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void tighten_kernel(int nq, int K, int capq, const int* __restrict__ qcnt,
                                                      const int* __restrict__ qover, const float* __restrict__ cl,
                                                      float* T, int64_t ldT, float* lkb, int* lrb, int* done,
                                                      int* zero16) {
  const int lane = threadIdx.x & 63;
  // the filter's record/tile counters for the next launch (bucket has read them)
  if (blockIdx.x == 0 && threadIdx.x < 16) zero16[threadIdx.x] = 0;
  const int q = blockIdx.x * kWavesPerWG + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  if (q >= nq) return;
  const int n = min(qcnt[q], capq);
  if (qover[q]) return;
  // incremental: the top-K candidate lower bounds so far are kept per query, and only the
  // candidates appended since the last call are offered
  const int d = done[q];
  float tk = d ? lkb[(size_t)q * 64 + lane] : -CWQ_INF;
  int tr = d ? lrb[(size_t)q * 64 + lane] : 0x7fffffff;
  const size_t base = (size_t)q * capq;
  for (int j0 = d; j0 < n; j0 += 64) {
    const int j = j0 + lane;
    list64_offer(tk, tr, lane, j < n ? cl[base + j] : -CWQ_INF, j, K);
  }
  lkb[(size_t)q * 64 + lane] = tk;
  lrb[(size_t)q * 64 + lane] = tr;
  if (lane == 0) done[q] = n;
  const float kth = rl_f2(tk, K - 1);
  if (lane == 0 && kth > T[(size_t)q * ldT]) T[(size_t)q * ldT] = kth;
}

hipError_t launch_tighten(int nq, int K, int capq, const int* qcnt, const int* qover, const float* cl, float* T,
                          int64_t ldT, float* lkb, int* lrb, int* done, int* zero16, hipStream_t s) {
  hipLaunchKernelGGL(tighten_kernel, dim3((unsigned)((nq + 3) / 4)), dim3(256), 0, s, nq, K, capq, qcnt, qover, cl, T,
                     ldT, lkb, lrb, done, zero16);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// final: per query (one wave), T2 = K-th largest l among the candidates, exact keys
// of the candidates with u >= T2 (bit-identical to the scan kernel's ISO arithmetic),
// exact top-K into partial-list slot 0.  X is the scan's interleaved query layout
// [q/16][v][q%16][16].
// ---------------------------------------------------------------------------
__device__ __forceinline__ float exact_iso_key(const float* __restrict__ X, const float* __restrict__ Mf, int DP,
                                               int q, int rr, const RowMeta& md, float pp, float& lp,
                                               int cat = 0, float dconst = 0.f) {
  const float* __restrict__ mr = Mf + (size_t)rr * DP;
  const int NV16 = DP / 16;
  const f32x16* __restrict__ xg = reinterpret_cast<const f32x16*>(X) + (size_t)(q / kXQ) * NV16 * kXQ + (q % kXQ);
  float acc = 0.f;
  auto slice = [&](const f32x16& xa, const float4* m4) {   // one 16-dim partial, scan order
    float part;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const float4 t4 = m4[j >> 2];
      const float mj = (j & 3) == 0 ? t4.x : (j & 3) == 1 ? t4.y : (j & 3) == 2 ? t4.z : t4.w;
      const float t = xa[j] - mj;
      part = (j == 0) ? t * t : fmaf(t, t, part);
    }
    acc += part;
  };
  // the row's slices are loaded CB at a time before any is used (one memory latency per
  // CB slices instead of per slice); the arithmetic order is unchanged
  constexpr int CB = 8;
  int v = 0;
  for (; v + CB <= NV16; v += CB) {
    float4 m4[CB][4];
#pragma unroll
    for (int u = 0; u < CB; ++u)
#pragma unroll
      for (int j = 0; j < 4; ++j) m4[u][j] = *reinterpret_cast<const float4*>(mr + (v + u) * 16 + j * 4);
    f32x16 xs[CB];
#pragma unroll
    for (int u = 0; u < CB; ++u) xs[u] = xg[(size_t)(v + u) * kXQ];
#pragma unroll
    for (int u = 0; u < CB; ++u) slice(xs[u], m4[u]);
  }
  for (; v < NV16; ++v) {
    float4 m4[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) m4[j] = *reinterpret_cast<const float4*>(mr + v * 16 + j * 4);
    slice(xg[(size_t)v * kXQ], m4);
  }
  return iso_key_tail(acc, md, pp, lp, cat, dconst);   // categorize: pp = BF[parent]
}

// Raw sum S = sum_d (x_d A_d - B_d)^2 of internal node i for query q in the exact scan's
// arithmetic (16-dim fma partials in dim order, summed in order): bit-identical to the
// scan_kernel / int_small_kernel values.  Ar/Br: row-major copies of int_A/int_B.
__device__ __forceinline__ float exact_aniso_S(const float* __restrict__ X, const float* __restrict__ Ar,
                                               const float* __restrict__ Br, int DP, int q, int i) {
  const float* __restrict__ ar = Ar + (size_t)i * DP;
  const float* __restrict__ br = Br + (size_t)i * DP;
  const int NV16 = DP / 16;
  const f32x16* __restrict__ xg = reinterpret_cast<const f32x16*>(X) + (size_t)(q / kXQ) * NV16 * kXQ + (q % kXQ);
  float acc = 0.f;
  for (int v = 0; v < NV16; ++v) {
    float4 a4[4], b4[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      a4[j] = *reinterpret_cast<const float4*>(ar + v * 16 + j * 4);
      b4[j] = *reinterpret_cast<const float4*>(br + v * 16 + j * 4);
    }
    const f32x16 xa = xg[(size_t)v * kXQ];
    float part;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const float4 ta = a4[j >> 2], tb = b4[j >> 2];
      const float aj = (j & 3) == 0 ? ta.x : (j & 3) == 1 ? ta.y : (j & 3) == 2 ? ta.z : ta.w;
      const float bj = (j & 3) == 0 ? tb.x : (j & 3) == 1 ? tb.y : (j & 3) == 2 ? tb.z : tb.w;
      const float t = fmaf(xa[j], aj, -bj);
      part = (j == 0) ? t * t : fmaf(t, t, part);
    }
    acc += part;
  }
  return acc;
}

// Exact path prefix P of internal node p (> 0) from the exact root prefix: the chain of
// prefix_level_kernel steps P = fmaf(w, lp', P[parent]) recomputed for p's ancestors.
// The chain is walked top-down by re-walking from p (depth^2 parent loads, no local
// array: a dynamically indexed one would put every caller on scratch memory).
__device__ __forceinline__ float exact_prefix(const float* __restrict__ X, const IntChain& ch, int DP, int q, int p,
                                              float proot) {
  int n = 0;
  for (int j = p; j > 0 && n < kMaxChain; j = ch.par_int[j]) ++n;
  float P = proot;
  for (int t = n - 1; t >= 0; --t) {
    int a = p;
    for (int u = 0; u < t; ++u) a = ch.par_int[a];   // the ancestor t levels above p
    const float S = exact_aniso_S(X, ch.Ar, ch.Br, DP, q, a);
    const float lp = -0.5f * (ch.logdet_int[a] + S);
    P = fmaf(ch.w_int[a], lp, P);
  }
  return P;
}

// Exact path prefixes of the candidates' parents for one query (one wave; every lane
// calls it, `need` marks the lanes with a parent p > 0), with exact_prefix's arithmetic
// node for node but each ancestor computed ONCE per query: the chains are walked top-down
// one depth per step, and at each step the lanes that need the same node (the top
// levels are shared by every candidate of a query) find it in a per-wave LDS table --
// the first lane to claim a node computes its exact S and P = fmaf(w, lp', P(parent)),
// the others read P after the wave barrier (a node's parent prefix is the same for
// every lane that reaches it).  A node that finds no free slot is computed by its lane.
constexpr int kChainSlots = 256;
__device__ __forceinline__ float chain_prefix_cached(const float* __restrict__ X, const IntChain& ch, int DP, int q,
                                                     bool need, int p, float proot, int* ck, float* cv) {
  int n = 0;
  if (need)
    for (int j = p; j > 0 && n < kMaxChain; j = ch.par_int[j]) ++n;
  int nmax = n;
  for (int off = 32; off > 0; off >>= 1) nmax = max(nmax, __shfl_xor(nmax, off, 64));
  float P = proot;
  for (int t = 0; t < nmax; ++t) {   // depth t + 1 for every lane
    const bool on = need && t < n;
    int a = -1, slot = -1;
    bool owner = false;
    if (on) {
      a = p;
      for (int u = 0; u < n - 1 - t; ++u) a = ch.par_int[a];
      int h = a & (kChainSlots - 1);
      for (int probe = 0; probe < 8; ++probe) {
        const int old = atomicCAS(ck + h, -1, a);
        if (old == -1 || old == a) {
          slot = h;
          owner = old == -1;
          break;
        }
        h = (h + 1) & (kChainSlots - 1);
      }
    }
    float Pa = 0.f;
    if (on && (owner || slot < 0)) {
      const float S = exact_aniso_S(X, ch.Ar, ch.Br, DP, q, a);
      const float lp = -0.5f * (ch.logdet_int[a] + S);
      Pa = fmaf(ch.w_int[a], lp, P);
      if (owner) cv[slot] = Pa;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (on && !owner && slot >= 0) Pa = cv[slot];
    if (on) P = Pa;
  }
  return P;
}

__global__ __launch_bounds__(256) void final_kernel(const float* __restrict__ X, const float* __restrict__ Mf, int DP,
                                                    int nq, int K, int capq, const int* __restrict__ qcnt,
                                                    const int* __restrict__ qover, const int* __restrict__ crow,
                                                    const float* __restrict__ cu, const float* __restrict__ cl,
                                                    const float* __restrict__ T, int64_t ldT,
                                                    const RowMeta* __restrict__ meta, const int* __restrict__ par,
                                                    const float* __restrict__ P, int64_t ldP, int seg_base,
                                                    float* pkey, float* paux, int* prow, int64_t lstride,
                                                    int* ok_flag, int* n_exact, const float* __restrict__ lkb,
                                                    const int* __restrict__ lrb, const int* __restrict__ done,
                                                    const IntChain chain, int use_chain, int cat,
                                                    float dconst) {
  __shared__ int s_pend[kWavesPerWG][128];
  __shared__ int s_ck[kWavesPerWG][kChainSlots];     // exact-prefix table (chain_prefix_cached)
  __shared__ float s_cv[kWavesPerWG][kChainSlots];
  const int lane = threadIdx.x & 63;
  const int q = blockIdx.x * kWavesPerWG + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  if (q >= nq) return;
  if (use_chain) {
    for (int i = lane; i < kChainSlots; i += 64) s_ck[threadIdx.x >> 6][i] = -1;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  const int n = qcnt[q];
  const float Tq = T[(size_t)q * ldT];
  bool ok = qover[q] == 0 && n >= K && n <= capq && Tq > -CWQ_INF;
  float lk = -CWQ_INF, la = 0.f;
  int lr = 0x7fffffff;
  int nx = 0;
  if (ok) {
    const size_t base = (size_t)q * capq;
    // pass 1: K-th largest lower bound (continuing tighten's list: only the candidates
    // of the last phase are offered)
    const int d = done[q];
    float tk = d ? lkb[(size_t)q * 64 + lane] : -CWQ_INF;
    int tr = d ? lrb[(size_t)q * 64 + lane] : 0x7fffffff;
    for (int j0 = d; j0 < n; j0 += 64) {
      const int j = j0 + lane;
      const float lv = j < n ? cl[base + j] : -CWQ_INF;
      list64_offer(tk, tr, lane, lv, j, K);
    }
    const float T2 = rl_f2(tk, K - 1);
    // pass 2: exact keys of the survivors (u >= T2), packed 64 to a round through a
    // per-wave LDS list so that every lane of a round has a row (C3: ~20 survivors
    // spread over ~3 chunks of candidates -> one round instead of three)
    int* pend = s_pend[threadIdx.x >> 6];
    int npend = 0;
    for (int j0 = 0; j0 < n || npend > 0; j0 += 64) {
      const int j = j0 + lane;
      const bool c = j < n && cu[base + j] >= T2;
      const uint64_t bm = __ballot(c);
      if (c) pend[npend + __popcll(bm & ((1ull << lane) - 1))] = j;
      npend += __popcll(bm);
      if (npend < 64 && j0 + 64 < n) continue;   // more candidates to pack first
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const bool act = lane < npend;
      const int jj = act ? pend[lane] : 0;
      const int rest = npend > 64 ? pend[64 + lane] : 0;   // lane < npend - 64 <= 63
      float key = -CWQ_INF, lp = 0.f;
      int rid = 0x7fffffff;
      const int rr = act ? crow[base + jj] : 0;
      const int p = act ? par[rr] : -1;
      // with the chain only the root's P[q][0] is read (ldP 1: node-major); every lane of
      // the wave takes part in the cached chain walk
      const float pc = use_chain ? chain_prefix_cached(X, chain, DP, q, act && p > 0, p, P[(size_t)q * ldP],
                                                       s_ck[threadIdx.x >> 6], s_cv[threadIdx.x >> 6])
                                 : 0.f;
      if (act) {
        const RowMeta md = meta[rr];
        // exact (cat: BF)
        float pp = p < 0 ? (cat ? CWQ_INF : 0.f) : (use_chain && p > 0 ? pc : P[(size_t)q * ldP + p]);
        key = exact_iso_key(X, Mf, DP, q, rr, md, pp, lp, cat, dconst);
        rid = seg_base + rr;
        ++nx;
      }
      __builtin_amdgcn_wave_barrier();
      if (npend > 64 && lane < npend - 64) pend[lane] = rest;
      npend = npend > 64 ? npend - 64 : 0;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const bool c2 = act;
      uint64_t mask = __ballot(c2);
      while (mask) {
        const int b = __builtin_ctzll(mask);
        mask &= mask - 1;
        const float ck = rl_f2(key, b), ca = rl_f2(lp, b);
        const int cr = __builtin_amdgcn_readlane(rid, b);
        // categorize lists: the smaller own lp first among equal keys (list_before<true>)
        const bool prec = lk > ck || (lk == ck && (cat && la != ca ? la < ca : lr < cr));
        const int pos = __popcll(__ballot(prec));
        if (pos < K) {
          const float sk = __int_as_float(wave_shr1(__float_as_int(lk)));
          const float sa = __int_as_float(wave_shr1(__float_as_int(la)));
          const int sr = wave_shr1(lr);
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
  }
  if (lane < K) {
    const size_t o = (size_t)q * lstride + lane;
    pkey[o] = ok ? lk : -CWQ_INF;
    paux[o] = la;
    prow[o] = ok ? lr : 0x7fffffff;
  }
  for (int off = 32; off > 0; off >>= 1) nx += __shfl_xor(nx, off, 64);
  if (lane == 0) {
    ok_flag[q] = ok ? 1 : 0;
    if (n_exact) n_exact[q] = nx;
  }
}

// final for small batches (nq <= kFinalWideMaxQ, the per-call paths): one 512-thread
// workgroup per query.  The exact keys are the same arithmetic as exact_iso_key, split
// differently over the threads: the 16-dim partials of up to 64 survivors are computed in
// parallel (one thread per (survivor, slice) -- every load of a round in flight at once),
// then lane s of wave 0 adds survivor s's partials in slice order (acc += part, as the
// scan does), so the keys are bit-identical; the per-lane form pays one row's dependent
// load chain per round (~33 us of a 1-query call at C3).
// Memory round trips are the cost at one query per call, so the query's counters and the
// first kFwThreads entries of its candidate lists arrive in ONE round (loaded before the
// count is known; entries past it are never used), and the survivors' row terms fly with
// their partials' row loads.  fx (optional): the fused expansion + host flags (FwExpand).
constexpr int kFwThreads = 512;
constexpr int kFwCand = 4096;   // candidates whose l, u are staged in LDS (= kFgCapQ)
constexpr int kFwMaxRows = 192;   // survivors per rerank round (three key waves)
constexpr int kFwDynMax = 56 * 1024;   // dynamic LDS budget (the static part is ~103 KiB of 160)
// Exact path prefixes of a round's survivor parents with the whole workgroup
// (final_wide_kernel, hierarchical trees): the distinct ancestors of every parent go into an
// LDS table (wave 0; a lane stops at the first node another lane has entered, whose
// ancestors that lane enters), then every (node, 16-dim slice) partial is computed in
// parallel, one thread per node adds them in slice order (exact_aniso_S's arithmetic), and
// the prefixes P = fmaf(w, lp', P(parent)) are stepped level by level from the root's exact
// prefix -- exact_prefix's values, without a depth x D serial chain per lane (226 of a
// 905 us one-query call on a depth-9 tree).  Returns false when the table overflows (the
// caller then takes the per-lane chain).
constexpr int kFwChainNodes = 1024, kFwChainHash = 2048, kFwChainPart = 8192;
struct FwChainLds {
  int hk[kFwChainHash];      // node id (-1: empty)
  int hv[kFwChainHash];      // its entry
  int node[kFwChainNodes];
  int depth[kFwChainNodes];
  float val[kFwChainNodes];  // lp', then P
  float part[kFwChainPart];  // [entries of a chunk][NV16] slice partials
  float pp[64];              // the result per wave-0 lane
  int m, maxd, over;
};
__device__ __forceinline__ int fw_hash(int a) { return (int)(((unsigned)a * 2654435761u) >> 21) & (kFwChainHash - 1); }
__device__ __forceinline__ int fw_find(const FwChainLds& L, int a) {
  int h = fw_hash(a);
  for (int t = 0; t < kFwChainHash; ++t) {
    const int k = L.hk[h];
    if (k == a) return L.hv[h];
    if (k == -1) return -1;
    h = (h + 1) & (kFwChainHash - 1);
  }
  return -1;
}
// every thread of the workgroup calls it; wave 0 lanes with `need` have parent p > 0
__device__ bool fw_chain_prefixes(FwChainLds& L, const f32x16* __restrict__ xg, const IntChain& ch, int DP, bool need,
                                  int p, float proot) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < kFwChainHash; i += kFwThreads) L.hk[i] = -1;
  if (tid == 0) {
    L.m = 0;
    L.maxd = 0;
    L.over = 0;
  }
  __syncthreads();
  if (wave == 0 && need) {
    int d = 0;
    for (int j = p; j > 0 && d < kMaxChain; j = ch.par_int[j]) ++d;
    atomicMax(&L.maxd, d);
    for (int a = p; a > 0 && d > 0; a = ch.par_int[a], --d) {
      int h = fw_hash(a), t = 0;
      bool stop = false;
      for (; t < kFwChainHash; ++t) {
        const int old = atomicCAS(&L.hk[h], -1, a);
        if (old == -1) {   // entered here: its entry, then on to its parent
          const int e = atomicAdd(&L.m, 1);
          if (e < kFwChainNodes) {
            L.node[e] = a;
            L.depth[e] = d;
          } else {
            L.over = 1;
          }
          L.hv[h] = e;
          break;
        }
        if (old == a) {   // entered by another lane, which enters its ancestors
          stop = true;
          break;
        }
        h = (h + 1) & (kFwChainHash - 1);
      }
      if (t == kFwChainHash) L.over = 1;
      if (stop) break;
    }
  }
  __syncthreads();
  if (L.over) return false;
  const int m = L.m, NV16 = DP / 16;
  const int chunk = kFwChainPart / NV16;
  for (int c0 = 0; c0 < m; c0 += chunk) {
    const int nc = min(chunk, m - c0);
    for (int it = tid; it < nc * NV16; it += kFwThreads) {
      const int e = it / NV16, v = it - e * NV16;
      const int a = L.node[c0 + e];
      const float* __restrict__ ar = ch.Ar + (size_t)a * DP + v * 16;
      const float* __restrict__ br = ch.Br + (size_t)a * DP + v * 16;
      float4 a4[4], b4[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        a4[j] = *reinterpret_cast<const float4*>(ar + j * 4);
        b4[j] = *reinterpret_cast<const float4*>(br + j * 4);
      }
      const f32x16 xa = xg[(size_t)v * kXQ];
      float part;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const float4 ta = a4[j >> 2], tb = b4[j >> 2];
        const float aj = (j & 3) == 0 ? ta.x : (j & 3) == 1 ? ta.y : (j & 3) == 2 ? ta.z : ta.w;
        const float bj = (j & 3) == 0 ? tb.x : (j & 3) == 1 ? tb.y : (j & 3) == 2 ? tb.z : tb.w;
        const float t = fmaf(xa[j], aj, -bj);
        part = (j == 0) ? t * t : fmaf(t, t, part);
      }
      L.part[it] = part;
    }
    __syncthreads();
    for (int e = tid; e < nc; e += kFwThreads) {
      const float acc = sum_in_order(L.part + e * NV16, NV16);
      L.val[c0 + e] = -0.5f * (ch.logdet_int[L.node[c0 + e]] + acc);
    }
    __syncthreads();
  }
  for (int d = 1; d <= L.maxd; ++d) {   // prefixes, root side first
    for (int e = tid; e < m; e += kFwThreads) {
      if (L.depth[e] != d) continue;
      const int a = L.node[e], pa = ch.par_int[a];
      const float Pp = pa > 0 ? L.val[fw_find(L, pa)] : proot;
      L.val[e] = fmaf(ch.w_int[a], L.val[e], Pp);
    }
    __syncthreads();
  }
  if (wave == 0 && need) L.pp[lane] = L.val[fw_find(L, p)];
  __syncthreads();
  return true;
}

#ifndef CWQ_STAMP
#define CWQ_STAMP 0   // diagnostic builds only (scripts/build_variant.py): wall-clock phase stamps
#endif
#if CWQ_STAMP
// final_wide_kernel's phases, per workgroup (the last launch's), 100 MHz wall clock
__device__ unsigned long long g_fw_stamp[256 * 16];
#define FW_ST(ph)                                                                       \
  do {                                                                                  \
    if (threadIdx.x == 0 && blockIdx.x < 256) g_fw_stamp[blockIdx.x * 16 + (ph)] = wall_clock64(); \
  } while (0)
extern "C" int cwq_debug_fw_stamp(unsigned long long* out, int n) {   // copies out, then clears
  static unsigned long long zero[256 * 16] = {};
  const hipError_t e =
      hipMemcpyFromSymbol(out, HIP_SYMBOL(g_fw_stamp), sizeof(unsigned long long) * (size_t)std::min(n, 4096));
  return e != hipSuccess ? (int)e : (int)hipMemcpyToSymbol(HIP_SYMBOL(g_fw_stamp), zero, sizeof(zero));
}
#else
#define FW_ST(ph) ((void)0)
#endif

__global__ __launch_bounds__(kFwThreads) void final_wide_kernel(
    const float* __restrict__ X, const float* __restrict__ Mf, int DP, int nq, int K, int capq,
    const int* __restrict__ qcnt, const int* __restrict__ qover, const int* __restrict__ crow,
    const float* __restrict__ cu, const float* __restrict__ cl, const float* __restrict__ T, int64_t ldT,
    const RowMeta* __restrict__ meta, const int* __restrict__ par, const float* __restrict__ P, int64_t ldP,
    int seg_base, float* pkey, float* paux, int* prow, int64_t lstride, int* ok_flag, int* n_exact,
    const float* __restrict__ lkb, const int* __restrict__ lrb, const int* __restrict__ done, const IntChain chain,
    int use_chain, int cat, float dconst, const FwExpand fx, int rows, int nopf) {
  extern __shared__ float s_dyn[];
  const int NV16 = DP / 16, LDP = NV16 + 1;                  // odd row pitch: conflict-free column reads
  float* s_part = s_dyn;                                      // [rows][LDP]
  int* s_surv = reinterpret_cast<int*>(s_dyn + rows * LDP);  // [capq] survivor positions
  __shared__ float s_wl[kFwCand], s_wu[kFwCand];              // candidates' l, u (the first kFwCand)
  __shared__ int s_wr[kFwThreads];                            // rows of candidates 0..kFwThreads-1
  __shared__ float s_ml[kFwThreads], s_ma[kFwThreads];        // per-wave top-K lists (T2 and key merges)
  __shared__ int s_mr[kFwThreads];
  __shared__ int s_rr[kFwMaxRows];
  __shared__ int s_nx;
  __shared__ int s_ns;
  __shared__ float s_T2;
  __shared__ FwChainLds s_chain;   // exact parent chains (fw_chain_prefixes)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int S = fx.split > 1 ? fx.split : 1;   // workgroups per query (FwExpand::split)
  const int q = blockIdx.x / S, sidx = blockIdx.x - q * S;
  const size_t base = (size_t)q * capq;
  // ---- one round trip: counters + the first window of the candidate lists ----
  FW_ST(0);
  const int n = qcnt[q];
  const float Tq = T[(size_t)q * ldT];
  const int ov = qover[q];
  (void)lkb;   // the stream select's list of the first done[q] candidates: not needed (T2 below)
  (void)lrb;
  (void)done;
  if (tid < capq) {
    s_wl[tid] = cl[base + tid];
    s_wu[tid] = cu[base + tid];
    s_wr[tid] = crow[base + tid];
  }
  if (tid == 0) {
    s_ns = 0;
    s_nx = 0;
  }
  // T = -inf (categorize lists whose probe saw fewer than K finite keys): every row with a
  // finite bound is a candidate, so the list is complete while it did not overflow
  const bool ok = ov == 0 && n <= capq && (Tq > -CWQ_INF ? n >= K : Tq == -CWQ_INF);   // uniform over the block
  // the rest of the lists' l and u (one more round trip, every load of it in flight at once)
  const int nst = ok ? min(n, kFwCand) : 0;
  {
    constexpr int B = kFwCand / kFwThreads - 1;
    float tl[B], tu[B];
#pragma unroll
    for (int i = 0; i < B; ++i) {
      const int j = kFwThreads * (i + 1) + tid;
      if (j < nst) {
        tl[i] = cl[base + j];
        tu[i] = cu[base + j];
      }
    }
#pragma unroll
    for (int i = 0; i < B; ++i) {
      const int j = kFwThreads * (i + 1) + tid;
      if (j < nst) {
        s_wl[j] = tl[i];
        s_wu[j] = tu[i];
      }
    }
  }
  float lk = -CWQ_INF, la = 0.f;
  int lr = 0x7fffffff, nx = 0;
  __syncthreads();
  FW_ST(1);
  if (ok) {
    // T2 = the K-th largest l over the whole list (multiplicity counted; -inf with fewer than
    // K candidates): a radix select of the ordered keys (ord_f32), 8 bits a pass -- an LDS
    // histogram of the keys under the prefix so far, one wave finds the digit holding the
    // K-th from the top.  (The list of the first `done` candidates the stream select kept is
    // not needed: every candidate's l is staged.)  Replaces per-wave top-K lists whose serial
    // inserts and merge took ~20 us of a categorize list's rerank
    // (profiles/r05_basic_percall_stamps_runmerge.log).
    {
      FW_ST(9);
      unsigned* s_hist = reinterpret_cast<unsigned*>(s_ml);   // [256] (s_ml is free until the merges)
      unsigned* s_rsel = reinterpret_cast<unsigned*>(s_ma);   // [2]: prefix, rank left
      unsigned pref = 0u, kk = (unsigned)K;
      if (n >= K) {
        for (int pass = 0; pass < 4; ++pass) {
          const int sh = 24 - 8 * pass;
          const unsigned hm = pass == 0 ? 0u : (~0u << (sh + 8));
          if (tid < 256) s_hist[tid] = 0u;
          __syncthreads();
          for (int j = tid; j < n; j += kFwThreads) {
            const unsigned u = ord_f32(j < kFwCand ? s_wl[j] : cl[base + j]);
            if ((u & hm) == pref) atomicAdd(&s_hist[(u >> sh) & 255u], 1u);
          }
          __syncthreads();
          if (wave == 0) {
            // lane L holds bins 255-4L .. 252-4L (lane 0: the top); inclusive prefix over lanes
            unsigned c[4], tot = 0u;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              c[i] = s_hist[255 - 4 * lane - i];
              tot += c[i];
            }
            unsigned inc = tot;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
              const unsigned t = __shfl_up(inc, o, 64);
              if (lane >= o) inc += t;
            }
            const unsigned exc = inc - tot;
            if (exc < kk && kk <= inc) {   // exactly one lane: the counts under the prefix reach kk
              unsigned above = exc;
              int dg = 252 - 4 * lane;
              bool got = false;   // the first bin (from the top) whose running count reaches kk
#pragma unroll
              for (int i = 0; i < 4; ++i) {
                if (!got && above + c[i] >= kk) {
                  dg = 255 - 4 * lane - i;
                  got = true;
                } else if (!got) {
                  above += c[i];
                }
              }
              s_rsel[0] = pref | ((unsigned)dg << sh);
              s_rsel[1] = kk - above;
            }
          }
          __syncthreads();
          pref = s_rsel[0];
          kk = s_rsel[1];
        }
      }
      if (tid == 0) s_T2 = n >= K ? unord_f32(pref) : -CWQ_INF;
      __syncthreads();
      FW_ST(2);
    }
    const float T2 = s_T2;
    // survivors u >= T2, compacted by all waves (their order does not matter: the top-K
    // list below is ordered by (key, row)); a split workgroup takes its slice of the list
    const int per = S > 1 ? (n + S * 64 - 1) / (S * 64) * 64 : n;
    const int jlo = min(n, sidx * per), jhi = min(n, jlo + per);
    for (int j0 = jlo + wave * 64; j0 < jhi; j0 += kFwThreads) {
      const int j = j0 + lane;
      const bool c = j < jhi && (j < kFwCand ? s_wu[j] : cu[base + j]) >= T2;
      const uint64_t bm = __ballot(c);
      int o = 0;
      if (lane == 0 && bm) o = atomicAdd(&s_ns, __popcll(bm));
      o = __shfl(o, 0, 64);
      if (c) s_surv[o + __popcll(bm & ((1ull << lane) - 1))] = j;
    }
    __syncthreads();
    FW_ST(3);
    const int ns = s_ns;
    const f32x16* __restrict__ xg = reinterpret_cast<const f32x16*>(X) + (size_t)(q / kXQ) * NV16 * kXQ + (q % kXQ);
    // survivors per round: `rows` (a multiple of 64: thread t < cnt forms survivor t's key in
    // key wave t / 64, each key wave keeping its own top-K list, merged below); 64 with the
    // exact parent chains (fw_chain_prefixes serves wave 0's lanes)
    const int RR = use_chain ? 64 : rows;
    for (int r0 = 0; r0 < ns; r0 += RR) {
      const int cnt = min(RR, ns - r0);
      if (tid < cnt) {
        const int j = s_surv[r0 + tid];
        s_rr[tid] = j < kFwThreads ? s_wr[j] : crow[base + j];
      }
      __syncthreads();   // s_rr visible; the previous round's partials consumed
      // the survivors' row terms (key threads), in flight with the partials' row loads
      RowMeta md;
      int p = -1, rr = 0;
      if (tid < cnt) {
        rr = s_rr[tid];
        md = meta[rr];
        p = par[rr];
      }
      // FB items per thread per batch: every row load of the batch is in flight before the
      // first partial is formed (one memory round trip per batch, not per item)
      constexpr int FB = 4;
      for (int t0 = tid; t0 < cnt * NV16; t0 += FB * kFwThreads) {
        float4 m4[FB][4];
#pragma unroll
        for (int b = 0; b < FB; ++b) {
          const int t = t0 + b * kFwThreads;
          if (t < cnt * NV16) {
            const int sv = t / NV16, v = t - sv * NV16;
            const float* __restrict__ mr = Mf + (size_t)s_rr[sv] * DP + v * 16;
#pragma unroll
            for (int j = 0; j < 4; ++j) m4[b][j] = *reinterpret_cast<const float4*>(mr + j * 4);
          }
        }
#pragma unroll
        for (int b = 0; b < FB; ++b) {
          const int t = t0 + b * kFwThreads;
          if (t >= cnt * NV16) break;
          const int sv = t / NV16, v = t - sv * NV16;
          const f32x16 xa = xg[(size_t)v * kXQ];
          float part;
#pragma unroll
          for (int j = 0; j < 16; ++j) {
            const float4 t4 = m4[b][j >> 2];
            const float mj = (j & 3) == 0 ? t4.x : (j & 3) == 1 ? t4.y : (j & 3) == 2 ? t4.z : t4.w;
            const float tt = xa[j] - mj;
            part = (j == 0) ? tt * tt : fmaf(tt, tt, part);
          }
          s_part[sv * LDP + v] = part;
        }
      }
      if (r0 == 0) FW_ST(12);
      float pp = 0.f;
      // exact parent chains (bounded internal prefixes): the whole workgroup, every distinct
      // ancestor once (fw_chain_prefixes); the per-lane chain if its table overflows
      const bool chained = use_chain && fw_chain_prefixes(s_chain, xg, chain, DP, tid < cnt && p > 0, p,
                                                          P[(size_t)q * ldP]);
      if (r0 == 0) FW_ST(13);
      if (tid < cnt) {
        pp = p < 0 ? (cat ? CWQ_INF : 0.f)
                   : (use_chain && p > 0 ? (chained ? s_chain.pp[lane] : exact_prefix(X, chain, DP, q, p, P[(size_t)q * ldP]))
                                         : P[(size_t)q * ldP + p]);
      }
      __syncthreads();
      if (wave * 64 < cnt) {
        const bool act = tid < cnt;
        float key = -CWQ_INF, lp = 0.f;
        int rid = 0x7fffffff;
        if (act) {
          float acc = 0.f;
          const float* pr = s_part + tid * LDP;
          int v = 0;
          for (; v + 8 <= NV16; v += 8) {   // 8 reads in flight, then the adds in slice order
            float t8[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) t8[u] = pr[v + u];
#pragma unroll
            for (int u = 0; u < 8; ++u) acc += t8[u];
          }
          for (; v < NV16; ++v) acc += pr[v];
          const float S = md.iv * acc;
          lp = -0.5f * (md.logdet + dconst + S);
          key = cat ? fminf(pp, lp) : fmaf(pp, md.invL, md.cw * lp);
          rid = seg_base + rr;
          ++nx;
        }
        // only keys that beat the list's K-th entry can enter (insertions are serial); the
        // wave's first round fills its empty list by a sort
        if (r0 == 0 && !nopf) {
          lk = key == key ? key : -CWQ_INF;   // a NaN key never enters (as the insertions)
          la = lp;
          lr = lk == -CWQ_INF ? 0x7fffffff : rid;
          wave_sort64<true>(lk, lr, la, lane, cat);
        }
        // the list order is list_before<cat> (categorize: equal keys by own lp ascending)
        const float tk = rl_f2(lk, K - 1), ta = rl_f2(la, K - 1);
        const int tr = __builtin_amdgcn_readlane(lr, K - 1);
        uint64_t mask = __ballot(act && r0 != 0 && (nopf || entry_before(key, lp, rid, tk, ta, tr, cat)));
        if (nopf && r0 == 0) mask = __ballot(act);
        while (mask) {
          const int b = __builtin_ctzll(mask);
          mask &= mask - 1;
          const float ck = rl_f2(key, b), ca = rl_f2(lp, b);
          const int cr = __builtin_amdgcn_readlane(rid, b);
          const bool prec = entry_before(lk, la, lr, ck, ca, cr, cat);
          const int pos = __popcll(__ballot(prec));
          if (pos < K) {
            const float sk = __int_as_float(wave_shr1(__float_as_int(lk)));
            const float sa = __int_as_float(wave_shr1(__float_as_int(la)));
            const int sr = wave_shr1(lr);
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
    }
    // the key waves' lists -> wave 0's (same insertion; a no-op with one key wave)
    FW_ST(4);
    const int nkw = ns > 0 ? (min(RR, ns) + 63) / 64 : 0;
    if (nkw > 1) {
      __syncthreads();
      if (wave > 0 && wave < nkw) {
        s_ml[tid] = lane < K ? lk : -CWQ_INF;
        s_ma[tid] = lane < K ? la : CWQ_INF;
        s_mr[tid] = lane < K ? lr : 0x7fffffff;
      }
      __syncthreads();
      if (wave == 0) {
        if (lane >= K) {
          lk = -CWQ_INF;
          la = CWQ_INF;
          lr = 0x7fffffff;
        }
        for (int w = 1; w < nkw; ++w) {
          const float key = s_ml[w * 64 + lane], lp = s_ma[w * 64 + lane];
          const int rid = s_mr[w * 64 + lane];
          if (cat) {   // (as the split merge below)
            list64_merge_aux(lk, la, lr, lane, key, lp, rid, true);
            continue;
          }
          const float tk = rl_f2(lk, K - 1), ta = rl_f2(la, K - 1);
          const int tr = __builtin_amdgcn_readlane(lr, K - 1);
          uint64_t mask = __ballot(rid != 0x7fffffff && entry_before(key, lp, rid, tk, ta, tr, cat));
          while (mask) {
            const int bb = __builtin_ctzll(mask);
            mask &= mask - 1;
            list64_insert_aux(lk, la, lr, lane, rl_f2(key, bb), rl_f2(lp, bb), __builtin_amdgcn_readlane(rid, bb), K,
                              cat);
          }
        }
      }
    }
  }
  for (int off = 32; off > 0; off >>= 1) nx += __shfl_xor(nx, off, 64);
  if (lane == 0 && nx) atomicAdd(&s_nx, nx);
  __syncthreads();
  FW_ST(5);
  if (wave != 0) return;
  nx = s_nx;
  if (S > 1) {
    // split: this workgroup's list out; the last of the query's S workgroups (release /
    // acquire at agent scope around the arrival count) merges the others' into its own
    const size_t so = ((size_t)q * S + sidx) * 64 + lane;
    fx.sk[so] = lk;
    fx.sa[so] = la;
    fx.sr[so] = lr;
    if (lane == 0 && nx) atomicAdd(&n_exact[q], nx);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    int last = 0;
    if (lane == 0) last = atomicAdd(fx.sctr ? &fx.sctr[q] : &ok_flag[q], 1) == S - 1;
    last = __shfl(last, 0, 64);
    if (!last) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    FW_ST(6);
    if (ok) {
      // the other workgroups' lists, 8 in flight per round trip, inserted into this one
      if (lane >= K) {
        lk = -CWQ_INF;
        la = CWQ_INF;
        lr = 0x7fffffff;
      }
      for (int w0 = 0; w0 < S; w0 += 8) {
        float mk[8], ma[8];
        int mr[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int w = w0 + u;
          const size_t o = ((size_t)q * S + (w < S ? w : sidx)) * 64 + lane;
          const bool use = w < S && w != sidx && lane < K;
          mk[u] = use ? __builtin_nontemporal_load(&fx.sk[o]) : -CWQ_INF;
          ma[u] = use ? __builtin_nontemporal_load(&fx.sa[o]) : CWQ_INF;
          mr[u] = use ? __builtin_nontemporal_load(&fx.sr[o]) : 0x7fffffff;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          // categorize lists (ties: most entries enter): a bitonic merge per list; Fast lists:
          // only entries that beat the K-th enter, a few serial inserts (a bitonic merge per
          // list, ~1.1 us, made C3's per-call rerank 36 -> 78 us:
          // profiles/r05_basic_percall_stamps_radix_s32.log, r05_bench_v2.log)
          if (cat) {
            if (w0 + u < S && w0 + u != sidx) list64_merge_aux(lk, la, lr, lane, mk[u], ma[u], mr[u], true);
            continue;
          }
          const float tk = rl_f2(lk, K - 1), ta = rl_f2(la, K - 1);
          const int tr = __builtin_amdgcn_readlane(lr, K - 1);
          uint64_t mask = __ballot(mr[u] != 0x7fffffff && entry_before(mk[u], ma[u], mr[u], tk, ta, tr, cat));
          while (mask) {
            const int bb = __builtin_ctzll(mask);
            mask &= mask - 1;
            list64_insert_aux(lk, la, lr, lane, rl_f2(mk[u], bb), rl_f2(ma[u], bb), __builtin_amdgcn_readlane(mr[u], bb),
                              K, cat);
          }
        }
      }
    }
    nx = __hip_atomic_load(&n_exact[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    FW_ST(7);
  }
  if (fx.ids) {
    // merge_expand_kernel's expansion of the (already sorted) top-K rows, in place
    if (!ok) {
      lk = -CWQ_INF;
      lr = 0x7fffffff;
    }
    const bool valid = lane < K && lk != -CWQ_INF && lr != 0x7fffffff;
    const uint64_t vm = __ballot(valid);
    const int nvalid = (~vm) ? __builtin_ctzll(~vm) : 64;
    int64_t s0 = 0;
    int cnt = 0;
    if (lane < nvalid) {
      s0 = fx.sent_ptr[lr];
      cnt = (int)(fx.sent_ptr[lr + 1] - s0);
    }
    int off = cnt;   // inclusive scan
    for (int dd = 1; dd < 64; dd <<= 1) {
      const int o = __shfl_up(off, dd, 64);
      if (lane >= dd) off += o;
    }
    const int total = __shfl(off, 63, 64);
    off -= cnt;
    const int k = fx.k;
    for (int j = 0; j < cnt && off + j < k; ++j) {
      fx.ids[(size_t)q * k + off + j] = fx.sent_ids[s0 + j];
      if (fx.scores) fx.scores[(size_t)q * k + off + j] = lk;
    }
    for (int t = total + lane; t < k; t += kWave) {
      fx.ids[(size_t)q * k + t] = -1;
      if (fx.scores) fx.scores[(size_t)q * k + t] = -CWQ_INF;
    }
    if (lane == 0) {
      fx.hflags[q] = n;
      fx.hflags[nq + q] = ok ? 1 : 0;
      fx.hflags[2 * nq + q] = nx;
    }
    return;
  }
  FW_ST(8);
  if (lane < K) {
    const size_t o = (size_t)q * lstride + lane;
    pkey[o] = ok ? lk : -CWQ_INF;
    paux[o] = la;
    prow[o] = ok ? lr : 0x7fffffff;
  }
  if (lane == 0) {
    ok_flag[q] = ok ? 1 : 0;
    if (n_exact) n_exact[q] = nx;
  }
}

// survivors per rerank round of final_wide_kernel: a multiple of 64 (<= kFwMaxRows) whose
// partials fit the dynamic LDS budget next to the survivor list; 0: the kernel cannot run
int final_wide_rows(int DP, int capq) {
  const int64_t avail = (int64_t)kFwDynMax - (int64_t)capq * 4;
  const int64_t r = avail > 0 ? avail / ((int64_t)(DP / 16 + 1) * 4) / 64 * 64 : 0;
  return (int)std::min<int64_t>(r, kFwMaxRows);
}
size_t final_wide_lds(int DP, int capq) {
  const int rows = final_wide_rows(DP, capq);
  return rows > 0 ? ((size_t)rows * (DP / 16 + 1) + (size_t)capq) * 4 : SIZE_MAX;
}

hipError_t launch_final(const float* X, const float* Mf, int DP, int nq, int K, int capq, const int* qcnt,
                        const int* qover, const int* crow, const float* cu, const float* cl, const float* T,
                        int64_t ldT, const RowMeta* meta, const int* par, const float* P, int64_t ldP, int seg_base,
                        float* pkey, float* paux, int* prow, int64_t lstride, int* ok_flag, int* n_exact,
                        const float* lkb, const int* lrb, const int* done, const IntChain* chain, int cat,
                        float dconst, hipStream_t s, const FwExpand* fx) {
  const IntChain ch = chain ? *chain : IntChain{nullptr, nullptr, nullptr, nullptr, nullptr};
  const FwExpand fe = fx ? *fx : FwExpand{nullptr, nullptr, nullptr, nullptr, 0, nullptr};
  const char* we = getenv("CWQ_FINAL_WIDE");   // largest nq for the workgroup-per-query form
  const int wide_max = we && *we ? atoi(we) : kFinalWideMaxQ;
  const size_t lds = final_wide_lds(DP, capq);
  if ((fx || nq <= wide_max) && lds <= (size_t)kFwDynMax) {
    if (fe.split > 1 && (!fe.sk || !fe.sa || !fe.sr || !(fe.sctr || ok_flag) || !n_exact)) return hipErrorInvalidValue;
    const unsigned grid = (unsigned)nq * (unsigned)(fe.split > 1 ? fe.split : 1);
    hipLaunchKernelGGL(final_wide_kernel, dim3(grid), dim3(kFwThreads), lds, s, X, Mf, DP, nq, K, capq, qcnt,
                       qover, crow, cu, cl, T, ldT, meta, par, P, ldP, seg_base, pkey, paux, prow, lstride, ok_flag,
                       n_exact, lkb, lrb, done, ch, chain ? 1 : 0, cat, dconst, fe,
                       getenv("CWQ_FW_ROWS") ? std::min(final_wide_rows(DP, capq), atoi(getenv("CWQ_FW_ROWS")))
                                             : final_wide_rows(DP, capq),
                       getenv("CWQ_FW_NOPF") ? 1 : 0);
    return hipGetLastError();
  }
  if (fx) return hipErrorInvalidValue;   // the fused tail exists in the workgroup-per-query form only
  hipLaunchKernelGGL(final_kernel, dim3((unsigned)((nq + 3) / 4)), dim3(256), 0, s, X, Mf, DP, nq, K, capq, qcnt, qover,
                     crow, cu, cl, T, ldT, meta, par, P, ldP, seg_base, pkey, paux, prow, lstride, ok_flag, n_exact,
                     lkb, lrb, done, ch, chain ? 1 : 0, cat, dconst);
  return hipGetLastError();
}

}  // namespace cwq
