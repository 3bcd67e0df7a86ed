// libcwq: small-batch "Cobweb Fast" filter (nq <= 64) -- the reference harness's mode,
// one cobweb_predict_fast(q, k) call at a time (benchmark_utils.py:801-805;
// CobwebWrapper.py:210-265).  Results are EXACT, as with the batch filter
// (cwq_mfma.hip): bf16-MFMA bounds select candidates, final_kernel scores them with the
// scan's fp32 arithmetic.
//
// At a few queries per call the batch filter's 256-query MFMA tiles are mostly padding
// and its pipeline (sample pass, select, five filter launches with bucket/tighten) costs
// a fixed ~0.6 ms.  Here the bound is the same but the pass is a single stream over the
// bf16 row panel (HBM-bound: 2*DPB + 32 bytes per isotropic row):
//
//   probe   (stream_kernel<1>): every `probe_stride`-th 16-row group; per query the max
//           lower bound l of the group goes to lb[q][g]; select_kernel (cwq_mfma.hip)
//           takes T0[q] = K-th largest of those maxima, a lower bound of the K-th
//           largest key (K distinct groups each hold a row with key >= l >= T0).
//   filter  (stream_kernel<0>): every isotropic row; (q, row) is a candidate iff
//           u >= T[q] (every true top-K row has u >= key >= tau_K >= T) and goes straight
//           to its query's candidate list (no record/bucket pass).  Optionally
//           (live_every > 0, CWQ_STREAM_LIVE) T rises during the pass: each candidate's l
//           is folded into Tb[row mod K][q] (atomicMax), the candidate's lane publishes
//           Tlive[q] = max(Tlive, min_b Tb[b][q]) -- K disjoint row blocks each holding a
//           row with key >= l >= that min, so still <= tau_K -- and waves raise T to
//           Tlive every live_every groups.  Measured at C3: 3x fewer candidates but a
//           slower pass (nq=1 276 -> 301 us, nq=64 378 -> 573 us), so it is off.
//   final_kernel (cwq_mfma.hip) then takes T2 = K-th largest l among the candidates and
//   computes exact keys for those with u >= T2.
//
// CDNA4 mapping: persistent 512-thread workgroups (8 waves); the queries' bf16 hi parts
// are staged once per workgroup into LDS in MFMA-fragment order (one conflict-free
// ds_read_b128 per fragment); a wave owns a 16-row group at a time: its 24 (D=768)
// A fragments (16 B per lane, the row panel is row-major [row][DPB]) are loaded straight
// into registers -- each row is used by one wave only, so there is nothing to share
// through LDS -- and v_mfma_f32_16x16x32_bf16 (rows x 16 queries) runs once per fragment
// and query block.  The MFMA work is ~5% of the pass time at 64 queries; the pass is
// bound by HBM (24 KB in flight per wave, 192 KB per CU).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <algorithm>

#include "cwq_internal.h"

namespace cwq {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CWQ_INF __builtin_inff()

constexpr int SK_WAVES = 8;
constexpr int SK_MAXQB = kStreamMaxQ / 16;   // query blocks of 16
constexpr int SK_CH = 8;                     // K fragments per chunk (8 x 32 = 256 dims)
// float <-> int order-preserving map for atomicMax on floats
__device__ __forceinline__ int f2ord(float f) {
  const int i = __float_as_int(f);
  return i >= 0 ? i : i ^ 0x7fffffff;
}
__device__ __forceinline__ float ord2f(int i) { return __int_as_float(i >= 0 ? i : i ^ 0x7fffffff); }

// MQB: query blocks the instantiation holds (1: nq <= 16, the per-call case, fewer live
// registers; SK_MAXQB otherwise)
template <int MODE, int MQB>
__global__ __launch_bounds__(512) void stream_kernel(const StreamArgs a) {
  extern __shared__ __attribute__((aligned(16))) char sq[];   // [nqb][nk][64 lanes][16 B]
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int nk = a.DPB / 32;
  const int nqb = a.nqb;
  // ---- stage the queries' bf16 fragments (B operand: k = 8*(l>>4).., query = l&15) ----
  for (int f = threadIdx.x; f < nqb * nk * 64; f += blockDim.x) {
    const int l = f & 63, ks = (f >> 6) % nk, qb = (f >> 6) / nk;
    const int q = qb * 16 + (l & 15);
    const uint4 v = *reinterpret_cast<const uint4*>(a.Xb + ((size_t)q * a.DPB + ks * 32 + 8 * (l >> 4)));
    *reinterpret_cast<uint4*>(sq + (size_t)f * 16) = v;
  }
  // per-lane query terms for the lane's column (query qb*16 + (lane & 15))
  float4 qi[MQB];
  float Tq[MQB];
  bool qok[MQB];
#pragma unroll
  for (int qb = 0; qb < MQB; ++qb) {
    const int q = qb * 16 + (lane & 15);
    qok[qb] = qb < nqb && q < a.nq;
    qi[qb] = qok[qb] ? a.qinfo[q] : make_float4(0.f, 0.f, 0.f, 0.f);
    Tq[qb] = CWQ_INF;
    if (MODE == 0 && qok[qb]) {
      Tq[qb] = a.T0[(size_t)q * a.ldT0 + (a.K - 1)];
      if (blockIdx.x == 0 && wave == 0 && lane < 16) a.T[q] = Tq[qb];   // for final_kernel
    }
  }
  __syncthreads();
  const int64_t ngroups = MODE == 1 ? a.n_probe : (int64_t)((a.nrows + 15) >> 4);
  const int64_t gstride = (int64_t)gridDim.x * SK_WAVES;
  const int c16 = lane >> 4, r16 = lane & 15;
  // probe: max of the lower bounds per query over the current group
  float pmax[MQB];
#pragma unroll
  for (int qb = 0; qb < MQB; ++qb) pmax[qb] = -CWQ_INF;
  // parent-prefix cache: pi = P[q][par] * invL changes only with the parent (flat trees:
  // one load per wave)
  int cpar = -3;
  float cP[MQB], cPh[MQB];   // lower / upper bound of the parent prefix (equal when exact)
#pragma unroll
  for (int qb = 0; qb < MQB; ++qb) cP[qb] = cPh[qb] = 0.f;
  const float* Pu = a.Phi ? a.Phi : a.P;
  auto panel = [&](int64_t gi) {
    const int64_t grp = MODE == 1 ? gi * a.probe_stride : gi;
    return reinterpret_cast<const char*>(a.Mb) + ((size_t)(grp * 16 + r16) * a.DPB + 8 * c16) * 2;
  };
  // K runs in chunks of SK_CH fragments (16 B per lane each: row r0 + (lane & 15),
  // k = ks*32 + 8*(lane >> 4)); the next chunk -- after the last one, the first chunk of
  // the wave's next group -- is in flight during this chunk's MFMAs and the epilogue.
  bf16x8 cur[SK_CH], nxt[SK_CH];
  // row terms of the rows this lane's accumulator columns hold (r0 + 4*c16 + j), one group
  // ahead like the panel chunks (at D = 256 a group is one chunk, so a load at the group's
  // start would put its latency on every group)
  constexpr bool PRE_RF = MQB == 1;
  RowF rfn[4];
  auto load_rf = [&](int64_t g) {
    const int64_t r0n = (MODE == 1 ? g * a.probe_stride : g) * 16;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t r = r0n + 4 * c16 + j;
      rfn[j] = r < a.nrows ? a.rf[r] : RowF{-CWQ_INF, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, -2};
    }
  };
  int64_t gi = (int64_t)blockIdx.x * SK_WAVES + wave;
  if (gi < ngroups) {
    const char* src = panel(gi);
#pragma unroll
    for (int i = 0; i < SK_CH; ++i)
      if (i < nk) cur[i] = *reinterpret_cast<const bf16x8*>(src + i * 64);
    if (PRE_RF) load_rf(gi);
  }
  int it = 0;
  for (; gi < ngroups; gi += gstride, ++it) {
    // live threshold every `live_every` groups, loaded now and used in the epilogue (the
    // load is in flight with the row panel): T = max(T, Tlive[q])
    const bool live = MODE == 0 && a.live_every > 0 && it % a.live_every == a.live_every - 1;
    int tlive[MQB];
#pragma unroll
    for (int qb = 0; qb < MQB; ++qb) tlive[qb] = (live && qok[qb]) ? a.Tlive[qb * 16 + r16] : 0x80000000;
    const int64_t grp = MODE == 1 ? gi * a.probe_stride : gi;
    const int64_t r0 = grp * 16;   // < nrows rounded up to 16 (probe: grp < ngroups of the panel)
    RowF rf[4];
    if (!PRE_RF) load_rf(gi);   // registers too tight for a group-ahead copy
#pragma unroll
    for (int j = 0; j < 4; ++j) rf[j] = rfn[j];   // PRE_RF: loaded with the group's first chunk
    const char* src = panel(gi);
    const int64_t gn = gi + gstride;
    const char* srcn = gn < ngroups ? panel(gn) : nullptr;
    f32x4 acc[MQB];
#pragma unroll
    for (int qb = 0; qb < MQB; ++qb) acc[qb] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int c0 = 0; c0 < nk; c0 += SK_CH) {
      if (c0 + SK_CH < nk) {
#pragma unroll
        for (int i = 0; i < SK_CH; ++i)
          if (c0 + SK_CH + i < nk) nxt[i] = *reinterpret_cast<const bf16x8*>(src + (c0 + SK_CH + i) * 64);
      } else if (srcn) {
#pragma unroll
        for (int i = 0; i < SK_CH; ++i)
          if (i < nk) nxt[i] = *reinterpret_cast<const bf16x8*>(srcn + i * 64);
        if (PRE_RF) load_rf(gn);   // the next group's row terms fly with its first chunk
      }
#pragma unroll
      for (int qb = 0; qb < MQB; ++qb) {
        if (qb >= nqb) break;
        const char* qs = sq + (((size_t)qb * nk + c0) * 64 + lane) * 16;
#pragma unroll
        for (int i = 0; i < SK_CH; ++i)
          if (c0 + i < nk)
            acc[qb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cur[i], *reinterpret_cast<const bf16x8*>(qs + i * 1024),
                                                              acc[qb], 0, 0, 0);
      }
#pragma unroll
      for (int i = 0; i < SK_CH; ++i) cur[i] = nxt[i];
    }
    if (live) {
#pragma unroll
      for (int qb = 0; qb < MQB; ++qb) Tq[qb] = fmaxf(Tq[qb], ord2f(tlive[qb]));
    }
    // ---- epilogue: rigorous bounds per (row, query); acc[qb][j] = dot of row
    // r0 + 4*c16 + j with query qb*16 + (lane & 15)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const bool rok = rf[j].par >= -1;
      if (rok && rf[j].par != cpar) {
        cpar = rf[j].par;
#pragma unroll
        for (int qb = 0; qb < MQB; ++qb) {
          const size_t o = (size_t)(qb * 16 + r16) * a.ldP + cpar;
          cP[qb] = (qok[qb] && cpar >= 0) ? a.P[o] : 0.f;
          cPh[qb] = (qok[qb] && cpar >= 0) ? Pu[o] : 0.f;
        }
      }
#pragma unroll
      for (int qb = 0; qb < MQB; ++qb) {
        if (qb >= nqb) break;
        if (!rok || !qok[qb]) continue;
        float u, l;
        fg_bounds2(acc[qb][j], 0x1p-23f * fabsf(acc[qb][j]), qi[qb], rf[j], cPh[qb] * rf[j].invL,
                   cP[qb] * rf[j].invL, a.eps_n, a.slack, u, l);
        if (MODE == 1) {
          pmax[qb] = fmaxf(pmax[qb], l);
        } else if (u >= Tq[qb]) {
          const int q = qb * 16 + r16;
          // live threshold: fold l into its row block, then publish min over the blocks
          // (rare: ~K x a few candidates per query after the first groups)
          if (a.live_every > 0) {
            const int64_t row = r0 + 4 * c16 + j;
            atomicMax(&a.Tb[(size_t)(row % a.K) * a.nq + q], f2ord(l));
            int m = 0x7fffffff;
            for (int b = 0; b < a.K; ++b)
              m = min(m, __hip_atomic_load(&a.Tb[(size_t)b * a.nq + q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            if (m != f2ord(-CWQ_INF)) atomicMax(&a.Tlive[q], m);
          }
          const int slot = atomicAdd(&a.qcnt[q], 1);
          if (slot < a.capq) {
            const size_t o = (size_t)q * a.capq + slot;
            a.crow[o] = (int)(r0 + 4 * c16 + j);
            a.cu[o] = u;
            a.cl[o] = l;
          } else {
            a.qover[q] = 1;
          }
        }
      }
    }
    if (MODE == 1) {   // the group's max lower bound per query -> lb[q][gi]
#pragma unroll
      for (int qb = 0; qb < MQB; ++qb) {
        float m = fmaxf(pmax[qb], __shfl_xor(pmax[qb], 16, 64));
        m = fmaxf(m, __shfl_xor(m, 32, 64));
        if (lane < 16 && qok[qb]) a.lb[(size_t)(qb * 16 + lane) * a.ldlb + gi] = m;
        pmax[qb] = -CWQ_INF;
      }
    }
  }
}

hipError_t launch_stream(const StreamArgs& a, int mode, int n_wg, hipStream_t s) {
  const int nk = a.DPB / 32;
  const size_t lds = stream_lds_bytes(a.nqb, a.DPB);
  if (a.nq <= 0 || a.nqb * 16 < a.nq || a.nqb > SK_MAXQB || a.DPB % 32 || a.K < 1 || a.K > 64 ||
      lds > (size_t)kStreamMaxLds)
    return hipErrorInvalidValue;
  static bool attr = false;   // dynamic LDS above the 64 KiB default
  if (!attr) {
    const void* fns[4] = {reinterpret_cast<const void*>(&stream_kernel<0, 1>),
                          reinterpret_cast<const void*>(&stream_kernel<0, SK_MAXQB>),
                          reinterpret_cast<const void*>(&stream_kernel<1, 1>),
                          reinterpret_cast<const void*>(&stream_kernel<1, SK_MAXQB>)};
    for (const void* f : fns) {
      const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, kStreamMaxLds);
      if (e != hipSuccess) return e;
    }
    attr = true;
  }
  const dim3 grid((unsigned)n_wg), block(64 * SK_WAVES);
  if (a.nqb == 1) {
    if (mode == 1) hipLaunchKernelGGL((stream_kernel<1, 1>), grid, block, lds, s, a);
    else hipLaunchKernelGGL((stream_kernel<0, 1>), grid, block, lds, s, a);
  } else {
    if (mode == 1) hipLaunchKernelGGL((stream_kernel<1, SK_MAXQB>), grid, block, lds, s, a);
    else hipLaunchKernelGGL((stream_kernel<0, SK_MAXQB>), grid, block, lds, s, a);
  }
  return hipGetLastError();
}

// Tb[b][q] and Tlive[q] = ordered(-inf) for the filter's atomicMax (Tlive follows Tb)
__global__ void stream_init_kernel(int* Tb, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) Tb[i] = f2ord(-CWQ_INF);
}

hipError_t launch_stream_init(int* Tb, int n, hipStream_t s) {
  hipLaunchKernelGGL(stream_init_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, Tb, n);
  return hipGetLastError();
}

}  // namespace cwq
