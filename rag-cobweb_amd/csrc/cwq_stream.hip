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
// and query block.  Chunks of 8 fragments alternate between two register buffers (the
// next chunk's 8 KB per wave in flight while the current one is multiplied), so the pass
// is bound by HBM: C3 nq=1 272 us (5.8 TB/s), nq=64 297 us (was 389 us with one buffer
// and a register copy per chunk that drained every load).
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
constexpr int SK_CH = kStreamChunk;         // K fragments per chunk (8 x 32 = 256 dims)
// float <-> int order-preserving map for atomicMax on floats
__device__ __forceinline__ int f2ord(float f) {
  const int i = __float_as_int(f);
  return i >= 0 ? i : i ^ 0x7fffffff;
}
__device__ __forceinline__ float ord2f(int i) { return __int_as_float(i >= 0 ? i : i ^ 0x7fffffff); }

// MODE 0: filter (candidates), 1: threshold probe, 2: the path-sum dots of the internal
// rows for a few queries (run_internal_bounds' small-batch form: rows x <= 64 queries
// streamed once instead of 256-query fgemm tiles that are mostly padding).
// MQB: query blocks the instantiation holds (1: nq <= 16, the per-call case, fewer live
// registers; SK_MAXQB otherwise)
template <int MODE, int MQB>
__global__ __launch_bounds__(512) void stream_kernel(const StreamArgs a) {
  extern __shared__ __attribute__((aligned(16))) char sq[];   // [nqb][nk][64 lanes][16 B]
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int nk = a.DPB / 32;
  const int nkp = (nk + SK_CH - 1) / SK_CH * SK_CH;   // K padded to whole chunks (zero fragments)
  const int nqb = a.nqb;
  // ---- stage the queries' bf16 fragments (B operand: k = 8*(l>>4).., query = l&15) ----
  for (int f = threadIdx.x; f < nqb * nkp * 64; f += blockDim.x) {
    const int l = f & 63, ks = (f >> 6) % nkp, qb = (f >> 6) / nkp;
    const int q = qb * 16 + (l & 15);
    const uint4 v = ks < nk ? *reinterpret_cast<const uint4*>(a.Xb + ((size_t)q * a.DPB + ks * 32 + 8 * (l >> 4)))
                            : make_uint4(0u, 0u, 0u, 0u);
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
  float proot[MQB];   // MODE 2: the root's exact prefix per query (fgemm_kernel<2>'s formula)
#pragma unroll
  for (int qb = 0; qb < MQB; ++qb)
    proot[qb] = (MODE == 2 && qok[qb]) ? a.root_w * (-0.5f * (a.root_ld + a.Sroot[qb * 16 + (lane & 15)])) : 0.f;
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
  // row terms of the rows this lane's accumulator columns hold (r0 + 4*c16 + j)
  auto load_rf = [&](RowF (&dst)[4], int64_t g) {
    const int64_t r0n = (MODE == 1 ? g * a.probe_stride : g) * 16;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t r = r0n + 4 * c16 + j;
      dst[j] = r < a.nrows ? a.rf[r] : RowF{-CWQ_INF, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, -2};
    }
  };
  int64_t gi = (int64_t)blockIdx.x * SK_WAVES + wave;
  if (gi >= ngroups) return;   // no barrier follows
  // K runs in chunks of SK_CH fragments (16 B per lane each: row r0 + (lane & 15),
  // k = ks*32 + 8*(lane >> 4)) over the wave's whole (group, chunk) sequence.  Two
  // register buffers alternate chunk by chunk: the loads of the next chunk (after a
  // group's last chunk, the first chunk of the wave's next group) go into one while the
  // MFMAs consume the other.  No buffer is ever copied: a copy of registers whose loads
  // are still in flight makes the compiler wait for every load (vmcnt(0)) before the
  // chunk's MFMAs, which left one chunk in flight per wave and the pass at 0.67 of HBM.
  // For the same reason nothing between a chunk's loads and its MFMAs is conditional:
  // a partial last chunk re-reads its last fragment (a cache hit) and multiplies the
  // extra copies by the zero query fragments of the LDS padding, and the wave's last
  // step re-reads its current chunk.
  bf16x8 bA[SK_CH], bB[SK_CH];
  auto issue = [&](bf16x8 (&b)[SK_CH], const char* p, int nfr) {
#pragma unroll
    for (int i = 0; i < SK_CH; ++i) b[i] = *reinterpret_cast<const bf16x8*>(p + min(i, nfr - 1) * 64);
  };
  f32x4 acc[MQB];
#pragma unroll
  for (int qb = 0; qb < MQB; ++qb) acc[qb] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto mma = [&](const bf16x8 (&b)[SK_CH], int c0) {
#pragma unroll
    for (int qb = 0; qb < MQB; ++qb) {
      if (qb >= nqb) break;
      const char* qs = sq + (((size_t)qb * nkp + c0) * 64 + lane) * 16;
#pragma unroll
      for (int i = 0; i < SK_CH; ++i)
        acc[qb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[i], *reinterpret_cast<const bf16x8*>(qs + i * 1024),
                                                          acc[qb], 0, 0, 0);
    }
  };
  issue(bA, panel(gi), min(SK_CH, nk));
  // the group's row terms are loaded at its start and used at its end (in flight with
  // its chunks)
  RowF rf[4];
  load_rf(rf, gi);
  int tlive[MQB];
  bool live = false;
  auto load_live = [&](int it) {
    // live threshold every `live_every` groups, loaded at the group's start and used in
    // its epilogue: T = max(T, Tlive[q])
    live = MODE == 0 && a.live_every > 0 && it % a.live_every == a.live_every - 1;
#pragma unroll
    for (int qb = 0; qb < MQB; ++qb) tlive[qb] = (live && qok[qb]) ? a.Tlive[qb * 16 + r16] : 0x80000000;
  };
  int it = 0;
  load_live(it);
  int c0 = 0;
  // one chunk: the next chunk's loads go into `oth`, the MFMAs consume `cur`; at a
  // group's last chunk the epilogue runs and the wave moves to its next group.  Returns
  // false after the wave's last group.  The loop below alternates step(bA, bB) and
  // step(bB, bA), so which buffer is in flight is static in the code.
  auto step = [&](const bf16x8 (&cur)[SK_CH], bf16x8 (&oth)[SK_CH]) -> bool {
    int64_t gn = gi;
    int cn = c0 + SK_CH;
    if (cn >= nk) {
      gn = gi + gstride;
      cn = 0;
    }
    const bool more = gn < ngroups;
    issue(oth, more ? panel(gn) + cn * 64 : panel(gi) + c0 * 64, more ? min(SK_CH, nk - cn) : min(SK_CH, nk - c0));
    mma(cur, c0);
    if (cn != 0) {
      c0 = cn;
      return true;
    }
    // ---- group gi done.  Epilogue: rigorous bounds per (row, query); acc[qb][j] = dot
    // of row r0 + 4*c16 + j with query qb*16 + (lane & 15)
    const int64_t r0 = (MODE == 1 ? gi * a.probe_stride : gi) * 16;
    if (live) {
#pragma unroll
      for (int qb = 0; qb < MQB; ++qb) Tq[qb] = fmaxf(Tq[qb], ord2f(tlive[qb]));
    }
    if (MODE == 2) {
      // path-sum dots, node-major: row r0 + 4 c16 + j is internal node row_id[r]; the
      // root's line gets its exact prefix (run_internal_bounds' fgemm_kernel<2> output)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t r = r0 + 4 * c16 + j;
        const int rid = (rf[j].par >= -1 && r < a.nrows) ? a.row_id[r] : -1;
        if (rid < 0) continue;
#pragma unroll
        for (int qb = 0; qb < MQB; ++qb) {
          if (qb >= nqb) break;
          if (!qok[qb]) continue;
          a.pout[(size_t)rid * a.ldpout + qb * 16 + r16] = rf[j].par < 0 ? proot[qb] : acc[qb][j];
        }
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (MODE == 2) break;
      const bool rok = rf[j].par >= -1;
      if (rok && rf[j].par != cpar) {
        cpar = rf[j].par;
#pragma unroll
        for (int qb = 0; qb < MQB; ++qb) {
          cP[qb] = cPh[qb] = 0.f;
          if (!qok[qb] || cpar < 0) continue;
          if (a.pb.dot) {
            pathb_bounds(a.pb, qb * 16 + r16, cpar, cP[qb], cPh[qb]);
          } else {
            const size_t o = pidx(a.ldP, a.pT, qb * 16 + r16, cpar);
            cP[qb] = a.P[o];
            cPh[qb] = Pu[o];
          }
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
    if (!more) return false;
    gi = gn;
    c0 = 0;
    load_rf(rf, gi);
    load_live(++it);
#pragma unroll
    for (int qb = 0; qb < MQB; ++qb) acc[qb] = f32x4{0.f, 0.f, 0.f, 0.f};
    return true;
  };
  while (step(bA, bB) && step(bB, bA)) {
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
    const void* fns[6] = {reinterpret_cast<const void*>(&stream_kernel<0, 1>),
                          reinterpret_cast<const void*>(&stream_kernel<0, SK_MAXQB>),
                          reinterpret_cast<const void*>(&stream_kernel<1, 1>),
                          reinterpret_cast<const void*>(&stream_kernel<1, SK_MAXQB>),
                          reinterpret_cast<const void*>(&stream_kernel<2, 1>),
                          reinterpret_cast<const void*>(&stream_kernel<2, SK_MAXQB>)};
    for (const void* f : fns) {
      const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, kStreamMaxLds);
      if (e != hipSuccess) return e;
    }
    attr = true;
  }
  const dim3 grid((unsigned)n_wg), block(64 * SK_WAVES);
  if (a.nqb == 1) {
    if (mode == 1) hipLaunchKernelGGL((stream_kernel<1, 1>), grid, block, lds, s, a);
    else if (mode == 2) hipLaunchKernelGGL((stream_kernel<2, 1>), grid, block, lds, s, a);
    else hipLaunchKernelGGL((stream_kernel<0, 1>), grid, block, lds, s, a);
  } else {
    if (mode == 1) hipLaunchKernelGGL((stream_kernel<1, SK_MAXQB>), grid, block, lds, s, a);
    else if (mode == 2) hipLaunchKernelGGL((stream_kernel<2, SK_MAXQB>), grid, block, lds, s, a);
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
