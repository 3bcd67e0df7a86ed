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
#include <type_traits>

#include "cwq_internal.h"

namespace cwq {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

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
// registers; SK_MAXQB otherwise).  I8 (filter only): int8 operands (launch_rows_i8) and
// v_mfma_i32_16x16x64_i8 -- half the bytes of the bf16 panel per row.  A 16-B fragment
// then holds 64 dims and the products are exact int32 sums; dot = acc * (s_x * s_r).  Both
// operands are loaded with the same byte -> (lane, element) map, so the instruction's
// internal k order inside a fragment does not matter for the dot product.
// CH: K fragments per load chunk (8; 12 for int8 rows of 12 fragments, D = 768, so that no
// chunk is partial and every wave keeps a whole chunk of HBM loads in flight).
// MINB: workgroups per CU the register allocation must allow (2: <= 128 VGPRs, twice the
// waves in flight per CU).
template <int MODE, int MQB, bool I8 = false, int CH = SK_CH, bool NT = false, int MINB = 1>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(MINB == 2 ? 4 : 1))) void stream_kernel(
    const StreamArgs a) {
  static_assert(!I8 || MODE == 0, "int8 operands: filter pass only");
  typedef typename std::conditional<I8, i32x4, bf16x8>::type frag_t;
  typedef typename std::conditional<I8, i32x4, f32x4>::type acc_t;
  constexpr int ES = I8 ? 1 : 2;   // operand bytes per dim
  extern __shared__ __attribute__((aligned(16))) char sq[];   // [nqb][nk][64 lanes][16 B]
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int nk = a.DPB / (I8 ? 64 : 32);
  const int nkp = (nk + CH - 1) / CH * CH;   // K padded to whole chunks (zero fragments)
  const int nqb = a.nqb;
  // filter: each workgroup collects its candidates in LDS (kStreamSlots per query) and
  // appends them with one global atomic per query at its end -- per-candidate atomics on
  // the query's counter serialise at ~1.5k candidates per query (int8 bounds, 64 queries:
  // pass 300 -> 449 us); a full buffer falls back to the global append
  const int SLB = MODE == 0 ? a.slots : 0;   // 0: no LDS buffer (it did not fit: per-candidate atomics)
  int* s_cnt = reinterpret_cast<int*>(sq + (size_t)nqb * ((nk + kStreamChunk - 1) / kStreamChunk * kStreamChunk) * 1024);
  int* s_base = s_cnt + nqb * 16;
  int* s_crow = s_base + nqb * 16;
  float* s_cu = reinterpret_cast<float*>(s_crow + nqb * 16 * SLB);
  float* s_cl = s_cu + nqb * 16 * SLB;
  if (SLB)
    for (int i = threadIdx.x; i < nqb * 16; i += blockDim.x) s_cnt[i] = 0;
  // fused prep (MODE 1, fprep): per-query terms and the root prefix, after the image
  const bool fprep = MODE == 1 && a.fprep;
  float4* s_qi = reinterpret_cast<float4*>(sq + (size_t)nqb * nkp * 1024);
  float* s_pr = reinterpret_cast<float*>(s_qi + 16);
  float* s_part = s_pr + 16;
  // ---- stage the queries' fragments (B operand: 16 B at k = (16/ES)*(l>>4).., query = l&15) ----
  for (int f = threadIdx.x; f < nqb * nkp * 64; f += blockDim.x) {
    const int l = f & 63, ks = (f >> 6) % nkp, qb = (f >> 6) / nkp;
    const int q = qb * 16 + (l & 15);
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (fprep) {
      // sb_prep_kernel's bf16 hi parts of x - c, 8 dims per fragment
      if (ks < nk && q < a.nq) {
        uint32_t w[4] = {0u, 0u, 0u, 0u};
        const int d0 = ks * 32 + 8 * (l >> 4);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int d = d0 + j;
          const float x = d < a.fD ? a.fq[(size_t)q * a.fD + d] - a.fc[d] : 0.f;
          const __bf16 h = (__bf16)x;
          w[j >> 1] |= (uint32_t)__builtin_bit_cast(uint16_t, h) << (16 * (j & 1));
        }
        v = make_uint4(w[0], w[1], w[2], w[3]);
      }
      if (blockIdx.x == 0 && ks < nk)   // the filter pass reads Xb (rows < 16 incl. zero padding)
        *reinterpret_cast<uint4*>(const_cast<char*>(reinterpret_cast<const char*>(a.Xb)) +
                                  ((size_t)q * a.DPB * ES + ks * 64 + 16 * (l >> 4))) = v;
    } else if (ks < nk) {
      v = *reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(a.Xb) +
                                          ((size_t)q * a.DPB * ES + ks * 64 + 16 * (l >> 4)));
    }
    *reinterpret_cast<uint4*>(sq + (size_t)f * 16) = v;
  }
  if (fprep) {
    // {|x'|^2, |x_hi|, |x_lo|} per query row (sb_prep_kernel's loop and reduction; rows
    // past nq are zero), one wave per row
    for (int r = wave; r < 16; r += SK_WAVES) {
      double sv = 0.0, slo = 0.0, shi = 0.0;
      for (int d = lane; d < a.DPB; d += 64) {
        const float x = (r < a.nq && d < a.fD) ? a.fq[(size_t)r * a.fD + d] - a.fc[d] : 0.f;
        const __bf16 h = (__bf16)x;
        const float hf = (float)h;
        const float lo = x - hf;
        sv += (double)x * (double)x;
        slo += (double)lo * (double)lo;
        shi += (double)hf * (double)hf;
      }
      for (int off = 32; off > 0; off >>= 1) {
        sv += __shfl_xor(sv, off, 64);
        slo += __shfl_xor(slo, off, 64);
        shi += __shfl_xor(shi, off, 64);
      }
      if (lane == 0) {
        const float4 v4 = make_float4((float)sv, (float)(sqrt(shi) * (1.0 + 0x1p-20)), (float)(sqrt(slo) * (1.0 + 0x1p-20)),
                                      0.f);
        s_qi[r] = v4;
        if (blockIdx.x == 0) const_cast<float4*>(a.qinfo)[r] = v4;
      }
    }
    // the root's exact prefix: 16-dim fma partials in dimension order, summed in slice order
    const int NV16 = a.fDP / 16;
    for (int t = threadIdx.x; t < a.nq * NV16; t += blockDim.x) {
      const int q = t / NV16, vv = t - q * NV16;
      float pp = 0.f;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int d = vv * 16 + j;
        const float x = d < a.fD ? a.fq[(size_t)q * a.fD + d] : 0.f;
        const float tt = fmaf(x, a.fA[(size_t)d * a.fld], -a.fB[(size_t)d * a.fld]);
        pp = (j == 0) ? tt * tt : fmaf(tt, tt, pp);
      }
      s_part[t] = pp;
    }
    __syncthreads();
    if ((int)threadIdx.x < a.nq) {
      const float acc = sum_in_order(s_part + threadIdx.x * NV16, NV16);
      const float P = a.fw0 * (-0.5f * (a.flogdet0 + acc));
      s_pr[threadIdx.x] = P;
      if (blockIdx.x == 0) a.fP[(size_t)threadIdx.x * a.fldP] = P;
    }
    if (blockIdx.x == 0) {
      // the scan layout X [r/kXQ][v][r%kXQ][16] of the first query group, and the counters
      for (int e = threadIdx.x; e < 16 * a.fDP; e += blockDim.x) {
        const int r = e / a.fDP, d = e - r * a.fDP;
        const size_t o = ((size_t)(d / 16) * kXQ + r) * 16 + (d % 16);
        a.fX[o] = (r < a.nq && d < a.fD) ? a.fq[(size_t)r * a.fD + d] : 0.f;
      }
      for (int e = threadIdx.x; e < 5 * a.nq; e += blockDim.x) a.fqcnt[e] = 0;
    }
  }
  // per-lane query terms for the lane's column (query qb*16 + (lane & 15))
  float4 qi[MQB];
  float Tq[MQB];
  bool qok[MQB];
  if (fprep) __syncthreads();   // s_qi, s_pr written
#pragma unroll
  for (int qb = 0; qb < MQB; ++qb) {
    const int q = qb * 16 + (lane & 15);
    qok[qb] = qb < nqb && q < a.nq;
    qi[qb] = qok[qb] ? (fprep ? s_qi[q] : a.qinfo[q]) : make_float4(0.f, 0.f, 0.f, 0.f);
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
  // groups of the pass: the probe's sampled groups, the live block list (group pruning), or
  // every 16-row block
  const bool lst = MODE == 0 && a.live;
  const int64_t ngroups = MODE == 1 ? a.n_probe : lst ? (int64_t)*a.live_n : (int64_t)((a.nrows + 15) >> 4);
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
  float cB[MQB];             // categorize: the parent's bottleneck (BFk)
#pragma unroll
  for (int qb = 0; qb < MQB; ++qb) cP[qb] = cPh[qb] = 0.f, cB[qb] = CWQ_INF;
  const float* Pu = a.Phi ? a.Phi : a.P;
  // the wave's groups are numbered gi; a group's 16-row block (its rows blk * 16 ..): the probe's
  // every probe_stride-th, or the live list's entry (a wave-uniform scalar load, issued one
  // group ahead so the next group's first loads never wait for it)
  auto bmap = [&](int64_t g) -> int64_t { return MODE == 1 ? g * a.probe_stride : lst ? (int64_t)a.live[g] : g; };
  auto panel = [&](int64_t blk) {
    return reinterpret_cast<const char*>(a.Mb) + (size_t)(blk * 16 + r16) * a.DPB * ES + 16 * c16;
  };
  // row terms of the rows this lane's accumulator columns hold (r0 + 4*c16 + j)
  auto load_rf = [&](RowF (&dst)[4], int64_t blk) {
    const int64_t r0n = blk * 16;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t r = r0n + 4 * c16 + j;
      dst[j] = r < a.nrows ? a.rf[r] : RowF{-CWQ_INF, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, -2};
    }
  };
  int64_t gi = (int64_t)blockIdx.x * SK_WAVES + wave;
  const bool idle = gi >= ngroups;   // no group for this wave (the filter's flush barrier follows)
  if (idle) gi = 0;
  int64_t bcur = idle ? 0 : bmap(gi);
  int64_t bnxt = (!idle && gi + gstride < ngroups) ? bmap(gi + gstride) : 0;
  // K runs in chunks of CH fragments (16 B per lane each: row r0 + (lane & 15),
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
  frag_t bA[CH], bB[CH];
  auto issue = [&](frag_t (&b)[CH], const char* p, int nfr) {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const frag_t* pp = reinterpret_cast<const frag_t*>(p + min(i, nfr - 1) * 64);
      if constexpr (NT)   // read once: nontemporal (the guide's streamed-once policy)
        b[i] = __builtin_nontemporal_load(pp);
      else
        b[i] = *pp;
    }
  };
  acc_t acc[MQB];
#pragma unroll
  for (int qb = 0; qb < MQB; ++qb) acc[qb] = acc_t{0, 0, 0, 0};
  auto mma = [&](const frag_t (&b)[CH], int c0) {
#pragma unroll
    for (int qb = 0; qb < MQB; ++qb) {
      if (qb >= nqb) break;
      const char* qs = sq + (((size_t)qb * nkp + c0) * 64 + lane) * 16;
#pragma unroll
      for (int i = 0; i < CH; ++i) {
        if constexpr (I8)
          acc[qb] = __builtin_amdgcn_mfma_i32_16x16x64_i8(b[i], *reinterpret_cast<const i32x4*>(qs + i * 1024), acc[qb],
                                                          0, 0, 0);
        else
          acc[qb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[i], *reinterpret_cast<const bf16x8*>(qs + i * 1024),
                                                            acc[qb], 0, 0, 0);
      }
    }
  };
  issue(bA, panel(bcur), min(CH, nk));
  // the group's row terms are loaded at its start and used at its end (in flight with
  // its chunks)
  RowF rf[4];
  load_rf(rf, bcur);
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
  auto step = [&](const frag_t (&cur)[CH], frag_t (&oth)[CH]) -> bool {
    int64_t gn = gi;
    int cn = c0 + CH;
    if (cn >= nk) {
      gn = gi + gstride;
      cn = 0;
    }
    const bool more = gn < ngroups;
    issue(oth, more ? panel(cn == 0 ? bnxt : bcur) + cn * 64 : panel(bcur) + c0 * 64,
          more ? min(CH, nk - cn) : min(CH, nk - c0));
    mma(cur, c0);
    if (cn != 0) {
      c0 = cn;
      return true;
    }
    // ---- group gi done.  Epilogue: rigorous bounds per (row, query); acc[qb][j] = dot
    // of row r0 + 4*c16 + j with query qb*16 + (lane & 15)
    const int64_t r0 = bcur * 16;
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
          a.pout[(size_t)rid * a.ldpout + qb * 16 + r16] = rf[j].par < 0 ? proot[qb] : (float)acc[qb][j];
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
          cB[qb] = CWQ_INF;
          if (!qok[qb] || cpar < 0) continue;
          if (MODE != 2 && a.BFk) cB[qb] = a.BFk[(size_t)(qb * 16 + r16) * a.ldBF + cpar];
          if (fprep) {   // flat tree: the root is every row's parent
            cP[qb] = cPh[qb] = s_pr[qb * 16 + r16];
          } else if (a.pb.dot) {
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
        if (MODE == 1 && a.probe_rows && qok[qb] && !rok)
          a.lb[(size_t)(qb * 16 + r16) * a.ldlb + gi * 16 + 4 * c16 + j] = -CWQ_INF;
        if (!rok || !qok[qb]) continue;
        float u, l;
        // int8: the int32 acc is exact (|acc| <= 127^2 * DPB); up to three fp32 roundings
        // follow -- int32 -> fp32 (exact while |acc| < 2^24, i.e. DPB <= 1040; the D = 1536
        // panels round here), s_x * s_r, and the product -- each within 2^-24 relative, so
        // |err| <= (3 * 2^-24 + O(2^-48)) |dot| < 2^-22 |dot|; 2^-21 is taken, and beta has
        // no accumulation term
        const float dot = I8 ? (float)acc[qb][j] * (qi[qb].w * rf[j].R0) : (float)acc[qb][j];
        fg_bounds2(dot, (I8 ? 0x1p-21f : 0x1p-23f) * fabsf(dot), qi[qb], rf[j], cPh[qb] * rf[j].invL,
                   cP[qb] * rf[j].invL, a.eps_n, a.slack, u, l);
        if (a.BFk) {   // categorize: min(BFk[parent], lp) is monotone in lp (CWQ_INF: no parent)
          u = fminf(u, cB[qb]);
          l = fminf(l, cB[qb]);
        }
        if (MODE == 1) {
          if (a.probe_rows) a.lb[(size_t)(qb * 16 + r16) * a.ldlb + gi * 16 + 4 * c16 + j] = l;
          else pmax[qb] = fmaxf(pmax[qb], l);
        } else if (u >= Tq[qb] && u > -CWQ_INF) {   // (a -inf bound: a -inf key, never listed)
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
          const int ls = SLB ? atomicAdd(&s_cnt[q], 1) : 0;
          if (ls < SLB) {
            s_crow[q * SLB + ls] = (int)(r0 + 4 * c16 + j);
            s_cu[q * SLB + ls] = u;
            s_cl[q * SLB + ls] = l;
            continue;
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
    if (MODE == 1 && !a.probe_rows) {   // the group's max lower bound per query -> lb[q][gi]
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
    bcur = bnxt;
    bnxt = gi + gstride < ngroups ? bmap(gi + gstride) : 0;
    load_rf(rf, bcur);
    load_live(++it);
#pragma unroll
    for (int qb = 0; qb < MQB; ++qb) acc[qb] = acc_t{0, 0, 0, 0};
    return true;
  };
  if (!idle)
    while (step(bA, bB) && step(bB, bA)) {
    }
  if (MODE == 1 && a.sel_ctr) {
    // fused select: the workgroup that finishes last (cross-workgroup protocol: every lb store
    // of the workgroup complete, barrier, agent-scope release, then the counter) reads all of
    // lb after an agent-scope acquire and writes the thresholds select_kernel would
    // the flag lives in the query image's first word: every wave is past its last LDS read
    // of it at the barrier below (a static __shared__ word would push the kernel past the
    // dynamic-LDS maximum launch_one requests)
    int& s_last = *reinterpret_cast<int*>(sq);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      const int prev = atomicAdd(a.sel_ctr, 1);
      s_last = prev == (int)gridDim.x - 1;
      if (s_last) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
    if (s_last) {
      if (2 * a.nq <= SK_WAVES) {
      // T0 = the K-th largest of the probe's values (group maxima, or every probed row's
      // bound with probe_rows; multiplicity counted, -inf with fewer than K): a radix select
      // of ord_f32 keys, 6-bit digits from the top (5 passes, then the last 2 bits), wpq waves
      // per query sharing an LDS histogram (past the flag word: the query image is no longer
      // read).  Only T0 = sel_lk[q][K-1] is read downstream (the pass's threshold; the rerank
      // forms its own).  All waves run the same passes and rounds, so the barriers are uniform.
      // (Per-wave top-K lists' serial inserts made the C2 categorize probe of list 1 -- 18.7k
      // finite bounds -- twice as long as list 2's, profiles/r05_basic_percall_c2_timeline_v3.txt;
      // with a wave per query -- nq >= SK_WAVES / 2 -- the lists are kept: six passes over
      // each query's values cost more there, C3 nq = 64 probe 0.16 -> 0.31 ms,
      // profiles/r05_bench_v4.log.)
      unsigned* s_h = reinterpret_cast<unsigned*>(sq) + 16;   // [qpr][64] histograms
      unsigned* s_rs = s_h + SK_WAVES * 64;                    // [qpr][2] prefix, rank left
      const int n = (int)(a.probe_rows ? a.n_probe * 16 : a.n_probe);
      const int wpq = a.nq >= SK_WAVES ? 1 : SK_WAVES / a.nq;
      const int qpr = SK_WAVES / wpq;   // queries per round
      const int sub = wave % wpq, g = wave / wpq;
      const bool enough = n >= a.K;
      for (int q0 = 0; q0 < a.nq; q0 += qpr) {
        const int q = q0 + g;
        const bool act = g < qpr && q < a.nq;
        const float* __restrict__ L = a.lb + (size_t)(act ? q : 0) * a.ldlb;
        unsigned pref = 0u, kk = (unsigned)a.K;
        for (int ps = 0; ps < 6; ++ps) {
          const int bits = ps < 5 ? 6 : 2, sh = ps < 5 ? 26 - 6 * ps : 0;
          const unsigned hm = ps == 0 ? 0u : (~0u << (sh + bits)), dm = (1u << bits) - 1u;
          if (act && sub == 0) s_h[g * 64 + lane] = 0u;
          __syncthreads();
          if (act && enough) {
            int j = sub * 64 + lane;
            for (; j + 3 * wpq * 64 < n; j += 4 * wpq * 64) {   // 4 loads in flight
              float v[4];
#pragma unroll
              for (int u = 0; u < 4; ++u) v[u] = L[j + u * wpq * 64];
#pragma unroll
              for (int u = 0; u < 4; ++u) {
                const unsigned o = ord_f32(v[u]);
                if ((o & hm) == pref) atomicAdd(&s_h[g * 64 + ((o >> sh) & dm)], 1u);
              }
            }
            for (; j < n; j += wpq * 64) {
              const unsigned o = ord_f32(L[j]);
              if ((o & hm) == pref) atomicAdd(&s_h[g * 64 + ((o >> sh) & dm)], 1u);
            }
          }
          __syncthreads();
          if (act && enough && sub == 0) {
            // lane l holds bin dm - l (lane 0: the top bin); inclusive prefix over the lanes
            const int bin = (int)dm - lane;
            const unsigned c = bin >= 0 ? s_h[g * 64 + bin] : 0u;
            unsigned inc = c;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
              const unsigned t = __shfl_up(inc, o, 64);
              if (lane >= o) inc += t;
            }
            const unsigned exc = inc - c;
            if (bin >= 0 && exc < kk && kk <= inc) {   // one lane: the counts under the prefix reach kk
              s_rs[g * 2] = pref | ((unsigned)bin << sh);
              s_rs[g * 2 + 1] = kk - exc;
            }
          }
          __syncthreads();
          if (act && enough) {
            pref = s_rs[g * 2];
            kk = s_rs[g * 2 + 1];
          }
        }
        if (act && sub == 0) {
          float T0 = enough ? unord_f32(pref) : -CWQ_INF;
          if (a.sel_floor) T0 = fmaxf(T0, a.sel_floor[q]);
          a.sel_lk[(size_t)q * 64 + lane] = lane == a.K - 1 ? T0 : -CWQ_INF;
          a.sel_lr[(size_t)q * 64 + lane] = 0x7fffffff;
        }
      }
      } else {
      // the K-th largest of the probe's values (group maxima, or every probed row's bound
      // with probe_rows) one by one: wpq waves per query on its value range, the first of
      // them merging the others' lists (LDS past the flag word: the query image is no
      // longer read); all waves run the same rounds, so the barriers are uniform
      float* s_lk = reinterpret_cast<float*>(sq) + 16;
      int* s_lr = reinterpret_cast<int*>(sq) + 16 + SK_WAVES * 64;
      const int n = (int)(a.probe_rows ? a.n_probe * 16 : a.n_probe);
      const int wpq = a.nq >= SK_WAVES ? 1 : SK_WAVES / a.nq;
      const int qpr = SK_WAVES / wpq;   // queries per round
      const int sub = wave % wpq;
      const int per = (n + wpq * 64 - 1) / (wpq * 64) * 64;
      for (int q0 = 0; q0 < a.nq; q0 += qpr) {
        const int q = q0 + wave / wpq;
        const bool act = wave / wpq < qpr && q < a.nq;
        float lk = -CWQ_INF;
        int lr = 0x7fffffff;
        if (act) {
          const int lo = min(n, sub * per);
          select_values_wave(a.lb + (size_t)q * a.ldlb, lo, min(n, lo + per), a.K, lane, lk, lr);
        }
        if (wpq > 1) {
          s_lk[wave * 64 + lane] = lk;
          s_lr[wave * 64 + lane] = lr;
          __syncthreads();
          if (act && sub == 0)
            for (int w = wave + 1; w < wave + wpq; ++w) {
              const int r = s_lr[w * 64 + lane];
              list64_offer(lk, lr, lane, lane < a.K && r != 0x7fffffff ? s_lk[w * 64 + lane] : -CWQ_INF, r, a.K);
            }
        }
        if (act && sub == 0) {
          if (a.sel_floor && lane == a.K - 1) lk = fmaxf(lk, a.sel_floor[q]);
          a.sel_lk[(size_t)q * 64 + lane] = lk;
          a.sel_lr[(size_t)q * 64 + lane] = lr;
        }
        if (wpq > 1) __syncthreads();
      }
      }
      if (threadIdx.x == 0) __hip_atomic_store(a.sel_ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }
  if (MODE != 0 || !SLB) return;
  // ---- flush the workgroup's candidate buffer: one global atomic per query ----
  __syncthreads();
  for (int i = threadIdx.x; i < a.nq; i += blockDim.x) {
    const int c = min(s_cnt[i], SLB);
    s_base[i] = c > 0 ? atomicAdd(&a.qcnt[i], c) : 0;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < a.nq * SLB; e += blockDim.x) {
    const int i = e / SLB, k = e - i * SLB;
    if (k >= min(s_cnt[i], SLB)) continue;
    const int slot = s_base[i] + k;
    if (slot < a.capq) {
      const size_t o = (size_t)i * a.capq + slot;
      a.crow[o] = s_crow[e];
      a.cu[o] = s_cu[e];
      a.cl[o] = s_cl[e];
    } else {
      a.qover[i] = 1;
    }
  }
}

template <int MODE, int MQB, bool I8 = false, int CH = SK_CH, bool NT = false, int MINB = 1>
static hipError_t launch_one(const StreamArgs& a, int n_wg, size_t lds, hipStream_t s) {
  // dynamic LDS above the 64 KiB default (once per kernel and device, thread-safe)
  if (hipError_t e = ensure_dyn_lds(reinterpret_cast<const void*>(&stream_kernel<MODE, MQB, I8, CH, NT, MINB>),
                                    kStreamMaxLds))
    return e;
  hipLaunchKernelGGL((stream_kernel<MODE, MQB, I8, CH, NT, MINB>), dim3((unsigned)(n_wg * MINB)), dim3(64 * SK_WAVES),
                     lds, s, a);
  return hipGetLastError();
}

// fragments per chunk of the two-workgroup int8 pass (4; CWQ_STREAM_CHI8=3 / 6 for A/Bs)
static int chi8() {
  const char* e = getenv("CWQ_STREAM_CHI8");
  const int v = e && *e ? atoi(e) : 4;
  return v == 3 || v == 6 ? v : 4;
}

// the bf16 pass's two-workgroup form (A/B: CWQ_STREAM_OCC2_BF16=1 until measured)
static bool occ2_bf16() {
  const char* e = getenv("CWQ_STREAM_OCC2_BF16");
  return e && *e == '1';
}

template <int MQB>
static hipError_t launch_mqb(const StreamArgs& a, int mode, bool i8, bool ch12, int n_wg, size_t lds, hipStream_t s) {
  if (mode == 1) return launch_one<1, MQB>(a, n_wg, lds, s);
  if (mode == 2) return launch_one<2, MQB>(a, n_wg, lds, s);
  // CWQ_STREAM_NT=1: the filter pass's row panel by nontemporal loads (A/B knob)
  const char* ne = getenv("CWQ_STREAM_NT");
  const bool ntc = ne && *ne && atoi(ne) != 0;
  // One query block (nq <= 16, the per-call case): half-size chunks at two workgroups per CU
  // -- twice the waves, so one wave's bounds epilogue no longer leaves its SIMD's loads idle
  // (C3 one query per call 252.0 -> 237.8 us, profiles/r06_stream_occ2_ab.log).
  // CWQ_STREAM_OCC2=0 restores one workgroup per CU.
  const char* oe = getenv("CWQ_STREAM_OCC2");
  const int occ = oe && *oe ? atoi(oe) : 1;
  const bool two = MQB == 1 && occ == 1 && !ntc && lds * 2 <= (size_t)kStreamMaxLds;
  if (i8) {
    if (ch12 && two) {
      const int c = chi8();
      if (c == 6) return launch_one<0, MQB, true, 6, false, 2>(a, n_wg, lds, s);
      if (c == 3) return launch_one<0, MQB, true, 3, false, 2>(a, n_wg, lds, s);
      return launch_one<0, MQB, true, 4, false, 2>(a, n_wg, lds, s);
    }
    if (ch12) return ntc ? launch_one<0, MQB, true, 12, true>(a, n_wg, lds, s) : launch_one<0, MQB, true, 12>(a, n_wg, lds, s);
    return launch_one<0, MQB, true>(a, n_wg, lds, s);
  }
  if (two && occ2_bf16()) return launch_one<0, MQB, false, 4, false, 2>(a, n_wg, lds, s);
  return ntc ? launch_one<0, MQB, false, SK_CH, true>(a, n_wg, lds, s) : launch_one<0, MQB>(a, n_wg, lds, s);
}

hipError_t launch_stream(const StreamArgs& a, int mode, int n_wg, hipStream_t s) {
  const bool i8 = mode == 0 && a.i8;
  // the filter's LDS candidate buffer when it fits next to the query image
  StreamArgs b = a;
  b.slots = mode == 0 && stream_lds_bytes(a.nqb, a.DPB, i8, true) <= (size_t)kStreamMaxLds && !getenv("CWQ_STREAM_NOBUF")
                ? kStreamSlots
                : 0;
  const size_t lds = stream_lds_bytes(a.nqb, a.DPB, i8, b.slots > 0) +
                     (mode == 1 && a.fprep ? (size_t)(16 + 16 + 16 * (a.fDP / 16)) * 16 : 0);
  if (mode == 1 && a.fprep && (a.nqb != 1 || a.nq > 16 || a.fDP % 16 || a.fDP > 1024 || !a.fq || !a.fX || !a.fP))
    return hipErrorInvalidValue;
  if (a.nq <= 0 || a.nqb * 16 < a.nq || a.nqb > SK_MAXQB || a.DPB % (i8 ? 64 : 32) || a.K < 1 || a.K > 64 ||
      lds > (size_t)kStreamMaxLds || n_wg < 1 || (mode == 1 ? a.n_probe : a.nrows) < 1)
    return hipErrorInvalidValue;
  // int8 rows of a multiple of 12 fragments: 12-fragment chunks (their K padding, a whole
  // number of chunks, is within stream_lds_bytes' 8-fragment padding)
  const bool ch12 = i8 && (a.DPB / 64) % 12 == 0 && !getenv("CWQ_STREAM_CH8");
  return a.nqb == 1 ? launch_mqb<1>(b, mode, i8, ch12, n_wg, lds, s)
                    : launch_mqb<SK_MAXQB>(b, mode, i8, ch12, n_wg, lds, s);
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
