// libcwq: PCA + ICA whitening transform (F4) on fp32 MFMA.
//
// Replaces PCAICAWhiteningModel.transform (src/whitening/pca_ica.py:30-51):
//   x_c   = x - mean                         (:40)
//   x_pca = (x_c @ components^T) / sqrt(explained_var + eps)   (:43-44)
//   x_ica = x_pca @ unmixing^T               (:48)
// as two GEMMs C[m][n] = sum_k (A[m][k] - ctr[k]) * B[n][k] with the centring fused
// into the A-tile load and the per-column division into the epilogue.  fp32 in, fp32
// accumulate on v_mfma_f32_32x32x2_f32 (an exact fp32 fma chain in k order, at the fp32
// vector rate): the path keeps the reference's fp32 numerics instead of dropping to
// bf16 -- its output feeds the tree statistics.  The divisor sqrt(var + eps) is passed
// in, computed by the caller exactly as numpy does (fp32 add, fp32 sqrt), so only the
// order of the dot-product accumulation differs from the reference's sgemm.
//
// Tiling: 256-thread workgroups, 128 x 128 output tile, 4 waves of 64 x 64 (2 x 2
// accumulators of 32 x 32), K staged 16 deep through LDS k-major ([k][m], rows padded
// to 132 floats), next tile's global loads in registers during the MFMAs.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cwq_internal.h"

namespace cwq {

typedef float f32x16w __attribute__((ext_vector_type(16)));

constexpr int WT = 128;        // output tile edge
constexpr int WK = 16;         // K per LDS stage
constexpr int WLD = WT + 4;    // padded LDS row (floats)

__global__ __launch_bounds__(256) void gemm_nt_f32_kernel(const float* __restrict__ A, int64_t M, int K,
                                                          const float* __restrict__ ctr, const float* __restrict__ B,
                                                          int N, const float* __restrict__ denom, float* __restrict__ C) {
  __shared__ float As[2][WK][WLD];
  __shared__ float Bs[2][WK][WLD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int64_t m0 = (int64_t)blockIdx.x * WT;
  const int n0 = blockIdx.y * WT;
  // global -> register staging: thread loads 8 consecutive k of one row of A and of B
  const int lr = tid >> 1, lk = (tid & 1) * 8;
  const int64_t am = m0 + lr;
  const int bn = n0 + lr;
  // raw values only: the centring is applied when the registers go to LDS (after the
  // MFMAs), so the 4 loads of a stage are all in flight at once (computing x - ctr at the
  // load made the compiler wait for each load in turn: 8 round trips per stage)
  float4 ra0, ra1, rb0, rb1, rc0, rc1;   // A, B and ctr values of this thread's 8 k
  const bool vec = (K & 3) == 0;   // 16-B aligned rows
  auto gload = [&](int k0) {
    const int kb = k0 + lk;
    const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
    if (vec && kb + 8 <= K) {
      typedef float v4f __attribute__((ext_vector_type(4)));
      auto ld4 = [](const float* p) {
        const v4f v = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(p));   // streamed once
        return make_float4(v[0], v[1], v[2], v[3]);
      };
      ra0 = ra1 = rb0 = rb1 = rc0 = rc1 = z;
      if (am < M) {
        ra0 = ld4(A + am * K + kb);
        ra1 = ld4(A + am * K + kb + 4);
      }
      if (bn < N) {
        const v4f* bp = reinterpret_cast<const v4f*>(B + (int64_t)bn * K + kb);
        const v4f x0 = bp[0], x1 = bp[1];
        rb0 = make_float4(x0[0], x0[1], x0[2], x0[3]);
        rb1 = make_float4(x1[0], x1[1], x1[2], x1[3]);
      }
      if (ctr) {
        const v4f* cp = reinterpret_cast<const v4f*>(ctr + kb);
        const v4f c0 = cp[0], c1 = cp[1];
        rc0 = make_float4(c0[0], c0[1], c0[2], c0[3]);
        rc1 = make_float4(c1[0], c1[1], c1[2], c1[3]);
      }
    } else {
      auto ld = [&](const float* base, bool rowok, int k) { return (rowok && k < K) ? base[k] : 0.f; };
      const float* ar = A + am * K;
      const float* br = B + (int64_t)bn * K;
      ra0 = make_float4(ld(ar, am < M, kb), ld(ar, am < M, kb + 1), ld(ar, am < M, kb + 2), ld(ar, am < M, kb + 3));
      ra1 = make_float4(ld(ar, am < M, kb + 4), ld(ar, am < M, kb + 5), ld(ar, am < M, kb + 6), ld(ar, am < M, kb + 7));
      rb0 = make_float4(ld(br, bn < N, kb), ld(br, bn < N, kb + 1), ld(br, bn < N, kb + 2), ld(br, bn < N, kb + 3));
      rb1 = make_float4(ld(br, bn < N, kb + 4), ld(br, bn < N, kb + 5), ld(br, bn < N, kb + 6), ld(br, bn < N, kb + 7));
      rc0 = ctr ? make_float4(ld(ctr, true, kb), ld(ctr, true, kb + 1), ld(ctr, true, kb + 2), ld(ctr, true, kb + 3)) : z;
      rc1 = ctr ? make_float4(ld(ctr, true, kb + 4), ld(ctr, true, kb + 5), ld(ctr, true, kb + 6), ld(ctr, true, kb + 7))
                : z;
    }
  };
  auto swrite = [&](int b, int k0) {
    // padding (rows past M, k past K) stays exactly 0: x - ctr only where both exist
    const bool row = am < M;
    const int kb = k0 + lk;
    auto put = [&](int j, float av, float cv, float bv) {
      As[b][lk + j][lr] = (row && kb + j < K) ? av - cv : 0.f;
      Bs[b][lk + j][lr] = bv;
    };
    put(0, ra0.x, rc0.x, rb0.x);
    put(1, ra0.y, rc0.y, rb0.y);
    put(2, ra0.z, rc0.z, rb0.z);
    put(3, ra0.w, rc0.w, rb0.w);
    put(4, ra1.x, rc1.x, rb1.x);
    put(5, ra1.y, rc1.y, rb1.y);
    put(6, ra1.z, rc1.z, rb1.z);
    put(7, ra1.w, rc1.w, rb1.w);
  };
  f32x16w acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
  const int nk = (K + WK - 1) / WK;
  gload(0);
  swrite(0, 0);
  __syncthreads();
  const int fi = lane & 31, fk = lane >> 5;
  for (int kt = 0; kt < nk; ++kt) {
    const int b = kt & 1;
    if (kt + 1 < nk) gload((kt + 1) * WK);
#pragma unroll
    for (int kk = 0; kk < WK; kk += 2) {
      float af[2], bf[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        af[t] = As[b][kk + fk][wm * 64 + t * 32 + fi];
        bf[t] = Bs[b][kk + fk][wn * 64 + t * 32 + fi];
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) swrite(b ^ 1, (kt + 1) * WK);
    __syncthreads();
  }
  // epilogue: C[i = row m][j = column n]; lane: n = lane&31, m = (e&3) + 8(e>>2) + 4(lane>>5)
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = n0 + wn * 64 + j * 32 + fi;
    if (n >= N) continue;
    const float dv = denom ? denom[n] : 1.f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int64_t m = m0 + wm * 64 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * fk;
        if (m < M) C[m * N + n] = denom ? acc[i][j][e] / dv : acc[i][j][e];
      }
  }
}

hipError_t launch_gemm_nt_f32(const float* A, int64_t M, int K, const float* ctr, const float* B, int N,
                              const float* denom, float* C, hipStream_t s) {
  if (M <= 0 || N <= 0) return hipSuccess;
  dim3 grid((unsigned)((M + WT - 1) / WT), (unsigned)((N + WT - 1) / WT));
  hipLaunchKernelGGL(gemm_nt_f32_kernel, grid, dim3(256), 0, s, A, M, K, ctr, B, N, denom, C);
  return hipGetLastError();
}

}  // namespace cwq
