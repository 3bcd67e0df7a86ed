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
  float ra[8], rb[8];
  auto gload = [&](int k0) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = k0 + lk + j;
      const bool kin = k < K;
      ra[j] = (am < M && kin) ? A[am * K + k] - (ctr ? ctr[k] : 0.f) : 0.f;
      rb[j] = (bn < N && kin) ? B[(int64_t)bn * K + k] : 0.f;
    }
  };
  auto swrite = [&](int b) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      As[b][lk + j][lr] = ra[j];
      Bs[b][lk + j][lr] = rb[j];
    }
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
  swrite(0);
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
    if (kt + 1 < nk) swrite(b ^ 1);
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
