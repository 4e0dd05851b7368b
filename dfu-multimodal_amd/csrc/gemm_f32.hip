// Small fp32 GEMM for the late-fusion head (train_multimodal_fusion.py:305-313 /
// grad_cam_visualization.py:289-302: Linear(2816, 512) -> ReLU -> Dropout -> Linear(512, 2)).
// The head is 1.44 MMAC per image pair (0.003 % of the step): it runs in exact fp32 so the
// logits carry no bf16 rounding of the features or head weights.  Generic strides cover the
// forward (X W^T), the input gradient (G W) and the weight gradient (G^T X) with one kernel.
//   C[m][n] = beta*C[m][n] + sum_k A[m*sam + k*sak] * B[n*sbn + k*sbk] (+ bias[n]) (relu)
#include "common.h"

namespace {

constexpr int T = 64, TK = 16;

__global__ __launch_bounds__(256) void k_gemm_f32(int M, int N, int K, const float* __restrict__ A,
                                                  int64_t sam, int64_t sak,
                                                  const float* __restrict__ B, int64_t sbn,
                                                  int64_t sbk, float* __restrict__ C, int64_t ldc,
                                                  const float* __restrict__ bias, int relu,
                                                  int accumulate) {
  __shared__ float As[TK][T + 1];
  __shared__ float Bs[TK][T + 1];
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const int m0 = blockIdx.y * T, n0 = blockIdx.x * T;
  float acc[4][4] = {};
  for (int k0 = 0; k0 < K; k0 += TK) {
    for (int i = threadIdx.x; i < T * TK; i += 256) {
      const int r = i / TK, kk = i % TK;
      const int m = m0 + r, n = n0 + r, k = k0 + kk;
      As[kk][r] = (m < M && k < K) ? A[(int64_t)m * sam + (int64_t)k * sak] : 0.f;
      Bs[kk][r] = (n < N && k < K) ? B[(int64_t)n * sbn + (int64_t)k * sbk] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < TK; ++kk) {
      float a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) { a[i] = As[kk][ty * 4 + i]; b[i] = Bs[kk][tx * 4 + i]; }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(a[i], b[j], acc[i][j]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + ty * 4 + i;
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + tx * 4 + j;
      if (n >= N) continue;
      float v = acc[i][j];
      if (bias) v += bias[n];
      if (accumulate) v += C[(int64_t)m * ldc + n];
      if (relu) v = fmaxf(v, 0.f);
      C[(int64_t)m * ldc + n] = v;
    }
  }
}

}  // namespace

extern "C" int dfu_gemm_f32(int32_t M, int32_t N, int32_t K, const float* A, int64_t sam,
                            int64_t sak, const float* B, int64_t sbn, int64_t sbk, float* C,
                            int64_t ldc, const float* bias, int32_t relu, int32_t accumulate,
                            void* stream) {
  DFU_CHECK_ARG(A && B && C && M > 0 && N > 0 && K > 0, "dfu_gemm_f32: bad args");
  dim3 grid((N + T - 1) / T, (M + T - 1) / T);
  hipLaunchKernelGGL(k_gemm_f32, grid, dim3(256), 0, (hipStream_t)stream, M, N, K, A, sam, sak, B,
                     sbn, sbk, C, ldc, bias, relu, accumulate);
  DFU_LAUNCH_CHECK();
  return DFU_OK;
}
