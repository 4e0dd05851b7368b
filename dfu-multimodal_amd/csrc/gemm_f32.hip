// Small fp32 GEMM for the late-fusion head (train_multimodal_fusion.py:305-313 /
// grad_cam_visualization.py:289-302: Linear(2816, 512) -> ReLU -> Dropout -> Linear(512, 2)).
// The head is 1.44 MMAC per image pair (0.003 % of the step): it runs in exact fp32 so the
// logits carry no bf16 rounding of the features or head weights.  Generic strides cover the
// forward (X W^T), the input gradient (G W) and the weight gradient (G^T X) with one kernel.
//   C[m][n] = beta*C[m][n] + sum_k A[m*sam + k*sak] * B[n*sbn + k*sbk] (+ bias[n]) (relu)
// The head's shapes have few output tiles (64 x 512 -> 8 tiles of 64x64) and long K (2816), so
// K is split across workgroups: each split writes an fp32 slab [split][M][N] of the caller's
// workspace and a second kernel sums the slabs in a fixed order and applies the epilogue —
// deterministic, and ~300 workgroups instead of 8.
#include "common.h"

namespace {

constexpr int T = 64, TK = 16;

__global__ __launch_bounds__(256) void k_gemm_f32(int M, int N, int K, const float* __restrict__ A,
                                                  int64_t sam, int64_t sak,
                                                  const float* __restrict__ B, int64_t sbn,
                                                  int64_t sbk, float* __restrict__ C, int64_t ldc,
                                                  const float* __restrict__ bias, int relu,
                                                  int accumulate, int k_per_split,
                                                  float* __restrict__ slab) {
  __shared__ float As[TK][T + 1];
  __shared__ float Bs[TK][T + 1];
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const int m0 = blockIdx.y * T, n0 = blockIdx.x * T;
  const int kb = blockIdx.z * k_per_split;
  const int ke = min(K, kb + k_per_split);
  float acc[4][4] = {};
  for (int k0 = kb; k0 < ke; k0 += TK) {
    for (int i = threadIdx.x; i < T * TK; i += 256) {
      const int r = i / TK, kk = i % TK;
      const int m = m0 + r, n = n0 + r, k = k0 + kk;
      As[kk][r] = (m < M && k < ke) ? A[(int64_t)m * sam + (int64_t)k * sak] : 0.f;
      Bs[kk][r] = (n < N && k < ke) ? B[(int64_t)n * sbn + (int64_t)k * sbk] : 0.f;
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
      if (slab) {  // split-K partial: plain store, epilogue in k_gemm_f32_reduce
        slab[((int64_t)blockIdx.z * M + m) * N + n] = v;
        continue;
      }
      if (bias) v += bias[n];
      if (accumulate) v += C[(int64_t)m * ldc + n];
      if (relu) v = fmaxf(v, 0.f);
      C[(int64_t)m * ldc + n] = v;
    }
  }
}

__global__ void k_gemm_f32_reduce(int M, int N, int splits, const float* __restrict__ slab,
                                  float* __restrict__ C, int64_t ldc, const float* __restrict__ bias,
                                  int relu, int accumulate) {
  const int64_t mn = (int64_t)M * N;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < mn;
       i += (int64_t)gridDim.x * blockDim.x) {
    float v = 0.f;
    for (int s = 0; s < splits; ++s) v += slab[s * mn + i];
    const int64_t m = i / N;
    const int n = (int)(i - m * N);
    if (bias) v += bias[n];
    float* c = C + m * ldc + n;
    if (accumulate) v += *c;
    if (relu) v = fmaxf(v, 0.f);
    *c = v;
  }
}

int splits_for(int M, int N, int K) {
  const int tiles = ((M + T - 1) / T) * ((N + T - 1) / T);
  int s = 512 / tiles;                       // aim at ~2 workgroups per CU
  const int kmax = (K + 63) / 64;            // at least 64 of K per split
  s = s < kmax ? s : kmax;
  return s < 1 ? 1 : s;
}

}  // namespace

extern "C" int64_t dfu_gemm_f32_workspace_bytes(int32_t M, int32_t N, int32_t K) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  const int s = splits_for(M, N, K);
  return s > 1 ? (int64_t)s * M * N * 4 : 0;
}

extern "C" int dfu_gemm_f32(int32_t M, int32_t N, int32_t K, const float* A, int64_t sam,
                            int64_t sak, const float* B, int64_t sbn, int64_t sbk, float* C,
                            int64_t ldc, const float* bias, int32_t relu, int32_t accumulate,
                            void* workspace, int64_t workspace_bytes, void* stream) {
  DFU_CHECK_ARG(A && B && C && M > 0 && N > 0 && K > 0, "dfu_gemm_f32: bad args");
  int splits = splits_for(M, N, K);
  if (workspace == nullptr || workspace_bytes < (int64_t)splits * M * N * 4) splits = 1;
  const int kps = (((K + splits - 1) / splits) + TK - 1) / TK * TK;
  splits = (K + kps - 1) / kps;
  float* slab = splits > 1 ? (float*)workspace : nullptr;
  hipStream_t s = (hipStream_t)stream;
  dim3 grid((N + T - 1) / T, (M + T - 1) / T, splits);
  hipLaunchKernelGGL(k_gemm_f32, grid, dim3(256), 0, s, M, N, K, A, sam, sak, B, sbn, sbk, C, ldc,
                     bias, relu, accumulate, kps, slab);
  DFU_LAUNCH_CHECK();
  if (slab) {
    const int64_t mn = (int64_t)M * N;
    int blocks = (int)((mn + 255) / 256);
    blocks = blocks > 2048 ? 2048 : blocks;
    hipLaunchKernelGGL(k_gemm_f32_reduce, dim3(blocks), dim3(256), 0, s, M, N, splits, slab, C,
                       ldc, bias, relu, accumulate);
    DFU_LAUNCH_CHECK();
  }
  return DFU_OK;
}
