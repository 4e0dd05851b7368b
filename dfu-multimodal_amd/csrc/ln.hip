// LayerNorm (timm vision_transformer.py: nn.LayerNorm(768, eps=1e-6) as norm1/norm2/norm) on
// the fp32 residual stream.  One wave per row, 4 floats per lane per step; statistics by
// wave-shuffle reductions (two-pass mean / variance in registers).
#include "common.h"

namespace {

constexpr int MAXV = 4;  // float4 chunks per lane -> D <= 64*4*4 = 1024

template <bool OUT_BF>
__global__ void k_ln_fwd(const float* __restrict__ x, int64_t ldx, int rows, int D,
                         const float* __restrict__ gamma, const float* __restrict__ beta,
                         float eps, void* __restrict__ out, int64_t ldo,
                         float* __restrict__ mean_out, float* __restrict__ rstd_out) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int nv = D / 4;
  const float* xr = x + (int64_t)row * ldx;
  f32x4 v[MAXV];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int j = lane + 64 * i;
    v[i] = j < nv ? *(const f32x4*)(xr + 4 * j) : (f32x4){0, 0, 0, 0};
    s += v[i][0] + v[i][1] + v[i][2] + v[i][3];
  }
  const float mean = wave_sum(s) / (float)D;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int j = lane + 64 * i;
    if (j < nv)
      for (int e = 0; e < 4; ++e) { const float d = v[i][e] - mean; q += d * d; }
  }
  const float rstd = rsqrtf(wave_sum(q) / (float)D + eps);
  if (lane == 0) {
    if (mean_out) mean_out[row] = mean;
    if (rstd_out) rstd_out[row] = rstd;
  }
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int j = lane + 64 * i;
    if (j >= nv) continue;
    const f32x4 g = *(const f32x4*)(gamma + 4 * j);
    const f32x4 b = *(const f32x4*)(beta + 4 * j);
    float o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = (v[i][e] - mean) * rstd * g[e] + b[e];
    if constexpr (OUT_BF) {
      bf16_t* orow = (bf16_t*)out + (int64_t)row * ldo + 4 * j;
      *(u32x2*)orow = (u32x2){pack2(o[0], o[1]), pack2(o[2], o[3])};
    } else {
      float* orow = (float*)out + (int64_t)row * ldo + 4 * j;
      *(f32x4*)orow = (f32x4){o[0], o[1], o[2], o[3]};
    }
  }
}

constexpr int LNB_ROWS = 16;  // rows per block in the backward (4 per wave): 788 blocks at B=64

template <bool DY_BF>
__global__ void k_ln_bwd(const void* __restrict__ dyv, int64_t lddy, const float* __restrict__ x,
                         int64_t ldx, const float* __restrict__ mean_in,
                         const float* __restrict__ rstd_in, const float* __restrict__ gamma,
                         int rows, int D, float* __restrict__ gx, int64_t ldg,
                         bf16_t* __restrict__ gx_bf, float* __restrict__ partial,
                         float* __restrict__ gsum_partial) {
  __shared__ float red[3][4][1024];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nv = D / 4;
  float dg[MAXV][4], db[MAXV][4], gs[MAXV][4];
#pragma unroll
  for (int i = 0; i < MAXV; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) { dg[i][e] = 0.f; db[i][e] = 0.f; gs[i][e] = 0.f; }
  f32x4 gm[MAXV];
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int j = lane + 64 * i;
    gm[i] = j < nv ? *(const f32x4*)(gamma + 4 * j) : (f32x4){0, 0, 0, 0};
  }
  for (int rr = 0; rr < LNB_ROWS / 4; ++rr) {
    const int row = blockIdx.x * LNB_ROWS + wave * (LNB_ROWS / 4) + rr;
    if (row >= rows) break;
    const float mu = mean_in[row], rs = rstd_in[row];
    float xh[MAXV][4], dy[MAXV][4];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
      const int j = lane + 64 * i;
      if (j < nv) {
        const f32x4 xv = *(const f32x4*)(x + (int64_t)row * ldx + 4 * j);
        if constexpr (DY_BF) {
          const u32x2 w = *(const u32x2*)((const bf16_t*)dyv + (int64_t)row * lddy + 4 * j);
          dy[i][0] = lo_bf(w[0]); dy[i][1] = hi_bf(w[0]); dy[i][2] = lo_bf(w[1]); dy[i][3] = hi_bf(w[1]);
        } else {
          const f32x4 w = *(const f32x4*)((const float*)dyv + (int64_t)row * lddy + 4 * j);
          dy[i][0] = w[0]; dy[i][1] = w[1]; dy[i][2] = w[2]; dy[i][3] = w[3];
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          xh[i][e] = (xv[e] - mu) * rs;
          const float dxh = dy[i][e] * gm[i][e];
          s1 += dxh;
          s2 += dxh * xh[i][e];
          dg[i][e] += dy[i][e] * xh[i][e];
          db[i][e] += dy[i][e];
        }
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) { xh[i][e] = 0.f; dy[i][e] = 0.f; }
      }
    }
    s1 = wave_sum(s1) / (float)D;
    s2 = wave_sum(s2) / (float)D;
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
      const int j = lane + 64 * i;
      if (j >= nv) continue;
      float* g = gx + (int64_t)row * ldg + 4 * j;
      f32x4 gv = *(f32x4*)g;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        gv[e] += rs * (dy[i][e] * gm[i][e] - s1 - xh[i][e] * s2);
        gs[i][e] += gv[e];
      }
      *(f32x4*)g = gv;
      if (gx_bf) {
        bf16_t* gb = gx_bf + (int64_t)row * ldg + 4 * j;
        *(u32x2*)gb = (u32x2){pack2(gv[0], gv[1]), pack2(gv[2], gv[3])};
      }
    }
  }
  // reduce dgamma/dbeta over the 4 waves
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int j = lane + 64 * i;
    if (j < nv)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        red[0][wave][4 * j + e] = dg[i][e];
        red[1][wave][4 * j + e] = db[i][e];
        red[2][wave][4 * j + e] = gs[i][e];
      }
  }
  __syncthreads();
  if (gsum_partial)  // column sums of the updated residual gradient (the upstream bias grad)
    for (int d = threadIdx.x; d < D; d += blockDim.x)
      gsum_partial[(int64_t)blockIdx.x * D + d] =
          red[2][0][d] + red[2][1][d] + red[2][2][d] + red[2][3][d];
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    partial[((int64_t)blockIdx.x * 2 + 0) * D + d] =
        red[0][0][d] + red[0][1][d] + red[0][2][d] + red[0][3][d];
    partial[((int64_t)blockIdx.x * 2 + 1) * D + d] =
        red[1][0][d] + red[1][1][d] + red[1][2][d] + red[1][3][d];
  }
}

}  // namespace

extern "C" int dfu_layernorm_fwd(const float* x, int64_t ldx, int32_t rows, int32_t D,
                                 const float* gamma, const float* beta, float eps, void* out,
                                 int64_t ldo, int32_t out_bf16, float* mean, float* rstd,
                                 void* stream) {
  DFU_CHECK_ARG(x && gamma && beta && out && rows > 0 && D % 4 == 0 && D <= 64 * 4 * MAXV,
                "dfu_layernorm_fwd: bad args (D=%d)", D);
  DFU_CHECK_ARG(ldx % 4 == 0 && ldo % 4 == 0, "dfu_layernorm_fwd: ld must be multiple of 4");
  dim3 grid((rows + 3) / 4);
  if (out_bf16)
    hipLaunchKernelGGL(k_ln_fwd<true>, grid, dim3(256), 0, (hipStream_t)stream, x, ldx, rows, D,
                       gamma, beta, eps, out, ldo, mean, rstd);
  else
    hipLaunchKernelGGL(k_ln_fwd<false>, grid, dim3(256), 0, (hipStream_t)stream, x, ldx, rows, D,
                       gamma, beta, eps, out, ldo, mean, rstd);
  DFU_LAUNCH_CHECK();
  return DFU_OK;
}

extern "C" int dfu_ln_bwd_blocks(int32_t rows) { return (rows + LNB_ROWS - 1) / LNB_ROWS; }

extern "C" int dfu_layernorm_bwd(const void* dy, int64_t lddy, int32_t dy_bf16, const float* x,
                                 int64_t ldx, const float* mean, const float* rstd,
                                 const float* gamma, int32_t rows, int32_t D, float* gx,
                                 int64_t ldg, void* gx_bf16, float* partial, float* gsum_partial,
                                 void* stream) {
  DFU_CHECK_ARG(dy && x && mean && rstd && gamma && gx && partial && rows > 0 && D % 4 == 0 &&
                    D <= 1024,
                "dfu_layernorm_bwd: bad args");
  DFU_CHECK_ARG(lddy % 4 == 0 && ldx % 4 == 0 && ldg % 4 == 0, "dfu_layernorm_bwd: bad ld");
  dim3 grid(dfu_ln_bwd_blocks(rows));
  if (dy_bf16)
    hipLaunchKernelGGL(k_ln_bwd<true>, grid, dim3(256), 0, (hipStream_t)stream, dy, lddy, x, ldx,
                       mean, rstd, gamma, rows, D, gx, ldg, (bf16_t*)gx_bf16, partial, gsum_partial);
  else
    hipLaunchKernelGGL(k_ln_bwd<false>, grid, dim3(256), 0, (hipStream_t)stream, dy, lddy, x, ldx,
                       mean, rstd, gamma, rows, D, gx, ldg, (bf16_t*)gx_bf16, partial, gsum_partial);
  DFU_LAUNCH_CHECK();
  return DFU_OK;
}
