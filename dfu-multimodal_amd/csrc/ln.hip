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

constexpr int LNB_ROWS = 32;  // rows per block in the backward (8 per wave): 394 blocks at B=64
constexpr int LNB_ILP = 2;    // rows per wave whose loads issue together (same box: 16/2 34.4 us, 32/2 31.7, 64/2 36.8, 32/4 41.5)

// Backward, one wave per row, 4 rows per wave processed two at a time: all loads of a row pair
// (x, dy, and the residual gradient gx it adds into) are issued before either row's
// reductions, so each pair costs one memory round trip.  NV = float4 chunks per lane
// (D <= 256 * NV).  dgamma / dbeta / column sums of the updated gx are reduced over the 4
// waves through one LDS buffer reused per quantity.
template <bool DY_BF, int NV>
__global__ __launch_bounds__(256) void k_ln_bwd(
    const void* __restrict__ dyv, int64_t lddy, const float* __restrict__ x, int64_t ldx,
    const float* __restrict__ mean_in, const float* __restrict__ rstd_in,
    const float* __restrict__ gamma, int rows, int D, float* __restrict__ gx, int64_t ldg,
    bf16_t* __restrict__ gx_bf, float* __restrict__ partial, float* __restrict__ gsum_partial) {
  __shared__ float red[4][256 * NV];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nv = D / 4;
  float dg[NV][4], db[NV][4], gs[NV][4];
  f32x4 gm[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int j = lane + 64 * i;
    gm[i] = j < nv ? *(const f32x4*)(gamma + 4 * j) : (f32x4){0, 0, 0, 0};
#pragma unroll
    for (int e = 0; e < 4; ++e) { dg[i][e] = 0.f; db[i][e] = 0.f; gs[i][e] = 0.f; }
  }
  const int row0 = blockIdx.x * LNB_ROWS + wave * (LNB_ROWS / 4);
#pragma unroll 1
  for (int rp = 0; rp < LNB_ROWS / 4; rp += LNB_ILP) {
    f32x4 xv[LNB_ILP][NV], gv[LNB_ILP][NV];
    float dy[LNB_ILP][NV][4], mu[LNB_ILP], rs[LNB_ILP];
    bool ok[LNB_ILP];
#pragma unroll
    for (int h = 0; h < LNB_ILP; ++h) {  // load phase: LNB_ILP rows
      const int row = row0 + rp + h;
      ok[h] = row < rows;
      mu[h] = ok[h] ? mean_in[row] : 0.f;
      rs[h] = ok[h] ? rstd_in[row] : 0.f;
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int j = lane + 64 * i;
        if (ok[h] && j < nv) {
          xv[h][i] = *(const f32x4*)(x + (int64_t)row * ldx + 4 * j);
          gv[h][i] = *(const f32x4*)(gx + (int64_t)row * ldg + 4 * j);
          if constexpr (DY_BF) {
            const u32x2 w = *(const u32x2*)((const bf16_t*)dyv + (int64_t)row * lddy + 4 * j);
            dy[h][i][0] = lo_bf(w[0]); dy[h][i][1] = hi_bf(w[0]);
            dy[h][i][2] = lo_bf(w[1]); dy[h][i][3] = hi_bf(w[1]);
          } else {
            const f32x4 w = *(const f32x4*)((const float*)dyv + (int64_t)row * lddy + 4 * j);
#pragma unroll
            for (int e = 0; e < 4; ++e) dy[h][i][e] = w[e];
          }
        } else {
          xv[h][i] = (f32x4){0, 0, 0, 0};
          gv[h][i] = (f32x4){0, 0, 0, 0};
#pragma unroll
          for (int e = 0; e < 4; ++e) dy[h][i][e] = 0.f;
        }
      }
    }
    float s1[LNB_ILP], s2[LNB_ILP];
#pragma unroll
    for (int h = 0; h < LNB_ILP; ++h) {
      s1[h] = 0.f;
      s2[h] = 0.f;
#pragma unroll
      for (int i = 0; i < NV; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float xh = (xv[h][i][e] - mu[h]) * rs[h];
          const float dxh = dy[h][i][e] * gm[i][e];
          s1[h] += dxh;
          s2[h] += dxh * xh;
          dg[i][e] += dy[h][i][e] * xh;
          db[i][e] += dy[h][i][e];
        }
    }
#pragma unroll
    for (int h = 0; h < LNB_ILP; ++h) {
      s1[h] = wave_sum(s1[h]) / (float)D;
      s2[h] = wave_sum(s2[h]) / (float)D;
    }
#pragma unroll
    for (int h = 0; h < LNB_ILP; ++h) {
      if (!ok[h]) continue;
      const int row = row0 + rp + h;
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int j = lane + 64 * i;
        if (j >= nv) continue;
        f32x4 g = gv[h][i];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float xh = (xv[h][i][e] - mu[h]) * rs[h];
          g[e] += rs[h] * (dy[h][i][e] * gm[i][e] - s1[h] - xh * s2[h]);
          gs[i][e] += g[e];
        }
        *(f32x4*)(gx + (int64_t)row * ldg + 4 * j) = g;
        if (gx_bf) {
          bf16_t* gb = gx_bf + (int64_t)row * ldg + 4 * j;
          *(u32x2*)gb = (u32x2){pack2(g[0], g[1]), pack2(g[2], g[3])};
        }
      }
    }
  }
  // reduce dgamma, dbeta (and the gx column sums) over the 4 waves, one quantity at a time
  auto wave_reduce = [&](float (&q)[NV][4], float* dst) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int j = lane + 64 * i;
      if (j < nv)
#pragma unroll
        for (int e = 0; e < 4; ++e) red[wave][4 * j + e] = q[i][e];
    }
    __syncthreads();
    for (int d = threadIdx.x; d < D; d += blockDim.x)
      dst[d] = red[0][d] + red[1][d] + red[2][d] + red[3][d];
    __syncthreads();
  };
  wave_reduce(dg, partial + ((int64_t)blockIdx.x * 2 + 0) * D);
  wave_reduce(db, partial + ((int64_t)blockIdx.x * 2 + 1) * D);
  if (gsum_partial)  // column sums of the updated residual gradient (the upstream bias grad)
    wave_reduce(gs, gsum_partial + (int64_t)blockIdx.x * D);
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
  auto kern = D <= 768 ? (dy_bf16 ? k_ln_bwd<true, 3> : k_ln_bwd<false, 3>)
                       : (dy_bf16 ? k_ln_bwd<true, 4> : k_ln_bwd<false, 4>);
  hipLaunchKernelGGL(kern, grid, dim3(256), 0, (hipStream_t)stream, dy, lddy, x, ldx, mean, rstd,
                     gamma, rows, D, gx, ldg, (bf16_t*)gx_bf16, partial, gsum_partial);
  DFU_LAUNCH_CHECK();
  return DFU_OK;
}
