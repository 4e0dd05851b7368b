// Training-mode BatchNorm2d over NHWC bf16 activations (torchvision resnet.py: every conv is
// followed by BatchNorm2d(eps=1e-5, momentum=0.1); train_multimodal_fusion.py:375 runs them
// in train mode).  Forward statistics come from the producing GEMM's epilogue slab
// (DFU_EPI_BF16_STATS: per 128-row tile, per channel (sum, M2)); this file combines them,
// applies the normalisation (+ residual, + ReLU), and implements the backward.
#include "common.h"

namespace {

// ---------------------------------------------------------------- forward finalize
// Block = 16 waves x 64 channel-lanes: a lane owns one channel (the 64 lanes of a wave read one
// contiguous 256-B row segment of the slab per tile), the waves stride the tiles; fp64 sums,
// then a 16-way LDS reduction.  Per tile t (nb rows): sum sb and M2 qb -> sum of squares
// qb + sb^2/nb.  fp64 sums of x and x^2 over <= 1e6 rows of bf16-scale values keep
// var = E[x^2] - mean^2 exact to ~1e-12 relative, and the tile loop is independent adds.
constexpr int FIN_WAVES = 16;  // (8 / 4 waves measured slower in the fusion step, round 3)

// CPW channels per block: a wave's 64 lanes cover CPW channels x (64 / CPW) tile slots, so
// narrow layers (C = 64 over up to 6272 stem tiles) spread their tile loop over more lanes.
// Slices (blockIdx.y, gridDim.y = S > 1): each block reduces tiles [y * tps, (y + 1) * tps)
// and publishes fp64 (sum, sum of squares) per channel with write-through (sc1) stores; one
// agent-scope counter per channel group counts the slices, and the LAST to arrive (told by the
// value its add returned; MI355X_MICROARCH.md hand-off table, row 1: sc1 stores, sc1 loads, no
// fence) sums the S records in slice order and finalizes — the result does not depend on the
// arrival order.  The counter is returned to zero (ops.tile_counters' invariant).
DFU_DEV void st_sc1_f64(double* p, double v) {
  __hip_atomic_store((unsigned long long*)p, (unsigned long long)__double_as_longlong(v),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
DFU_DEV double ld_sc1_f64(const double* p) {
  return __longlong_as_double((long long)__hip_atomic_load((unsigned long long*)p, __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_AGENT));
}

// Slice hand-off: every block's lane-0 record stores are drained, the block's add is counted;
// returns (in every thread) whether this block is the last of its channel group.
DFU_DEV bool last_slice(int* counter, int S, int* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const int old = __hip_atomic_fetch_add(counter, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = old == S - 1;
    if (last) __hip_atomic_store(counter, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = last;
  }
  __syncthreads();
  return *flag != 0;
}

template <int CPW>
__global__ __launch_bounds__(64 * FIN_WAVES) void k_bn_finalize(
    const float* __restrict__ stats, int tiles, int tps, int M, int C,
    const float* __restrict__ gamma, const float* __restrict__ beta, float eps, float momentum,
    float* __restrict__ rmean, float* __restrict__ rvar, int64_t* __restrict__ nbt,
    float* __restrict__ mean_out, float* __restrict__ invstd_out, float* __restrict__ scale_out,
    float* __restrict__ shift_out, double* __restrict__ ws, int* __restrict__ counters) {
  constexpr int TS = 64 / CPW;  // tile slots per wave
  __shared__ double sh_s[FIN_WAVES][64], sh_q[FIN_WAVES][64];
  __shared__ int flag;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int cl = lane % CPW, slot = lane / CPW;
  const int c = blockIdx.x * CPW + cl;
  const int S = gridDim.y;
  const int t0 = blockIdx.y * tps, t1 = min(tiles, t0 + tps);
  double sx = 0.0, sxx = 0.0;
  if (c < C) {
    const int last = tiles - 1;
    const double inv_last = 1.0 / (double)(M - last * 128);
#pragma unroll 4
    for (int t = t0 + w * TS + slot; t < t1; t += FIN_WAVES * TS) {
      const double sb = stats[((int64_t)t * 2 + 0) * C + c];
      const double qb = stats[((int64_t)t * 2 + 1) * C + c];
      sx += sb;
      sxx += qb + sb * sb * (t == last ? inv_last : (1.0 / 128.0));
    }
  }
  sh_s[w][lane] = sx;
  sh_q[w][lane] = sxx;
  __syncthreads();
  const bool owner = w == 0 && slot == 0 && c < C;
  if (owner) {
    sx = sxx = 0.0;
    for (int k = 0; k < FIN_WAVES; ++k)
      for (int j = 0; j < TS; ++j) {
        sx += sh_s[k][j * CPW + cl];
        sxx += sh_q[k][j * CPW + cl];
      }
  }
  if (S > 1) {
    if (owner) {
      st_sc1_f64(ws + ((int64_t)blockIdx.y * 2 + 0) * C + c, sx);
      st_sc1_f64(ws + ((int64_t)blockIdx.y * 2 + 1) * C + c, sxx);
    }
    if (!last_slice(counters + blockIdx.x, S, &flag)) return;
    if (owner) {
      sx = sxx = 0.0;
      for (int y = 0; y < S; ++y) {
        sx += ld_sc1_f64(ws + ((int64_t)y * 2 + 0) * C + c);
        sxx += ld_sc1_f64(ws + ((int64_t)y * 2 + 1) * C + c);
      }
    }
  }
  if (owner) {
    const double nn = (double)M;
    const double mu = sx / nn;
    const double var = fmax(sxx / nn - mu * mu, 0.0);  // biased, used to normalise
    const float invstd = (float)(1.0 / sqrt(var + (double)eps));
    const float g = gamma ? gamma[c] : 1.f;
    const float b = beta ? beta[c] : 0.f;
    mean_out[c] = (float)mu;
    invstd_out[c] = invstd;
    scale_out[c] = g * invstd;
    shift_out[c] = b - (float)mu * g * invstd;
    if (rmean) rmean[c] = (1.f - momentum) * rmean[c] + momentum * (float)mu;
    if (rvar) {
      const double unb = nn > 1.0 ? var * nn / (nn - 1.0) : var;
      rvar[c] = (1.f - momentum) * rvar[c] + momentum * (float)unb;
    }
  }
  if (nbt && blockIdx.x == 0 && threadIdx.x == 0) *nbt += 1;  // one finalizing block
}

__global__ void k_bn_eval_coeffs(const float* gamma, const float* beta, const float* rm,
                                 const float* rv, float eps, int C, float* scale, float* shift) {
  for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < C; c += gridDim.x * blockDim.x) {
    const float inv = 1.0f / sqrtf(rv[c] + eps);
    const float g = gamma ? gamma[c] : 1.f;
    scale[c] = g * inv;
    shift[c] = (beta ? beta[c] : 0.f) - rm[c] * g * inv;
  }
}

// ---------------------------------------------------------------- forward apply
// Grid-stride elementwise kernels over [M][C] bf16 in 8-channel vectors.  With 256-thread
// blocks and C/8 a power of two <= 256 (every ResNet-50 width) the stride is a multiple of C/8,
// so a thread's channel group never changes: FIXED kernels decode it once and keep the
// per-channel constants in registers (no per-vector 64-bit modulo, no per-element loads).
// mask (optional): bit e of byte i = (stored output element 8i + e > 0), the ReLU mask the
// backward needs (dfu_bn_bwd_* relu = 3) at 1/16 of the bytes of re-reading the output.
DFU_DEV unsigned positive_bits8(const u32x4 pk) {
  unsigned m = 0;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    const unsigned lo = pk[w] & 0xffffu, hi = pk[w] >> 16;
    // bf16 bits of a value > 0: +denormal .. +inf (0x0001 .. 0x7f80); not +-0, negatives, NaN
    m |= (unsigned)(lo - 1u < 0x7f80u) << (2 * w);
    m |= (unsigned)(hi - 1u < 0x7f80u) << (2 * w + 1);
  }
  return m;
}

template <bool FIXED>
__global__ void k_bn_apply(const bf16_t* __restrict__ y, const float* __restrict__ scale,
                           const float* __restrict__ shift, const bf16_t* __restrict__ res,
                           int relu, bf16_t* __restrict__ out, uint8_t* __restrict__ mask,
                           int64_t M, int C) {
  const int cv = C / 8;
  const int64_t n = M * cv;
  float sc[8], sf[8];
  auto load_coef = [&](int c0) {
    const f32x4 s0 = *(const f32x4*)(scale + c0), s1 = *(const f32x4*)(scale + c0 + 4);
    const f32x4 h0 = *(const f32x4*)(shift + c0), h1 = *(const f32x4*)(shift + c0 + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      sc[e] = s0[e]; sc[e + 4] = s1[e]; sf[e] = h0[e]; sf[e + 4] = h1[e];
    }
  };
  if (FIXED) load_coef((threadIdx.x & (cv - 1)) * 8);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    if (!FIXED) load_coef((int)(i % cv) * 8);
    float f[8];
    unpack8(*(const u32x4*)(y + i * 8), f);
    float r[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (res) unpack8(*(const u32x4*)(res + i * 8), r);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float v = fmaf(f[e], sc[e], sf[e]) + r[e];
      f[e] = relu ? fmaxf(v, 0.f) : v;
    }
    const u32x4 pk = pack8(f);
    *(u32x4*)(out + i * 8) = pk;
    if (mask) mask[i] = (uint8_t)positive_bits8(pk);
  }
}

inline bool fixed_channels(int C) {
  const int cv = C / 8;
  return cv > 0 && cv <= 256 && (cv & (cv - 1)) == 0;
}

// ---------------------------------------------------------------- backward
// Block of 256 threads = CT column-threads (8 channels each) x (256/CT) row-lanes; each thread
// keeps RED_U rows' loads in flight per iteration.  Rows per block: a multiple of
// rl_n * RED_U, grown until at most ~2048 row-blocks exist (8 per CU: the loop is latency-bound,
// parallelism is what feeds it); the sliced finalize reduces any number of them in parallel.
constexpr int RED_U = 4;
inline int bwd_rows_per_block(int64_t M, int C) {
  const int cv = C / 8;
  const int ct_n = cv < 64 ? cv : 64;
  const int rl_n = 256 / ct_n;
  int64_t rpb = (int64_t)rl_n * RED_U;
  const int64_t col_groups = cv / ct_n;
  while ((M + rpb - 1) / rpb * col_groups > 2048 && rpb < M) rpb *= 2;
  return (int)rpb;
}

// RELU: 0 none; 1 mask = out > 0 (the stored output: BN + residual + ReLU); 2 mask =
// fma(y, scale, shift) > 0, the forward's own pre-ReLU value recomputed from y (BN + ReLU with
// no residual: the same fp32 value k_bn_apply rounded, so the same mask, without reading out).
// A compile-time mode: every load of an iteration is issued before any of them is used.
template <int RELU>
DFU_DEV void relu_mask8(const float* oo, const float* yy, const float* sc, const float* sf,
                        float* g, unsigned mb = 0) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    if constexpr (RELU == 1) g[e] = oo[e] > 0.f ? g[e] : 0.f;
    if constexpr (RELU == 3) g[e] = ((mb >> e) & 1u) ? g[e] : 0.f;
    if constexpr (RELU == 2) g[e] = (fmaf(yy[e], sc[e], sf[e]) + 0.f) > 0.f ? g[e] : 0.f;
  }
}

template <int RELU>
__global__ void k_bn_bwd_reduce(const bf16_t* __restrict__ dout, const bf16_t* __restrict__ y,
                                const bf16_t* __restrict__ out,
                                const float* __restrict__ scale, const float* __restrict__ shift,
                                const float* __restrict__ mean, const float* __restrict__ invstd,
                                int64_t M, int C, int rows_per_block, float* __restrict__ partial) {
  __shared__ float red[2][256][8];
  const int cv = C / 8;
  const int ct_n = min(cv, 64);
  const int rl_n = 256 / ct_n;
  const int ct = threadIdx.x % ct_n, rl = threadIdx.x / ct_n;
  const int c8 = blockIdx.x * ct_n + ct;
  const int c0 = c8 * 8;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_block;
  const int64_t r1 = min(M, r0 + rows_per_block);
  float sg[8] = {0, 0, 0, 0, 0, 0, 0, 0}, sgx[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  float mu[8], is[8], sc[8] = {}, sf[8] = {};
#pragma unroll
  for (int e = 0; e < 8; ++e) { mu[e] = mean[c0 + e]; is[e] = invstd[c0 + e]; }
  if constexpr (RELU == 2) {
#pragma unroll
    for (int e = 0; e < 8; ++e) { sc[e] = scale[c0 + e]; sf[e] = shift[c0 + e]; }
  }
  // RED_U rows per iteration, every load of the iteration issued before any is used (rows past
  // r1 load row r0 again and are masked out of the sums)
  for (int64_t rb = r0 + rl; rb < r1; rb += (int64_t)rl_n * RED_U) {
    u32x4 gv[RED_U], yv[RED_U], ov[RED_U];
#pragma unroll
    for (int u = 0; u < RED_U; ++u) {
      const int64_t r = rb + (int64_t)u * rl_n;
      const int64_t o = (r < r1 ? r : r0) * C + c0;
      gv[u] = *(const u32x4*)(dout + o);
      yv[u] = *(const u32x4*)(y + o);
      ov[u] = (u32x4){0u, 0u, 0u, 0u};
      if constexpr (RELU == 1) ov[u] = *(const u32x4*)(out + o);
      if constexpr (RELU == 3) ov[u][0] = ((const uint8_t*)out)[o / 8];
    }
#pragma unroll
    for (int u = 0; u < RED_U; ++u) {
      if (rb + (int64_t)u * rl_n >= r1) continue;
      float g[8], yy[8], oo[8];
      unpack8(gv[u], g);
      unpack8(yv[u], yy);
      unpack8(ov[u], oo);
      relu_mask8<RELU>(oo, yy, sc, sf, g, ov[u][0]);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        sg[e] += g[e];
        sgx[e] += g[e] * (yy[e] - mu[e]) * is[e];
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) { red[0][threadIdx.x][e] = sg[e]; red[1][threadIdx.x][e] = sgx[e]; }
  __syncthreads();
  if (rl == 0) {
    for (int l = 1; l < rl_n; ++l) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        sg[e] += red[0][l * ct_n + ct][e];
        sgx[e] += red[1][l * ct_n + ct][e];
      }
    }
    float* p0 = partial + ((int64_t)blockIdx.y * 2 + 0) * C + c0;
    float* p1 = partial + ((int64_t)blockIdx.y * 2 + 1) * C + c0;
#pragma unroll
    for (int e = 0; e < 8; ++e) { p0[e] = sg[e]; p1[e] = sgx[e]; }
  }
}

// 16 waves x 64 channel-lanes per workgroup (coalesced 256-B row segments of the partials, the
// waves stride the row-blocks); fp64 sums, 16-way LDS reduction.
// Slices over the row-blocks as k_bn_finalize (blockIdx.y, last arriver sums in slice order).
__global__ __launch_bounds__(64 * FIN_WAVES) void k_bn_bwd_finalize(
    const float* __restrict__ partial, int blocks, int bps, int64_t M, int C,
    const float* __restrict__ gamma, const float* __restrict__ invstd, int batch_stats,
    float* __restrict__ dgamma, float* __restrict__ dbeta, float* __restrict__ coef,
    double* __restrict__ ws, int* __restrict__ counters) {
  __shared__ double red[2][FIN_WAVES][64];
  __shared__ int flag;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  const int S = gridDim.y;
  const int b0 = blockIdx.y * bps, b1 = min(blocks, b0 + bps);
  double sg = 0.0, sgx = 0.0;
  if (c < C) {
#pragma unroll 4
    for (int b = b0 + w; b < b1; b += FIN_WAVES) {
      sg += partial[((int64_t)b * 2 + 0) * C + c];
      sgx += partial[((int64_t)b * 2 + 1) * C + c];
    }
  }
  red[0][w][lane] = sg;
  red[1][w][lane] = sgx;
  __syncthreads();
  if (w == 0 && c < C)
    for (int k = 1; k < FIN_WAVES; ++k) { sg += red[0][k][lane]; sgx += red[1][k][lane]; }
  if (S > 1) {
    if (w == 0 && c < C) {
      st_sc1_f64(ws + ((int64_t)blockIdx.y * 2 + 0) * C + c, sg);
      st_sc1_f64(ws + ((int64_t)blockIdx.y * 2 + 1) * C + c, sgx);
    }
    if (!last_slice(counters + blockIdx.x, S, &flag)) return;
    if (w == 0 && c < C) {
      sg = sgx = 0.0;
      for (int y = 0; y < S; ++y) {
        sg += ld_sc1_f64(ws + ((int64_t)y * 2 + 0) * C + c);
        sgx += ld_sc1_f64(ws + ((int64_t)y * 2 + 1) * C + c);
      }
    }
  }
  if (w == 0 && c < C) {
    if (dbeta) dbeta[c] += (float)sg;
    if (dgamma) dgamma[c] += (float)sgx;
    const float g = gamma ? gamma[c] : 1.f;
    coef[3 * c + 0] = g * invstd[c];
    coef[3 * c + 1] = batch_stats ? (float)(sg / (double)M) : 0.f;
    coef[3 * c + 2] = batch_stats ? (float)(sgx / (double)M) : 0.f;
  }
}

// dy = k (g - m1 - xhat m2), xhat = (y - mean) invstd  ==  a g + b y + c per channel with
// a = k, b = -k m2 invstd, c = k (m2 invstd mean - m1).
template <int RELU, bool FIXED>
__global__ void k_bn_bwd_apply(const bf16_t* __restrict__ dout, const bf16_t* __restrict__ y,
                               const bf16_t* __restrict__ out,
                               const float* __restrict__ scale, const float* __restrict__ shift,
                               const float* __restrict__ mean, const float* __restrict__ invstd,
                               const float* __restrict__ coef, int64_t M, int C,
                               bf16_t* __restrict__ dy, bf16_t* __restrict__ dres) {
  const int cv = C / 8;
  const int64_t n = M * cv;
  float ka[8], kb[8], kc[8], sc[8] = {}, sf[8] = {};
  auto load_coef = [&](int c0) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int c = c0 + e;
      const float k = coef[3 * c], m1 = coef[3 * c + 1], m2 = coef[3 * c + 2];
      const float is = invstd[c];
      ka[e] = k;
      kb[e] = -k * m2 * is;
      kc[e] = k * (m2 * is * mean[c] - m1);
      if constexpr (RELU == 2) { sc[e] = scale[c]; sf[e] = shift[c]; }
    }
  };
  if (FIXED) load_coef((threadIdx.x & (cv - 1)) * 8);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    if (!FIXED) load_coef((int)(i % cv) * 8);
    float g[8], yy[8], oo[8];
    const u32x4 gv = *(const u32x4*)(dout + i * 8), yv = *(const u32x4*)(y + i * 8);
    u32x4 ov = {};
    if constexpr (RELU == 1) ov = *(const u32x4*)(out + i * 8);
    if constexpr (RELU == 3) ov[0] = ((const uint8_t*)out)[i];
    unpack8(gv, g);
    unpack8(yv, yy);
    unpack8(ov, oo);
    relu_mask8<RELU>(oo, yy, sc, sf, g, ov[0]);
    if (dres) *(u32x4*)(dres + i * 8) = pack8(g);
    float d[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) d[e] = fmaf(ka[e], g[e], fmaf(kb[e], yy[e], kc[e]));
    *(u32x4*)(dy + i * 8) = pack8(d);
  }
}

// ---------------------------------------------------------------- standalone statistics
// The (sum, M2) record per 128-row tile and channel that the GEMM's BN-statistics epilogue
// writes, computed from stored bf16 rows instead (a BatchNorm2d not fused behind a conv).
// Block = 64 channel lanes x 4 row groups of 32 rows; pass 1 sums (tile mean), pass 2 sums the
// squared deviations from it over the same rows (L1/L2-resident).
__global__ __launch_bounds__(256) void k_bn_tile_stats(const bf16_t* __restrict__ x, int M, int C,
                                                       float* __restrict__ stats) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int c = blockIdx.y * 64 + lane;
  const int r0 = blockIdx.x * 128, nb = min(128, M - r0);
  const int ra = r0 + g * 32, rb = min(r0 + nb, ra + 32);
  float v[32];
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    const int r = ra + i;
    v[i] = (c < C && r < rb) ? bf2f(x[(int64_t)r * C + c]) : 0.f;
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 32; ++i) s += v[i];
  red[g][lane] = s;
  __syncthreads();
  const float tot = red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane];
  const float mu = tot / (float)nb;
  __syncthreads();
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    const float d = ra + i < rb ? v[i] - mu : 0.f;
    q += d * d;
  }
  red[g][lane] = q;
  __syncthreads();
  if (g == 0 && c < C) {
    stats[((int64_t)blockIdx.x * 2 + 0) * C + c] = tot;
    stats[((int64_t)blockIdx.x * 2 + 1) * C + c] = red[0][lane] + red[1][lane] + red[2][lane] +
                                                    red[3][lane];
  }
}

inline unsigned grid_for(int64_t n) {
  int64_t b = (n + 255) / 256;
  if (b > 65536) b = 65536;
  return (unsigned)(b < 1 ? 1 : b);
}

}  // namespace

namespace {
constexpr int FIN_TPS = 128;  // stats tiles (or bwd row-blocks) per finalize slice
inline int fin_cpw(int C) { return C <= 64 ? 16 : (C <= 128 ? 32 : 64); }
}  // namespace

extern "C" int64_t dfu_bn_finalize_ws_bytes(int32_t tiles, int32_t C) {
  const int S = (tiles + FIN_TPS - 1) / FIN_TPS;
  return S > 1 ? (int64_t)S * 2 * C * 8 : 0;
}

extern "C" int dfu_bn_finalize(const float* stats, int32_t tiles, int32_t M, int32_t C,
                               const float* gamma, const float* beta, float eps, float momentum,
                               float* running_mean, float* running_var, int64_t* num_batches,
                               float* mean_out, float* invstd_out, float* scale_out,
                               float* shift_out, double* ws, int32_t* counters, int32_t ncounters,
                               void* stream) {
  DFU_CHECK_ARG(stats && tiles == (M + 127) / 128 && C > 0 && mean_out && invstd_out &&
                    scale_out && shift_out,
                "dfu_bn_finalize: bad args (tiles=%d M=%d)", tiles, M);
  // 16 channels per block up to C = 64, 32 up to 128, else 64; the tiles in slices of FIN_TPS
  // when a workspace and zeroed counters are given (else one slice: a long serial tile loop)
  const int cpw = fin_cpw(C);
  const int gx = (C + cpw - 1) / cpw;
  int S = (tiles + FIN_TPS - 1) / FIN_TPS;
  if (ws == nullptr || counters == nullptr || ncounters < gx) S = 1;
  const int tps = S > 1 ? FIN_TPS : tiles;
  auto kern = C <= 64 ? k_bn_finalize<16> : (C <= 128 ? k_bn_finalize<32> : k_bn_finalize<64>);
  hipLaunchKernelGGL(kern, dim3(gx, S), dim3(64 * FIN_WAVES), 0, (hipStream_t)stream, stats,
                     tiles, tps, M, C, gamma, beta, eps, momentum, running_mean, running_var,
                     num_batches, mean_out, invstd_out, scale_out, shift_out, ws, counters);
  DFU_LAUNCH_CHECK();
  return DFU_OK;
}

extern "C" int dfu_bn_tile_stats(const void* x, int64_t M, int32_t C, float* stats,
                                 void* stream) {
  DFU_CHECK_ARG(x && stats && M > 0 && M < (1ll << 31) && C > 0, "dfu_bn_tile_stats: bad args");
  hipLaunchKernelGGL(k_bn_tile_stats, dim3((unsigned)((M + 127) / 128), (C + 63) / 64), dim3(256),
                     0, (hipStream_t)stream, (const bf16_t*)x, (int)M, C, stats);
  DFU_LAUNCH_CHECK();
  return DFU_OK;
}

extern "C" int dfu_bn_eval_coeffs(const float* gamma, const float* beta, const float* running_mean,
                                  const float* running_var, float eps, int32_t C,
                                  float* scale_out, float* shift_out, void* stream) {
  DFU_CHECK_ARG(running_mean && running_var && scale_out && shift_out && C > 0,
                "dfu_bn_eval_coeffs: bad args");
  hipLaunchKernelGGL(k_bn_eval_coeffs, dim3((C + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                     gamma, beta, running_mean, running_var, eps, C, scale_out, shift_out);
  DFU_LAUNCH_CHECK();
  return DFU_OK;
}

extern "C" int dfu_bn_apply_mask(const void* y, const float* scale, const float* shift,
                                 const void* residual, int32_t relu, void* out, uint8_t* mask,
                                 int64_t M, int32_t C, void* stream) {
  DFU_CHECK_ARG(y && scale && shift && out && C % 8 == 0 && M > 0, "dfu_bn_apply: bad args");
  hipLaunchKernelGGL(fixed_channels(C) ? k_bn_apply<true> : k_bn_apply<false>,
                     dim3(grid_for(M * C / 8)), dim3(256), 0, (hipStream_t)stream,
                     (const bf16_t*)y, scale, shift, (const bf16_t*)residual, relu, (bf16_t*)out,
                     mask, M, C);
  DFU_LAUNCH_CHECK();
  return DFU_OK;
}

extern "C" int dfu_bn_apply(const void* y, const float* scale, const float* shift,
                            const void* residual, int32_t relu, void* out, int64_t M, int32_t C,
                            void* stream) {
  return dfu_bn_apply_mask(y, scale, shift, residual, relu, out, nullptr, M, C, stream);
}

extern "C" int dfu_bn_bwd_blocks(int64_t M, int32_t C) {
  const int rpb = bwd_rows_per_block(M, C);
  return (int)((M + rpb - 1) / rpb);
}

extern "C" int dfu_bn_bwd_reduce(const void* dout, const void* y, const void* out, int32_t relu,
                                 const float* scale, const float* shift, const float* mean,
                                 const float* invstd, int64_t M, int32_t C, float* partial,
                                 void* stream) {
  DFU_CHECK_ARG(dout && y && mean && invstd && partial && C % 8 == 0 && M > 0 && relu >= 0 &&
                    relu <= 3,
                "dfu_bn_bwd_reduce: bad args");
  DFU_CHECK_ARG((relu != 1 && relu != 3) || out, "dfu_bn_bwd_reduce: relu=1/3 needs out/mask");
  DFU_CHECK_ARG(relu != 2 || (scale && shift), "dfu_bn_bwd_reduce: relu=2 needs scale/shift");
  const int cv = C / 8;
  const int ct_n = cv < 64 ? cv : 64;
  DFU_CHECK_ARG(256 % ct_n == 0 && cv % ct_n == 0, "dfu_bn_bwd_reduce: C=%d unsupported", C);
  const int rpb = bwd_rows_per_block(M, C);
  dim3 grid(cv / ct_n, dfu_bn_bwd_blocks(M, C));
  auto kern = relu == 1   ? k_bn_bwd_reduce<1>
              : relu == 2 ? k_bn_bwd_reduce<2>
              : relu == 3 ? k_bn_bwd_reduce<3>
                          : k_bn_bwd_reduce<0>;
  hipLaunchKernelGGL(kern, grid, dim3(256), 0, (hipStream_t)stream, (const bf16_t*)dout,
                     (const bf16_t*)y, (const bf16_t*)out, scale, shift, mean, invstd, M, C, rpb,
                     partial);
  DFU_LAUNCH_CHECK();
  return DFU_OK;
}

extern "C" int64_t dfu_bn_bwd_finalize_ws_bytes(int32_t blocks, int32_t C) {
  const int S = (blocks + FIN_TPS - 1) / FIN_TPS;
  return S > 1 ? (int64_t)S * 2 * C * 8 : 0;
}

extern "C" int dfu_bn_bwd_finalize(const float* partial, int32_t blocks, int64_t M, int32_t C,
                                   const float* gamma, const float* invstd, int32_t batch_stats,
                                   float* dgamma, float* dbeta, float* coef, double* ws,
                                   int32_t* counters, int32_t ncounters, void* stream) {
  DFU_CHECK_ARG(partial && invstd && coef && blocks > 0 && C > 0, "dfu_bn_bwd_finalize: bad args");
  const int gx = (C + 63) / 64;
  int S = (blocks + FIN_TPS - 1) / FIN_TPS;
  if (ws == nullptr || counters == nullptr || ncounters < gx) S = 1;
  const int bps = S > 1 ? FIN_TPS : blocks;
  hipLaunchKernelGGL(k_bn_bwd_finalize, dim3(gx, S), dim3(64 * FIN_WAVES), 0, (hipStream_t)stream,
                     partial, blocks, bps, M, C, gamma, invstd, batch_stats, dgamma, dbeta, coef,
                     ws, counters);
  DFU_LAUNCH_CHECK();
  return DFU_OK;
}

// The whole BN backward in one call (reduce -> finalize -> apply, the same three launches): the
// host's per-layer cost is one C call and one workspace instead of five calls and three
// allocations (~53 BatchNorms a step).  Workspace: [finalize slices (f64)] [partial sums
// blocks x 2 x C (f32)] [coef C x 3 (f32)].
extern "C" int64_t dfu_bn_bwd_ws_bytes(int64_t M, int32_t C) {
  if (M <= 0 || C <= 0) return 0;
  const int blocks = dfu_bn_bwd_blocks(M, C);
  return dfu_bn_bwd_finalize_ws_bytes(blocks, C) + ((int64_t)blocks * 2 * C + 3LL * C) * 4;
}

extern "C" int dfu_bn_bwd(const void* dout, const void* y, const void* out, int32_t relu,
                          const float* scale, const float* shift, const float* mean,
                          const float* invstd, const float* gamma, int64_t M, int32_t C,
                          int32_t batch_stats, float* dgamma, float* dbeta, void* dy, void* dres,
                          void* ws, int64_t ws_bytes, int32_t* counters, int32_t ncounters,
                          void* stream) {
  DFU_CHECK_ARG(ws && M > 0 && C > 0 && ws_bytes >= dfu_bn_bwd_ws_bytes(M, C) &&
                    ((uintptr_t)ws & 15) == 0,
                "dfu_bn_bwd: workspace of dfu_bn_bwd_ws_bytes(M, C) bytes (16-B aligned) needed");
  const int blocks = dfu_bn_bwd_blocks(M, C);
  const int64_t fin = dfu_bn_bwd_finalize_ws_bytes(blocks, C);
  double* fws = fin > 0 ? (double*)ws : nullptr;
  float* partial = (float*)((char*)ws + fin);
  float* coef = partial + (int64_t)blocks * 2 * C;
  int rc = dfu_bn_bwd_reduce(dout, y, out, relu, scale, shift, mean, invstd, M, C, partial,
                             stream);
  if (rc != DFU_OK) return rc;
  rc = dfu_bn_bwd_finalize(partial, blocks, M, C, gamma, invstd, batch_stats, dgamma, dbeta, coef,
                           fws, fws ? counters : nullptr, fws ? ncounters : 0, stream);
  if (rc != DFU_OK) return rc;
  return dfu_bn_bwd_apply(dout, y, out, relu, scale, shift, mean, invstd, coef, M, C, dy, dres,
                          stream);
}

extern "C" int dfu_bn_bwd_apply(const void* dout, const void* y, const void* out, int32_t relu,
                                const float* scale, const float* shift, const float* mean,
                                const float* invstd, const float* coef, int64_t M, int32_t C,
                                void* dy, void* dres, void* stream) {
  DFU_CHECK_ARG(dout && y && mean && invstd && coef && dy && C % 8 == 0 && M > 0 && relu >= 0 &&
                    relu <= 3,
                "dfu_bn_bwd_apply: bad args");
  DFU_CHECK_ARG((relu != 1 && relu != 3) || out, "dfu_bn_bwd_apply: relu=1/3 needs out/mask");
  DFU_CHECK_ARG(relu != 2 || (scale && shift), "dfu_bn_bwd_apply: relu=2 needs scale/shift");
  const bool fx = fixed_channels(C);
  auto kern = relu == 1   ? (fx ? k_bn_bwd_apply<1, true> : k_bn_bwd_apply<1, false>)
              : relu == 2 ? (fx ? k_bn_bwd_apply<2, true> : k_bn_bwd_apply<2, false>)
              : relu == 3 ? (fx ? k_bn_bwd_apply<3, true> : k_bn_bwd_apply<3, false>)
                          : (fx ? k_bn_bwd_apply<0, true> : k_bn_bwd_apply<0, false>);
  hipLaunchKernelGGL(kern, dim3(grid_for(M * C / 8)), dim3(256), 0, (hipStream_t)stream,
                     (const bf16_t*)dout, (const bf16_t*)y, (const bf16_t*)out, scale, shift, mean,
                     invstd, coef, M, C, (bf16_t*)dy, (bf16_t*)dres);
  DFU_LAUNCH_CHECK();
  return DFU_OK;
}
