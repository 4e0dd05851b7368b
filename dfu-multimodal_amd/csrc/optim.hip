// Loss and optimizer of the training step:
//   weighted CrossEntropy (train_multimodal_fusion.py:342-346, 376),
//   AdamW(lr=1e-4, weight_decay=1e-4, betas (0.9, 0.999), eps 1e-8) (:347, 380),
// with the step counter kept on the device so a captured graph replays the bias correction.
#include "common.h"

namespace {

// Single block.  loss = sum_i w[y_i] * (lse_i - z_i[y_i]) / sum_i w[y_i]
__global__ void k_ce_fwd(const float* __restrict__ z, const int64_t* __restrict__ y,
                         const float* __restrict__ w, int B, int C, float* __restrict__ loss,
                         float* __restrict__ dz) {
  __shared__ float s_num[256], s_den[256];
  float num = 0.f, den = 0.f;
  for (int i = threadIdx.x; i < B; i += blockDim.x) {
    const int64_t yi = y[i];
    const float wi = (yi >= 0 && yi < C) ? (w ? w[yi] : 1.f) : 0.f;
    float mx = -INFINITY;
    for (int c = 0; c < C; ++c) mx = fmaxf(mx, z[(int64_t)i * C + c]);
    float se = 0.f;
    for (int c = 0; c < C; ++c) se += expf(z[(int64_t)i * C + c] - mx);
    const float lse = mx + logf(se);
    if (wi != 0.f) num += wi * (lse - z[(int64_t)i * C + yi]);
    den += wi;
  }
  s_num[threadIdx.x] = num;
  s_den[threadIdx.x] = den;
  __syncthreads();
  for (int s = blockDim.x / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) {
      s_num[threadIdx.x] += s_num[threadIdx.x + s];
      s_den[threadIdx.x] += s_den[threadIdx.x + s];
    }
    __syncthreads();
  }
  const float D = s_den[0];
  if (threadIdx.x == 0) loss[0] = s_num[0] / D;
  if (dz) {
    for (int i = threadIdx.x; i < B; i += blockDim.x) {
      const int64_t yi = y[i];
      const float wi = (yi >= 0 && yi < C) ? (w ? w[yi] : 1.f) : 0.f;
      float mx = -INFINITY;
      for (int c = 0; c < C; ++c) mx = fmaxf(mx, z[(int64_t)i * C + c]);
      float se = 0.f;
      for (int c = 0; c < C; ++c) se += expf(z[(int64_t)i * C + c] - mx);
      for (int c = 0; c < C; ++c) {
        const float pc = expf(z[(int64_t)i * C + c] - mx) / se;
        dz[(int64_t)i * C + c] = wi * (pc - (c == yi ? 1.f : 0.f)) / D;
      }
    }
  }
}

__global__ void k_ce_bwd(const float* __restrict__ saved, const float* __restrict__ g, int n,
                         float* __restrict__ out) {
  const float gg = g[0];
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    out[i] = saved[i] * gg;
}

struct AdamCoef {
  float step_size, bc2_sqrt_inv, decay;
};

DFU_DEV AdamCoef adam_coef(int64_t step, float lr, float b1, float b2, float wd) {
  const double t = (double)step;
  const double bc1 = 1.0 - pow((double)b1, t);
  const double bc2 = 1.0 - pow((double)b2, t);
  AdamCoef a;
  a.step_size = (float)(lr / bc1);
  a.bc2_sqrt_inv = (float)(1.0 / sqrt(bc2));
  a.decay = 1.f - lr * wd;
  return a;
}

DFU_DEV void adam_update(float& p, float g, float& m, float& v, const AdamCoef& a, float b1,
                         float b2, float eps) {
  p *= a.decay;
  m = m + (1.f - b1) * (g - m);  // lerp_(grad, 1 - beta1)
  v = v * b2 + (1.f - b2) * g * g;
  const float denom = sqrtf(v) * a.bc2_sqrt_inv + eps;
  p -= a.step_size * (m / denom);
}

// The interleaved-pair bf16x3 shadow (dfu_adamw_flat's shadow_x3): elements [x3_begin,
// x3_end) of the range, per 32-element block [hi 32 | lo 32] (hi = bf16(p), lo = bf16(p - hi)).
struct X3Shadow {
  bf16_t* base;
  int64_t begin, end;  // element range (relative to the AdamW range); begin % 4 == 0
};

// Optionally also writes the bf16 shadow of the updated parameters (the GEMM operand copy),
// so no per-step cast kernels are needed, an fp16 shadow (the "parity" precision mode's ViT
// forward operands) and the interleaved-pair split of a sub-range (its ResNet forward's conv
// weight operands: FlatParams.enable_x3).
__device__ __forceinline__ void adamw_vec4(float* __restrict__ p, const float* __restrict__ g,
                                           float* __restrict__ m, float* __restrict__ v,
                                           bf16_t* __restrict__ shadow,
                                           bf16_t* __restrict__ shadow16, const X3Shadow& x3,
                                           int64_t i, f32x4 pp,
                                           f32x4 gg, f32x4 mm, f32x4 vv, const AdamCoef& a,
                                           float b1, float b2, float eps) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    float pe = pp[e], me = mm[e], ve = vv[e];
    adam_update(pe, gg[e], me, ve, a, b1, b2, eps);
    pp[e] = pe; mm[e] = me; vv[e] = ve;
  }
  ((f32x4*)p)[i] = pp;
  ((f32x4*)m)[i] = mm;
  ((f32x4*)v)[i] = vv;
  if (shadow) ((u32x2*)shadow)[i] = (u32x2){pack2(pp[0], pp[1]), pack2(pp[2], pp[3])};
  if (shadow16) ((u32x2*)shadow16)[i] = (u32x2){pack2h(pp[0], pp[1]), pack2h(pp[2], pp[3])};
  const int64_t e = 4 * i - x3.begin;
  if (x3.base && e >= 0 && 4 * i < x3.end) {
    float hi[4], lo[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      hi[k] = bf2f(f2bf(pp[k]));
      lo[k] = pp[k] - hi[k];
    }
    bf16_t* o = x3.base + 2 * e - (e & 31);  // block e / 32 at 64 (e / 32): [hi | lo]
    *(u32x2*)o = (u32x2){pack2(hi[0], hi[1]), pack2(hi[2], hi[3])};
    *(u32x2*)(o + 32) = (u32x2){pack2(lo[0], lo[1]), pack2(lo[2], lo[3])};
  }
}

// Each thread handles ADAM_UNROLL float4 groups per grid-stride pass, spaced one grid apart so
// every wave's accesses stay contiguous; all 4 x ADAM_UNROLL loads issue before the first
// update.  The optimizer is a pure streaming pass (4 reads + 3 writes of fp32 and one bf16
// write per parameter, 30 B).  Measured on MI355X at 110.75M parameters (same box): one block
// per CU beats a wide grid by ~20% (601 vs 767 us; 4096 blocks keep 7 streams x 16 waves per
// CU fighting over HBM pages), and unrolling does not help at that grid (unroll 2/4: 656/625 us).
template <int ADAM_UNROLL>
__global__ void __launch_bounds__(256) k_adamw_flat(float* __restrict__ p,
                                                    const float* __restrict__ g,
                                                    float* __restrict__ m, float* __restrict__ v,
                                                    int64_t n, float lr, float b1, float b2,
                                                    float eps, float wd,
                                                    const int64_t* __restrict__ step_dev,
                                                    bf16_t* __restrict__ shadow,
                                                    bf16_t* __restrict__ shadow16,
                                                    const X3Shadow x3) {
  const AdamCoef a = adam_coef(*step_dev, lr, b1, b2, wd);
  const int64_t n4 = n / 4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  for (; i + (ADAM_UNROLL - 1) * stride < n4; i += ADAM_UNROLL * stride) {
    f32x4 pp[ADAM_UNROLL], gg[ADAM_UNROLL], mm[ADAM_UNROLL], vv[ADAM_UNROLL];
#pragma unroll
    for (int u = 0; u < ADAM_UNROLL; ++u) {
      const int64_t j = i + u * stride;
      gg[u] = ((const f32x4*)g)[j];
      pp[u] = ((f32x4*)p)[j];
      mm[u] = ((f32x4*)m)[j];
      vv[u] = ((f32x4*)v)[j];
    }
#pragma unroll
    for (int u = 0; u < ADAM_UNROLL; ++u)
      adamw_vec4(p, g, m, v, shadow, shadow16, x3, i + u * stride, pp[u], gg[u], mm[u], vv[u], a,
                 b1, b2, eps);
  }
  for (; i < n4; i += stride)
    adamw_vec4(p, g, m, v, shadow, shadow16, x3, i, ((f32x4*)p)[i], ((const f32x4*)g)[i],
               ((f32x4*)m)[i],
               ((f32x4*)v)[i], a, b1, b2, eps);
  for (int64_t k = n4 * 4 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < n;
       k += stride) {
    float pe = p[k], me = m[k], ve = v[k];
    adam_update(pe, g[k], me, ve, a, b1, b2, eps);
    p[k] = pe; m[k] = me; v[k] = ve;
    if (shadow) shadow[k] = f2bf(pe);
    if (shadow16) shadow16[k] = (bf16_t)(pack2h(pe, 0.f) & 0xffffu);
  }
}

// Tensor-table form: chunk c covers elements [chunk_offsets[c], chunk_offsets[c+1]) of the
// virtual concatenation; each block finds its tensor by binary search over tensor starts.
constexpr int ADAM_CHUNK = 65536;
__global__ void k_adamw_table(float* const* __restrict__ P, float* const* __restrict__ G,
                              float* const* __restrict__ M, float* const* __restrict__ V,
                              const int64_t* __restrict__ numel, int ntensors,
                              const int64_t* __restrict__ chunk_tensor, int nchunks, float lr,
                              float b1, float b2, float eps, float wd,
                              const int64_t* __restrict__ step_dev) {
  const AdamCoef a = adam_coef(*step_dev, lr, b1, b2, wd);
  for (int c = blockIdx.x; c < nchunks; c += gridDim.x) {
    // chunk_tensor[c] packs (tensor index << 32) | chunk index within the tensor
    const int64_t ct = chunk_tensor[c];
    const int t = (int)(ct >> 32);
    const int64_t start = (int64_t)(ct & 0xffffffff) * ADAM_CHUNK;
    const int64_t end = min(numel[t], start + ADAM_CHUNK);
    float* p = P[t];
    float* gp = G[t];
    float* m = M[t];
    float* v = V[t];
    for (int64_t i = start + threadIdx.x; i < end; i += blockDim.x) {
      float pe = p[i], me = m[i], ve = v[i];
      adam_update(pe, gp ? gp[i] : 0.f, me, ve, a, b1, b2, eps);
      p[i] = pe; m[i] = me; v[i] = ve;
    }
  }
}

__global__ void k_step_inc(int64_t* s) {
  if (threadIdx.x == 0 && blockIdx.x == 0) *s += 1;
}

}  // namespace

extern "C" int dfu_ce_weighted_fwd(const float* logits, const int64_t* labels, const float* weight,
                                   int32_t B, int32_t C, float* loss, float* dlogits,
                                   void* stream) {
  DFU_CHECK_ARG(logits && labels && loss && B > 0 && C > 0, "dfu_ce_weighted_fwd: bad args");
  hipLaunchKernelGGL(k_ce_fwd, dim3(1), dim3(256), 0, (hipStream_t)stream, logits, labels, weight,
                     B, C, loss, dlogits);
  DFU_LAUNCH_CHECK();
  return DFU_OK;
}

extern "C" int dfu_ce_weighted_bwd(const float* saved, const float* grad_loss, int32_t B,
                                   int32_t C, float* dlogits, void* stream) {
  DFU_CHECK_ARG(saved && grad_loss && dlogits, "dfu_ce_weighted_bwd: bad args");
  const int n = B * C;
  hipLaunchKernelGGL(k_ce_bwd, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, saved,
                     grad_loss, n, dlogits);
  DFU_LAUNCH_CHECK();
  return DFU_OK;
}

extern "C" int dfu_adamw_flat(float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                              int64_t n, float lr, float beta1, float beta2, float eps,
                              float weight_decay, const int64_t* step_dev, void* shadow_bf16,
                              void* shadow_f16, void* shadow_x3, int64_t x3_begin,
                              int64_t x3_end, void* stream) {
  DFU_CHECK_ARG(param && grad && exp_avg && exp_avg_sq && step_dev && n > 0,
                "dfu_adamw_flat: bad args");
  // the pair blocks of 32 must sit inside whole float4 groups of the range, which must cover
  // them: n % 4 == 0 there (the scalar tail writes no pairs)
  DFU_CHECK_ARG(!shadow_x3 || (x3_begin >= 0 && x3_begin % 4 == 0 && x3_end >= x3_begin &&
                               x3_end <= n / 4 * 4 && (x3_end - x3_begin) % 32 == 0 &&
                               ((uintptr_t)shadow_x3 & 7) == 0),
                "dfu_adamw_flat: x3 range [%lld, %lld) must be 4-aligned, a multiple of 32 long, "
                "inside the range's float4 groups (n=%lld)", (long long)x3_begin,
                (long long)x3_end, (long long)n);
  DFU_CHECK_ARG(((uintptr_t)param & 15) == 0 && ((uintptr_t)grad & 15) == 0 &&
                    ((uintptr_t)exp_avg & 15) == 0 && ((uintptr_t)exp_avg_sq & 15) == 0 &&
                    ((uintptr_t)shadow_bf16 & 7) == 0 && ((uintptr_t)shadow_f16 & 7) == 0,
                "dfu_adamw_flat: buffers must be 16-byte aligned (shadows 8-byte)");
  int64_t blocks = (n / 4 + 255) / 256;
  static const int64_t cap = [] {  // one block per CU (see k_adamw_flat)
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
    return (int64_t)cus;
  }();
  if (blocks > cap) blocks = cap;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(k_adamw_flat<1>, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, param,
                     grad, exp_avg, exp_avg_sq, n, lr, beta1, beta2, eps, weight_decay, step_dev,
                     (bf16_t*)shadow_bf16, (bf16_t*)shadow_f16,
                     X3Shadow{(bf16_t*)shadow_x3, x3_begin, shadow_x3 ? x3_end : 0});
  DFU_LAUNCH_CHECK();
  return DFU_OK;
}

extern "C" int dfu_adamw(float* const* params, float* const* grads, float* const* exp_avg,
                         float* const* exp_avg_sq, const int64_t* numels, int32_t ntensors,
                         const int64_t* chunk_offsets, int32_t nchunks, float lr, float beta1,
                         float beta2, float eps, float weight_decay, int64_t* step_dev,
                         void* stream) {
  DFU_CHECK_ARG(params && exp_avg && exp_avg_sq && numels && chunk_offsets && step_dev &&
                    ntensors > 0 && nchunks > 0,
                "dfu_adamw: bad args");
  const int blocks = nchunks < 8192 ? nchunks : 8192;
  hipLaunchKernelGGL(k_adamw_table, dim3(blocks), dim3(256), 0, (hipStream_t)stream, params, grads,
                     exp_avg, exp_avg_sq, numels, ntensors, chunk_offsets, nchunks, lr, beta1,
                     beta2, eps, weight_decay, step_dev);
  DFU_LAUNCH_CHECK();
  return DFU_OK;
}

extern "C" int dfu_step_increment(int64_t* step_dev, void* stream) {
  DFU_CHECK_ARG(step_dev, "dfu_step_increment: null counter");
  hipLaunchKernelGGL(k_step_inc, dim3(1), dim3(64), 0, (hipStream_t)stream, step_dev);
  DFU_LAUNCH_CHECK();
  return DFU_OK;
}
