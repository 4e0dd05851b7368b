// Grad-CAM path (BASELINE.json config C5; grad_cam_visualization.py:327-429, 561-632): input
// gradients through the two stems (the training step never needs them) and the CAM / saliency
// reductions the reference does with torch ops on hooked tensors.
//   dfu_col2im_f32      adjoint of dfu_im2col_f32: resnet conv1 7x7/s2 input gradient
//   dfu_unpatchify_f32  adjoint of dfu_patchify_f32: ViT patch_embed.proj input gradient
//   dfu_gradcam         w_c = mean_p grad; cam = relu(sum_c w_c act); cam /= max cam (:415-429)
//   dfu_saliency        mean_c |dx|, / max (the ViT fallback, :401-413)
#include "common.h"

namespace {

constexpr int TPB = 256;

inline unsigned grid_for(int64_t n) {
  int64_t b = (n + TPB - 1) / TPB;
  if (b > 65536) b = 65536;
  return (unsigned)(b < 1 ? 1 : b);
}

// dx[b][c][h][w] = sum over the taps (r, s) whose output (oh, ow) reads (h, w) of
// dcol[(b, oh, ow)][c*R*S + r*S + s]; one thread per input element (a gather: no atomics, a
// fixed summation order r-major, s-minor).
__global__ void k_col2im_f32(const float* __restrict__ dcol, int B, int C, int H, int W, int R,
                             int S, int stride, int pad, int P, int Q, int Kp,
                             float* __restrict__ dx) {
  const int64_t n = (int64_t)B * C * H * W;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int w = (int)(i % W);
    int64_t t = i / W;
    const int h = (int)(t % H);
    t /= H;
    const int c = (int)(t % C);
    const int b = (int)(t / C);
    float s = 0.f;
    for (int r = 0; r < R; ++r) {
      const int hh = h + pad - r;
      if (hh < 0 || hh % stride) continue;
      const int oh = hh / stride;
      if (oh >= P) continue;
      for (int q = 0; q < S; ++q) {
        const int ww = w + pad - q;
        if (ww < 0 || ww % stride) continue;
        const int ow = ww / stride;
        if (ow >= Q) continue;
        s += dcol[((int64_t)(b * P + oh) * Q + ow) * Kp + (c * R + r) * S + q];
      }
    }
    dx[i] = s;
  }
}

// Non-overlapping patches: a permutation, dx[b][c][h][w] = dpatch[(b, h/ps, w/ps)][(c, h%ps, w%ps)].
__global__ void k_unpatchify_f32(const float* __restrict__ dp, int B, int C, int H, int W, int ps,
                                 float* __restrict__ dx) {
  const int gh = H / ps, gw = W / ps, K = C * ps * ps;
  const int64_t n = (int64_t)B * C * H * W;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int w = (int)(i % W);
    int64_t t = i / W;
    const int h = (int)(t % H);
    t /= H;
    const int c = (int)(t % C);
    const int b = (int)(t / C);
    dx[i] = dp[((int64_t)(b * gh + h / ps) * gw + w / ps) * K + (c * ps + h % ps) * ps + w % ps];
  }
}

DFU_DEV float ld_any(const void* p, int64_t i, int bf) {
  return bf ? bf2f(((const bf16_t*)p)[i]) : ((const float*)p)[i];
}

DFU_DEV float block_max(float v, float* sh) {
  v = wave_max(v);
  const int wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if ((threadIdx.x & 63) == 0) sh[wave] = v;
  __syncthreads();
  float m = sh[0];
  for (int k = 1; k < nw; ++k) m = fmaxf(m, sh[k]);
  __syncthreads();
  return m;
}

// One workgroup per image.  act element (b, p, c) at b*sab + p*sap + c*sac (an NCHW or
// channels_last view of the hooked (B, Ca, h, w) output), grad likewise with (Cg, sgb, sgp, sgc).
// Weights come from the Cg gradient channels and the map runs over the first min(Ca, Cg)
// activation channels: the reference's "channel mismatch" branch (:418-422).  Its hooks reach
// that branch on a torchvision Bottleneck, whose `relu` runs three times per block: the stored
// activation is the last call's output (2048 channels), the stored gradient the FIRST call's
// (the 512-wide conv1 output), because tensor hooks fire in reverse order.  cam: [B][HW] fp32.
__global__ __launch_bounds__(256) void k_gradcam(const void* __restrict__ act, int Ca,
                                                 int64_t sab, int64_t sap, int64_t sac,
                                                 const void* __restrict__ grad, int Cg,
                                                 int64_t sgb, int64_t sgp, int64_t sgc, int bf,
                                                 int HW, float* __restrict__ cam) {
  extern __shared__ float shm[];  // [Cg] weights, [HW] cam, [4] reduction
  float* wts = shm;
  float* cm = shm + Cg;
  float* red = cm + HW;
  const int b = blockIdx.x;
  for (int c = threadIdx.x; c < Cg; c += blockDim.x) {  // weights = gradients.mean(dim=(2, 3))
    float s = 0.f;
    for (int p = 0; p < HW; ++p) s += ld_any(grad, b * sgb + p * sgp + c * sgc, bf);
    wts[c] = s / (float)HW;
  }
  __syncthreads();
  const int nc = Ca < Cg ? Ca : Cg;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int p = wave; p < HW; p += nw) {  // cam[p] = sum_c w_c * act[c][p], then ReLU
    float s = 0.f;
    for (int c = lane; c < nc; c += 64) s += wts[c] * ld_any(act, b * sab + p * sap + c * sac, bf);
    s = wave_sum(s);
    if (lane == 0) cm[p] = fmaxf(s, 0.f);
  }
  __syncthreads();
  float mx = 0.f;
  for (int p = threadIdx.x; p < HW; p += blockDim.x) mx = fmaxf(mx, cm[p]);
  mx = block_max(mx, red);
  const float inv = mx > 0.f ? 1.f / mx : 1.f;
  for (int p = threadIdx.x; p < HW; p += blockDim.x)
    cam[(int64_t)b * HW + p] = mx > 0.f ? cm[p] * inv : cm[p];
}

// One workgroup per image: s[p] = mean_c |dx[b][c][p]|, then / max if max > 0.
__global__ __launch_bounds__(1024) void k_saliency(const float* __restrict__ dx, int C, int HW,
                                                   float* __restrict__ out) {
  __shared__ float red[16];
  const float* x = dx + (int64_t)blockIdx.x * C * HW;
  float* o = out + (int64_t)blockIdx.x * HW;
  float mx = 0.f;
  for (int p = threadIdx.x; p < HW; p += blockDim.x) {
    float s = 0.f;
    for (int c = 0; c < C; ++c) s += fabsf(x[(int64_t)c * HW + p]);
    s /= (float)C;
    o[p] = s;
    mx = fmaxf(mx, s);
  }
  mx = block_max(mx, red);
  if (mx > 0.f) {
    const float inv = 1.f / mx;
    for (int p = threadIdx.x; p < HW; p += blockDim.x) o[p] *= inv;
  }
}

}  // namespace

extern "C" int dfu_col2im_f32(const float* dcol, int32_t B, int32_t C, int32_t H, int32_t W,
                              int32_t R, int32_t S, int32_t stride, int32_t pad, int32_t P,
                              int32_t Q, int32_t Kp, float* dx, void* stream) {
  DFU_CHECK_ARG(dcol && dx && B > 0 && C > 0 && R > 0 && S > 0 && stride > 0 && Kp >= C * R * S,
                "dfu_col2im_f32: bad args");
  DFU_CHECK_ARG(P == (H + 2 * pad - R) / stride + 1 && Q == (W + 2 * pad - S) / stride + 1,
                "dfu_col2im_f32: bad P/Q");
  const int64_t n = (int64_t)B * C * H * W;
  hipLaunchKernelGGL(k_col2im_f32, dim3(grid_for(n)), dim3(TPB), 0, (hipStream_t)stream, dcol,
                     B, C, H, W, R, S, stride, pad, P, Q, Kp, dx);
  DFU_LAUNCH_CHECK();
  return DFU_OK;
}

extern "C" int dfu_unpatchify_f32(const float* dpatch, int32_t B, int32_t C, int32_t H,
                                  int32_t W, int32_t ps, float* dx, void* stream) {
  DFU_CHECK_ARG(dpatch && dx && ps > 0 && H % ps == 0 && W % ps == 0,
                "dfu_unpatchify_f32: bad patch size %d for %dx%d", ps, H, W);
  const int64_t n = (int64_t)B * C * H * W;
  hipLaunchKernelGGL(k_unpatchify_f32, dim3(grid_for(n)), dim3(TPB), 0, (hipStream_t)stream,
                     dpatch, B, C, H, W, ps, dx);
  DFU_LAUNCH_CHECK();
  return DFU_OK;
}

extern "C" int dfu_gradcam(const void* act, int32_t Ca, int64_t sab, int64_t sap, int64_t sac,
                           const void* grad, int32_t Cg, int64_t sgb, int64_t sgp, int64_t sgc,
                           int32_t is_bf16, int32_t B, int32_t HW, float* cam, void* stream) {
  DFU_CHECK_ARG(act && grad && cam && B > 0 && HW > 0 && Ca > 0 && Cg > 0,
                "dfu_gradcam: bad args");
  const size_t lds = (size_t)(Cg + HW + 4) * sizeof(float);
  DFU_CHECK_ARG(lds <= 64 * 1024, "dfu_gradcam: C + HW too large (%d + %d)", Cg, HW);
  hipLaunchKernelGGL(k_gradcam, dim3(B), dim3(256), lds, (hipStream_t)stream, act, Ca, sab, sap,
                     sac, grad, Cg, sgb, sgp, sgc, is_bf16, HW, cam);
  DFU_LAUNCH_CHECK();
  return DFU_OK;
}

extern "C" int dfu_saliency(const float* dx, int32_t B, int32_t C, int32_t HW, float* out,
                            void* stream) {
  DFU_CHECK_ARG(dx && out && B > 0 && C > 0 && HW > 0, "dfu_saliency: bad args");
  hipLaunchKernelGGL(k_saliency, dim3(B), dim3(1024), 0, (hipStream_t)stream, dx, C, HW, out);
  DFU_LAUNCH_CHECK();
  return DFU_OK;
}
