// GPU input pipeline: the reference's per-sample torchvision transforms
// (notebooks/train_multimodal_fusion.py:172-205) on a decoded batch, bit-exact with the PIL
// backend torchvision drives for PIL images.  The host only decodes (PIL, as the reference's
// DataLoader workers do) and packs bytes; everything after decode runs here:
//   Resize((224, 224))            PIL Image.resize(BILINEAR): separable antialiased resample,
//                                 22-bit fixed-point taps, horizontal pass then vertical, each
//                                 rounded to u8 (k_resize_h, k_resize_v; taps from
//                                 dfu_resize_coeffs on the host)
//   Random{Horizontal,Vertical}Flip, RandomRotation(30), ColorJitter(0.3, 0.3, 0.3),
//   RandomAffine(20, (0.1, 0.1), (0.8, 1.2)), ToTensor, Normalize
//                                 one gather kernel per output pixel (k_augment_apply): PIL's
//                                 16.16 fixed-point nearest-neighbour affine maps (fill 0), the
//                                 ImageEnhance blends in fp32 with truncation, /255 and the
//                                 normalisation in fp32 with IEEE division -> fp32 NCHW
//   ImageEnhance.Contrast needs the mean grey level of the image it is applied to: one block
//   per image reduces it first (k_augment_stats).
// Random parameters are drawn on the host (data/gpu_transforms.py) and arrive per image as
// dfu_aug_params; all arithmetic here is integer except the blends and the normalisation.
#include <cmath>
#include <vector>

#include "common.h"

#pragma clang fp contract(off)  // the blends and the normalisation round like the CPU code

namespace {

constexpr int kPrec = 22;  // PIL Resample.c PRECISION_BITS (32 - 8 - 2)
constexpr int TPB = 256;

DFU_DEV int clip8(int s) {
  const int v = s >> kPrec;
  return v < 0 ? 0 : (v > 255 ? 255 : v);
}

// Horizontal pass: tmp[img][y][x] for every source row y, out width OW; one thread per output
// pixel, the source bytes through L1/L2 (a wave-per-row LDS-staged variant measured 1.6x
// slower: its load and compute phases do not overlap at the occupancy its LDS allows).
__global__ void k_resize_h(const uint8_t* __restrict__ src, const dfu_resize_desc* __restrict__ d,
                           const int32_t* __restrict__ coefs, int OW, uint8_t* __restrict__ tmp) {
  const dfu_resize_desc D = d[blockIdx.y];
  const int32_t* bnd = coefs + D.coef_off;
  const int32_t* kk = bnd + 2 * OW;
  const int64_t n = (int64_t)D.h * OW;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int y = (int)(i / OW), x = (int)(i % OW);
    const int xmin = bnd[2 * x], cnt = bnd[2 * x + 1];
    const int32_t* k = kk + (int64_t)x * D.ksh;
    const uint8_t* p = src + D.src_off + ((int64_t)y * D.w + xmin) * 3;
    int s0 = 1 << (kPrec - 1), s1 = s0, s2 = s0;
    for (int j = 0; j < cnt; ++j) {
      const int w = k[j];
      s0 += p[3 * j] * w;
      s1 += p[3 * j + 1] * w;
      s2 += p[3 * j + 2] * w;
    }
    uint8_t* o = tmp + D.tmp_off + i * 3;
    o[0] = (uint8_t)clip8(s0);
    o[1] = (uint8_t)clip8(s1);
    o[2] = (uint8_t)clip8(s2);
  }
}

// Vertical pass over the horizontal result: dst[img][y][x][3], OH x OW.
__global__ void k_resize_v(const uint8_t* __restrict__ tmp, const dfu_resize_desc* __restrict__ d,
                           const int32_t* __restrict__ coefs, int OW, int OH,
                           uint8_t* __restrict__ dst) {
  const dfu_resize_desc D = d[blockIdx.y];
  const int32_t* bnd = coefs + D.coef_off + 2 * OW + (int64_t)OW * D.ksh;
  const int32_t* kk = bnd + 2 * OH;
  const int n = OH * OW;
  uint8_t* out = dst + (int64_t)blockIdx.y * n * 3;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int y = i / OW, x = i % OW;
    const int ymin = bnd[2 * y], cnt = bnd[2 * y + 1];
    const int32_t* k = kk + (int64_t)y * D.ksv;
    const uint8_t* p = tmp + D.tmp_off + ((int64_t)ymin * OW + x) * 3;
    int s0 = 1 << (kPrec - 1), s1 = s0, s2 = s0;
    for (int j = 0; j < cnt; ++j) {
      const int w = k[j];
      const uint8_t* q = p + (int64_t)j * OW * 3;
      s0 += q[0] * w;
      s1 += q[1] * w;
      s2 += q[2] * w;
    }
    out[i * 3] = (uint8_t)clip8(s0);
    out[i * 3 + 1] = (uint8_t)clip8(s1);
    out[i * 3 + 2] = (uint8_t)clip8(s2);
  }
}

struct Px {
  int c[3];
};

// PIL Geometry.c affine_fixed: source = ((a2 + y*a1 + x*a0) >> 16, (a5 + y*a4 + x*a3) >> 16).
DFU_DEV bool affine_src(const int32_t* a, int x, int y, int W, int H, int& xs, int& ys) {
  xs = (a[2] + y * a[1] + x * a[0]) >> 16;
  ys = (a[5] + y * a[4] + x * a[3]) >> 16;
  return xs >= 0 && xs < W && ys >= 0 && ys < H;
}

// The flipped + rotated resized image at (x, y); rotation fill is black.
DFU_DEV Px rotated(const uint8_t* im, const dfu_aug_params& P, int W, int H, int x, int y) {
  Px p = {{0, 0, 0}};
  if (P.rotate && !affine_src(P.rot, x, y, W, H, x, y)) return p;
  if (P.hflip) x = W - 1 - x;
  if (P.vflip) y = H - 1 - y;
  const uint8_t* q = im + ((int64_t)y * W + x) * 3;
  p.c[0] = q[0];
  p.c[1] = q[1];
  p.c[2] = q[2];
  return p;
}

// PIL Convert.c rgb2l: L = (19595 R + 38470 G + 7471 B + 0x8000) >> 16.
DFU_DEV int grey(const Px& p) { return (p.c[0] * 19595 + p.c[1] * 38470 + p.c[2] * 7471 + 0x8000) >> 16; }

// PIL ImagingBlend(degenerate, image, alpha): float(in1) + alpha * float(in2 - in1), clipped
// to [0, 255] and truncated.
DFU_DEV int blend(int in1, int in2, float alpha) {
  const float t = (float)in1 + alpha * (float)(in2 - in1);
  return t <= 0.f ? 0 : (t >= 255.f ? 255 : (int)t);
}

// ColorJitter ops [0, upto) in their drawn order; `mean` is the contrast op's grey mean.
DFU_DEV Px colour(Px p, const dfu_aug_params& P, int upto, int mean) {
  for (int k = 0; k < upto; ++k) {
    const float f = P.factor[k];
    if (f == 1.f) continue;  // ImagingBlend copies the image for alpha == 1
    int deg[3];
    if (P.op[k] == DFU_AUG_BRIGHTNESS) {
      deg[0] = deg[1] = deg[2] = 0;
    } else if (P.op[k] == DFU_AUG_CONTRAST) {
      deg[0] = deg[1] = deg[2] = mean;
    } else {
      deg[0] = deg[1] = deg[2] = grey(p);
    }
    if (f == 0.f) {
      for (int c = 0; c < 3; ++c) p.c[c] = deg[c];
    } else {
      for (int c = 0; c < 3; ++c) p.c[c] = blend(deg[c], p.c[c], f);
    }
  }
  return p;
}

DFU_DEV int contrast_slot(const dfu_aug_params& P) {
  for (int k = 0; k < P.n_ops; ++k)
    if (P.op[k] == DFU_AUG_CONTRAST) return k;
  return -1;
}

// ImageEnhance.Contrast needs int(mean(L) + 0.5) of the image entering the contrast op:
// kStatBlocks blocks per image add their grey sums into sums[img] (integer atomics: the
// order does not matter).  sum <= 255 * H * W fits int32 for H * W < 8.4M.
constexpr int kStatBlocks = 8;

__global__ void __launch_bounds__(256) k_augment_stats(const uint8_t* __restrict__ img,
                                                       const dfu_aug_params* __restrict__ params,
                                                       int H, int W, int32_t* __restrict__ sums) {
  const dfu_aug_params P = params[blockIdx.y];
  const int slot = contrast_slot(P);
  if (slot < 0) return;
  const uint8_t* im = img + (int64_t)blockIdx.y * H * W * 3;
  int s = 0;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < H * W; i += gridDim.x * blockDim.x) {
    const Px p = colour(rotated(im, P, W, H, i % W, i / W), P, slot, 0);
    s += grey(p);
  }
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if ((threadIdx.x & 63) == 0) atomicAdd(sums + blockIdx.y, s);
}

__global__ void k_augment_apply(const uint8_t* __restrict__ img,
                                const dfu_aug_params* __restrict__ params,
                                const int32_t* __restrict__ means, int H, int W, float m0, float m1,
                                float m2, float s0, float s1, float s2, float* __restrict__ out) {
  const dfu_aug_params P = params[blockIdx.y];
  const uint8_t* im = img + (int64_t)blockIdx.y * H * W * 3;
  const int n = H * W;
  // == int(sum / n + 0.5), ImageStat's mean rounded as ImageEnhance.Contrast does
  const int mean = contrast_slot(P) >= 0 ? (int)((2 * (int64_t)means[blockIdx.y] + n) / (2 * (int64_t)n)) : 0;
  float* o = out + (int64_t)blockIdx.y * 3 * n;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    int x = i % W, y = i / W;
    Px p = {{0, 0, 0}};
    if (!P.affine || affine_src(P.aff, x, y, W, H, x, y))
      p = colour(rotated(im, P, W, H, x, y), P, P.n_ops, mean);
    o[i] = ((float)p.c[0] / 255.f - m0) / s0;
    o[n + i] = ((float)p.c[1] / 255.f - m1) / s1;
    o[2 * n + i] = ((float)p.c[2] / 255.f - m2) / s2;
  }
}

}  // namespace

// PIL Resample.c precompute_coeffs + normalize_coeffs_8bpc for the bilinear filter (support 1):
// kernel width of an in_size -> out_size pass.
extern "C" int dfu_resize_ksize(int32_t in_size, int32_t out_size) {
  if (in_size <= 0 || out_size <= 0) return -1;
  double filterscale = (double)in_size / out_size;
  if (filterscale < 1.0) filterscale = 1.0;
  return (int)ceil(1.0 * filterscale) * 2 + 1;
}

extern "C" int dfu_resize_coeffs(int32_t in_size, int32_t out_size, int32_t* bounds,
                                 int32_t* kk) {
  DFU_CHECK_ARG(in_size > 0 && out_size > 0 && bounds && kk, "dfu_resize_coeffs: bad args");
  const double scale = (double)in_size / out_size;
  const double filterscale = scale < 1.0 ? 1.0 : scale;
  const double support = 1.0 * filterscale;
  const int ksize = dfu_resize_ksize(in_size, out_size);
  std::vector<double> w(ksize);
  for (int xx = 0; xx < out_size; ++xx) {
    const double center = (xx + 0.5) * scale;
    const double ss = 1.0 / filterscale;
    int xmin = (int)(center - support + 0.5);
    if (xmin < 0) xmin = 0;
    int xmax = (int)(center + support + 0.5);
    if (xmax > in_size) xmax = in_size;
    xmax -= xmin;
    double ww = 0.0;
    for (int x = 0; x < xmax; ++x) {
      double t = (x + xmin - center + 0.5) * ss;
      if (t < 0) t = -t;
      w[x] = t < 1.0 ? 1.0 - t : 0.0;
      ww += w[x];
    }
    for (int x = 0; x < ksize; ++x) {
      double v = x < xmax ? (ww != 0.0 ? w[x] / ww : w[x]) : 0.0;
      kk[(int64_t)xx * ksize + x] =
          (int32_t)(v < 0 ? -0.5 + v * (1 << kPrec) : 0.5 + v * (1 << kPrec));
    }
    bounds[2 * xx] = xmin;
    bounds[2 * xx + 1] = xmax;
  }
  return DFU_OK;
}

extern "C" int dfu_resize_batch(const uint8_t* src, const dfu_resize_desc* descs,
                                const int32_t* coefs, int32_t n, int32_t out_w, int32_t out_h,
                                uint8_t* tmp, uint8_t* dst, void* stream) {
  DFU_CHECK_ARG(src && descs && coefs && tmp && dst && n > 0 && out_w > 0 && out_h > 0,
                "dfu_resize_batch: bad args");
  hipLaunchKernelGGL(k_resize_h, dim3(96, n), dim3(TPB), 0, (hipStream_t)stream, src, descs,
                     coefs, out_w, tmp);
  DFU_LAUNCH_CHECK();
  const int gx = (out_w * out_h + TPB - 1) / TPB;
  hipLaunchKernelGGL(k_resize_v, dim3(gx < 64 ? gx : 64, n), dim3(TPB), 0, (hipStream_t)stream,
                     tmp, descs, coefs, out_w, out_h, dst);
  DFU_LAUNCH_CHECK();
  return DFU_OK;
}

extern "C" int dfu_augment_normalize(const uint8_t* img, const dfu_aug_params* params, int32_t n,
                                     int32_t H, int32_t W, const float* mean3, const float* std3,
                                     int32_t* contrast_means, float* out, void* stream) {
  DFU_CHECK_ARG(img && params && mean3 && std3 && contrast_means && out && n > 0 && H > 0 &&
                    W > 0 && (int64_t)H * W * 255 < (1ll << 31),
                "dfu_augment_normalize: bad args");
  hipError_t e = hipMemsetAsync(contrast_means, 0, sizeof(int32_t) * n, (hipStream_t)stream);
  DFU_CHECK_ARG(e == hipSuccess, "dfu_augment_normalize: memset: %s", hipGetErrorString(e));
  hipLaunchKernelGGL(k_augment_stats, dim3(kStatBlocks, n), dim3(256), 0, (hipStream_t)stream,
                     img, params, H, W, contrast_means);
  DFU_LAUNCH_CHECK();
  const int gx = (H * W + TPB - 1) / TPB;
  hipLaunchKernelGGL(k_augment_apply, dim3(gx < 64 ? gx : 64, n), dim3(TPB), 0,
                     (hipStream_t)stream, img, params, contrast_means, H, W, mean3[0], mean3[1],
                     mean3[2], std3[0], std3[1], std3[2], out);
  DFU_LAUNCH_CHECK();
  return DFU_OK;
}
