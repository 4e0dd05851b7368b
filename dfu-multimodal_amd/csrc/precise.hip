// Split-bf16 forward ("bf16x3" precision mode) of the DFU fusion step.
//
// bf16 storage of the ViT/ResNet weights and activations moves the fusion logits ~2e-3 away
// from the reference's fp32 CPU path, above north_star's 1e-3 bar.  This mode
// keeps the forward pass within fp32 rounding of that path on the same MFMA GEMM kernels:
// every contraction A·Bᵀ of the forward runs as ONE bf16 GEMM over a tripled K,
//     A3 = [hi(A) | lo(A) | hi(A)],   B3 = [hi(B) | hi(B) | lo(B)]   (K' = 3K)
//     A3·B3ᵀ = hi(A)hi(B)ᵀ + lo(A)hi(B)ᵀ + hi(A)lo(B)ᵀ,
// with hi = bf16(x), lo = bf16(x - hi): |x - hi - lo| <= 2^-17 |x|, and the dropped lo·lo term
// is <= 2^-18 of |a||b|, so each product carries ~16 mantissa bits (fp32 accumulate).  For an
// implicit-GEMM convolution the tripled K is a tripled channel axis (C' = 3C: the loaders and
// the NHWC layout are unchanged).  Between kernels the forward keeps fp32 (or the triple,
// which holds hi + lo exactly): GEMM outputs leave as fp32 (F32 / F32_RESID / F32_STATS /
// PATCH epilogues), and the kernels below turn them into the next GEMM's triple while also
// writing the plain bf16 tensors the (unchanged, bf16) backward pass saves.
//
// Layout of a triple: bf16 [rows][3C], segment s at columns [sC, (s+1)C).  The ResNet's
// activations use the split-pair form instead (round 4): the plain bf16 tensor IS the hi
// buffer and a second [rows][C] buffer holds lo; the GEMM reads the tripled K from the two
// (dfu_gemm_desc.a_seg), so each BN output is written as 2 + 2 bytes instead of 6 + 2.
#include "common.h"

namespace {

constexpr int TPB = 256;

inline unsigned nblocks(int64_t n, int per_block = TPB) {
  int64_t b = (n + per_block - 1) / per_block;
  if (b > 65535 * 4) b = 65535 * 4;
  return (unsigned)(b < 1 ? 1 : b);
}

DFU_DEV void split8(const float* f, float* hi, float* lo) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    hi[e] = bf2f(f2bf(f[e]));
    lo[e] = f[e] - hi[e];
  }
}

// Store the triple of 8 values at column c of row `row` (3C columns): pattern 0 = A (hi, lo,
// hi), 1 = B (hi, hi, lo).
DFU_DEV void st_triple8(bf16_t* row, int C, int c, const float* f, int pattern) {
  float hi[8], lo[8];
  split8(f, hi, lo);
  const u32x4 h = pack8(hi), l = pack8(lo);
  *(u32x4*)(row + c) = h;
  *(u32x4*)(row + C + c) = pattern ? h : l;
  *(u32x4*)(row + 2 * C + c) = pattern ? l : h;
}

DFU_DEV void ld8_f32(const float* p, float* f) {
  const f32x4 a = *(const f32x4*)p, b = *(const f32x4*)(p + 4);
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    f[e] = a[e];
    f[e + 4] = b[e];
  }
}
DFU_DEV void st8_f32(float* p, const float* f) {
  *(f32x4*)p = (f32x4){f[0], f[1], f[2], f[3]};
  *(f32x4*)(p + 4) = (f32x4){f[4], f[5], f[6], f[7]};
}
// hi + lo of a triple's 8 values at column c (segments 0 and 1 of either pattern A row).
DFU_DEV void ld8_triple(const bf16_t* row, int C, int c, float* f) {
  float h[8], l[8];
  unpack8(*(const u32x4*)(row + c), h);
  unpack8(*(const u32x4*)(row + C + c), l);
#pragma unroll
  for (int e = 0; e < 8; ++e) f[e] = h[e] + l[e];
}

// ---------------------------------------------------------------- generic split
// fp32 [rows][cols] (any ld_in) -> triple [rows][3 seg], seg >= cols (% 8), columns past cols
// zero (the stem's 147 weight columns padded to 160).  Scalar loads (weights: any alignment).
__global__ void k_split_x3(const float* __restrict__ in, int64_t ld_in, int rows, int cols,
                           int seg, bf16_t* __restrict__ out, int pattern,
                           bf16_t* __restrict__ hi_out, int64_t ld_hi) {
  const int cv = seg / 8;
  const int64_t n = (int64_t)rows * cv;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / cv;
    const int c = (int)(i - r * cv) * 8;
    float f[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] = c + e < cols ? in[r * ld_in + c + e] : 0.f;
    if (pattern == 2) {  // interleaved pairs [rows][2 seg]: per 32 columns [hi 32 | lo 32]
      float hi[8], lo[8];
      split8(f, hi, lo);
      bf16_t* o = out + r * 2 * seg + 2 * (c & ~31) + (c & 31);
      *(u32x4*)o = pack8(hi);
      *(u32x4*)(o + 32) = pack8(lo);
    } else {
      st_triple8(out + r * 3 * seg, seg, c, f, pattern);
    }
    if (hi_out) *(u32x4*)(hi_out + r * ld_hi + c) = pack8(f);
  }
}

// fp32 OIHW conv weight -> bf16 KRSC' (pattern 1: C' = 3C, [hi | hi | lo] along channels;
// pattern 2: C' = 2C interleaved pairs, per 32 channels [hi 32 | lo 32]).
__global__ void k_pack_conv_weight_x3(const float* __restrict__ w, bf16_t* __restrict__ out, int K,
                                      int C, int R, int S, int pattern) {
  const int64_t n = (int64_t)K * R * S * C;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    int64_t t = i / C;  // (k, r, s)
    const int s = (int)(t % S);
    int64_t t2 = t / S;
    const int r = (int)(t2 % R);
    const int k = (int)(t2 / R);
    const float v = w[(((int64_t)k * C + c) * R + r) * S + s];
    const bf16_t h = f2bf(v);
    const bf16_t l = f2bf(v - bf2f(h));
    if (pattern == 2) {
      bf16_t* o = out + t * 2 * C + 2 * (c & ~31) + (c & 31);
      o[0] = h;
      o[32] = l;
    } else {
      bf16_t* o = out + t * 3 * C + c;
      o[0] = h;
      o[C] = h;
      o[2 * C] = l;
    }
  }
}

// hi = bf16(f), lo = bf16(f - hi) of 8 values into the pair buffers at element e
DFU_DEV void st_pair8(bf16_t* hi, bf16_t* lo, int64_t e, const float* f) {
  float h[8], l[8];
  split8(f, h, l);
  *(u32x4*)(hi + e) = pack8(h);
  *(u32x4*)(lo + e) = pack8(l);
}
// hi + lo of 8 values of a pair at element e
DFU_DEV void ld8_pair(const bf16_t* hi, const bf16_t* lo, int64_t e, float* f) {
  float h[8], l[8];
  unpack8(*(const u32x4*)(hi + e), h);
  unpack8(*(const u32x4*)(lo + e), l);
#pragma unroll
  for (int i = 0; i < 8; ++i) f[i] = h[i] + l[i];
}

// ---------------------------------------------------------------- BatchNorm apply
// out = act(y*scale + shift + res) from the fp32 conv output y (F32_STATS epilogue), or from
// the split pair (y = hi, y_lo = lo) that epilogue writes with aux_out (hi is then the BN
// backward's bf16 y itself, so y_bf is not written).  res_mode 0 none, 1 fp32 [M][C], 2 split
// pair (res = hi, res_lo = lo, [M][C] each).  Outputs
// (each optional): the pair hi = out_bf (the plain bf16 tensor the backward saves and the next
// convolution's hi operand) and out_lo, fp32 (a residual), y rounded to bf16 (the BN backward's
// input), and the ReLU bitmask (bit k of byte i = output element 8i + k > 0: the BN backward's
// relu = 3 mask, 1/16 of the bytes of re-reading the output; k_bn_apply's format).
__global__ void k_bn_apply_x3(const void* __restrict__ y, const bf16_t* __restrict__ y_lo,
                              const float* __restrict__ scale,
                              const float* __restrict__ shift, const void* __restrict__ res,
                              const bf16_t* __restrict__ res_lo, int res_mode, int relu,
                              bf16_t* __restrict__ out_lo, bf16_t* __restrict__ out_bf,
                              float* __restrict__ out_f32, bf16_t* __restrict__ y_bf,
                              uint8_t* __restrict__ relu_mask, int64_t M, int C, int cv_log2) {
  const int cv = C / 8;  // a power of two (every ResNet-50 width; host-checked): no division
  const int64_t n = M * cv;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = i >> cv_log2;
    const int c = (int)(i & (cv - 1)) * 8;
    const int64_t e = m * C + c;
    float f[8], r[8], sc[8], sh[8];
    {
      const f32x4 s0 = *(const f32x4*)(scale + c), s1 = *(const f32x4*)(scale + c + 4);
      const f32x4 h0 = *(const f32x4*)(shift + c), h1 = *(const f32x4*)(shift + c + 4);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        sc[k] = s0[k];
        sc[k + 4] = s1[k];
        sh[k] = h0[k];
        sh[k + 4] = h1[k];
      }
    }
    if (y_lo) {
      ld8_pair((const bf16_t*)y, y_lo, e, f);
    } else {
      ld8_f32((const float*)y + e, f);
      if (y_bf) *(u32x4*)(y_bf + e) = pack8(f);
    }
    if (res_mode == 1) ld8_f32((const float*)res + e, r);
    else if (res_mode == 2) ld8_pair((const bf16_t*)res, res_lo, e, r);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float v = fmaf(f[k], sc[k], sh[k]);
      if (res_mode) v += r[k];
      f[k] = relu ? fmaxf(v, 0.f) : v;
    }
    if (out_lo) st_pair8(out_bf, out_lo, e, f);
    else if (out_bf) *(u32x4*)(out_bf + e) = pack8(f);
    if (out_f32) st8_f32(out_f32 + e, f);
    if (relu_mask) {
      unsigned bits = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) bits |= (unsigned)(f[k] > 0.f) << k;
      relu_mask[i] = (uint8_t)bits;
    }
  }
}

// ---------------------------------------------------------------- pooling
// resnet maxpool 3x3/s2/p1 over fp32 NHWC -> split pair (plain bf16 = hi, y_lo) + argmax
// (first max in row-major window order wins, as k_maxpool_fwd).
__global__ void k_maxpool_fwd_x3(const float* __restrict__ x, int B, int H, int W, int C,
                                 bf16_t* __restrict__ y_lo, bf16_t* __restrict__ y_bf,
                                 uint8_t* __restrict__ am, int P, int Q) {
  const int cv = C / 8;
  const int64_t n = (int64_t)B * P * Q * cv;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int c8 = (int)(i % cv);
    const int64_t pix = i / cv;
    const int q = (int)(pix % Q);
    const int64_t t = pix / Q;
    const int p = (int)(t % P);
    const int b = (int)(t / P);
    float best[8];
    int arg[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) { best[e] = -INFINITY; arg[e] = 0; }
    for (int wi = 0; wi < 3; ++wi) {
      const int ih = 2 * p - 1 + wi;
      if ((unsigned)ih >= (unsigned)H) continue;
      for (int wj = 0; wj < 3; ++wj) {
        const int iw = 2 * q - 1 + wj;
        if ((unsigned)iw >= (unsigned)W) continue;
        float f[8];
        ld8_f32(x + (((int64_t)b * H + ih) * W + iw) * C + c8 * 8, f);
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (f[e] > best[e] || (f[e] != f[e] && best[e] == best[e])) {
            best[e] = f[e];
            arg[e] = wi * 3 + wj;
          }
      }
    }
    st_pair8(y_bf, y_lo, pix * C + c8 * 8, best);
    uint64_t packed = 0;
#pragma unroll
    for (int e = 0; e < 8; ++e) packed |= (uint64_t)arg[e] << (8 * e);
    *(uint64_t*)(am + pix * C + c8 * 8) = packed;
  }
}

// The stem's bn1 + ReLU + maxpool 3x3/s2/p1 in one pass over the conv output's split pair
// (y = hi, y_lo = lo; NHWC [B*H*W][C]): each window element is relu(fmaf(hi + lo, scale, shift))
// -- k_bn_apply_x3's arithmetic -- and the max / argmax are k_maxpool_fwd_x3's, so the result
// is bitwise the two-kernel path's, without its fp32 BN output (4 B written and read per conv
// output element).  The BN backward's ReLU bitmask (k_bn_apply_x3's format) is written by the
// window that owns each input element (its taps wi, wj in {1, 2}: rows 2p, 2p+1, columns 2q,
// 2q+1 -- every element once, since H <= 2P and W <= 2Q).  One thread per (output pixel,
// 8 channels); the nine taps' loads are all issued before the first compare.
__global__ __launch_bounds__(256) void k_maxpool_bn_fwd_x3(
    const bf16_t* __restrict__ yhi, const bf16_t* __restrict__ ylo,
    const float* __restrict__ scale, const float* __restrict__ shift, int B, int H, int W, int C,
    bf16_t* __restrict__ out_lo, bf16_t* __restrict__ out_bf, uint8_t* __restrict__ am,
    uint8_t* __restrict__ relu_mask, int P, int Q, int cv_log2) {
  const int cv = C >> 3;
  const int n = B * P * Q * cv;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int c8 = i & (cv - 1);
    const int pix = i >> cv_log2;
    const int q = pix % Q;
    const int t = pix / Q;
    const int p = t % P;
    const int b = t / P;
    float sc[8], sh[8];
    ld8_f32(scale + 8 * c8, sc);
    ld8_f32(shift + 8 * c8, sh);
    u32x4 hv[9], lv[9];
    int64_t eo[9];
    bool ok[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const int ih = 2 * p - 1 + k / 3, iw = 2 * q - 1 + k % 3;
      ok[k] = (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
      eo[k] = ok[k] ? ((int64_t)(b * H + ih) * W + iw) * C + 8 * c8 : 0;
      hv[k] = *(const u32x4*)(yhi + eo[k]);
      lv[k] = *(const u32x4*)(ylo + eo[k]);
    }
    float best[8];
    int arg[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) { best[e] = -INFINITY; arg[e] = 0; }
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      if (!ok[k]) continue;
      float h[8], l[8], f[8];
      unpack8(hv[k], h);
      unpack8(lv[k], l);
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] = fmaxf(fmaf(h[e] + l[e], sc[e], sh[e]), 0.f);
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (f[e] > best[e] || (f[e] != f[e] && best[e] == best[e])) {
          best[e] = f[e];
          arg[e] = k;
        }
      if (relu_mask && k / 3 >= 1 && k % 3 >= 1) {  // this window owns the element
        unsigned bits = 0;
#pragma unroll
        for (int e = 0; e < 8; ++e) bits |= (unsigned)(f[e] > 0.f) << e;
        relu_mask[eo[k] >> 3] = (uint8_t)bits;
      }
    }
    st_pair8(out_bf, out_lo, (int64_t)pix * C + 8 * c8, best);
    uint64_t packed = 0;
#pragma unroll
    for (int e = 0; e < 8; ++e) packed |= (uint64_t)arg[e] << (8 * e);
    *(uint64_t*)(am + (int64_t)pix * C + 8 * c8) = packed;
  }
}

// AdaptiveAvgPool2d(1) over a split pair (hi, lo: [B*HW][C] each) -> fp32 [B][C].
__global__ void k_avgpool_fwd_x3(const bf16_t* __restrict__ hi, const bf16_t* __restrict__ lo,
                                 int B, int HW, int C, float* __restrict__ y) {
  const int cv = C / 8;
  const int64_t n = (int64_t)B * cv;
  const float inv = 1.0f / (float)HW;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int c8 = (int)(i % cv);
    const int b = (int)(i / cv);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int t = 0; t < HW; ++t) {
      float f[8];
      ld8_pair(hi, lo, ((int64_t)b * HW + t) * C + c8 * 8, f);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += f[e];
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] *= inv;
    st8_f32(y + (int64_t)b * C + c8 * 8, acc);
  }
}

// ---------------------------------------------------------------- LayerNorm
// timm LayerNorm over fp32 rows of D (one wave per row, as k_ln_fwd) -> triple [rows][3D]
// (H16: fp16 [rows][D], the fp16 forward's GEMM operand) and plain bf16 [rows][D]; mean / rstd
// saved for the backward.
template <bool H16>
__global__ void k_ln_fwd_x3(const float* __restrict__ x, int64_t ldx, int rows, int D,
                            const float* __restrict__ gamma, const float* __restrict__ beta,
                            float eps, bf16_t* __restrict__ out3, bf16_t* __restrict__ out_bf,
                            float* __restrict__ mean_out, float* __restrict__ rstd_out) {
  constexpr int MAXV = 2;  // 8-float chunks per lane: D <= 1024
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int nv = D / 8;
  const float* xr = x + (int64_t)row * ldx;
  float v[MAXV][8];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int j = lane + 64 * i;
    if (j < nv) ld8_f32(xr + 8 * j, v[i]);
    else
#pragma unroll
      for (int e = 0; e < 8; ++e) v[i][e] = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) s += v[i][e];
  }
  const float mean = wave_sum(s) / (float)D;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int j = lane + 64 * i;
    if (j < nv)
#pragma unroll
      for (int e = 0; e < 8; ++e) { const float d = v[i][e] - mean; q += d * d; }
  }
  const float rstd = 1.0f / sqrtf(wave_sum(q) / (float)D + eps);
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int j = lane + 64 * i;
    if (j >= nv) continue;
    float g[8], b[8], o[8];
    ld8_f32(gamma + 8 * j, g);
    ld8_f32(beta + 8 * j, b);
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (v[i][e] - mean) * rstd * g[e] + b[e];
    if constexpr (H16)
      *(u32x4*)(out3 + (int64_t)row * D + 8 * j) = pack8h(o);
    else
      st_triple8(out3 + (int64_t)row * 3 * D, D, 8 * j, o, 0);
    *(u32x4*)(out_bf + (int64_t)row * D + 8 * j) = pack8(o);
  }
}

// ---------------------------------------------------------------- GELU
// h = gelu(hpre) (exact erf, timm nn.GELU) from the fp32 fc1 output -> h triple [rows][3N],
// plain bf16 h and gelu'(hpre) (the backward's fc2-wgrad operand and dGELU factor).
__global__ void k_gelu_x3(const float* __restrict__ hpre, int64_t rows, int N,
                          bf16_t* __restrict__ h3, bf16_t* __restrict__ h_bf,
                          bf16_t* __restrict__ dg_bf) {
  const int cv = N / 8;
  const int64_t n = rows * cv;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / cv;
    const int c = (int)(i - r * cv) * 8;
    float f[8], g[8], d[8];
    ld8_f32(hpre + r * N + c, f);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float cdf = 0.5f * erfcf(-f[e] * 0.70710678118654752f);
      g[e] = f[e] * cdf;
      d[e] = fmaf(f[e], 0.39894228040143268f * expf(-0.5f * f[e] * f[e]), cdf);
    }
    st_triple8(h3 + r * 3 * N, N, c, g, 0);
    *(u32x4*)(h_bf + r * N + c) = pack8(g);
    *(u32x4*)(dg_bf + r * N + c) = pack8(d);
  }
}

}  // namespace

extern "C" int dfu_split_x3(const float* in, int64_t ld_in, int32_t rows, int32_t cols,
                            int32_t seg, void* out, int32_t pattern, void* hi_out, int64_t ld_hi,
                            void* stream) {
  DFU_CHECK_ARG(in && out && rows >= 0 && cols > 0 && seg % 8 == 0 && seg >= cols &&
                    ld_in >= cols && (pattern >= 0 && pattern <= 2) &&
                    (pattern != 2 || seg % 32 == 0) &&
                    (!hi_out || (ld_hi % 8 == 0 && ld_hi >= seg)),
                "dfu_split_x3: bad args (seg %% 8 == 0, seg >= cols, pattern 0/1/2; 2: seg %% 32 == 0)");
  const int64_t n = (int64_t)rows * (seg / 8);
  if (n == 0) return DFU_OK;
  hipLaunchKernelGGL(k_split_x3, dim3(nblocks(n)), dim3(TPB), 0, (hipStream_t)stream, in, ld_in,
                     rows, cols, seg, (bf16_t*)out, pattern, (bf16_t*)hi_out, ld_hi);
  DFU_LAUNCH_CHECK();
  return DFU_OK;
}

extern "C" int dfu_pack_conv_weight_x3(const float* w, void* out, int32_t K, int32_t C, int32_t R,
                                       int32_t S, int32_t pattern, void* stream) {
  DFU_CHECK_ARG(w && out && K > 0 && C > 0 && R > 0 && S > 0 &&
                    (pattern == 1 || (pattern == 2 && C % 32 == 0)),
                "dfu_pack_conv_weight_x3: bad args (pattern 1, or 2 with C %% 32 == 0)");
  const int64_t n = (int64_t)K * R * S * C;
  hipLaunchKernelGGL(k_pack_conv_weight_x3, dim3(nblocks(n)), dim3(TPB), 0, (hipStream_t)stream,
                     w, (bf16_t*)out, K, C, R, S, pattern);
  DFU_LAUNCH_CHECK();
  return DFU_OK;
}

extern "C" int dfu_bn_apply_x3(const void* y, const void* y_lo, const float* scale,
                               const float* shift, const void* residual,
                               const void* residual_lo, int32_t res_mode,
                               int32_t relu, void* out_lo, void* out_bf16, float* out_f32,
                               void* y_bf16, uint8_t* relu_mask, int64_t M, int32_t C,
                               void* stream) {
  const int cv = C / 8;
  int cv_log2 = 0;
  while ((1 << cv_log2) < cv) ++cv_log2;
  DFU_CHECK_ARG(C % 8 == 0 && cv > 0 && (1 << cv_log2) == cv,
                "dfu_bn_apply_x3: C / 8 must be a power of two (C=%d)", C);
  DFU_CHECK_ARG((((uintptr_t)scale | (uintptr_t)shift) & 15) == 0,
                "dfu_bn_apply_x3: scale/shift must be 16-byte aligned");
  DFU_CHECK_ARG(y && scale && shift && C % 8 == 0 && M >= 0 && res_mode >= 0 && res_mode <= 2 &&
                    (res_mode == 0 || residual) && (res_mode != 2 || residual_lo) &&
                    (!out_lo || out_bf16),
                "dfu_bn_apply_x3: bad args");
  const int64_t n = M * (C / 8);
  if (n == 0) return DFU_OK;
  hipLaunchKernelGGL(k_bn_apply_x3, dim3(nblocks(n)), dim3(TPB), 0, (hipStream_t)stream, y,
                     (const bf16_t*)y_lo, scale, shift, residual, (const bf16_t*)residual_lo,
                     res_mode, relu, (bf16_t*)out_lo,
                     (bf16_t*)out_bf16, out_f32, (bf16_t*)y_bf16, relu_mask, M, C, cv_log2);
  DFU_LAUNCH_CHECK();
  return DFU_OK;
}

extern "C" int dfu_maxpool_fwd_x3(const float* x, int32_t B, int32_t H, int32_t W, int32_t C,
                                  void* y_lo, void* y_bf16, uint8_t* argmax, int32_t P, int32_t Q,
                                  void* stream) {
  DFU_CHECK_ARG(x && y_lo && y_bf16 && argmax && C % 8 == 0, "dfu_maxpool_fwd_x3: bad args");
  const int64_t n = (int64_t)B * P * Q * (C / 8);
  hipLaunchKernelGGL(k_maxpool_fwd_x3, dim3(nblocks(n)), dim3(TPB), 0, (hipStream_t)stream, x, B,
                     H, W, C, (bf16_t*)y_lo, (bf16_t*)y_bf16, argmax, P, Q);
  DFU_LAUNCH_CHECK();
  return DFU_OK;
}

extern "C" int dfu_maxpool_bn_fwd_x3(const void* y, const void* y_lo, const float* scale,
                                     const float* shift, int32_t B, int32_t H, int32_t W,
                                     int32_t C, void* out_lo, void* out_bf16, uint8_t* argmax,
                                     uint8_t* relu_mask, int32_t P, int32_t Q, void* stream) {
  const int cv = C / 8;
  int cv_log2 = 0;
  while ((1 << cv_log2) < cv) ++cv_log2;
  DFU_CHECK_ARG(y && y_lo && scale && shift && out_lo && out_bf16 && argmax && C % 8 == 0 &&
                    cv > 0 && (1 << cv_log2) == cv && P == (H - 1) / 2 + 1 &&
                    Q == (W - 1) / 2 + 1 && (int64_t)B * H * W * C < (int64_t)1 << 31 &&
                    (((uintptr_t)scale | (uintptr_t)shift) & 15) == 0,
                "dfu_maxpool_bn_fwd_x3: bad args (C / 8 a power of two, P, Q of a 3x3/s2/p1 "
                "pool, < 2^31 elements, 16-B aligned scale / shift)");
  const int64_t n = (int64_t)B * P * Q * cv;
  if (n == 0) return DFU_OK;
  hipLaunchKernelGGL(k_maxpool_bn_fwd_x3, dim3(nblocks(n)), dim3(TPB), 0, (hipStream_t)stream,
                     (const bf16_t*)y, (const bf16_t*)y_lo, scale, shift, B, H, W, C,
                     (bf16_t*)out_lo, (bf16_t*)out_bf16, argmax, relu_mask, P, Q, cv_log2);
  DFU_LAUNCH_CHECK();
  return DFU_OK;
}

extern "C" int dfu_avgpool_fwd_x3(const void* hi, const void* lo, int32_t B, int32_t HW,
                                  int32_t C, float* y, void* stream) {
  DFU_CHECK_ARG(hi && lo && y && C % 8 == 0, "dfu_avgpool_fwd_x3: bad args");
  const int64_t n = (int64_t)B * (C / 8);
  hipLaunchKernelGGL(k_avgpool_fwd_x3, dim3(nblocks(n)), dim3(TPB), 0, (hipStream_t)stream,
                     (const bf16_t*)hi, (const bf16_t*)lo, B, HW, C, y);
  DFU_LAUNCH_CHECK();
  return DFU_OK;
}

extern "C" int dfu_layernorm_fwd_x3(const float* x, int64_t ldx, int32_t rows, int32_t D,
                                    const float* gamma, const float* beta, float eps, void* out3,
                                    void* out_bf16, float* mean, float* rstd, void* stream) {
  DFU_CHECK_ARG(x && gamma && beta && out3 && out_bf16 && mean && rstd && D % 8 == 0 &&
                    D <= 1024 && ldx % 4 == 0,
                "dfu_layernorm_fwd_x3: bad args (D %% 8 == 0, D <= 1024)");
  if (rows == 0) return DFU_OK;
  const int wpb = 4;
  hipLaunchKernelGGL(k_ln_fwd_x3<false>, dim3((rows + wpb - 1) / wpb), dim3(64 * wpb), 0,
                     (hipStream_t)stream, x, ldx, rows, D, gamma, beta, eps, (bf16_t*)out3,
                     (bf16_t*)out_bf16, mean, rstd);
  DFU_LAUNCH_CHECK();
  return DFU_OK;
}

extern "C" int dfu_layernorm_fwd_h16(const float* x, int64_t ldx, int32_t rows, int32_t D,
                                     const float* gamma, const float* beta, float eps,
                                     void* out_f16, void* out_bf16, float* mean, float* rstd,
                                     void* stream) {
  DFU_CHECK_ARG(x && gamma && beta && out_f16 && out_bf16 && mean && rstd && D % 8 == 0 &&
                    D <= 1024 && ldx % 4 == 0,
                "dfu_layernorm_fwd_h16: bad args (D %% 8 == 0, D <= 1024)");
  if (rows == 0) return DFU_OK;
  const int wpb = 4;
  hipLaunchKernelGGL(k_ln_fwd_x3<true>, dim3((rows + wpb - 1) / wpb), dim3(64 * wpb), 0,
                     (hipStream_t)stream, x, ldx, rows, D, gamma, beta, eps, (bf16_t*)out_f16,
                     (bf16_t*)out_bf16, mean, rstd);
  DFU_LAUNCH_CHECK();
  return DFU_OK;
}

extern "C" int dfu_gelu_x3(const float* hpre, int64_t rows, int32_t N, void* h3, void* h_bf16,
                           void* dgelu_bf16, void* stream) {
  DFU_CHECK_ARG(hpre && h3 && h_bf16 && dgelu_bf16 && N % 8 == 0, "dfu_gelu_x3: bad args");
  const int64_t n = rows * (N / 8);
  if (n == 0) return DFU_OK;
  hipLaunchKernelGGL(k_gelu_x3, dim3(nblocks(n)), dim3(TPB), 0, (hipStream_t)stream, hpre, rows,
                     N, (bf16_t*)h3, (bf16_t*)h_bf16, (bf16_t*)dgelu_bf16);
  DFU_LAUNCH_CHECK();
  return DFU_OK;
}
