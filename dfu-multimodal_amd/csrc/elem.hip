// Layout, pooling and elementwise kernels of the DFU training step (HBM-bound; every kernel
// moves 16-B vectors per lane).  Reference ops replaced are named per entry point in
// include/dfu_hip.h.
#include "common.h"

namespace {

constexpr int TPB = 256;

inline unsigned nblocks(int64_t n, int per_block = TPB) {
  int64_t b = (n + per_block - 1) / per_block;
  return (unsigned)(b < 1 ? 1 : b);
}

// ---------------------------------------------------------------- weight packing
__global__ void k_pack_conv_weight(const float* __restrict__ w, bf16_t* __restrict__ out, int K,
                                   int C, int R, int S) {
  const int64_t n = (int64_t)K * R * S * C;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    // out index i = ((k*R + r)*S + s)*C + c
    int c = (int)(i % C);
    int64_t t = i / C;
    int s = (int)(t % S);
    t /= S;
    int r = (int)(t % R);
    int k = (int)(t / R);
    out[i] = f2bf(w[(((int64_t)k * C + c) * R + r) * S + s]);
  }
}

// oihw[k][c][r][s] += krsc[k][r][s][c]; one thread per OIHW element (coalesced writes).
__global__ void k_conv_grad_krsc_to_oihw(const float* __restrict__ krsc, float* __restrict__ oihw,
                                         int K, int C, int R, int S) {
  const int64_t n = (int64_t)K * C * R * S;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int s = (int)(i % S);
    int64_t t = i / S;
    const int r = (int)(t % R);
    t /= R;
    const int c = (int)(t % C);
    const int k = (int)(t / C);
    oihw[i] += krsc[(((int64_t)k * R + r) * S + s) * C + c];
  }
}

__global__ void k_cast_rows_bf16(const float* __restrict__ in, int64_t ld_in,
                                 bf16_t* __restrict__ out, int64_t ld_out, int rows, int cols) {
  const int64_t n = (int64_t)rows * ld_out;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / ld_out;
    const int c = (int)(i - r * ld_out);
    out[i] = c < cols ? f2bf(in[r * ld_in + c]) : (bf16_t)0;
  }
}

__global__ void k_cast_rows_f16(const float* __restrict__ in, int64_t ld_in,
                                bf16_t* __restrict__ out, int64_t ld_out, int rows, int cols) {
  const int64_t n = (int64_t)rows * ld_out;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / ld_out;
    const int c = (int)(i - r * ld_out);
    out[i] = c < cols ? (bf16_t)(pack2h(in[r * ld_in + c], 0.f) & 0xffffu) : (bf16_t)0;
  }
}

__global__ void k_cast_rows_f32(const bf16_t* __restrict__ in, int64_t ld_in,
                                float* __restrict__ out, int64_t ld_out, int rows, int cols) {
  const int64_t n = (int64_t)rows * cols;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / cols;
    const int c = (int)(i - r * cols);
    out[r * ld_out + c] = bf2f(in[r * ld_in + c]);
  }
}

// ---------------------------------------------------------------- stem im2col / patchify
// 8 values as the split-bf16 triple of csrc/precise.hip: hi | lo | hi, segments C apart.
DFU_DEV void store_triple8(bf16_t* row, int C, int c, const float* f) {
  float hi[8], lo[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    hi[e] = bf2f(f2bf(f[e]));
    lo[e] = f[e] - hi[e];
  }
  const u32x4 h = pack8(hi);
  *(u32x4*)(row + c) = h;
  *(u32x4*)(row + C + c) = pack8(lo);
  *(u32x4*)(row + 2 * C + c) = h;
}
// 8 values as a split pair (csrc/precise.hip): hi at hi[e], lo = bf16(f - hi) at lo[e]
DFU_DEV void store_pair8(bf16_t* hi, bf16_t* lo, int64_t e, const float* f) {
  float h[8], l[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    h[i] = bf2f(f2bf(f[i]));
    l[i] = f[i] - h[i];
  }
  *(u32x4*)(hi + e) = pack8(h);
  *(u32x4*)(lo + e) = pack8(l);
}

// out[m][k], m = (b, oh, ow), k = c*R*S + r*S + s; each thread writes one 16-B vector (8 k).
// Stem im2col: fp32 NCHW input -> bf16 [B*P*Q][Kp] rows, k = (c, r, s) (OIHW weight order),
// zero-padded to Kp.  Each thread owns one 16-byte chunk kv of the row (its 8 taps decoded
// once); a block of VPR*RPB threads covers RPB consecutive rows per iteration, so a wave's
// stores are contiguous row bytes.  One division per row decodes (b, oh, ow).
// X3: the split pair (hi rows in out, lo rows in out_lo, both row stride Kp; csrc/precise.hip).
template <int VPR, bool X3 = false>
__global__ __launch_bounds__(VPR * 16) void k_im2col_f32(
    const float* __restrict__ x, int64_t sn, int64_t sc, int64_t sh, int64_t sw, int B, int C,
    int H, int W, int R, int S, int stride, int pad, int P, int Q, bf16_t* __restrict__ out,
    bf16_t* __restrict__ out_lo = nullptr) {
  constexpr int RPB = 16;
  constexpr int Kp = VPR * 8;
  const int kv = threadIdx.x % VPR, rsub = threadIdx.x / VPR;
  const int KK = C * R * S;
  int tc[8], tr[8], ts[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int k = kv * 8 + e;
    const int c = k / (R * S), rs = k - (k / (R * S)) * (R * S);
    tc[e] = k < KK ? c : -1;
    tr[e] = rs / S;
    ts[e] = rs - (rs / S) * S;
  }
  const int rows = B * P * Q;
  for (int m = blockIdx.x * RPB + rsub; m < rows; m += gridDim.x * RPB) {
    const int b = m / (P * Q);
    const int rem = m - b * P * Q;
    const int oh = rem / Q, ow = rem - (rem / Q) * Q;
    const int ih0 = oh * stride - pad, iw0 = ow * stride - pad;
    const float* xb = x + b * sn;
    float f[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int ih = ih0 + tr[e], iw = iw0 + ts[e];
      const bool ok = tc[e] >= 0 && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
      f[e] = ok ? xb[tc[e] * sc + ih * sh + iw * sw] : 0.f;
    }
    if constexpr (X3) {
      store_pair8(out, out_lo, (int64_t)m * Kp + kv * 8, f);
    } else {
      *(u32x4*)(out + (int64_t)m * Kp + kv * 8) = pack8(f);
    }
  }
}

// Any Kp (a standalone conv with few input channels, nn.Conv2d): one thread per 16-B output
// vector, taps decoded per vector.
__global__ __launch_bounds__(256) void k_im2col_f32_any(
    const float* __restrict__ x, int64_t sn, int64_t sc, int64_t sh, int64_t sw, int B, int C,
    int H, int W, int R, int S, int stride, int pad, int P, int Q, int Kp,
    bf16_t* __restrict__ out) {
  const int vpr = Kp / 8, RS = R * S, KK = C * RS;
  const int64_t n = (int64_t)B * P * Q * vpr;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = i / vpr;
    const int kv = (int)(i - m * vpr);
    const int b = (int)(m / ((int64_t)P * Q));
    const int rem = (int)(m - (int64_t)b * P * Q);
    const int oh = rem / Q, ow = rem - (rem / Q) * Q;
    const int ih0 = oh * stride - pad, iw0 = ow * stride - pad;
    const float* xb = x + b * sn;
    float f[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int k = kv * 8 + e;
      const int c = k / RS, rs = k - (k / RS) * RS;
      const int ih = ih0 + rs / S, iw = iw0 + (rs - (rs / S) * S);
      const bool ok = k < KK && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
      f[e] = ok ? xb[c * sc + ih * sh + iw * sw] : 0.f;
    }
    *(u32x4*)(out + m * Kp + kv * 8) = pack8(f);
  }
}

// The same rows staged through LDS: one block per output row (b, oh) loads the C x R input rows
// that row's windows touch (rows outside the image as zeros) with coalesced fp32 reads, then
// writes the Q x Kp output row segment with 16-B stores.  A thread owns one 8-tap chunk kv of
// the row (its taps' LDS row offsets and columns decoded once, kept in registers) and walks the
// output positions ow = lane group, + 256 / VPR, ...; no division in either loop.  The gather
// kernel above issues 8 scattered global reads per 16-B store and ran at ~1.3 TB/s of output.
template <bool X3>
__global__ __launch_bounds__(256) void k_im2col_lds(
    const float* __restrict__ x, int64_t sn, int64_t sc, int64_t sh, int64_t sw, int B, int C,
    int H, int W, int R, int S, int stride, int pad, int P, int Q, int Kp,
    bf16_t* __restrict__ out, bf16_t* __restrict__ out_lo = nullptr) {
  extern __shared__ float tile[];  // [C * R][W]
  const int KK = C * R * S;
  const int VPR = Kp / 8;
  const int groups = 256 / VPR;  // output positions in flight per block
  const int kv = threadIdx.x % VPR, og = threadIdx.x / VPR;
  int off[8], tsx[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int k = kv * 8 + e;
    const int c = k / (R * S), rs = k - c * (R * S);
    const int r = rs / S;
    off[e] = k < KK ? (c * R + r) * W : -1;
    tsx[e] = rs - r * S;
  }
  const int CR = C * R;
  const int64_t ldo = Kp;
  for (int row = blockIdx.x; row < B * P; row += gridDim.x) {
    const int b = row / P, oh = row - b * P;
    __syncthreads();  // the previous row's gathers are done
    // every input row's load issued before any is stored (W <= 256, C * R <= 24: host-checked)
    const float* xb = x + b * sn;
    const int iw = threadIdx.x;
    float v[24];
#pragma unroll
    for (int cr = 0; cr < 24; ++cr) {
      v[cr] = 0.f;
      if (cr < CR) {
        const int c = cr / R, r = cr - c * R;
        const int ih = oh * stride - pad + r;
        if ((unsigned)ih < (unsigned)H && iw < W) v[cr] = xb[c * sc + (int64_t)ih * sh + iw * sw];
      }
    }
#pragma unroll
    for (int cr = 0; cr < 24; ++cr)
      if (cr < CR && iw < W) tile[cr * W + iw] = v[cr];
    __syncthreads();
    if (og >= groups) continue;
    const int64_t orow = (int64_t)row * Q * ldo + kv * 8;
    for (int ow = og; ow < Q; ow += groups) {
      const int iw0 = ow * stride - pad;
      float f[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int iw = iw0 + tsx[e];
        f[e] = (off[e] >= 0 && (unsigned)iw < (unsigned)W) ? tile[off[e] + iw] : 0.f;
      }
      if constexpr (X3) {
        store_pair8(out, out_lo, orow + ow * ldo, f);
      } else {
        *(u32x4*)(out + orow + ow * ldo) = pack8(f);
      }
    }
  }
}

// VEC: unit-stride rows with 16-byte aligned 8-float runs (two float4 loads per thread; the
// host checks); the vector count fits 32 bits (host-checked), so the index math is 32-bit.
template <bool X3 = false, bool VEC = false>
__global__ void k_patchify_f32(const float* __restrict__ x, int64_t sn, int64_t sc, int64_t sh,
                               int64_t sw, int B, int C, int H, int W, int ps,
                               bf16_t* __restrict__ out) {
  const int gh = H / ps, gw = W / ps;
  const int K = C * ps * ps;
  const int vec_per_row = K / 8;
  const int n = B * gh * gw * vec_per_row;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int m = i / vec_per_row;
    const int kv = i - m * vec_per_row;
    const int b = m / (gh * gw);
    const int pidx = m - b * gh * gw;
    const int py = pidx / gw, px = pidx - (pidx / gw) * gw;
    const int k0 = kv * 8;
    const int c = k0 / (ps * ps);
    const int rem = k0 - c * ps * ps;
    const int kh = rem / ps, kw0 = rem - (rem / ps) * ps;  // ps % 8 == 0: 8 consecutive kw
    const float* src = x + b * sn + c * sc + (py * ps + kh) * sh + (px * ps + kw0) * sw;
    float f[8];
    if constexpr (VEC) {
      const f32x4 a = *(const f32x4*)src, a2 = *(const f32x4*)(src + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        f[e] = a[e];
        f[4 + e] = a2[e];
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] = src[e * sw];
    }
    if constexpr (X3) {
      store_triple8(out + m * 3 * K, K, k0, f);
    } else {
      *(u32x4*)(out + m * K + k0) = pack8(f);
    }
  }
}

// ---------------------------------------------------------------- max / avg pooling
// 3x3 / stride 2 / pad 1 (torchvision resnet maxpool; first max in row-major window order wins,
// as ATen's max_pool2d_with_indices) on one output row per blockIdx.y = (b, p): 32-bit index
// math only (a grid-stride form decoding (b, p, q, c8) with 64-bit divisions per vector ran
// 110 us on the stem's 64 x 112 x 112 x 64 input).  BN:
// the input is the stem conv output y and every window element is first mapped to the value
// k_bn_apply would have stored, bf16(relu(fma(y, scale, shift) + 0)) (bn.hip), so the pooled
// output and argmax equal maxpool(bn_apply(y)) bit for bit without the BN output in HBM.
template <bool BN>
__global__ __launch_bounds__(256) void k_maxpool_rows(const bf16_t* __restrict__ x,
                                                      const float* __restrict__ scale,
                                                      const float* __restrict__ shift, int H,
                                                      int W, int C, bf16_t* __restrict__ y,
                                                      uint8_t* __restrict__ am, int P, int Q) {
  const int cv = C / 8;
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= Q * cv) return;
  const int b = blockIdx.y / P, p = blockIdx.y - b * P;
  const int q = t / cv, c8 = t - q * cv;
  float sc[8], sf[8];
  if constexpr (BN) {
#pragma unroll
    for (int e = 0; e < 8; ++e) { sc[e] = scale[c8 * 8 + e]; sf[e] = shift[c8 * 8 + e]; }
  }
  float best[8];
  int arg[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { best[e] = -INFINITY; arg[e] = 0; }
  const bf16_t* xb = x + (int64_t)b * H * W * C + c8 * 8;
  // all nine window loads issued first (out-of-image taps read a clamped in-image address and
  // are skipped below), so they are in flight together
  u32x4 win[9];
#pragma unroll
  for (int wi = 0; wi < 3; ++wi)
#pragma unroll
    for (int wj = 0; wj < 3; ++wj) {
      const int ih = min(max(2 * p - 1 + wi, 0), H - 1);
      const int iw = min(max(2 * q - 1 + wj, 0), W - 1);
      win[wi * 3 + wj] = *(const u32x4*)(xb + (int64_t)(ih * W + iw) * C);
    }
#pragma unroll
  for (int wi = 0; wi < 3; ++wi) {
    const int ih = 2 * p - 1 + wi;
    if ((unsigned)ih >= (unsigned)H) continue;
#pragma unroll
    for (int wj = 0; wj < 3; ++wj) {
      const int iw = 2 * q - 1 + wj;
      if ((unsigned)iw >= (unsigned)W) continue;
      float f[8];
      unpack8(win[wi * 3 + wj], f);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        if constexpr (BN) f[e] = bf2f(f2bf(fmaxf(fmaf(f[e], sc[e], sf[e]) + 0.f, 0.f)));
        if (f[e] > best[e] || (f[e] != f[e] && best[e] == best[e])) {
          best[e] = f[e];
          arg[e] = wi * 3 + wj;
        }
      }
    }
  }
  const int64_t o = ((int64_t)blockIdx.y * Q + q) * C + c8 * 8;
  *(u32x4*)(y + o) = pack8(best);
  uint64_t packed = 0;
#pragma unroll
  for (int e = 0; e < 8; ++e) packed |= (uint64_t)arg[e] << (8 * e);
  *(uint64_t*)(am + o) = packed;
}

// Backward, one input row pair per blockIdx.y = (b, h / 2): a thread owns the 2 x 2 input
// pixels (2i .. 2i+1, 2j .. 2j+1) of one 8-channel group.  Every one of them can only be the
// argmax of the windows (p, q) in {i, i+1} x {j, j+1} (window p covers rows 2p-1 .. 2p+1), so
// the thread loads those four windows' dy and argmax once (not once per pixel) and each pixel
// sums the windows whose argmax it is in row-major window order (deterministic; the same
// order and values as a per-pixel gather).
__global__ __launch_bounds__(256) void k_maxpool_bwd_2x2(const bf16_t* __restrict__ dy,
                                                         const uint8_t* __restrict__ am, int H,
                                                         int W, int C, int P, int Q,
                                                         bf16_t* __restrict__ dx) {
  const int cv = C / 8;
  const int W2 = (W + 1) / 2, H2 = (H + 1) / 2;
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= W2 * cv) return;
  const int b = blockIdx.y / H2, i = blockIdx.y - b * H2;
  const int j = t / cv, c8 = t - j * cv;
  uint64_t a4[4];
  u32x4 g4[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {  // every load from a clamped address; invalid windows skipped
    const int p = min(i + (k >> 1), P - 1), q = min(j + (k & 1), Q - 1);
    const int64_t o = (((int64_t)b * P + p) * Q + q) * C + c8 * 8;
    a4[k] = *(const uint64_t*)(am + o);
    g4[k] = *(const u32x4*)(dy + o);
  }
  float f4[4][8];
#pragma unroll
  for (int k = 0; k < 4; ++k) unpack8(g4[k], f4[k]);
#pragma unroll
  for (int dh = 0; dh < 2; ++dh)
#pragma unroll
    for (int dw = 0; dw < 2; ++dw) {
      const int h = 2 * i + dh, w = 2 * j + dw;
      if (h >= H || w >= W) continue;
      float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int p = i + (k >> 1), q = j + (k & 1);
        const int wi = h - (2 * p - 1), wj = w - (2 * q - 1);
        if (p >= P || q >= Q || wi < 0 || wi > 2 || wj < 0 || wj > 2) continue;
        const int want = wi * 3 + wj;
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if ((int)((a4[k] >> (8 * e)) & 0xff) == want) acc[e] += f4[k][e];
      }
      *(u32x4*)(dx + (((int64_t)b * H + h) * W + w) * C + c8 * 8) = pack8(acc);
    }
}

__global__ void k_avgpool_fwd(const bf16_t* __restrict__ x, int B, int HW, int C,
                              float* __restrict__ y) {
  const int cv = C / 8;
  const int64_t n = (int64_t)B * cv;
  const float inv = 1.0f / (float)HW;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int c8 = (int)(i % cv);
    const int b = (int)(i / cv);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const bf16_t* src = x + (int64_t)b * HW * C + c8 * 8;
    for (int t = 0; t < HW; ++t) {
      float f[8];
      unpack8(*(const u32x4*)(src + (int64_t)t * C), f);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += f[e];
    }
    float* dst = y + (int64_t)b * C + c8 * 8;
    *(f32x4*)dst = (f32x4){acc[0] * inv, acc[1] * inv, acc[2] * inv, acc[3] * inv};
    *(f32x4*)(dst + 4) = (f32x4){acc[4] * inv, acc[5] * inv, acc[6] * inv, acc[7] * inv};
  }
}

__global__ void k_avgpool_bwd(const float* __restrict__ dy, int B, int HW, int C,
                              bf16_t* __restrict__ dx) {
  const int cv = C / 8;
  const int64_t n = (int64_t)B * HW * cv;
  const float inv = 1.0f / (float)HW;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int c8 = (int)(i % cv);
    const int64_t pix = i / cv;
    const int b = (int)(pix / HW);
    const float* g = dy + (int64_t)b * C + c8 * 8;
    float f[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] = g[e] * inv;
    *(u32x4*)(dx + pix * C + c8 * 8) = pack8(f);
  }
}

// ---------------------------------------------------------------- column sums (bias grads)
// Block = 64 column-threads (8 columns each = 512 columns) x 4 row-lanes; ROWS rows per block.
constexpr int CS_ROWS = 64;  // rows per partial (same box, ViT bias grads: 128 rows 55 us, 64 rows 47, 32 rows 51 for N = 768+2304+3072)
template <bool BF>
__global__ void k_colsum(const void* __restrict__ xv, int64_t ld, int rows, int N,
                         float* __restrict__ partial) {
  __shared__ float red[4][512];
  const int ct = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int col = blockIdx.x * 512 + ct * 8;
  const int r0 = blockIdx.y * CS_ROWS;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (col < N) {
#pragma unroll 8
    for (int r = r0 + rl; r < min(rows, r0 + CS_ROWS); r += 4) {
      if constexpr (BF) {
        const bf16_t* x = (const bf16_t*)xv + (int64_t)r * ld + col;
        if (col + 8 <= N) {
          float f[8];
          unpack8(*(const u32x4*)x, f);
#pragma unroll
          for (int e = 0; e < 8; ++e) acc[e] += f[e];
        } else {
          for (int e = 0; e < 8 && col + e < N; ++e) acc[e] += bf2f(x[e]);
        }
      } else {
        const float* x = (const float*)xv + (int64_t)r * ld + col;
        for (int e = 0; e < 8 && col + e < N; ++e) acc[e] += x[e];
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) red[rl][ct * 8 + e] = acc[e];
  __syncthreads();
  if (rl == 0 && col < N) {
    for (int e = 0; e < 8 && col + e < N; ++e) {
      const float s = red[0][ct * 8 + e] + red[1][ct * 8 + e] + red[2][ct * 8 + e] +
                      red[3][ct * 8 + e];
      partial[(int64_t)blockIdx.y * N + col + e] = s;
    }
  }
}

// out_v[d] += sum_b partial[b][v][d]; 32 block-lanes x 8 columns per workgroup.
__global__ void k_reduce_partials(const float* __restrict__ partial, int blocks, int nvec, int D,
                                  float* __restrict__ out0, float* __restrict__ out1) {
  __shared__ float red[32][8];
  const int cl = threadIdx.x & 7, bl = threadIdx.x >> 3;
  const int64_t i = (int64_t)blockIdx.x * 8 + cl;  // flattened (v, d)
  const bool ok = i < (int64_t)nvec * D;
  float s = 0.f;
  if (ok) {
    // loads issued 8 ahead, added in the same order (bitwise the same sum)
    const int64_t st = (int64_t)nvec * D;
#pragma unroll 8
    for (int b = bl; b < blocks; b += 32) s += partial[(int64_t)b * st + i];
  }
  red[bl][cl] = s;
  __syncthreads();
  if (bl == 0 && ok) {
    for (int l = 1; l < 32; ++l) s += red[l][cl];
    const int v = (int)(i / D);
    const int d = (int)(i - (int64_t)v * D);
    float* o = v == 0 ? out0 : out1;
    if (o) o[d] += s;
  }
}

// ---------------------------------------------------------------- rows gather / scatter
__global__ void k_gather_rows(const float* __restrict__ in, int64_t ld_in, int stride, int offset,
                              int rows, int D, float* __restrict__ out, int64_t ld_out) {
  const int64_t n = (int64_t)rows * D;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int r = (int)(i / D);
    const int d = (int)(i - (int64_t)r * D);
    out[(int64_t)r * ld_out + d] = in[((int64_t)r * stride + offset) * ld_in + d];
  }
}
__global__ void k_scatter_rows(const float* __restrict__ in, int64_t ld_in, int stride, int offset,
                               int rows, int D, float* __restrict__ out, int64_t ld_out) {
  const int64_t n = (int64_t)rows * D;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int r = (int)(i / D);
    const int d = (int)(i - (int64_t)r * D);
    out[((int64_t)r * stride + offset) * ld_out + d] += in[(int64_t)r * ld_in + d];
  }
}

// ---------------------------------------------------------------- relu / dropout
template <bool BF>
__global__ void k_relu_fwd(const void* __restrict__ x, void* __restrict__ y, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    if constexpr (BF) {
      const bf16_t v = ((const bf16_t*)x)[i];
      ((bf16_t*)y)[i] = (v & 0x8000) ? (bf16_t)0 : v;
    } else {
      ((float*)y)[i] = fmaxf(((const float*)x)[i], 0.f);
    }
  }
}
template <bool BF>
__global__ void k_relu_bwd(const void* __restrict__ dy, const void* __restrict__ y,
                           void* __restrict__ dx, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    if constexpr (BF) {
      const float yy = bf2f(((const bf16_t*)y)[i]);
      ((bf16_t*)dx)[i] = yy > 0.f ? ((const bf16_t*)dy)[i] : (bf16_t)0;
    } else {
      const float yy = ((const float*)y)[i];
      ((float*)dx)[i] = yy > 0.f ? ((const float*)dy)[i] : 0.f;
    }
  }
}

DFU_DEV uint32_t hash_u32(uint64_t seed, uint64_t ctr) {
  // splitmix64 finaliser on (seed ^ counter): counter-based, stateless, graph-replay safe
  uint64_t z = seed + 0x9E3779B97F4A7C15ull * (ctr + 1);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (uint32_t)(z >> 32);
}

template <bool BF>
__global__ void k_dropout_fwd(const void* __restrict__ x, void* __restrict__ y,
                              uint8_t* __restrict__ mask, int64_t n, float p, uint64_t seed,
                              const int64_t* __restrict__ offset_dev) {
  const uint64_t base = (uint64_t)(*offset_dev);
  const float scale = 1.0f / (1.0f - p);
  const uint32_t thr = (uint32_t)fminf(p * 4294967296.0f, 4294967295.0f);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const bool keep = hash_u32(seed, base + (uint64_t)i) >= thr;
    mask[i] = keep ? 1 : 0;
    if constexpr (BF) {
      ((bf16_t*)y)[i] = f2bf(keep ? bf2f(((const bf16_t*)x)[i]) * scale : 0.f);
    } else {
      ((float*)y)[i] = keep ? ((const float*)x)[i] * scale : 0.f;
    }
  }
}
__global__ void k_advance(int64_t* off, int64_t n) {
  if (threadIdx.x == 0 && blockIdx.x == 0) *off += n;
}
template <bool BF>
__global__ void k_dropout_bwd(const void* __restrict__ dy, const uint8_t* __restrict__ mask,
                              void* __restrict__ dx, int64_t n, float p) {
  const float scale = 1.0f / (1.0f - p);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const bool keep = mask[i] != 0;
    if constexpr (BF) {
      ((bf16_t*)dx)[i] = f2bf(keep ? bf2f(((const bf16_t*)dy)[i]) * scale : 0.f);
    } else {
      ((float*)dx)[i] = keep ? ((const float*)dy)[i] * scale : 0.f;
    }
  }
}

// ---------------------------------------------------------------- concat / split
__global__ void k_concat2(const void* __restrict__ a, int a_bf, int Na, const void* __restrict__ b,
                          int b_bf, int Nb, int rows, bf16_t* __restrict__ out) {
  const int N = Na + Nb;
  const int64_t n = (int64_t)rows * N;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int r = (int)(i / N);
    const int c = (int)(i - (int64_t)r * N);
    float v;
    if (c < Na) v = a_bf ? bf2f(((const bf16_t*)a)[(int64_t)r * Na + c]) : ((const float*)a)[(int64_t)r * Na + c];
    else v = b_bf ? bf2f(((const bf16_t*)b)[(int64_t)r * Nb + c - Na]) : ((const float*)b)[(int64_t)r * Nb + c - Na];
    out[i] = f2bf(v);
  }
}
__global__ void k_split2(const void* __restrict__ g, int g_bf, int rows, int Na, int Nb,
                         float* __restrict__ ga, float* __restrict__ gb) {
  const int N = Na + Nb;
  const int64_t n = (int64_t)rows * N;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int r = (int)(i / N);
    const int c = (int)(i - (int64_t)r * N);
    const float v = g_bf ? bf2f(((const bf16_t*)g)[i]) : ((const float*)g)[i];
    if (c < Na) { if (ga) ga[(int64_t)r * Na + c] = v; }
    else if (gb) gb[(int64_t)r * Nb + c - Na] = v;
  }
}

// ---------------------------------------------------------------- ViT embedding
__global__ void k_vit_cls_rows(const float* __restrict__ cls, const float* __restrict__ pos,
                               float* __restrict__ x, int B, int T, int D) {
  const int64_t n = (int64_t)B * D;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int b = (int)(i / D);
    const int d = (int)(i - (int64_t)b * D);
    x[(int64_t)b * T * D + d] = cls[d] + pos[d];
  }
}
// one thread per (t, d): sum over the batch
__global__ void k_vit_embed_bwd(const float* __restrict__ gx, int B, int T, int D,
                                float* __restrict__ dcls, float* __restrict__ dpos,
                                bf16_t* __restrict__ gpatch, float* __restrict__ partial) {
  const int64_t n = (int64_t)T * D;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int t = (int)(i / D);
    const int d = (int)(i - (int64_t)t * D);
    float s = 0.f;
    // eight images' loads in flight before their stores (a load issued behind a store would
    // wait for it: vmcnt retires in issue order); the sum keeps the image order
    constexpr int U = 8;
    for (int b0 = 0; b0 < B; b0 += U) {
      float v[U];
#pragma unroll
      for (int u = 0; u < U; ++u)
        v[u] = b0 + u < B ? gx[((int64_t)(b0 + u) * T + t) * D + d] : 0.f;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (b0 + u >= B) break;
        s += v[u];
        if (t > 0) gpatch[((int64_t)(b0 + u) * (T - 1) + t - 1) * D + d] = f2bf(v[u]);
      }
    }
    if (dpos) dpos[i] += s;
    if (t == 0) {
      if (dcls) dcls[d] += s;
      partial[i] = 0.f;
    } else {
      partial[i] = s;
    }
  }
}
// out[d] += sum_t partial[t][d]: 16 columns x 16 row lanes per block (lane r sums rows r, r + 16,
// ..., then the 16 lane sums are added in r order), D / 16 blocks.
constexpr int SRA_C = 16, SRA_R = 16;
__global__ __launch_bounds__(SRA_C * SRA_R) void k_sum_rows_add(const float* __restrict__ partial,
                                                                int T, int D,
                                                                float* __restrict__ out) {
  __shared__ float red[SRA_R][SRA_C];
  const int c = threadIdx.x % SRA_C, r = threadIdx.x / SRA_C;
  const int d = blockIdx.x * SRA_C + c;
  float s = 0.f;
  if (d < D) {
#pragma unroll 4
    for (int t = r; t < T; t += SRA_R) s += partial[(int64_t)t * D + d];
  }
  red[r][c] = s;
  __syncthreads();
  if (r == 0 && d < D) {
    float a = 0.f;
    for (int k = 0; k < SRA_R; ++k) a += red[k][c];
    out[d] += a;
  }
}

__global__ void k_argmax_rows(const float* __restrict__ x, int rows, int C,
                              int64_t* __restrict__ out) {
  for (int r = blockIdx.x * blockDim.x + threadIdx.x; r < rows; r += gridDim.x * blockDim.x) {
    int best = 0;
    float bv = x[(int64_t)r * C];
    for (int c = 1; c < C; ++c) {
      const float v = x[(int64_t)r * C + c];
      if (v > bv) { bv = v; best = c; }
    }
    out[r] = best;
  }
}

// torch.softmax(outputs, dim=1) of the reference's test phase (train_multimodal_fusion.py:477):
// out[r][c] = exp(x[r][c] - max_r) / sum_c' exp(x[r][c'] - max_r), fp32 with expf.
__global__ void k_softmax_rows(const float* __restrict__ x, int rows, int C,
                               float* __restrict__ out) {
  for (int r = blockIdx.x * blockDim.x + threadIdx.x; r < rows; r += gridDim.x * blockDim.x) {
    const float* xr = x + (int64_t)r * C;
    float mx = xr[0];
    for (int c = 1; c < C; ++c) mx = fmaxf(mx, xr[c]);
    float s = 0.f;
    for (int c = 0; c < C; ++c) s += expf(xr[c] - mx);
    const float inv = 1.0f / s;
    for (int c = 0; c < C; ++c) out[(int64_t)r * C + c] = expf(xr[c] - mx) * inv;
  }
}

inline unsigned grid_for(int64_t n) {
  int64_t b = (n + TPB - 1) / TPB;
  if (b > 65536) b = 65536;
  return (unsigned)(b < 1 ? 1 : b);
}

// Per-step training metrics kept on the device (train_multimodal_fusion.py:383-388 does
// loss.item(), torch.max(outputs, 1) and .cpu() every step): confusion[label][argmax] += 1 per
// row (first maximum wins, as torch.max) and, from one lane, loss_sum += loss, batches += 1.
// Integer atomics and a single-lane fp64 add: the totals are exact and order-independent.
__global__ void k_metrics_accumulate(const float* __restrict__ logits,
                                     const int64_t* __restrict__ labels, int rows, int C,
                                     const float* __restrict__ loss,
                                     unsigned long long* __restrict__ confusion,
                                     double* __restrict__ loss_sum,
                                     unsigned long long* __restrict__ batches) {
  for (int r = blockIdx.x * blockDim.x + threadIdx.x; r < rows; r += gridDim.x * blockDim.x) {
    int best = 0;
    float bv = logits[(int64_t)r * C];
    for (int c = 1; c < C; ++c) {
      const float v = logits[(int64_t)r * C + c];
      if (v > bv) { bv = v; best = c; }
    }
    const int64_t y = labels[r];
    if (y >= 0 && y < C) atomicAdd(confusion + y * C + best, 1ull);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (loss) *loss_sum += (double)*loss;
    *batches += 1ull;
  }
}

// Up to DFU_REDUCE_BATCH independent "sum the per-block partials into a gradient vector"
// reductions in ONE launch (a ViT block's backward has eight: two LayerNorms' dgamma / dbeta and
// four bias column sums).  Block j works on entry e = the one whose [first_block, +ceil(D/8))
// range holds j, 8 columns x 32 row-lanes as k_reduce_partials, same summation order.
struct ReduceBatch {
  const float* partial[DFU_REDUCE_BATCH];
  int64_t stride[DFU_REDUCE_BATCH];
  float* out[DFU_REDUCE_BATCH];
  int blocks[DFU_REDUCE_BATCH];
  int D[DFU_REDUCE_BATCH];
  int first[DFU_REDUCE_BATCH + 1];
  int n;
};

__global__ void k_reduce_partials_batch(const ReduceBatch b) {
  __shared__ float red[32][8];
  int e = 0;
  while (e + 1 < b.n && (int)blockIdx.x >= b.first[e + 1]) ++e;
  const int cl = threadIdx.x & 7, bl = threadIdx.x >> 3;
  const int d = ((int)blockIdx.x - b.first[e]) * 8 + cl;
  const bool ok = d < b.D[e];
  const float* p = b.partial[e];
  const int64_t st = b.stride[e];
  float s = 0.f;
  if (ok) {
#pragma unroll 8
    for (int r = bl; r < b.blocks[e]; r += 32) s += p[(int64_t)r * st + d];
  }
  red[bl][cl] = s;
  __syncthreads();
  if (bl == 0 && ok) {
    for (int l = 1; l < 32; ++l) s += red[l][cl];
    b.out[e][d] += s;
  }
}

}  // namespace

// k_patchify_f32's vector form: unit-stride rows, 16-byte aligned 8-float runs
inline bool patchify_vec(const float* x, int64_t sn, int64_t sc, int64_t sh, int64_t sw) {
  return sw == 1 && ((uintptr_t)x & 15) == 0 && sn % 4 == 0 && sc % 4 == 0 && sh % 4 == 0;
}

#define LAUNCH(kern, n, stream, ...)                                                     \
  do {                                                                                   \
    hipLaunchKernelGGL(kern, dim3(grid_for(n)), dim3(TPB), 0, (hipStream_t)(stream),     \
                       __VA_ARGS__);                                                     \
    DFU_LAUNCH_CHECK();                                                                  \
  } while (0)

extern "C" int dfu_pack_conv_weight(const float* w, void* out, int32_t K, int32_t C, int32_t R,
                                    int32_t S, void* stream) {
  DFU_CHECK_ARG(w && out && K > 0 && C > 0 && R > 0 && S > 0, "dfu_pack_conv_weight: bad args");
  LAUNCH(k_pack_conv_weight, (int64_t)K * C * R * S, stream, w, (bf16_t*)out, K, C, R, S);
  return DFU_OK;
}

extern "C" int dfu_conv_grad_krsc_to_oihw(const float* krsc, float* oihw, int32_t K, int32_t C,
                                          int32_t R, int32_t S, void* stream) {
  DFU_CHECK_ARG(krsc && oihw && K > 0 && C > 0 && R > 0 && S > 0, "dfu_conv_grad_krsc_to_oihw: bad args");
  LAUNCH(k_conv_grad_krsc_to_oihw, (int64_t)K * C * R * S, stream, krsc, oihw, K, C, R, S);
  return DFU_OK;
}

// Batched bf16 transpose (include/dfu_hip.h dfu_transpose_bf16): one 256-thread workgroup per
// 64x64 tile; the tile goes through LDS as 16-B row chunks and leaves as 16-B column chunks
// (row stride 65 dwords of bf16 pairs: the column reads of a 16-lane group hit distinct banks).
__global__ __launch_bounds__(256) void k_transpose_bf16(const dfu_transpose_job* __restrict__ jobs,
                                                        int njobs) {
  __shared__ uint16_t t[64][66];
  const int tile = blockIdx.x;
  int j = 0;
  while (j + 1 < njobs && jobs[j + 1].tile0 <= tile) ++j;
  const dfu_transpose_job jb = jobs[j];
  const int tn = (jb.cols + 63) / 64;
  const int lt = tile - jb.tile0;
  const int r0 = (lt / tn) * 64, c0 = (lt % tn) * 64;
  const uint16_t* src = (const uint16_t*)jb.src;
  uint16_t* dst = (uint16_t*)jb.dst;
  const int64_t lds = jb.ld_src ? jb.ld_src : jb.cols, ldd = jb.ld_dst ? jb.ld_dst : jb.rows;
#pragma unroll
  for (int h = 0; h < 2; ++h) {  // 64 rows x 8 chunks of 8 columns
    const int q = threadIdx.x + 256 * h;
    const int r = q >> 3, cc = (q & 7) * 8;
    if (r0 + r < jb.rows && c0 + cc < jb.cols) {
      const u32x4 v = *(const u32x4*)(src + (int64_t)(r0 + r) * lds + c0 + cc);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        t[r][cc + 2 * e] = (uint16_t)(v[e] & 0xffffu);
        t[r][cc + 2 * e + 1] = (uint16_t)(v[e] >> 16);
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int h = 0; h < 2; ++h) {  // 64 dst rows (src columns) x 8 chunks of 8 src rows
    const int q = threadIdx.x + 256 * h;
    const int c = q >> 3, rr = (q & 7) * 8;
    if (c0 + c < jb.cols && r0 + rr < jb.rows) {
      u32x4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e)
        v[e] = (uint32_t)t[rr + 2 * e][c] | ((uint32_t)t[rr + 2 * e + 1][c] << 16);
      *(u32x4*)(dst + (int64_t)(c0 + c) * ldd + r0 + rr) = v;
    }
  }
}

extern "C" int dfu_transpose_bf16(const dfu_transpose_job* jobs, int32_t njobs, int32_t ntiles,
                                  void* stream) {
  DFU_CHECK_ARG(jobs && njobs > 0 && ntiles > 0, "dfu_transpose_bf16: bad args");
  hipLaunchKernelGGL(k_transpose_bf16, dim3(ntiles), dim3(256), 0, (hipStream_t)stream, jobs,
                     njobs);
  DFU_LAUNCH_CHECK();
  return DFU_OK;
}

extern "C" int dfu_cast_rows_bf16(const float* in, int64_t ld_in, void* out, int64_t ld_out,
                                  int32_t rows, int32_t cols, void* stream) {
  DFU_CHECK_ARG(in && out && rows > 0 && cols > 0 && ld_out >= cols && ld_in >= cols,
                "dfu_cast_rows_bf16: bad args");
  LAUNCH(k_cast_rows_bf16, (int64_t)rows * ld_out, stream, in, ld_in, (bf16_t*)out, ld_out, rows,
         cols);
  return DFU_OK;
}

extern "C" int dfu_cast_rows_f16(const float* in, int64_t ld_in, void* out, int64_t ld_out,
                                 int32_t rows, int32_t cols, void* stream) {
  DFU_CHECK_ARG(in && out && rows > 0 && cols > 0 && ld_out >= cols && ld_in >= cols,
                "dfu_cast_rows_f16: bad args");
  LAUNCH(k_cast_rows_f16, (int64_t)rows * ld_out, stream, in, ld_in, (bf16_t*)out, ld_out, rows,
         cols);
  return DFU_OK;
}

extern "C" int dfu_cast_rows_f32(const void* in, int64_t ld_in, float* out, int64_t ld_out,
                                 int32_t rows, int32_t cols, void* stream) {
  DFU_CHECK_ARG(in && out && rows > 0 && cols > 0, "dfu_cast_rows_f32: bad args");
  LAUNCH(k_cast_rows_f32, (int64_t)rows * cols, stream, (const bf16_t*)in, ld_in, out, ld_out,
         rows, cols);
  return DFU_OK;
}

// The LDS-staged kernel when the C x R input rows of one output row fit (the stem: 3 x 7 x 224
// fp32 = 18.4 KiB); the per-chunk gather otherwise.
static bool im2col_lds_fits(int C, int R, int W, int Kp) {
  return Kp <= 256 * 8 / 2 && C * R <= 24 && W <= 256 && (int64_t)C * R * W * 4 <= 48 * 1024;
}

extern "C" int dfu_im2col_f32(const float* x, int64_t sn, int64_t sc, int64_t sh, int64_t sw,
                              int32_t B, int32_t C, int32_t H, int32_t W, int32_t R, int32_t S,
                              int32_t stride, int32_t pad, int32_t P, int32_t Q, void* out,
                              int32_t Kp, void* stream) {
  DFU_CHECK_ARG(x && out && Kp % 8 == 0 && Kp >= C * R * S, "dfu_im2col_f32: bad Kp=%d", Kp);
  DFU_CHECK_ARG(((uintptr_t)out & 15) == 0, "dfu_im2col_f32: out must be 16-B aligned");
  const int64_t rows = (int64_t)B * P * Q;
  DFU_CHECK_ARG(rows < (1ll << 31), "dfu_im2col_f32: too many rows");
  hipStream_t st = (hipStream_t)stream;
  if (im2col_lds_fits(C, R, W, Kp)) {
    hipLaunchKernelGGL(k_im2col_lds<false>, dim3(B * P), dim3(256), (size_t)C * R * W * 4, st, x,
                       sn, sc, sh, sw, B, C, H, W, R, S, stride, pad, P, Q, Kp, (bf16_t*)out);
    DFU_LAUNCH_CHECK();
    return DFU_OK;
  }
  const int blocks = (int)((rows + 15) / 16 < 8192 ? (rows + 15) / 16 : 8192);
  switch (Kp) {
    case 160:
      hipLaunchKernelGGL(k_im2col_f32<20>, dim3(blocks), dim3(320), 0, st, x, sn, sc, sh, sw, B,
                         C, H, W, R, S, stride, pad, P, Q, (bf16_t*)out);
      break;
    default: {
      const int64_t n = rows * (Kp / 8);
      const unsigned g = (unsigned)((n + 255) / 256 < 65536 ? (n + 255) / 256 : 65536);
      hipLaunchKernelGGL(k_im2col_f32_any, dim3(g), dim3(256), 0, st, x, sn, sc, sh, sw, B, C, H,
                         W, R, S, stride, pad, P, Q, Kp, (bf16_t*)out);
    }
  }
  DFU_LAUNCH_CHECK();
  return DFU_OK;
}

extern "C" int dfu_patchify_f32(const float* x, int64_t sn, int64_t sc, int64_t sh, int64_t sw,
                                int32_t B, int32_t C, int32_t H, int32_t W, int32_t ps, void* out,
                                void* stream) {
  DFU_CHECK_ARG(x && out && ps % 8 == 0 && H % ps == 0 && W % ps == 0,
                "dfu_patchify_f32: bad patch size %d for %dx%d", ps, H, W);
  const int64_t n = (int64_t)B * (H / ps) * (W / ps) * (C * ps * ps / 8);
  DFU_CHECK_ARG(n < (1ll << 31), "dfu_patchify_f32: too many vectors");
  if (patchify_vec(x, sn, sc, sh, sw))
    LAUNCH((k_patchify_f32<false, true>), n, stream, x, sn, sc, sh, sw, B, C, H, W, ps, (bf16_t*)out);
  else
    LAUNCH((k_patchify_f32<false, false>), n, stream, x, sn, sc, sh, sw, B, C, H, W, ps, (bf16_t*)out);
  return DFU_OK;
}

extern "C" int dfu_im2col_f32_x3(const float* x, int64_t sn, int64_t sc, int64_t sh, int64_t sw,
                                 int32_t B, int32_t C, int32_t H, int32_t W, int32_t R, int32_t S,
                                 int32_t stride, int32_t pad, int32_t P, int32_t Q, void* out,
                                 void* out_lo, int32_t Kp, void* stream) {
  DFU_CHECK_ARG(x && out && out_lo && Kp == 160 && Kp >= C * R * S, "dfu_im2col_f32_x3: bad Kp=%d",
                Kp);
  DFU_CHECK_ARG(((uintptr_t)out & 15) == 0 && ((uintptr_t)out_lo & 15) == 0,
                "dfu_im2col_f32_x3: out and out_lo must be 16-B aligned");
  const int64_t rows = (int64_t)B * P * Q;
  DFU_CHECK_ARG(rows < (1ll << 31), "dfu_im2col_f32_x3: too many rows");
  if (im2col_lds_fits(C, R, W, Kp)) {
    hipLaunchKernelGGL(k_im2col_lds<true>, dim3(B * P), dim3(256), (size_t)C * R * W * 4,
                       (hipStream_t)stream, x, sn, sc, sh, sw, B, C, H, W, R, S, stride, pad, P, Q,
                       Kp, (bf16_t*)out, (bf16_t*)out_lo);
    DFU_LAUNCH_CHECK();
    return DFU_OK;
  }
  const int blocks = (int)((rows + 15) / 16 < 8192 ? (rows + 15) / 16 : 8192);
  hipLaunchKernelGGL((k_im2col_f32<20, true>), dim3(blocks), dim3(320), 0, (hipStream_t)stream,
                     x, sn, sc, sh, sw, B, C, H, W, R, S, stride, pad, P, Q, (bf16_t*)out,
                     (bf16_t*)out_lo);
  DFU_LAUNCH_CHECK();
  return DFU_OK;
}

extern "C" int dfu_patchify_f32_x3(const float* x, int64_t sn, int64_t sc, int64_t sh, int64_t sw,
                                   int32_t B, int32_t C, int32_t H, int32_t W, int32_t ps,
                                   void* out, void* stream) {
  DFU_CHECK_ARG(x && out && ps % 8 == 0 && H % ps == 0 && W % ps == 0,
                "dfu_patchify_f32_x3: bad patch size %d for %dx%d", ps, H, W);
  const int64_t n = (int64_t)B * (H / ps) * (W / ps) * (C * ps * ps / 8);
  DFU_CHECK_ARG(n < (1ll << 31), "dfu_patchify_f32_x3: too many vectors");
  if (patchify_vec(x, sn, sc, sh, sw))
    LAUNCH((k_patchify_f32<true, true>), n, stream, x, sn, sc, sh, sw, B, C, H, W, ps, (bf16_t*)out);
  else
    LAUNCH((k_patchify_f32<true, false>), n, stream, x, sn, sc, sh, sw, B, C, H, W, ps, (bf16_t*)out);
  return DFU_OK;
}

extern "C" int dfu_maxpool_fwd(const void* x, int32_t B, int32_t H, int32_t W, int32_t C, void* y,
                               uint8_t* argmax, int32_t P, int32_t Q, void* stream) {
  return dfu_maxpool_bn_fwd(x, nullptr, nullptr, B, H, W, C, y, argmax, P, Q, stream);
}

extern "C" int dfu_maxpool_bn_fwd(const void* x, const float* scale, const float* shift, int32_t B,
                                  int32_t H, int32_t W, int32_t C, void* y, uint8_t* argmax,
                                  int32_t P, int32_t Q, void* stream) {
  DFU_CHECK_ARG(x && y && argmax && C % 8 == 0, "dfu_maxpool_fwd: C %% 8 != 0");
  DFU_CHECK_ARG(P == (H - 1) / 2 + 1 && Q == (W - 1) / 2 + 1, "dfu_maxpool_fwd: bad P/Q");
  DFU_CHECK_ARG((scale == nullptr) == (shift == nullptr), "dfu_maxpool_bn_fwd: scale and shift");
  DFU_CHECK_ARG((int64_t)B * P < 65536 && Q * (C / 8) < (1 << 24), "dfu_maxpool_fwd: size");
  const dim3 grid((Q * (C / 8) + 255) / 256, B * P);
  hipLaunchKernelGGL(scale ? k_maxpool_rows<true> : k_maxpool_rows<false>, grid, dim3(256), 0,
                     (hipStream_t)stream, (const bf16_t*)x, scale, shift, H, W, C, (bf16_t*)y,
                     argmax, P, Q);
  DFU_LAUNCH_CHECK();
  return DFU_OK;
}

extern "C" int dfu_maxpool_bwd(const void* dy, const uint8_t* argmax, int32_t B, int32_t H,
                               int32_t W, int32_t C, int32_t P, int32_t Q, void* dx,
                               void* stream) {
  DFU_CHECK_ARG(dy && dx && argmax && C % 8 == 0, "dfu_maxpool_bwd: C %% 8 != 0");
  DFU_CHECK_ARG((int64_t)B * ((H + 1) / 2) < 65536 && W * (C / 8) < (1 << 24),
                "dfu_maxpool_bwd: size");
  const dim3 grid(((W + 1) / 2 * (C / 8) + 255) / 256, B * ((H + 1) / 2));
  hipLaunchKernelGGL(k_maxpool_bwd_2x2, grid, dim3(256), 0, (hipStream_t)stream,
                     (const bf16_t*)dy, argmax, H, W, C, P, Q, (bf16_t*)dx);
  DFU_LAUNCH_CHECK();
  return DFU_OK;
}

extern "C" int dfu_avgpool_fwd(const void* x, int32_t B, int32_t HW, int32_t C, float* y,
                               void* stream) {
  DFU_CHECK_ARG(x && y && C % 8 == 0, "dfu_avgpool_fwd: C %% 8 != 0");
  LAUNCH(k_avgpool_fwd, (int64_t)B * (C / 8), stream, (const bf16_t*)x, B, HW, C, y);
  return DFU_OK;
}

extern "C" int dfu_avgpool_bwd(const float* dy, int32_t B, int32_t HW, int32_t C, void* dx,
                               void* stream) {
  DFU_CHECK_ARG(dy && dx && C % 8 == 0, "dfu_avgpool_bwd: C %% 8 != 0");
  LAUNCH(k_avgpool_bwd, (int64_t)B * HW * (C / 8), stream, dy, B, HW, C, (bf16_t*)dx);
  return DFU_OK;
}

extern "C" int dfu_colsum_blocks(int32_t rows) { return (rows + CS_ROWS - 1) / CS_ROWS; }

extern "C" int dfu_colsum(const void* x, int32_t is_bf16, int64_t ld, int32_t rows, int32_t N,
                          float* out, float* partial, void* stream) {
  DFU_CHECK_ARG(x && partial && rows > 0 && N > 0, "dfu_colsum: bad args");
  if (is_bf16) DFU_CHECK_ARG(ld % 8 == 0 && ((uintptr_t)x & 15) == 0, "dfu_colsum: bf16 needs ld%%8==0");
  const int blocks = dfu_colsum_blocks(rows);
  dim3 grid((N + 511) / 512, blocks);
  if (is_bf16)
    hipLaunchKernelGGL(k_colsum<true>, grid, dim3(256), 0, (hipStream_t)stream, x, ld, rows, N, partial);
  else
    hipLaunchKernelGGL(k_colsum<false>, grid, dim3(256), 0, (hipStream_t)stream, x, ld, rows, N, partial);
  DFU_LAUNCH_CHECK();
  if (out == nullptr) return DFU_OK;  // partials only (reduced later, dfu_reduce_partials_batch)
  hipLaunchKernelGGL(k_reduce_partials, dim3((N + 7) / 8), dim3(256), 0, (hipStream_t)stream,
                     partial, blocks, 1, N, out, (float*)nullptr);
  DFU_LAUNCH_CHECK();
  return DFU_OK;
}

extern "C" int dfu_reduce_partials(const float* partial, int32_t blocks, int32_t nvec, int32_t D,
                                   float* out0, float* out1, void* stream) {
  DFU_CHECK_ARG(partial && blocks > 0 && nvec >= 1 && nvec <= 2 && D > 0, "dfu_reduce_partials: bad args");
  hipLaunchKernelGGL(k_reduce_partials, dim3((unsigned)(((int64_t)nvec * D + 7) / 8)), dim3(256), 0,
                     (hipStream_t)stream, partial, blocks, nvec, D, out0, out1);
  DFU_LAUNCH_CHECK();
  return DFU_OK;
}

extern "C" int dfu_gather_rows_f32(const float* in, int64_t ld_in, int32_t stride, int32_t offset,
                                   int32_t rows, int32_t D, float* out, int64_t ld_out,
                                   void* stream) {
  DFU_CHECK_ARG(in && out && rows > 0 && D > 0, "dfu_gather_rows_f32: bad args");
  LAUNCH(k_gather_rows, (int64_t)rows * D, stream, in, ld_in, stride, offset, rows, D, out, ld_out);
  return DFU_OK;
}

extern "C" int dfu_scatter_rows_f32(const float* in, int64_t ld_in, int32_t stride, int32_t offset,
                                    int32_t rows, int32_t D, float* out, int64_t ld_out,
                                    void* stream) {
  DFU_CHECK_ARG(in && out && rows > 0 && D > 0, "dfu_scatter_rows_f32: bad args");
  LAUNCH(k_scatter_rows, (int64_t)rows * D, stream, in, ld_in, stride, offset, rows, D, out, ld_out);
  return DFU_OK;
}

extern "C" int dfu_relu_fwd(const void* x, void* y, int64_t n, int32_t is_bf16, void* stream) {
  DFU_CHECK_ARG(x && y && n >= 0, "dfu_relu_fwd: bad args");
  if (n == 0) return DFU_OK;
  if (is_bf16) LAUNCH(k_relu_fwd<true>, n, stream, x, y, n);
  else LAUNCH(k_relu_fwd<false>, n, stream, x, y, n);
  return DFU_OK;
}

extern "C" int dfu_relu_bwd(const void* dy, const void* y, void* dx, int64_t n, int32_t is_bf16,
                            void* stream) {
  DFU_CHECK_ARG(dy && y && dx && n >= 0, "dfu_relu_bwd: bad args");
  if (n == 0) return DFU_OK;
  if (is_bf16) LAUNCH(k_relu_bwd<true>, n, stream, dy, y, dx, n);
  else LAUNCH(k_relu_bwd<false>, n, stream, dy, y, dx, n);
  return DFU_OK;
}

extern "C" int dfu_dropout_fwd(const void* x, void* y, uint8_t* mask, int64_t n, float p,
                               uint64_t seed, int64_t* offset_dev, int32_t is_bf16, void* stream) {
  DFU_CHECK_ARG(x && y && mask && offset_dev && p >= 0.f && p < 1.f, "dfu_dropout_fwd: bad args");
  if (n == 0) return DFU_OK;
  if (is_bf16) LAUNCH(k_dropout_fwd<true>, n, stream, x, y, mask, n, p, seed, offset_dev);
  else LAUNCH(k_dropout_fwd<false>, n, stream, x, y, mask, n, p, seed, offset_dev);
  hipLaunchKernelGGL(k_advance, dim3(1), dim3(64), 0, (hipStream_t)stream, offset_dev, n);
  DFU_LAUNCH_CHECK();
  return DFU_OK;
}

extern "C" int dfu_dropout_bwd(const void* dy, const uint8_t* mask, void* dx, int64_t n, float p,
                               int32_t is_bf16, void* stream) {
  DFU_CHECK_ARG(dy && mask && dx && p >= 0.f && p < 1.f, "dfu_dropout_bwd: bad args");
  if (n == 0) return DFU_OK;
  if (is_bf16) LAUNCH(k_dropout_bwd<true>, n, stream, dy, mask, dx, n, p);
  else LAUNCH(k_dropout_bwd<false>, n, stream, dy, mask, dx, n, p);
  return DFU_OK;
}

extern "C" int dfu_concat2_bf16(const void* a, int32_t a_bf16, int32_t Na, const void* b,
                                int32_t b_bf16, int32_t Nb, int32_t rows, void* out, void* stream) {
  DFU_CHECK_ARG(a && b && out && rows > 0, "dfu_concat2_bf16: bad args");
  LAUNCH(k_concat2, (int64_t)rows * (Na + Nb), stream, a, a_bf16, Na, b, b_bf16, Nb, rows,
         (bf16_t*)out);
  return DFU_OK;
}

extern "C" int dfu_split2_f32(const void* g, int32_t g_bf16, int32_t rows, int32_t Na, int32_t Nb,
                              float* ga, float* gb, void* stream) {
  DFU_CHECK_ARG(g && rows > 0, "dfu_split2_f32: bad args");
  LAUNCH(k_split2, (int64_t)rows * (Na + Nb), stream, g, g_bf16, rows, Na, Nb, ga, gb);
  return DFU_OK;
}

extern "C" int dfu_vit_cls_rows(const float* cls, const float* pos, float* x, int32_t B, int32_t T,
                                int32_t D, void* stream) {
  DFU_CHECK_ARG(cls && pos && x && B > 0 && T > 0 && D > 0, "dfu_vit_cls_rows: bad args");
  LAUNCH(k_vit_cls_rows, (int64_t)B * D, stream, cls, pos, x, B, T, D);
  return DFU_OK;
}

extern "C" int dfu_vit_embed_bwd(const float* gx, int32_t B, int32_t T, int32_t D, float* dcls,
                                 float* dpos, float* dbias, void* gpatch, float* partial,
                                 void* stream) {
  DFU_CHECK_ARG(gx && gpatch && partial && B > 0 && T > 1 && D > 0, "dfu_vit_embed_bwd: bad args");
  LAUNCH(k_vit_embed_bwd, (int64_t)T * D, stream, gx, B, T, D, dcls, dpos, (bf16_t*)gpatch, partial);
  if (dbias) {
    hipLaunchKernelGGL(k_sum_rows_add, dim3((D + SRA_C - 1) / SRA_C), dim3(SRA_C * SRA_R), 0,
                       (hipStream_t)stream, partial, T, D, dbias);
    DFU_LAUNCH_CHECK();
  }
  return DFU_OK;
}

extern "C" int dfu_argmax_rows(const float* x, int32_t rows, int32_t C, int64_t* out,
                               void* stream) {
  DFU_CHECK_ARG(x && out && rows > 0 && C > 0, "dfu_argmax_rows: bad args");
  LAUNCH(k_argmax_rows, (int64_t)rows, stream, x, rows, C, out);
  return DFU_OK;
}

extern "C" int dfu_softmax_rows(const float* x, int32_t rows, int32_t C, float* out,
                                void* stream) {
  DFU_CHECK_ARG(x && out && rows > 0 && C > 0, "dfu_softmax_rows: bad args");
  LAUNCH(k_softmax_rows, (int64_t)rows, stream, x, rows, C, out);
  return DFU_OK;
}

extern "C" int dfu_metrics_accumulate(const float* logits, const int64_t* labels, int32_t rows,
                                      int32_t C, const float* loss, int64_t* confusion,
                                      double* loss_sum, int64_t* batches, void* stream) {
  DFU_CHECK_ARG(logits && labels && confusion && loss_sum && batches && rows > 0 && C > 0,
                "dfu_metrics_accumulate: bad args");
  hipLaunchKernelGGL(k_metrics_accumulate, dim3(1), dim3(256), 0, (hipStream_t)stream, logits,
                     labels, rows, C, loss, (unsigned long long*)confusion, loss_sum,
                     (unsigned long long*)batches);
  DFU_LAUNCH_CHECK();
  return DFU_OK;
}

extern "C" int dfu_reduce_partials_batch(const dfu_reduce_entry* entries, int32_t n, void* stream) {
  DFU_CHECK_ARG(entries && n >= 0 && n <= DFU_REDUCE_BATCH,
                "dfu_reduce_partials_batch: 0..%d entries", DFU_REDUCE_BATCH);
  if (n == 0) return DFU_OK;
  ReduceBatch b;
  b.n = n;
  int total = 0;
  for (int i = 0; i < n; ++i) {
    const dfu_reduce_entry& en = entries[i];
    DFU_CHECK_ARG(en.partial && en.out && en.blocks > 0 && en.D > 0 && en.stride >= en.D,
                  "dfu_reduce_partials_batch: bad entry %d", i);
    b.partial[i] = en.partial;
    b.stride[i] = en.stride;
    b.out[i] = en.out;
    b.blocks[i] = en.blocks;
    b.D[i] = en.D;
    b.first[i] = total;
    total += (en.D + 7) / 8;
  }
  b.first[n] = total;
  hipLaunchKernelGGL(k_reduce_partials_batch, dim3(total), dim3(256), 0, (hipStream_t)stream, b);
  DFU_LAUNCH_CHECK();
  return DFU_OK;
}
