// The bf16x3 ResNet stem convolution (torchvision resnet50 conv1: 7x7 / stride 2 / pad 3,
// 3 -> 64 channels; train_multimodal_fusion.py:294) as ONE implicit-GEMM kernel, for the
// "parity" precision mode.
//
// The explicit path (k_im2col_lds<true> + the interleaved-pair GEMM) writes the im2col rows as a
// split pair (hi, lo: 2 x 160 bf16 per output pixel, 514 MB at B = 64) and reads them back.
// Here each workgroup stages the input rows its 128 output pixels touch (fp32, all 3 channels,
// <= 11 rows) in LDS once, builds every lane's A fragments from them in registers (hi =
// bf16(x), lo = bf16(x - hi), the 147 taps padded to 160 with zeros), and runs the same three
// products per 32-tap step as the pair GEMM (hi.hi + lo.hi + hi.lo, in that order, on
// v_mfma_f32_16x16x32_bf16 with the B operand first), so the fp32 result is the pair GEMM's.
// The weights are split into hi / lo planes in LDS once per (persistent) workgroup.  Outputs:
// the conv result as the split pair (y = bf16 hi, y_lo), the BN tile statistics of the unrounded
// values (sum, M2 per 128-row block: the F32_STATS epilogue's records, merged across the four
// waves by Chan's formula), and the hi im2col rows the weight gradient reads (col, optional).
// Bytes: input 39 MB + y pair 205 MB + col 257 MB (B = 64), against 1.27 GB for the two-kernel
// path.
//
// Geometry: a tile is 128 consecutive output pixels m (one stats block).  P*Q % 128 == 0 keeps
// a tile inside one image and Q >= 64 inside three output rows, i.e. 11 staged input rows.
// 256 threads = 4 waves; wave w owns tile rows 32w .. 32w+31 (two 16-row fragments) x all 64
// output channels (four 16-column fragments).
#include "common.h"

namespace {

constexpr int SC = 3, SR = 7, SK = 64, SKR = 147, SKP = 160;
constexpr int STM = 128;       // output pixels per tile
constexpr int SRR = 11;        // staged input rows per tile
constexpr int SWP = 168;       // weight plane row stride (bf16): 336 B rows
constexpr int SNT = 256;

template <int CTRL>
DFU_DEV float dpp_s(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL,
                                                               0xF, 0xF, false));
}
DFU_DEV float row16_sum_s(float v) {  // sum over the 16 lanes of a DPP row (gemm_kernel.h)
  v += dpp_s<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_s<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_s<0x141>(v);  // row_half_mirror
  v += dpp_s<0x140>(v);  // row_mirror
  return v;
}

__global__ __launch_bounds__(SNT, 2) void k_stem_conv_x3(
    const float* __restrict__ x, int64_t sn, int64_t sc, int64_t sh, int64_t sw, int H, int W,
    int P, int Q, int tiles, const float* __restrict__ w, bf16_t* __restrict__ y,
    bf16_t* __restrict__ y_lo, float* __restrict__ stats, bf16_t* __restrict__ col) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int WP = W + 6;  // staged columns: iw = -3 .. W + 2
  float* xin = (float*)smem;                                     // [SC][SRR][WP]
  const int xin_bytes = (SC * SRR * WP * 4 + 4 + 15) / 16 * 16;  // + the zero slot
  bf16_t* whi = (bf16_t*)(smem + xin_bytes);                     // [SK][SWP]
  bf16_t* wlo = whi + SK * SWP;
  float* red = (float*)(wlo + SK * SWP);                         // [4][SK][2]
  int* koff = (int*)(red + 4 * SK * 2);                          // [SKP] tap -> xin offset
  const int ZERO = SC * SRR * WP;  // a zero slot past the staged rows: the padded taps read it
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lrow = lane & 15, kc = lane >> 4;

  // weight planes, once per workgroup: w [64][147] fp32 -> hi / lo bf16 [64][160 (168)]; the
  // taps 147..159 zero.  All of a thread's loads go out before its first LDS store (a
  // load-then-store loop serialised 40 global round trips at the kernel's start).
  {
    constexpr int NW4 = SK * SKR / 4;                  // 2352 float4 of the contiguous weight
    constexpr int PER = (NW4 + SNT - 1) / SNT;         // 10 per thread
    f32x4 wv[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int i = min(tid + j * SNT, NW4 - 1);
      wv[j] = ((const f32x4*)w)[i];
    }
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int i = tid + j * SNT;
      if (i < NW4) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int f = 4 * i + e;
          const int n = f / SKR, k = f - n * SKR;
          const bf16_t h = f2bf(wv[j][e]);
          whi[n * SWP + k] = h;
          wlo[n * SWP + k] = f2bf(wv[j][e] - bf2f(h));
        }
      }
    }
    for (int i = tid; i < SK * (SKP - SKR); i += SNT) {
      const int n = i / (SKP - SKR), k = SKR + i - n * (SKP - SKR);
      whi[n * SWP + k] = 0;
      wlo[n * SWP + k] = 0;
    }
    // tap k = (c, r, s) of OIHW -> offset (c * SRR + r) * WP + s in the staged rows; the
    // padded taps -> past every pixel's base, clamped to the zero slot at the read
    if (tid < SKP) {
      const unsigned k = tid, c = k / 49u, rem = k - 49u * c, r = rem / 7u, s_ = rem - 7u * r;
      koff[k] = k < (unsigned)SKR ? (int)((c * SRR + r) * WP + s_) : (1 << 24);
    }
    if (tid == 0) xin[ZERO] = 0.f;
  }

  const int PQ = P * Q;
  // The input rows of the NEXT tile are loaded into registers (a thread per staged column, all
  // 33 rows' loads in flight at once) while the current tile computes, and written to LDS at the
  // top of the next iteration: the global-load latency hides under the MFMAs.
  const int cc = tid;  // staged column of this thread (W + 6 <= 256 threads: host-checked)
  float v[SC * SRR];
  auto load_rows = [&](int t) {
    const int m0 = t * STM;
    const int b = m0 / PQ;
    const int pa = (m0 - b * PQ) / Q;
    const float* xb = x + b * sn;
    const int iw = cc - 3;
    const bool okw = cc < WP && (unsigned)iw < (unsigned)W;
    const int iwc = min(max(iw, 0), W - 1);
    // every load from a clamped in-image address, the zero padding by a select afterwards (a
    // load under a runtime condition becomes a branch and a vmcnt(0) wait per element)
#pragma unroll
    for (int cr = 0; cr < SC * SRR; ++cr) {
      const int c = cr / SRR, rr = cr - c * SRR;
      const int ih = 2 * pa - 3 + rr;
      const int ihc = min(max(ih, 0), H - 1);
      v[cr] = xb[c * sc + (int64_t)ihc * sh + (int64_t)iwc * sw];
    }
#pragma unroll
    for (int cr = 0; cr < SC * SRR; ++cr) {
      const int ih = 2 * pa - 3 + cr % SRR;
      v[cr] = okw && (unsigned)ih < (unsigned)H ? v[cr] : 0.f;
    }
  };
  if ((int)blockIdx.x < tiles) load_rows(blockIdx.x);
  for (int t = blockIdx.x; t < tiles; t += gridDim.x) {
    const int m0 = t * STM;
    const int b = m0 / PQ;
    const int pq0 = m0 - b * PQ;
    const int pa = pq0 / Q;  // first output row of the tile
    __syncthreads();         // the previous tile's reads of xin / red are done
    if (cc < WP) {  // input rows 2 pa - 3 .. 2 pa + 7 of image b (zero outside the image)
#pragma unroll
      for (int cr = 0; cr < SC * SRR; ++cr) xin[cr * WP + cc] = v[cr];
    }
    __syncthreads();
    if (t + (int)gridDim.x < tiles) load_rows(t + gridDim.x);

    f32x4 acc[2][4];
#pragma unroll
    for (int rf = 0; rf < 2; ++rf)
#pragma unroll
      for (int cf = 0; cf < 4; ++cf) acc[rf][cf] = (f32x4){0.f, 0.f, 0.f, 0.f};
    int base[2];
#pragma unroll
    for (int rf = 0; rf < 2; ++rf) {
      const int pq = pq0 + 32 * wave + 16 * rf + lrow;
      const int p = pq / Q, q = pq - p * Q;
      base[rf] = 2 * (p - pa) * WP + 2 * q;
    }
#pragma unroll
    for (int ks = 0; ks < SKP / 32; ++ks) {
      const int k0 = 32 * ks + 8 * kc;
      const u32x4 o0 = *(const u32x4*)(koff + k0), o1 = *(const u32x4*)(koff + k0 + 4);
      const int off[8] = {(int)o0[0], (int)o0[1], (int)o0[2], (int)o0[3],
                          (int)o1[0], (int)o1[1], (int)o1[2], (int)o1[3]};
      bf16x8 ahi[2], alo[2];
#pragma unroll
      for (int rf = 0; rf < 2; ++rf) {
        float h[8], l[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {  // every read unconditional (a conditional LDS read
          // became an exec-masked branch per element)
          const float v = xin[min(base[rf] + off[e], ZERO)];
          h[e] = bf2f(f2bf(v));
          l[e] = v - h[e];
        }
        const u32x4 hp = pack8(h), lp = pack8(l);
        ahi[rf] = __builtin_bit_cast(bf16x8, hp);
        alo[rf] = __builtin_bit_cast(bf16x8, lp);
        if (col) *(u32x4*)(col + (int64_t)(m0 + 32 * wave + 16 * rf + lrow) * SKP + k0) = hp;
      }
      bf16x8 bhi[4], blo[4];
#pragma unroll
      for (int cf = 0; cf < 4; ++cf) {
        const int n = 16 * cf + lrow;
        bhi[cf] = *(const bf16x8*)(whi + n * SWP + k0);
        blo[cf] = *(const bf16x8*)(wlo + n * SWP + k0);
      }
      // the pair GEMM's order per 32-tap step: hi.hi, lo.hi (A lo), hi.lo (B lo)
#pragma unroll
      for (int tt = 0; tt < 3; ++tt)
#pragma unroll
        for (int rf = 0; rf < 2; ++rf)
#pragma unroll
          for (int cf = 0; cf < 4; ++cf)
            acc[rf][cf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                tt == 2 ? blo[cf] : bhi[cf], tt == 1 ? alo[rf] : ahi[rf], acc[rf][cf], 0, 0, 0);
    }

    // epilogue: lane holds rows 32 wave + 16 rf + lrow, channels 16 cf + 4 kc + r
#pragma unroll
    for (int rf = 0; rf < 2; ++rf) {
      const int64_t m = m0 + 32 * wave + 16 * rf + lrow;
#pragma unroll
      for (int cf = 0; cf < 4; ++cf) {
        float h[4], l[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          h[r] = bf2f(f2bf(acc[rf][cf][r]));
          l[r] = acc[rf][cf][r] - h[r];
        }
        const int n = 16 * cf + 4 * kc;
        *(u32x2*)(y + m * SK + n) = (u32x2){pack2(h[0], h[1]), pack2(h[2], h[3])};
        *(u32x2*)(y_lo + m * SK + n) = (u32x2){pack2(l[0], l[1]), pack2(l[2], l[3])};
      }
    }
    // BN tile statistics of the unrounded values: per wave (32 rows) two-pass, then Chan's
    // merge of the four waves (as the F32_STATS epilogue)
#pragma unroll
    for (int cf = 0; cf < 4; ++cf)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float s = row16_sum_s(acc[0][cf][r] + acc[1][cf][r]);
        const float mean = s * (1.0f / 32.0f);
        const float d0 = acc[0][cf][r] - mean, d1 = acc[1][cf][r] - mean;
        const float q = row16_sum_s(d0 * d0 + d1 * d1);
        if (lrow == 0) {
          const int n = 16 * cf + 4 * kc + r;
          red[(wave * SK + n) * 2 + 0] = s;
          red[(wave * SK + n) * 2 + 1] = q;
        }
      }
    __syncthreads();
    if (tid < SK) {
      float S = 0.f, Qm = 0.f, Cn = 0.f;
#pragma unroll
      for (int wv = 0; wv < 4; ++wv) {
        const float s1 = red[(wv * SK + tid) * 2 + 0], q1 = red[(wv * SK + tid) * 2 + 1];
        if (Cn > 0.f) {
          const float d = s1 / 32.0f - S / Cn;
          Qm += q1 + d * d * Cn * 32.0f / (Cn + 32.0f);
        } else {
          Qm = q1;
        }
        S += s1;
        Cn += 32.0f;
      }
      stats[((int64_t)t * 2 + 0) * SK + tid] = S;
      stats[((int64_t)t * 2 + 1) * SK + tid] = Qm;
    }
  }
}

// ---------------------------------------------------------------- weight gradient
// dW[n][k] += sum_m dy[m][n] * bf16(x at tap k of output pixel m): the stem's weight gradient
// straight from the fp32 image (the bf16 backward's operand is bf16(x), the hi rows the
// explicit path's im2col held), so no im2col rows are written in the forward or read here.
// A persistent workgroup walks tiles of TWO output rows (2Q pixels of one image: the 9 input
// rows they touch are staged once, where 128-pixel tiles restaged 11 rows per 1.14 output rows)
// and stages the tile's input rows (fp32, 3 channels) and dy rows ([2Q][64] bf16, row stride
// 72) in LDS; per 32-pixel step it builds
//   Y fragments (the dy side: 16 channels x 8 consecutive pixels per lane) by two
//     ds_read_b64_tr_b16 each -- the compiler's builtin: no LDS-DMA here, so its waits are exact;
//   X fragments (the im2col side: 16 taps x the same 8 pixels) by reads of x at
//     base(pixel) + koff(tap) + 2e (8 consecutive pixels lie in one output row: Q % 16 == 0;
//     one address per fragment, so the reads pair into ds_read2_b32),
// and accumulates D[n][k] over all its tiles in registers: wave w owns the tap fragments
// w, w + 4, w + 8 (< 10) x all four channel fragments.  Its partial D goes to slab[blockIdx]
// ([64][147] fp32); k_stem_wgrad_reduce adds the slabs into dW in a fixed order.
constexpr int SDYS = 72;       // dy LDS row stride (bf16): 144-B rows
constexpr int WRR = 9;         // staged input rows per two-output-row tile
constexpr int WDV = 7;         // dy 16-B loads per thread per tile: 2Q <= 224 rows

typedef short s16x4 __attribute__((ext_vector_type(4)));
DFU_DEV bf16x4 tr16_b64(const bf16_t* p) {
  const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)(p));
  return __builtin_bit_cast(bf16x4, v);
}

__global__ __launch_bounds__(SNT, 2) void k_stem_wgrad(
    const float* __restrict__ x, int64_t sn, int64_t sc, int64_t sh, int64_t sw, int H, int W,
    int P, int Q, int tiles, const bf16_t* __restrict__ dy, float* __restrict__ slab) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int WP = W + 6;
  const int TP = 2 * Q;  // pixels per tile
  float* xin = (float*)smem;                                       // [SC][WRR][WP]
  const int xin_bytes = (SC * WRR * WP * 4 + 64 + 15) / 16 * 16;   // + 16 zeros
  bf16_t* dys = (bf16_t*)(smem + xin_bytes);                       // [TP][SDYS]
  int* koff = (int*)(dys + TP * SDYS);                             // [SKP]
  const int ZERO = SC * WRR * WP;  // 16 zero floats: a padded tap's 8 pixel reads land there
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lrow = lane & 15, kc = lane >> 4;
  if (tid < SKP) {
    const unsigned k = tid, c = k / 49u, rem = k - 49u * c, r = rem / 7u, s_ = rem - 7u * r;
    koff[k] = k < (unsigned)SKR ? (int)((c * WRR + r) * WP + s_) : (1 << 24);
  }
  if (tid < 16) xin[ZERO + tid] = 0.f;

  const int P2 = P / 2;
  const int cc = tid;  // staged input column of this thread (W + 6 <= 256: host-checked)
  float v[SC * WRR];
  u32x4 dv[WDV];
  auto load_tile = [&](int t) {  // into registers: the tile's input rows and dy rows
    const int b = t / P2;
    const int pa = 2 * (t - b * P2);
    const float* xb = x + b * sn;
    const int iw = cc - 3;
    const bool okw = cc < WP && (unsigned)iw < (unsigned)W;
    const int iwc = min(max(iw, 0), W - 1);
#pragma unroll
    for (int cr = 0; cr < SC * WRR; ++cr) {
      const int c = cr / WRR, rr = cr - c * WRR;
      const int ihc = min(max(2 * pa - 3 + rr, 0), H - 1);
      v[cr] = xb[c * sc + (int64_t)ihc * sh + (int64_t)iwc * sw];
    }
    const int64_t m0 = ((int64_t)b * P + pa) * Q;
#pragma unroll
    for (int i = 0; i < WDV; ++i) {  // rows past the tile (2Q < 224) reload its last row
      const int row = min((tid >> 3) + 32 * i, TP - 1);
      dv[i] = *(const u32x4*)(dy + (m0 + row) * SK + 8 * (tid & 7));
    }
#pragma unroll
    for (int cr = 0; cr < SC * WRR; ++cr) {
      const int ih = 2 * pa - 3 + cr % WRR;
      v[cr] = okw && (unsigned)ih < (unsigned)H ? v[cr] : 0.f;
    }
  };
  f32x4 acc[4][3];
#pragma unroll
  for (int rf = 0; rf < 4; ++rf)
#pragma unroll
    for (int j = 0; j < 3; ++j) acc[rf][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  __syncthreads();  // koff
  int ko[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int cf = wave + 4 * j;
    ko[j] = koff[min(16 * cf + lrow, SKP - 1)];
  }
  const int tq = lane & 15, tp = tq & 3, tr = tq >> 2;  // transposed-read lane roles
  const int ksteps = TP / 32;
  if ((int)blockIdx.x < tiles) load_tile(blockIdx.x);
  for (int t = blockIdx.x; t < tiles; t += gridDim.x) {
    __syncthreads();  // the previous tile's reads of xin / dys are done
    if (cc < WP) {
#pragma unroll
      for (int cr = 0; cr < SC * WRR; ++cr) xin[cr * WP + cc] = v[cr];
    }
#pragma unroll
    for (int i = 0; i < WDV; ++i) {
      const int row = (tid >> 3) + 32 * i;
      if (row < TP) *(u32x4*)(dys + row * SDYS + 8 * (tid & 7)) = dv[i];
    }
    __syncthreads();
    if (t + (int)gridDim.x < tiles) load_tile(t + gridDim.x);
    for (int ks = 0; ks < ksteps; ++ks) {
      // this lane's 8 pixels: tile pixels 32 ks + 8 kc + 0..7 (one output row)
      const int lp = 32 * ks + 8 * kc;
      const int pr = lp >= Q ? 1 : 0, q = lp - pr * Q;
      const int base = 2 * pr * WP + 2 * q;
      bf16x8 yf[4];
#pragma unroll
      for (int rf = 0; rf < 4; ++rf) {
        const bf16_t* a0 = dys + (32 * ks + 8 * kc + tr) * SDYS + 16 * rf + 4 * tp;
        const bf16x4 lo4 = tr16_b64(a0), hi4 = tr16_b64(a0 + 4 * SDYS);
        yf[rf] = __builtin_shufflevector(lo4, hi4, 0, 1, 2, 3, 4, 5, 6, 7);
      }
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        if (wave + 4 * j >= SKP / 16) continue;  // (wave-uniform)
        const float* xp = xin + (ko[j] < (1 << 24) ? base + ko[j] : ZERO);
        float h[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) h[e] = xp[2 * e];
        const bf16x8 xf = __builtin_bit_cast(bf16x8, pack8(h));  // bf16(x): the hi rows
#pragma unroll
        for (int rf = 0; rf < 4; ++rf)
          acc[rf][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xf, yf[rf], acc[rf][j], 0, 0, 0);
      }
    }
  }
  // lane holds D[n = 16 rf + lrow][k = 16 cf + 4 kc + r]
  float* sl = slab + (int64_t)blockIdx.x * SK * SKR;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int cf = wave + 4 * j;
    if (cf >= SKP / 16) continue;
#pragma unroll
    for (int rf = 0; rf < 4; ++rf)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int k = 16 * cf + 4 * kc + r;
        if (k < SKR) sl[(16 * rf + lrow) * SKR + k] = acc[rf][j][r];
      }
  }
}

// dW[i] += sum over the G slabs of slab[g][i], i < 64 x 147, in a fixed order: 16 slices of
// the slabs per element (waves), each slice's loads all in flight (four running sums), then the
// slices merged in order.
__global__ __launch_bounds__(1024) void k_stem_wgrad_reduce(const float* __restrict__ slab,
                                                            int G, float* __restrict__ dw) {
  __shared__ float part[16][64];
  const int l = threadIdx.x & 63, sl = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + l;
  constexpr int NE = SK * SKR;
  const int ic = min(i, NE - 1);
  float s4[4] = {0.f, 0.f, 0.f, 0.f};
  int g = sl;
  for (; g + 48 < G; g += 64) {
#pragma unroll
    for (int u = 0; u < 4; ++u) s4[u] += slab[(int64_t)(g + 16 * u) * NE + ic];
  }
  for (; g < G; g += 16) s4[0] += slab[(int64_t)g * NE + ic];
  part[sl][l] = (s4[0] + s4[1]) + (s4[2] + s4[3]);
  __syncthreads();
  if (sl == 0 && i < NE) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) t += part[k][l];
    dw[i] += t;
  }
}

}  // namespace

extern "C" int64_t dfu_stem_wgrad_ws_bytes(int32_t B, int32_t H, int32_t W) {
  const int P = (H + 6 - 7) / 2 + 1;
  const int64_t tiles = (int64_t)B * (P / 2);
  const int64_t g = tiles < 512 ? tiles : 512;
  return (g > 0 ? g : 1) * SK * SKR * 4;
}

extern "C" int dfu_stem_wgrad_x3(const float* x, int64_t sn, int64_t sc, int64_t sh, int64_t sw,
                                 int32_t B, int32_t C, int32_t H, int32_t W, const void* dy,
                                 int32_t K, int32_t R, int32_t S, int32_t stride, int32_t pad,
                                 float* dw, float* slab, int64_t slab_bytes, void* stream) {
  const int P = (H + 2 * pad - R) / stride + 1, Q = (W + 2 * pad - S) / stride + 1;
  DFU_CHECK_ARG(x && dy && dw && slab && C == SC && K == SK && R == SR && S == SR &&
                    stride == 2 && pad == 3 && B > 0 && H >= SR && W >= SR,
                "dfu_stem_wgrad_x3: the 7x7/s2/p3 3->64 stem only");
  DFU_CHECK_ARG(P % 2 == 0 && Q % 16 == 0 && 2 * Q <= 32 * WDV && W + 6 <= SNT &&
                    (int64_t)B * P * Q < (1LL << 31),
                "dfu_stem_wgrad_x3: needs P even, Q %% 16 == 0, Q <= 112, W <= 250 (P=%d Q=%d)",
                P, Q);
  DFU_CHECK_ARG((((uintptr_t)dy) & 15) == 0, "dfu_stem_wgrad_x3: dy must be 16-byte aligned");
  const int tiles = B * (P / 2);
  const int grid = tiles < 512 ? tiles : 512;
  DFU_CHECK_ARG(slab_bytes >= (int64_t)grid * SK * SKR * 4,
                "dfu_stem_wgrad_x3: slab needs dfu_stem_wgrad_ws_bytes bytes");
  const int xin_bytes = (SC * WRR * (W + 6) * 4 + 64 + 15) / 16 * 16;
  const size_t lds = xin_bytes + 2 * Q * SDYS * 2 + SKP * 4;
  hipLaunchKernelGGL(k_stem_wgrad, dim3(grid), dim3(SNT), lds, (hipStream_t)stream, x, sn, sc, sh,
                     sw, H, W, P, Q, tiles, (const bf16_t*)dy, slab);
  DFU_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_stem_wgrad_reduce, dim3((SK * SKR + 63) / 64), dim3(1024), 0,
                     (hipStream_t)stream, slab, grid, dw);
  DFU_LAUNCH_CHECK();
  return DFU_OK;
}

extern "C" int dfu_stem_conv_x3(const float* x, int64_t sn, int64_t sc, int64_t sh, int64_t sw,
                                int32_t B, int32_t C, int32_t H, int32_t W, const float* w,
                                int32_t K, int32_t R, int32_t S, int32_t stride, int32_t pad,
                                void* y, void* y_lo, float* stats, void* col, void* stream) {
  const int P = (H + 2 * pad - R) / stride + 1, Q = (W + 2 * pad - S) / stride + 1;
  DFU_CHECK_ARG(x && w && y && y_lo && stats && C == SC && K == SK && R == SR && S == SR &&
                    stride == 2 && pad == 3 && B > 0 && H >= SR && W >= SR,
                "dfu_stem_conv_x3: the 7x7/s2/p3 3->64 stem only (C=%d K=%d R=%d S=%d st=%d "
                "pad=%d)", C, K, R, S, stride, pad);
  DFU_CHECK_ARG((P * Q) % STM == 0 && Q >= 64 && W + 6 <= SNT && (int64_t)B * P * Q < (1LL << 31),
                "dfu_stem_conv_x3: needs P*Q %% 128 == 0, Q >= 64, W <= 250 (P=%d Q=%d)", P, Q);
  DFU_CHECK_ARG((((uintptr_t)y | (uintptr_t)y_lo | (uintptr_t)col | (uintptr_t)w) & 15) == 0,
                "dfu_stem_conv_x3: outputs and w must be 16-byte aligned");
  const int tiles = B * P * Q / STM;
  const int xin_bytes = (SC * SRR * (W + 6) * 4 + 4 + 15) / 16 * 16;
  const size_t lds = xin_bytes + 2 * SK * SWP * 2 + 4 * SK * 2 * 4 + SKP * 4;
  static const int cus = [] {
    int dev = 0, n = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      n = 256;
    return n;
  }();
  const int grid = tiles < 2 * cus ? tiles : 2 * cus;  // persistent: two per CU
  hipLaunchKernelGGL(k_stem_conv_x3, dim3(grid), dim3(SNT), lds, (hipStream_t)stream, x, sn, sc,
                     sh, sw, H, W, P, Q, tiles, w, (bf16_t*)y, (bf16_t*)y_lo, stats,
                     (bf16_t*)col);
  DFU_LAUNCH_CHECK();
  return DFU_OK;
}
