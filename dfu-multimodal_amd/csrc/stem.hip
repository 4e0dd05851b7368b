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

}  // namespace

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
