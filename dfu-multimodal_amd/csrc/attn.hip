// Multi-head self-attention of timm ViT-B/16 (vision_transformer.py Attention with
// F.scaled_dot_product_attention; N = 197 tokens, 12 heads, head dim 64, scale 1/8).
//
// One workgroup (4 waves) per (batch, head).  The whole key/value (or query/dO) sequence is
// resident in LDS (N padded to a multiple of 32, <= 256), so the softmax is exact over the
// full row — no online rescaling.  All products are v_mfma_f32_16x16x32_bf16:
//   forward  S^T = K Q^T (lane owns one query), P in registers, O^T = V^T P^T;
//   dQ pass  recompute S, P; dP^T = V dO^T; dS = P (dP - delta); dQ^T = K^T dS^T;
//   dK/dV    key-owned: S = Q K^T, dP = dO V^T; dV^T += dO^T P; dK^T += Q^T dS.
// Products that contract over the token index use a k-slot permutation (slot 8g+j <-> token
// 32u + 4g + j for j < 4, 32u + 16 + 4g + j - 4 otherwise) so that accumulator registers
// feed the next MFMA directly; the matching operand is read with ds_read_b64_tr_b16.
#include "common.h"

namespace {

// [rows][64] bf16 image, 128-B rows; 16-B chunk index XOR ((row >> 1) & 3) << 1 makes both
// the ds_read_b128 row reads and the tr_b16 column reads conflict-free.
DFU_DEV int r128_off(int row, int chunk) { return row * 128 + ((chunk ^ (((row >> 1) & 3) << 1)) << 4); }

typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

DFU_DEV bf16x8 row_frag(const char* lds, int rb, int ks, int lane) {
  return *(const bf16x8*)(lds + r128_off(rb + (lane & 15), ks * 4 + (lane >> 4)));
}
// Transposed fragment over token chunk u (32 tokens, slot-permuted), feature tile d0.
DFU_DEV bf16x8 tr_frag(const char* lds, int u, int d0, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int col = d0 + 4 * p;
  const int chunk = col >> 3, half = (col >> 2) & 1;
  const int r0 = 32 * u + 4 * g + q;
  const char* a0 = lds + r128_off(r0, chunk) + half * 8;
  const char* a1 = lds + r128_off(r0 + 16, chunk) + half * 8;
  bf16x4 x0 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)a0);
  bf16x4 x1 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)a1);
  return __builtin_shufflevector(x0, x1, 0, 1, 2, 3, 4, 5, 6, 7);
}
// The same fragment by asm reads (common.h lds_tr16_b64), for kernels that stage by LDS-DMA:
// retire them (lds_reads_retired + pin) before the first use.
DFU_DEV bf16x8 tr_frag_asm(const char* lds, int u, int d0, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int col = d0 + 4 * p;
  const int chunk = col >> 3, half = (col >> 2) & 1;
  const int r0 = 32 * u + 4 * g + q;
  bf16x4 x0 = lds_tr16_b64(lds + r128_off(r0, chunk) + half * 8);
  bf16x4 x1 = lds_tr16_b64(lds + r128_off(r0 + 16, chunk) + half * 8);
  return __builtin_shufflevector(x0, x1, 0, 1, 2, 3, 4, 5, 6, 7);
}
template <bool H16 = false>
DFU_DEV bf16x8 pack_frag(const f32x4& a, const f32x4& b) {
  u32x4 w;
  if constexpr (H16) {
    w[0] = pack2h(a[0], a[1]);
    w[1] = pack2h(a[2], a[3]);
    w[2] = pack2h(b[0], b[1]);
    w[3] = pack2h(b[2], b[3]);
  } else {
    w[0] = pack2(a[0], a[1]);
    w[1] = pack2(a[2], a[3]);
    w[2] = pack2(b[0], b[1]);
    w[3] = pack2(b[2], b[3]);
  }
  return __builtin_bit_cast(bf16x8, w);
}
// One 16x16x32 MFMA on 16-bit operands held as bf16x8 bits: bf16, or fp16 (H16).
template <bool H16>
DFU_DEV f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  if constexpr (H16)
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a),
                                                  __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// Copy rows [0, NPAD) of one (b, h) slice of qkv (which = 0 q, 1 k, 2 v) or of a [B*N][H][64]
// tensor into an r128 LDS image; rows >= N are zero.
DFU_DEV void stage_rows(char* lds, const bf16_t* base, int64_t row_stride, int N, int NPAD,
                        int tid, int nthr = 256) {
  for (int idx = tid; idx < NPAD * 8; idx += nthr) {
    const int row = idx >> 3, chunk = idx & 7;
    u32x4 v = {0u, 0u, 0u, 0u};
    if (row < N) v = *(const u32x4*)(base + (int64_t)row * row_stride + chunk * 8);
    *(u32x4*)(lds + r128_off(row, chunk)) = v;
  }
}

// Two images at once (e.g. K and V), every load of the thread issued before any LDS write: one
// memory round trip for the whole staging (a load-then-write loop pays one per iteration).
template <int NPAD, int NTHR>
DFU_DEV void stage_rows2(char* lds0, const bf16_t* base0, char* lds1, const bf16_t* base1,
                         int64_t row_stride, int N, int tid) {
  // branch-free: padding rows load row N-1 (in bounds) and are zeroed at the LDS write, so the
  // loads are not split into exec-masked blocks that each wait for their own data
  constexpr int IT = (NPAD * 8 + NTHR - 1) / NTHR;
  u32x4 v0[IT], v1[IT];
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int idx = tid + i * NTHR, row = idx >> 3, chunk = idx & 7;
    const int64_t o = (int64_t)(row < N ? row : N - 1) * row_stride + chunk * 8;
    v0[i] = *(const u32x4*)(base0 + o);
    v1[i] = *(const u32x4*)(base1 + o);
  }
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int idx = tid + i * NTHR, row = idx >> 3, chunk = idx & 7;
    const u32x4 z = {0u, 0u, 0u, 0u};
    if (idx < NPAD * 8) {
      *(u32x4*)(lds0 + r128_off(row, chunk)) = row < N ? v0[i] : z;
      *(u32x4*)(lds1 + r128_off(row, chunk)) = row < N ? v1[i] : z;
    }
  }
}

constexpr float LOG2E = 1.4426950408889634f;

// 2^x by the bare v_exp_f32 (softmax arguments are <= 0 and only need ~1 ulp; below 2^-126 the
// hardware result flushes to 0, which a probability that small may).  exp2f would wrap it in
// range-reduction code (cmp, cndmask, ldexp) that made the attention kernels VALU-bound.
DFU_DEV float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// 16 zero bytes: the LDS-DMA source of padding rows
__device__ __attribute__((aligned(16))) const uint32_t g_attn_zero16[4] = {0u, 0u, 0u, 0u};

typedef __attribute__((address_space(3))) void attn_lds_void;
typedef const __attribute__((address_space(1))) void attn_glb_void;

// Issue this wave's share of the LDS-DMA that stages the K and V images of one (b, h) slice
// (rows >= N zero) into `img` (K at 0, V at NPAD*128).  One wave instruction fills 1 KiB = 8 rows
// of an r128 image at a wave-uniform base, lane l at base + 16 l: row 8j + (l >> 3), position
// l & 7, which in the r128 image holds 16-B chunk (l & 7) ^ swizzle(row).  The images' 4*KT
// instructions are spread over the NW waves, KT/2 each (KT even: NPAD is a multiple of 32).
template <int KT, int NW>
DFU_DEV void stage_kv_dma(char* img, const bf16_t* kbase, const bf16_t* vbase,
                          int64_t tok_stride, int N, int wave, int lane) {
  constexpr int PER_IMG = 2 * KT;  // NPAD * 128 / 1024
  constexpr int PER_WAVE = 4 * KT / NW;
  static_assert((4 * KT) % NW == 0, "DMA instructions split evenly over the waves");
#pragma unroll
  for (int i = 0; i < PER_WAVE; ++i) {
    const int j = wave + NW * i;
    const int im = j / PER_IMG, blk = j - im * PER_IMG;
    const int row = 8 * blk + (lane >> 3);
    const int chunk = (lane & 7) ^ (((row >> 1) & 3) << 1);
    const bf16_t* base = im ? vbase : kbase;
    const void* src = row < N ? (const void*)(base + (int64_t)row * tok_stride + chunk * 8)
                              : (const void*)g_attn_zero16;
    char* dst = img + im * (KT * 16 * 128) + blk * 1024;
    __builtin_amdgcn_global_load_lds((attn_glb_void*)src, (attn_lds_void*)dst, 16, 0, 0);
  }
}

// Persistent forward: one 8-wave workgroup per CU walks the (b, h) slices blockIdx.x,
// + gridDim.x, ...; the K/V images live in two LDS buffers, and the next slice's images are
// DMA'd (global_load_lds, no register round trip) while this one is computed, so the staging
// latency that a one-slice-per-workgroup launch exposed (216 VGPRs: one workgroup per CU)
// overlaps the math.  13 query tiles of 16 at N = 197: at most 2 per wave.
// H16: fp16 qkv and P (the "parity" precision mode's ViT forward): o is written in fp16 (the
// proj GEMM's operand) and in bf16 to o_bf (what the bf16 backward reads).
template <int KT, int NW = 8, bool H16 = false>
__global__ __launch_bounds__(64 * NW) void k_attn_fwd(const bf16_t* __restrict__ qkv, int N, int H,
                                                      int BH, float scale,
                                                      bf16_t* __restrict__ o,
                                                      float* __restrict__ lse,
                                                      bf16_t* __restrict__ o_bf = nullptr) {
  constexpr int NPAD = KT * 16;
  constexpr int IMG2 = 2 * NPAD * 128;  // K + V images of one slice
  constexpr int QPW = 2;                // query tiles per wave and slice (QT <= 2 * NW)
  __shared__ __attribute__((aligned(16))) char smem[2 * IMG2];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4;
  const int64_t tok_stride = (int64_t)3 * H * 64;
  const int QT = (N + 15) / 16;
  const float c = scale * LOG2E;
  auto slice_base = [&](int bh) {
    const int b = bh / H, h = bh - b * H;
    return qkv + (int64_t)b * N * tok_stride + h * 64;
  };
  // Query tile of slot j of this wave in the it-th slice: the QT <= 2 NW tiles sit in the
  // slots wave + NW j rotated by it & 3, so the SIMD holding the surplus tile (13 tiles on 4
  // SIMDs at N = 197) changes from slice to slice: 10 instead of 12 tiles on the busiest SIMD
  // over a CU's three slices at B = 64.
  auto qtile = [&](int j, int itv) { return (wave + NW * j + 2 * NW - (itv & 3)) % (2 * NW); };
  // this wave's query fragments of a slice (exactly 2 QPW loads per lane, branch-free: rows
  // past N re-read row N - 1, unused)
  auto load_q = [&](int bh, int itv, u32x4 (&v)[QPW][2]) {
    const bf16_t* qbase = slice_base(bh);
#pragma unroll
    for (int j = 0; j < QPW; ++j) {
      const int q = qtile(j, itv) * 16 + (lane & 15);
      const int64_t qo = (int64_t)(q < N ? q : N - 1) * tok_stride + 8 * g;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) v[j][ks] = *(const u32x4*)(qbase + qo + 32 * ks);
    }
  };
  u32x4 qn[QPW][2];
  {
    const bf16_t* qb = slice_base(blockIdx.x);
    stage_kv_dma<KT, NW>(smem, qb + H * 64, qb + 2 * H * 64, tok_stride, N, wave, lane);
    load_q(blockIdx.x, 0, qn);
  }
  int it = 0;
  for (int bh = blockIdx.x; bh < BH; bh += gridDim.x, ++it) {
    const char* Ks = smem + (it & 1) * IMG2;
    const char* Vs = Ks + NPAD * 128;
    const int b = bh / H, h = bh - b * H;
    // this slice's images and query fragments have landed (and the previous slice's stores):
    // one wait, pinned to the query registers so the compiler's own wait for them happens
    // here and not in front of the first MFMA (where it would also drain the next DMA)
    u32x4 qv[QPW][2];
#pragma unroll
    for (int j = 0; j < QPW; ++j)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) qv[j][ks] = qn[j][ks];
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(qv[0][0]), "+v"(qv[0][1]), "+v"(qv[1][0]),
                 "+v"(qv[1][1])::"memory");
    // after the barrier every wave is past the previous slice, so the other buffer is free:
    // stage the next slice into it, and prefetch the next slice's query fragments (the last
    // slice re-stages / re-loads itself: unconditional, fixed-count issues)
    __builtin_amdgcn_s_barrier();  // (no fence: the wait above is the one needed)
    {
      const int nb = bh + (int)gridDim.x < BH ? bh + (int)gridDim.x : bh;
      const bf16_t* nq = slice_base(nb);
      stage_kv_dma<KT, NW>(smem + ((it + 1) & 1) * IMG2, nq + H * 64, nq + 2 * H * 64,
                           tok_stride, N, wave, lane);
      load_q(nb, it + 1, qn);
    }
#pragma unroll
    for (int j = 0; j < QPW; ++j) {
      const int qt = qtile(j, it);
      if (qt >= QT) continue;
      const int q = qt * 16 + (lane & 15);
      bf16x8 qf[2];
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) qf[ks] = __builtin_bit_cast(bf16x8, qv[j][ks]);
      f32x4 s[KT];
#pragma unroll
      for (int t = 0; t < KT; ++t) {
        s[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
        if (t >= KT - 2 && 16 * t >= N) continue;  // all keys past N: masked below, no MFMAs
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
          s[t] = mfma16<H16>(row_frag(Ks, 16 * t, ks, lane), qf[ks], s[t]);
      }
      // lane holds S[q][key = 16t + 4g + r]; padding keys: NPAD rounds N up to a multiple of
      // 32, so only the last two key tiles (a compile-time set) can hold them
      float mx = -INFINITY;
#pragma unroll
      for (int t = 0; t < KT; ++t) {
        if (t >= KT - 2) {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (16 * t + 4 * g + r >= N) s[t][r] = -INFINITY;
        }
        mx = fmaxf(mx, fmaxf(fmaxf(s[t][0], s[t][1]), fmaxf(s[t][2], s[t][3])));
      }
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      // exponent arguments and the row sum on packed pairs (v_pk_fma_f32 / v_pk_add_f32)
      const f32x2 c2 = {c, c}, b2 = {-mx * c, -mx * c};
      f32x2 l2 = {0.f, 0.f};
#pragma unroll
      for (int t = 0; t < KT; ++t)
#pragma unroll
        for (int r = 0; r < 4; r += 2) {
          f32x2 a = {s[t][r], s[t][r + 1]};
          a = a * c2 + b2;
          a[0] = fast_exp2(a[0]);
          a[1] = fast_exp2(a[1]);
          s[t][r] = a[0];
          s[t][r + 1] = a[1];
          l2 += a;
        }
      float l = l2[0] + l2[1];
      l += __shfl_xor(l, 16, 64);
      l += __shfl_xor(l, 32, 64);
      f32x4 acc[4];
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) acc[dt] = (f32x4){0.f, 0.f, 0.f, 0.f};
      // V^T fragments one 32-token chunk ahead: chunk u+1's reads go out before chunk u's MFMAs
      bf16x8 vf[4];
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) vf[dt] = tr_frag_asm(Vs, 0, 16 * dt, lane);
#pragma unroll
      for (int u = 0; u < KT / 2; ++u) {
        const bf16x8 pb = pack_frag<H16>(s[2 * u], s[2 * u + 1]);
        lds_reads_retired();
        bf16x8 cur[4];
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          pin(vf[dt]);
          cur[dt] = vf[dt];
        }
        if (u + 1 < KT / 2) {
#pragma unroll
          for (int dt = 0; dt < 4; ++dt) vf[dt] = tr_frag_asm(Vs, u + 1, 16 * dt, lane);
        }
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) acc[dt] = mfma16<H16>(cur[dt], pb, acc[dt]);
      }
      if (q < N) {
        const float inv = 1.0f / l;
        const int64_t oe = ((int64_t)b * N + q) * H * 64 + h * 64 + 4 * g;
        bf16_t* orow = o + oe;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          const float o0 = acc[dt][0] * inv, o1 = acc[dt][1] * inv;
          const float o2 = acc[dt][2] * inv, o3 = acc[dt][3] * inv;
          if constexpr (H16) {
            *(u32x2*)(orow + 16 * dt) = (u32x2){pack2h(o0, o1), pack2h(o2, o3)};
            *(u32x2*)(o_bf + oe + 16 * dt) = (u32x2){pack2(o0, o1), pack2(o2, o3)};
          } else {
            *(u32x2*)(orow + 16 * dt) = (u32x2){pack2(o0, o1), pack2(o2, o3)};
          }
        }
        if (g == 0) lse[(int64_t)bh * NPAD + q] = mx * scale + logf(l);
      }
    }
  }
  // the last (redundant) DMA lands before the workgroup's LDS is released
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// Fused backward: one workgroup (8 waves) per (b, h).  Q, K, V, dO are staged once into LDS
// (4 r128 images), with LSE and delta = rowsum(dO * O); then the waves share one pool of work
// items: QT query tiles (dQ: recompute S and P, dP^T = V dO^T, dS = P (dP - delta),
// dQ^T = K^T dS^T) and QT key tiles (dK/dV: S = Q K^T, dP = dO V^T; dV^T += dO^T P,
// dK^T += Q^T dS).
// Q16: qkv is the fp16 tensor of the "parity" mode's forward, rounded to bf16 while staging
// (the bf16 backward's operands; no bf16 copy of qkv is written in the forward).
DFU_DEV u32x4 f16x8_to_bf16x8(u32x4 v) {
  const f16x8 h = __builtin_bit_cast(f16x8, v);
  float f[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) f[e] = (float)h[e];
  return pack8(f);
}

template <int KT, bool Q16 = false>
__global__ __launch_bounds__(512) void k_attn_bwd_fused(const bf16_t* __restrict__ qkv,
                                                        const bf16_t* __restrict__ o,
                                                        const bf16_t* __restrict__ dout,
                                                        const float* __restrict__ lse, int N,
                                                        int H, float scale,
                                                        bf16_t* __restrict__ dqkv) {
  constexpr int NPAD = KT * 16;
  constexpr int NTH = 512, NWAVES = 8;
  __shared__ __attribute__((aligned(16))) char smem[4 * NPAD * 128 + 2 * NPAD * 4];
  char* Qs = smem;
  char* Ks = smem + NPAD * 128;
  char* Vs = smem + 2 * NPAD * 128;
  char* Ds = smem + 3 * NPAD * 128;
  float* Ls = (float*)(smem + 4 * NPAD * 128);
  float* Es = Ls + NPAD;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4;
  const int bh = blockIdx.x, b = bh / H, h = bh - b * H;
  const int64_t tok_stride = (int64_t)3 * H * 64;
  const int64_t o_stride = (int64_t)H * 64;
  const bf16_t* qbase = qkv + (int64_t)b * N * tok_stride + h * 64;
  const bf16_t* obase = o + (int64_t)b * N * o_stride + h * 64;
  const bf16_t* dobase = dout + (int64_t)b * N * o_stride + h * 64;
  // all of a thread's staging loads (IT iterations x 5 tensors) issued before any is used
  constexpr int IT = (NPAD * 8 + NTH - 1) / NTH;
  u32x4 pq[IT], pk[IT], pv[IT], pd[IT], po[IT];
#pragma unroll
  for (int i = 0; i < IT; ++i) {  // branch-free as stage_rows2: padding rows load row N-1
    const int idx = tid + i * NTH, row = idx >> 3, chunk = idx & 7;
    const int rr = row < N ? row : N - 1;
    const bf16_t* t = qbase + (int64_t)rr * tok_stride + chunk * 8;
    pq[i] = *(const u32x4*)t;
    pk[i] = *(const u32x4*)(t + H * 64);
    pv[i] = *(const u32x4*)(t + 2 * H * 64);
    pd[i] = *(const u32x4*)(dobase + (int64_t)rr * o_stride + chunk * 8);
    po[i] = *(const u32x4*)(obase + (int64_t)rr * o_stride + chunk * 8);
  }
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int idx = tid + i * NTH, row = idx >> 3, chunk = idx & 7;
    if (idx >= NPAD * 8) break;
    const u32x4 z = {0u, 0u, 0u, 0u};
    const bool in = row < N;
    if constexpr (Q16) {
      pq[i] = f16x8_to_bf16x8(pq[i]);
      pk[i] = f16x8_to_bf16x8(pk[i]);
      pv[i] = f16x8_to_bf16x8(pv[i]);
    }
    const u32x4 vq = in ? pq[i] : z, vk = in ? pk[i] : z, vv = in ? pv[i] : z,
                vd = in ? pd[i] : z, vo = in ? po[i] : z;
    const int off = r128_off(row, chunk);
    *(u32x4*)(Qs + off) = vq;
    *(u32x4*)(Ks + off) = vk;
    *(u32x4*)(Vs + off) = vv;
    *(u32x4*)(Ds + off) = vd;
    float fd[8], fo[8];
    unpack8(vd, fd);
    unpack8(vo, fo);
    float d = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) d += fd[e] * fo[e];
    d += __shfl_xor(d, 1, 64);  // the 8 chunks of a row are 8 consecutive lanes
    d += __shfl_xor(d, 2, 64);
    d += __shfl_xor(d, 4, 64);
    // padding queries get LSE = +inf: every probability of theirs is exp2(-inf) = 0, so no
    // element needs a query mask below; padding keys need none either (their K, V rows are 0,
    // so they add nothing to dQ, and their own dK / dV rows are never stored)
    if (chunk == 0) {
      Es[row] = row < N ? d : 0.f;
      Ls[row] = row < N ? lse[(int64_t)bh * NPAD + row] * LOG2E : INFINITY;
    }
  }
  __syncthreads();
  const float c = scale * LOG2E;
  const int QT = (N + 15) / 16;
  for (int it = wave; it < 2 * QT; it += NWAVES) {
    if (it < QT) {  // ---------------- dQ for query tile it
      const int qt = it;
      const int q = qt * 16 + (lane & 15);
      const bool qv = q < N;
      bf16x8 qf[2], df[2];
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        qf[ks] = row_frag(Qs, 16 * qt, ks, lane);
        df[ks] = row_frag(Ds, 16 * qt, ks, lane);
      }
      const float dsum = Es[q], lq = Ls[q];
      f32x4 s[KT];
#pragma unroll
      for (int t = 0; t < KT; ++t) {
        s[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
        // key tiles past N (the last of NPAD's 32-row rounding) hold only zero K rows: their
        // dS adds exactly 0 to dQ, so they are skipped (bit-identical)
        if (t >= KT - 2 && 16 * t >= N) continue;
        f32x4 st = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          st = __builtin_amdgcn_mfma_f32_16x16x32_bf16(row_frag(Ks, 16 * t, ks, lane), qf[ks], st, 0, 0, 0);
          dp = __builtin_amdgcn_mfma_f32_16x16x32_bf16(row_frag(Vs, 16 * t, ks, lane), df[ks], dp, 0, 0, 0);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) st[r] = fast_exp2(fmaf(st[r], c, -lq)) * (dp[r] - dsum);
        s[t] = st;
      }
      f32x4 acc[4];
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) acc[dt] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int u = 0; u < KT / 2; ++u) {
        const bf16x8 dsb = pack_frag(s[2 * u], s[2 * u + 1]);
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
          acc[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(tr_frag(Ks, u, 16 * dt, lane), dsb, acc[dt], 0, 0, 0);
      }
      if (qv) {
        bf16_t* dst = dqkv + ((int64_t)b * N + q) * tok_stride + h * 64 + 4 * g;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
          *(u32x2*)(dst + 16 * dt) = (u32x2){pack2(acc[dt][0] * scale, acc[dt][1] * scale),
                                             pack2(acc[dt][2] * scale, acc[dt][3] * scale)};
      }
    } else {  // ---------------- dK, dV for key tile it - QT
      const int kt = it - QT;
      const int key = kt * 16 + (lane & 15);
      const bool kv = key < N;
      bf16x8 kf[2], vf[2];
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        kf[ks] = row_frag(Ks, 16 * kt, ks, lane);
        vf[ks] = row_frag(Vs, 16 * kt, ks, lane);
      }
      f32x4 dv[4], dk[4];
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        dv[dt] = (f32x4){0.f, 0.f, 0.f, 0.f};
        dk[dt] = (f32x4){0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll 1
      for (int u = 0; u < KT / 2; ++u) {
        f32x4 ph[2], dsh[2];
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          const int qt = 2 * u + hh;
          if (qt >= QT) {  // a query tile past N: P = 0 (LSE = +inf), nothing to add
            ph[hh] = dsh[hh] = (f32x4){0.f, 0.f, 0.f, 0.f};
            continue;
          }
          f32x4 st = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) {
            st = __builtin_amdgcn_mfma_f32_16x16x32_bf16(row_frag(Qs, 16 * qt, ks, lane), kf[ks], st, 0, 0, 0);
            dp = __builtin_amdgcn_mfma_f32_16x16x32_bf16(row_frag(Ds, 16 * qt, ks, lane), vf[ks], dp, 0, 0, 0);
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int q = 16 * qt + 4 * g + r;
            const float pv = fast_exp2(fmaf(st[r], c, -Ls[q]));
            ph[hh][r] = pv;
            dsh[hh][r] = pv * (dp[r] - Es[q]);
          }
        }
        const bf16x8 pb = pack_frag(ph[0], ph[1]);
        const bf16x8 db = pack_frag(dsh[0], dsh[1]);
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          dv[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(tr_frag(Ds, u, 16 * dt, lane), pb, dv[dt], 0, 0, 0);
          dk[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(tr_frag(Qs, u, 16 * dt, lane), db, dk[dt], 0, 0, 0);
        }
      }
      if (kv) {
        bf16_t* dst = dqkv + ((int64_t)b * N + key) * tok_stride + h * 64 + 4 * g;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          *(u32x2*)(dst + H * 64 + 16 * dt) = (u32x2){pack2(dk[dt][0] * scale, dk[dt][1] * scale),
                                                      pack2(dk[dt][2] * scale, dk[dt][3] * scale)};
          *(u32x2*)(dst + 2 * H * 64 + 16 * dt) = (u32x2){pack2(dv[dt][0], dv[dt][1]),
                                                          pack2(dv[dt][2], dv[dt][3])};
        }
      }
    }
  }
}

// ------------------------------------------------------------------ bf16x3 forward
// fp32-accurate attention for the "bf16x3" precision mode (include/dfu_hip.h): the same MFMA
// dataflow as k_attn_fwd on split operands x = hi + lo (hi = bf16(x), lo = bf16(x - hi)):
//   S^T = Khi Qhi^T + Khi Qlo^T + Klo Qhi^T,   O^T = Vhi^T Phi^T + Vhi^T Plo^T + Vlo^T Phi^T
// with the softmax in fp32 between them, i.e. every product keeps 16 mantissa bits (the
// dropped lo*lo term and the split remainders are ~2^-17 relative per product, against
// bf16's 2^-9).  One 8-wave workgroup per (b, h): K and V are read from the fp32 qkv GEMM
// output and split into four r128 LDS images while staging; each wave owns query tiles
// wave, wave + 8.  The kernel also writes the plain bf16 copy of qkv (hi: the bf16 backward's
// operand; every element is read exactly once here), o as the A-operand triple
// [hi | lo | hi] of the proj GEMM, o bf16 and the LSE, exactly as k_attn_fwd's.
DFU_DEV void split_f4(const f32x4 v, u32x2& hi, u32x2& lo) {
  hi = (u32x2){pack2(v[0], v[1]), pack2(v[2], v[3])};
  const f32x4 r = {v[0] - lo_bf(hi[0]), v[1] - hi_bf(hi[0]), v[2] - lo_bf(hi[1]),
                   v[3] - hi_bf(hi[1])};
  lo = (u32x2){pack2(r[0], r[1]), pack2(r[2], r[3])};
}

template <int KT>
__global__ __launch_bounds__(512) void k_attn_fwd_x3(const float* __restrict__ qkv, int N, int H,
                                                     float scale, int npad,
                                                     bf16_t* __restrict__ qkv_bf,
                                                     bf16_t* __restrict__ o3,
                                                     bf16_t* __restrict__ o_bf,
                                                     float* __restrict__ lse) {
  constexpr int NPAD = KT * 16;
  constexpr int IMG = NPAD * 128;
  constexpr int NTH = 512, NW = 8;
  __shared__ __attribute__((aligned(16))) char smem[4 * IMG];  // K hi, K lo, V hi, V lo
  char* Kh = smem;
  char* Kl = smem + IMG;
  char* Vh = smem + 2 * IMG;
  char* Vl = smem + 3 * IMG;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4;
  const int bh = blockIdx.x, b = bh / H, h = bh - b * H;
  const int D = H * 64;
  const int64_t tok = (int64_t)3 * D;
  const float* base = qkv + (int64_t)b * N * tok + h * 64;
  bf16_t* bbase = qkv_bf ? qkv_bf + (int64_t)b * N * tok + h * 64 : nullptr;
  // staging, one tensor at a time (K, then V): 16 float4 per row; every load of the tensor
  // issued before any conversion
  constexpr int IT = (NPAD * 16 + NTH - 1) / NTH;
#pragma unroll
  for (int which = 1; which <= 2; ++which) {
    char* dh = which == 1 ? Kh : Vh;
    char* dl = which == 1 ? Kl : Vl;
    f32x4 v[IT];
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int idx = tid + i * NTH, row = idx >> 4, c4 = idx & 15;
      const int64_t o = (int64_t)(row < N ? row : N - 1) * tok + 4 * c4;
      v[i] = *(const f32x4*)(base + which * D + o);
    }
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int idx = tid + i * NTH, row = idx >> 4, c4 = idx & 15;
      if (idx < NPAD * 16) {
        const bool in = row < N;
        const int off = r128_off(row, c4 >> 1) + (c4 & 1) * 8;
        u32x2 hi, lo;
        split_f4(v[i], hi, lo);
        const u32x2 z = {0u, 0u};
        *(u32x2*)(dh + off) = in ? hi : z;
        *(u32x2*)(dl + off) = in ? lo : z;
        if (bbase && in) *(u32x2*)(bbase + (int64_t)row * tok + which * D + 4 * c4) = hi;
      }
    }
  }
  __syncthreads();
  const float c = scale * LOG2E;
  const int QT = (N + 15) / 16;
  for (int qt = wave; qt < QT; qt += NW) {
    const int q = qt * 16 + (lane & 15);
    const bool qvalid = q < N;
    bf16x8 qh[2], ql[2];
    {
      const int64_t qo = (int64_t)(qvalid ? q : N - 1) * tok + 8 * g;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const f32x4 a = *(const f32x4*)(base + qo + 32 * ks);
        const f32x4 bq = *(const f32x4*)(base + qo + 32 * ks + 4);
        u32x2 ha, la, hb, lb;
        split_f4(a, ha, la);
        split_f4(bq, hb, lb);
        qh[ks] = __builtin_bit_cast(bf16x8, (u32x4){ha[0], ha[1], hb[0], hb[1]});
        ql[ks] = __builtin_bit_cast(bf16x8, (u32x4){la[0], la[1], lb[0], lb[1]});
        if (bbase && qvalid)
          *(u32x4*)(bbase + (int64_t)q * tok + 8 * g + 32 * ks) = (u32x4){ha[0], ha[1], hb[0], hb[1]};
      }
    }
    f32x4 s[KT];
#pragma unroll
    for (int t = 0; t < KT; ++t) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const bf16x8 khf = row_frag(Kh, 16 * t, ks, lane);
        const bf16x8 klf = row_frag(Kl, 16 * t, ks, lane);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(klf, qh[ks], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(khf, ql[ks], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(khf, qh[ks], acc, 0, 0, 0);
      }
      s[t] = acc;
      // bound the scheduler's hoisting of later tiles' LDS reads (each is 8 VGPRs: hoisting
      // them all spilled)
      if (t % 2 == 1) __builtin_amdgcn_sched_barrier(0);
    }
    float mx = -INFINITY;
#pragma unroll
    for (int t = 0; t < KT; ++t) {
      if (t >= KT - 2) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (16 * t + 4 * g + r >= N) s[t][r] = -INFINITY;
      }
      mx = fmaxf(mx, fmaxf(fmaxf(s[t][0], s[t][1]), fmaxf(s[t][2], s[t][3])));
    }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    float l = 0.f;
#pragma unroll
    for (int t = 0; t < KT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = fast_exp2(fmaf(s[t][r], c, -mx * c));
        s[t][r] = p;
        l += p;
      }
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
    f32x4 acc[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) acc[dt] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < KT / 2; ++u) {
      f32x4 r0, r1;
      const bf16x8 ph = pack_frag(s[2 * u], s[2 * u + 1]);
      {
        const u32x4 w = __builtin_bit_cast(u32x4, ph);
        r0 = (f32x4){s[2 * u][0] - lo_bf(w[0]), s[2 * u][1] - hi_bf(w[0]),
                     s[2 * u][2] - lo_bf(w[1]), s[2 * u][3] - hi_bf(w[1])};
        r1 = (f32x4){s[2 * u + 1][0] - lo_bf(w[2]), s[2 * u + 1][1] - hi_bf(w[2]),
                     s[2 * u + 1][2] - lo_bf(w[3]), s[2 * u + 1][3] - hi_bf(w[3])};
      }
      const bf16x8 pl = pack_frag(r0, r1);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const bf16x8 vhf = tr_frag(Vh, u, 16 * dt, lane);
        const bf16x8 vlf = tr_frag(Vl, u, 16 * dt, lane);
        acc[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vlf, ph, acc[dt], 0, 0, 0);
        acc[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vhf, pl, acc[dt], 0, 0, 0);
        acc[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vhf, ph, acc[dt], 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if (qvalid) {
      const float inv = 1.0f / l;
      const int64_t row = (int64_t)b * N + q;
      const int col = h * 64 + 4 * g;
      bf16_t* r3 = o3 + row * 3 * D + col;
      bf16_t* rb = o_bf + row * D + col;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        u32x2 hi, lo;
        split_f4(acc[dt] * inv, hi, lo);
        *(u32x2*)(rb + 16 * dt) = hi;
        *(u32x2*)(r3 + 16 * dt) = hi;
        *(u32x2*)(r3 + D + 16 * dt) = lo;
        *(u32x2*)(r3 + 2 * D + 16 * dt) = hi;
      }
      if (g == 0) lse[(int64_t)bh * npad + q] = mx * scale + logf(l);
    }
  }
}

#define DISPATCH_KT(KTV, CALL) \
  switch (KTV) {               \
    case 2: CALL(2); break;    \
    case 4: CALL(4); break;    \
    case 6: CALL(6); break;    \
    case 8: CALL(8); break;    \
    case 10: CALL(10); break;  \
    case 12: CALL(12); break;  \
    case 14: CALL(14); break;  \
    case 16: CALL(16); break;  \
    default: break;            \
  }

int attn_cus() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
    cus = n;
  }
  return cus;
}

}  // namespace

extern "C" int dfu_attention_npad(int32_t N) { return ((N + 31) / 32) * 32; }

extern "C" int dfu_attention_fwd(const void* qkv, int32_t B, int32_t N, int32_t H, int32_t dh,
                                 float scale, void* o, float* lse, void* stream) {
  DFU_CHECK_ARG(qkv && o && lse && B > 0 && H > 0, "dfu_attention_fwd: bad args");
  DFU_CHECK_ARG(dh == 64, "dfu_attention_fwd: head dim %d unsupported (64 only)", dh);
  DFU_CHECK_ARG(N > 0 && N <= 256, "dfu_attention_fwd: N=%d unsupported (<= 256)", N);
  const int KT = dfu_attention_npad(N) / 16;
  hipStream_t s = (hipStream_t)stream;
  const int BH = B * H;
  const int grid = BH < attn_cus() ? BH : attn_cus();  // persistent: one workgroup per CU
#define CALL(K) hipLaunchKernelGGL(k_attn_fwd<K>, dim3(grid), dim3(512), 0, s, (const bf16_t*)qkv, N, H, BH, scale, (bf16_t*)o, lse)
  DISPATCH_KT(KT, CALL)
#undef CALL
  DFU_LAUNCH_CHECK();
  return DFU_OK;
}

extern "C" int dfu_attention_fwd_f16(const void* qkv, int32_t B, int32_t N, int32_t H, int32_t dh,
                                     float scale, void* o, void* o_bf16, float* lse,
                                     void* stream) {
  DFU_CHECK_ARG(qkv && o && o_bf16 && lse && B > 0 && H > 0, "dfu_attention_fwd_f16: bad args");
  DFU_CHECK_ARG(dh == 64, "dfu_attention_fwd_f16: head dim %d unsupported (64 only)", dh);
  DFU_CHECK_ARG(N > 0 && N <= 256, "dfu_attention_fwd_f16: N=%d unsupported (<= 256)", N);
  const int KT = dfu_attention_npad(N) / 16;
  hipStream_t s = (hipStream_t)stream;
  const int BH = B * H;
  const int grid = BH < attn_cus() ? BH : attn_cus();
#define CALL(K) hipLaunchKernelGGL((k_attn_fwd<K, 8, true>), dim3(grid), dim3(512), 0, s, (const bf16_t*)qkv, N, H, BH, scale, (bf16_t*)o, lse, (bf16_t*)o_bf16)
  DISPATCH_KT(KT, CALL)
#undef CALL
  DFU_LAUNCH_CHECK();
  return DFU_OK;
}

extern "C" int dfu_attention_fwd_f32(const float* qkv, int32_t B, int32_t N, int32_t H,
                                     int32_t dh, float scale, int32_t npad, void* qkv_bf16,
                                     void* o3, void* o_bf16, float* lse, void* stream) {
  DFU_CHECK_ARG(qkv && o3 && o_bf16 && lse && B > 0 && H > 0,
                "dfu_attention_fwd_f32: bad args");
  DFU_CHECK_ARG(dh == 64, "dfu_attention_fwd_f32: head dim %d unsupported (64 only)", dh);
  DFU_CHECK_ARG(N > 0 && N <= 224 && npad >= dfu_attention_npad(N),
                "dfu_attention_fwd_f32: N=%d unsupported (<= 224) or npad %d < %d", N, npad,
                dfu_attention_npad(N));
  const int KT = dfu_attention_npad(N) / 16;
  hipStream_t s = (hipStream_t)stream;
#define CALL(K) hipLaunchKernelGGL(k_attn_fwd_x3<K>, dim3(B * H), dim3(512), 0, s, qkv, N, H, scale, npad, (bf16_t*)qkv_bf16, (bf16_t*)o3, (bf16_t*)o_bf16, lse)
  switch (KT) {
    case 2: CALL(2); break;
    case 4: CALL(4); break;
    case 6: CALL(6); break;
    case 8: CALL(8); break;
    case 10: CALL(10); break;
    case 12: CALL(12); break;
    case 14: CALL(14); break;
    default: break;
  }
#undef CALL
  DFU_LAUNCH_CHECK();
  return DFU_OK;
}

namespace {
template <bool Q16>
int attention_bwd(const void* qkv, const void* o, const void* dout, const float* lse, int32_t B,
                  int32_t N, int32_t H, int32_t dh, float scale, float* delta, void* dqkv,
                  void* stream) {
  DFU_CHECK_ARG(qkv && o && dout && lse && delta && dqkv && B > 0 && H > 0,
                "dfu_attention_bwd: bad args");
  DFU_CHECK_ARG(dh == 64, "dfu_attention_bwd: head dim %d unsupported (64 only)", dh);
  DFU_CHECK_ARG(N > 0 && N <= 256, "dfu_attention_bwd: N=%d unsupported (<= 256)", N);
  const int KT = dfu_attention_npad(N) / 16;
  hipStream_t s = (hipStream_t)stream;
#define CALL(K) hipLaunchKernelGGL((k_attn_bwd_fused<K, Q16>), dim3(B * H), dim3(512), 0, s, (const bf16_t*)qkv, (const bf16_t*)o, (const bf16_t*)dout, lse, N, H, scale, (bf16_t*)dqkv)
  DISPATCH_KT(KT, CALL)
#undef CALL
  DFU_LAUNCH_CHECK();
  return DFU_OK;
}
}  // namespace

extern "C" int dfu_attention_bwd(const void* qkv, const void* o, const void* dout,
                                 const float* lse, int32_t B, int32_t N, int32_t H, int32_t dh,
                                 float scale, float* delta, void* dqkv, void* stream) {
  return attention_bwd<false>(qkv, o, dout, lse, B, N, H, dh, scale, delta, dqkv, stream);
}

extern "C" int dfu_attention_bwd_qkv16(const void* qkv16, const void* o, const void* dout,
                                       const float* lse, int32_t B, int32_t N, int32_t H,
                                       int32_t dh, float scale, float* delta, void* dqkv,
                                       void* stream) {
  return attention_bwd<true>(qkv16, o, dout, lse, B, N, H, dh, scale, delta, dqkv, stream);
}
