// bf16 MFMA GEMM template for gfx950 with implicit-GEMM convolution loaders and fused
// epilogues.  One kernel body serves every contraction of the DFU training step
// (SURVEY.md §2.2): ViT Linear fwd/dgrad/wgrad, NHWC conv fwd/dgrad/wgrad, fusion head.
//
// Geometry: 256 threads = 4 waves (2 x 2), block tile 128 x 128, K-step 64, each wave owns a
// 64 x 64 sub-tile = 4 x 4 v_mfma_f32_16x16x32_bf16 accumulators (fp32).
// Operands are staged global -> registers -> LDS (two LDS stages, one barrier per K-step):
// the register stage is what lets one loader serve plain, transposed and gathered (im2col)
// operands.  Two LDS images:
//   K-contiguous  [128 rows][64 k]  128-B rows, 16-B chunk index ^= (row & 7)  -> ds_read_b128
//   MN-contiguous [64 k][128 cols]  256-B rows, 16-B chunk index ^= f(k)       -> ds_read_b64_tr_b16
// both conflict-free for their reads and for the 16-B register-staged writes.
// The MFMA is issued with the operands swapped (B fragment as "A"), so each lane ends with 4
// consecutive output COLUMNS of one row: 8-B (bf16) / 16-B (fp32) epilogue stores.
#pragma once
#include "common.h"

namespace dfu {

constexpr int BM = 128, BN = 128, BK = 64, NT = 256;
constexpr int TILE_BYTES = 128 * 64 * 2;  // 16 KiB per operand tile
constexpr int STAGE_BYTES = 2 * TILE_BYTES;
constexpr int LDS_BYTES = 2 * STAGE_BYTES;  // 64 KiB -> 2 workgroups per CU

struct GemmArgs {
  int M, N, K;
  int ktiles, kt_per_split;
  int tiles_m, tiles_n;
  const bf16_t* A;
  int64_t lda;
  const bf16_t* B;
  int64_t ldb;
  void* C;
  int64_t ldc;
  float alpha;
  const float* bias;
  const void* aux;
  int64_t ldaux;
  void* aux_out;
  int64_t ldaux_out;
  float* stats;
  int split;
  int ep_tokens;
  // conv geometry
  int cn, ch, cw, cc, ck, cr, cs, cstride, cpad, cp, cq;
  FastDiv div_pq, div_q, div_hw, div_w, div_c, div_k, div_s;
  int m_ld_bound;  // rows of MN-contiguous operands may be read up to this column bound
  int n_ld_bound;
};

// ------------------------------------------------------------------------------ LDS maps
DFU_DEV int kc_off(int row, int chunk) { return row * 128 + ((chunk ^ (row & 7)) << 4); }
DFU_DEV int mn_swz(int k) { return ((k & 3) << 1) | (((k >> 3) & 1) << 3); }
DFU_DEV int mn_off(int krow, int chunk) { return krow * 256 + ((chunk ^ mn_swz(krow)) << 4); }

DFU_DEV bool is_kcontig(int mode) {
  return mode == DFU_OPND_KMAJOR || mode == DFU_OPND_CONV_FWD || mode == DFU_OPND_CONV_DGRAD;
}

// ------------------------------------------------------------------------------ loaders
// Each thread moves 4 x 16 B per operand per K-step.
struct Stage {
  u32x4 v[4];
};

// Per-thread precomputed state for one operand (rows fixed across the K loop).
struct LoadState {
  const bf16_t* ptr[4];  // row base pointers (KMAJOR) / unused
  int i0[4], i1[4];      // conv: ih0/iw0 (fwd) or h/w (dgrad) per row; wgrad: r,s per chunk
  int valid[4];
  int bofs[4];           // conv: batch offset index
  int col;               // MN-contiguous: column (mn) of this thread's chunk
  int c_in;              // wgrad: channel of this thread's chunk
};

template <int MODE>
DFU_DEV void load_init(const GemmArgs& p, LoadState& st, const bf16_t* base, int64_t ld, int mn0,
                       int MN, int tid) {
  if constexpr (MODE == DFU_OPND_KMAJOR) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = mn0 + (tid >> 3) + 32 * i;
      st.valid[i] = row < MN;
      st.ptr[i] = base + (int64_t)(st.valid[i] ? row : 0) * ld + (tid & 7) * 8;
    }
  } else if constexpr (MODE == DFU_OPND_CONV_FWD) {
    // rows = output positions m = (b, oh, ow)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = mn0 + (tid >> 3) + 32 * i;
      st.valid[i] = m < MN;
      const uint32_t mm = st.valid[i] ? m : 0;
      const uint32_t b = fdiv(mm, p.div_pq);
      const uint32_t rem = mm - b * (uint32_t)(p.cp * p.cq);
      const uint32_t oh = fdiv(rem, p.div_q);
      const uint32_t ow = rem - oh * p.cq;
      st.i0[i] = (int)oh * p.cstride - p.cpad;
      st.i1[i] = (int)ow * p.cstride - p.cpad;
      st.bofs[i] = (int)b;
    }
  } else if constexpr (MODE == DFU_OPND_CONV_DGRAD) {
    // rows = input positions m = (b, h, w) of dX
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = mn0 + (tid >> 3) + 32 * i;
      st.valid[i] = m < MN;
      const uint32_t mm = st.valid[i] ? m : 0;
      const uint32_t b = fdiv(mm, p.div_hw);
      const uint32_t rem = mm - b * (uint32_t)(p.ch * p.cw);
      const uint32_t h = fdiv(rem, p.div_w);
      const uint32_t w = rem - h * p.cw;
      st.i0[i] = (int)h + p.cpad;
      st.i1[i] = (int)w + p.cpad;
      st.bofs[i] = (int)b;
    }
  } else if constexpr (MODE == DFU_OPND_MNMAJOR || MODE == DFU_OPND_CONV_DGRAD_W) {
    st.col = mn0 + (tid & 15) * 8;
  } else if constexpr (MODE == DFU_OPND_CONV_WGRAD_X) {
    st.col = mn0 + (tid & 15) * 8;  // n' = (r, s, c)
    const uint32_t n = st.col;
    const uint32_t rs = fdiv(n, p.div_c);
    st.c_in = (int)(n - rs * p.cc);
    const uint32_t r = fdiv(rs, p.div_s);
    st.i0[0] = (int)r;
    st.i1[0] = (int)(rs - r * p.cs);
  }
}

// Global -> registers for K-step kt.  MN is the extent of the operand's row/col dimension.
template <int MODE>
DFU_DEV void load_tile(const GemmArgs& p, const LoadState& st, const bf16_t* base, int64_t ld,
                       int MN_bound, int kt, int kend, int tid, Stage& s) {
  const int k0 = kt * BK;
  const u32x4 z = {0u, 0u, 0u, 0u};
  if constexpr (MODE == DFU_OPND_KMAJOR) {
    const int k = k0 + (tid & 7) * 8;
    const bool kin = k < kend;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      s.v[i] = (st.valid[i] && kin) ? *(const u32x4*)(st.ptr[i] + k0) : z;
  } else if constexpr (MODE == DFU_OPND_CONV_FWD) {
    // whole K-step lies in one filter tap (C % 64 == 0, host-checked)
    const uint32_t rs = fdiv((uint32_t)k0, p.div_c);
    const int c0 = k0 - (int)rs * p.cc + (tid & 7) * 8;
    const uint32_t r = fdiv(rs, p.div_s);
    const int sx = (int)(rs - r * p.cs);
    const bool kin = k0 < kend;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int ih = st.i0[i] + (int)r, iw = st.i1[i] + sx;
      const bool ok = kin && st.valid[i] && (unsigned)ih < (unsigned)p.ch && (unsigned)iw < (unsigned)p.cw;
      const int64_t off = (((int64_t)st.bofs[i] * p.ch + ih) * p.cw + iw) * p.cc + c0;
      s.v[i] = ok ? *(const u32x4*)(base + off) : z;
    }
  } else if constexpr (MODE == DFU_OPND_CONV_DGRAD) {
    // K' = (r, s, kout); gather dY[b][(h+pad-r)/st][(w+pad-s)/st][kout]
    const uint32_t rs = fdiv((uint32_t)k0, p.div_k);
    const int k_0 = k0 - (int)rs * p.ck + (tid & 7) * 8;
    const uint32_t r = fdiv(rs, p.div_s);
    const int sx = (int)(rs - r * p.cs);
    const bool kin = k0 < kend;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int hn = st.i0[i] - (int)r, wn = st.i1[i] - sx;
      bool ok = kin && st.valid[i] && hn >= 0 && wn >= 0;
      int oh = hn, ow = wn;
      if (p.cstride != 1) {
        ok = ok && (hn % p.cstride == 0) && (wn % p.cstride == 0);
        oh = hn / p.cstride;
        ow = wn / p.cstride;
      }
      ok = ok && oh < p.cp && ow < p.cq;
      const int64_t off = (((int64_t)st.bofs[i] * p.cp + oh) * p.cq + ow) * p.ck + k_0;
      s.v[i] = ok ? *(const u32x4*)(base + off) : z;
    }
  } else if constexpr (MODE == DFU_OPND_MNMAJOR) {
    const bool cin = st.col < MN_bound;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int k = k0 + (tid >> 4) + 16 * i;
      s.v[i] = (cin && k < kend) ? *(const u32x4*)(base + (int64_t)k * ld + st.col) : z;
    }
  } else if constexpr (MODE == DFU_OPND_CONV_DGRAD_W) {
    // B[k'=(r,s,kout)][c] = Wkrsc[kout][r][s][c];  ld = R*S*C
    const uint32_t rs = fdiv((uint32_t)k0, p.div_k);
    const int kout0 = k0 - (int)rs * p.ck;
    const bool cin = st.col < MN_bound && k0 < kend;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int kout = kout0 + (tid >> 4) + 16 * i;
      s.v[i] = cin ? *(const u32x4*)(base + (int64_t)kout * ld + (int64_t)rs * p.cc + st.col) : z;
    }
  } else if constexpr (MODE == DFU_OPND_CONV_WGRAD_X) {
    // B[k'=m (b,oh,ow)][n'=(r,s,c)] = X[b][oh*st-pad+r][ow*st-pad+s][c]
    const bool cin = st.col < MN_bound;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = k0 + (tid >> 4) + 16 * i;
      bool ok = cin && m < kend;
      const uint32_t mm = ok ? m : 0;
      const uint32_t b = fdiv(mm, p.div_pq);
      const uint32_t rem = mm - b * (uint32_t)(p.cp * p.cq);
      const uint32_t oh = fdiv(rem, p.div_q);
      const uint32_t ow = rem - oh * p.cq;
      const int ih = (int)oh * p.cstride - p.cpad + st.i0[0];
      const int iw = (int)ow * p.cstride - p.cpad + st.i1[0];
      ok = ok && (unsigned)ih < (unsigned)p.ch && (unsigned)iw < (unsigned)p.cw;
      const int64_t off = (((int64_t)b * p.ch + ih) * p.cw + iw) * p.cc + st.c_in;
      s.v[i] = ok ? *(const u32x4*)(base + off) : z;
    }
  }
}

template <int MODE>
DFU_DEV void store_tile(char* lds, int tid, const Stage& s) {
  if constexpr (MODE == DFU_OPND_KMAJOR || MODE == DFU_OPND_CONV_FWD ||
                MODE == DFU_OPND_CONV_DGRAD) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      *(u32x4*)(lds + kc_off((tid >> 3) + 32 * i, tid & 7)) = s.v[i];
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      *(u32x4*)(lds + mn_off((tid >> 4) + 16 * i, tid & 15)) = s.v[i];
  }
}

// ------------------------------------------------------------------------------ fragments
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

// Fragment of a 16-row (or 16-col) subtile at base `rb`, k-half ks (0/1): lane holds
// X[rb + (lane&15)][ks*32 + 8*(lane>>4) + j], j = 0..7.
template <bool KCONTIG>
DFU_DEV bf16x8 read_frag(const char* lds, int rb, int ks, int lane) {
  if constexpr (KCONTIG) {
    const int row = rb + (lane & 15);
    const int chunk = ks * 4 + (lane >> 4);
    return *(const bf16x8*)(lds + kc_off(row, chunk));
  } else {
    const int g = lane >> 4, i = lane & 15, q = i >> 2, pp = i & 3;
    const int krow = ks * 32 + 8 * g + q;
    const int col = rb + 4 * pp;
    const int chunk = col >> 3, half = (col >> 2) & 1;
    const char* a0 = lds + mn_off(krow, chunk) + half * 8;
    const char* a1 = lds + mn_off(krow + 4, chunk) + half * 8;
    bf16x4 x0 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(a0));
    bf16x4 x1 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(a1));
    return __builtin_shufflevector(x0, x1, 0, 1, 2, 3, 4, 5, 6, 7);
  }
}

// ------------------------------------------------------------------------------ kernel
template <int AMODE, int BMODE, int EPI>
__global__ __launch_bounds__(NT, 2) void gemm_kernel(const GemmArgs p) {
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;

  // XCD-aware bijective remap: blocks b and b+8 share an XCD; give each XCD a contiguous
  // range of tiles so neighbouring tiles (shared A panel) hit the same L2.
  const int nwg = gridDim.x;
  const int bid = blockIdx.x;
  int wgid = bid;
  if (nwg >= 16) {
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  const int tn = wgid % p.tiles_n;
  const int tm = wgid / p.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;

  const int kt_begin = blockIdx.y * p.kt_per_split;
  const int kt_end = min(p.ktiles, kt_begin + p.kt_per_split);
  const int kend = p.K;

  LoadState sa, sb;
  load_init<AMODE>(p, sa, p.A, p.lda, m0, p.M, tid);
  load_init<BMODE>(p, sb, p.B, p.ldb, n0, p.N, tid);

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  constexpr bool AK = (AMODE == DFU_OPND_KMAJOR || AMODE == DFU_OPND_CONV_FWD ||
                       AMODE == DFU_OPND_CONV_DGRAD);
  constexpr bool BKc = (BMODE == DFU_OPND_KMAJOR || BMODE == DFU_OPND_CONV_FWD ||
                        BMODE == DFU_OPND_CONV_DGRAD);

  if (kt_begin < kt_end) {
    Stage ra, rb;
    load_tile<AMODE>(p, sa, p.A, p.lda, p.m_ld_bound, kt_begin, kend, tid, ra);
    load_tile<BMODE>(p, sb, p.B, p.ldb, p.n_ld_bound, kt_begin, kend, tid, rb);
    store_tile<AMODE>(smem, tid, ra);
    store_tile<BMODE>(smem + TILE_BYTES, tid, rb);
    __syncthreads();

    for (int kt = kt_begin; kt < kt_end; ++kt) {
      const int cur = (kt - kt_begin) & 1;
      const bool has_next = kt + 1 < kt_end;
      if (has_next) {
        load_tile<AMODE>(p, sa, p.A, p.lda, p.m_ld_bound, kt + 1, kend, tid, ra);
        load_tile<BMODE>(p, sb, p.B, p.ldb, p.n_ld_bound, kt + 1, kend, tid, rb);
      }
      const char* la = smem + cur * STAGE_BYTES;
      const char* lb = la + TILE_BYTES;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8 fa[4], fb[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) fa[i] = read_frag<AK>(la, wr * 64 + i * 16, ks, lane);
#pragma unroll
        for (int j = 0; j < 4; ++j) fb[j] = read_frag<BKc>(lb, wc * 64 + j * 16, ks, lane);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
      }
      if (has_next) {
        char* ln = smem + (cur ^ 1) * STAGE_BYTES;
        store_tile<AMODE>(ln, tid, ra);
        store_tile<BMODE>(ln + TILE_BYTES, tid, rb);
      }
      __syncthreads();
    }
  }

  // ---------------------------------------------------------------- epilogue
  // lane holds C[m = m0 + wr*64 + 16i + (lane&15)][n = n0 + wc*64 + 16j + 4*(lane>>4) + r]
  const int lrow = lane & 15, lcol = 4 * (lane >> 4);

  if constexpr (EPI == DFU_EPI_BF16_STATS) {
    // Store bf16 and emit per-column (sum, M2) of this 128-row tile over the rounded values.
    float* red = (float*)smem;  // [2 waves-rows][128 cols][2]
    float cnt_w = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) cnt_w += (m0 + wr * 64 + 16 * i + lrow < p.M) ? 1.f : 0.f;
    // rows valid per wave: sum over the 16 lanes sharing a column
    float cnt = cnt_w;
    cnt += __shfl_xor(cnt, 1, 64);
    cnt += __shfl_xor(cnt, 2, 64);
    cnt += __shfl_xor(cnt, 4, 64);
    cnt += __shfl_xor(cnt, 8, 64);
    float sum[4][4], m2[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int m = m0 + wr * 64 + 16 * i + lrow;
          float v = bf2f(f2bf(acc[i][j][r] * p.alpha));
          acc[i][j][r] = v;
          s += (m < p.M) ? v : 0.f;
        }
        s += __shfl_xor(s, 1, 64);
        s += __shfl_xor(s, 2, 64);
        s += __shfl_xor(s, 4, 64);
        s += __shfl_xor(s, 8, 64);
        sum[j][r] = s;
        const float mean = cnt > 0.f ? s / cnt : 0.f;
        float q = 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int m = m0 + wr * 64 + 16 * i + lrow;
          const float d = acc[i][j][r] - mean;
          q += (m < p.M) ? d * d : 0.f;
        }
        q += __shfl_xor(q, 1, 64);
        q += __shfl_xor(q, 2, 64);
        q += __shfl_xor(q, 4, 64);
        q += __shfl_xor(q, 8, 64);
        m2[j][r] = q;
      }
    }
    // bf16 stores
    bf16_t* C = (bf16_t*)p.C;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + wr * 64 + 16 * i + lrow;
      if (m >= p.M) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = n0 + wc * 64 + 16 * j + lcol;
        if (n + 3 < p.N) {
          u32x2 w;
          w[0] = pack2(acc[i][j][0], acc[i][j][1]);
          w[1] = pack2(acc[i][j][2], acc[i][j][3]);
          *(u32x2*)(C + (int64_t)m * p.ldc + n) = w;
        } else {
          for (int r = 0; r < 4; ++r)
            if (n + r < p.N) C[(int64_t)m * p.ldc + n + r] = f2bf(acc[i][j][r]);
        }
      }
    }
    // combine the two row-waves with Chan's formula
    __syncthreads();
    if (lrow == 0 && wr == 1) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int c = wc * 64 + 16 * j + lcol + r;
          red[c * 3 + 0] = sum[j][r];
          red[c * 3 + 1] = m2[j][r];
          red[c * 3 + 2] = cnt;
        }
    }
    __syncthreads();
    if (lrow == 0 && wr == 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int cl = wc * 64 + 16 * j + lcol + r;
          const int n = n0 + cl;
          if (n >= p.N) continue;
          const float s1 = red[cl * 3 + 0], q1 = red[cl * 3 + 1], c1 = red[cl * 3 + 2];
          const float s0 = sum[j][r], q0 = m2[j][r], c0 = cnt;
          const float ct = c0 + c1;
          float M2 = q0 + q1;
          if (c0 > 0.f && c1 > 0.f) {
            const float d = s1 / c1 - s0 / c0;
            M2 += d * d * c0 * c1 / ct;
          }
          p.stats[((int64_t)tm * 2 + 0) * p.N + n] = s0 + s1;
          p.stats[((int64_t)tm * 2 + 1) * p.N + n] = M2;
        }
    }
    return;
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + wr * 64 + 16 * i + lrow;
      if (m >= p.M) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = n0 + wc * 64 + 16 * j + lcol;
        if (n >= p.N) continue;
        const bool full = (n + 3 < p.N);
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = acc[i][j][r] * p.alpha;
        if constexpr (EPI == DFU_EPI_BF16 || EPI == DFU_EPI_BF16_RELU || EPI == DFU_EPI_F32 ||
                      EPI == DFU_EPI_F32_RESID || EPI == DFU_EPI_BF16_GELU ||
                      EPI == DFU_EPI_PATCH) {
          if (p.bias) {
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] += (n + r < p.N) ? p.bias[n + r] : 0.f;
          }
        }
        if constexpr (EPI == DFU_EPI_BF16 || EPI == DFU_EPI_BF16_RELU) {
          if constexpr (EPI == DFU_EPI_BF16_RELU) {
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
          }
          bf16_t* C = (bf16_t*)p.C + (int64_t)m * p.ldc + n;
          if (full) {
            *(u32x2*)C = (u32x2){pack2(v[0], v[1]), pack2(v[2], v[3])};
          } else {
            for (int r = 0; r < 4; ++r)
              if (n + r < p.N) C[r] = f2bf(v[r]);
          }
        } else if constexpr (EPI == DFU_EPI_BF16_GELU) {
          bf16_t* C = (bf16_t*)p.C + (int64_t)m * p.ldc + n;
          bf16_t* Pre = (bf16_t*)p.aux_out + (int64_t)m * p.ldaux_out + n;
          float g[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) g[r] = gelu_f(bf2f(f2bf(v[r])));
          if (full) {
            *(u32x2*)Pre = (u32x2){pack2(v[0], v[1]), pack2(v[2], v[3])};
            *(u32x2*)C = (u32x2){pack2(g[0], g[1]), pack2(g[2], g[3])};
          } else {
            for (int r = 0; r < 4; ++r)
              if (n + r < p.N) { Pre[r] = f2bf(v[r]); C[r] = f2bf(g[r]); }
          }
        } else if constexpr (EPI == DFU_EPI_F32) {
          float* C = (float*)p.C + (int64_t)m * p.ldc + n;
          if (full) {
            *(f32x4*)C = (f32x4){v[0], v[1], v[2], v[3]};
          } else {
            for (int r = 0; r < 4; ++r)
              if (n + r < p.N) C[r] = v[r];
          }
        } else if constexpr (EPI == DFU_EPI_F32_RESID) {
          float* C = (float*)p.C + (int64_t)m * p.ldc + n;
          const float* R = (const float*)p.aux + (int64_t)m * p.ldaux + n;
          if (full) {
            const f32x4 rr = *(const f32x4*)R;
            *(f32x4*)C = (f32x4){v[0] + rr[0], v[1] + rr[1], v[2] + rr[2], v[3] + rr[3]};
          } else {
            for (int r = 0; r < 4; ++r)
              if (n + r < p.N) C[r] = v[r] + R[r];
          }
        } else if constexpr (EPI == DFU_EPI_BF16_DGELU || EPI == DFU_EPI_BF16_ADD) {
          bf16_t* C = (bf16_t*)p.C + (int64_t)m * p.ldc + n;
          const bf16_t* X = (const bf16_t*)p.aux + (int64_t)m * p.ldaux + n;
          float x[4];
          if (full) {
            const u32x2 xv = *(const u32x2*)X;
            x[0] = lo_bf(xv[0]); x[1] = hi_bf(xv[0]); x[2] = lo_bf(xv[1]); x[3] = hi_bf(xv[1]);
          } else {
            for (int r = 0; r < 4; ++r) x[r] = (n + r < p.N) ? bf2f(X[r]) : 0.f;
          }
#pragma unroll
          for (int r = 0; r < 4; ++r)
            v[r] = (EPI == DFU_EPI_BF16_DGELU) ? v[r] * gelu_grad_f(x[r]) : v[r] + x[r];
          if (full) {
            *(u32x2*)C = (u32x2){pack2(v[0], v[1]), pack2(v[2], v[3])};
          } else {
            for (int r = 0; r < 4; ++r)
              if (n + r < p.N) C[r] = f2bf(v[r]);
          }
        } else if constexpr (EPI == DFU_EPI_F32_ACC) {
          float* C = (float*)p.C + (int64_t)m * p.ldc + n;
          if (p.split > 1) {
            for (int r = 0; r < 4; ++r)
              if (n + r < p.N) atomicAdd(C + r, v[r]);
          } else if (full) {
            f32x4 c = *(f32x4*)C;
            *(f32x4*)C = (f32x4){c[0] + v[0], c[1] + v[1], c[2] + v[2], c[3] + v[3]};
          } else {
            for (int r = 0; r < 4; ++r)
              if (n + r < p.N) C[r] += v[r];
          }
        } else if constexpr (EPI == DFU_EPI_F32_ACC_CONVW) {
          // m = kout, n = (r, s, c) -> OIHW offset kout*C*R*S + c*R*S + r*S + s
          float* C = (float*)p.C;
          const int RS = p.cr * p.cs;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int nn = n + r;
            if (nn >= p.N) continue;
            const int rs = nn / p.cc, c = nn - rs * p.cc;
            const int64_t off = (int64_t)m * p.ldc + (int64_t)c * RS + rs;
            if (p.split > 1) atomicAdd(C + off, v[r]);
            else C[off] += v[r];
          }
        } else if constexpr (EPI == DFU_EPI_PATCH) {
          // m = b*T + t  ->  row b*(T+1) + 1 + t of the fp32 token matrix
          const int T = p.ep_tokens;
          const int b = m / T, t = m - b * T;
          float* C = (float*)p.C + ((int64_t)b * (T + 1) + 1 + t) * p.ldc + n;
          const float* P = (const float*)p.aux + (int64_t)(1 + t) * p.ldaux + n;
          if (full) {
            const f32x4 pp = *(const f32x4*)P;
            *(f32x4*)C = (f32x4){v[0] + pp[0], v[1] + pp[1], v[2] + pp[2], v[3] + pp[3]};
          } else {
            for (int r = 0; r < 4; ++r)
              if (n + r < p.N) C[r] = v[r] + P[r];
          }
        }
      }
    }
  }
}

}  // namespace dfu
