// bf16 MFMA GEMM template for gfx950 with implicit-GEMM convolution loaders and fused
// epilogues.  One kernel body serves every contraction of the DFU training step
// (SURVEY.md §2.2): ViT Linear fwd/dgrad/wgrad, NHWC conv fwd/dgrad/wgrad, patch-embed.
//
// Geometry: 512 threads = 8 waves (2 per SIMD), one workgroup per CU, output tile TM x TN
// (128x128, 256x128, 128x256 or 256x256), K-step 64, v_mfma_f32_16x16x32_bf16 with fp32
// accumulators.  Operands move global -> LDS by LDS-DMA (global_load_lds_dwordx4) into an
// NSTAGE-deep ring (3 stages when they fit in 160 KiB, else 2), tracked by counted vmcnt and
// published with a raw s_barrier — no VGPR staging, so gathered (im2col) and transposed
// operands cost no registers.  Two LDS images:
//   K-contiguous  [rows][64 k]         128-B rows, 16-B chunk ^= (row & 7)   -> ds_read_b128
//   MN-contiguous [64 k][128 cols] x n 256-B rows, 16-B chunk ^= f(k)        -> ds_read_b64_tr_b16
// both conflict-free; the swizzle is applied on the DMA SOURCE (the LDS write is lane-linear).
// The MFMA is issued with the operands swapped (B fragment as "A"), so each lane ends with 4
// consecutive output COLUMNS of one row: 8-B (bf16) / 16-B (fp32) epilogue stores.
#pragma once
#include "common.h"

namespace dfu {

constexpr int BK = 64, NT = 512, NWAVE = 8;
constexpr int LDS_MAX = 160 * 1024;

// OCC = workgroups per CU the variant is built for (launch bounds); OCC 2 forces a 2-stage
// ring so two workgroups' LDS fit (their prologues/epilogues overlap each other's main loop).
template <int TM_, int TN_, int OCC_ = 1, int NST_ = 0>
struct Tile {
  static constexpr int TM = TM_, TN = TN_, OCC = OCC_;
  static constexpr int WGM = (TM == 256 && TN == 128) ? 4 : 2;  // wave grid
  static constexpr int WGN = NWAVE / WGM;
  static constexpr int WTM = TM / WGM, WTN = TN / WGN;         // per-wave sub-tile
  static constexpr int FM = WTM / 16, FN = WTN / 16;           // MFMA accumulators per wave
  static constexpr int NLDA = TM / 64, NLDB = TN / 64;         // DMA instructions per thread
  static constexpr int A_BYTES = TM * BK * 2, B_BYTES = TN * BK * 2;
  static constexpr int STAGE_BYTES = A_BYTES + B_BYTES;
  // ring depth: NST_ if given, else 3 when it fits one workgroup per CU, else 2
  static constexpr int NSTAGE =
      NST_ ? NST_ : ((OCC == 1 && 3 * STAGE_BYTES <= LDS_MAX) ? 3 : 2);
  static constexpr int LDS_BYTES = NSTAGE * STAGE_BYTES;
  static constexpr int DMA_PER_STAGE = NLDA + NLDB;
  static_assert(OCC * LDS_BYTES <= LDS_MAX, "LDS for the requested occupancy");
};

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
  float* slab;  // split-K partial slabs [split][M][N] (F32_ACC with a workspace)
  int split;
  int ep_tokens;
  // conv geometry
  int cn, ch, cw, cc, ck, cr, cs, cstride, cpad, cp, cq;
  int cpad_w;  // padding along W (== cpad except for stride-phase dgrad launches)
  // Stride-phase dgrad (ph_st > 0): this launch computes the dX rows h = h'*st + ph_h,
  // w = w'*st + ph_w with only the live taps r = ph_r0 + st*ri, s = ph_s0 + st*si.  The
  // geometry above is then the phase's stride-1 equivalent (ch, cw = phase grid; cr, cs = live
  // tap counts; cpad, cpad_w = tap origins); ph_H/ph_W/ph_S are the real dX dims / filter width.
  int ph_st, ph_h, ph_w, ph_r0, ph_s0, ph_H, ph_W, ph_S;
  FastDiv div_pq, div_q, div_hw, div_w, div_c, div_k, div_s;
  int m_ld_bound;  // MN-contiguous operands may be read up to this column bound
  int n_ld_bound;
};

// ------------------------------------------------------------------------------ LDS maps
DFU_DEV int kc_off(int row, int chunk) { return row * 128 + ((chunk ^ (row & 7)) << 4); }
DFU_DEV int mn_swz(int k) { return ((k & 3) << 1) | (((k >> 3) & 1) << 3); }
DFU_DEV int mn_off(int krow, int chunk) { return krow * 256 + ((chunk ^ mn_swz(krow)) << 4); }

template <int MODE>
constexpr bool kcontig() {
  return MODE == DFU_OPND_KMAJOR || MODE == DFU_OPND_CONV_FWD || MODE == DFU_OPND_CONV_DGRAD;
}

// ------------------------------------------------------------------------------ loaders
// One DMA wave-instruction writes 1 KiB of LDS at a wave-uniform base, lane l at base+16*l.
// Instruction i of wave w lands at byte 1024*(w + 8*i) of the operand tile.
//   K-contiguous tile: that is rows 8*(w+8i) .. +7, i.e. thread row (tid>>3) + 64*i, and the
//     lane at LDS slot (lane&7) of its row fetches chunk (lane&7) ^ (row&7) = kc_lane_chunk.
//   MN-contiguous tile (128-column sub-images of 16 KiB): 1-KiB piece q = w + 8*i is k-rows
//     4*(q&15) .. +3 of sub-image q>>4, i.e. k-row (tid>>4) + 32*(i&1), columns
//     128*(i>>1) + 8*chunk with chunk = (lane&15) ^ f(k-row) (same f for every i).
// Out-of-range lanes fetch 16 zero bytes from g_zero16.
__device__ __attribute__((aligned(16))) const uint32_t g_zero16[4] = {0u, 0u, 0u, 0u};

DFU_DEV int kc_lane_chunk(int lane) { return (lane & 7) ^ ((lane >> 3) & 7); }
DFU_DEV int mn_lane_chunk(int tid) { return (tid & 15) ^ mn_swz(tid >> 4); }

template <int NLD>
struct LoadState {
  const bf16_t* ptr[NLD];  // KMAJOR: row pointer incl. the swizzled chunk offset
  int i0[NLD], i1[NLD];    // conv: ih0/iw0 (fwd) or h+pad/w+pad (dgrad); wgrad: r, s per sub
  int valid[NLD];
  int bofs[NLD];           // conv: batch index
  int cin[NLD];            // wgrad: channel per sub-image
  int kc;                  // K-contiguous: element offset of this lane's (swizzled) chunk
  int col;                 // MN-contiguous: first column (sub-image 0) of this lane's chunk
};

template <int MODE, int NLD>
DFU_DEV void load_init(const GemmArgs& p, LoadState<NLD>& st, const bf16_t* base, int64_t ld,
                       int mn0, int MN, int tid) {
  const int lane = tid & 63;
  if constexpr (kcontig<MODE>()) {
    st.kc = kc_lane_chunk(lane) * 8;
  } else {
    st.col = mn0 + mn_lane_chunk(tid) * 8;
  }
  if constexpr (MODE == DFU_OPND_KMAJOR) {
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      const int row = mn0 + (tid >> 3) + 64 * i;
      st.valid[i] = row < MN;
      st.ptr[i] = base + (int64_t)(st.valid[i] ? row : 0) * ld + st.kc;
    }
  } else if constexpr (MODE == DFU_OPND_CONV_FWD) {
#pragma unroll
    for (int i = 0; i < NLD; ++i) {  // rows = output positions (b, oh, ow)
      const int m = mn0 + (tid >> 3) + 64 * i;
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
#pragma unroll
    for (int i = 0; i < NLD; ++i) {  // rows = input positions (b, h, w) of dX
      const int m = mn0 + (tid >> 3) + 64 * i;
      st.valid[i] = m < MN;
      const uint32_t mm = st.valid[i] ? m : 0;
      const uint32_t b = fdiv(mm, p.div_hw);
      const uint32_t rem = mm - b * (uint32_t)(p.ch * p.cw);
      const uint32_t h = fdiv(rem, p.div_w);
      const uint32_t w = rem - h * p.cw;
      st.i0[i] = (int)h + p.cpad;
      st.i1[i] = (int)w + p.cpad_w;
      st.bofs[i] = (int)b;
    }
  } else if constexpr (MODE == DFU_OPND_CONV_WGRAD_X) {
    constexpr int NSUB = NLD >= 2 ? NLD / 2 : 1;
#pragma unroll
    for (int sub = 0; sub < NSUB; ++sub) {  // n' = (r, s, c) per sub-image
      const uint32_t n = st.col + 128 * sub;
      const uint32_t rs = fdiv(n, p.div_c);
      st.cin[sub] = (int)(n - rs * p.cc);
      const uint32_t r = fdiv(rs, p.div_s);
      st.i0[sub] = (int)r;
      st.i1[sub] = (int)(rs - r * p.cs);
    }
  }
}

typedef __attribute__((address_space(3))) void lds_void;
typedef const __attribute__((address_space(1))) void glb_void;

DFU_DEV void glds16(const void* src, char* lds_dst) {
  __builtin_amdgcn_global_load_lds((glb_void*)src, (lds_void*)lds_dst, 16, 0, 0);
}

// Issue this thread's NLD LDS-DMA instructions for K-step kt into `tile`.
template <int MODE, int NLD>
DFU_DEV void issue_tile(const GemmArgs& p, const LoadState<NLD>& st, const bf16_t* base,
                        int64_t ld, int MN_bound, int kt, int kend, int tid, char* tile) {
  const int k0 = kt * BK;
  char* dst = tile + 1024 * (tid >> 6);
  const void* zero = (const void*)g_zero16;
  if constexpr (MODE == DFU_OPND_KMAJOR) {
    const bool kin = k0 + st.kc < kend;
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      const bool ok = st.valid[i] && kin;
      glds16(ok ? (const void*)(st.ptr[i] + k0) : zero, dst + 8192 * i);
    }
  } else if constexpr (MODE == DFU_OPND_CONV_FWD) {
    // whole K-step lies in one filter tap (C % 64 == 0, host-checked)
    const uint32_t rs = fdiv((uint32_t)k0, p.div_c);
    const int c0 = k0 - (int)rs * p.cc + st.kc;
    const uint32_t r = fdiv(rs, p.div_s);
    const int sx = (int)(rs - r * p.cs);
    const bool kin = k0 < kend;
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      const int ih = st.i0[i] + (int)r, iw = st.i1[i] + sx;
      const bool ok = kin && st.valid[i] && (unsigned)ih < (unsigned)p.ch && (unsigned)iw < (unsigned)p.cw;
      const int64_t off = (((int64_t)st.bofs[i] * p.ch + ih) * p.cw + iw) * p.cc + c0;
      glds16(ok ? (const void*)(base + off) : zero, dst + 8192 * i);
    }
  } else if constexpr (MODE == DFU_OPND_CONV_DGRAD) {
    // K' = (r, s, kout); gather dY[b][(h+pad-r)/st][(w+pad-s)/st][kout]
    const uint32_t rs = fdiv((uint32_t)k0, p.div_k);
    const int k_0 = k0 - (int)rs * p.ck + st.kc;
    const uint32_t r = fdiv(rs, p.div_s);
    const int sx = (int)(rs - r * p.cs);
    const bool kin = k0 < kend;
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
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
      glds16(ok ? (const void*)(base + off) : zero, dst + 8192 * i);
    }
  } else if constexpr (MODE == DFU_OPND_MNMAJOR) {
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      const int k = k0 + (tid >> 4) + 32 * (i & 1);
      const int col = st.col + 128 * (i >> 1);
      const bool ok = col < MN_bound && k < kend;
      glds16(ok ? (const void*)(base + (int64_t)k * ld + col) : zero, dst + 8192 * i);
    }
  } else if constexpr (MODE == DFU_OPND_CONV_DGRAD_W) {
    // B[k'=(r,s,kout)][c] = Wkrsc[kout][r][s][c];  ld = R*S*C
    const uint32_t rs = fdiv((uint32_t)k0, p.div_k);
    const int kout0 = k0 - (int)rs * p.ck;
    int64_t tap_off = (int64_t)rs * p.cc;
    if (p.ph_st) {  // phase launch: live tap (ri, si) -> filter tap (r0 + st ri, s0 + st si)
      const uint32_t ri = fdiv(rs, p.div_s);
      const int si = (int)(rs - ri * p.cs);
      tap_off = ((int64_t)(p.ph_r0 + p.ph_st * (int)ri) * p.ph_S + p.ph_s0 + p.ph_st * si) * p.cc;
    }
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      const int kout = kout0 + (tid >> 4) + 32 * (i & 1);
      const int col = st.col + 128 * (i >> 1);
      const bool ok = col < MN_bound && k0 < kend;
      glds16(ok ? (const void*)(base + (int64_t)kout * ld + tap_off + col) : zero,
             dst + 8192 * i);
    }
  } else if constexpr (MODE == DFU_OPND_CONV_WGRAD_X) {
    // B[k'=m (b,oh,ow)][n'=(r,s,c)] = X[b][oh*st-pad+r][ow*st-pad+s][c]
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      const int sub = i >> 1;
      const int m = k0 + (tid >> 4) + 32 * (i & 1);
      bool ok = (st.col + 128 * sub) < MN_bound && m < kend;
      const uint32_t mm = ok ? m : 0;
      const uint32_t b = fdiv(mm, p.div_pq);
      const uint32_t rem = mm - b * (uint32_t)(p.cp * p.cq);
      const uint32_t oh = fdiv(rem, p.div_q);
      const uint32_t ow = rem - oh * p.cq;
      const int ih = (int)oh * p.cstride - p.cpad + st.i0[sub];
      const int iw = (int)ow * p.cstride - p.cpad + st.i1[sub];
      ok = ok && (unsigned)ih < (unsigned)p.ch && (unsigned)iw < (unsigned)p.cw;
      const int64_t off = (((int64_t)b * p.ch + ih) * p.cw + iw) * p.cc + st.cin[sub];
      glds16(ok ? (const void*)(base + off) : zero, dst + 8192 * i);
    }
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
    const char* img = lds + 16384 * (rb >> 7);
    const int g = lane >> 4, i = lane & 15, q = i >> 2, pp = i & 3;
    const int krow = ks * 32 + 8 * g + q;
    const int col = (rb & 127) + 4 * pp;
    const int chunk = col >> 3, half = (col >> 2) & 1;
    const char* a0 = img + mn_off(krow, chunk) + half * 8;
    const char* a1 = img + mn_off(krow + 4, chunk) + half * 8;
    bf16x4 x0 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(a0));
    bf16x4 x1 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(a1));
    return __builtin_shufflevector(x0, x1, 0, 1, 2, 3, 4, 5, 6, 7);
  }
}

template <int N>
DFU_DEV void wait_vmcnt() {
  static_assert(N >= 0 && N <= 63, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Wait until at most k stages (DPS DMA instructions each) issued after the current one are
// still in flight; k is runtime (the ring drains at the end), vmcnt needs an immediate.
template <int DPS, int KMAX>
DFU_DEV void wait_stages(int k) {
  if constexpr (KMAX > 0) {
    if (k >= KMAX) {
      wait_vmcnt<DPS * KMAX>();
      return;
    }
    wait_stages<DPS, KMAX - 1>(k);
  } else {
    wait_vmcnt<0>();
  }
}

// Output row of GEMM row m: identity, or for a stride-phase dgrad launch the dX row
// (b, h'*st + ph_h, w'*st + ph_w) of phase-grid row m = (b, h', w').
DFU_DEV int64_t out_row(const GemmArgs& p, int m) {
  if (!p.ph_st) return m;
  const uint32_t b = fdiv((uint32_t)m, p.div_hw);
  const uint32_t rem = (uint32_t)m - b * (uint32_t)(p.ch * p.cw);
  const uint32_t h = fdiv(rem, p.div_w);
  const uint32_t w = rem - h * (uint32_t)p.cw;
  return ((int64_t)b * p.ph_H + (int)h * p.ph_st + p.ph_h) * p.ph_W + (int)w * p.ph_st + p.ph_w;
}

// ------------------------------------------------------------------------------ kernel
template <int AMODE, int BMODE, int EPI, int TM, int TN, int OCC = 1, int NST = 0>
__global__ __launch_bounds__(NT, OCC) void gemm_kernel(const GemmArgs p) {
  using T = Tile<TM, TN, OCC, NST>;
  constexpr int WGM = T::WGM, WGN = T::WGN, WTM = T::WTM, WTN = T::WTN;
  constexpr int FM = T::FM, FN = T::FN, NSTAGE = T::NSTAGE;
  __shared__ __attribute__((aligned(16))) char smem[T::LDS_BYTES];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wr = wave / WGN, wc = wave % WGN;

  // XCD-aware bijective remap (blocks b and b+8 share an XCD): each XCD gets a contiguous
  // range of tile ids; then a grouped raster (GROUP_M x tiles_n bands walked column by
  // column) keeps the tiles live on one XCD sharing A and B panels in its L2.
  const int nwg = gridDim.x;
  const int bid = blockIdx.x;
  int wgid = bid;
  if (nwg >= 16) {
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  constexpr int GROUP_M = 4;
  const int band = GROUP_M * p.tiles_n;
  const int g0 = (wgid / band) * GROUP_M;
  const int gm = min(GROUP_M, p.tiles_m - g0);
  const int within = wgid - (wgid / band) * band;
  const int tm = g0 + within % gm;
  const int tn = within / gm;
  const int m0 = tm * TM, n0 = tn * TN;

  const int kt_begin = blockIdx.y * p.kt_per_split;
  const int kt_end = min(p.ktiles, kt_begin + p.kt_per_split);
  const int kend = p.K;

  LoadState<T::NLDA> sa;
  LoadState<T::NLDB> sb;
  load_init<AMODE, T::NLDA>(p, sa, p.A, p.lda, m0, p.M, tid);
  load_init<BMODE, T::NLDB>(p, sb, p.B, p.ldb, n0, p.N, tid);

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  constexpr bool AK = kcontig<AMODE>();
  constexpr bool BKc = kcontig<BMODE>();

  auto issue = [&](int kt, char* stage) {
    issue_tile<AMODE, T::NLDA>(p, sa, p.A, p.lda, p.m_ld_bound, kt, kend, tid, stage);
    issue_tile<BMODE, T::NLDB>(p, sb, p.B, p.ldb, p.n_ld_bound, kt, kend, tid,
                               stage + T::A_BYTES);
  };
  // All fragment reads of the K-step (both 32-wide halves) are issued before the first MFMA,
  // so the LDS latency overlaps MFMAs (counted lgkmcnt waits) instead of draining per group.
  auto compute = [&](const char* la) {
    const char* lb = la + T::A_BYTES;
    bf16x8 fa[2][FM], fb[2][FN];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
      for (int i = 0; i < FM; ++i) fa[ks][i] = read_frag<AK>(la, wr * WTM + i * 16, ks, lane);
#pragma unroll
      for (int j = 0; j < FN; ++j) fb[ks][j] = read_frag<BKc>(lb, wc * WTN + j * 16, ks, lane);
    }
    __builtin_amdgcn_sched_barrier(0);  // keep the reads ahead (the scheduler sinks them)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[ks][j], fa[ks][i], acc[i][j], 0, 0, 0);
  };
  // Pipeline: K-step i+NSTAGE-1 is issued (into the slot K-step i-1 vacated) right after the
  // barrier that publishes K-step i; completion is tracked with counted vmcnt (the DMA is
  // invisible to the compiler's waits).
  const int nk = kt_end - kt_begin;
#pragma unroll
  for (int s = 0; s < NSTAGE - 1; ++s)
    if (s < nk) issue(kt_begin + s, smem + s * T::STAGE_BYTES);
  for (int i = 0; i < nk; ++i) {
    // stage i must have landed; the min(nk-i-1, NSTAGE-2) stages issued after it may fly on
    wait_stages<T::DMA_PER_STAGE, NSTAGE - 2>(nk - i - 1);
    __builtin_amdgcn_s_barrier();
    if (i + NSTAGE - 1 < nk)
      issue(kt_begin + i + NSTAGE - 1, smem + ((i + NSTAGE - 1) % NSTAGE) * T::STAGE_BYTES);
    compute(smem + (i % NSTAGE) * T::STAGE_BYTES);
  }
  __syncthreads();

  // ---------------------------------------------------------------- epilogue
  // lane holds C[m = m0 + wr*WTM + 16i + (lane&15)][n = n0 + wc*WTN + 16j + 4*(lane>>4) + r]
  const int lrow = lane & 15, lcol = 4 * (lane >> 4);

  if constexpr (EPI == DFU_EPI_BF16_STATS) {
    // bf16 store + per-column (sum, M2) of this TM-row tile over the rounded values:
    // per wave two-pass in registers, then Chan's merge across the WGM row-waves in LDS.
    static_assert(WGM * TN * 3 * 4 <= T::LDS_BYTES, "stats scratch");
    float* red = (float*)smem;  // [WGM][TN][3]
    float cnt = 0.f;
#pragma unroll
    for (int i = 0; i < FM; ++i) cnt += (m0 + wr * WTM + 16 * i + lrow < p.M) ? 1.f : 0.f;
    cnt += __shfl_xor(cnt, 1, 64);
    cnt += __shfl_xor(cnt, 2, 64);
    cnt += __shfl_xor(cnt, 4, 64);
    cnt += __shfl_xor(cnt, 8, 64);
    bf16_t* C = (bf16_t*)p.C;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const int m = m0 + wr * WTM + 16 * i + lrow;
          const float v = bf2f(f2bf(acc[i][j][r] * p.alpha));
          acc[i][j][r] = v;
          s += (m < p.M) ? v : 0.f;
        }
        s += __shfl_xor(s, 1, 64);
        s += __shfl_xor(s, 2, 64);
        s += __shfl_xor(s, 4, 64);
        s += __shfl_xor(s, 8, 64);
        const float mean = cnt > 0.f ? s / cnt : 0.f;
        float q = 0.f;
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const int m = m0 + wr * WTM + 16 * i + lrow;
          const float d = acc[i][j][r] - mean;
          q += (m < p.M) ? d * d : 0.f;
        }
        q += __shfl_xor(q, 1, 64);
        q += __shfl_xor(q, 2, 64);
        q += __shfl_xor(q, 4, 64);
        q += __shfl_xor(q, 8, 64);
        if (lrow == 0) {
          const int c = wc * WTN + 16 * j + lcol + r;
          red[(wr * TN + c) * 3 + 0] = s;
          red[(wr * TN + c) * 3 + 1] = q;
          red[(wr * TN + c) * 3 + 2] = cnt;
        }
      }
    }
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int m = m0 + wr * WTM + 16 * i + lrow;
      if (m >= p.M) continue;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int n = n0 + wc * WTN + 16 * j + lcol;
        if (n + 3 < p.N) {
          *(u32x2*)(C + (int64_t)m * p.ldc + n) =
              (u32x2){pack2(acc[i][j][0], acc[i][j][1]), pack2(acc[i][j][2], acc[i][j][3])};
        } else {
          for (int r = 0; r < 4; ++r)
            if (n + r < p.N) C[(int64_t)m * p.ldc + n + r] = f2bf(acc[i][j][r]);
        }
      }
    }
    __syncthreads();
    // one (sum, M2) record per 128-row block: merge the row-waves that cover each block
    constexpr int HALVES = TM / 128;
    for (int idx = tid; idx < TN * HALVES; idx += NT) {
      const int c = idx % TN, h = idx / TN;
      const int n = n0 + c;
      if (n >= p.N || m0 + 128 * h >= p.M) continue;
      float S = 0.f, Q = 0.f, Cn = 0.f;
      for (int w = 0; w < WGM; ++w) {
        if ((w * WTM) / 128 != h) continue;
        const float s1 = red[(w * TN + c) * 3 + 0], q1 = red[(w * TN + c) * 3 + 1];
        const float c1 = red[(w * TN + c) * 3 + 2];
        if (c1 <= 0.f) continue;
        if (Cn > 0.f) {
          const float d = s1 / c1 - S / Cn;
          Q += q1 + d * d * Cn * c1 / (Cn + c1);
        } else {
          Q = q1;
        }
        S += s1;
        Cn += c1;
      }
      const int64_t blk = m0 / 128 + h;
      p.stats[(blk * 2 + 0) * p.N + n] = S;
      p.stats[(blk * 2 + 1) * p.N + n] = Q;
    }
    return;
  } else {
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int m = m0 + wr * WTM + 16 * i + lrow;
      if (m >= p.M) continue;
      const int64_t mo = AMODE == DFU_OPND_CONV_DGRAD ? out_row(p, m) : (int64_t)m;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int n = n0 + wc * WTN + 16 * j + lcol;
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
          bf16_t* C = (bf16_t*)p.C + mo * p.ldc + n;
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
          for (int r = 0; r < 4; ++r) g[r] = gelu_f(v[r]);
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
          bf16_t* C = (bf16_t*)p.C + mo * p.ldc + n;
          const bf16_t* X = (const bf16_t*)p.aux + mo * p.ldaux + n;
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
          if (p.slab != nullptr) {
            // split-K partial: plain coalesced store into this split's slab
            float* S = p.slab + ((int64_t)blockIdx.y * p.M + m) * p.N + n;
            if (full) {
              *(f32x4*)S = (f32x4){v[0], v[1], v[2], v[3]};
            } else {
              for (int r = 0; r < 4; ++r)
                if (n + r < p.N) S[r] = v[r];
            }
          } else {
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
          }
        } else if constexpr (EPI == DFU_EPI_PATCH) {
          // m = b*T + t  ->  row b*(T+1) + 1 + t of the fp32 token matrix
          const int Tt = p.ep_tokens;
          const int b = m / Tt, t = m - b * Tt;
          float* C = (float*)p.C + ((int64_t)b * (Tt + 1) + 1 + t) * p.ldc + n;
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
