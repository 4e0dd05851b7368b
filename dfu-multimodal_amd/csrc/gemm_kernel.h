// bf16 MFMA GEMM template for gfx950 with implicit-GEMM convolution loaders and fused
// epilogues.  One kernel body serves every contraction of the DFU training step
// (SURVEY.md §2.2): ViT Linear fwd/dgrad/wgrad, NHWC conv fwd/dgrad/wgrad, patch-embed.
//
// Geometry: 512 threads = 8 waves (2 per SIMD) or 256 threads = 4 waves, output tile TM x TN
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
//
// Persistent schedule: the grid is at most one wave of workgroups (CUs x occupancy); each
// workgroup walks the work units u = wg, wg + G, ... (unit = output tile x K-split) as ONE
// continuous K-step stream, so the ring never drains at a tile boundary: the next tile's first
// stages are in flight while the current tile's epilogue runs, and the epilogue's stores drain
// under the next tile's MFMAs.  Epilogue stores are buffer stores masked by an out-of-range
// offset (never by a branch), so every wave issues a fixed count of them and the counted vmcnt
// waits of the K-loop stay exact across tile boundaries (vmcnt retires loads, stores and
// LDS-DMA of a wave in issue order; MI355X_MICROARCH.md).
#pragma once
#include "common.h"

namespace dfu {

constexpr int BK = 64;
constexpr int LDS_MAX = 160 * 1024;

// OCC = workgroups per CU the variant is built for (launch bounds); OCC 2 forces a 2-stage
// ring so two workgroups' LDS fit (their prologues/epilogues overlap each other's main loop).
// NW = waves per workgroup: 8 (2x4 or 4x2 wave grid) or 4 (2x2: 64x64 per wave on a 128x128
// tile, a third less LDS read traffic per MFMA than 64x32).
template <int TM_, int TN_, int OCC_ = 1, int NST_ = 0, int NW_ = 8>
struct Tile {
  static constexpr int TM = TM_, TN = TN_, OCC = OCC_, NW = NW_, NT = 64 * NW_;
  static constexpr int WGM = NW == 4 ? 2 : (TM == 256 && TN == 128) ? 4 : 2;  // wave grid
  static constexpr int WGN = NW / WGM;
  static constexpr int WTM = TM / WGM, WTN = TN / WGN;         // per-wave sub-tile
  static constexpr int FM = WTM / 16, FN = WTN / 16;           // MFMA accumulators per wave
  static constexpr int NLDA = TM / (8 * NW), NLDB = TN / (8 * NW);  // DMA instrs per thread
  static constexpr int A_BYTES = TM * BK * 2, B_BYTES = TN * BK * 2;
  static constexpr int STAGE_BYTES = A_BYTES + B_BYTES;
  // BF16_STATS epilogue scratch (per-wave column partials), after the ring in the same array
  static constexpr int STATS_BYTES = WGM * TN * 3 * 4;
  // ring depth: NST_ if given, else 3 when it fits one workgroup per CU, else 2
  static constexpr int NSTAGE =
      NST_ ? NST_ : ((OCC == 1 && 3 * STAGE_BYTES + STATS_BYTES <= LDS_MAX) ? 3 : 2);
  static constexpr int LDS_BYTES = NSTAGE * STAGE_BYTES;
  static constexpr int DMA_PER_STAGE = NLDA + NLDB;
  static_assert(OCC * (LDS_BYTES + STATS_BYTES) <= LDS_MAX, "LDS for the requested occupancy");
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
  int* counters;  // per-tile arrival counters: in-kernel slab reduction (zero in, zero out)
  int split;    // K-splits; work units = tiles_m * tiles_n * split
  // Tail split (tail_r > 0, split == 1): units [0, tail_full) are whole tiles; the tail_r tiles
  // left over after the last complete round of workgroups are each split over tail_s
  // workgroups along K (tail_kps K-steps each) instead of leaving most CUs idle for a whole
  // round.  Each split stores its fp32 accumulators to tslab; the last to arrive on the tile's
  // counter sums the slabs in split order and runs the normal epilogue.
  int tail_full, tail_r, tail_s, tail_kps;
  float* tslab;  // [tail_s][tail_r][FM*FN][threads] f32x4, lane-linear
  // Split-pair A (dfu_gemm_desc.a_seg > 0, the bf16x3 ResNet forward): the tripled K is read
  // as segments [hi | lo | hi] of width a_seg from two buffers of row (pixel) stride a_seg,
  // hi at A and lo at A + a_lo_delta (elements); a_pix = the conv gather's pixel stride.
  // Interleaved pairs (the kernel's X3 instantiations, dfu_gemm_desc.x3_pairs): K = 2 a_seg,
  // each K-step of 64 is [hi | lo] of 32 real k, and the kernel forms the three products.
  int a_seg, a_pix;
  int64_t a_lo_delta;
  int n4;       // N and every leading dimension % 4 == 0: one vector access per 4 columns
  int n8;       // N, ldc (, ldaux_out) % 8 == 0 and 16-B aligned bf16 outputs: paired stores
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
  int dbg;  // timing experiments only (DFU_GEMM_DEBUG): 1 no epilogue, 2 no MFMA, 4 no DMA
  int a_bytes, b_bytes;  // operand extents in bytes (buffer-resource DMA of gemm_ps.hip)
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
// Instruction i of wave w (of NW) lands at byte 1024*(w + NW*i) of the operand tile.
//   K-contiguous tile: that is rows 8*(w+NW*i) .. +7, i.e. thread row (tid>>3) + 8*NW*i, and
//     the lane at LDS slot (lane&7) of its row fetches chunk (lane&7) ^ (row&7).
//   MN-contiguous tile (128-column sub-images of 16 KiB = 16 pieces, PPS = 16/NW pieces per
//     wave): piece q = w + NW*(i%PPS) of sub-image i/PPS is k-rows 4q .. 4q+3, i.e. k-row
//     (tid>>4) + 4*NW*(i%PPS), columns 128*(i/PPS) + 8*chunk with chunk = (lane&15) ^ f(k-row)
//     (the same f for every i: f reads k-row bits 0, 1 and 3 only).
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

template <int MODE, int NLD, int NW>
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
      const int row = mn0 + (tid >> 3) + 8 * NW * i;
      st.valid[i] = row < MN;
      st.ptr[i] = base + (int64_t)(st.valid[i] ? row : 0) * ld + st.kc;
    }
  } else if constexpr (MODE == DFU_OPND_CONV_FWD) {
#pragma unroll
    for (int i = 0; i < NLD; ++i) {  // rows = output positions (b, oh, ow)
      const int m = mn0 + (tid >> 3) + 8 * NW * i;
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
      const int m = mn0 + (tid >> 3) + 8 * NW * i;
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
    constexpr int PPS = 16 / NW;
    constexpr int NSUB = NLD >= PPS ? NLD / PPS : 1;
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

// Issue this thread's NLD LDS-DMA instructions for K-step kt into `tile` (IS_A: the A operand,
// which may be in split-pair form, GemmArgs::a_seg).
template <int MODE, int NLD, int NW, bool IS_A = false, bool X3 = false>
DFU_DEV void issue_tile(const GemmArgs& p, const LoadState<NLD>& st, const bf16_t* base,
                        int64_t ld, int MN_bound, int kt, int kend, int tid, char* tile) {
  constexpr bool is_a = IS_A;
  constexpr int PPS = 16 / NW;  // MN-contiguous pieces per wave and 128-column sub-image
  constexpr int STEP = 1024 * NW;
  const int k0 = kt * BK;
  char* dst = tile + 1024 * (tid >> 6);
  const void* zero = (const void*)g_zero16;
  if constexpr (MODE == DFU_OPND_KMAJOR) {
    const bool kin = k0 + st.kc < kend;
    // split-pair A: segment 1 of the tripled K from the lo buffer, segment 2 from hi again, by
    // this lane's 16-B chunk (a_seg % 8 == 0, host-checked: no chunk straddles two segments)
    int64_t adj = 0;
    if (is_a && p.a_seg) {
      const int k = k0 + st.kc;
      if constexpr (X3) {  // k = 64q + 32 seg + r -> real column 32q + r of hi (seg 0) or lo
        const int seg = (k >> 5) & 1;
        adj = (seg ? p.a_lo_delta : 0) - 32 * ((k >> 6) + seg);
      } else {
        adj = k >= 2 * p.a_seg ? -2 * (int64_t)p.a_seg
                               : (k >= p.a_seg ? p.a_lo_delta - p.a_seg : 0);
      }
    }
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      const bool ok = st.valid[i] && kin;
      glds16(ok ? (const void*)(st.ptr[i] + k0 + adj) : zero, dst + STEP * i);
    }
  } else if constexpr (MODE == DFU_OPND_CONV_FWD) {
    // whole K-step lies in one filter tap (C % 64 == 0, host-checked)
    const uint32_t rs = fdiv((uint32_t)k0, p.div_c);
    int c0 = k0 - (int)rs * p.cc;
    int64_t adj = 0;
    if constexpr (X3) {  // interleaved pairs: this lane's chunk is hi (kc < 32) or lo of the
      c0 = (c0 >> 1) + (st.kc & 31);  // 32 real channels from c0 / 2
      adj = (st.kc & 32) ? p.a_lo_delta : 0;
    } else {
      if (p.a_seg) {  // split-pair input: channel segment 1 from the lo buffer, 2 from hi again
        const int seg = c0 >= 2 * p.a_seg ? 2 : (c0 >= p.a_seg ? 1 : 0);
        c0 -= seg * p.a_seg;
        adj = seg == 1 ? p.a_lo_delta : 0;
      }
      c0 += st.kc;
    }
    const uint32_t r = fdiv(rs, p.div_s);
    const int sx = (int)(rs - r * p.cs);
    const bool kin = k0 < kend;
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      const int ih = st.i0[i] + (int)r, iw = st.i1[i] + sx;
      const bool ok = kin && st.valid[i] && (unsigned)ih < (unsigned)p.ch && (unsigned)iw < (unsigned)p.cw;
      const int64_t off = (((int64_t)st.bofs[i] * p.ch + ih) * p.cw + iw) * p.a_pix + c0 + adj;
      glds16(ok ? (const void*)(base + off) : zero, dst + STEP * i);
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
      glds16(ok ? (const void*)(base + off) : zero, dst + STEP * i);
    }
  } else if constexpr (MODE == DFU_OPND_MNMAJOR) {
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      const int k = k0 + (tid >> 4) + 4 * NW * (i % PPS);
      const int col = st.col + 128 * (i / PPS);
      const bool ok = col < MN_bound && k < kend;
      glds16(ok ? (const void*)(base + (int64_t)k * ld + col) : zero, dst + STEP * i);
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
      const int kout = kout0 + (tid >> 4) + 4 * NW * (i % PPS);
      const int col = st.col + 128 * (i / PPS);
      const bool ok = col < MN_bound && k0 < kend;
      glds16(ok ? (const void*)(base + (int64_t)kout * ld + tap_off + col) : zero,
             dst + STEP * i);
    }
  } else if constexpr (MODE == DFU_OPND_CONV_WGRAD_X) {
    // B[k'=m (b,oh,ow)][n'=(r,s,c)] = X[b][oh*st-pad+r][ow*st-pad+s][c]
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      const int sub = i / PPS;
      const int m = k0 + (tid >> 4) + 4 * NW * (i % PPS);
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
      glds16(ok ? (const void*)(base + off) : zero, dst + STEP * i);
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
    // asm reads (common.h lds_tr16_b64): the caller retires them before the first use
    bf16x4 x0 = lds_tr16_b64(a0);
    bf16x4 x1 = lds_tr16_b64(a1);
    return __builtin_shufflevector(x0, x1, 0, 1, 2, 3, 4, 5, 6, 7);
  }
}

template <int N>
DFU_DEV void wait_vmcnt() {
  static_assert(N >= 0 && N <= 63, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Wait until at most n of this wave's youngest vector-memory operations are outstanding.  n is
// wave-uniform but known only at run time, and vmcnt takes an immediate: wait for the largest
// rung <= n of a ladder of immediates (a smaller count only waits longer).
constexpr int vm_rung_below(int v) {
  return v > 48 ? 48 : v > 40 ? 40 : v > 32 ? 32 : v > 24 ? 24 : v > 20 ? 20 : v > 16 ? 16
         : v > 12 ? 12 : v - 1;
}
template <int V>
DFU_DEV void wait_vm_le(int n) {
  if constexpr (V <= 0) {
    wait_vmcnt<0>();
  } else {
    if (n >= V) {
      wait_vmcnt<V>();
      return;
    }
    wait_vm_le<vm_rung_below(V)>(n);
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

// ------------------------------------------------------------------------------ epilogue I/O
// Buffer descriptors with a 2 GiB range over each output / operand base: an element is masked
// by the out-of-range offset kOOB (the store is dropped, the load reads 0), never by a branch.
constexpr int kRsrcBytes = 0x7fffff00;
constexpr uint32_t kOOB = 0x7fffff80u;
typedef __amdgpu_buffer_rsrc_t rsrc_t;

DFU_DEV rsrc_t make_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, kRsrcBytes,
                                           0x00020000);
}
DFU_DEV int boff(bool ok, int64_t byte_off) { return (int)(ok ? (uint32_t)byte_off : kOOB); }

// Four consecutive columns n..n+3 at element index e of a row-major fp32 / bf16 matrix; okr =
// row in range.  n4 (launch-uniform): one vector access, else four scalar accesses.
// AUX = cache-policy bits of the buffer instruction (16 = sc1: write-through stores / loads
// that bypass non-coherent caches, for data handed between workgroups; HIP guide G16 R1).
template <int AUX = 0>
DFU_DEV void st4_f32(rsrc_t r, int64_t e, bool okr, int n, int N, bool n4, const float* v) {
  if (n4) {
    const u32x4 x = {__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]),
                     __float_as_uint(v[3])};
    __builtin_amdgcn_raw_buffer_store_b128(x, r, boff(okr && n < N, e * 4), 0, AUX);
  } else {
#pragma unroll
    for (int q = 0; q < 4; ++q)
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v[q]), r,
                                            boff(okr && n + q < N, (e + q) * 4), 0, AUX);
  }
}
template <bool H16 = false>
DFU_DEV void st4_bf16(rsrc_t r, int64_t e, bool okr, int n, int N, bool n4, const float* v) {
  if (n4) {
    const u32x2 x = H16 ? (u32x2){pack2h(v[0], v[1]), pack2h(v[2], v[3])}
                        : (u32x2){pack2(v[0], v[1]), pack2(v[2], v[3])};
    __builtin_amdgcn_raw_buffer_store_b64(x, r, boff(okr && n < N, e * 2), 0, 0);
  } else {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint16_t h = H16 ? (uint16_t)(pack2h(v[q], 0.f) & 0xffffu) : f2bf(v[q]);
      __builtin_amdgcn_raw_buffer_store_b16(h, r, boff(okr && n + q < N, (e + q) * 2), 0, 0);
    }
  }
}
template <int AUX = 0>
DFU_DEV void ld4_f32(rsrc_t r, int64_t e, bool okr, int n, int N, bool n4, float* v) {
  if (n4) {
    const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(r, boff(okr && n < N, e * 4), 0, AUX);
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = __uint_as_float(x[q]);
  } else {
#pragma unroll
    for (int q = 0; q < 4; ++q)
      v[q] = __uint_as_float(
          __builtin_amdgcn_raw_buffer_load_b32(r, boff(okr && n + q < N, (e + q) * 4), 0, AUX));
  }
}
DFU_DEV void ld4_bf16(rsrc_t r, int64_t e, bool okr, int n, int N, bool n4, float* v) {
  if (n4) {
    const u32x2 x = __builtin_amdgcn_raw_buffer_load_b64(r, boff(okr && n < N, e * 2), 0, 0);
    v[0] = lo_bf(x[0]);
    v[1] = hi_bf(x[0]);
    v[2] = lo_bf(x[1]);
    v[3] = hi_bf(x[1]);
  } else {
#pragma unroll
    for (int q = 0; q < 4; ++q)
      v[q] = bf2f(
          __builtin_amdgcn_raw_buffer_load_b16(r, boff(okr && n + q < N, (e + q) * 2), 0, 0));
  }
}

// Raw epilogue loads (unpacked where used, so the load can be issued steps ahead): four fp32 /
// bf16 columns n..n+3 at element e; out-of-range lanes read zeros (kOOB offset).
template <bool N4>
DFU_DEV u32x4 ldraw_f32(rsrc_t r, int64_t e, bool okr, int n, int N) {
  if constexpr (N4) return __builtin_amdgcn_raw_buffer_load_b128(r, boff(okr && n < N, e * 4), 0, 0);
  u32x4 x;
#pragma unroll
  for (int q = 0; q < 4; ++q)
    x[q] = __builtin_amdgcn_raw_buffer_load_b32(r, boff(okr && n + q < N, (e + q) * 4), 0, 0);
  return x;
}
template <bool N4>
DFU_DEV u32x2 ldraw_bf16(rsrc_t r, int64_t e, bool okr, int n, int N) {
  if constexpr (N4) return __builtin_amdgcn_raw_buffer_load_b64(r, boff(okr && n < N, e * 2), 0, 0);
  uint32_t h[4];
#pragma unroll
  for (int q = 0; q < 4; ++q)
    h[q] = __builtin_amdgcn_raw_buffer_load_b16(r, boff(okr && n + q < N, (e + q) * 2), 0, 0);
  return (u32x2){h[0] | (h[1] << 16), h[2] | (h[3] << 16)};
}

// Sum over the 16 lanes of a DPP row (the 16 rows of one MFMA fragment column), result in every
// lane: quad swaps, then half-row and row mirrors — four DPP adds instead of ds_bpermute
// shuffles, pairing the lanes as xor 1, 2, 4, 8 would (the same additions, bitwise).
template <int CTRL>
DFU_DEV float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL,
                                                               0xF, 0xF, false));
}
DFU_DEV float row16_sum(float v) {
  v += dpp_f<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_f<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_f<0x141>(v);  // row_half_mirror
  v += dpp_f<0x140>(v);  // row_mirror
  return v;
}

// Bias of the 4 columns n0w + 16j + 4*(lane>>4) + r (j < FN) by SCALAR loads (lgkmcnt, not
// vmcnt: a vector load here would make hipcc drain the in-flight DMA of the next tile), then a
// per-lane select among the 16 columns of each fragment.
template <int FN>
DFU_DEV void load_bias(const float* bias, int n0w, int N, int lane, float (&b)[FN][4]) {
  typedef const __attribute__((address_space(4))) float cfloat;
  const cfloat* bp = (const cfloat*)bias;
  const int g = lane >> 4;
  // n0w is wave-uniform (the wave's column base) but derived from threadIdx.x: without the
  // readfirstlane hipcc cannot prove it and emits VECTOR loads plus s_waitcnt vmcnt(0), which
  // drains the next tile's in-flight DMA (and the previous epilogue's stores) at every epilogue
  n0w = __builtin_amdgcn_readfirstlane(n0w);
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int nb = n0w + 16 * j;
    float s[16];
    if (nb + 16 <= N) {
#pragma unroll
      for (int q = 0; q < 16; ++q) s[q] = bp[nb + q];
    } else {
#pragma unroll
      for (int q = 0; q < 16; ++q) s[q] = nb + q < N ? bp[nb + q] : 0.f;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r)
      b[j][r] = g == 0 ? s[r] : g == 1 ? s[4 + r] : g == 2 ? s[8 + r] : s[12 + r];
  }
}

// One 16-row block of bf16 outputs (row element offset rowe; fragment j holds columns
// n0w + 16j + 4*(lane>>4) + r).  With n8, fragments j and j+1 are merged by one
// v_permlane16_swap per dword so every lane stores 8 consecutive columns (16 B): lane group g
// takes columns 16j + 16(g&1) + 8(g>>1) .. +7, the 4 lanes of a row cover 64 contiguous bytes,
// and one dwordx4 replaces two dwordx2 (HIP guide T21, for the 16x16 accumulator layout).
// H16: fp16 outputs instead of bf16 (the same 16-bit layout).
template <int FN, int AUX = 0, bool H16 = false>
DFU_DEV void st_row_bf16(rsrc_t r, int64_t rowe, bool okm, int n0w, int N, bool n8, bool n4,
                         int lane, const float (&v)[FN][4]) {
  static_assert(FN % 2 == 0, "fragment pairs");
  auto pk = [](float a, float b) { return H16 ? pack2h(a, b) : pack2(a, b); };
  if (n8) {
    const int g = lane >> 4;
    const int cofs = ((g & 1) << 4) + ((g >> 1) << 3);
#pragma unroll
    for (int j = 0; j < FN; j += 2) {
      const uint32_t a0 = pk(v[j][0], v[j][1]), a1 = pk(v[j][2], v[j][3]);
      const uint32_t b0 = pk(v[j + 1][0], v[j + 1][1]), b1 = pk(v[j + 1][2], v[j + 1][3]);
      const auto rx = __builtin_amdgcn_permlane16_swap(a0, b0, false, false);
      const auto ry = __builtin_amdgcn_permlane16_swap(a1, b1, false, false);
      const u32x4 q = {rx[0], ry[0], rx[1], ry[1]};
      const int col = n0w + 16 * j + cofs;
      __builtin_amdgcn_raw_buffer_store_b128(q, r, boff(okm && col < N, (rowe + col) * 2), 0, AUX);
    }
  } else {
    const int lcol = 4 * (lane >> 4);
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = n0w + 16 * j + lcol;
      st4_bf16<H16>(r, rowe + n, okm, n, N, n4, v[j]);
    }
  }
}

// Vector-memory instructions every wave issues in one epilogue AFTER its last load (its tile
// stores); the K-loop's waits count them.  0 = not fixed (fp32 atomics: never persistent).
template <int EPI, class T>
DFU_DEV int epi_stores(const GemmArgs& p) {
  constexpr bool bf16_out = EPI == DFU_EPI_BF16 || EPI == DFU_EPI_BF16_RELU ||
                            EPI == DFU_EPI_BF16_GELU || EPI == DFU_EPI_BF16_DGELU ||
                            EPI == DFU_EPI_BF16_ADD || EPI == DFU_EPI_BF16_STATS;
  const int per = bf16_out && p.n8 ? T::FM * T::FN / 2 : T::FM * T::FN * (p.n4 ? 1 : 4);
  if constexpr (EPI == DFU_EPI_BF16_GELU) return 2 * per;
  if constexpr (EPI == DFU_EPI_F32_STATS)  // split-pair output: two bf16 rows per fragment row
    if (p.aux_out) return 2 * (p.n8 ? T::FM * T::FN / 2 : T::FM * T::FN * (p.n4 ? 1 : 4));
  if constexpr (EPI == DFU_EPI_F32_ACC)
    if ((p.slab == nullptr && p.split > 1) || p.counters != nullptr) return 0;
  return per;
}

// C += slab 0 + ... + slab S-1 over this workgroup's tile (the last split to arrive).
template <class T, int S>
DFU_DEV void splitk_sum(const GemmArgs& p, int m0, int n0, int tid) {
  constexpr int FM = T::FM, FN = T::FN, WTM = T::WTM, WTN = T::WTN;
  const int lane = tid & 63, wave = tid >> 6;
  const int wr = wave / T::WGN, wc = wave % T::WGN;
  const int lrow = lane & 15, lcol = 4 * (lane >> 4);
  const int M = p.M, N = p.N;
  const bool n4 = p.n4 != 0;
  const rsrc_t rs = make_rsrc(p.slab);
  const rsrc_t rc = make_rsrc(p.C);
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int m = m0 + wr * WTM + 16 * i + lrow;
    const bool okm = m < M;
    const int mc = okm ? m : 0;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = n0 + wc * WTN + 16 * j + lcol;
      float x[S][4], c[4];
#pragma unroll
      for (int k = 0; k < S; ++k) ld4_f32<16>(rs, ((int64_t)k * M + mc) * N + n, okm, n, N, n4, x[k]);
      ld4_f32(rc, (int64_t)mc * p.ldc + n, okm, n, N, n4, c);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float sum = x[0][r];
#pragma unroll
        for (int k = 1; k < S; ++k) sum += x[k][r];
        c[r] += sum;
      }
      st4_f32(rc, (int64_t)mc * p.ldc + n, okm, n, N, n4, c);
    }
  }
}

// In-kernel split-K reduction (after this split's slab tile is stored, write-through): count the
// tile's arrivals; the last split to arrive adds slab 0 + ... + slab S-1 (that order, as the
// separate reduce kernel) into C and resets the counter.  No workgroup ever waits for another
// (the publish is: own stores drained -> barrier -> one agent-scope atomic), so it is correct
// for any placement of the splits over XCDs and CUs (HIP guide G16 R1: sc1 stores and loads).
template <class T>
DFU_DEV void splitk_finish(const GemmArgs& p, int m0, int n0, float* red, int tid) {
  const int t = (m0 / T::TM) * p.tiles_n + n0 / T::TN;
  int* flag = (int*)red;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (tid == 0) {
    const int old = __hip_atomic_fetch_add(p.counters + t, 1, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
    const int last = old == p.split - 1;
    if (last) __hip_atomic_store(p.counters + t, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = last;
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  const int last = *flag;
  if (!last) return;
  switch (p.split) {  // compile-time split counts: every slab load of the tile issued up front
    case 2: splitk_sum<T, 2>(p, m0, n0, tid); break;
    case 3: splitk_sum<T, 3>(p, m0, n0, tid); break;
    case 4: splitk_sum<T, 4>(p, m0, n0, tid); break;
    case 5: splitk_sum<T, 5>(p, m0, n0, tid); break;
    case 6: splitk_sum<T, 6>(p, m0, n0, tid); break;
    case 7: splitk_sum<T, 7>(p, m0, n0, tid); break;
    default: splitk_sum<T, 8>(p, m0, n0, tid); break;
  }
}

// Tail-split hand-off (GemmArgs::tail_*): store this split's accumulators (write-through),
// count the tile's arrivals, and in the last split to arrive replace acc by the sum of all the
// tile's splits in split order (its own from registers: the same values it stored), so the
// result does not depend on arrival order.  Returns whether this workgroup runs the epilogue.
// Same publish protocol as splitk_finish (no workgroup waits for another).
template <class T>
DFU_DEV bool tail_reduce(const GemmArgs& p, f32x4 (&acc)[T::FM][T::FN], int v, float* red,
                         int tid) {
  constexpr int NF = T::FM * T::FN, NT = T::NT;
  const int R = p.tail_r, S = p.tail_s;
  const int s = v / R, r = v - s * R;
  const rsrc_t rs = make_rsrc(p.tslab);
  auto off = [&](int k, int f) { return (int)(((((int64_t)k * R + r) * NF + f) * NT + tid) * 16); };
#pragma unroll
  for (int i = 0; i < T::FM; ++i)
#pragma unroll
    for (int j = 0; j < T::FN; ++j)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i][j]), rs,
                                             off(s, i * T::FN + j), 0, 16);
  int* flag = (int*)red;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (tid == 0) {
    const int old = __hip_atomic_fetch_add(p.counters + r, 1, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
    const int last = old == S - 1;
    if (last) __hip_atomic_store(p.counters + r, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = last;
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (!*flag) return false;
  // acc = slab 0 + slab 1 + ... in split order (this split's own slab re-read: the same
  // values); two slabs' loads in flight per round trip (an odd count reads slab S-1 twice and
  // adds it once: the out-of-range partner is clamped, not added).
  for (int k = 0; k < S; k += 2) {
    const int k1 = k + 1 < S ? k + 1 : k;
    f32x4 x0[T::FM][T::FN], x1[T::FM][T::FN];
#pragma unroll
    for (int i = 0; i < T::FM; ++i)
#pragma unroll
      for (int j = 0; j < T::FN; ++j) {
        x0[i][j] = __builtin_bit_cast(
            f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off(k, i * T::FN + j), 0, 16));
        x1[i][j] = __builtin_bit_cast(
            f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off(k1, i * T::FN + j), 0, 16));
      }
#pragma unroll
    for (int i = 0; i < T::FM; ++i)
#pragma unroll
      for (int j = 0; j < T::FN; ++j) {
        f32x4 a = k == 0 ? x0[i][j] : acc[i][j] + x0[i][j];
        if (k1 != k) a = a + x1[i][j];
        acc[i][j] = a;
      }
  }
  return true;
}

// ------------------------------------------------------------------------------ epilogue
// Epilogue side input (bf16 aux: the dGELU factor, the addend, the BN input y) prefetched into
// registers during the tile's LAST K-step, so its latency hides under that step's MFMAs instead
// of stalling the epilogue (which would also wait out the next tile's in-flight DMA first).
// Each lane's 4 columns of fragment (i, j) as two packed bf16 pairs.
template <int EPI, class T>
constexpr bool aux_prefetch() {
  return (EPI == DFU_EPI_BF16_DGELU || EPI == DFU_EPI_BF16_ADD) && T::FM * T::FN <= 16;
}
template <class T>
struct AuxPre {
  u32x2 v[T::FM][T::FN];
};

DFU_DEV int64_t out_row(const GemmArgs& p, int m);

template <int AMODE, int EPI, class T>
DFU_DEV void aux_load(const GemmArgs& p, int m0, int n0, int tid, AuxPre<T>& pre) {
  const int lane = tid & 63, wave = tid >> 6;
  const int wr = wave / T::WGN, wc = wave % T::WGN;
  const int lrow = lane & 15, lcol = 4 * (lane >> 4);
  const rsrc_t ra = make_rsrc(p.aux);
  const bool n4 = p.n4 != 0;
#pragma unroll
  for (int i = 0; i < T::FM; ++i) {
    const int m = m0 + wr * T::WTM + 16 * i + lrow;
    const bool okm = m < p.M;
    const int mc = okm ? m : 0;
    const int64_t mo = AMODE == DFU_OPND_CONV_DGRAD ? out_row(p, mc) : (int64_t)mc;
#pragma unroll
    for (int j = 0; j < T::FN; ++j) {
      const int n = n0 + wc * T::WTN + 16 * j + lcol;
      const int64_t e = mo * p.ldaux + n;
      if (n4) {
        pre.v[i][j] = __builtin_amdgcn_raw_buffer_load_b64(ra, boff(okm && n < p.N, e * 2), 0, 0);
      } else {
        uint32_t h[4];
#pragma unroll
        for (int q = 0; q < 4; ++q)
          h[q] = __builtin_amdgcn_raw_buffer_load_b16(ra, boff(okm && n + q < p.N, (e + q) * 2), 0, 0);
        pre.v[i][j] = (u32x2){h[0] | (h[1] << 16), h[2] | (h[3] << 16)};
      }
    }
  }
}
DFU_DEV void unpack4(u32x2 x, float* v) {
  v[0] = lo_bf(x[0]);
  v[1] = hi_bf(x[0]);
  v[2] = lo_bf(x[1]);
  v[3] = hi_bf(x[1]);
}

// lane holds C[m = m0 + wr*WTM + 16i + (lane&15)][n = n0 + wc*WTN + 16j + 4*(lane>>4) + r]
template <int AMODE, int EPI, class T>
DFU_DEV void epilogue(const GemmArgs& p, f32x4 (&acc)[T::FM][T::FN], int m0, int n0, int sidx,
                      float* red, int tid, const AuxPre<T>& pre) {
  constexpr bool kPre = aux_prefetch<EPI, T>();
  constexpr int FM = T::FM, FN = T::FN, WTM = T::WTM, WTN = T::WTN, WGM = T::WGM;
  constexpr int TM = T::TM, TN = T::TN;
  const int lane = tid & 63, wave = tid >> 6;
  const int wr = wave / T::WGN, wc = wave % T::WGN;
  const int lrow = lane & 15, lcol = 4 * (lane >> 4);
  const bool n4 = p.n4 != 0;
  const int M = p.M, N = p.N;
  const rsrc_t rc = make_rsrc(p.C);

  if constexpr (EPI == DFU_EPI_BF16_STATS || EPI == DFU_EPI_F32_STATS) {
    // bf16 (fp32) store + per-column (sum, M2) of this TM-row tile over the stored values: per
    // wave two-pass in registers, then Chan's merge across the WGM row-waves in LDS.  The stats
    // records are stored before the tile (the K-loop's waits count only the tile stores).
    float cnt = 0.f;
#pragma unroll
    for (int i = 0; i < FM; ++i) cnt += (m0 + wr * WTM + 16 * i + lrow < M) ? 1.f : 0.f;
    cnt = row16_sum(cnt);
#pragma unroll
    for (int j = 0; j < FN; ++j) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const int m = m0 + wr * WTM + 16 * i + lrow;
          const float v = EPI == DFU_EPI_BF16_STATS ? bf2f(f2bf(acc[i][j][r] * p.alpha))
                                                    : acc[i][j][r] * p.alpha;
          acc[i][j][r] = v;
          s += (m < M) ? v : 0.f;
        }
        s = row16_sum(s);
        const float mean = cnt > 0.f ? s / cnt : 0.f;
        float q = 0.f;
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const int m = m0 + wr * WTM + 16 * i + lrow;
          const float d = acc[i][j][r] - mean;
          q += (m < M) ? d * d : 0.f;
        }
        q = row16_sum(q);
        if (lrow == 0) {
          const int c = wc * WTN + 16 * j + lcol + r;
          red[(wr * TN + c) * 3 + 0] = s;
          red[(wr * TN + c) * 3 + 1] = q;
          red[(wr * TN + c) * 3 + 2] = cnt;
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    // one (sum, M2) record per 128-row block: merge the row-waves that cover each block
    const rsrc_t rs = make_rsrc(p.stats);
    constexpr int HALVES = TM / 128;
    for (int idx = tid; idx < TN * HALVES; idx += T::NT) {
      const int c = idx % TN, h = idx / TN;
      const int n = n0 + c;
      float S = 0.f, Q = 0.f, Cn = 0.f;
#pragma unroll
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
      const bool ok = n < N && m0 + 128 * h < M;
      const int64_t blk = m0 / 128 + h;
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(S), rs,
                                            boff(ok, ((blk * 2 + 0) * N + n) * 4), 0, 0);
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(Q), rs,
                                            boff(ok, ((blk * 2 + 1) * N + n) * 4), 0, 0);
    }
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int m = m0 + wr * WTM + 16 * i + lrow;
      float v[FN][4];
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) v[j][r] = acc[i][j][r];
      if constexpr (EPI == DFU_EPI_BF16_STATS) {
        st_row_bf16<FN>(rc, (int64_t)m * p.ldc, m < M, n0 + wc * WTN, N, p.n8, n4, lane, v);
      } else if (p.aux_out) {
        // split pair (the bf16x3 ResNet forward): hi = bf16(v) into C, lo = bf16(v - hi) into
        // aux_out; the BN apply reads the pair and hi is also the BN backward's bf16 y
        float lo[FN][4];
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float h = bf2f(f2bf(v[j][r]));
            lo[j][r] = v[j][r] - h;
            v[j][r] = h;
          }
        st_row_bf16<FN>(rc, (int64_t)m * p.ldc, m < M, n0 + wc * WTN, N, p.n8, n4, lane, v);
        st_row_bf16<FN>(make_rsrc(p.aux_out), (int64_t)m * p.ldaux_out, m < M, n0 + wc * WTN, N,
                        p.n8, n4, lane, lo);
      } else {
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int n = n0 + wc * WTN + 16 * j + lcol;
          st4_f32(rc, (int64_t)(m < M ? m : 0) * p.ldc + n, m < M, n, N, n4, v[j]);
        }
      }
    }
  } else {
    constexpr bool kBias = EPI == DFU_EPI_BF16 || EPI == DFU_EPI_BF16_RELU || EPI == DFU_EPI_F32 ||
                           EPI == DFU_EPI_F32_RESID || EPI == DFU_EPI_BF16_GELU ||
                           EPI == DFU_EPI_PATCH;
    float bias[FN][4];
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) bias[j][r] = 0.f;
    if (kBias && p.bias) load_bias<FN>(p.bias, n0 + wc * WTN, N, lane, bias);
    const rsrc_t ra = make_rsrc(p.aux);
    const rsrc_t ro = make_rsrc(EPI == DFU_EPI_F32_ACC ? (const void*)p.slab : p.aux_out);
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int m = m0 + wr * WTM + 16 * i + lrow;
      const bool okm = m < M;
      const int mc = okm ? m : 0;
      const int64_t mo = AMODE == DFU_OPND_CONV_DGRAD ? out_row(p, mc) : (int64_t)mc;
      const int n0w = n0 + wc * WTN;
      float v[FN][4];
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) v[j][r] = acc[i][j][r] * p.alpha + bias[j][r];
      if constexpr (EPI == DFU_EPI_BF16 || EPI == DFU_EPI_BF16_RELU) {
        if constexpr (EPI == DFU_EPI_BF16_RELU) {
#pragma unroll
          for (int j = 0; j < FN; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) v[j][r] = fmaxf(v[j][r], 0.f);
        }
        st_row_bf16<FN>(rc, mo * p.ldc, okm, n0w, N, p.n8, n4, lane, v);
      } else if constexpr (EPI == DFU_EPI_BF16_GELU) {
        // GELU and its derivative from one erfc/exp evaluation: the backward's dGELU
        // epilogue then only multiplies (no transcendental work in the dgrad GEMM)
        float g[FN][4], d[FN][4];
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) gelu_and_grad(v[j][r], g[j][r], d[j][r]);
        st_row_bf16<FN>(ro, mo * p.ldaux_out, okm, n0w, N, p.n8, n4, lane, d);
        st_row_bf16<FN>(rc, mo * p.ldc, okm, n0w, N, p.n8, n4, lane, g);
      } else if constexpr (EPI == DFU_EPI_BF16_DGELU || EPI == DFU_EPI_BF16_ADD) {
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int n = n0w + 16 * j + lcol;
          float x[4];
          if constexpr (kPre)
            unpack4(pre.v[i][j], x);
          else
            ld4_bf16(ra, mo * p.ldaux + n, okm, n, N, n4, x);
#pragma unroll
          for (int r = 0; r < 4; ++r)
            v[j][r] = (EPI == DFU_EPI_BF16_DGELU) ? v[j][r] * x[r] : v[j][r] + x[r];
        }
        st_row_bf16<FN>(rc, mo * p.ldc, okm, n0w, N, p.n8, n4, lane, v);
      } else {
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int n = n0w + 16 * j + lcol;
          if constexpr (EPI == DFU_EPI_F32) {
            st4_f32(rc, mo * p.ldc + n, okm, n, N, n4, v[j]);
          } else if constexpr (EPI == DFU_EPI_F32_RESID) {
            float x[4];
            ld4_f32(ra, mo * p.ldaux + n, okm, n, N, n4, x);
#pragma unroll
            for (int r = 0; r < 4; ++r) v[j][r] += x[r];
            st4_f32(rc, mo * p.ldc + n, okm, n, N, n4, v[j]);
          } else if constexpr (EPI == DFU_EPI_F32_ACC) {
            if (p.slab != nullptr) {
              // split-K partial into this split's slab (write-through when reduced in-kernel)
              if (p.counters != nullptr)
                st4_f32<16>(ro, ((int64_t)sidx * M + mc) * N + n, okm, n, N, n4, v[j]);
              else
                st4_f32(ro, ((int64_t)sidx * M + mc) * N + n, okm, n, N, n4, v[j]);
            } else if (p.split > 1) {  // fp32 atomics: launched one unit per workgroup (host)
              float* C = (float*)p.C + (int64_t)mc * p.ldc + n;
              for (int r = 0; r < 4; ++r)
                if (okm && n + r < N) atomicAdd(C + r, v[j][r]);
            } else {
              float c[4];
              ld4_f32(rc, (int64_t)mc * p.ldc + n, okm, n, N, n4, c);
#pragma unroll
              for (int r = 0; r < 4; ++r) v[j][r] += c[r];
              st4_f32(rc, (int64_t)mc * p.ldc + n, okm, n, N, n4, v[j]);
            }
          } else if constexpr (EPI == DFU_EPI_PATCH) {
            // m = b*T + t -> row b*(T+1) + 1 + t of the fp32 token matrix, + pos-embed row 1+t
            const int Tt = p.ep_tokens;
            const int b = mc / Tt, t = mc - b * Tt;
            float pe[4];
            ld4_f32(ra, (int64_t)(1 + t) * p.ldaux + n, okm, n, N, n4, pe);
#pragma unroll
            for (int r = 0; r < 4; ++r) v[j][r] += pe[r];
            st4_f32(rc, ((int64_t)b * (Tt + 1) + 1 + t) * p.ldc + n, okm, n, N, n4, v[j]);
          }
        }
      }
    }
    if constexpr (EPI == DFU_EPI_F32_ACC) {
      if (p.slab != nullptr && p.counters != nullptr) splitk_finish<T>(p, m0, n0, red, tid);
    }
  }
}

// ------------------------------------------------------------------------------ kernel
template <int AMODE, int BMODE, int EPI, int TM, int TN, int OCC = 1, int NST = 0, int NW = 8,
          bool X3 = false>
__global__ __launch_bounds__(64 * NW, OCC) void gemm_kernel(const GemmArgs p) {
  using T = Tile<TM, TN, OCC, NST, NW>;
  constexpr int WGN = T::WGN, WTM = T::WTM, WTN = T::WTN;
  constexpr int FM = T::FM, FN = T::FN, NSTAGE = T::NSTAGE;
  constexpr int SCRATCH = (EPI == DFU_EPI_BF16_STATS || EPI == DFU_EPI_F32_STATS)
                              ? T::STATS_BYTES
                              : 16;  // stats / flag
  // ALL LDS in one array: a second __shared__ object can make hipcc drain the DMA per K-step
  __shared__ __attribute__((aligned(16))) char smem[T::LDS_BYTES + SCRATCH];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wr = wave / WGN, wc = wave % WGN;

  // Tail split (GemmArgs::tail_*) is built into the 8-wave 128x128 variants only (8 accumulator
  // fragments per lane); in the larger ones its code costs register spills, and the host never
  // requests it from them (gemm.hip kTailOK).
  constexpr bool kTail = NW == 8 && FM * FN <= 8 && EPI != DFU_EPI_F32_ACC;
  const int tiles = p.tiles_m * p.tiles_n;
  const int units = kTail && p.tail_r ? p.tail_full + p.tail_r * p.tail_s : tiles * p.split;
  // Units by rounds: in round i workgroup b takes unit i*G + w(b).  In complete rounds w is
  // the XCD-aware bijective remap (blocks b and b+8 share an XCD): each XCD gets a contiguous
  // range of units, neighbours in the grouped raster below that share A and B panels in its
  // L2.  In the last, partial round w(b) = b, so its units spread over all XCDs and CUs (the
  // dispatcher places block b on XCD b % 8) instead of piling onto the first XCDs.
  const int nwg = gridDim.x;
  const int bid = blockIdx.x;
  int wg = bid;
  if (nwg >= 16) {
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  const int full = units / nwg;
  const int rounds = full + (bid < units - full * nwg ? 1 : 0);
  if (rounds == 0) return;
  auto unit_at = [&](int i) { return i * nwg + (i < full ? wg : bid); };

  // unit u -> split s = u / tiles and tile t = u % tiles in a grouped raster (GROUP_M x
  // tiles_n bands walked column by column)
  // (tail units: v = u - tail_full -> split v / tail_r of tail tile tail_full + v % tail_r)
  auto unit_geom = [&](int u, int& m0, int& n0, int& kb, int& nk) {
    constexpr int GROUP_M = 4;
    int s, t, kps;
    if (kTail && p.tail_r && u >= p.tail_full) {
      const int v = u - p.tail_full;
      s = v / p.tail_r;
      t = p.tail_full + (v - s * p.tail_r);
      kps = p.tail_kps;
    } else {
      s = u / tiles;
      t = u - s * tiles;
      kps = p.kt_per_split;
    }
    const int band = GROUP_M * p.tiles_n;
    const int g0 = (t / band) * GROUP_M;
    const int gm = min(GROUP_M, p.tiles_m - g0);
    const int within = t - (t / band) * band;
    m0 = (g0 + within % gm) * TM;
    n0 = (within / gm) * TN;
    kb = s * kps;
    nk = min(p.ktiles, kb + kps) - kb;
  };
  int total = 0;  // K-steps over all of this workgroup's units
  for (int i = 0; i < rounds; ++i) {
    int m0_, n0_, kb_, nk_;
    unit_geom(unit_at(i), m0_, n0_, kb_, nk_);
    total += nk_;
  }

  // issue cursor: the round / K-step the next DMA stage loads
  LoadState<T::NLDA> sa;
  LoadState<T::NLDB> sb;
  int iu = 0, ik = 0, im0, in0, ikb, ink;
  unit_geom(unit_at(0), im0, in0, ikb, ink);
  load_init<AMODE, T::NLDA, NW>(p, sa, p.A, p.lda, im0, p.M, tid);
  load_init<BMODE, T::NLDB, NW>(p, sb, p.B, p.ldb, in0, p.N, tid);
  auto issue_next = [&](char* stage) {
    if (!(p.dbg & 4)) {
    issue_tile<AMODE, T::NLDA, NW, true, X3>(p, sa, p.A, p.lda, p.m_ld_bound, ikb + ik, p.K, tid,
                                         stage);
    issue_tile<BMODE, T::NLDB, NW>(p, sb, p.B, p.ldb, p.n_ld_bound, ikb + ik, p.K, tid,
                               stage + T::A_BYTES);
    }
    if (++ik == ink) {
      ik = 0;
      if (++iu < rounds) {
        unit_geom(unit_at(iu), im0, in0, ikb, ink);
        load_init<AMODE, T::NLDA, NW>(p, sa, p.A, p.lda, im0, p.M, tid);
        load_init<BMODE, T::NLDB, NW>(p, sb, p.B, p.ldb, in0, p.N, tid);
      }
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  constexpr bool AK = kcontig<AMODE>();
  constexpr bool BKc = kcontig<BMODE>();
  // All fragment reads of the K-step (both 32-wide halves) are issued before the first MFMA,
  // so the LDS latency overlaps MFMAs (counted lgkmcnt waits) instead of draining per group.
  auto compute = [&](const char* la) {
    const char* lb = la + T::A_BYTES;
    static_assert(!X3 || (FM * FN < 32 && AK && BKc),
                  "interleaved pairs: K-contiguous operands, at most 64x64 per wave");
    if constexpr (FM * FN >= 32) {
      // 256x256: 128 accumulator registers leave room for one k-half of fragments at a time
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8 fa[FM], fb[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i) fa[i] = read_frag<AK>(la, wr * WTM + i * 16, ks, lane);
#pragma unroll
        for (int j = 0; j < FN; ++j) fb[j] = read_frag<BKc>(lb, wc * WTN + j * 16, ks, lane);
        if constexpr (!AK || !BKc) {  // asm (MN-major) reads: retired before the MFMAs
          lds_reads_retired();
#pragma unroll
          for (int i = 0; i < FM; ++i) pin(fa[i]);
#pragma unroll
          for (int j = 0; j < FN; ++j) pin(fb[j]);
        }
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
      }
    } else {
      bf16x8 fa[2][FM], fb[2][FN];
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
        for (int i = 0; i < FM; ++i) fa[ks][i] = read_frag<AK>(la, wr * WTM + i * 16, ks, lane);
#pragma unroll
        for (int j = 0; j < FN; ++j) fb[ks][j] = read_frag<BKc>(lb, wc * WTN + j * 16, ks, lane);
      }
      __builtin_amdgcn_sched_barrier(0);  // keep the reads ahead (the scheduler sinks them)
      if constexpr (!AK || !BKc) {  // asm (MN-major) reads: retired before the MFMAs
        lds_reads_retired();
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
          for (int i = 0; i < FM; ++i) pin(fa[ks][i]);
#pragma unroll
          for (int j = 0; j < FN; ++j) pin(fb[ks][j]);
        }
      }
      if constexpr (X3) {
        // interleaved pairs: k-half 0 holds hi and 1 holds lo of the same 32 real k, so the
        // step is hi·hi + lo·hi + hi·lo (the tripled-K sum, from 2 operand tiles instead of 3)
#pragma unroll
        for (int t = 0; t < 3; ++t)
#pragma unroll
          for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[t == 2][j], fa[t == 1][i],
                                                                 acc[i][j], 0, 0, 0);
      } else {
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j)
              acc[i][j] =
                  __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[ks][j], fa[ks][i], acc[i][j], 0, 0, 0);
      }
    }
  };

  // Pipeline over the flattened K-step stream: step g+NSTAGE-1 is issued (into the slot step
  // g-1 vacated) right after the barrier that publishes step g.  Before that barrier each wave
  // waits until its share of step g's DMA has landed; younger than it are the
  // min(NSTAGE-2, total-1-g) stages issued after it and the stores of every epilogue run since
  // (bit k of `hist`: an epilogue ran k+1 steps ago).
  const int E = (p.dbg & 1) ? 0 : epi_stores<EPI, T>(p);
  AuxPre<T> pre;
  float* red = (float*)(smem + T::LDS_BYTES);
  unsigned hist = 0;
  int ci = 0, cu = unit_at(0), ck = 0, cm0, cn0, ckb, cnk;
  unit_geom(cu, cm0, cn0, ckb, cnk);
#pragma unroll
  for (int s = 0; s < NSTAGE - 1; ++s)
    if (s < total) issue_next(smem + s * T::STAGE_BYTES);
  int slot = 0;
  for (int g = 0; g < total; ++g) {
    const int later = min(NSTAGE - 2, total - 1 - g);
    const unsigned win = hist & ((1u << (NSTAGE - 1)) - 1u);
    if (win == 0 && later == NSTAGE - 2)  // steady state: a fixed count, no ladder
      wait_vmcnt<T::DMA_PER_STAGE * (NSTAGE - 2)>();
    else
      wait_vm_le<63>(T::DMA_PER_STAGE * later + E * __builtin_popcount(win));
    __builtin_amdgcn_s_barrier();
    if (g + NSTAGE - 1 < total) {
      const int is = slot == 0 ? NSTAGE - 1 : slot - 1;  // (g + NSTAGE - 1) % NSTAGE
      issue_next(smem + is * T::STAGE_BYTES);
    }
    if constexpr (aux_prefetch<EPI, T>())
      if (ck + 1 == cnk) aux_load<AMODE, EPI, T>(p, cm0, cn0, tid, pre);
    if (!(p.dbg & 2)) compute(smem + slot * T::STAGE_BYTES);
    slot = slot == NSTAGE - 1 ? 0 : slot + 1;
    hist <<= 1;
    if (++ck == cnk) {
      // a tail split ends its workgroup's stream: hand off, and only the tile's last runs on
      bool epi = true;
      if constexpr (kTail)
        if (p.tail_r && cu >= p.tail_full) epi = tail_reduce<T>(p, acc, cu - p.tail_full, red, tid);
      if (epi && !(p.dbg & 1))
        epilogue<AMODE, EPI, T>(p, acc, cm0, cn0, cu / tiles, red, tid, pre);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
      hist |= 1u;
      ck = 0;
      if (++ci < rounds) {
        cu = unit_at(ci);
        unit_geom(cu, cm0, cn0, ckb, cnk);
      }
    }
  }
}

}  // namespace dfu
