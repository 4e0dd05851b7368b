// 256x256 phased GEMM (the ViT linears: forward, dgrad and wgrad): the K-step is split
// into four phases, each {one barrier; this phase's fragment reads; one half-tile of the NEXT
// K-step's LDS-DMA; a 16-MFMA cluster}, so LDS reads, DMA issue and MFMAs interleave at a fine
// grain instead of one burst each per K-step (cdna_hip_programming.md "The 256² 8-phase
// template": the per-phase interleave is the lever).
//
// Geometry: 8 waves as 2 (M) x 4 (N); wave (wr, wc) owns rows {h*128 + wr*64 + 0..63 : h = 0,1}
// and columns {h*128 + wc*32 + 0..31 : h = 0,1}, i.e. one quarter of each operand HALF-tile
// (A rows 0-127 / 128-255, B columns 0-127 / 128-255).  Phase q computes the quadrant
// (A half, B half) = (top, left), (top, right), (bottom, right), (bottom, left): every wave reads
// the same half-tiles in the same phase, so each phase waits only for the half-tile(s) it
// reads.  The next K-step's half-tiles are issued in phases 1-4 in the order of first use (A-top,
// B-left, B-right, A-bottom) into the other of two LDS buffers (2 x 64 KiB).
//   RAW: phase 1 needs A-top + B-left (younger: 2 half-tiles = 4 DMA per thread -> vmcnt(4)),
//        phase 2 B-right (younger: A-bottom + next A-top -> 4), phase 3 A-bottom (younger: next
//        A-top + B-left -> 4), phase 4 reads B-left again (retired at phase 1).  Each wave waits
//        for its own DMA, then the phase barrier publishes everyone's.
//   WAR: a half-tile of the other buffer is re-filled at least one barrier after its last read
//        (A-top: read phase 1, re-filled next phase 1; B-left 4 -> 2; B-right 2 -> 3;
//        A-bottom 3 -> 4), and reads are retired (lgkmcnt(0)) before each MFMA cluster.
// One workgroup per CU; workgroups walk tiles (grouped raster, XCD-aware) one at a time.
// A and B K-contiguous (forward), B MN-major (dgrad), or both MN-major (wgrad, split-K units
// into fp32 slabs) -- MN-major halves are 128-column tr16 sub-images.
// Epilogues: BF16 (+bias), BF16_GELU (GELU'(pre) to aux_out), F32_RESID; dgrad: BF16,
// BF16_DGELU, BF16_ADD.
#include "gemm_table.h"

namespace dfu {
namespace {

constexpr int P8_IMG = 256 * 128;     // one operand image: 256 rows x 64 k x 2 B
constexpr int P8_BUF = 2 * P8_IMG;    // A + B
constexpr int P8_LDS = 2 * P8_BUF;    // two buffers: 128 KiB

// One half-tile (128 rows x 64 k) of a K-contiguous operand into rows 128h.. of `img`: two
// wave-instructions per thread; piece q = wave + 8i covers image rows 128h + 8q .. +7.
DFU_DEV void p8_issue_half(const bf16_t* base, int64_t ld, int row0, int rows, int k0, int K,
                           int h, char* img, int tid) {
  const int lane = tid & 63, wave = tid >> 6;
  const int c = kc_lane_chunk(lane);
  const bool kin = k0 + c * 8 < K;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int q = wave + 8 * i;
    const int r = 128 * h + 8 * q + (lane >> 3);
    const int g = row0 + r;
    const bool ok = kin && g < rows;
    glds16(ok ? (const void*)(base + (int64_t)g * ld + k0 + c * 8) : (const void*)g_zero16,
           img + h * 16384 + q * 1024);
  }
}

// One half-tile (64 k x 128 columns = one 16 KiB MN-contiguous sub-image) of an MN-major
// operand X[k][mn] into sub-image h of `img`: the layout of gemm_kernel.h's MN images (piece q
// = k-rows 4q .. 4q+3, lane chunk swizzled by the k-row), two wave-instructions per thread.
DFU_DEV void p8_issue_half_mn(const bf16_t* base, int64_t ld, int col0, int col_bound, int k0,
                              int K, int h, char* img, int tid) {
  const int wave = tid >> 6;
  const int col = col0 + 128 * h + 8 * mn_lane_chunk(tid);
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int k = k0 + (tid >> 4) + 32 * i;
    const bool ok = col < col_bound && k < K;
    glds16(ok ? (const void*)(base + (int64_t)k * ld + col) : (const void*)g_zero16,
           img + 16384 * h + 8192 * i + 1024 * wave);
  }
}

// Epilogue, compiled per n4 (N4) so that no control flow surrounds its loads and hipcc's wait
// counts stay exact.  Bias by scalar loads (load_bias: the wave's column base is uniform); the
// reading epilogues (residual, gelu', addend, C) issue each step's load PD steps ahead of the
// stores between (vmcnt retires in issue order: a load issued behind a store waits for it).
template <int EPI, bool N4>
DFU_DEV void p8_epilogue_n(const GemmArgs& p, f32x4 (&acc)[8][4], int m0, int n0, int wr, int wc,
                           int lane, int sidx) {
  constexpr bool n4 = N4;
  const int M = p.M, N = p.N;
  const rsrc_t rc = make_rsrc(p.C);
  const rsrc_t ra = make_rsrc(p.aux);
  const rsrc_t ro = make_rsrc(p.aux_out);
  constexpr bool kLdF = EPI == DFU_EPI_F32_RESID || EPI == DFU_EPI_F32_ACC;
  constexpr bool kLdH = EPI == DFU_EPI_BF16_DGELU || EPI == DFU_EPI_BF16_ADD;
  constexpr int NS = 32, PD = 4;  // steps (j, i): fragment column j outer, row i inner
  const bool ld_c = EPI == DFU_EPI_F32_RESID || p.slab == nullptr;
  u32x4 af[NS];
  u32x2 ah[NS];
  auto col_of = [&](int j) { return n0 + (j >> 1) * 128 + wc * 32 + (j & 1) * 16 + 4 * (lane >> 4); };
  auto row_of = [&](int i) { return m0 + (i >> 2) * 128 + wr * 64 + (i & 3) * 16 + (lane & 15); };
  auto load_step = [&](int st) {
    if constexpr (kLdF || kLdH) {
      const int n = col_of(st >> 3), m = row_of(st & 7);
      const bool okm = m < M;
      const int64_t mc = okm ? m : 0;
      if constexpr (EPI == DFU_EPI_F32_RESID)
        af[st] = ldraw_f32<N4>(ra, mc * p.ldaux + n, okm, n, N);
      else if constexpr (EPI == DFU_EPI_F32_ACC) {
        if (ld_c) af[st] = ldraw_f32<N4>(rc, mc * p.ldc + n, okm, n, N);
      } else
        ah[st] = ldraw_bf16<N4>(ra, mc * p.ldaux + n, okm, n, N);
    }
  };
  float bias[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) bias[j][r] = 0.f;
  if (p.bias) {  // (before the loads: no control flow between a load and its use)
    float b2[2][4];
#pragma unroll
    for (int hb = 0; hb < 2; ++hb) {
      load_bias<2>(p.bias, n0 + hb * 128 + wc * 32, N, lane, b2);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        bias[2 * hb][r] = b2[0][r];
        bias[2 * hb + 1][r] = b2[1][r];
      }
    }
  }
#pragma unroll
  for (int st = 0; st < PD; ++st) load_step(st);
#pragma unroll
  for (int st = 0; st < NS; ++st) {
    if (st + PD < NS) load_step(st + PD);
    if constexpr (kLdF || kLdH) __builtin_amdgcn_sched_barrier(0);
    const int j = st >> 3, i = st & 7;
    const int n = col_of(j);
    const int m = row_of(i);
    const bool okm = m < M;
    const int64_t mc = okm ? m : 0;
    float v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = acc[i][j][r] * p.alpha + bias[j][r];
    if constexpr (EPI == DFU_EPI_BF16) {
      st4_bf16(rc, mc * p.ldc + n, okm, n, N, n4, v);
    } else if constexpr (EPI == DFU_EPI_BF16_GELU) {
      float g[4], d[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) gelu_and_grad(v[r], g[r], d[r]);
      st4_bf16(ro, mc * p.ldaux_out + n, okm, n, N, n4, d);
      st4_bf16(rc, mc * p.ldc + n, okm, n, N, n4, g);
    } else if constexpr (EPI == DFU_EPI_BF16_DGELU || EPI == DFU_EPI_BF16_ADD) {
      float x[4];
      unpack4(ah[st], x);
#pragma unroll
      for (int r = 0; r < 4; ++r)
        v[r] = EPI == DFU_EPI_BF16_DGELU ? v[r] * x[r] : v[r] + x[r];
      st4_bf16(rc, mc * p.ldc + n, okm, n, N, n4, v);
    } else if constexpr (EPI == DFU_EPI_F32_ACC) {  // split-K slab, or C += acc unsplit
      if (p.slab != nullptr) {
        st4_f32(make_rsrc(p.slab), ((int64_t)sidx * M + mc) * N + n, okm, n, N, n4, v);
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += __uint_as_float(af[st][r]);
        st4_f32(rc, mc * p.ldc + n, okm, n, N, n4, v);
      }
    } else {  // DFU_EPI_F32_RESID
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] += __uint_as_float(af[st][r]);
      st4_f32(rc, mc * p.ldc + n, okm, n, N, n4, v);
    }
  }
}
template <int EPI>
DFU_DEV void p8_epilogue(const GemmArgs& p, f32x4 (&acc)[8][4], int m0, int n0, int wr, int wc,
                         int lane, int sidx) {
  if (p.n4)
    p8_epilogue_n<EPI, true>(p, acc, m0, n0, wr, wc, lane, sidx);
  else
    p8_epilogue_n<EPI, false>(p, acc, m0, n0, wr, wc, lane, sidx);
}

template <int AMODE, int BMODE, int EPI>
__global__ __launch_bounds__(512) void gemm_p8(const GemmArgs p) {
  constexpr bool AK_ = AMODE == DFU_OPND_KMAJOR;  // A K-contiguous (else MN-major: wgrad)
  constexpr bool BK_ = BMODE == DFU_OPND_KMAJOR;  // B K-contiguous (else MN-major: dgrad, wgrad)
  auto issue_a = [&](int m0_, int k0_, int h, char* img) {
    if constexpr (AK_)
      p8_issue_half(p.A, p.lda, m0_, p.M, k0_, p.K, h, img, threadIdx.x);
    else
      p8_issue_half_mn(p.A, p.lda, m0_, p.m_ld_bound, k0_, p.K, h, img, threadIdx.x);
  };
  auto issue_b = [&](int n0_, int k0_, int h, char* img) {
    if constexpr (BK_)
      p8_issue_half(p.B, p.ldb, n0_, p.N, k0_, p.K, h, img, threadIdx.x);
    else
      p8_issue_half_mn(p.B, p.ldb, n0_, p.n_ld_bound, k0_, p.K, h, img, threadIdx.x);
  };
  __shared__ __attribute__((aligned(16))) char smem[P8_LDS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;
  const int tiles = p.tiles_m * p.tiles_n;
  const int nwg = gridDim.x, bid = blockIdx.x;
  int wg = bid;
  if (nwg >= 16) {  // bijective XCD-aware remap: blocks b and b+8 share an XCD
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  // work units: tile x K-split (split s covers K-steps [s*kps, (s+1)*kps) and stores an fp32
  // slab for the reduce kernel; F32_ACC only)
  const int units = tiles * p.split;
  for (int u = wg; u < units; u += nwg) {
    const int sidx = u / tiles, t = u - sidx * tiles;
    const int kb = sidx * p.kt_per_split;
    const int nk = min(p.ktiles, kb + p.kt_per_split) - kb;
    constexpr int GROUP_M = 4;
    const int band = GROUP_M * p.tiles_n;
    const int g0 = (t / band) * GROUP_M;
    const int gm = min(GROUP_M, p.tiles_m - g0);
    const int within = t - (t / band) * band;
    const int m0 = (g0 + within % gm) * 256, n0 = (within / gm) * 256;

    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

    // the previous tile's last reads of buffer 0 must be done before its prologue refills it
    __builtin_amdgcn_s_barrier();
    // prologue: K-step 0 into buffer 0, in first-use order (A-top, B-left, B-right, A-bottom)
    issue_a(m0, kb * BK, 0, smem);
    issue_b(n0, kb * BK, 0, smem + P8_IMG);
    issue_b(n0, kb * BK, 1, smem + P8_IMG);
    issue_a(m0, kb * BK, 1, smem);

    for (int kt = 0; kt < nk; ++kt) {
      const char* la = smem + (kt & 1) * P8_BUF;
      const char* lb = la + P8_IMG;
      char* na = smem + ((kt & 1) ^ 1) * P8_BUF;
      char* nb = na + P8_IMG;
      const bool nxt = kt + 1 < nk;
      const int k1 = (kb + kt + 1) * BK;
      bf16x8 fa[4][2], fb[2][2];
      auto read_a = [&](int h) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int ks = 0; ks < 2; ++ks)
            fa[i][ks] = read_frag<AK_>(la, h * 128 + wr * 64 + i * 16, ks, lane);
      };
      auto read_b = [&](int h) {
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int ks = 0; ks < 2; ++ks)
            fb[j][ks] = read_frag<BK_>(lb, h * 128 + wc * 32 + j * 16, ks, lane);
      };
      auto mfma = [&](int ha, int hb) {
        lds_reads_retired();
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {  // (asm MN-major reads: ordered after the wait)
#pragma unroll
          for (int i = 0; i < 4; ++i) pin(fa[i][ks]);
#pragma unroll
          for (int j = 0; j < 2; ++j) pin(fb[j][ks]);
        }
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
              acc[ha * 4 + i][hb * 2 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                  fb[j][ks], fa[i][ks], acc[ha * 4 + i][hb * 2 + j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
      };
      // one barrier per K-step (all of this K-step's half-tiles landed and published); the next
      // K-step's DMA goes out in phases 1 and 2, leaving phases 3-4 of MFMAs to cover it; waves
      // drift freely through phases 2-4 (no LDS hazard inside a K-step)
      wait_vmcnt<0>();
      __builtin_amdgcn_s_barrier();
      read_a(0);
      read_b(0);
      if (nxt) {
        issue_a(m0, k1, 0, na);
        issue_b(n0, k1, 0, nb);
      }
      mfma(0, 0);
      read_b(1);
      if (nxt) {
        issue_b(n0, k1, 1, nb);
        issue_a(m0, k1, 1, na);
      }
      mfma(0, 1);
      read_a(1);
      mfma(1, 1);
      read_b(0);
      mfma(1, 0);
    }
    p8_epilogue<EPI>(p, acc, m0, n0, wr, wc, lane, sidx);
  }
}

}  // namespace

#define P8(A, B, E) {A, B, E, T256x256p8, &gemm_p8<A, B, E>, P8_LDS, 512}
const Entry kTable256x256p8[] = {
    P8(DFU_OPND_KMAJOR, DFU_OPND_KMAJOR, DFU_EPI_BF16),
    P8(DFU_OPND_KMAJOR, DFU_OPND_KMAJOR, DFU_EPI_BF16_GELU),
    P8(DFU_OPND_KMAJOR, DFU_OPND_KMAJOR, DFU_EPI_F32_RESID),
    P8(DFU_OPND_KMAJOR, DFU_OPND_MNMAJOR, DFU_EPI_BF16),
    P8(DFU_OPND_KMAJOR, DFU_OPND_MNMAJOR, DFU_EPI_BF16_DGELU),
    P8(DFU_OPND_KMAJOR, DFU_OPND_MNMAJOR, DFU_EPI_BF16_ADD),
    P8(DFU_OPND_MNMAJOR, DFU_OPND_MNMAJOR, DFU_EPI_F32_ACC),  // weight gradients (split-K slabs)
};
#undef P8
const int kTable256x256p8N = sizeof(kTable256x256p8) / sizeof(Entry);

}  // namespace dfu
