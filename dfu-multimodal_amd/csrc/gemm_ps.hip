// Persistent phased 256x256 GEMM (tile 8): the K-step body of gemm_p8.hip (four 16-MFMA
// quadrant phases, the next K-step's half-tile DMA issued in phases 1-2, one barrier per K-step)
// run over ONE continuous stream of K-steps per workgroup, across its work units: the DMA of a
// unit's first K-step is issued during the previous unit's last K-step, so the 64 KiB stage
// fill never starts cold after the first unit, and the epilogue's stores drain under the next
// unit's MFMAs (the K-step wait counts them, as gemm_kernel.h's persistent loop does).
//
// Geometry (as gemm_p8): 8 waves as 2 (M) x 4 (N); wave (wr, wc) owns rows
// {h*128 + wr*64 + 0..63 : h = 0,1} and columns {h*128 + wc*32 + 0..31 : h = 0,1}.  Two LDS
// buffers of 64 KiB (A 256 x 64, B 256 x 64).  Work units as gemm_kernel: output tile x K-split
// (F32_ACC split-K into fp32 slabs), XCD-aware bijective remap, grouped raster.
//   RAW: the K-step g barrier follows every wave's wait for its own DMA of K-step g (issued in
//        K-step g-1, phases 1-2; younger than it are only the stores of an epilogue run at the
//        end of K-step g-1: a fixed count per wave).
//   WAR: buffer (g+1)&1 is refilled after the K-step g barrier, which every wave passes only
//        after its K-step g-1 MFMAs consumed every fragment read from that buffer.
// Epilogue stores are buffer stores masked by an out-of-range offset (a fixed count per wave).
#include "gemm_table.h"

namespace dfu {
namespace {

// Timing ablations (tools/build_ablate.sh builds a separate library with -DDFU_PS_ABLATE=mask;
// the product build is 0): 1 no epilogue, 2 no MFMA, 4 no DMA, 8 no fragment reads (zero
// fragments), 16 no K-step barrier, 32 epilogue accesses out of range (issued, no traffic),
// 64 / 128 no B DMA / no B fragment reads, 256 / 512 the same for A.  The DMA and read
// ablations keep the first K-step's (random) data in LDS / in the fragments: MFMAs on zero
// operands would run at a higher clock (MI355X_MICROARCH.md, DVFS give-back).  Results are wrong in every ablated build.
#ifndef DFU_PS_ABLATE
#define DFU_PS_ABLATE 0
#endif
constexpr int kAbl = DFU_PS_ABLATE;

constexpr int PS_IMG = 256 * 128;   // one operand image: 256 rows x 64 k x 2 B
constexpr int PS_BUF = 2 * PS_IMG;  // A + B
constexpr int PS_LDS = 2 * PS_BUF;  // two buffers: 128 KiB

// DMA of one operand half-tile by buffer_load ... lds (a buffer resource over the operand, 32-bit
// per-lane byte offsets): a lane out of range carries offset kOOB and the hardware fills its 16
// bytes with zeros -- no per-lane pointer select, no branch.  Per-lane state for the current
// issue unit (computed once per unit; the K-step loop adds a wave-uniform k offset):
//   K-contiguous: image row (tid>>3) + 64i (i = 0..3; half h = rows 128h.. = i in {2h, 2h+1}),
//     this lane's 16-B chunk kc_lane_chunk(lane) of the K-step (gemm_kernel.h's KMAJOR image);
//   MN-major: half h = 128 columns from col0 + 128h (lane chunk mn_lane_chunk(tid)), k-rows
//     (tid>>4) + 32i (i = 0, 1) of the K-step (gemm_kernel.h's MN sub-images).
template <bool KC>
struct PsSrc {
  uint32_t off[4];  // byte offset of this lane's first element (K-contiguous: row base + chunk)
  bool ok[4];
};

template <bool KC>
DFU_DEV void ps_src_init(PsSrc<KC>& s, int64_t ld, int mn0, int bound, int tid) {
  if constexpr (KC) {
    const int kc = kc_lane_chunk(tid & 63) * 8;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = mn0 + (tid >> 3) + 64 * i;
      s.ok[i] = row < bound;
      s.off[i] = (uint32_t)(((int64_t)(s.ok[i] ? row : 0) * ld + kc) * 2);
    }
  } else {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int col = mn0 + 128 * h + 8 * mn_lane_chunk(tid);
      s.ok[h] = col < bound;
      s.off[h] = (uint32_t)((s.ok[h] ? col : 0) * 2);
    }
  }
}

typedef __attribute__((address_space(3))) void lds_void_t;
DFU_DEV void bl16(rsrc_t r, uint32_t off, char* lds_dst) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_t*)lds_dst, 16, off, 0, 0, 0);
}

// Half-tile h of K-step k0 into `img` (two wave-instructions per thread; wave = tid >> 6, kept
// wave-uniform by the caller so the LDS destination is scalar).
// NCH: 64-row chunks of a K-contiguous image (4; 3 for the 192-row A operand: chunk 3 unused).
template <bool KC, int NCH = 4>
DFU_DEV void ps_issue(const PsSrc<KC>& s, rsrc_t r, int64_t ld, int k0, int K, int h, char* img,
                      int tid, int wave) {
  if constexpr (KC) {
    // (bitwise &, not &&: no short-circuit control flow around the loads)
    const bool kin = k0 + kc_lane_chunk(tid & 63) * 8 < K;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      if (2 * h + i >= NCH) continue;  // (h is a literal at every call: folds)
      const bool ok = kin & s.ok[2 * h + i];
      bl16(r, ok ? s.off[2 * h + i] + 2u * (uint32_t)k0 : kOOB,
           img + h * 16384 + i * 8192 + wave * 1024);
    }
  } else {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int k = k0 + (tid >> 4) + 32 * i;
      const bool ok = s.ok[h] & (k < K);
      bl16(r, ok ? s.off[h] + (uint32_t)((int64_t)k * ld * 2) : kOOB,
           img + 16384 * h + 8192 * i + 1024 * wave);
    }
  }
}

// Vector-memory instructions a wave issues in one epilogue after its last waited load
// (FMH: 16-row fragments per wave per tile half; 2 FMH fragment rows per wave).
template <int EPI, int FMH = 4>
DFU_DEV int ps_epi_stores(const GemmArgs& p) {
  constexpr bool bf16_out = EPI == DFU_EPI_BF16 || EPI == DFU_EPI_BF16_GELU ||
                            EPI == DFU_EPI_BF16_DGELU || EPI == DFU_EPI_BF16_ADD;
  constexpr int NI = 2 * FMH;
  const int per = bf16_out && p.n8 ? 2 * NI : 4 * NI * (p.n4 ? 1 : 4);
  // dGELU with column sums (p.stats): four more 16-B stores per wave (scalar: sixteen)
  const int cs = EPI == DFU_EPI_BF16_DGELU && p.stats ? (p.n4 ? 4 : 16) : 0;
  const int per16 = p.n8 ? 2 * NI : 4 * NI * (p.n4 ? 1 : 4);  // one 16-bit output
  if constexpr (EPI == DFU_EPI_X3_GELU) return 4 * per16;
  if constexpr (EPI == DFU_EPI_F16_DUAL) return (p.aux_out ? 2 : 1) * per16;
  if constexpr (EPI == DFU_EPI_F16_GELU) return 3 * per16;
  return (EPI == DFU_EPI_BF16_GELU ? 2 * per : per) + cs;
}

// lane holds C[m0 + (i / FMH) * 32 FMH + wr * 16 FMH + (i % FMH) * 16 + (lane&15)]
//              [n0 + (j>>1)*128 + wc*32 + (j&1)*16 + 4*(lane>>4) + r]
// (FMH = 4: the 256-row tile, m0 + (i>>2)*128 + wr*64 + (i&3)*16; FMH = 3: the 192-row tile)
// N4 (p.n4 at compile time): no control flow around the epilogue's loads, so hipcc's wait
// counts stay exact instead of falling back to vmcnt(0) where branches join.
template <int EPI, int FMH, bool N4>
DFU_DEV void ps_epilogue_n(const GemmArgs& p, f32x4 (&acc)[2 * FMH][4], int m0, int n0, int wr,
                           int wc, int lane, int sidx) {
  constexpr bool n4 = N4;
  const int M = p.M, N = p.N;
  const rsrc_t rc = make_rsrc(p.C);
  const rsrc_t ra = make_rsrc(p.aux);
  const rsrc_t ro = make_rsrc(p.aux_out);
  // dGELU + p.stats: per-column sums of the stored (bf16) values over this wave's 128 rows,
  // the bias gradient of the Linear whose output gradient this is (timm Mlp fc1.bias)
  float cs[2][2][4];
#pragma unroll
  for (int hb = 0; hb < 2; ++hb)
#pragma unroll
    for (int jj = 0; jj < 2; ++jj)
#pragma unroll
      for (int r = 0; r < 4; ++r) cs[hb][jj][r] = 0.f;
  float bias[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) bias[j][r] = 0.f;
  constexpr bool kBias = EPI == DFU_EPI_BF16 || EPI == DFU_EPI_BF16_GELU ||
                         EPI == DFU_EPI_F32_RESID || EPI == DFU_EPI_F32 ||
                         EPI == DFU_EPI_X3_GELU || EPI == DFU_EPI_F16_DUAL ||
                         EPI == DFU_EPI_F16_GELU;
  if (kBias && p.bias) {
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
  // The epilogue walks its 4 FMH steps (fragment row i, column half hb).  Epilogues that read
  // (the residual / C for RESID and unsplit ACC, gelu' or the addend for DGELU / ADD) issue a
  // step's loads PD steps ahead, in front of the stores of the steps between: vmcnt retires in
  // issue order, so a load issued after a store would wait for that store too, and the loads of
  // one step after the previous step's stores serialised the epilogue on memory latency (one
  // round trip per step: 19 us of the 89 us fc2 forward, standalone).
  constexpr bool kLdF = EPI == DFU_EPI_F32_RESID || EPI == DFU_EPI_F32_ACC;
  constexpr bool kLdH = EPI == DFU_EPI_BF16_DGELU || EPI == DFU_EPI_BF16_ADD;
  constexpr int NS = 4 * FMH, PD = 2;
  const bool ld_c = EPI == DFU_EPI_F32_RESID || p.slab == nullptr;  // ACC: C += acc unsplit
  u32x4 af[NS][2];
  u32x2 ah[NS][2];
  auto row_of = [&](int i) {
    return m0 + (i / FMH) * 32 * FMH + wr * 16 * FMH + (i % FMH) * 16 + (lane & 15);
  };
  auto load_step = [&](int st) {
    if constexpr (kLdF || kLdH) {
      const int i = st >> 1, hb = st & 1;
      const int m = row_of(i);
      const bool okm = (kAbl & 32) ? (m < 0) : (m < M);
      const int64_t mc = okm ? m : 0;
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const int n = n0 + hb * 128 + wc * 32 + jj * 16 + 4 * (lane >> 4);
        if constexpr (EPI == DFU_EPI_F32_RESID)
          af[st][jj] = ldraw_f32<N4>(ra, mc * p.ldaux + n, okm, n, N);
        else if constexpr (EPI == DFU_EPI_F32_ACC) {
          if (ld_c) af[st][jj] = ldraw_f32<N4>(rc, mc * p.ldc + n, okm, n, N);
        } else
          ah[st][jj] = ldraw_bf16<N4>(ra, mc * p.ldaux + n, okm, n, N);
      }
    }
  };
#pragma unroll
  for (int st = 0; st < PD; ++st) load_step(st);
#pragma unroll
  for (int st = 0; st < NS; ++st) {
    if (st + PD < NS) load_step(st + PD);
    if constexpr (kLdF || kLdH) __builtin_amdgcn_sched_barrier(0);
    const int i = st >> 1, hb = st & 1;
    const int m = row_of(i);
    const bool okm = (kAbl & 32) ? (m < 0) : (m < M);  // ablation 32: every access out of range
    const int64_t mc = okm ? m : 0;
    {
      const int n0w = n0 + hb * 128 + wc * 32;
      float v[2][4];
#pragma unroll
      for (int jj = 0; jj < 2; ++jj)
#pragma unroll
        for (int r = 0; r < 4; ++r) v[jj][r] = acc[i][2 * hb + jj][r] * p.alpha + bias[2 * hb + jj][r];
      if constexpr (EPI == DFU_EPI_BF16) {
        st_row_bf16<2, 0>(rc, mc * p.ldc, okm, n0w, N, p.n8, n4, lane, v);
      } else if constexpr (EPI == DFU_EPI_BF16_GELU) {
        float g[2][4], d[2][4];
#pragma unroll
        for (int jj = 0; jj < 2; ++jj)
#pragma unroll
          for (int r = 0; r < 4; ++r) gelu_and_grad(v[jj][r], g[jj][r], d[jj][r]);
        st_row_bf16<2, 0>(ro, mc * p.ldaux_out, okm, n0w, N, p.n8, n4, lane, d);
        st_row_bf16<2, 0>(rc, mc * p.ldc, okm, n0w, N, p.n8, n4, lane, g);
      } else if constexpr (EPI == DFU_EPI_X3_GELU) {
        // gelu(pre) as the split triple hi = bf16(g), lo = bf16(g - hi): segments hi | lo | hi
        float g[2][4], d[2][4], lo[2][4];
#pragma unroll
        for (int jj = 0; jj < 2; ++jj)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            gelu_and_grad(v[jj][r], g[jj][r], d[jj][r]);
            lo[jj][r] = g[jj][r] - bf2f(f2bf(g[jj][r]));
          }
        st_row_bf16<2, 0>(ro, mc * p.ldaux_out, okm, n0w, N, p.n8, n4, lane, d);
        st_row_bf16<2, 0>(rc, mc * p.ldc, okm, n0w, N, p.n8, n4, lane, g);
        st_row_bf16<2, 0>(rc, mc * p.ldc + N, okm, n0w, N, p.n8, n4, lane, lo);
        st_row_bf16<2, 0>(rc, mc * p.ldc + 2 * N, okm, n0w, N, p.n8, n4, lane, g);
      } else if constexpr (EPI == DFU_EPI_F16_DUAL) {
        // fp16 operand of the next fp16 step, bf16 copy for the backward
        st_row_bf16<2, 0, true>(rc, mc * p.ldc, okm, n0w, N, p.n8, n4, lane, v);
        if (p.aux_out) st_row_bf16<2, 0>(ro, mc * p.ldaux_out, okm, n0w, N, p.n8, n4, lane, v);
      } else if constexpr (EPI == DFU_EPI_F16_GELU) {
        // gelu(pre) as fp16 (fc2's operand, column 0) and bf16 (the backward's h, column N)
        float g[2][4], d[2][4];
#pragma unroll
        for (int jj = 0; jj < 2; ++jj)
#pragma unroll
          for (int r = 0; r < 4; ++r) gelu_and_grad(v[jj][r], g[jj][r], d[jj][r]);
        st_row_bf16<2, 0>(ro, mc * p.ldaux_out, okm, n0w, N, p.n8, n4, lane, d);
        st_row_bf16<2, 0, true>(rc, mc * p.ldc, okm, n0w, N, p.n8, n4, lane, g);
        st_row_bf16<2, 0>(rc, mc * p.ldc + N, okm, n0w, N, p.n8, n4, lane, g);
      } else if constexpr (EPI == DFU_EPI_F32) {
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
          const int n = n0w + jj * 16 + 4 * (lane >> 4);
          st4_f32<0>(rc, mc * p.ldc + n, okm, n, N, n4, v[jj]);
        }
      } else if constexpr (EPI == DFU_EPI_BF16_DGELU || EPI == DFU_EPI_BF16_ADD) {
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
          const int n = n0w + jj * 16 + 4 * (lane >> 4);
          float x[4];
          unpack4(ah[st][jj], x);
#pragma unroll
          for (int r = 0; r < 4; ++r)
            v[jj][r] = EPI == DFU_EPI_BF16_DGELU ? v[jj][r] * x[r] : v[jj][r] + x[r];
        }
        if constexpr (EPI == DFU_EPI_BF16_DGELU) {
#pragma unroll
          for (int jj = 0; jj < 2; ++jj)
#pragma unroll
            for (int r = 0; r < 4; ++r) cs[hb][jj][r] += okm ? bf2f(f2bf(v[jj][r])) : 0.f;
        }
        st_row_bf16<2, 0>(rc, mc * p.ldc, okm, n0w, N, p.n8, n4, lane, v);
      } else if constexpr (EPI == DFU_EPI_F32_ACC) {  // split-K slab, or C += acc unsplit
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
          const int n = n0w + jj * 16 + 4 * (lane >> 4);
          if (p.slab != nullptr) {
            st4_f32(make_rsrc(p.slab), ((int64_t)sidx * M + mc) * N + n, okm, n, N, n4, v[jj]);
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) v[jj][r] += __uint_as_float(af[st][jj][r]);
            st4_f32<0>(rc, mc * p.ldc + n, okm, n, N, n4, v[jj]);
          }
        }
      } else {  // DFU_EPI_F32_RESID
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
          const int n = n0w + jj * 16 + 4 * (lane >> 4);
#pragma unroll
          for (int r = 0; r < 4; ++r) v[jj][r] += __uint_as_float(af[st][jj][r]);
          st4_f32<0>(rc, mc * p.ldc + n, okm, n, N, n4, v[jj]);
        }
      }
    }
  }
  if constexpr (EPI == DFU_EPI_BF16_DGELU) {
    if (p.stats) {  // row (m0 / TM) * 2 + wr of the [2 * tiles_m][N] partial slab
      const rsrc_t rs = make_rsrc(p.stats);
      const int64_t prow = (int64_t)(m0 / (64 * FMH)) * 2 + wr;
      const bool lead = (lane & 15) == 0;
#pragma unroll
      for (int hb = 0; hb < 2; ++hb)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
          float t[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) t[r] = row16_sum(cs[hb][jj][r]);
          const int n = n0 + hb * 128 + wc * 32 + jj * 16 + 4 * (lane >> 4);
          st4_f32(rs, prow * N + n, lead, n, N, n4, t);
        }
    }
  }
}

template <int EPI, int FMH>
DFU_DEV void ps_epilogue(const GemmArgs& p, f32x4 (&acc)[2 * FMH][4], int m0, int n0, int wr,
                         int wc, int lane, int sidx) {
  if (p.n4)
    ps_epilogue_n<EPI, FMH, true>(p, acc, m0, n0, wr, wc, lane, sidx);
  else
    ps_epilogue_n<EPI, FMH, false>(p, acc, m0, n0, wr, wc, lane, sidx);
}

// TMH: rows per tile half (128: the 256 x 256 tile; 96: 192 x 256, K-contiguous A only -- for
// N = 768 outputs, whose 256-row tiling leaves 41 % of the CUs idle: 150 tiles at M = 12608).
// H16: fp16 A and B (v_mfma_f32_16x16x32_f16, the same fragment layout and rate as bf16): the
// "parity" precision mode's ViT forward (dfu_gemm_desc.operand_type 1).
template <int AMODE, int BMODE, int EPI, int TMH = 128, bool H16 = false>
__global__ __launch_bounds__(512) void gemm_ps(const GemmArgs p) {
  constexpr bool AK_ = AMODE == DFU_OPND_KMAJOR;  // A K-contiguous (else MN-major: wgrad)
  constexpr bool BK_ = BMODE == DFU_OPND_KMAJOR;  // B K-contiguous (else MN-major)
  constexpr int FMH = TMH / 32;  // 16-row fragments per wave per half
  constexpr int TMt = 2 * TMH;
  static_assert(TMH == 128 || (TMH == 96 && AK_), "192-row tile: K-contiguous A only");
  __shared__ __attribute__((aligned(16))) char smem[PS_LDS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;
  const int tiles = p.tiles_m * p.tiles_n;
  const int units = tiles * p.split;
  const int nwg = gridDim.x, bid = blockIdx.x;
  int wg = bid;
  if (nwg >= 16) {  // bijective XCD-aware remap: blocks b and b+8 share an XCD
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  // rounds: in complete rounds workgroup b takes unit i*G + wg(b); in the last, partial round
  // unit i*G + b (spread over every XCD)
  const int full = units / nwg;
  const int rounds = full + (bid < units - full * nwg ? 1 : 0);
  if (rounds == 0) return;
  auto unit_at = [&](int i) { return i * nwg + (i < full ? wg : bid); };
  auto unit_geom = [&](int u, int& m0, int& n0, int& kb, int& nk) {
    constexpr int GROUP_M = 4;
    const int s = u / tiles, t = u - s * tiles;
    const int band = GROUP_M * p.tiles_n;
    const int g0 = (t / band) * GROUP_M;
    const int gm = min(GROUP_M, p.tiles_m - g0);
    const int within = t - (t / band) * band;
    m0 = (g0 + within % gm) * TMt;
    n0 = (within / gm) * 256;
    kb = s * p.kt_per_split;
    nk = min(p.ktiles, kb + p.kt_per_split) - kb;
  };
  int total = 0;
  for (int i = 0; i < rounds; ++i) {
    int a_, b_, c_, nk_;
    unit_geom(unit_at(i), a_, b_, c_, nk_);
    total += nk_;
  }
  PsSrc<AK_> sa;
  PsSrc<BK_> sb;
  auto src_init = [&](int m0_, int n0_) {
    ps_src_init<AK_>(sa, p.lda, m0_, AK_ ? p.M : p.m_ld_bound, tid);
    ps_src_init<BK_>(sb, p.ldb, n0_, BK_ ? p.N : p.n_ld_bound, tid);
  };
  const rsrc_t ra_ = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(p.A), (short)0,
                                                        p.a_bytes, 0x00020000);
  const rsrc_t rb_ = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(p.B), (short)0,
                                                        p.b_bytes, 0x00020000);
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  auto issue_a = [&](int k0_, int h, char* img) {
    ps_issue<AK_, TMt / 64>(sa, ra_, p.lda, k0_, p.K, h, img, tid, wave_u);
  };
  auto issue_b = [&](int k0_, int h, char* img) {
    ps_issue<BK_>(sb, rb_, p.ldb, k0_, p.K, h, img, tid, wave_u);
  };

  // issue cursor (the K-step whose DMA goes out next) and compute cursor
  int iu = 0, ik = 0, im0, in0, ikb, ink;
  unit_geom(unit_at(0), im0, in0, ikb, ink);
  src_init(im0, in0);
  int ci = 0, ck = 0, cm0, cn0, ckb, cnk;
  int cu = unit_at(0);
  unit_geom(cu, cm0, cn0, ckb, cnk);
  auto advance_issue = [&]() {
    if (++ik == ink) {
      ik = 0;
      if (++iu < rounds) {
        unit_geom(unit_at(iu), im0, in0, ikb, ink);
        src_init(im0, in0);
      }
    }
  };

  f32x4 acc[2 * FMH][4];
#pragma unroll
  for (int i = 0; i < 2 * FMH; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // prologue: K-step 0 into buffer 0, in first-use order (A-top, B-left, B-right, A-bottom)
  {
    const int k0 = (ikb + ik) * BK;
    issue_a(k0, 0, smem);
    issue_b(k0, 0, smem + PS_IMG);
    issue_b(k0, 1, smem + PS_IMG);
    issue_a(k0, 1, smem);
    if constexpr ((kAbl & (4 | 64 | 256)) != 0) {  // ablated DMA: both buffers hold K-step 0
      issue_a(k0, 0, smem + PS_BUF);
      issue_b(k0, 0, smem + PS_BUF + PS_IMG);
      issue_b(k0, 1, smem + PS_BUF + PS_IMG);
      issue_a(k0, 1, smem + PS_BUF);
    }
    advance_issue();
  }
  constexpr bool kDmaA = (kAbl & (4 | 256)) == 0, kDmaB = (kAbl & (4 | 64)) == 0;
  bool rd_on = true;  // read ablations: fragments read in K-step 0 only
  const int E = (kAbl & 1) ? 0 : ps_epi_stores<EPI, FMH>(p);
  bool epi_last = false;  // an epilogue ran at the end of the previous K-step
  // Fragment registers hold one A half (fa) and one B half (fb); each phase's MFMAs run one
  // k-half (ks) at a time, and the reads the NEXT group needs go out as soon as the group before
  // it has consumed the registers they overwrite, so every read has a group of 8 MFMAs (this
  // wave's and its SIMD partner's) to land under instead of stalling the pipe (the compiler's
  // lgkmcnt waits are the exact ones for K-contiguous reads; MN-major ones are asm, retired by an
  // lgkmcnt(0) in front of each group).
  // (Measured and dropped, round 3: both B halves kept in registers, the next K-step's barrier
  // moved in front of the last MFMA group, the DMA spread over all four groups, the two wave rows
  // issuing their DMA at different points, s_setprio around the groups, per-XCD runs for the
  // partial round -- all within noise.  Round 5: the operand tiles through VGPRs
  // (buffer_load_dwordx4, then ds_write_b128 two phases later, same LDS images) instead of
  // LDS-DMA: 10-13 % slower on 4096^3 and the ViT shapes, same box.  And the ping-pong schedule
  // of cdna_hip_programming.md's 256^2 template on this tile (wave row 1 one barrier behind row
  // 0, two barriers per quadrant phase, MFMAs at priority 1, both B halves in registers, one
  // half-tile of DMA per phase): level at 4096^3 and fc2, 4-7 % slower at K = 768.  And the
  // DMA issued by wave row 0 alone (its pieces and row 1's, so one wave per SIMD keeps issuing
  // MFMAs): level everywhere.)
  bf16x8 fa[FMH][2], fb[2][2];
  auto rd_a = [&](const char* la, int h, int ks) {
    if constexpr ((kAbl & (8 | 512)) != 0)
      if (!rd_on) return;
#pragma unroll
    for (int i = 0; i < FMH; ++i)
      fa[i][ks] = read_frag<AK_>(la, h * TMH + wr * (TMH / 2) + i * 16, ks, lane);
  };
  auto rd_b = [&](const char* lb, int h, int ks) {
    if constexpr ((kAbl & (8 | 128)) != 0)
      if (!rd_on) return;
#pragma unroll
    for (int j = 0; j < 2; ++j)
      fb[j][ks] = read_frag<BK_>(lb, h * 128 + wc * 32 + j * 16, ks, lane);
  };
  // the first group's reads of a K-step (A-top, B-left, both k-halves)
  auto rd_first = [&](const char* la) {
    rd_a(la, 0, 0);
    rd_b(la + PS_IMG, 0, 0);
    rd_a(la, 0, 1);
    rd_b(la + PS_IMG, 0, 1);
  };
  auto mf = [&](int ha, int hb, int ks) {
    if constexpr ((kAbl & 2) != 0) {
      __builtin_amdgcn_sched_barrier(0);
      return;
    }
    if constexpr (!AK_ || !BK_) {  // asm (MN-major) fragment reads: retired before use
      lds_reads_retired();
#pragma unroll
      for (int i = 0; i < FMH; ++i) pin(fa[i][ks]);
#pragma unroll
      for (int j = 0; j < 2; ++j) pin(fb[j][ks]);
    }
#pragma unroll
    for (int i = 0; i < FMH; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        if constexpr (H16)
          acc[ha * FMH + i][hb * 2 + j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(
              __builtin_bit_cast(f16x8, fb[j][ks]),
              __builtin_bit_cast(f16x8, fa[i][ks]), acc[ha * FMH + i][hb * 2 + j], 0, 0, 0);
        else
          acc[ha * FMH + i][hb * 2 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              fb[j][ks], fa[i][ks], acc[ha * FMH + i][hb * 2 + j], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  };
  for (int g = 0; g < total; ++g) {
    const char* la = smem + (g & 1) * PS_BUF;
    const char* lb = la + PS_IMG;
    char* na = smem + ((g & 1) ^ 1) * PS_BUF;
    char* nb = na + PS_IMG;
    const bool nxt = g + 1 < total;
    const int k1 = (ikb + ik) * BK;  // the next K-step (issue cursor)
    // this K-step's DMA landed (younger: only the previous epilogue's stores), then published
    if (epi_last)
      wait_vm_le<63>(E);
    else
      wait_vmcnt<0>();
    if constexpr (!(kAbl & 16)) __builtin_amdgcn_s_barrier();
    if constexpr ((kAbl & (8 | 128 | 512)) != 0) rd_on = g == 0;
    rd_first(la);
    if (nxt) {
      if (kDmaA) issue_a(k1, 0, na);
      if (kDmaB) issue_b(k1, 0, nb);
    }
    __builtin_amdgcn_sched_barrier(0);
    mf(0, 0, 0);   // A-top x B-left
    rd_b(lb, 1, 0);
    mf(0, 0, 1);
    rd_b(lb, 1, 1);
    if (nxt) {
      if (kDmaB) issue_b(k1, 1, nb);
      if (kDmaA) issue_a(k1, 1, na);
      advance_issue();
    }
    __builtin_amdgcn_sched_barrier(0);
    mf(0, 1, 0);   // A-top x B-right
    rd_a(la, 1, 0);
    mf(0, 1, 1);
    rd_a(la, 1, 1);
    mf(1, 1, 0);   // A-bottom x B-right
    rd_b(lb, 0, 0);
    mf(1, 1, 1);
    rd_b(lb, 0, 1);
    mf(1, 0, 0);   // A-bottom x B-left
    mf(1, 0, 1);
    epi_last = false;
    if (++ck == cnk) {
      if constexpr (!(kAbl & 1)) {
        ps_epilogue<EPI, FMH>(p, acc, cm0, cn0, wr, wc, lane, cu / tiles);
      } else {  // keep the accumulators (and so every MFMA) alive without storing them
#pragma unroll
        for (int i = 0; i < 2 * FMH; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) asm volatile("" ::"v"(acc[i][j]));
      }
#pragma unroll
      for (int i = 0; i < 2 * FMH; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
      epi_last = true;
      ck = 0;
      if (++ci < rounds) {
        cu = unit_at(ci);
        unit_geom(cu, cm0, cn0, ckb, cnk);
      }
    }
  }
}

}  // namespace

#define PS(A, B, E) {A, B, E, T256x256ps, &gemm_ps<A, B, E>, PS_LDS, 512}
#define PSH(E)                                                                            \
  {DFU_OPND_KMAJOR, DFU_OPND_KMAJOR, (E) | kF16Key, T256x256ps,                           \
   &gemm_ps<DFU_OPND_KMAJOR, DFU_OPND_KMAJOR, E, 128, true>, PS_LDS, 512}
const Entry kTable256x256ps[] = {
    PS(DFU_OPND_KMAJOR, DFU_OPND_KMAJOR, DFU_EPI_BF16),
    PS(DFU_OPND_KMAJOR, DFU_OPND_KMAJOR, DFU_EPI_BF16_GELU),
    PS(DFU_OPND_KMAJOR, DFU_OPND_KMAJOR, DFU_EPI_F32_RESID),
    PS(DFU_OPND_KMAJOR, DFU_OPND_KMAJOR, DFU_EPI_F32),      // bf16x3 forward (qkv)
    PS(DFU_OPND_KMAJOR, DFU_OPND_KMAJOR, DFU_EPI_X3_GELU),  // bf16x3 forward (fc1 + GELU)
    PS(DFU_OPND_KMAJOR, DFU_OPND_KMAJOR, DFU_EPI_BF16_DGELU),  // dgrads on a transposed weight
    PS(DFU_OPND_KMAJOR, DFU_OPND_MNMAJOR, DFU_EPI_BF16),
    PS(DFU_OPND_KMAJOR, DFU_OPND_MNMAJOR, DFU_EPI_BF16_DGELU),
    PS(DFU_OPND_KMAJOR, DFU_OPND_MNMAJOR, DFU_EPI_BF16_ADD),
    PS(DFU_OPND_MNMAJOR, DFU_OPND_MNMAJOR, DFU_EPI_F32_ACC),  // weight gradients (split-K slabs)
    // fp16 operands (epilogue key | kF16Key): the "parity" mode's ViT forward
    PSH(DFU_EPI_F32),        // qkv (fp32 out: unused by the product path, tests)
    PSH(DFU_EPI_F32_RESID),  // proj / fc2 with the fp32 residual
    PSH(DFU_EPI_F16_DUAL),   // qkv: fp16 for the attention, bf16 for the backward
    PSH(DFU_EPI_F16_GELU),   // fc1 + GELU
};
#undef PS
#undef PSH
const int kTable256x256psN = sizeof(kTable256x256ps) / sizeof(Entry);

// 192 x 256 (K-contiguous A): the N = 768 ViT GEMMs (forward proj / fc2 with the fp32 residual,
// their bf16x3 forms, and the input gradients to 768 on the transposed weights)
#define PS192(A, B, E) {A, B, E, T192x256ps, &gemm_ps<A, B, E, 96>, PS_LDS, 512}
const Entry kTable192x256ps[] = {
    PS192(DFU_OPND_KMAJOR, DFU_OPND_KMAJOR, DFU_EPI_BF16),
    PS192(DFU_OPND_KMAJOR, DFU_OPND_KMAJOR, DFU_EPI_F32_RESID),
    PS192(DFU_OPND_KMAJOR, DFU_OPND_KMAJOR, DFU_EPI_F32),
    PS192(DFU_OPND_KMAJOR, DFU_OPND_MNMAJOR, DFU_EPI_BF16),
    PS192(DFU_OPND_KMAJOR, DFU_OPND_MNMAJOR, DFU_EPI_BF16_ADD),
    {DFU_OPND_KMAJOR, DFU_OPND_KMAJOR, DFU_EPI_F32_RESID | kF16Key, T192x256ps,
     &gemm_ps<DFU_OPND_KMAJOR, DFU_OPND_KMAJOR, DFU_EPI_F32_RESID, 96, true>, PS_LDS, 512},
};
#undef PS192
const int kTable192x256psN = sizeof(kTable192x256ps) / sizeof(Entry);

}  // namespace dfu
