// Host dispatch for the MFMA GEMM template (include/dfu_hip.h: dfu_gemm): picks the tile
// shape and split-K by a wave-quantisation cost model (one 512-thread workgroup per CU),
// launches the kernel, and for split-K with a caller workspace reduces the fp32 slabs.
#include <math.h>
#include <stdlib.h>

#include <type_traits>

#include "gemm_table.h"

using namespace dfu;

namespace {

constexpr int kCUs = 256;
constexpr int kTM[NTILES] = {128, 256, 128, 256, 128, 128, 256, 256, 192, 256, 128};
constexpr int kTN[NTILES] = {128, 128, 256, 256, 128, 128, 256, 256, 256, 64, 64};
constexpr int kOcc[NTILES] = {1, 1, 1, 1, 2, 2, 1, 1, 1, 1, 2};  // workgroups per CU
// the tile whose fitted step time a variant borrows (the persistent phased 256x256: the phased)
constexpr int kBase[NTILES] = {0, 1, 2, 3, 4, 5, 6, 6, 6, 9, 10};
constexpr bool kTailOK[NTILES] = {true, false, false, false, true, false, false, false, false,
                                  false, false};
// Wave-quantisation cost model: a launch takes ceil(tiles * splits / 256) rounds (one 512-thread
// workgroup per CU), each costing kRoundUs (prologue fill + epilogue) + k-steps * kStepUs.
// Fitted on MI355X to tools/gemm_bench.py --sweep (ViT qkv K=768 vs fc2 K=3072 forward rows,
// r01): 128x128 0.57 us/step + 4.8 us/round ... 256x256 1.41 us/step + 13.9 us/round, i.e.
// 256x256 moves 1.62x more MFMA work per microsecond than 128x128.
// The 2-per-CU 128x128 variant: two co-resident workgroups share the MFMA pipe (step cost per
// workgroup ~doubles) but hide each other's fill and epilogue.
// (the phased 256x256 kernels are priced high: only the offline-tuned table selects them)
// (the 64-column tiles are priced high too: only tuned plans select them)
constexpr double kStepUs[NTILES] = {0.57, 0.89, 0.90, 1.41, 0.70, 0.65, 3.0, 3.0, 3.0, 3.0, 3.0};
constexpr double kRoundUs[NTILES] = {4.8, 8.3, 7.4, 13.9, 6.1, 6.1, 20.0, 20.0, 20.0, 20.0, 20.0};
constexpr double kSlabGBs = 5000.0;  // split-K: slab write + reduce (read slabs, RMW C)
constexpr double kReduceLaunchUs = 2.0;
// Persistent schedule (gemm_kernel.h): a workgroup owning several work units pays one
// prologue fill for all of them plus, per unit, the epilogue time its MFMAs do not hide.
constexpr double kUnitUs[NTILES] = {1.0, 1.8, 1.7, 3.0, 1.2, 1.2, 3.0, 3.0, 3.0, 3.0, 3.0};
// Persistent launches (at most one wave of workgroups, each walking its work units) for the
// generic tiles (g_persistent) and the persistent phased 256-wide tiles (g_persistent_ps);
// otherwise one workgroup per unit, which the hardware dispatcher hands to CUs as they free up.
// Round 6 (final tree, same box, three rounds): the generic tiles one workgroup per unit ran the
// fusion step 0.4 % faster and the GEMM replay 0.7 %; the phased tiles level either way in the
// step, persistent faster alone.  dfu_gemm_set_persistent (bit 0 generic, bit 1 phased); env
// DFU_GEMM_PERSISTENT / DFU_GEMM_PERSISTENT_PS: A/B.
int g_persistent = getenv("DFU_GEMM_PERSISTENT") ? atoi(getenv("DFU_GEMM_PERSISTENT")) : 0;
int g_persistent_ps = getenv("DFU_GEMM_PERSISTENT_PS") ? atoi(getenv("DFU_GEMM_PERSISTENT_PS")) : 1;
// dfu_gemm_set_inkernel_reduce (measured slower: off); env DFU_GEMM_INKERNEL_REDUCE: A/B
int g_inkernel_reduce =
    getenv("DFU_GEMM_INKERNEL_REDUCE") ? atoi(getenv("DFU_GEMM_INKERNEL_REDUCE")) : 0;
// the wave-split reduce for small planes (DFU_GEMM_WIDE_REDUCE=0 disables it: A/B timing)
const int g_wide_reduce = getenv("DFU_GEMM_WIDE_REDUCE") ? atoi(getenv("DFU_GEMM_WIDE_REDUCE")) : 1;
// dfu_gemm_set_tail_split; env DFU_GEMM_TAIL_SPLIT: A/B
int g_tail_split = getenv("DFU_GEMM_TAIL_SPLIT") ? atoi(getenv("DFU_GEMM_TAIL_SPLIT")) : 1;

const Entry* find_entry(int a, int b, int e, int tile) {
  const Entry* tabs[NTILES] = {kTable128x128, kTable256x128, kTable128x256, kTable256x256,
                               kTable128x128o2, kTable128x128w4, kTable256x256p8,
                               kTable256x256ps, kTable192x256ps, kTable256x64,
                               kTable128x64o2};
  const int ns[NTILES] = {kTable128x128N, kTable256x128N, kTable128x256N, kTable256x256N,
                          kTable128x128o2N, kTable128x128w4N, kTable256x256p8N,
                          kTable256x256psN, kTable192x256psN, kTable256x64N,
                          kTable128x64o2N};
  for (int i = 0; i < ns[tile]; ++i) {
    const Entry& en = tabs[tile][i];
    if (en.a == a && en.b == b && en.e == e) return &en;
  }
  return nullptr;
}

inline int round8(int x) { return (x + 7) & ~7; }
inline int cdiv(int a, int b) { return (a + b - 1) / b; }

struct Plan {
  const Entry* entry = nullptr;
  int tile = 0, split = 1;
  double cost = 1e30;
};

// Offline-tuned plans (tools/gemm_tune.py on MI355X: every distinct GEMM of the training step,
// all tiles x split-K candidates timed, fastest kept) take precedence over the cost model.
struct TunedPlan {
  int a, b, e, M, N, K, cn, ch, cw, cc, ck, cr, cs, cstride, cpad;
  int tile, split;  // tile id 1..NTILES, split-K (1 = none)
};
const TunedPlan kTuned[] = {
#include "gemm_tuned.inc"
    {-1, -1, -1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}};

// the dispatch key of a descriptor's kernel: its epilogue, | kF16Key for fp16 operands,
// | kX3Key for interleaved bf16x3 pairs (also the tuned-plan table's epilogue field)
inline int epi_key(const dfu_gemm_desc* d) {
  return d->epilogue | (d->operand_type == 1 ? kF16Key : 0) | (d->x3_pairs ? kX3Key : 0);
}

// An fp16-operand descriptor takes its own entry (epilogue | kF16Key) if tuned, else the bf16
// entry of the same shape.
const TunedPlan* find_tuned_key(const dfu_gemm_desc* d, int epi) {
  const bool conv = d->a_mode >= DFU_OPND_CONV_FWD || d->b_mode >= DFU_OPND_CONV_FWD;
  for (const TunedPlan& t : kTuned) {
    if (t.a != d->a_mode || t.b != d->b_mode || t.e != epi || t.M != d->M ||
        t.N != d->N || t.K != d->K)
      continue;
    if (conv && (t.cn != d->conv_n || t.ch != d->conv_h || t.cw != d->conv_w ||
                 t.cc != d->conv_c || t.ck != d->conv_k || t.cr != d->conv_r ||
                 t.cs != d->conv_s || t.cstride != d->conv_stride || t.cpad != d->conv_pad))
      continue;
    return &t;
  }
  return nullptr;
}

const TunedPlan* find_tuned(const dfu_gemm_desc* d) {
  const int epi = d->epilogue | (d->x3_pairs ? kX3Key : 0);
#ifndef DFU_NO_F16_TUNED  // (A/B builds only: the fp16 GEMMs on the bf16 shapes' plans)
  if (d->operand_type == 1)
    if (const TunedPlan* t = find_tuned_key(d, epi | kF16Key)) return t;
#endif
  return find_tuned_key(d, epi);
}

Plan plan_gemm(const dfu_gemm_desc* d) {
  const bool acc_epi = d->epilogue == DFU_EPI_F32_ACC;
  if (d->tile == 0 && d->split_k == 0) {
    if (const TunedPlan* tp = find_tuned(d)) {
      Plan pl;
      pl.tile = tp->tile - 1;
      pl.entry = find_entry(d->a_mode, d->b_mode, epi_key(d), pl.tile);
      pl.split = acc_epi ? tp->split : 1;
      pl.cost = 0.0;
      if (pl.entry) return pl;
    }
  }
  const int ktiles = cdiv(d->K, BK);
  Plan best;
  for (int t = 0; t < NTILES; ++t) {
    if (d->tile > 0 && d->tile - 1 != t) continue;
    const Entry* en = find_entry(d->a_mode, d->b_mode, epi_key(d), t);
    if (!en) continue;
    const int tiles = cdiv(d->M, kTM[t]) * cdiv(d->N, kTN[t]);
    int s_lo = 1, s_hi = 1;
    if (acc_epi) {
      if (d->split_k > 0) s_lo = s_hi = d->split_k;
      else s_hi = ktiles < 256 ? ktiles : 256;  // long-K weight gradients: up to 1 split per CU
    }
    for (int s = s_lo; s <= s_hi; ++s) {
      const int kps = cdiv(ktiles, s);
      const int se = cdiv(ktiles, kps);
      if (se != s && s != s_lo) continue;
      const int slots = kCUs * kOcc[t];
      const int rounds = cdiv(tiles * se, slots);
      double cost = (g_persistent && tiles * se > slots)
                        ? kRoundUs[t] + rounds * (kps * kStepUs[t] + kUnitUs[t])
                        : rounds * (kRoundUs[t] + kps * kStepUs[t]);
      if (se > 1)
        cost += kReduceLaunchUs + 4.0 * (se + 2) * (double)d->M * d->N / (kSlabGBs * 1e3);
      if (cost < best.cost) {
        best.cost = cost;
        best.entry = en;
        best.tile = t;
        best.split = se;
      }
    }
  }
  return best;
}

__global__ void k_splitk_reduce(const float* __restrict__ slab, int splits, int M, int N,
                                float* __restrict__ C, int64_t ldc) {
  const int64_t n4 = (int64_t)M * N / 4;
  const int64_t plane = (int64_t)M * N;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x) {
    f32x4 s = ((const f32x4*)slab)[i];
    for (int k = 1; k < splits; ++k) {
      const f32x4 v = *(const f32x4*)(slab + k * plane + 4 * i);
      s[0] += v[0]; s[1] += v[1]; s[2] += v[2]; s[3] += v[3];
    }
    const int64_t e = 4 * i;
    const int64_t m = e / N;
    const int n = (int)(e - m * N);
    float* c = C + m * ldc + n;  // N % 4 == 0, ldc % 4 == 0, C 16-B aligned (host-checked)
    f32x4 cv = *(f32x4*)c;
    *(f32x4*)c = (f32x4){cv[0] + s[0], cv[1] + s[1], cv[2] + s[2], cv[3] + s[3]};
  }
}

// Any N (e.g. the stem's 7x7x3 = 147 weight columns): one thread per (row, column); rows on
// blockIdx.y, so no per-element 64-bit division.
__global__ void k_splitk_reduce_scalar(const float* __restrict__ slab, int splits, int M, int N,
                                       float* __restrict__ C, int64_t ldc) {
  const int64_t plane = (int64_t)M * N;
  for (int m = blockIdx.y; m < M; m += gridDim.y)
    for (int n = blockIdx.x * blockDim.x + threadIdx.x; n < N; n += gridDim.x * blockDim.x) {
      const int64_t i = (int64_t)m * N + n;
      float s = 0.f;
      for (int k = 0; k < splits; ++k) s += slab[k * plane + i];
      C[(int64_t)m * ldc + n] += s;
    }
}

// Small planes with many splits (the ResNet weight gradients: 64x64 .. 512x512 tiles of
// K = 12544 .. 802816 split 16-256 ways): one lane per element (f32x4 when VEC), the waves of a
// block split the slabs between them (wave w sums slabs w, w + nw, ...) and combine in wave
// order through LDS — a fixed summation order, so still bitwise reproducible.
template <bool VEC>
__global__ void __launch_bounds__(1024) k_splitk_reduce_wide(const float* __restrict__ slab,
                                                             int splits, int M, int N,
                                                             float* __restrict__ C, int64_t ldc) {
  using V = typename std::conditional<VEC, f32x4, float>::type;
  __shared__ V red[16][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int64_t plane = (int64_t)M * N;
  const int64_t units = VEC ? plane / 4 : plane;
  const int64_t e = (int64_t)blockIdx.x * 64 + lane;
  V s = {};
  if (e < units) {
    const V* p = (const V*)slab + e;
    const int64_t step = VEC ? plane / 4 : plane;
#pragma unroll 4
    for (int k = w; k < splits; k += nw) s += p[k * step];
  }
  red[w][lane] = s;
  __syncthreads();
  if (w != 0 || e >= units) return;
  for (int j = 1; j < nw; ++j) s += red[j][lane];
  if (VEC) {
    const int64_t m = 4 * e / N;
    const int n = (int)(4 * e - m * N);
    V* c = (V*)(C + m * ldc + n);  // N % 4 == 0, ldc % 4 == 0, C 16-B aligned (host-checked)
    *c += s;
  } else {
    const int64_t m = e / N;
    C[m * ldc + (e - m * N)] += *(const float*)&s;
  }
}

// Tail split (GemmArgs::tail_*) for an unsplit launch of `tiles` tiles over `slots`
// workgroup slots: the R = tiles mod slots tiles of the last, partial round are each split
// S ways along K, S = as many as the idle slots allow (<= 8, >= 2 K-steps per split).
struct Tail {
  int full = 0, r = 0, s = 0, kps = 0;
  int64_t bytes = 0;  // fp32 slab workspace
};

// The split count maximises the K-step time it takes off the tail round minus the slab hand-off,
// which all the tail workgroups do at once at the end of the launch: each stores its fp32 tile
// and the last of each tile reads them all back, ~2 x R x S x TM x TN x 4 bytes at ~5 TB/s, plus
// ~3 us (fitted on MI355X with tools/gemm_step_profile.py --tail-ab: K >= ~2304 launches gain
// 7-40 us, K <= 1024 ones would lose up to 11).  Used only if the net gain is positive.
Tail tail_plan(int tiles, int slots, int ktiles, int tm, int tn, double step_us) {
  Tail best;
  if (!g_tail_split) return best;
  const int R = tiles % slots;
  if (R == 0) return best;
  int smax = slots / R;
  if (smax > 8) smax = 8;
  if (smax > ktiles / 2) smax = ktiles / 2;
  double best_gain = 0.0;
  for (int S = 2; S <= smax; ++S) {
    const int kps = cdiv(ktiles, S);
    const int se = cdiv(ktiles, kps);
    if (se != S) continue;
    const double bytes = (double)R * S * tm * tn * 4;
    const double gain = (ktiles - kps) * step_us - (3.0 + 2.0 * bytes / 5e6);
    if (gain > best_gain) {
      best_gain = gain;
      best.s = S;
      best.kps = kps;
    }
  }
  if (best.s < 2) return Tail();
  best.full = tiles - R;
  best.r = R;
  best.bytes = (int64_t)best.s * R * tm * tn * 4;
  return best;
}

Tail tail_for(const dfu_gemm_desc* d, const Plan& pl) {
  if (!pl.entry || d->epilogue == DFU_EPI_F32_ACC || !kTailOK[pl.tile]) return Tail();
  const int tiles = cdiv(d->M, kTM[pl.tile]) * cdiv(d->N, kTN[pl.tile]);
  return tail_plan(tiles, kCUs * kOcc[pl.tile], cdiv(d->K, BK), kTM[pl.tile], kTN[pl.tile],
                   kStepUs[kBase[pl.tile]]);
}

}  // namespace

extern "C" int dfu_gemm_stats_tiles(int32_t M) { return (M + 127) / 128; }

extern "C" int64_t dfu_gemm_workspace_bytes(const dfu_gemm_desc* d) {
  if (!d) return 0;
  const Plan pl = plan_gemm(d);
  if (!pl.entry) return 0;
  if (d->epilogue != DFU_EPI_F32_ACC) {
    // tail-split slabs (at most one split per workgroup slot); a strided dgrad's phase launches
    // re-plan their own tiles: the bound over every tile shape
    if (!g_tail_split) return 0;
    if (d->a_mode == DFU_OPND_CONV_DGRAD && d->conv_stride > 1) {
      int64_t b = 0;
      for (int t = 0; t < NTILES; ++t) {
        const int64_t bt = kTailOK[t] ? (int64_t)kCUs * kOcc[t] * kTM[t] * kTN[t] * 4 : 0;
        if (bt > b) b = bt;
      }
      return b;
    }
    return tail_for(d, pl).bytes;
  }
  return pl.split > 1 ? (int64_t)pl.split * d->M * d->N * 4 : 0;
}

extern "C" int dfu_gemm_plan(const dfu_gemm_desc* d, int32_t* tile, int32_t* split_k) {
  DFU_CHECK_ARG(d != nullptr && tile != nullptr && split_k != nullptr, "dfu_gemm_plan: null");
  DFU_CHECK_ARG(d->operand_type == 0 || d->operand_type == 1, "dfu_gemm: bad operand_type %d",
                d->operand_type);
  if (d->epilogue == DFU_EPI_F16_DUAL || d->epilogue == DFU_EPI_F16_GELU) {
    DFU_CHECK_ARG(d->operand_type == 1, "dfu_gemm: the F16 epilogues need operand_type 1");
    DFU_CHECK_ARG((d->epilogue == DFU_EPI_F16_DUAL && d->aux_out == nullptr) ||
                      (d->aux_out != nullptr && d->ldaux_out >= d->N),
                  "dfu_gemm: F16_GELU needs aux_out (F16_DUAL: NULL or ldaux_out >= N)");
    DFU_CHECK_ARG(d->epilogue != DFU_EPI_F16_GELU || d->ldc >= 2LL * d->N,
                  "dfu_gemm: F16_GELU needs ldc >= 2N");
  }
  const Plan pl = plan_gemm(d);
  if (!pl.entry) {
    dfu_set_error("dfu_gemm_plan: unsupported combination");
    return DFU_E_UNSUPPORTED;
  }
  *tile = pl.tile + 1;
  *split_k = pl.split;
  return DFU_OK;
}

extern "C" int dfu_gemm_set_persistent(int32_t mode) {
  const int old = (g_persistent ? 1 : 0) | (g_persistent_ps ? 2 : 0);
  g_persistent = (mode & 1) != 0;
  g_persistent_ps = (mode & 2) != 0;
  return old;
}

extern "C" int dfu_gemm_set_tail_split(int32_t enable) {
  const int old = g_tail_split;
  g_tail_split = enable != 0;
  return old;
}

extern "C" int dfu_gemm_set_inkernel_reduce(int32_t enable) {
  const int old = g_inkernel_reduce;
  g_inkernel_reduce = enable != 0;
  return old;
}

namespace {

// One stride phase of a strided dgrad (see GemmArgs::ph_*): rows h = h'*st + ph, taps
// r = r0 + st*ri; qh = (ph + pad - r0) / st is the phase's stride-1 "padding".
struct Phase {
  int ph, pw, r0, s0, nr, ns, qh, qw, Hs, Ws;
};

Phase make_phase(const dfu_gemm_desc* d, int ph, int pw) {
  const int st = d->conv_stride, pad = d->conv_pad;
  Phase f;
  f.ph = ph;
  f.pw = pw;
  f.r0 = (ph + pad) % st;
  f.s0 = (pw + pad) % st;
  f.nr = f.r0 < d->conv_r ? (d->conv_r - f.r0 + st - 1) / st : 0;
  f.ns = f.s0 < d->conv_s ? (d->conv_s - f.s0 + st - 1) / st : 0;
  f.qh = (ph + pad - f.r0) / st;
  f.qw = (pw + pad - f.s0) / st;
  f.Hs = ph < d->conv_h ? (d->conv_h - ph + st - 1) / st : 0;
  f.Ws = pw < d->conv_w ? (d->conv_w - pw + st - 1) / st : 0;
  return f;
}

// dX rows of a phase without live taps: 0 (BF16) or the addend (BF16_ADD).
__global__ void k_phase_fill(bf16_t* __restrict__ C, int64_t ldc, const bf16_t* __restrict__ aux,
                             int64_t ldaux, int B, int Hs, int Ws, int H, int W, int st, int ph,
                             int pw, int N) {
  const int64_t rows = (int64_t)B * Hs * Ws;
  const int nv = N / 8;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < rows * nv;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = i / nv;
    const int c = (int)(i - m * nv) * 8;
    const int b = (int)(m / ((int64_t)Hs * Ws));
    const int rem = (int)(m - (int64_t)b * Hs * Ws);
    const int h = rem / Ws, w = rem - (rem / Ws) * Ws;
    const int64_t row = ((int64_t)b * H + h * st + ph) * W + w * st + pw;
    const u32x4 v = aux ? *(const u32x4*)(aux + row * ldaux + c) : (u32x4){0u, 0u, 0u, 0u};
    *(u32x4*)(C + row * ldc + c) = v;
  }
}

int launch(const dfu_gemm_desc* d, const Plan& pl, const Phase* ph, hipStream_t s);

}  // namespace

extern "C" int dfu_gemm(const dfu_gemm_desc* d, void* stream) {
  DFU_CHECK_ARG(d != nullptr, "dfu_gemm: null descriptor");
  DFU_CHECK_ARG(d->M > 0 && d->N > 0 && d->K > 0, "dfu_gemm: bad shape M=%d N=%d K=%d", d->M,
                d->N, d->K);
  const bool a_kc = d->a_mode == DFU_OPND_KMAJOR || d->a_mode == DFU_OPND_CONV_FWD ||
                    d->a_mode == DFU_OPND_CONV_DGRAD;
  const bool b_kc = d->b_mode == DFU_OPND_KMAJOR;
  DFU_CHECK_ARG(!(a_kc || b_kc) || d->K % 8 == 0,
                "dfu_gemm: K=%d must be a multiple of 8 for K-contiguous operands", d->K);
  DFU_CHECK_ARG(d->tile >= 0 && d->tile <= NTILES, "dfu_gemm: bad tile hint %d", d->tile);
  const bool acc_epi = d->epilogue == DFU_EPI_F32_ACC;
  DFU_CHECK_ARG(d->split_k >= 0, "dfu_gemm: split_k must be >= 0 (0 = auto)");
  DFU_CHECK_ARG(d->split_k <= 1 || acc_epi, "dfu_gemm: split_k > 1 needs the F32_ACC epilogue");
  DFU_CHECK_ARG(d->operand_type == 0 || d->operand_type == 1, "dfu_gemm: bad operand_type %d",
                d->operand_type);
  if (d->epilogue == DFU_EPI_F16_DUAL || d->epilogue == DFU_EPI_F16_GELU) {
    DFU_CHECK_ARG(d->operand_type == 1, "dfu_gemm: the F16 epilogues need operand_type 1");
    DFU_CHECK_ARG((d->epilogue == DFU_EPI_F16_DUAL && d->aux_out == nullptr) ||
                      (d->aux_out != nullptr && d->ldaux_out >= d->N),
                  "dfu_gemm: F16_GELU needs aux_out (F16_DUAL: NULL or ldaux_out >= N)");
    DFU_CHECK_ARG(d->epilogue != DFU_EPI_F16_GELU || d->ldc >= 2LL * d->N,
                  "dfu_gemm: F16_GELU needs ldc >= 2N");
  }
  const Plan pl = plan_gemm(d);
  if (!pl.entry) {
    dfu_set_error("dfu_gemm: unsupported combination a_mode=%d b_mode=%d epilogue=%d tile=%d "
                  "operand_type=%d", d->a_mode, d->b_mode, d->epilogue, d->tile,
                  d->operand_type);
    return DFU_E_UNSUPPORTED;
  }
  if (d->epilogue == DFU_EPI_BF16_DGELU && d->stats != nullptr && pl.tile != T256x256ps) {
    // the dGELU column sums exist in the persistent phased 256x256 epilogue only; the caller
    // then sums the columns itself
    dfu_set_error("dfu_gemm: dGELU column sums need the persistent 256x256 tile (plan: %d)",
                  pl.tile + 1);
    return DFU_E_UNSUPPORTED;
  }
  if (d->epilogue == DFU_EPI_X3_GELU) {
    DFU_CHECK_ARG(pl.tile == T256x256ps, "dfu_gemm: X3_GELU needs the persistent 256x256 tile");
    DFU_CHECK_ARG(d->aux_out != nullptr && d->ldaux_out >= d->N && d->ldc >= 3LL * d->N,
                  "dfu_gemm: X3_GELU needs aux_out (ldaux_out >= N) and ldc >= 3N");
  }
  DFU_CHECK_ARG(((uintptr_t)d->A & 15) == 0 && ((uintptr_t)d->B & 15) == 0,
                "dfu_gemm: A and B must be 16-byte aligned");
  if (d->a_mode == DFU_OPND_KMAJOR || d->a_mode == DFU_OPND_MNMAJOR)
    DFU_CHECK_ARG(d->lda % 8 == 0, "dfu_gemm: lda=%lld must be a multiple of 8", (long long)d->lda);
  if (d->b_mode == DFU_OPND_KMAJOR || d->b_mode == DFU_OPND_MNMAJOR)
    DFU_CHECK_ARG(d->ldb % 8 == 0, "dfu_gemm: ldb=%lld must be a multiple of 8", (long long)d->ldb);
  if (d->a_mode == DFU_OPND_MNMAJOR)
    DFU_CHECK_ARG(d->lda >= round8(d->M), "dfu_gemm: MN-major A needs lda >= round8(M)");
  if (d->b_mode == DFU_OPND_MNMAJOR)
    DFU_CHECK_ARG(d->ldb >= round8(d->N), "dfu_gemm: MN-major B needs ldb >= round8(N)");
  if (d->epilogue == DFU_EPI_BF16_STATS || d->epilogue == DFU_EPI_F32_STATS)
    DFU_CHECK_ARG(d->stats != nullptr, "dfu_gemm: STATS epilogue needs a stats slab");
  DFU_CHECK_ARG(d->x3_pairs == 0 || (d->x3_pairs == 1 && d->a_seg > 0 && d->operand_type == 0),
                "dfu_gemm: x3_pairs (0/1) needs split-pair A (a_seg > 0) and bf16 operands");
  if (d->a_seg) {
    const bool conv_a = d->a_mode == DFU_OPND_CONV_FWD;
    const int nseg = d->x3_pairs ? 2 : 3;  // interleaved pairs: K = 2 a_seg (a_seg % 32 == 0)
    const int align = d->x3_pairs ? 32 : (conv_a ? 64 : 8);
    DFU_CHECK_ARG(d->a_lo != nullptr && d->a_seg > 0 && d->a_seg % align == 0 &&
                      (d->a_mode == DFU_OPND_KMAJOR || conv_a) &&
                      (conv_a ? d->conv_c == nseg * d->a_seg : (d->K == nseg * d->a_seg &&
                                                                d->lda == d->a_seg)) &&
                      ((uintptr_t)d->a_lo & 15) == 0 &&
                      ((const char*)d->a_lo - (const char*)d->A) % 2 == 0,
                  "dfu_gemm: split-pair A needs a_lo, a_seg %% 8 == 0 (conv forward: %% 64; "
                  "x3_pairs: %% 32), K-contiguous or conv-forward A with K (conv_c) = 3 a_seg "
                  "(x3_pairs: 2 a_seg) and lda = a_seg");
    DFU_CHECK_ARG(pl.tile != T256x256p8 && pl.tile != T256x256ps && pl.tile != T192x256ps,
                  "dfu_gemm: split-pair A is not supported on the phased tiles (plan %d)",
                  pl.tile + 1);
  }
  if (d->epilogue == DFU_EPI_BF16_DSTATS) {  // retired in round 4 (measured slower); reserved
    dfu_set_error("dfu_gemm: the DSTATS epilogue is retired");
    return DFU_E_UNSUPPORTED;
  }

  const bool conv = d->a_mode >= DFU_OPND_CONV_FWD || d->b_mode >= DFU_OPND_CONV_FWD;
  if (conv) {
    DFU_CHECK_ARG(d->conv_n > 0 && d->conv_h > 0 && d->conv_w > 0 && d->conv_c > 0 &&
                      d->conv_k > 0 && d->conv_r > 0 && d->conv_s > 0 && d->conv_stride > 0 &&
                      d->conv_p > 0 && d->conv_q > 0,
                  "dfu_gemm: conv geometry missing");
    if (d->a_mode == DFU_OPND_CONV_FWD) {
      DFU_CHECK_ARG(d->conv_c % BK == 0, "dfu_gemm: implicit conv fwd needs C %% 64 == 0");
      DFU_CHECK_ARG(d->K == d->conv_r * d->conv_s * d->conv_c, "dfu_gemm: conv fwd K != RSC");
      DFU_CHECK_ARG(d->M == d->conv_n * d->conv_p * d->conv_q, "dfu_gemm: conv fwd M != NPQ");
    }
    if (d->a_mode == DFU_OPND_CONV_DGRAD) {
      DFU_CHECK_ARG(d->conv_k % BK == 0, "dfu_gemm: conv dgrad needs Kout %% 64 == 0");
      DFU_CHECK_ARG(d->K == d->conv_r * d->conv_s * d->conv_k, "dfu_gemm: conv dgrad K != RSK");
      DFU_CHECK_ARG(d->M == d->conv_n * d->conv_h * d->conv_w, "dfu_gemm: conv dgrad M != NHW");
      DFU_CHECK_ARG(d->conv_c % 8 == 0, "dfu_gemm: conv dgrad needs C %% 8 == 0");
      DFU_CHECK_ARG(d->b_mode == DFU_OPND_CONV_DGRAD_W, "dfu_gemm: conv dgrad needs DGRAD_W B");
    }
    if (d->b_mode == DFU_OPND_CONV_WGRAD_X) {
      DFU_CHECK_ARG(d->conv_c % 8 == 0, "dfu_gemm: conv wgrad needs C %% 8 == 0");
      DFU_CHECK_ARG(d->N == d->conv_r * d->conv_s * d->conv_c, "dfu_gemm: conv wgrad N != RSC");
      DFU_CHECK_ARG(d->K == d->conv_n * d->conv_p * d->conv_q, "dfu_gemm: conv wgrad K != NPQ");
    }
  }
  hipStream_t s = (hipStream_t)stream;
  if (d->a_mode != DFU_OPND_CONV_DGRAD || d->conv_stride == 1) return launch(d, pl, nullptr, s);

  // Strided dgrad: stride^2 phase launches, each a dense stride-1 gather over its live taps
  // (a dense launch would spend (1 - 1/stride^2) of its MFMA work on zero taps).
  const int st = d->conv_stride;
  for (int ph = 0; ph < st; ++ph)
    for (int pw = 0; pw < st; ++pw) {
      const Phase f = make_phase(d, ph, pw);
      if (f.Hs == 0 || f.Ws == 0) continue;
      if (f.nr == 0 || f.ns == 0) {  // no live tap: the rows are 0 (or the addend)
        DFU_CHECK_ARG(d->epilogue == DFU_EPI_BF16 || d->epilogue == DFU_EPI_BF16_ADD,
                      "dfu_gemm: strided dgrad supports the BF16 / BF16_ADD epilogues");
        if (d->epilogue == DFU_EPI_BF16_ADD && d->aux == d->C && d->ldaux == d->ldc) continue;
        const int64_t n = (int64_t)d->conv_n * f.Hs * f.Ws * (d->N / 8);
        const int blocks = (int)((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096);
        hipLaunchKernelGGL(k_phase_fill, dim3(blocks), dim3(256), 0, s, (bf16_t*)d->C, d->ldc,
                           d->epilogue == DFU_EPI_BF16_ADD ? (const bf16_t*)d->aux : nullptr,
                           d->ldaux, d->conv_n, f.Hs, f.Ws, d->conv_h, d->conv_w, st, ph, pw,
                           d->N);
        DFU_LAUNCH_CHECK();
        continue;
      }
      dfu_gemm_desc pd = *d;
      pd.M = d->conv_n * f.Hs * f.Ws;
      pd.K = f.nr * f.ns * d->conv_k;
      const Plan pp = plan_gemm(&pd);
      if (!pp.entry) {
        dfu_set_error("dfu_gemm: no kernel for a dgrad phase");
        return DFU_E_UNSUPPORTED;
      }
      const int rc = launch(&pd, pp, &f, s);
      if (rc != DFU_OK) return rc;
    }
  return DFU_OK;
}

namespace {

int launch(const dfu_gemm_desc* d, const Plan& pl, const Phase* ph, hipStream_t s) {
  const bool acc_epi = d->epilogue == DFU_EPI_F32_ACC;
  GemmArgs a;
  const int TM = kTM[pl.tile], TN = kTN[pl.tile];
  a.M = d->M; a.N = d->N; a.K = d->K;
  a.ktiles = cdiv(d->K, BK);
  a.kt_per_split = cdiv(a.ktiles, pl.split);
  const int splits = cdiv(a.ktiles, a.kt_per_split);
  a.tiles_m = cdiv(d->M, TM);
  a.tiles_n = cdiv(d->N, TN);
  a.A = (const bf16_t*)d->A; a.lda = d->lda;
  a.B = (const bf16_t*)d->B; a.ldb = d->ldb;
  a.C = d->C; a.ldc = d->ldc;
  a.alpha = d->alpha;
  a.bias = d->bias;
  a.aux = d->aux; a.ldaux = d->ldaux;
  a.aux_out = d->aux_out; a.ldaux_out = d->ldaux_out;
  a.stats = d->stats;
  a.split = splits;
  a.n4 = (d->N % 4 == 0 && d->ldc % 4 == 0 && (d->aux == nullptr || d->ldaux % 4 == 0) &&
          (d->aux_out == nullptr || d->ldaux_out % 4 == 0))
             ? 1
             : 0;
  a.n8 = (a.n4 && d->N % 8 == 0 && d->ldc % 8 == 0 && ((uintptr_t)d->C & 15) == 0 &&
          (d->aux_out == nullptr || (d->ldaux_out % 8 == 0 && ((uintptr_t)d->aux_out & 15) == 0)))
             ? 1
             : 0;
  a.slab = nullptr;
  if (acc_epi && splits > 1 && d->workspace != nullptr &&
      d->workspace_bytes >= (int64_t)splits * d->M * d->N * 4)
    a.slab = (float*)d->workspace;
  // in-kernel split-K reduction: the last split of a tile to finish adds the slabs into C
  a.counters = nullptr;
  if (a.slab != nullptr && g_inkernel_reduce && splits <= 8 && d->tile_counters != nullptr &&
      d->tile_counters_len >= a.tiles_m * a.tiles_n && pl.tile != T256x256p8 &&
      pl.tile != T256x256ps && pl.tile != T192x256ps)
    a.counters = d->tile_counters;
  // the phased kernel has neither fp32 atomics nor the in-kernel reduction: split-K needs slabs
  DFU_CHECK_ARG(!((pl.tile == T256x256p8 || pl.tile == T256x256ps || pl.tile == T192x256ps) &&
                  acc_epi && splits > 1 &&
                  a.slab == nullptr),
                "dfu_gemm: split-K on the phased 256x256 tile needs a workspace "
                "(dfu_gemm_workspace_bytes)");
  a.ep_tokens = d->ep_tokens;
  a.cn = d->conv_n; a.ch = d->conv_h; a.cw = d->conv_w; a.cc = d->conv_c;
  a.ck = d->conv_k; a.cr = d->conv_r; a.cs = d->conv_s;
  a.cstride = d->conv_stride; a.cpad = d->conv_pad; a.cp = d->conv_p; a.cq = d->conv_q;
  a.cpad_w = d->conv_pad;
  // split-pair A (the bf16x3 ResNet forward's activations): hi at A, lo at a_lo, both with
  // row / pixel stride a_seg; the tripled K reads segments hi | lo | hi
  a.a_seg = d->a_seg;
  a.a_pix = d->a_seg ? d->a_seg : d->conv_c;
  a.a_lo_delta = d->a_seg ? ((const bf16_t*)d->a_lo - (const bf16_t*)d->A) : 0;
  a.ph_st = a.ph_h = a.ph_w = a.ph_r0 = a.ph_s0 = a.ph_H = a.ph_W = a.ph_S = 0;
  if (ph) {  // the phase's stride-1 equivalent geometry (GemmArgs::ph_*)
    a.ch = ph->Hs; a.cw = ph->Ws; a.cr = ph->nr; a.cs = ph->ns;
    a.cstride = 1; a.cpad = ph->qh; a.cpad_w = ph->qw;
    a.ph_st = d->conv_stride; a.ph_h = ph->ph; a.ph_w = ph->pw;
    a.ph_r0 = ph->r0; a.ph_s0 = ph->s0;
    a.ph_H = d->conv_h; a.ph_W = d->conv_w; a.ph_S = d->conv_s;
  }
  static const int dbg = getenv("DFU_GEMM_DEBUG") ? atoi(getenv("DFU_GEMM_DEBUG")) : 0;
  a.dbg = dbg;
  a.m_ld_bound = round8(d->M);
  a.n_ld_bound = round8(d->N);
  {
    // operand extents (elements): K-contiguous [MN][ld], MN-major [K][ld]
    const int64_t ea = d->a_mode == DFU_OPND_MNMAJOR ? (int64_t)(d->K - 1) * d->lda + a.m_ld_bound
                                                     : (int64_t)(d->M - 1) * d->lda + d->K;
    const int64_t eb = d->b_mode == DFU_OPND_MNMAJOR ? (int64_t)(d->K - 1) * d->ldb + a.n_ld_bound
                                                     : (int64_t)(d->N - 1) * d->ldb + d->K;
    if (pl.tile == T256x256ps || pl.tile == T192x256ps)
      DFU_CHECK_ARG(2 * ea < kRsrcBytes && 2 * eb < kRsrcBytes,
                    "dfu_gemm: operands over 2 GiB need another tile than the buffer-DMA 256x256");
    a.a_bytes = (int)(2 * ea < kRsrcBytes ? 2 * ea : kRsrcBytes);
    a.b_bytes = (int)(2 * eb < kRsrcBytes ? 2 * eb : kRsrcBytes);
  }
  if (d->a_mode >= DFU_OPND_CONV_FWD || d->b_mode >= DFU_OPND_CONV_FWD) {
    a.div_pq = make_fastdiv(a.cp * a.cq);
    a.div_q = make_fastdiv(a.cq);
    a.div_hw = make_fastdiv(a.ch * a.cw);
    a.div_w = make_fastdiv(a.cw);
    a.div_c = make_fastdiv(a.cc);
    a.div_k = make_fastdiv(a.ck);
    a.div_s = make_fastdiv(a.cs);
    if (d->b_mode == DFU_OPND_CONV_WGRAD_X) a.n_ld_bound = d->N;
  }
  // the epilogue addresses its outputs by 32-bit offsets within a 2 GiB buffer range
  const bool c32 = d->epilogue == DFU_EPI_F32 || d->epilogue == DFU_EPI_F32_RESID ||
                   d->epilogue == DFU_EPI_F32_ACC || d->epilogue == DFU_EPI_PATCH ||
                   d->epilogue == DFU_EPI_F32_STATS;
  int64_t c_rows = d->M;
  if (ph) c_rows = (int64_t)d->conv_n * d->conv_h * d->conv_w;
  if (d->epilogue == DFU_EPI_PATCH && d->ep_tokens > 0)
    c_rows = (int64_t)(d->M / d->ep_tokens) * (d->ep_tokens + 1);
  DFU_CHECK_ARG(c_rows * d->ldc * (c32 ? 4 : 2) < kRsrcBytes &&
                    (a.slab == nullptr || (int64_t)splits * d->M * d->N * 4 < kRsrcBytes),
                "dfu_gemm: output larger than the 2 GiB epilogue buffer range");
  // Persistent schedule: at most one wave of workgroups (CUs x occupancy), each walking its
  // work units as one K-step stream; split-K by fp32 atomics (no workspace) keeps one unit
  // per workgroup (its atomics have no fixed vmcnt count).
  const int slots = kCUs * kOcc[pl.tile];
  a.tail_full = a.tail_r = a.tail_s = a.tail_kps = 0;
  a.tslab = nullptr;
  if (!acc_epi && splits == 1 && kTailOK[pl.tile]) {
    const Tail t =
        tail_plan(a.tiles_m * a.tiles_n, slots, a.ktiles, TM, TN, kStepUs[kBase[pl.tile]]);
    if (t.r > 0 && d->workspace != nullptr && d->workspace_bytes >= t.bytes &&
        d->tile_counters != nullptr && d->tile_counters_len >= t.r) {
      a.tail_full = t.full; a.tail_r = t.r; a.tail_s = t.s; a.tail_kps = t.kps;
      a.tslab = (float*)d->workspace;
      a.counters = d->tile_counters;
    }
  }
  const int units = a.tail_r ? a.tail_full + a.tail_r * a.tail_s : a.tiles_m * a.tiles_n * splits;
  const bool atomics = acc_epi && splits > 1 && a.slab == nullptr;
  const bool pers = (pl.tile == T256x256ps || pl.tile == T192x256ps) ? g_persistent_ps
                                                                     : g_persistent;
  const int nwg = (pers && !atomics && units > slots) ? slots : units;
  hipLaunchKernelGGL(pl.entry->fn, dim3(nwg), dim3(pl.entry->threads), 0, s, a);
  DFU_LAUNCH_CHECK();
  if (a.slab != nullptr && a.counters == nullptr) {
    const int64_t n = (int64_t)d->M * d->N;
    const bool vec = d->N % 4 == 0 && d->ldc % 4 == 0 && ((uintptr_t)d->C & 15) == 0;
    int64_t blocks = (vec ? n / 4 : n) / 256 + 1;
    if (blocks > 8192) blocks = 8192;
    if (blocks < kCUs && splits >= 8 && g_wide_reduce) {
      // too few elements to fill the chip one lane each: split the slabs over waves too
      const int nw = splits < 16 ? splits : 16;
      const int64_t units = vec ? n / 4 : n;
      const unsigned wb = (unsigned)((units + 63) / 64);
      if (vec)
        hipLaunchKernelGGL(k_splitk_reduce_wide<true>, dim3(wb), dim3(64 * nw), 0, s, a.slab,
                           splits, d->M, d->N, (float*)d->C, d->ldc);
      else
        hipLaunchKernelGGL(k_splitk_reduce_wide<false>, dim3(wb), dim3(64 * nw), 0, s, a.slab,
                           splits, d->M, d->N, (float*)d->C, d->ldc);
    } else if (vec)
      hipLaunchKernelGGL(k_splitk_reduce, dim3((unsigned)blocks), dim3(256), 0, s, a.slab, splits,
                         d->M, d->N, (float*)d->C, d->ldc);
    else
      hipLaunchKernelGGL(k_splitk_reduce_scalar,
                         dim3((unsigned)((d->N + 255) / 256), (unsigned)(d->M < 4096 ? d->M : 4096)),
                         dim3(256), 0, s, a.slab, splits, d->M, d->N, (float*)d->C, d->ldc);
    DFU_LAUNCH_CHECK();
  }
  return DFU_OK;
}

}  // namespace
