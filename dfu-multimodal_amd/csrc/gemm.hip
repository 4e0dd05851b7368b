// Host dispatch for the MFMA GEMM template (include/dfu_hip.h: dfu_gemm).
// Only the (A mode, B mode, epilogue) combinations the training step uses are instantiated.
#include "gemm_kernel.h"

using namespace dfu;

namespace {

typedef void (*gemm_fn)(const GemmArgs);

template <int A, int B, int E>
constexpr gemm_fn K() {
  return &gemm_kernel<A, B, E>;
}

struct Entry {
  int a, b, e;
  gemm_fn fn;
};

#define E3(a, b, e) {a, b, e, K<a, b, e>()}
const Entry kTable[] = {
    // Linear forward: Y = X W^T (+ epilogue)         (timm qkv/proj/fc1/fc2, patch-embed, head)
    E3(DFU_OPND_KMAJOR, DFU_OPND_KMAJOR, DFU_EPI_BF16),
    E3(DFU_OPND_KMAJOR, DFU_OPND_KMAJOR, DFU_EPI_BF16_RELU),
    E3(DFU_OPND_KMAJOR, DFU_OPND_KMAJOR, DFU_EPI_BF16_GELU),
    E3(DFU_OPND_KMAJOR, DFU_OPND_KMAJOR, DFU_EPI_F32),
    E3(DFU_OPND_KMAJOR, DFU_OPND_KMAJOR, DFU_EPI_F32_RESID),
    E3(DFU_OPND_KMAJOR, DFU_OPND_KMAJOR, DFU_EPI_PATCH),
    // 1x1/s1 conv and the stem (explicit im2col) forward with BN statistics
    E3(DFU_OPND_KMAJOR, DFU_OPND_KMAJOR, DFU_EPI_BF16_STATS),
    // Linear / 1x1 conv dgrad: dX = dY W
    E3(DFU_OPND_KMAJOR, DFU_OPND_MNMAJOR, DFU_EPI_BF16),
    E3(DFU_OPND_KMAJOR, DFU_OPND_MNMAJOR, DFU_EPI_BF16_DGELU),
    E3(DFU_OPND_KMAJOR, DFU_OPND_MNMAJOR, DFU_EPI_BF16_ADD),
    E3(DFU_OPND_KMAJOR, DFU_OPND_MNMAJOR, DFU_EPI_F32),
    // Linear / 1x1 conv wgrad: dW += dY^T X
    E3(DFU_OPND_MNMAJOR, DFU_OPND_MNMAJOR, DFU_EPI_F32_ACC),
    // implicit-GEMM conv (3x3, strided 1x1)
    E3(DFU_OPND_CONV_FWD, DFU_OPND_KMAJOR, DFU_EPI_BF16_STATS),
    E3(DFU_OPND_CONV_DGRAD, DFU_OPND_CONV_DGRAD_W, DFU_EPI_BF16),
    E3(DFU_OPND_CONV_DGRAD, DFU_OPND_CONV_DGRAD_W, DFU_EPI_BF16_ADD),
    E3(DFU_OPND_MNMAJOR, DFU_OPND_CONV_WGRAD_X, DFU_EPI_F32_ACC_CONVW),
};
#undef E3

inline int round8(int x) { return (x + 7) & ~7; }

}  // namespace

extern "C" int dfu_gemm_stats_tiles(int32_t M) { return (M + BM - 1) / BM; }

extern "C" int dfu_gemm(const dfu_gemm_desc* d, void* stream) {
  DFU_CHECK_ARG(d != nullptr, "dfu_gemm: null descriptor");
  DFU_CHECK_ARG(d->M > 0 && d->N > 0 && d->K > 0, "dfu_gemm: bad shape M=%d N=%d K=%d", d->M,
                d->N, d->K);
  const bool a_kc = d->a_mode == DFU_OPND_KMAJOR || d->a_mode == DFU_OPND_CONV_FWD ||
                    d->a_mode == DFU_OPND_CONV_DGRAD;
  const bool b_kc = d->b_mode == DFU_OPND_KMAJOR;
  DFU_CHECK_ARG(!(a_kc || b_kc) || d->K % 8 == 0,
                "dfu_gemm: K=%d must be a multiple of 8 for K-contiguous operands", d->K);
  gemm_fn fn = nullptr;
  for (const Entry& e : kTable)
    if (e.a == d->a_mode && e.b == d->b_mode && e.e == d->epilogue) fn = e.fn;
  if (!fn) {
    dfu_set_error("dfu_gemm: unsupported combination a_mode=%d b_mode=%d epilogue=%d",
                  d->a_mode, d->b_mode, d->epilogue);
    return DFU_E_UNSUPPORTED;
  }
  const bool acc_epi = d->epilogue == DFU_EPI_F32_ACC || d->epilogue == DFU_EPI_F32_ACC_CONVW;
  DFU_CHECK_ARG(d->split_k >= 1, "dfu_gemm: split_k must be >= 1");
  DFU_CHECK_ARG(d->split_k == 1 || acc_epi, "dfu_gemm: split_k > 1 needs an F32_ACC epilogue");
  DFU_CHECK_ARG(((uintptr_t)d->A & 15) == 0 && ((uintptr_t)d->B & 15) == 0,
                "dfu_gemm: A and B must be 16-byte aligned");
  // leading dims must keep every 16-B vector aligned
  if (d->a_mode == DFU_OPND_KMAJOR || d->a_mode == DFU_OPND_MNMAJOR)
    DFU_CHECK_ARG(d->lda % 8 == 0, "dfu_gemm: lda=%lld must be a multiple of 8", (long long)d->lda);
  if (d->b_mode == DFU_OPND_KMAJOR || d->b_mode == DFU_OPND_MNMAJOR)
    DFU_CHECK_ARG(d->ldb % 8 == 0, "dfu_gemm: ldb=%lld must be a multiple of 8", (long long)d->ldb);
  if (d->a_mode == DFU_OPND_MNMAJOR)
    DFU_CHECK_ARG(d->lda >= round8(d->M), "dfu_gemm: MN-major A needs lda >= round8(M)");
  if (d->b_mode == DFU_OPND_MNMAJOR)
    DFU_CHECK_ARG(d->ldb >= round8(d->N), "dfu_gemm: MN-major B needs ldb >= round8(N)");
  if (d->epilogue == DFU_EPI_BF16_STATS)
    DFU_CHECK_ARG(d->stats != nullptr, "dfu_gemm: STATS epilogue needs a stats slab");

  GemmArgs a;
  a.M = d->M; a.N = d->N; a.K = d->K;
  a.ktiles = (d->K + BK - 1) / BK;
  a.kt_per_split = (a.ktiles + d->split_k - 1) / d->split_k;
  const int splits = (a.ktiles + a.kt_per_split - 1) / a.kt_per_split;
  a.tiles_m = (d->M + BM - 1) / BM;
  a.tiles_n = (d->N + BN - 1) / BN;
  a.A = (const bf16_t*)d->A; a.lda = d->lda;
  a.B = (const bf16_t*)d->B; a.ldb = d->ldb;
  a.C = d->C; a.ldc = d->ldc;
  a.alpha = d->alpha;
  a.bias = d->bias;
  a.aux = d->aux; a.ldaux = d->ldaux;
  a.aux_out = d->aux_out; a.ldaux_out = d->ldaux_out;
  a.stats = d->stats;
  a.split = splits;
  a.ep_tokens = d->ep_tokens;
  a.cn = d->conv_n; a.ch = d->conv_h; a.cw = d->conv_w; a.cc = d->conv_c;
  a.ck = d->conv_k; a.cr = d->conv_r; a.cs = d->conv_s;
  a.cstride = d->conv_stride; a.cpad = d->conv_pad; a.cp = d->conv_p; a.cq = d->conv_q;
  a.m_ld_bound = round8(d->M);
  a.n_ld_bound = round8(d->N);
  const bool conv = d->a_mode >= DFU_OPND_CONV_FWD || d->b_mode >= DFU_OPND_CONV_FWD ||
                    d->epilogue == DFU_EPI_F32_ACC_CONVW;
  if (conv) {
    DFU_CHECK_ARG(d->conv_n > 0 && d->conv_h > 0 && d->conv_w > 0 && d->conv_c > 0 &&
                      d->conv_k > 0 && d->conv_r > 0 && d->conv_s > 0 && d->conv_stride > 0 &&
                      d->conv_p > 0 && d->conv_q > 0,
                  "dfu_gemm: conv geometry missing");
    a.div_pq = make_fastdiv(d->conv_p * d->conv_q);
    a.div_q = make_fastdiv(d->conv_q);
    a.div_hw = make_fastdiv(d->conv_h * d->conv_w);
    a.div_w = make_fastdiv(d->conv_w);
    a.div_c = make_fastdiv(d->conv_c);
    a.div_k = make_fastdiv(d->conv_k);
    a.div_s = make_fastdiv(d->conv_s);
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
    }
    if (d->b_mode == DFU_OPND_CONV_WGRAD_X) {
      DFU_CHECK_ARG(d->conv_c % 8 == 0, "dfu_gemm: conv wgrad needs C %% 8 == 0");
      DFU_CHECK_ARG(d->N == d->conv_r * d->conv_s * d->conv_c, "dfu_gemm: conv wgrad N != RSC");
      DFU_CHECK_ARG(d->K == d->conv_n * d->conv_p * d->conv_q, "dfu_gemm: conv wgrad K != NPQ");
      a.n_ld_bound = d->N;
    }
  }
  dim3 grid(a.tiles_m * a.tiles_n, splits);
  hipLaunchKernelGGL(fn, grid, dim3(NT), 0, (hipStream_t)stream, a);
  DFU_LAUNCH_CHECK();
  return DFU_OK;
}
