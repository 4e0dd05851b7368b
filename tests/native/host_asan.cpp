// Host-side sanitizer driver ("-fsanitize=address CPU build of the host C++").
// Built by `make -C dfu-multimodal_amd asan` with AddressSanitizer + UBSan on the HOST half of
// every libdfu_hip translation unit (-Xarch_host; the gfx950 device code is unchanged) and run
// by tests/test_host_asan_cpu.py.  It drives only the host logic, with no GPU:
//   - the GEMM planner (tile / split-K cost model, offline-tuned table lookup, tail-split plan,
//     workspace sizing) over every contraction of the training step and a random shape sweep;
//   - the argument validation of every launching entry point (each rejects before any launch);
//   - the error-string buffer (truncation of long messages);
//   - the resize tap computation (PIL precompute_coeffs restatement) into exactly-sized
//     buffers, so an out-of-bounds write is a sanitizer report;
//   - the BatchNorm / LayerNorm / colsum / attention sizing helpers.
// Exit status 0 and no sanitizer report = pass.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "../../include/dfu_hip.h"

extern "C" void dfu_set_error(const char* fmt, ...);

static int g_fail = 0;
#define EXPECT(cond, ...)                                  \
  do {                                                     \
    if (!(cond)) {                                         \
      fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      fprintf(stderr, __VA_ARGS__);                        \
      fprintf(stderr, "\n");                               \
      ++g_fail;                                            \
    }                                                      \
  } while (0)

static dfu_gemm_desc linear(int M, int N, int K, int a, int b, int e) {
  dfu_gemm_desc d;
  memset(&d, 0, sizeof(d));
  d.M = M; d.N = N; d.K = K;
  d.a_mode = a; d.b_mode = b; d.epilogue = e;
  d.lda = a == DFU_OPND_MNMAJOR ? (M + 7) / 8 * 8 : K;
  d.ldb = b == DFU_OPND_MNMAJOR ? (N + 7) / 8 * 8 : K;
  d.ldc = N;
  d.alpha = 1.f;
  return d;
}

// conv geometry: input B x H x W x C, K filters R x S, stride, pad
static void set_conv(dfu_gemm_desc& d, int B, int H, int W, int C, int K, int R, int st, int pad) {
  d.conv_n = B; d.conv_h = H; d.conv_w = W; d.conv_c = C;
  d.conv_k = K; d.conv_r = R; d.conv_s = R; d.conv_stride = st; d.conv_pad = pad;
  d.conv_p = (H + 2 * pad - R) / st + 1;
  d.conv_q = (W + 2 * pad - R) / st + 1;
}

static void check_plan(const dfu_gemm_desc& d, const char* what) {
  int32_t tile = -1, split = -1;
  const int rc = dfu_gemm_plan(&d, &tile, &split);
  EXPECT(rc == DFU_OK, "%s: plan rc %d (%s)", what, rc, dfu_last_error_string());
  if (rc != DFU_OK) return;
  EXPECT(tile >= 1 && tile <= 11, "%s: tile %d", what, tile);
  EXPECT(split >= 1 && split <= 256, "%s: split %d", what, split);
  EXPECT(split == 1 || d.epilogue == DFU_EPI_F32_ACC, "%s: split %d on a non-ACC epilogue", what,
         split);
  const int64_t ws = dfu_gemm_workspace_bytes(&d);
  EXPECT(ws >= 0, "%s: workspace %lld", what, (long long)ws);
  if (d.epilogue == DFU_EPI_F32_ACC && split > 1)
    EXPECT(ws == (int64_t)split * d.M * d.N * 4, "%s: slab bytes %lld", what, (long long)ws);
}

// Every contraction of one fusion training step (B = 64): ViT-B/16 linears and the ResNet-50
// convolutions (fwd, dgrad incl. strided phases, wgrad).
static void step_shapes() {
  const int B = 64, T = 197, D = 768;
  const int M = B * T;
  const int lin[][2] = {{3 * D, D}, {D, D}, {4 * D, D}, {D, 4 * D}};  // N, K of the forward
  for (auto& l : lin) {
    const int N = l[0], K = l[1];
    for (int e : {DFU_EPI_BF16, DFU_EPI_BF16_GELU, DFU_EPI_F32_RESID})
      check_plan(linear(M, N, K, DFU_OPND_KMAJOR, DFU_OPND_KMAJOR, e), "vit fwd");
    for (int e : {DFU_EPI_BF16, DFU_EPI_BF16_DGELU})
      check_plan(linear(M, K, N, DFU_OPND_KMAJOR, DFU_OPND_MNMAJOR, e), "vit dgrad");
    dfu_gemm_desc w = linear(N, K, M, DFU_OPND_MNMAJOR, DFU_OPND_MNMAJOR, DFU_EPI_F32_ACC);
    check_plan(w, "vit wgrad");
    w.split_k = 3;
    check_plan(w, "vit wgrad split 3");
  }
  check_plan(linear(B * 196, D, D, DFU_OPND_KMAJOR, DFU_OPND_KMAJOR, DFU_EPI_PATCH), "patch");

  struct Conv { int H, C, K, R, st; };
  const Conv convs[] = {{56, 64, 64, 1, 1},    {56, 64, 64, 3, 1},    {56, 64, 256, 1, 1},
                        {56, 256, 64, 1, 1},   {56, 256, 128, 1, 1},  {56, 128, 128, 3, 2},
                        {28, 128, 512, 1, 1},  {56, 256, 512, 1, 2},  {28, 512, 128, 1, 1},
                        {28, 128, 128, 3, 1},  {28, 512, 256, 1, 1},  {28, 256, 256, 3, 2},
                        {14, 256, 1024, 1, 1}, {28, 512, 1024, 1, 2}, {14, 1024, 256, 1, 1},
                        {14, 256, 256, 3, 1},  {14, 1024, 512, 1, 1}, {14, 512, 512, 3, 2},
                        {7, 512, 2048, 1, 1},  {14, 1024, 2048, 1, 2}, {7, 2048, 512, 1, 1},
                        {7, 512, 512, 3, 1}};
  for (const Conv& c : convs) {
    const int pad = c.R / 2;
    dfu_gemm_desc f;
    memset(&f, 0, sizeof(f));
    set_conv(f, B, c.H, c.H, c.C, c.K, c.R, c.st, pad);
    const int P = f.conv_p;
    const int Mo = B * P * P, Kc = c.R * c.R * c.C;
    // forward
    dfu_gemm_desc d = f;
    d.M = Mo; d.N = c.K; d.K = Kc; d.alpha = 1.f; d.ldc = c.K;
    d.a_mode = c.R == 1 && c.st == 1 ? DFU_OPND_KMAJOR : DFU_OPND_CONV_FWD;
    d.lda = c.C; d.b_mode = DFU_OPND_KMAJOR; d.ldb = Kc;
    d.epilogue = DFU_EPI_BF16_STATS;
    check_plan(d, "conv fwd");
    // dgrad (strided: one plan per phase inside dfu_gemm; the planner sees the dense shape)
    d = f;
    d.M = B * c.H * c.H; d.N = c.C; d.K = c.R * c.R * c.K; d.alpha = 1.f; d.ldc = c.C;
    d.a_mode = DFU_OPND_CONV_DGRAD; d.lda = c.K;
    d.b_mode = DFU_OPND_CONV_DGRAD_W; d.ldb = Kc;
    d.epilogue = DFU_EPI_BF16_ADD;
    check_plan(d, "conv dgrad");
    // wgrad
    d = f;
    d.M = c.K; d.N = Kc; d.K = Mo; d.alpha = 1.f; d.ldc = Kc;
    d.a_mode = DFU_OPND_MNMAJOR; d.lda = c.K;
    d.b_mode = DFU_OPND_CONV_WGRAD_X; d.ldb = c.C;
    d.epilogue = DFU_EPI_F32_ACC;
    check_plan(d, "conv wgrad");
  }
}

// Random shapes through every (a, b, epilogue) combination the planner knows; unsupported ones
// must be reported, never crash.
static void random_sweep() {
  srand(1234);
  const int epis[] = {DFU_EPI_BF16, DFU_EPI_BF16_RELU, DFU_EPI_BF16_GELU, DFU_EPI_F32,
                      DFU_EPI_F32_RESID, DFU_EPI_BF16_DGELU, DFU_EPI_BF16_ADD, DFU_EPI_F32_ACC,
                      DFU_EPI_BF16_STATS, DFU_EPI_PATCH, DFU_EPI_F32_STATS};
  int planned = 0;
  for (int it = 0; it < 20000; ++it) {
    const int M = 1 + rand() % 300000, N = 8 * (1 + rand() % 512), K = 8 * (1 + rand() % 2048);
    const int a = rand() % 2, b = rand() % 2;
    const int e = epis[rand() % 11];
    dfu_gemm_desc d = linear(M, N, K, a, b, e);
    if (rand() % 4 == 0) d.tile = 1 + rand() % 8;
    if (e == DFU_EPI_F32_ACC && rand() % 3 == 0) d.split_k = 1 + rand() % 64;
    int32_t tile = 0, split = 0;
    const int rc = dfu_gemm_plan(&d, &tile, &split);
    EXPECT(rc == DFU_OK || rc == DFU_E_UNSUPPORTED, "sweep: rc %d", rc);
    if (rc == DFU_OK) {
      ++planned;
      EXPECT(tile >= 1 && tile <= 11 && split >= 1, "sweep: tile %d split %d", tile, split);
      EXPECT(dfu_gemm_workspace_bytes(&d) >= 0, "sweep: workspace");
    } else {
      EXPECT(strlen(dfu_last_error_string()) > 0, "sweep: empty error");
    }
  }
  EXPECT(planned > 2000, "sweep: only %d plans", planned);
}

// Descriptors every check in dfu_gemm must reject before launching anything.
static void gemm_rejects() {
  EXPECT(dfu_gemm(nullptr, nullptr) == DFU_E_INVALID, "null desc");
  static char buf[4096] __attribute__((aligned(16)));
  dfu_gemm_desc ok = linear(256, 256, 256, DFU_OPND_KMAJOR, DFU_OPND_KMAJOR, DFU_EPI_BF16);
  ok.A = buf; ok.B = buf; ok.C = buf;
  struct Bad { const char* what; dfu_gemm_desc d; };
  std::vector<Bad> bad;
  dfu_gemm_desc d;
  d = ok; d.M = 0; bad.push_back({"M=0", d});
  d = ok; d.K = -8; bad.push_back({"K<0", d});
  d = ok; d.K = 100; d.lda = d.ldb = 100; bad.push_back({"K%8", d});
  d = ok; d.A = buf + 2; bad.push_back({"misaligned A", d});
  d = ok; d.lda = 260; d.K = 256; d.lda = 257; bad.push_back({"lda%8", d});
  d = ok; d.split_k = -1; bad.push_back({"split<0", d});
  d = ok; d.split_k = 4; bad.push_back({"split on BF16", d});
  d = ok; d.tile = 99; bad.push_back({"tile 99", d});
  d = ok; d.epilogue = DFU_EPI_BF16_STATS; bad.push_back({"stats slab", d});
  d = ok; d.a_mode = DFU_OPND_MNMAJOR; d.lda = 8; bad.push_back({"lda < M", d});
  d = ok; d.a_mode = DFU_OPND_CONV_FWD; bad.push_back({"conv geometry", d});
  d = ok; d.a_mode = DFU_OPND_CONV_FWD;
  set_conv(d, 1, 16, 16, 32, 256, 3, 1, 1); d.K = 288; bad.push_back({"conv C%64", d});
  d = ok; d.a_mode = DFU_OPND_CONV_DGRAD; d.b_mode = DFU_OPND_KMAJOR;
  set_conv(d, 1, 16, 16, 256, 64, 1, 1, 0); d.K = 64; bad.push_back({"dgrad B mode", d});
  for (auto& x : bad) {
    const int rc = dfu_gemm(&x.d, nullptr);
    EXPECT(rc == DFU_E_INVALID || rc == DFU_E_UNSUPPORTED, "%s: rc %d", x.what, rc);
    EXPECT(strlen(dfu_last_error_string()) > 0, "%s: no message", x.what);
  }
}

// Other launching entry points with a missing operand: each returns DFU_E_INVALID first.
static void entry_rejects() {
  float f = 0.f;
  int rc;
  rc = dfu_bn_finalize(nullptr, 1, 128, 64, nullptr, nullptr, 1e-5f, 0.1f, nullptr, nullptr,
                       nullptr, &f, &f, &f, &f, nullptr, nullptr, 0, nullptr);
  EXPECT(rc == DFU_E_INVALID, "bn_finalize rc %d", rc);
  rc = dfu_bn_finalize(&f, 3, 128, 64, nullptr, nullptr, 1e-5f, 0.1f, nullptr, nullptr, nullptr,
                       &f, &f, &f, &f, nullptr, nullptr, 0, nullptr);
  EXPECT(rc == DFU_E_INVALID, "bn_finalize tiles rc %d", rc);
  rc = dfu_bn_apply(nullptr, &f, &f, nullptr, 1, &f, 128, 64, nullptr);
  EXPECT(rc == DFU_E_INVALID, "bn_apply rc %d", rc);
  rc = dfu_bn_apply(&f, &f, &f, nullptr, 1, &f, 128, 60, nullptr);
  EXPECT(rc == DFU_E_INVALID, "bn_apply C%%8 rc %d", rc);
  rc = dfu_bn_bwd_reduce(&f, &f, nullptr, 1, nullptr, nullptr, &f, &f, 128, 64, &f, nullptr);
  EXPECT(rc == DFU_E_INVALID, "bn_bwd_reduce relu1 without out rc %d", rc);
  rc = dfu_bn_bwd_reduce(&f, &f, nullptr, 3, nullptr, nullptr, &f, &f, 128, 64, &f, nullptr);
  EXPECT(rc == DFU_E_INVALID, "bn_bwd_reduce relu3 rc %d", rc);
  rc = dfu_bn_bwd_apply(&f, &f, &f, 2, nullptr, nullptr, &f, &f, &f, 128, 64, &f, nullptr,
                        nullptr);
  EXPECT(rc == DFU_E_INVALID, "bn_bwd_apply relu2 without scale rc %d", rc);
  rc = dfu_reduce_partials_batch(nullptr, 1, nullptr);
  EXPECT(rc == DFU_E_INVALID, "reduce batch null rc %d", rc);
  dfu_reduce_entry ents[DFU_REDUCE_BATCH + 1];
  memset(ents, 0, sizeof(ents));
  rc = dfu_reduce_partials_batch(ents, DFU_REDUCE_BATCH + 1, nullptr);
  EXPECT(rc == DFU_E_INVALID, "reduce batch overflow rc %d", rc);
  rc = dfu_metrics_accumulate(nullptr, nullptr, 4, 2, nullptr, nullptr, nullptr, nullptr, nullptr);
  EXPECT(rc == DFU_E_INVALID, "metrics rc %d", rc);
  rc = dfu_attention_fwd(nullptr, 1, 197, 12, 64, 0.125f, nullptr, nullptr, nullptr);
  EXPECT(rc == DFU_E_INVALID, "attention rc %d", rc);
  rc = dfu_attention_fwd(&f, 1, 300, 12, 64, 0.125f, &f, &f, nullptr);
  EXPECT(rc == DFU_E_INVALID, "attention N=300 rc %d", rc);
  rc = dfu_split_x3(nullptr, 8, 8, 8, 8, nullptr, 0, nullptr, 0, nullptr);
  EXPECT(rc == DFU_E_INVALID, "split_x3 rc %d", rc);
}

static void error_buffer() {
  std::vector<char> big(5000, 'x');
  big.back() = 0;
  dfu_set_error("%s", big.data());
  const size_t n = strlen(dfu_last_error_string());
  EXPECT(n > 0 && n < 1024, "error string length %zu", n);
  dfu_set_error("short %d", 7);
  EXPECT(strcmp(dfu_last_error_string(), "short 7") == 0, "error string '%s'",
         dfu_last_error_string());
}

// Resize taps into buffers of exactly the documented size (heap: ASan sees any overrun).
static void resize_taps() {
  const int sizes[] = {1, 2, 3, 7, 31, 64, 100, 224, 225, 256, 299, 333, 480, 512, 640, 1024, 4032};
  for (int in : sizes)
    for (int out : {1, 2, 112, 224, 256, 299, 512}) {
      const int ks = dfu_resize_ksize(in, out);
      EXPECT(ks >= 1, "ksize(%d, %d) = %d", in, out, ks);
      std::vector<int32_t>* bounds = new std::vector<int32_t>(2 * out);
      std::vector<int32_t>* kk = new std::vector<int32_t>((size_t)out * ks);
      const int rc = dfu_resize_coeffs(in, out, bounds->data(), kk->data());
      EXPECT(rc == DFU_OK, "resize_coeffs(%d, %d) rc %d", in, out, rc);
      for (int o = 0; o < out && rc == DFU_OK; ++o) {
        const int x0 = (*bounds)[2 * o], cnt = (*bounds)[2 * o + 1];
        EXPECT(x0 >= 0 && cnt >= 1 && cnt <= ks && x0 + cnt <= in,
               "taps(%d->%d)[%d] = (%d, %d), ksize %d", in, out, o, x0, cnt, ks);
        int64_t sum = 0;
        for (int k = 0; k < cnt; ++k) sum += (*kk)[(size_t)o * ks + k];
        EXPECT(sum > (1 << 22) - 64 && sum < (1 << 22) + 64, "taps(%d->%d)[%d] sum %lld", in,
               out, o, (long long)sum);
      }
      delete bounds;
      delete kk;
    }
}

static void sizing_helpers() {
  for (int M : {1, 127, 128, 129, 12544, 200704, 802816}) {
    EXPECT(dfu_gemm_stats_tiles(M) == (M + 127) / 128, "stats tiles %d", M);
    for (int C : {64, 128, 256, 512, 1024, 2048}) {
      const int blocks = dfu_bn_bwd_blocks(M, C);
      EXPECT(blocks >= 1 && blocks <= M, "bn bwd blocks M=%d C=%d: %d", M, C, blocks);
      EXPECT(dfu_bn_bwd_finalize_ws_bytes(blocks, C) >= 0, "bn bwd ws");
      EXPECT(dfu_bn_finalize_ws_bytes(dfu_gemm_stats_tiles(M), C) >= 0, "bn fwd ws");
    }
    EXPECT(dfu_ln_bwd_blocks(M) >= 1, "ln blocks %d", M);
    EXPECT(dfu_colsum_blocks(M) >= 1, "colsum blocks %d", M);
  }
  for (int N : {1, 50, 197, 208}) EXPECT(dfu_attention_npad(N) >= N, "npad %d", N);
  EXPECT(dfu_gemm_f32_workspace_bytes(64, 512, 2816) >= 0, "f32 ws");
}

int main() {
  EXPECT(dfu_version() >= 1, "version");
  step_shapes();
  random_sweep();
  gemm_rejects();
  entry_rejects();
  error_buffer();
  resize_taps();
  sizing_helpers();
  if (g_fail) {
    fprintf(stderr, "%d host check(s) failed\n", g_fail);
    return 1;
  }
  printf("host_asan: all host checks passed\n");
  return 0;
}
