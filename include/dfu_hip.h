/*
 * dfu_hip.h — C ABI of libdfu_hip.so, the MI355X (gfx950) kernel library behind the
 * DFU multimodal-fusion training step (ResNet50 RGB branch + ViT-B/16 thermal branch +
 * 2816->512->2 late-fusion MLP).
 *
 * The reference (ShreenathKR2000/DFU-Multimodal) has no FFI layer: its hot path is
 * `MultimodalFusionModel.forward` (notebooks/train_multimodal_fusion.py:315-326) calling
 * torchvision resnet50 (hub v0.13.1, :294) and timm vit_base_patch16_224 (:299-302), whose
 * arithmetic ATen dispatches to cuDNN/cuBLAS.  Each entry point below replaces one of those
 * implicit ATen ops; the comment on each names the reference call site.
 *
 * Conventions:
 *   - the library NEVER allocates device memory; every pointer is caller-owned;
 *   - activations are NHWC (ResNet) / [tokens][features] (ViT), bf16 = raw uint16 bits;
 *   - every call takes the HIP stream to enqueue on and returns 0 on success, otherwise a
 *     hipError_t value or a DFU_E_* code; dfu_last_error_string() gives the message;
 *   - no call synchronises the device or the host (all calls are graph-capturable).
 */
#ifndef DFU_HIP_H
#define DFU_HIP_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DFU_OK 0
#define DFU_E_INVALID 1001     /* bad shape, stride, alignment or mode */
#define DFU_E_UNSUPPORTED 1002 /* valid request this build does not implement */

/* ---------------------------------------------------------------- library ---------- */
const char* dfu_last_error_string(void);
int dfu_version(void);
/* Fill `bytes` of device memory with zero on `stream` (grad buckets, BN slabs). */
int dfu_zero(void* ptr, int64_t bytes, void* stream);

/* Library-owned non-blocking HIP streams at a HIP priority (lower = higher; 0 default). */
int dfu_stream_create(int32_t priority, void** stream);
int dfu_stream_destroy(void* stream);
/* `waiter` waits for the work enqueued on `producer` so far (torch Stream.wait_stream without an
 * Event object per call: one of a per-device ring of events, recorded on `producer` and waited
 * on by `waiter`; capturable).  Both streams belong to the current device. */
int dfu_stream_wait(void* waiter, void* producer);
/* Capture status of `stream`: 0 none, 1 active, 2 invalidated (hipStreamCaptureStatus). */
int dfu_stream_capture_status(void* stream, int32_t* status);
/* End a HIP stream capture left active on any of `streams` (n <= 64) after a failed capture
 * (e.g. unjoined work: the origin's end fails and the origin and its forked streams stay in
 * capture mode): the capturing streams are joined to each other inside the capture, the capture
 * is ended on its origin and the partial graph dropped, so the streams run eager work again.
 * *still_capturing (optional) = streams still capturing afterwards (0 on success). */
int dfu_streams_abort_capture(void* const* streams, int32_t n, int32_t* still_capturing);

/* ---------------------------------------------------------------- GEMM -------------
 * C[M,N] (+)= epilogue(alpha * sum_k A[m,k] * B[n,k]) on bf16 MFMA tiles, fp32 accumulate.
 * Replaces every cuBLAS / cuDNN contraction of the hot path:
 *   timm Linear fwd/dgrad/wgrad (qkv, proj, fc1, fc2, patch-embed; vision_transformer.py),
 *   torchvision conv fwd/dgrad/wgrad as NHWC implicit GEMM (resnet.py Bottleneck, stem),
 *   the fusion head Linear layers (train_multimodal_fusion.py:305-313, grad_cam :289-302).
 */
enum dfu_operand_mode {
  DFU_OPND_KMAJOR = 0,        /* X[mn][k], k contiguous, leading dim ld                    */
  DFU_OPND_MNMAJOR = 1,       /* X[k][mn], mn contiguous, leading dim ld                   */
  DFU_OPND_CONV_FWD = 2,      /* A only: NHWC input gathered as im2col rows (r,s,c)        */
  DFU_OPND_CONV_DGRAD = 3,    /* A only: NHWC dY gathered for dX rows, k = (r,s,kout)      */
  DFU_OPND_CONV_DGRAD_W = 4,  /* B only: KRSC weight viewed as [(r,s,kout)][c]             */
  DFU_OPND_CONV_WGRAD_X = 5   /* B only: NHWC input as [m=(b,oh,ow)][(r,s,c)]              */
};
enum dfu_epilogue {
  DFU_EPI_BF16 = 0,          /* C bf16 = alpha*acc + bias                                  */
  DFU_EPI_BF16_RELU = 1,     /* C bf16 = relu(alpha*acc + bias)                             */
  DFU_EPI_BF16_GELU = 2,     /* pre = acc + bias: C bf16 = gelu(pre), aux_out bf16 = gelu'(pre) */
  DFU_EPI_F32 = 3,           /* C f32 = alpha*acc + bias                                    */
  DFU_EPI_F32_RESID = 4,     /* C f32 = aux f32 + alpha*acc + bias  (residual stream)       */
  DFU_EPI_BF16_DGELU = 5,    /* C bf16 = acc * aux bf16 (aux = the GELU epilogue's gelu');
                                with `stats`: also the column sums of the stored C over each
                                128-row half of every 256-row tile, fp32 [2*ceil(M/256)][N]
                                (the bias gradient's partials; persistent 256x256 tile only,
                                DFU_E_UNSUPPORTED otherwise)                                 */
  DFU_EPI_BF16_ADD = 6,      /* C bf16 = acc + aux bf16                                     */
  DFU_EPI_F32_ACC = 7,       /* C f32 += acc   (split-K: fp32 slabs + reduce, or atomics)   */
  DFU_EPI_F32_ACC_CONVW = 8, /* retired: conv wgrad accumulates KRSC + dfu_conv_grad_krsc... */
  DFU_EPI_BF16_STATS = 9,    /* C bf16 = acc; per-column (sum, M2) of each 128-row tile     */
  DFU_EPI_PATCH = 10,        /* ViT patch-embed: C f32 [B][T+1][N] row 1+p = acc+bias+pos   */
  DFU_EPI_F32_STATS = 11,    /* C f32 = acc; per-column (sum, M2) of each 128-row tile (the
                                split-bf16 "bf16x3" forward: BN statistics of unrounded y)  */
  DFU_EPI_BF16_DSTATS = 12,  /* retired (round 4: BN backward sums in the dgrad epilogue
                                measured slower than the separate reduce); reserved, returns
                                DFU_E_UNSUPPORTED                                            */
  DFU_EPI_X3_GELU = 13,      /* bf16x3 forward of timm Mlp.fc1 + GELU: pre = acc + bias (fp32),
                                C = the A-operand triple [hi | lo | hi] of gelu(pre), bf16
                                [M][3N] (ldc >= 3N; segments at columns 0, N, 2N), aux_out
                                bf16 = gelu'(pre).  Persistent 256x256 tile only.            */
  DFU_EPI_F16_DUAL = 14,     /* v = alpha*acc + bias: C fp16 = v (the next fp16 GEMM's or the
                                fp16 attention's operand), aux_out bf16 = v when non-NULL (a
                                bf16 copy for the backward).  operand_type 1 only.            */
  DFU_EPI_F16_GELU = 15      /* fp16 forward of timm Mlp.fc1 + GELU: pre = acc + bias: C =
                                [fp16 gelu(pre) | bf16 gelu(pre)], 16-bit [M][2N] (ldc >= 2N;
                                fc2's fp16 operand at column 0, the backward's bf16 h at
                                column N), aux_out bf16 = gelu'(pre).  operand_type 1 only.  */
};

typedef struct dfu_gemm_desc {
  int32_t M, N, K;
  int32_t a_mode, b_mode;
  const void* A;
  int64_t lda;
  const void* B;
  int64_t ldb;
  void* C;
  int64_t ldc;
  int32_t epilogue;
  float alpha;
  const float* bias;   /* [N] or NULL                                          */
  const void* aux;     /* residual / pre-activation / pos-embed operand         */
  int64_t ldaux;
  void* aux_out;       /* GELU pre-activation output                            */
  int64_t ldaux_out;
  float* stats;        /* DFU_EPI_{BF16,F32}_STATS: [ceil(M/128)][2][N] fp32 (sum, M2) */
  int32_t split_k;     /* F32_ACC only: 0 = auto (cost model), 1 = none, >1 fixed */
  int32_t ep_tokens;   /* DFU_EPI_PATCH: patches per image                      */
  /* implicit-GEMM convolution geometry (modes 2-5 and the CONVW epilogue)       */
  int32_t conv_n, conv_h, conv_w, conv_c; /* input  N,H,W,C                        */
  int32_t conv_k, conv_r, conv_s;         /* output channels, filter R,S           */
  int32_t conv_stride, conv_pad;
  int32_t conv_p, conv_q;                 /* output H,W                            */
  int32_t tile;        /* 0 = auto; 1..7 = 128x128, 256x128, 128x256, 256x256,
                          128x128 at 2 workgroups/CU (8 waves, 4 waves), phased
                          256x256 (K-contiguous A and B only); 8 = persistent
                          phased 256x256 (K-contiguous or MN-major A and B);
                          9 = persistent phased 192x256 (K-contiguous A);
                          10, 11 = 4-wave 256x64, 128x64 at 2/CU (K-contiguous
                          or implicit-conv A, K-contiguous B)                  */
  void* workspace;     /* split-K fp32 slabs (dfu_gemm_workspace_bytes); NULL =  */
  int64_t workspace_bytes; /*   split-K partials accumulate with fp32 atomics     */
  /* Split-K with slabs: NULL = a second kernel adds the slabs into C.  Otherwise a zeroed
   * int32[tile_counters_len] the launch returns zeroed: the last of a tile's splits to finish
   * adds all its slabs into C inside the GEMM (same order, bitwise the same result).  One
   * buffer per stream (launches on one stream never overlap). */
  int32_t* tile_counters;
  int32_t tile_counters_len;
  int32_t operand_type; /* 0 = bf16 A and B; 1 = fp16 A and B (the "parity" precision
                           mode's ViT forward: persistent tiles 8 / 9, K-contiguous A and B,
                           epilogues F32, F32_RESID, F16_DUAL, F16_GELU)                   */
  /* Split-pair A (a_seg > 0; the bf16x3 ResNet forward's activations): the tripled K (or the
   * conv's tripled channel axis, conv_c = 3 a_seg) reads its three segments hi | lo | hi of
   * width a_seg from two bf16 buffers of row (pixel) stride a_seg: hi at A, lo at a_lo.
   * K-contiguous (lda = a_seg, K = 3 a_seg; a_seg % 8 == 0) or conv-forward A (a_seg % 64
   * == 0); not on the phased 256x256 tiles (7-9). */
  int32_t a_seg;
  const void* a_lo;
  /* 1 = interleaved pairs (with a_seg, a_seg % 32 == 0): K (conv: conv_c) = 2 a_seg, and each
   * 64-wide K-step is [hi | lo] of 32 real k -- A read so from the split pair, B stored so
   * (dfu_split_x3 / dfu_pack_conv_weight_x3 pattern 2); the kernel forms hi·hi + lo·hi + hi·lo
   * per step, the tripled-K sum from 2 operand tiles instead of 3.  Tiles 1, 2, 10, 11
   * (F32_STATS). */
  int32_t x3_pairs;
} dfu_gemm_desc;

int dfu_gemm(const dfu_gemm_desc* desc, void* stream);
/* 128-row blocks (rows of the stats slab) produced by DFU_EPI_BF16_STATS for M rows. */
int dfu_gemm_stats_tiles(int32_t M);
/* Workspace bytes for this descriptor: deterministic split-K slabs (F32_ACC) or tail-split
 * slabs (other epilogues); 0 if the launch needs none. */
int64_t dfu_gemm_workspace_bytes(const dfu_gemm_desc* desc);
/* The tile (1..11, as dfu_gemm_desc.tile) and split-K the cost model picks for this descriptor. */
int dfu_gemm_plan(const dfu_gemm_desc* desc, int32_t* tile, int32_t* split_k);
/* GEMM schedule switch (tests, A/B timing), a bit mask: bit 0 the generic tiles, bit 1 the
 * persistent phased 256-wide tiles; set = persistent workgroups, each walking several work units
 * as one continuous K-step stream; clear = one workgroup per work unit.  Default 2 (round 6).
 * Every setting gives bitwise-identical results.  Returns the previous mask. */
int dfu_gemm_set_persistent(int32_t mode);
/* Split-K reduction switch: 1 = inside the GEMM when the descriptor carries tile
 * counters, 0 (default: measured faster) = the separate reduce kernel.  Bitwise-identical; returns the
 * previous setting. */
int dfu_gemm_set_inkernel_reduce(int32_t enable);
/* Tail-split switch: 1 (default) = when the tiles of an unsplit launch leave a last, partial
 * round of workgroups, split each of those tiles along K over the idle workgroups (fp32 slabs
 * in the descriptor's workspace, dfu_gemm_workspace_bytes; the tile's last split to finish sums
 * them in split order and runs the epilogue; needs tile_counters).  0 = off.  Deterministic
 * either way (not bitwise equal to each other).  Returns the previous setting. */
int dfu_gemm_set_tail_split(int32_t enable);
/* Exact fp32 GEMM for the tiny fusion head (train_multimodal_fusion.py:305-313):
 * C[m][n] = accumulate*C[m][n] + sum_k A[m*sam + k*sak] * B[n*sbn + k*sbk] (+bias[n]) (relu). */
int dfu_gemm_f32(int32_t M, int32_t N, int32_t K, const float* A, int64_t sam, int64_t sak,
                 const float* B, int64_t sbn, int64_t sbk, float* C, int64_t ldc,
                 const float* bias, int32_t relu, int32_t accumulate, void* workspace,
                 int64_t workspace_bytes, void* stream);
/* Workspace for dfu_gemm_f32's deterministic split-K slabs (0 = runs unsplit). With a smaller
 * or NULL workspace dfu_gemm_f32 runs unsplit (correct, slower). */
int64_t dfu_gemm_f32_workspace_bytes(int32_t M, int32_t N, int32_t K);

/* ---------------------------------------------------------------- layout / packing -- */
/* fp32 OIHW conv weight -> bf16 KRSC ([K][R][S][C]) for the implicit-GEMM convs
 * (torchvision resnet.py conv3x3/conv1x1 weights; state_dict stays OIHW fp32). */
int dfu_pack_conv_weight(const float* w, void* out_bf16, int32_t K, int32_t C, int32_t R,
                         int32_t S, void* stream);
/* Conv weight gradient accumulated in KRSC fp32 (coalesced GEMM epilogue) -> ADD into the
 * OIHW fp32 parameter gradient: oihw[k][c][r][s] += krsc[k][r][s][c]. */
int dfu_conv_grad_krsc_to_oihw(const float* krsc, float* oihw, int32_t K, int32_t C, int32_t R,
                               int32_t S, void* stream);
/* fp32 [rows][cols] -> bf16 [rows][ld_out] (cols..ld_out-1 zero-filled). */
int dfu_cast_rows_bf16(const float* in, int64_t ld_in, void* out, int64_t ld_out, int32_t rows,
                       int32_t cols, void* stream);
/* Batched bf16 transpose: for each job, dst[c][r] = src[r][c] (src [rows][cols] with row
 * stride ld_src, dst [cols][rows] with row stride ld_dst, in elements, 0 = dense; rows, cols
 * and the strides multiples of 8, both 16-B aligned).  Keeps a transposed copy of the ViT
 * Linear weights' bf16 shadow so the input-gradient GEMMs read their weight operand
 * K-contiguous (dX = dY W: B = W^T [in][out]) instead of MN-major, and, one job per filter tap,
 * the flipped channel-transposed copy of the 3x3 conv weights the stride-1 conv dgrads run as
 * forward convolutions on (W'[c][R-1-r][S-1-s][k] = W[k][r][s][c]).  `jobs` lives in DEVICE
 * memory; job j covers the launch's 64x64 tiles [tile0_j, tile0_j + ceil(rows/64) *
 * ceil(cols/64)), in job order; `ntiles` is the total. */
typedef struct dfu_transpose_job {
  const void* src;
  void* dst;
  int32_t rows, cols;
  int32_t tile0;
  int32_t ld_src, ld_dst;
  int32_t pad_;
} dfu_transpose_job;
int dfu_transpose_bf16(const dfu_transpose_job* jobs, int32_t njobs, int32_t ntiles,
                       void* stream);
/* fp32 [rows][cols] -> fp16 [rows][ld_out] (RNE; cols..ld_out-1 zero-filled): the fp16
 * operands of the "parity" precision mode's ViT forward. */
int dfu_cast_rows_f16(const float* in, int64_t ld_in, void* out, int64_t ld_out, int32_t rows,
                      int32_t cols, void* stream);
/* bf16 [rows][cols] (ld_in) -> fp32 [rows][cols] (ld_out). */
int dfu_cast_rows_f32(const void* in, int64_t ld_in, float* out, int64_t ld_out, int32_t rows,
                      int32_t cols, void* stream);
/* Stem im2col (resnet conv1 7x7/s2/p3, train_multimodal_fusion.py:294): fp32 input with
 * arbitrary NCHW strides -> bf16 [B*P*Q][Kp], k = c*R*S + r*S + s (OIHW flatten order), any
 * Kp % 8 == 0 >= C*R*S (dfu_hip.nn.Conv2d's explicit path for other channel counts). */
int dfu_im2col_f32(const float* x, int64_t sn, int64_t sc, int64_t sh, int64_t sw, int32_t B,
                   int32_t C, int32_t H, int32_t W, int32_t R, int32_t S, int32_t stride,
                   int32_t pad, int32_t P, int32_t Q, void* out, int32_t Kp, void* stream);
/* ViT patchify (timm PatchEmbed.proj conv16/s16): fp32 strided input -> bf16
 * [B*(H/ps)*(W/ps)][C*ps*ps], k = c*ps*ps + kh*ps + kw. */
int dfu_patchify_f32(const float* x, int64_t sn, int64_t sc, int64_t sh, int64_t sw, int32_t B,
                     int32_t C, int32_t H, int32_t W, int32_t ps, void* out, void* stream);

/* ---------------------------------------------------------------- Grad-CAM (C5) ----- */
/* Input gradients of the two stems, which Grad-CAM needs (grad_cam_visualization.py:374-386:
 * the input requires grad) and the training step does not.
 * col2im: adjoint of dfu_im2col_f32 (resnet conv1): fp32 dcol [B*P*Q][Kp] -> fp32 NCHW dx. */
int dfu_col2im_f32(const float* dcol, int32_t B, int32_t C, int32_t H, int32_t W, int32_t R,
                   int32_t S, int32_t stride, int32_t pad, int32_t P, int32_t Q, int32_t Kp,
                   float* dx, void* stream);
/* unpatchify: adjoint of dfu_patchify_f32 (timm patch_embed.proj): fp32
 * [B*(H/ps)*(W/ps)][C*ps*ps] -> fp32 NCHW dx. */
int dfu_unpatchify_f32(const float* dpatch, int32_t B, int32_t C, int32_t H, int32_t W,
                       int32_t ps, float* dx, void* stream);
/* Grad-CAM map per image (grad_cam_visualization.py:415-429): w_c = mean_p grad[b][p][c] over
 * the Cg gradient channels, cam[b][p] = relu(sum_{c < min(Ca, Cg)} w_c act[b][p][c]) / max_p
 * (when > 0).  Per-tensor element strides (batch, position, channel): NCHW or channels_last
 * views; both bf16 or both fp32; cam fp32 [B][HW]. */
int dfu_gradcam(const void* act, int32_t Ca, int64_t sab, int64_t sap, int64_t sac,
                const void* grad, int32_t Cg, int64_t sgb, int64_t sgp, int64_t sgc,
                int32_t is_bf16, int32_t B, int32_t HW, float* cam, void* stream);
/* Input-gradient saliency (grad_cam_visualization.py:401-413, the ViT fallback):
 * out[b][p] = mean_c |dx[b][c][p]|, divided by its per-image max when that is > 0. */
int dfu_saliency(const float* dx, int32_t B, int32_t C, int32_t HW, float* out, void* stream);

/* ---------------------------------------------------------------- BatchNorm (train) -- */
/* torchvision BatchNorm2d(eps 1e-5, momentum 0.1) in training mode over NHWC [M][C].
 * finalize: combine the (sum, M2) tile slab of the producing GEMM into mean / invstd,
 * scale = gamma*invstd, shift = beta - mean*scale; update running stats (unbiased var) and
 * num_batches_tracked. */
int dfu_bn_finalize(const float* stats, int32_t tiles, int32_t M, int32_t C, const float* gamma,
                    const float* beta, float eps, float momentum, float* running_mean,
                    float* running_var, int64_t* num_batches, float* mean_out,
                    float* invstd_out, float* scale_out, float* shift_out, double* ws,
                    int32_t* counters, int32_t ncounters, void* stream);
/* With ws (dfu_bn_finalize_ws_bytes) and >= C/16 zeroed int32 counters (returned zeroed), the
 * tiles are reduced in parallel slices whose last block combines them in slice order (same
 * result for any arrival order); ws or counters NULL: one serial pass per channel group. */
int64_t dfu_bn_finalize_ws_bytes(int32_t tiles, int32_t C);
/* The per-128-row-tile (sum, M2) records of dfu_bn_finalize's `stats` ([ceil(M/128)][2][C],
 * M2 about the tile mean) computed from stored bf16 rows x[M][C] -- a BatchNorm2d that does not
 * follow a conv with the statistics epilogue (torch.nn.BatchNorm2d.forward, train mode). */
int dfu_bn_tile_stats(const void* x, int64_t M, int32_t C, float* stats, void* stream);
/* Eval-mode BN: scale/shift from running stats. */
int dfu_bn_eval_coeffs(const float* gamma, const float* beta, const float* running_mean,
                       const float* running_var, float eps, int32_t C, float* scale_out,
                       float* shift_out, void* stream);
/* out = act(y*scale[c] + shift[c] (+ residual)), bf16 NHWC; act = relu if relu != 0. */
int dfu_bn_apply(const void* y, const float* scale, const float* shift, const void* residual,
                 int32_t relu, void* out, int64_t M, int32_t C, void* stream);
/* dfu_bn_apply that also writes the ReLU mask of its output: bit e of mask[i] = (out element
 * 8i + e > 0), M*C/8 bytes (the backward's relu = 3 input; mask may be NULL). */
int dfu_bn_apply_mask(const void* y, const float* scale, const float* shift,
                      const void* residual, int32_t relu, void* out, uint8_t* mask, int64_t M,
                      int32_t C, void* stream);
/* Backward of out = act(bn(y) (+res)).  reduce: per-channel partial sums of g and g*xhat,
 * g = dout * mask; written as [blocks][2][C] (dfu_bn_bwd_blocks(M, C)).  relu: 0 no mask;
 * 1 mask = out > 0 (BN + residual + ReLU: reads out); 2 mask = y*scale + shift > 0 with the
 * forward's scale/shift (BN + ReLU, no residual: recomputed from y, out not read); 3 the same
 * mask as 1 from the bitmask dfu_bn_apply_mask wrote, passed as `out` (1/16 of the bytes). */
int dfu_bn_bwd_blocks(int64_t M, int32_t C);
int dfu_bn_bwd_reduce(const void* dout, const void* y, const void* out, int32_t relu,
                      const float* scale, const float* shift, const float* mean,
                      const float* invstd, int64_t M, int32_t C, float* partial, void* stream);
/* finalize: sums -> dgamma, dbeta (accumulated into grad buffers, may be NULL) and the
 * per-channel coefficients used by apply.  batch_stats = 0 for eval-mode BN (running
 * statistics are constants: dy = gamma*invstd*g). */
int dfu_bn_bwd_finalize(const float* partial, int32_t blocks, int64_t M, int32_t C,
                        const float* gamma, const float* invstd, int32_t batch_stats,
                        float* dgamma, float* dbeta, float* coef, double* ws, int32_t* counters,
                        int32_t ncounters, void* stream);
/* Workspace of dfu_bn_bwd_finalize's sliced form (as dfu_bn_finalize's). */
int64_t dfu_bn_bwd_finalize_ws_bytes(int32_t blocks, int32_t C);
/* dy = gamma*invstd*(g - mean(g) - xhat*mean(g*xhat)); optionally dres = g (bf16). */
int dfu_bn_bwd_apply(const void* dout, const void* y, const void* out, int32_t relu,
                     const float* scale, const float* shift, const float* mean,
                     const float* invstd, const float* coef, int64_t M, int32_t C, void* dy,
                     void* dres, void* stream);
/* The three above in one call (the same launches, bitwise the same results) on one workspace of
 * dfu_bn_bwd_ws_bytes(M, C) bytes, 16-B aligned: finalize slices, the partial sums and coef;
 * counters: zeroed per-stream tile counters (zero in, zero out) for the sliced finalize. */
int64_t dfu_bn_bwd_ws_bytes(int64_t M, int32_t C);
int dfu_bn_bwd(const void* dout, const void* y, const void* out, int32_t relu, const float* scale,
               const float* shift, const float* mean, const float* invstd, const float* gamma,
               int64_t M, int32_t C, int32_t batch_stats, float* dgamma, float* dbeta, void* dy,
               void* dres, void* ws, int64_t ws_bytes, int32_t* counters, int32_t ncounters,
               void* stream);

/* ---------------------------------------------------------------- pooling ----------- */
/* resnet maxpool 3x3/s2/p1 on NHWC bf16; argmax (0..8 window index) saved as uint8. */
int dfu_maxpool_fwd(const void* x, int32_t B, int32_t H, int32_t W, int32_t C, void* y,
                    uint8_t* argmax, int32_t P, int32_t Q, void* stream);
/* The stem's bn1 + relu + maxpool in one pass (resnet.py: maxpool(relu(bn1(conv1 x))))): x is
 * the conv output y, each window element is bf16(relu(y * scale + shift)) exactly as
 * dfu_bn_apply(relu=1) stores it, so y/argmax equal dfu_bn_apply followed by dfu_maxpool_fwd
 * bit for bit.  scale = shift = NULL is dfu_maxpool_fwd. */
int dfu_maxpool_bn_fwd(const void* x, const float* scale, const float* shift, int32_t B,
                       int32_t H, int32_t W, int32_t C, void* y, uint8_t* argmax, int32_t P,
                       int32_t Q, void* stream);
int dfu_maxpool_bwd(const void* dy, const uint8_t* argmax, int32_t B, int32_t H, int32_t W,
                    int32_t C, int32_t P, int32_t Q, void* dx, void* stream);
/* resnet AdaptiveAvgPool2d(1) + flatten: NHWC bf16 [B][HW][C] -> fp32 [B][C]. */
int dfu_avgpool_fwd(const void* x, int32_t B, int32_t HW, int32_t C, float* y, void* stream);
int dfu_avgpool_bwd(const float* dy, int32_t B, int32_t HW, int32_t C, void* dx, void* stream);

/* ---------------------------------------------------------------- LayerNorm --------- */
/* timm LayerNorm(eps 1e-6) over rows of D: fp32 x (row stride ldx) -> out (bf16 if
 * out_bf16 else fp32, row stride ldo); saves mean / rstd per row. */
int dfu_layernorm_fwd(const float* x, int64_t ldx, int32_t rows, int32_t D, const float* gamma,
                      const float* beta, float eps, void* out, int64_t ldo, int32_t out_bf16,
                      float* mean, float* rstd, void* stream);
/* dx (fp32, += into gx which is also read as the incoming residual grad) and a bf16 copy of
 * the updated residual grad; dgamma/dbeta partials [blocks][2][D] (dfu_ln_bwd_blocks).
 * gsum_partial (optional, [blocks][D]): column sums of the UPDATED gx — the bias gradient of
 * the Linear whose output is that residual stream (timm Block proj / fc2), so no separate
 * pass over the fp32 gradient is needed. */
int dfu_ln_bwd_blocks(int32_t rows);
int dfu_layernorm_bwd(const void* dy, int64_t lddy, int32_t dy_bf16, const float* x,
                      int64_t ldx, const float* mean, const float* rstd, const float* gamma,
                      int32_t rows, int32_t D, float* gx, int64_t ldg, void* gx_bf16,
                      float* partial, float* gsum_partial, void* stream);
/* Sum a [blocks][nvec][D] partial slab over blocks and ADD into out[v] (v < nvec). */
int dfu_reduce_partials(const float* partial, int32_t blocks, int32_t nvec, int32_t D,
                        float* out0, float* out1, void* stream);
/* Several such reductions in one launch: out[d] += sum_b partial[b * stride + d], d < D, per
 * entry (host array of n <= DFU_REDUCE_BATCH entries; same sums as dfu_reduce_partials). */
#define DFU_REDUCE_BATCH 8
typedef struct dfu_reduce_entry {
  const float* partial;
  int64_t stride; /* elements between consecutive blocks' rows */
  float* out;
  int32_t blocks;
  int32_t D;
} dfu_reduce_entry;
int dfu_reduce_partials_batch(const dfu_reduce_entry* entries, int32_t n, void* stream);

/* ---------------------------------------------------------------- attention --------- */
/* timm Attention with F.scaled_dot_product_attention: qkv bf16 [B*N][3][H][dh] (the qkv
 * Linear output), o bf16 [B*N][H][dh], lse fp32 [B*H][Npad]. dh == 64, N <= 256. */
int dfu_attention_fwd(const void* qkv, int32_t B, int32_t N, int32_t H, int32_t dh, float scale,
                      void* o, float* lse, void* stream);
/* The "parity" precision mode's fp16 forward: qkv fp16 (the DFU_EPI_F16_DUAL output), the same
 * kernel on v_mfma_f32_16x16x32_f16 with fp16 probabilities; o fp16 (the proj GEMM's operand)
 * and o_bf16 (what the bf16 backward reads), lse as dfu_attention_fwd. */
int dfu_attention_fwd_f16(const void* qkv, int32_t B, int32_t N, int32_t H, int32_t dh,
                          float scale, void* o, void* o_bf16, float* lse, void* stream);
/* Backward: writes dq, dk, dv into dqkv (same layout as qkv); delta scratch [B*H][Npad]. */
int dfu_attention_bwd(const void* qkv, const void* o, const void* dout, const float* lse,
                      int32_t B, int32_t N, int32_t H, int32_t dh, float scale, float* delta,
                      void* dqkv, void* stream);
/* The same backward reading the "parity" forward's fp16 qkv (rounded to bf16 while staging: no
 * bf16 copy of qkv is stored in the forward); o, dout and dqkv bf16 as above. */
int dfu_attention_bwd_qkv16(const void* qkv16, const void* o, const void* dout, const float* lse,
                            int32_t B, int32_t N, int32_t H, int32_t dh, float scale,
                            float* delta, void* dqkv, void* stream);
int dfu_attention_npad(int32_t N);

/* ---------------------------------------------------------------- ViT embedding ----- */
/* Row 0 of every image: x[b][0][:] = cls + pos[0] (timm _pos_embed, class token). */
int dfu_vit_cls_rows(const float* cls, const float* pos, float* x, int32_t B, int32_t T,
                     int32_t D, void* stream);
/* Backward of the embedding sum: from gx fp32 [B][T][D]:
 *   dcls += sum_b gx[b][0], dpos[t] += sum_b gx[b][t], dbias += sum_{b,t>0} gx[b][t],
 *   gpatch bf16 [B*(T-1)][D] = gx[:,1:]. */
int dfu_vit_embed_bwd(const float* gx, int32_t B, int32_t T, int32_t D, float* dcls,
                      float* dpos, float* dbias, void* gpatch, float* partial, void* stream);

/* ---------------------------------------------------------------- elementwise ------- */
/* Column sums of a bf16/fp32 [rows][N] matrix ADDED into out fp32 [N] (bias grads); out NULL:
 * only the per-block partials [dfu_colsum_blocks(rows)][N] are written. */
int dfu_colsum(const void* x, int32_t is_bf16, int64_t ld, int32_t rows, int32_t N, float* out,
               float* partial, void* stream);
int dfu_colsum_blocks(int32_t rows);
/* Gather rows: out[i][:] = in[i*stride + offset][:] (fp32 -> fp32), D columns. */
int dfu_gather_rows_f32(const float* in, int64_t ld_in, int32_t stride, int32_t offset,
                        int32_t rows, int32_t D, float* out, int64_t ld_out, void* stream);
/* Scatter rows (add): out[i*stride + offset][:] += in[i][:] (fp32). */
int dfu_scatter_rows_f32(const float* in, int64_t ld_in, int32_t stride, int32_t offset,
                         int32_t rows, int32_t D, float* out, int64_t ld_out, void* stream);
/* y = relu(x) / dx = dy * (y > 0), bf16 or fp32 (is_bf16). */
int dfu_relu_fwd(const void* x, void* y, int64_t n, int32_t is_bf16, void* stream);
int dfu_relu_bwd(const void* dy, const void* y, void* dx, int64_t n, int32_t is_bf16,
                 void* stream);
/* Inverted dropout (nn.Dropout training mode): counter-based hash RNG keyed by
 * (seed, *offset_dev); mask saved as uint8; offset advanced on device (graph-replay safe). */
int dfu_dropout_fwd(const void* x, void* y, uint8_t* mask, int64_t n, float p, uint64_t seed,
                    int64_t* offset_dev, int32_t is_bf16, void* stream);
int dfu_dropout_bwd(const void* dy, const uint8_t* mask, void* dx, int64_t n, float p,
                    int32_t is_bf16, void* stream);
/* Copy two fp32/bf16 feature matrices into one concatenated bf16 buffer (torch.cat at
 * train_multimodal_fusion.py:321) and its backward split. */
int dfu_concat2_bf16(const void* a, int32_t a_bf16, int32_t Na, const void* b, int32_t b_bf16,
                     int32_t Nb, int32_t rows, void* out, void* stream);
int dfu_split2_f32(const void* g, int32_t g_bf16, int32_t rows, int32_t Na, int32_t Nb,
                   float* ga, float* gb, void* stream);

/* ---------------------------------------------------------------- loss / optimizer -- */
/* nn.CrossEntropyLoss(weight=w) mean reduction (train_multimodal_fusion.py:342-346,376):
 * loss = sum_i w[y_i]*(lse_i - z_i[y_i]) / sum_i w[y_i]; dlogits = grad*d(loss)/dz. */
int dfu_ce_weighted_fwd(const float* logits, const int64_t* labels, const float* weight,
                        int32_t B, int32_t C, float* loss, float* dlogits, void* stream);
int dfu_ce_weighted_bwd(const float* dlogits_saved, const float* grad_loss, int32_t B,
                        int32_t C, float* dlogits, void* stream);
/* torch.optim.AdamW (lr, betas, eps, weight_decay) over a table of tensors
 * (train_multimodal_fusion.py:347,380).  step_dev is an int64 device counter incremented by
 * the launch (graph-capturable bias correction).  Tensors are described by device arrays of
 * pointers and element counts. */
int dfu_adamw(float* const* params, float* const* grads, float* const* exp_avg,
              float* const* exp_avg_sq, const int64_t* numels, int32_t ntensors,
              const int64_t* chunk_offsets, int32_t nchunks, float lr, float beta1,
              float beta2, float eps, float weight_decay, int64_t* step_dev, void* stream);
/* Flat form: one contiguous buffer of n parameters (the fused flat-parameter layout).
 * shadow_bf16 (optional, n bf16): also receives bf16(updated param) — the GEMM operand copy
 * of every weight, so the forward pass needs no cast kernels; shadow_f16 (optional, n fp16):
 * fp16(updated param), the operands of the "parity" precision mode's fp16 ViT forward;
 * shadow_x3 (optional, bf16, 2 (x3_end - x3_begin) elements): elements [x3_begin, x3_end) of
 * the range split into interleaved pairs, per 32-element block [hi 32 | lo 32] (hi =
 * bf16(p), lo = bf16(p - hi)) -- for conv weights of C % 32 == 0 channels starting on a
 * 32-element boundary, exactly the dfu_gemm_desc.x3_pairs B operand (dfu_split_x3 /
 * dfu_pack_conv_weight_x3 pattern 2), so the bf16x3 ResNet forward needs no per-layer split
 * launches.  x3_begin % 4 == 0, (x3_end - x3_begin) % 32 == 0, x3_end <= n rounded down to 4. */
int dfu_adamw_flat(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                   float lr, float beta1, float beta2, float eps, float weight_decay,
                   const int64_t* step_dev, void* shadow_bf16, void* shadow_f16, void* shadow_x3,
                   int64_t x3_begin, int64_t x3_end, void* stream);
int dfu_step_increment(int64_t* step_dev, void* stream);
/* argmax over C for each row (torch.max(outputs, 1), :384) -> int64. */
int dfu_argmax_rows(const float* x, int32_t rows, int32_t C, int64_t* out, void* stream);
/* torch.softmax(outputs, dim=1) over fp32 rows of C logits (the test phase's ulcer
 * probability softmax[:, 1], train_multimodal_fusion.py:477) -> fp32 [rows][C]. */
int dfu_softmax_rows(const float* x, int32_t rows, int32_t C, float* out, void* stream);
/* The per-step metrics of train_multimodal_fusion.py:383-388 (loss.item(), torch.max(outputs,
 * 1), .cpu()) accumulated on the device, read back once per epoch: confusion int64 [C][C]
 * (row = label, column = argmax, first maximum wins) += 1 per row; *loss_sum (fp64) += *loss
 * (if loss != NULL); *batches += 1.  Exact, order-independent totals. */
int dfu_metrics_accumulate(const float* logits, const int64_t* labels, int32_t rows, int32_t C,
                           const float* loss, int64_t* confusion, double* loss_sum,
                           int64_t* batches, void* stream);

/* ---------------------------------------------------------------- bf16x3 forward ---- */
/* The "bf16x3" precision mode (csrc/precise.hip): the forward pass of the training step at
 * fp32 accuracy on the bf16 MFMA GEMM, so the fusion logits meet north_star's 1e-3 bar against
 * the reference's fp32 CPU path.  A contraction A.B^T runs as one GEMM over a tripled K with
 * A3 = [hi(A) | lo(A) | hi(A)] ("pattern 0"), B3 = [hi(B) | hi(B) | lo(B)] ("pattern 1"),
 * hi = bf16(x), lo = bf16(x - hi); a triple is bf16 [rows][3C].  GEMM outputs stay fp32
 * (DFU_EPI_F32 / F32_RESID / F32_STATS / PATCH); the kernels below also write the plain bf16
 * tensors the (bf16) backward pass saves.  Reference ops: the same as their bf16 twins above. */
/* fp32 [rows][cols] (ld_in) -> triple [rows][3 seg] of `pattern`, seg >= cols (seg % 8 == 0,
 * columns past cols zero); optional plain bf16 copy hi_out [rows][ld_hi >= seg].  Pattern 2:
 * interleaved pairs [rows][2 seg] (seg % 32 == 0), per 32 columns [hi 32 | lo 32] (the B
 * operand of dfu_gemm_desc.x3_pairs). */
int dfu_split_x3(const float* in, int64_t ld_in, int32_t rows, int32_t cols, int32_t seg,
                 void* out, int32_t pattern, void* hi_out, int64_t ld_hi, void* stream);
/* fp32 OIHW conv weight -> bf16 KRSC': pattern 1, C' = 3C along the channels; pattern 2,
 * C' = 2C interleaved pairs (C % 32 == 0; dfu_gemm_desc.x3_pairs). */
int dfu_pack_conv_weight_x3(const float* w, void* out, int32_t K, int32_t C, int32_t R, int32_t S,
                            int32_t pattern, void* stream);
/* dfu_im2col_f32 writing the split pair: hi rows to out, lo rows to out_lo (row stride Kp each:
 * the stem GEMM's split-pair A, dfu_gemm_desc.a_seg = Kp); dfu_patchify_f32_x3 writes the
 * pattern-0 triple (row stride 3 K). */
int dfu_im2col_f32_x3(const float* x, int64_t sn, int64_t sc, int64_t sh, int64_t sw, int32_t B,
                      int32_t C, int32_t H, int32_t W, int32_t R, int32_t S, int32_t stride,
                      int32_t pad, int32_t P, int32_t Q, void* out, void* out_lo, int32_t Kp,
                      void* stream);
int dfu_patchify_f32_x3(const float* x, int64_t sn, int64_t sc, int64_t sh, int64_t sw, int32_t B,
                        int32_t C, int32_t H, int32_t W, int32_t ps, void* out, void* stream);
/* BN apply on the conv output y: v = act(y*scale + shift (+ residual)).  y is fp32 [M][C]
 * (y_lo null) or the split pair the F32_STATS epilogue writes with aux_out (y = hi, y_lo = lo,
 * bf16 each; hi is then the BN backward's bf16 y and y_bf16 is not written).  Residual mode 0
 * none, 1 fp32 [M][C], 2 split pair (residual = hi, residual_lo = lo, [M][C] bf16 each).
 * Optional outputs: the split pair out_bf16 (hi, also the plain bf16 activation) + out_lo
 * (out_lo requires out_bf16), out_f32, y_bf16 (= bf16(y) for an fp32 y), relu_mask (M*C/8
 * bytes: bit k of byte i = output element 8i + k > 0, the dfu_bn_bwd_* relu = 3 mask). */
int dfu_bn_apply_x3(const void* y, const void* y_lo, const float* scale, const float* shift,
                    const void* residual, const void* residual_lo, int32_t res_mode, int32_t relu,
                    void* out_lo, void* out_bf16, float* out_f32, void* y_bf16,
                    uint8_t* relu_mask, int64_t M, int32_t C, void* stream);
/* resnet maxpool 3x3/s2/p1 on fp32 NHWC -> split pair (y_bf16 = hi, y_lo) and uint8 argmax. */
int dfu_maxpool_fwd_x3(const float* x, int32_t B, int32_t H, int32_t W, int32_t C, void* y_lo,
                       void* y_bf16, uint8_t* argmax, int32_t P, int32_t Q, void* stream);
/* AdaptiveAvgPool2d(1) on a split pair (hi, lo: [B*HW][C] bf16 each) -> fp32 [B][C]. */
/* The bf16x3 stem convolution (torchvision resnet50 conv1 7x7/s2/p3, 3 -> 64 channels; the
 * "parity" mode) as one implicit-GEMM kernel: x fp32 NCHW with element strides (sn, sc, sh,
 * sw), w fp32 OIHW [64][3][7][7] -> the conv output as a split pair y / y_lo (bf16 [B*P*Q][64]
 * each: hi = bf16(v), lo = bf16(v - hi)), the BN tile statistics stats [B*P*Q / 128][2][64]
 * (sum, M2 of each 128-row block, as the F32_STATS epilogue) and optionally col, the hi
 * im2col rows [B*P*Q][160] bf16 (taps 147.. zero; the library's own backward reads x instead:
 * dfu_stem_wgrad_x3).  The same fp32
 * values as dfu_im2col_f32_x3 + the interleaved-pair dfu_gemm, without the pair im2col in
 * HBM.  Needs P*Q % 128 == 0, Q >= 64, W <= 250. */
int dfu_stem_conv_x3(const float* x, int64_t sn, int64_t sc, int64_t sh, int64_t sw, int32_t B,
                     int32_t C, int32_t H, int32_t W, const float* w, int32_t K, int32_t R,
                     int32_t S, int32_t stride, int32_t pad, void* y, void* y_lo, float* stats,
                     void* col, void* stream);
/* The bf16x3 stem's weight gradient without im2col rows (replaces the MN x MN F32_ACC dfu_gemm
 * over col in StemFn.backward, resnet50 conv1 weight.grad): dw [64][147] fp32 (OIHW order,
 * contiguous) += sum over the B*P*Q output pixels m of dy[m][n] * bf16(x at tap k of m), from
 * x fp32 NCHW with element strides (sn, sc, sh, sw) and dy bf16 [B*P*Q][64] (16-B aligned).
 * Deterministic: per-workgroup partials into slab (dfu_stem_wgrad_ws_bytes bytes), summed in a
 * fixed order.  The 7x7/s2/p3 3 -> 64 stem with P even, Q % 16 == 0, Q <= 112, W <= 250. */
int64_t dfu_stem_wgrad_ws_bytes(int32_t B, int32_t H, int32_t W);
int dfu_stem_wgrad_x3(const float* x, int64_t sn, int64_t sc, int64_t sh, int64_t sw, int32_t B,
                      int32_t C, int32_t H, int32_t W, const void* dy, int32_t K, int32_t R,
                      int32_t S, int32_t stride, int32_t pad, float* dw, float* slab,
                      int64_t slab_bytes, void* stream);
/* bn1 + ReLU + maxpool 3x3/s2/p1 of the bf16x3 stem in one pass (bitwise dfu_bn_apply_x3 with
 * out_f32 then dfu_maxpool_fwd_x3, without the fp32 intermediate): the conv output split pair
 * y / y_lo (bf16 NHWC [B*H*W][C] each), BN scale / shift (fp32 [C], 16-B aligned) -> pooled
 * pair out_bf16 / out_lo [B*P*Q][C], argmax (uint8, window index) and optionally the BN
 * backward's ReLU bitmask (bit k of byte i: element 8i + k > 0), each input element written
 * once.  P = (H - 1) / 2 + 1, Q = (W - 1) / 2 + 1; C / 8 a power of two.  Replaces the
 * torchvision stem's bn1 / relu / maxpool (resnet.py _forward_impl) in the parity mode. */
int dfu_maxpool_bn_fwd_x3(const void* y, const void* y_lo, const float* scale, const float* shift,
                          int32_t B, int32_t H, int32_t W, int32_t C, void* out_lo,
                          void* out_bf16, uint8_t* argmax, uint8_t* relu_mask, int32_t P,
                          int32_t Q, void* stream);
int dfu_avgpool_fwd_x3(const void* hi, const void* lo, int32_t B, int32_t HW, int32_t C, float* y,
                       void* stream);
/* timm LayerNorm -> triple [rows][3D] + plain bf16 [rows][D]; mean / rstd per row. */
int dfu_layernorm_fwd_x3(const float* x, int64_t ldx, int32_t rows, int32_t D,
                         const float* gamma, const float* beta, float eps, void* out3,
                         void* out_bf16, float* mean, float* rstd, void* stream);
/* timm LayerNorm -> fp16 [rows][D] (the fp16 forward's GEMM operand) + plain bf16 [rows][D];
 * mean / rstd per row. */
int dfu_layernorm_fwd_h16(const float* x, int64_t ldx, int32_t rows, int32_t D,
                          const float* gamma, const float* beta, float eps, void* out_f16,
                          void* out_bf16, float* mean, float* rstd, void* stream);
/* exact GELU of the fp32 fc1 output -> triple [rows][3N], bf16 h and bf16 gelu'(pre) (the
 * DFU_EPI_BF16_DGELU operand, as DFU_EPI_BF16_GELU's aux_out). */
int dfu_gelu_x3(const float* hpre, int64_t rows, int32_t N, void* h3, void* h_bf16,
                void* dgelu_bf16, void* stream);
/* fp32-accurate softmax attention (SDPA) on the fp32 qkv GEMM output [B*N][3][H][dh]: the
 * bf16 MFMA attention on split operands (S = Qhi Khi + Qhi Klo + Qlo Khi, O = Phi Vhi + Plo Vhi +
 * Phi Vlo, fp32 softmax; ~2^-17 relative per product) -> o triple [B*N][3*H*dh], o bf16, lse
 * fp32 [B*H][npad] (as dfu_attention_fwd's: the bf16 backward's inputs) and, when qkv_bf16 is
 * not NULL, the plain bf16 copy of qkv (the backward's operand).  dh == 64, N <= 224. */
int dfu_attention_fwd_f32(const float* qkv, int32_t B, int32_t N, int32_t H, int32_t dh,
                          float scale, int32_t npad, void* qkv_bf16, void* o3, void* o_bf16,
                          float* lse, void* stream);

/* ---------------------------------------------------------------- input pipeline ---- */
/* The torchvision transforms of train_multimodal_fusion.py:172-205 on a decoded batch,
 * bit-exact with torchvision's PIL backend (replaces the DataLoader workers' per-sample
 * transform calls, :270-275 and MultimodalDataset.__getitem__ :151-165; decode stays PIL). */
typedef struct dfu_resize_desc {
  int64_t src_off;  /* byte offset of the image in the packed source (H x W x 3 u8) */
  int64_t tmp_off;  /* byte offset of its horizontal-pass rows (h x out_w x 3) in the scratch */
  int64_t coef_off; /* int32 offset of its taps: [out_w][2] bounds, [out_w][ksh] weights,
                       [out_h][2] bounds, [out_h][ksv] weights (dfu_resize_coeffs) */
  int32_t w, h;     /* source size */
  int32_t ksh, ksv; /* tap counts of the two passes (dfu_resize_ksize) */
} dfu_resize_desc;

enum dfu_aug_op { DFU_AUG_BRIGHTNESS = 0, DFU_AUG_CONTRAST = 1, DFU_AUG_SATURATION = 2 };

/* Per-image random parameters, drawn on the host in torchvision's order.  rot / aff are PIL's
 * 16.16 fixed-point inverse maps (Geometry.c affine_fixed): a0 a1 a2' a3 a4 a5' with the
 * half-pixel terms folded into a2' / a5'. */
typedef struct dfu_aug_params {
  int32_t hflip, vflip;
  int32_t rotate;
  int32_t rot[6];
  int32_t affine;
  int32_t aff[6];
  int32_t n_ops;     /* ColorJitter ops applied, in order (RandomApply may give 0) */
  int32_t op[3];     /* enum dfu_aug_op */
  float factor[3];   /* ImageEnhance factors of op[k] */
} dfu_aug_params;

/* Host-only (no GPU): taps of one bilinear antialiased resize pass (PIL Resample.c
 * precompute_coeffs + normalize_coeffs_8bpc).  ksize = dfu_resize_ksize(in, out);
 * bounds [out][2] = (first source index, count), kk [out][ksize] 22-bit fixed point. */
int dfu_resize_ksize(int32_t in_size, int32_t out_size);
int dfu_resize_coeffs(int32_t in_size, int32_t out_size, int32_t* bounds, int32_t* kk);
/* Resize n packed images to out_h x out_w (HWC u8): tmp holds sum_i h_i*out_w*3 bytes,
 * dst n*out_h*out_w*3.  descs and coefs are device arrays; src is read in whole aligned
 * dwords, so it must stay readable up to 3 bytes past the last image. */
int dfu_resize_batch(const uint8_t* src, const dfu_resize_desc* descs, const int32_t* coefs,
                     int32_t n, int32_t out_w, int32_t out_h, uint8_t* tmp, uint8_t* dst,
                     void* stream);
/* Flips, rotation, colour jitter, affine, ToTensor and Normalize on n resized H x W x 3 u8
 * images -> out fp32 [n][3][H][W].  params and contrast_means (n int32 scratch) are device
 * arrays (contrast_means receives the per-image grey sums); mean3 / std3 are host
 * arrays of 3 floats. */
int dfu_augment_normalize(const uint8_t* img, const dfu_aug_params* params, int32_t n,
                          int32_t H, int32_t W, const float* mean3, const float* std3,
                          int32_t* contrast_means, float* out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* DFU_HIP_H */
