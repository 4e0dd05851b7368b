// GEMM instantiations, 128x128 tiles at 2 workgroups per CU (2-stage ring, 64 KiB LDS):
// memory-bound shapes (small K or small N) overlap one workgroup's loads/epilogue with the other.
#include "gemm_table.h"
#define E(A, B, Ep) DFU_ENTRY_OCC(A, B, Ep, 128, 128, 2, dfu::T128x128o2)
#define EX(A, B, Ep) DFU_ENTRY_X3(A, B, Ep, 128, 128, 2, 8, dfu::T128x128o2)
namespace dfu {
const Entry kTable128x128o2[] = {
    E(DFU_OPND_KMAJOR, DFU_OPND_KMAJOR, DFU_EPI_BF16),
    E(DFU_OPND_KMAJOR, DFU_OPND_KMAJOR, DFU_EPI_BF16_RELU),
    E(DFU_OPND_KMAJOR, DFU_OPND_KMAJOR, DFU_EPI_BF16_GELU),
    E(DFU_OPND_KMAJOR, DFU_OPND_KMAJOR, DFU_EPI_F32),
    E(DFU_OPND_KMAJOR, DFU_OPND_KMAJOR, DFU_EPI_F32_RESID),
    E(DFU_OPND_KMAJOR, DFU_OPND_KMAJOR, DFU_EPI_PATCH),
    E(DFU_OPND_KMAJOR, DFU_OPND_KMAJOR, DFU_EPI_BF16_STATS),
    E(DFU_OPND_KMAJOR, DFU_OPND_MNMAJOR, DFU_EPI_BF16),
    E(DFU_OPND_KMAJOR, DFU_OPND_MNMAJOR, DFU_EPI_BF16_DGELU),
    E(DFU_OPND_KMAJOR, DFU_OPND_MNMAJOR, DFU_EPI_BF16_ADD),
    E(DFU_OPND_KMAJOR, DFU_OPND_MNMAJOR, DFU_EPI_F32),
    E(DFU_OPND_MNMAJOR, DFU_OPND_MNMAJOR, DFU_EPI_F32_ACC),
    E(DFU_OPND_CONV_FWD, DFU_OPND_KMAJOR, DFU_EPI_BF16_STATS),
    // split-K forms of the bf16x3 forward's long-K, few-tile convolutions (fp32 slabs; the BN
    // statistics and the output pair by dfu_stats_pair_f32 after the reduction)
    E(DFU_OPND_KMAJOR, DFU_OPND_KMAJOR, DFU_EPI_F32_ACC),
    E(DFU_OPND_CONV_FWD, DFU_OPND_KMAJOR, DFU_EPI_F32_ACC),
    E(DFU_OPND_CONV_FWD, DFU_OPND_KMAJOR, DFU_EPI_BF16),  // stride-1 dgrad on flipped weights
    E(DFU_OPND_CONV_DGRAD, DFU_OPND_CONV_DGRAD_W, DFU_EPI_BF16),
    E(DFU_OPND_CONV_DGRAD, DFU_OPND_CONV_DGRAD_W, DFU_EPI_BF16_ADD),
    E(DFU_OPND_MNMAJOR, DFU_OPND_CONV_WGRAD_X, DFU_EPI_F32_ACC),
    // bf16x3 forward on interleaved split pairs (dfu_gemm_desc.x3_pairs)
    EX(DFU_OPND_KMAJOR, DFU_OPND_KMAJOR, DFU_EPI_F32_ACC),
    EX(DFU_OPND_CONV_FWD, DFU_OPND_KMAJOR, DFU_EPI_F32_ACC),
};
const int kTable128x128o2N = sizeof(kTable128x128o2) / sizeof(Entry);
}  // namespace dfu
