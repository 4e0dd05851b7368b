// GEMM instantiations, 256x64 tiles of 4 waves (2x2, 128x32 per wave), one workgroup per CU
// (3-stage ring, 120 KiB LDS): the ResNet's 64-channel outputs (stem, layer-1 convs), where a
// 128-column tile leaves half of every MFMA's columns unused.  K-contiguous / implicit-conv A,
// K-contiguous B (the MN-major loader works in 128-column sub-images).
#include "gemm_table.h"
#define E(A, B, Ep) DFU_ENTRY_W4(A, B, Ep, 256, 64, 1, dfu::T256x64)
#define EX(A, B, Ep) DFU_ENTRY_X3(A, B, Ep, 256, 64, 1, 4, dfu::T256x64)
namespace dfu {
const Entry kTable256x64[] = {
    E(DFU_OPND_KMAJOR, DFU_OPND_KMAJOR, DFU_EPI_BF16),
    E(DFU_OPND_KMAJOR, DFU_OPND_KMAJOR, DFU_EPI_BF16_STATS),
    E(DFU_OPND_KMAJOR, DFU_OPND_KMAJOR, DFU_EPI_F32_STATS),
    E(DFU_OPND_KMAJOR, DFU_OPND_KMAJOR, DFU_EPI_BF16_ADD),  // 1x1 dgrad on the transposed weight
    E(DFU_OPND_CONV_FWD, DFU_OPND_KMAJOR, DFU_EPI_BF16_STATS),
    E(DFU_OPND_CONV_FWD, DFU_OPND_KMAJOR, DFU_EPI_F32_STATS),
    E(DFU_OPND_CONV_FWD, DFU_OPND_KMAJOR, DFU_EPI_BF16),  // stride-1 dgrad on flipped weights
    // bf16x3 forward on interleaved split pairs (dfu_gemm_desc.x3_pairs)
    EX(DFU_OPND_KMAJOR, DFU_OPND_KMAJOR, DFU_EPI_F32_STATS),
    EX(DFU_OPND_CONV_FWD, DFU_OPND_KMAJOR, DFU_EPI_F32_STATS),
};
const int kTable256x64N = sizeof(kTable256x64) / sizeof(Entry);
}  // namespace dfu
