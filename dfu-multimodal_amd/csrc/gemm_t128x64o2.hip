// GEMM instantiations, 128x64 tiles of 4 waves (2x2, 64x32 per wave), two workgroups per CU
// (2-stage ring, 48 KiB LDS each): the ResNet's 64-channel outputs (stem, layer-1 convs), where a
// 128-column tile leaves half of every MFMA's columns unused.  K-contiguous / implicit-conv A,
// K-contiguous B (the MN-major loader works in 128-column sub-images).
#include "gemm_table.h"
#define E(A, B, Ep) DFU_ENTRY_W4(A, B, Ep, 128, 64, 2, dfu::T128x64o2)
#define EX(A, B, Ep) DFU_ENTRY_X3(A, B, Ep, 128, 64, 2, 4, dfu::T128x64o2)
namespace dfu {
const Entry kTable128x64o2[] = {
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
const int kTable128x64o2N = sizeof(kTable128x64o2) / sizeof(Entry);
}  // namespace dfu
