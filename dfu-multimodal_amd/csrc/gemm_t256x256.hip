// GEMM instantiations, 256x256 tiles (2-stage ring; long-K weight gradients, big products).
#include "gemm_table.h"
#define E(A, B, Ep) DFU_ENTRY(A, B, Ep, 256, 256, dfu::T256x256)
namespace dfu {
const Entry kTable256x256[] = {
    E(DFU_OPND_KMAJOR, DFU_OPND_KMAJOR, DFU_EPI_BF16),
    E(DFU_OPND_KMAJOR, DFU_OPND_KMAJOR, DFU_EPI_BF16_GELU),
    E(DFU_OPND_KMAJOR, DFU_OPND_KMAJOR, DFU_EPI_F32_RESID),
    E(DFU_OPND_KMAJOR, DFU_OPND_MNMAJOR, DFU_EPI_BF16),
    E(DFU_OPND_KMAJOR, DFU_OPND_MNMAJOR, DFU_EPI_BF16_DGELU),
    E(DFU_OPND_MNMAJOR, DFU_OPND_MNMAJOR, DFU_EPI_F32_ACC),
    E(DFU_OPND_MNMAJOR, DFU_OPND_CONV_WGRAD_X, DFU_EPI_F32_ACC),
};
const int kTable256x256N = sizeof(kTable256x256) / sizeof(Entry);
}  // namespace dfu
