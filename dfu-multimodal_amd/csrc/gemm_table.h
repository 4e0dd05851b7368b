// Dispatch-table entries of the GEMM template, one table per tile shape (gemm_t*.hip).
#pragma once
#include "gemm_kernel.h"

namespace dfu {
typedef void (*gemm_fn)(const GemmArgs);
// Entry.e of an fp16-operand kernel (dfu_gemm_desc.operand_type 1): the epilogue | kF16Key
constexpr int kF16Key = 64;
// Entry.e of an interleaved-pair bf16x3 kernel (dfu_gemm_desc.x3_pairs): the epilogue | kX3Key
constexpr int kX3Key = 128;
struct Entry {
  int a, b, e, tile;
  gemm_fn fn;
  int lds_bytes;
  int threads;
};
enum TileId {
  T128x128 = 0, T256x128 = 1, T128x256 = 2, T256x256 = 3, T128x128o2 = 4, T128x128w4 = 5,
  T256x256p8 = 6,  // phased 256x256 (gemm_p8.hip): K-contiguous A and B only
  T256x256ps = 7,  // persistent phased 256x256 (gemm_ps.hip)
  T192x256ps = 8,  // persistent phased 192x256 (gemm_ps.hip): K-contiguous A
  T256x64 = 9,     // 4-wave 256x64 (64-channel convs; K-contiguous B)
  T128x64o2 = 10,  // 4-wave 128x64 at 2 workgroups per CU
  NTILES = 11
};
extern const Entry kTable128x128[];
extern const int kTable128x128N;
extern const Entry kTable256x128[];
extern const int kTable256x128N;
extern const Entry kTable128x256[];
extern const int kTable128x256N;
extern const Entry kTable256x256[];
extern const int kTable256x256N;
extern const Entry kTable128x128o2[];
extern const int kTable128x128o2N;
extern const Entry kTable128x128w4[];
extern const int kTable128x128w4N;
extern const Entry kTable256x256p8[];
extern const int kTable256x256p8N;
extern const Entry kTable256x256ps[];
extern const int kTable256x256psN;
extern const Entry kTable192x256ps[];
extern const int kTable192x256psN;
extern const Entry kTable256x64[];
extern const int kTable256x64N;
extern const Entry kTable128x64o2[];
extern const int kTable128x64o2N;
}  // namespace dfu

#define DFU_ENTRY(A, B, E, TMv, TNv, TID)                                             \
  {                                                                                   \
    A, B, E, TID, &dfu::gemm_kernel<A, B, E, TMv, TNv>, dfu::Tile<TMv, TNv>::LDS_BYTES, \
        dfu::Tile<TMv, TNv>::NT                                                       \
  }
#define DFU_ENTRY_OCC(A, B, E, TMv, TNv, OCCv, TID)                       \
  {                                                                       \
    A, B, E, TID, &dfu::gemm_kernel<A, B, E, TMv, TNv, OCCv>,             \
        dfu::Tile<TMv, TNv, OCCv>::LDS_BYTES, dfu::Tile<TMv, TNv, OCCv>::NT   \
  }
#define DFU_ENTRY_NST(A, B, E, TMv, TNv, NSTv, TID)                       \
  {                                                                       \
    A, B, E, TID, &dfu::gemm_kernel<A, B, E, TMv, TNv, 1, NSTv>,          \
        dfu::Tile<TMv, TNv, 1, NSTv>::LDS_BYTES, dfu::Tile<TMv, TNv, 1, NSTv>::NT \
  }
// 4-wave workgroups (2x2 waves of 64x64), OCCv per CU
#define DFU_ENTRY_W4(A, B, E, TMv, TNv, OCCv, TID)                              \
  {                                                                             \
    A, B, E, TID, &dfu::gemm_kernel<A, B, E, TMv, TNv, OCCv, 0, 4>,             \
        dfu::Tile<TMv, TNv, OCCv, 0, 4>::LDS_BYTES, dfu::Tile<TMv, TNv, OCCv, 0, 4>::NT \
  }
// interleaved-pair bf16x3 kernels (gemm_kernel<..., X3 = true>), keyed epilogue | kX3Key
#define DFU_ENTRY_X3(A, B, E, TMv, TNv, OCCv, NWv, TID)                                      \
  {                                                                                          \
    A, B, (E) | dfu::kX3Key, TID, &dfu::gemm_kernel<A, B, E, TMv, TNv, OCCv, 0, NWv, true>,   \
        dfu::Tile<TMv, TNv, OCCv, 0, NWv>::LDS_BYTES, dfu::Tile<TMv, TNv, OCCv, 0, NWv>::NT  \
  }
