"""Yardstick: the persistent 256x256 GEMM (tile 8) and the library's plan on square shapes and
the ViT forward shapes, beside torch.matmul (hipBLASLt) on the same random bf16 operands.
Separates what the K-loop delivers (long K, many tiles) from what the ViT shapes cost (K = 768,
150-600 tiles).  HIP events, 20 launches each.
  python tools/gemm_square.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dfu-multimodal_amd")]
import torch  # noqa: E402

from dfu_hip import _lib as L  # noqa: E402
from dfu_hip import ops  # noqa: E402


def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


SHAPES = [(4096, 4096, 4096), (8192, 8192, 8192), (12608, 2304, 768), (12608, 3072, 768),
          (12608, 768, 3072), (12608, 768, 768), (16384, 4096, 768), (12608, 768, 12288)]
print(f"{'shape':>22s} {'tile':>6s} {'us':>9s} {'TF/s':>7s}")
for M, N, K in SHAPES:
    A = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    B = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    C = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    fl = 2.0 * M * N * K
    for tile in (0, 8):
        us = timeit(lambda: ops.gemm(M, N, K, A, K, B, K, C, N, epilogue=L.EPI_BF16, tile=tile))
        print(f"{M:>6d}x{N:>5d}x{K:>5d} {('auto' if tile == 0 else tile):>6} {us:9.1f} "
              f"{fl / us / 1e6:7.0f}", flush=True)
    us = timeit(lambda: torch.matmul(A, B.t(), out=C))
    print(f"{M:>6d}x{N:>5d}x{K:>5d} {'blaslt':>6s} {us:9.1f} {fl / us / 1e6:7.0f}", flush=True)
