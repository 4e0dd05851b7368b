"""Layer 1's N = 64 1x1 input gradients (dX[M][64] = dY[M][K] W[K][64]): the MN-major weight
view against the transposed [64][K] weight on each tile that runs it (HIP events, us).
Usage (GPU box): python tools/t1x1_time.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dfu-multimodal_amd")]
import torch  # noqa: E402

from dfu_hip import _lib as L  # noqa: E402
from dfu_hip import ops  # noqa: E402

dev, bf = "cuda", torch.bfloat16
M = 64 * 56 * 56
NAMES = {0: "auto", 6: "128x128w4", 10: "256x64", 11: "128x64o2"}


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


for K, add in ((64, False), (256, False), (256, True)):
    dy = (torch.randn(M, K, device=dev) * 0.1).to(bf)
    W = (torch.randn(K, 64, device=dev) * 0.1).to(bf)  # [out][in]
    Wt = W.t().contiguous()
    aux = (torch.randn(M, 64, device=dev) * 0.1).to(bf) if add else None
    epi = L.EPI_BF16_ADD if add else L.EPI_BF16
    ref = dy.float() @ W.float() + (aux.float() if add else 0)
    out = torch.empty(M, 64, dtype=bf, device=dev)
    cells = []

    def mn(tile=0):
        ops.gemm(M, 64, K, dy, K, W, 64, out, 64, b_mode=L.OPND_MNMAJOR, epilogue=epi, aux=aux,
                 ldaux=64 if add else 0, tile=tile)

    def km(tile=0):
        ops.gemm(M, 64, K, dy, K, Wt, K, out, 64, epilogue=epi, aux=aux, ldaux=64 if add else 0,
                 tile=tile)
    for name, fn, tiles in (("MN-major W", mn, (0, 6)), ("W^T", km, (0, 6, 10, 11))):
        for t in tiles:
            try:
                us = timeit(lambda: fn(t))
            except L.DfuError:
                cells.append(f"{name}/{NAMES[t]} -")
                continue
            err = ((out.float() - ref).norm() / ref.norm()).item()
            cells.append(f"{name}/{NAMES[t]} {us:6.1f}us (rel {err:.1e})")
    print(f"{M}x64x{K}{' ADD' if add else ''}: " + "  ".join(cells), flush=True)
