"""Calibration only (not a product path): the library GEMM (torch.matmul -> hipBLASLt) against
dfu's MFMA template on the ViT GEMM shapes of the B=64 step, same layouts, bf16 in, plain bf16
(fwd/dgrad) or fp32 (wgrad) out, random operands.  Tells how far the template is from what the
vendor library reaches on this chip and clock.
Usage (GPU box): python tools/blas_compare.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dfu-multimodal_amd")]
import torch  # noqa: E402

from dfu_hip import _lib as L  # noqa: E402
from dfu_hip import ops  # noqa: E402

dev = "cuda"
bf = torch.bfloat16


def T(*s):
    return (torch.randn(*s, device=dev) * 0.1).to(bf)


def timeit(fn, iters=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


print(f"{'case':34s} {'hipBLASLt':>16s} {'dfu':>16s}")
M = 12608
for name, N, K in (("qkv", 2304, 768), ("proj", 768, 768), ("fc1", 3072, 768), ("fc2", 768, 3072)):
    A, W, dY = T(M, K), T(N, K), T(M, N)
    C, dX = torch.empty(M, N, dtype=bf, device=dev), torch.empty(M, K, dtype=bf, device=dev)
    dW = torch.zeros(N, K, device=dev)
    fl = 2 * M * N * K
    rows = [
        (f"fwd  {name} {M}x{N}x{K}", lambda: torch.matmul(A, W.t(), out=C),
         lambda: ops.gemm(M, N, K, A, K, W, K, C, N, epilogue=L.EPI_BF16)),
        (f"dgrd {name} {M}x{K}x{N}", lambda: torch.matmul(dY, W, out=dX),
         lambda: ops.gemm(M, K, N, dY, N, W, K, dX, K, b_mode=L.OPND_MNMAJOR, epilogue=L.EPI_BF16)),
        (f"wgrd {name} {N}x{K}x{M}", lambda: torch.mm(dY.t(), A, out_dtype=torch.float32),
         lambda: ops.gemm(N, K, M, dY, N, A, K, dW, K, a_mode=L.OPND_MNMAJOR,
                          b_mode=L.OPND_MNMAJOR, epilogue=L.EPI_F32_ACC)),
    ]
    for label, blas, ours in rows:
        try:
            tb = timeit(blas)
            sb = f"{tb:7.1f}us {fl / tb / 1e6:5.0f}T"
        except Exception as e:  # out_dtype may be unsupported: fall back to a bf16 product
            if label.startswith("wgrd"):
                tb = timeit(lambda: torch.mm(dY.t(), A))
                sb = f"{tb:7.1f}us {fl / tb / 1e6:5.0f}T*"
            else:
                sb = f"err {type(e).__name__}"
        to = timeit(ours)
        print(f"{label:34s} {sb:>16s} {to:7.1f}us {fl / to / 1e6:5.0f}T", flush=True)
print("(* = bf16 output: torch.mm out_dtype=float32 unavailable)")
