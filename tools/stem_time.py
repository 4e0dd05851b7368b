"""Time the parity mode's stem conv at B = 64: the fused implicit-GEMM kernel
(dfu_stem_conv_x3) against the pair im2col + split weights + interleaved-pair GEMM it
replaces; and its weight gradient from x (dfu_stem_wgrad_x3) against the MN x MN GEMM over the
hi im2col rows.  python tools/stem_time.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "dfu-multimodal_amd"))
from dfu_hip import _lib as L  # noqa: E402
from dfu_hip import ops  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
x = torch.randn(B, 3, 224, 224, device="cuda")
w = torch.randn(64, 3, 7, 7, device="cuda") * 0.05
M = B * 112 * 112


def old():
    (chi, clo), P, Q = ops.im2col_f32_x3(x, 7, 7, 2, 3, 160)
    w3 = ops.split_x3(w.reshape(64, -1), ops.X3_PAIRS, seg=160)
    y = torch.empty(M, 64, dtype=torch.bfloat16, device="cuda")
    ylo = torch.empty_like(y)
    st = torch.empty(M // 128, 2, 64, device="cuda")
    ops.gemm(M, 64, 320, chi, 160, w3, 320, y, 64, epilogue=L.EPI_F32_STATS, stats=st, x3=True,
             a_lo=clo, x3_pairs=True, aux_out=ylo, ldaux_out=64)


def new():
    ops.stem_conv_x3(x, w)


def new_nocol():
    ops.stem_conv_x3(x, w, want_col=False)


dy = (torch.randn(M, 64, device="cuda") * 0.1).to(torch.bfloat16)
col = ops.im2col_f32(x, 7, 7, 2, 3, 160)[0]
dw = torch.zeros(64, 147, device="cuda")


def wgrad_gemm():
    ops.gemm(64, 147, M, dy, 64, col, 160, dw, 147, a_mode=L.OPND_MNMAJOR,
             b_mode=L.OPND_MNMAJOR, epilogue=L.EPI_F32_ACC)


def wgrad_x():
    ops.stem_wgrad_x3(x, dy, dw)


for name, fn in (("pair im2col + GEMM", old), ("fused stem kernel", new),
                 ("fused, no col rows", new_nocol), ("wgrad: GEMM over col", wgrad_gemm),
                 ("wgrad: from x", wgrad_x)):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        fn()
    e1.record()
    torch.cuda.synchronize()
    print(f"{name:20s}: {e0.elapsed_time(e1) * 1e3 / 20:8.1f} us per stem (B = {B})", flush=True)
