"""Time the ResNet50 strided 3x3 input gradients (layer2-4 block 0 conv2, B = 64) under every
tile hint (0 = the library plan), and the stride-1 GEMM of each stride phase alone.
  python tools/dgrad_strided_time.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dfu-multimodal_amd")]
import torch  # noqa: E402

from dfu_hip import _lib as L  # noqa: E402
from dfu_hip import ops  # noqa: E402

B = 64
SHAPES = [(56, 128), (28, 256), (14, 512)]  # input H = W, channels (C = K)


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


for H, C in SHAPES:
    g = ops.ConvGeom(B, H, H, C, C, 3, 3, 2, 1)
    dy = (torch.randn(B * g.p * g.q, C, device="cuda") * 0.1).to(torch.bfloat16)
    w = (torch.randn(C, 3, 3, C, device="cuda") * 0.1).to(torch.bfloat16)  # KRSC
    dx = torch.empty(B * H * H, C, device="cuda", dtype=torch.bfloat16)
    Mx, K = B * H * H, 9 * C
    flop = 2 * Mx * C * K / 4  # algorithmic: a quarter of the taps are live per phase

    def run(tile):
        return lambda: ops.gemm(Mx, C, K, dy, 0, w, K, dx, C, a_mode=L.OPND_CONV_DGRAD,
                                b_mode=L.OPND_CONV_DGRAD_W, epilogue=L.EPI_BF16, conv=g,
                                tile=tile)
    line = []
    for t in range(0, 12):
        try:
            us = timed(run(t))
            line.append(f"t{t} {us:6.1f}")
        except RuntimeError:
            line.append(f"t{t}     --")
    print(f"dgrad s2 {Mx}x{C}x{K} (H={H}, C={C}) [{flop / 1e9:.1f} GFLOP]: " + "  ".join(line),
          flush=True)
    # each stride phase as the dense stride-1 GEMM it is: M = B * (H/2)^2, K = live taps x C
    Mp = B * (H // 2) * (H // 2)
    for taps in (4, 2, 1):
        A = (torch.randn(Mp, taps * C, device="cuda") * 0.1).to(torch.bfloat16)
        Bw = (torch.randn(C, taps * C, device="cuda") * 0.1).to(torch.bfloat16)
        Cc = torch.empty(Mp, C, device="cuda", dtype=torch.bfloat16)
        us = timed(lambda: ops.gemm(Mp, C, taps * C, A, taps * C, Bw, taps * C, Cc, C,
                                    epilogue=L.EPI_BF16))
        print(f"   dense phase GEMM {Mp}x{C}x{taps * C}: {us:6.1f} us "
              f"({2 * Mp * C * taps * C / us / 1e6:.0f} TF/s)", flush=True)
