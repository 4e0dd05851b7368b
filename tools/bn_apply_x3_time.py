"""Time dfu_bn_apply_x3 (the parity mode's BN apply over split pairs) at the ResNet-50 B = 64
shapes of the step: conv output pair in, optional residual (pair, or fp32 for the downsample
branch), out pair + ReLU bitmask.  Bytes: 4 (y pair) [+ 4 residual pair] + 4 (out pair) +
1/8 (mask) per element.   python tools/bn_apply_x3_time.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "dfu-multimodal_amd"))
from dfu_hip import ops  # noqa: E402

B = 64
# (rows, C, residual pair?, count per step): bn1/bn2 (no residual) and bn3 (+ residual pair)
shapes = [(B * 56 * 56, 64, False, 6), (B * 56 * 56, 256, True, 3), (B * 28 * 28, 128, False, 7),
          (B * 28 * 28, 512, True, 4), (B * 14 * 14, 256, False, 11), (B * 14 * 14, 1024, True, 6),
          (B * 7 * 7, 512, False, 5), (B * 7 * 7, 2048, True, 3)]
tot_us = tot_b = 0.0
for M, C, res, cnt in shapes:
    y = torch.randn(M, C, device="cuda").to(torch.bfloat16)
    ylo = (torch.randn(M, C, device="cuda") * 1e-3).to(torch.bfloat16)
    r = torch.randn(M, C, device="cuda").to(torch.bfloat16) if res else None
    rlo = (torch.randn(M, C, device="cuda") * 1e-3).to(torch.bfloat16) if res else None
    out, lo = torch.empty_like(y), torch.empty_like(y)
    mask = torch.empty(M * C // 8, dtype=torch.uint8, device="cuda")
    sc, sh = torch.rand(C, device="cuda"), torch.rand(C, device="cuda")

    def run():
        ops.bn_apply_x3(y, sc, sh, r, 2 if res else 0, True, M, C, out_lo=lo, out_bf16=out,
                        residual_lo=rlo, y_lo=ylo, relu_mask=mask)
    for _ in range(3):
        run()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 50
    e0.record()
    for _ in range(reps):
        run()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    nb = M * C * ((8 if res else 4) + 4 + 0.125)
    tot_us += us * cnt
    tot_b += nb * cnt
    print(f"M={M:7d} C={C:5d} res={int(res)}: {us:7.1f} us  {nb / us / 1e3:6.0f} GB/s  (x{cnt})",
          flush=True)
print(f"per step: {tot_us / 1e3:.3f} ms, {tot_b / 1e9:.2f} GB, {tot_b / tot_us / 1e3:.0f} GB/s")
