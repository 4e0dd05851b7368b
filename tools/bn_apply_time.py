"""Time dfu_bn_apply (BN scale/shift + residual + ReLU, bf16 NHWC) at the ResNet50 B=64 shapes.

  python tools/bn_apply_time.py   (on the GPU box; DFU_BN_BLOCKS caps the grid for sweeps)
Algorithmic bytes: y read + residual read (if any) + out written, 2 B each per element.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dfu-multimodal_amd"))
from dfu_hip import ops  # noqa: E402

B = 64
shapes = [(B * 112 * 112, 64, False), (B * 56 * 56, 64, False), (B * 56 * 56, 256, True),
          (B * 28 * 28, 512, True), (B * 14 * 14, 1024, True), (B * 7 * 7, 2048, True)]
tot = 0.0
for M, C, res in shapes:
    y = torch.randn(M, C, device="cuda").to(torch.bfloat16)
    r = torch.randn(M, C, device="cuda").to(torch.bfloat16) if res else None
    out = torch.empty_like(y)
    sc = torch.rand(C, device="cuda")
    sh = torch.rand(C, device="cuda")
    for _ in range(3):
        ops.bn_apply(y, sc, sh, r, True, out, M, C)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 50
    e0.record()
    for _ in range(reps):
        ops.bn_apply(y, sc, sh, r, True, out, M, C)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    nb = M * C * 2 * (3 if res else 2)
    tot += us
    print(f"bn_apply M={M} C={C} res={res}: {us:.1f} us, {nb / us / 1e3:.0f} GB/s")
print(f"total {tot:.1f} us")
