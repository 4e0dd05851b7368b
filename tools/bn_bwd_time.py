"""Time the BatchNorm backward (reduce -> finalize -> apply) at the ResNet50 B=64 shapes.

  python tools/bn_bwd_time.py   (on the GPU box; DFU_HIP_LIB selects another build for A/B)
Algorithmic bytes: reduce reads dout, y (+ out for the residual mask); apply reads the same and
writes dy (+ dres); 2 B per element each.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dfu-multimodal_amd"))
from dfu_hip import ops  # noqa: E402

B = 64
# (M, C, relu mode, residual): conv1/conv2 BN+ReLU recompute the mask (2); block output BN +
# residual + ReLU masks from the stored output (1) and emits dres
shapes = [(B * 112 * 112, 64, 2, False), (B * 56 * 56, 64, 2, False), (B * 56 * 56, 256, 1, True),
          (B * 28 * 28, 128, 2, False), (B * 28 * 28, 512, 1, True), (B * 14 * 14, 256, 2, False),
          (B * 14 * 14, 1024, 1, True), (B * 7 * 7, 512, 2, False), (B * 7 * 7, 2048, 1, True)]
tot = 0.0
for M, C, relu, res in shapes:
    bf = torch.bfloat16
    dout = torch.randn(M, C, device="cuda").to(bf)
    y = torch.randn(M, C, device="cuda").to(bf)
    out = torch.relu(torch.randn(M, C, device="cuda")).to(bf)
    mean = torch.randn(C, device="cuda") * 0.1
    invstd = torch.rand(C, device="cuda") + 0.5
    gamma = torch.randn(C, device="cuda")
    sc, sh = gamma * invstd, -mean * gamma * invstd
    dy = torch.empty_like(y)
    dres = torch.empty_like(y) if res else None
    dg = torch.zeros(C, device="cuda")
    db = torch.zeros(C, device="cuda")

    def run():
        ops.bn_bwd(dout, y, out, relu, mean, invstd, gamma, M, C, dy, dres, dg, db,
                   scale=sc, shift=sh)

    for _ in range(3):
        run()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 30
    e0.record()
    for _ in range(reps):
        run()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    nrd = 3 if relu == 1 else 2
    nb = M * C * 2 * (2 * nrd + 1 + (1 if res else 0))
    tot += us
    print(f"bn_bwd M={M} C={C} relu={relu} res={res}: {us:.1f} us, {nb / us / 1e3:.0f} GB/s")
print(f"total {tot:.1f} us  lib={os.environ.get('DFU_HIP_LIB', 'in-tree')}")
