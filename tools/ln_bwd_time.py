"""Time the ViT LayerNorm backward (dfu_layernorm_bwd + dgamma/dbeta reduction) at B=64.

  python tools/ln_bwd_time.py   (on the GPU box; DFU_HIP_LIB selects another build for A/B)
rows = 64 x 197, D = 768; dy bf16, gx fp32 read-modify-write + bf16 copy, column sums of gx.
Algorithmic bytes per row: x 4D + gx 8D + dy 2D + gx_bf16 2D = 16 D.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dfu-multimodal_amd"))
from dfu_hip import ops  # noqa: E402

rows, D = 64 * 197, 768
dev = "cuda"
x = torch.randn(rows, D, device=dev)
dy = torch.randn(rows, D, device=dev).to(torch.bfloat16)
gx = torch.randn(rows, D, device=dev)
gxb = torch.empty(rows, D, dtype=torch.bfloat16, device=dev)
mean = x.mean(1)
rstd = torch.rsqrt(x.var(1, unbiased=False) + 1e-6)
gamma = torch.randn(D, device=dev)
dg = torch.empty(D, device=dev)
db = torch.empty(D, device=dev)


def run():
    ops.layernorm_bwd(dy, D, True, x, D, mean, rstd, gamma, rows, D, gx, D, gxb, dg, db, gsum=True)


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
print(f"ln_bwd rows={rows} D={D} lib={os.environ.get('DFU_HIP_LIB', 'in-tree')}: {us:.1f} us, "
      f"{16 * D * rows / us / 1e3:.0f} GB/s algorithmic")
