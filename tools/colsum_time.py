"""Time the bias-gradient column sum (dfu_colsum: partial sums + reduce) at the ViT B=64 shapes.

  python tools/colsum_time.py   (on the GPU box; DFU_HIP_LIB selects another build for A/B)
Algorithmic bytes: the bf16 dY read once (2 B per element).
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dfu-multimodal_amd"))
from dfu_hip import ops  # noqa: E402

rows = 64 * 197
tot = 0.0
for N in (768, 2304, 3072):
    x = torch.randn(rows, N, device="cuda").to(torch.bfloat16)
    out = torch.zeros(N, device="cuda")
    for _ in range(3):
        ops.colsum_add(x, out)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 50
    e0.record()
    for _ in range(reps):
        ops.colsum_add(x, out)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    tot += us
    print(f"colsum rows={rows} N={N}: {us:.1f} us, {rows * N * 2 / us / 1e3:.0f} GB/s")
print(f"total {tot:.1f} us  lib={os.environ.get('DFU_HIP_LIB', 'in-tree')}")
