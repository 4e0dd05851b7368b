"""Time the flat AdamW kernel at the fusion model's parameter count (110.75M) with HIP events.

  python tools/adamw_time.py   (on the GPU box)
Algorithmic bytes per parameter: p, g, m, v read (16 B) + p, m, v written (12 B) + bf16 shadow (2 B).
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dfu-multimodal_amd"))
from dfu_hip import ops  # noqa: E402

n = 110_750_000
dev = "cuda"
p = torch.randn(n, device=dev)
g = torch.randn(n, device=dev)
m = torch.zeros(n, device=dev)
v = torch.zeros(n, device=dev)
sh = torch.empty(n, dtype=torch.bfloat16, device=dev)
step = torch.ones((), dtype=torch.int64, device=dev)
for _ in range(3):
    ops.adamw_flat(p, g, m, v, 1e-4, 0.9, 0.999, 1e-8, 1e-4, step, sh)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
reps = 20
e0.record()
for _ in range(reps):
    ops.adamw_flat(p, g, m, v, 1e-4, 0.9, 0.999, 1e-8, 1e-4, step, sh)
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) * 1e3 / reps
print(f"adamw_flat n={n}: {us:.1f} us, {30 * n / us / 1e3:.0f} GB/s algorithmic")
