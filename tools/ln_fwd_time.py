"""Time the ViT LayerNorm forward (fp32 residual stream in, bf16 out + mean/rstd) at B=64.

  python tools/ln_fwd_time.py   (on the GPU box; DFU_HIP_LIB selects another build for A/B)
rows = 64 x 197, D = 768.  Algorithmic bytes per row: 4 D in + 2 D out.  Prints a checksum of
the output so two builds can be compared bit for bit.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dfu-multimodal_amd"))
from dfu_hip import ops  # noqa: E402

rows, D = 64 * 197, 768
g = torch.Generator(device="cpu").manual_seed(0)
x = torch.randn(rows, D, generator=g).cuda()
gamma = torch.randn(D, generator=g).cuda()
beta = torch.randn(D, generator=g).cuda()
out = torch.empty(rows, D, dtype=torch.bfloat16, device="cuda")
mean = torch.empty(rows, device="cuda")
rstd = torch.empty(rows, device="cuda")


def run():
    ops.layernorm_fwd(x, D, rows, D, gamma, beta, 1e-6, out, D, True, mean, rstd)


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
ck = (out.view(torch.int16).long().sum().item(), mean.double().sum().item(), rstd.double().sum().item())
print(f"ln_fwd rows={rows} D={D} lib={os.environ.get('DFU_HIP_LIB', 'in-tree')}: {us:.1f} us, "
      f"{6 * D * rows / us / 1e3:.0f} GB/s algorithmic; checksum {ck}")
