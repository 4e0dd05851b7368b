"""Time the stem's max-pool backward (dfu_maxpool_bwd) at C3's shape: dy [64][56][56][64] bf16
-> dx [64][112][112][64]; HIP events over 50 launches.  python tools/pool_time.py"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "dfu-multimodal_amd"))
import torch  # noqa: E402

from dfu_hip import ops  # noqa: E402

B, H, W, C = 64, 112, 112, 64
x = torch.randn(B * H * W, C, device="cuda").to(torch.bfloat16)
y, am, P, Q = ops.maxpool_fwd(x, B, H, W, C)
dy = torch.randn(B * P * Q, C, device="cuda").to(torch.bfloat16)
ops.maxpool_bwd(dy, am, B, H, W, C, P, Q)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(50):
    dx = ops.maxpool_bwd(dy, am, B, H, W, C, P, Q)
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) / 50 * 1e3
nbytes = B * H * W * C * 2 + B * P * Q * C * 3
print(f"maxpool bwd {B}x{H}x{W}x{C}: {us:.1f} us, {nbytes / us / 1e6:.2f} TB/s algorithmic")
