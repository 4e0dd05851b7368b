"""Time the attention kernels at the ViT-B/16 B=64 shape (HIP events): forward and fused
backward, us per launch and TFLOP/s (fwd 4*N^2*dh per head, bwd 2.5x).
Usage (GPU box): python tools/attn_time.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dfu-multimodal_amd")]
import torch  # noqa: E402

from dfu_hip import ops  # noqa: E402

B, N, H, dh = 64, 197, 12, 64
qkv = (torch.randn(B * N, 3 * H * dh, device="cuda") * 0.5).to(torch.bfloat16)
dout = (torch.randn(B * N, H * dh, device="cuda") * 0.1).to(torch.bfloat16)
scale = dh ** -0.5


def timeit(fn, iters=50):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


o, lse = ops.attention_fwd(qkv, B, N, H, dh, scale)
dq = torch.empty_like(qkv)
fl = 4.0 * N * N * dh * B * H
tf = timeit(lambda: ops.attention_fwd(qkv, B, N, H, dh, scale))
tb = timeit(lambda: ops.attention_bwd(qkv, o, dout, lse, B, N, H, dh, scale, dq))
qf = qkv.float()
qb = torch.empty_like(qkv)
tx = timeit(lambda: ops.attention_fwd_f32(qf, B, N, H, dh, scale, qkv_bf16=qb))
q16 = qkv.to(torch.float16)
th = timeit(lambda: ops.attention_fwd_f16(q16, B, N, H, dh, scale))
print(f"attention fwd {tf:.1f} us ({fl / tf / 1e6:.0f} TFLOP/s)  fwd fp16 {th:.1f} us  bwd "
      f"{tb:.1f} us ({2.5 * fl / tb / 1e6:.0f} TFLOP/s)  fwd bf16x3 {tx:.1f} us")
