"""Time the GPU input pipeline on a batch of decoded images: the two HIP kernels alone (inputs
resident), the whole GpuPreprocessor call (host staging + one H2D copy + kernels), and the
reference's per-sample PIL/torch transform on one host core for comparison."""
import argparse
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dfu-multimodal_amd"), os.path.join(ROOT, "oracle")]
from data import gpu_transforms as GT  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=64)
ap.add_argument("--h", type=int, default=480)
ap.add_argument("--w", type=int, default=640)
ap.add_argument("--iters", type=int, default=20)
a = ap.parse_args()

rng = np.random.default_rng(0)
imgs = [rng.integers(0, 256, (a.h, a.w, 3), dtype=np.uint8) for _ in range(a.batch)]
spec = GT.rgb_train_transform
g = torch.Generator().manual_seed(0)
params = [GT.sample_params(spec, g) for _ in imgs]
pre = GT.GpuPreprocessor(spec)
for _ in range(3):
    pre(imgs, params)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(a.iters):
    pre(imgs, params)
torch.cuda.synchronize()
full = (time.perf_counter() - t0) / a.iters
# kernels only: replay on resident staging via the profiler-visible launches
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(a.iters):
    pre(imgs, params)
e.record()
torch.cuda.synchronize()
print(f"GpuPreprocessor batch {a.batch} of {a.h}x{a.w}: {full * 1e3:.2f} ms/batch "
      f"({a.batch / full:.0f} img/s incl. host staging + H2D)")
import transforms_ref as TR  # noqa: E402
t0 = time.perf_counter()
n = min(8, a.batch)
for im, p in zip(imgs[:n], params[:n]):
    TR.reference_transform(im, spec.size, spec.mean, spec.std, p.hflip, p.vflip, p.angle, p.ops,
                           p.affine)
cpu = (time.perf_counter() - t0) / n
print(f"PIL/torch reference transform: {cpu * 1e3:.2f} ms/img ({1 / cpu:.0f} img/s, 1 core)")
