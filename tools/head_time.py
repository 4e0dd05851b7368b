"""How long the fusion step's serial head section runs (no profiler): HIP events on the head's
stream at ConcatFn's forward (both encoders' features ready) and at the end of its backward
(the features' gradients split off: the encoders' backwards start), median over steps.
Usage (GPU box): python tools/head_time.py [--steps 20]"""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dfu-multimodal_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from dfu_hip import functional as Fn  # noqa: E402
from dfu_hip import nn as hnn  # noqa: E402
from dfu_hip.optim import FusedAdamW  # noqa: E402

marks = []
f0, b0 = Fn.ConcatFn.forward, Fn.ConcatFn.backward


def fwd(ctx, a, b):
    e = torch.cuda.Event(enable_timing=True)
    e.record()
    marks.append(("fwd", e))
    return f0(ctx, a, b)


def bwd(ctx, g):
    r = b0(ctx, g)
    e = torch.cuda.Event(enable_timing=True)
    e.record()
    marks.append(("bwd", e))
    return r


Fn.ConcatFn.forward, Fn.ConcatFn.backward = staticmethod(fwd), staticmethod(bwd)
dev = torch.device("cuda", 0)
torch.manual_seed(42)
model, f = bench.build("fusion", dev)
opt = FusedAdamW(model.parameters(), lr=1e-4, weight_decay=1e-4)
crit = hnn.CrossEntropyLoss(weight=torch.tensor([2.0, 2.0], device=dev))
rgb, th, y = bench.synthetic(64, dev, 42)
steps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 20
t_step = []
for i in range(steps + 3):
    s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s0.record()
    opt.zero_grad()
    crit(f(model, rgb, th), y).backward()
    opt.step()
    s1.record()
    t_step.append((s0, s1))
torch.cuda.synchronize()
pairs = [(marks[k][1], marks[k + 1][1]) for k in range(0, len(marks) - 1, 2)][3:]
head = [a.elapsed_time(b) for a, b in pairs]
step = [a.elapsed_time(b) for a, b in t_step[3:]]
print(f"head section (concat fwd -> split of the feature gradients): median "
      f"{statistics.median(head) * 1e3:.0f} us; step median {statistics.median(step):.2f} ms")
