"""Where the eager C3 step's runtime copies and fills come from (tools, not a product path): one
profiled step (torch.profiler, Python stacks), the ATen copy / fill / zero ops grouped by their
calling site in this repository.

  python tools/copy_sites.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dfu-multimodal_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from dfu_hip import functional as Fn  # noqa: E402
from dfu_hip import nn as hnn  # noqa: E402
from dfu_hip.optim import FusedAdamW  # noqa: E402

OPS = ("aten::copy_", "aten::clone", "aten::contiguous", "aten::to", "aten::_to_copy",
       "aten::fill_", "aten::zero_", "aten::zeros", "aten::zeros_like", "aten::cat",
       "aten::index", "aten::mul", "aten::add", "aten::sub", "aten::div")


def main():
    dev = torch.device("cuda", 0)
    torch.manual_seed(42)
    model, fwd = bench.build("fusion", dev)
    opt = FusedAdamW(model.parameters(), lr=1e-4, weight_decay=1e-4)
    crit = hnn.CrossEntropyLoss(weight=torch.tensor([2.0, 2.0], device=dev))
    rgb, th, y = bench.synthetic(64, dev, seed=42)

    def step():
        opt.zero_grad()
        crit(fwd(model, rgb, th), y).backward()
        Fn.join_grad_streams()
        opt.step()
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    torch.autograd.set_multithreading_enabled(False)  # backward frames on this thread
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU], with_stack=True) as prof:
        step()
        torch.cuda.synchronize()
    sites = {}
    for ev in prof.events():
        if ev.name not in OPS:
            continue
        frames = [f for f in (ev.stack or []) if "dfu-multimodal_amd" in f or "bench.py" in f]
        key = (ev.name, frames[0] if frames else "(no repo frame)")
        sites[key] = sites.get(key, 0) + 1
    for (name, frame), n in sorted(sites.items(), key=lambda kv: -kv[1]):
        print(f"{n:4d}  {name:18s} {frame}")


if __name__ == "__main__":
    main()
