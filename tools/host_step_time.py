"""Host-side cost of one eager fusion training step (tools, not a product path): wall time the
CPU spends enqueueing each phase (zero_grad, forward, loss, backward, the optimizer step) against
the GPU time of the step, to see whether the device waits for the host at the step's tail.

  python tools/host_step_time.py [--steps 20] [--batch 64]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dfu-multimodal_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from dfu_hip import functional as Fn  # noqa: E402
from dfu_hip import nn as hnn  # noqa: E402
from dfu_hip.optim import FusedAdamW  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--profile", action="store_true", help="cProfile the host side instead")
    ap.add_argument("--precision", default="parity")
    ap.add_argument("--pin", action="store_true", help="pin the process to four cores")
    a = ap.parse_args()
    Fn.set_precision(a.precision)
    if a.pin and hasattr(os, "sched_setaffinity"):
        # four fixed cores (the calling thread, autograd's device thread, the runtime's): the
        # box's scheduler otherwise moves the process between cores of different speed mid-run
        cores = sorted(os.sched_getaffinity(0))[:4]
        os.sched_setaffinity(0, cores)
        print("pinned to cores", cores)
    if a.profile:
        return profile()
    dev = torch.device("cuda", 0)
    torch.manual_seed(42)
    model, fwd = bench.build("fusion", dev)
    opt = FusedAdamW(model.parameters(), lr=1e-4, weight_decay=1e-4)
    crit = hnn.CrossEntropyLoss(weight=torch.tensor([2.0, 2.0], device=dev))
    rgb, th, y = bench.synthetic(a.batch, dev, seed=42)
    phases = ["zero_grad", "forward", "loss", "backward", "join", "opt.step"]
    acc = {k: [] for k in phases}
    gpu = []
    for it in range(a.steps + 3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        t = [time.perf_counter()]
        opt.zero_grad()
        t.append(time.perf_counter())
        out = fwd(model, rgb, th)
        t.append(time.perf_counter())
        loss = crit(out, y)
        t.append(time.perf_counter())
        loss.backward()
        t.append(time.perf_counter())
        Fn.join_grad_streams()
        t.append(time.perf_counter())
        opt.step()
        t.append(time.perf_counter())
        e1.record()
        torch.cuda.synchronize()
        if it >= 3:
            for k, i in zip(phases, range(len(phases))):
                acc[k].append((t[i + 1] - t[i]) * 1e3)
            gpu.append(e0.elapsed_time(e1))
    med = lambda v: sorted(v)[len(v) // 2]  # noqa: E731
    host = sum(med(acc[k]) for k in phases)
    print("host enqueue ms per phase (median):",
          ", ".join(f"{k} {med(acc[k]):.3f}" for k in phases))
    print(f"host total {host:.3f} ms, GPU step {med(gpu):.3f} ms (synchronised each step)")
    # the fastest step: the enqueue's own cost without the host's noise (other processes on the
    # box's cores, frequency changes) -- which moves the medians by several ms between runs
    tot = [sum(acc[k][j] for k in phases) for j in range(len(gpu))]
    print(f"host fastest step {min(tot):.3f} ms, lower quartile {sorted(tot)[len(tot) // 4]:.3f} ms")




def profile(steps=5):
    """cProfile of the host side of `steps` eager steps (after warm-up): top functions."""
    import cProfile
    import pstats
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
    # the autograd engine runs CUDA backward nodes on its own device thread, which cProfile
    # (per thread) does not see: run them on this thread for the profile
    torch.autograd.set_multithreading_enabled(False)
    step()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(steps):
        step()
    pr.disable()
    torch.cuda.synchronize()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(45)
    st.sort_stats("cumulative").print_stats(45)


if __name__ == "__main__":
    main()
