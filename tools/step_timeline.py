"""Host vs device timeline of the eager fusion step (no profiler: rocprofv3's per-dispatch host
cost makes the host look like the bottleneck).  Synchronise, then run N steps back to back; at
each phase boundary (forward, loss, backward, optimizer step) record a HIP event on the current
stream and the host clock.  The device reaches boundary i at event time g[i] (from the first
event); the host enqueued it at h[i].  g[i] - h[i] is how far the device runs behind the host:
where it is small the device has caught up and waits for the host's enqueue.
  python tools/step_timeline.py [--steps 8] [--precision parity]"""
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
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--precision", default=None)
    a = ap.parse_args()
    if a.precision:
        Fn.set_precision(a.precision)
    dev = torch.device("cuda", 0)
    torch.manual_seed(42)
    model, fwd = bench.build("fusion", dev)
    opt = FusedAdamW(model.parameters(), lr=1e-4, weight_decay=1e-4)
    crit = hnn.CrossEntropyLoss(weight=torch.tensor([2.0, 2.0], device=dev))
    rgb, th, y = bench.synthetic(64, dev, seed=42)
    names = []
    evs, hs = [], []
    # per-encoder end-of-backward events (recorded on the stream each backward runs on)
    ends = {}

    def wrap(fn_cls, key):
        orig = fn_cls.backward

        def bwd(ctx, *g):
            r = orig(ctx, *g)
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            ends.setdefault(key, []).append(e)
            return r
        fn_cls.backward = staticmethod(bwd)
    wrap(Fn.StemFn, "resnet backward end")
    wrap(Fn.PatchEmbedFn, "vit backward end")

    def wrapf(fn_cls, key):
        orig = fn_cls.forward

        def fwd_(ctx, *a_):
            r = orig(ctx, *a_)
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            ends.setdefault(key, []).append(e)
            return r
        fn_cls.forward = staticmethod(fwd_)
    wrapf(Fn.AvgPoolFn, "resnet forward end")
    wrapf(Fn.TokenNormFn, "vit forward end")

    def mark(name):
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        evs.append(e)
        hs.append(time.perf_counter())
        names.append(name)

    def step():
        opt.zero_grad()
        out = fwd(model, rgb, th)
        mark("forward enqueued")
        loss = crit(out, y)
        mark("loss enqueued")
        loss.backward()
        Fn.join_grad_streams()
        mark("backward enqueued")
        opt.step()
        mark("step enqueued")

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    names.clear(), evs.clear(), hs.clear()
    ends.clear()
    mark("start")
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    h0 = hs[0]
    print(f"{'boundary':>20s} {'host ms':>9s} {'device ms':>10s} {'device behind host':>19s}")
    for i, n in enumerate(names):
        g = evs[0].elapsed_time(evs[i])
        h = (hs[i] - h0) * 1e3
        print(f"{n:>20s} {h:9.2f} {g:10.2f} {g - h:19.2f}")
    for key, es in ends.items():
        es = es[-a.steps:]
        ts = [evs[0].elapsed_time(e) for e in es]
        print(f"{key:>20s} (device ms): " + " ".join(f"{t:.2f}" for t in ts))
    bw = [evs[0].elapsed_time(evs[i]) for i, n in enumerate(names) if n == "backward enqueued"]
    print("backward joined (device ms): " + " ".join(f"{t:.2f}" for t in bw))
    k = len(names) - 1
    print(f"per step: host {(hs[k] - h0) * 1e3 / a.steps:.2f} ms, device "
          f"{evs[0].elapsed_time(evs[k]) / a.steps:.2f} ms")


if __name__ == "__main__":
    main()
