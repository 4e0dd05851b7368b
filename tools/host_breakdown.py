"""Where the host time of an eager fusion step goes (tools, not a product path).

  python tools/host_breakdown.py [--micro]

1. Launch micro-costs on this host: one library launch through ctypes (dfu_zero), one dfu_gemm
   through ops.gemm (descriptor built in Python) against the same descriptor replayed (ctypes +
   the C side only), and torch's own elementwise launch, each as host microseconds per call.
2. cProfile of eager steps with the backward on the calling thread: the callers of torch.empty /
   torch.empty_like / ops.gemm (which layer allocates and launches how often per step).
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dfu-multimodal_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from dfu_hip import _lib as L  # noqa: E402
from dfu_hip import functional as Fn  # noqa: E402
from dfu_hip import nn as hnn  # noqa: E402
from dfu_hip import ops  # noqa: E402
from dfu_hip.optim import FusedAdamW  # noqa: E402


def _host_us(fn, n=400):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    dt = time.perf_counter() - t
    torch.cuda.synchronize()
    return dt / n * 1e6


def micro(dev):
    z = torch.empty(4096, device=dev)
    M = N = K = 256
    A = torch.randn(M, K, device=dev).to(torch.bfloat16)
    B = torch.randn(N, K, device=dev).to(torch.bfloat16)
    C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    ops.gemm_record = []
    ops.gemm(M, N, K, A, K, B, K, C, N)
    rec, ops.gemm_record = ops.gemm_record, None
    r = {
        "dfu_zero (ctypes, 3 args)": _host_us(lambda: ops.zero_(z)),
        "ops.gemm (Python descriptor + 2 ctypes calls)": _host_us(
            lambda: ops.gemm(M, N, K, A, K, B, K, C, N)),
        "dfu_gemm replay (ctypes + C only)": _host_us(lambda: ops.gemm_replay(rec)),
        "torch add_ (ATen launch)": _host_us(lambda: z.add_(1.0)),
        "torch.empty (caching allocator, 1 MiB)": _host_us(
            lambda: torch.empty(1 << 18, device=dev)),
        "ops.stream_ptr": _host_us(ops.stream_ptr, 4000),
    }
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def ctx():
        with torch.cuda.stream(s1):
            pass
    t = torch.empty(16, device=dev)
    r.update({
        "torch.cuda.current_stream()": _host_us(torch.cuda.current_stream, 2000),
        "with torch.cuda.stream(s): pass": _host_us(ctx, 2000),
        "s1.wait_stream(s2)": _host_us(lambda: s1.wait_stream(s2), 2000),
        "t.record_stream(s1)": _host_us(lambda: t.record_stream(s1), 2000),
        "torch.cuda.Event()": _host_us(torch.cuda.Event, 2000),
        "ops.current_stream()": _host_us(ops.current_stream, 2000),
    })
    for k, v in r.items():
        print(f"  {k:48s} {v:7.2f} us")


def profile(dev, steps=5):
    import cProfile
    import pstats
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
    st.sort_stats("tottime").print_stats(30)
    st.sort_stats("ncalls").print_stats(40)
    st.print_callers(r"\{built-in method torch.empty\}|\{built-in method torch.empty_like\}")
    st.print_callers(r"ops.py:\d+\(gemm\)")
    st.print_callers(r"module.py:\d+\(__getattr__\)")
    st.print_callers(r"__init__.py:\d+\(current_stream\)")


def main():
    dev = torch.device("cuda", 0)
    Fn.set_precision("parity")
    print("launch micro-costs (host us per call):")
    micro(dev)
    if "--micro" not in sys.argv:
        profile(dev)


if __name__ == "__main__":
    main()
