"""Calibration only (not a product path): one ViT GEMM of the B = 64 step through torch.matmul
(-> hipBLASLt), repeated, for rocprofv3 kernel-trace / --pmc passes beside tools/gemm_one.py's
dfu run of the same case (profiles/r16_blas_counters.md).
  python tools/blas_one.py <case> [--iters N]
  cases: qkv_fwd, fc1_fwd, fc2_fwd (A [M,K] W[N,K]^T), qkv_dgrad_t, fc1_dgrad_t (dY [M,K] W [K,N])"""
import argparse

import torch

SHAPES = {"qkv_fwd": (12608, 2304, 768), "fc1_fwd": (12608, 3072, 768),
          "fc2_fwd": (12608, 768, 3072), "qkv_dgrad_t": (12608, 768, 2304),
          "fc1_dgrad_t": (12608, 768, 3072)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("case", choices=sorted(SHAPES))
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    M, N, K = SHAPES[a.case]
    bf = torch.bfloat16
    A = (torch.randn(M, K, device="cuda") * 0.1).to(bf)
    C = torch.empty(M, N, dtype=bf, device="cuda")
    if a.case.endswith("_fwd"):
        W = (torch.randn(N, K, device="cuda") * 0.1).to(bf)
        fn = lambda: torch.matmul(A, W.t(), out=C)  # noqa: E731
    else:
        W = (torch.randn(K, N, device="cuda") * 0.1).to(bf)
        fn = lambda: torch.matmul(A, W, out=C)  # noqa: E731
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / a.iters * 1e3
    print(f"blas {a.case} {M}x{N}x{K}: {us:.1f} us {2 * M * N * K / us / 1e6:.0f} TFLOP/s")


if __name__ == "__main__":
    main()
