"""Run one GEMM of the step repeatedly (for rocprofv3 --pmc counter passes on a single kernel).

  python tools/gemm_one.py <case> [--tile T] [--iters N]
  cases: fc1_fwd (12608x3072x768, KM x KM, BF16), fc1_gelu (same, GELU epilogue),
         fc2_dgrad (12608x3072x768, KM x MN, DGELU), fc1_wgrad (3072x768x12608, MN x MN, F32_ACC),
         l1c3_fwd (200704x256x64 1x1 conv, STATS), fc2_fwd_resid (12608x768x3072, F32_RESID),
         fc2_wgrad / qkv_wgrad / proj_wgrad (768x3072 / 2304x768 / 768x768 x 12608, F32_ACC),
         l1c3x3_fwd / l1c1x3_fwd / l3c2x3_fwd (bf16x3 pair convs; FLOPs: the MFMA work, 3 products)
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dfu-multimodal_amd")]
import torch  # noqa: E402

from dfu_hip import _lib as L  # noqa: E402
from dfu_hip import ops  # noqa: E402


def T(*s, dtype=torch.bfloat16):
    return (torch.randn(*s, device="cuda") * 0.1).to(dtype)


CHECK = []  # (HIP result, fp32 reference) thunks for --check


def build(case, tile):
    if case in ("qkv_fwd", "proj_fwd", "fc2_fwd"):
        M, N, K = {"qkv_fwd": (12608, 2304, 768), "proj_fwd": (12608, 768, 768),
                   "fc2_fwd": (12608, 768, 3072)}[case]
        A, B, C = T(M, K), T(N, K), T(M, N)
        bias = T(N, dtype=torch.float32)
        CHECK.append(lambda: (C.float(), A.float() @ B.float().t() + bias))
        return 2 * M * N * K, lambda: ops.gemm(M, N, K, A, K, B, K, C, N, epilogue=L.EPI_BF16,
                                               bias=bias, tile=tile)
    if case in ("fc1_fwd", "fc1_gelu"):
        M, N, K = 12608, 3072, 768
        A, B, C, pre = T(M, K), T(N, K), T(M, N), T(M, N)
        epi = L.EPI_BF16_GELU if case == "fc1_gelu" else L.EPI_BF16
        kw = dict(aux_out=pre, ldaux_out=N) if case == "fc1_gelu" else {}
        return 2 * M * N * K, lambda: ops.gemm(M, N, K, A, K, B, K, C, N, epilogue=epi, tile=tile, **kw)
    if case == "fc2_dgrad":
        M, N, K = 12608, 3072, 768
        A, B, C, h = T(M, K), T(K, N), T(M, N), T(M, N)
        return 2 * M * N * K, lambda: ops.gemm(M, N, K, A, K, B, N, C, N, b_mode=L.OPND_MNMAJOR,
                                               epilogue=L.EPI_BF16_DGELU, aux=h, ldaux=N, tile=tile)
    if case in ("fc1_dgrad", "qkv_dgrad"):
        M, N, K = {"fc1_dgrad": (12608, 768, 3072), "qkv_dgrad": (12608, 768, 2304)}[case]
        A, B, C = T(M, K), T(K, N), T(M, N)
        CHECK.append(lambda: (C.float(), A.float() @ B.float()))
        return 2 * M * N * K, lambda: ops.gemm(M, N, K, A, K, B, N, C, N, b_mode=L.OPND_MNMAJOR,
                                               epilogue=L.EPI_BF16, tile=tile)
    if case in ("fc1_dgrad_t", "qkv_dgrad_t", "fc2_dgrad_t"):
        # the dgrads with a pre-transposed weight: B K-contiguous (KM x KM)
        M, N, K = {"fc1_dgrad_t": (12608, 768, 3072), "qkv_dgrad_t": (12608, 768, 2304),
                   "fc2_dgrad_t": (12608, 3072, 768)}[case]
        A, B, C, h = T(M, K), T(N, K), T(M, N), T(M, N)
        if case == "fc2_dgrad_t":
            return 2 * M * N * K, lambda: ops.gemm(M, N, K, A, K, B, K, C, N,
                                                   epilogue=L.EPI_BF16_DGELU, aux=h, ldaux=N,
                                                   tile=tile)
        CHECK.append(lambda: (C.float(), A.float() @ B.float().t()))
        return 2 * M * N * K, lambda: ops.gemm(M, N, K, A, K, B, K, C, N, epilogue=L.EPI_BF16,
                                               tile=tile)
    if case == "proj_dgrad_t":
        M, N, K = 12608, 768, 768
        A, B, C = T(M, K), T(N, K), T(M, N)
        CHECK.append(lambda: (C.float(), A.float() @ B.float().t()))
        return 2 * M * N * K, lambda: ops.gemm(M, N, K, A, K, B, K, C, N, epilogue=L.EPI_BF16,
                                               tile=tile)
    if case in ("proj_fwd_resid", "fc2x3_fwd_resid", "projx3_fwd_resid"):
        M, N, K = {"proj_fwd_resid": (12608, 768, 768), "fc2x3_fwd_resid": (12608, 768, 9216),
                   "projx3_fwd_resid": (12608, 768, 2304)}[case]
        A, B = T(M, K), T(N, K)
        C, X = T(M, N, dtype=torch.float32), T(M, N, dtype=torch.float32)
        bias = T(N, dtype=torch.float32)
        CHECK.append(lambda: (C - X, A.float() @ B.float().t() + bias))
        return 2 * M * N * K, lambda: ops.gemm(M, N, K, A, K, B, K, C, N,
                                               epilogue=L.EPI_F32_RESID, bias=bias, aux=X,
                                               ldaux=N, tile=tile)
    if case == "fc2_fwd_resid":  # the step's fc2 forward: fp32 residual-stream epilogue
        M, N, K = 12608, 768, 3072
        A, B = T(M, K), T(N, K)
        C, X = T(M, N, dtype=torch.float32), T(M, N, dtype=torch.float32)
        bias = T(N, dtype=torch.float32)
        CHECK.append(lambda: (C - X, A.float() @ B.float().t() + bias))
        return 2 * M * N * K, lambda: ops.gemm(M, N, K, A, K, B, K, C, N,
                                               epilogue=L.EPI_F32_RESID, bias=bias, aux=X,
                                               ldaux=N, tile=tile)
    if case in ("fc2_wgrad", "qkv_wgrad", "proj_wgrad"):
        M, N, K = {"fc2_wgrad": (768, 3072, 12608), "qkv_wgrad": (2304, 768, 12608),
                   "proj_wgrad": (768, 768, 12608)}[case]
        A, B = T(K, M), T(K, N)
        C = torch.zeros(M, N, device="cuda")
        CHECK.append(lambda: (C.clone(), A.float().t() @ B.float()))
        return 2 * M * N * K, lambda: ops.gemm(M, N, K, A, M, B, N, C, N, a_mode=L.OPND_MNMAJOR,
                                               b_mode=L.OPND_MNMAJOR, epilogue=L.EPI_F32_ACC,
                                               tile=tile)
    if case == "fc1_wgrad":
        M, N, K = 3072, 768, 12608
        A, B = T(K, M), T(K, N)
        C = torch.zeros(M, N, device="cuda")
        return 2 * M * N * K, lambda: ops.gemm(M, N, K, A, M, B, N, C, N, a_mode=L.OPND_MNMAJOR,
                                               b_mode=L.OPND_MNMAJOR, epilogue=L.EPI_F32_ACC,
                                               tile=tile)
    if case in ("l1c3x3_fwd", "l1c1x3_fwd", "l3c2x3_fwd"):
        # the parity mode's bf16x3 ResNet convs on interleaved hi/lo pairs (functional.conv_fwd_x3):
        # layer-1 conv3 (1x1, 64 -> 256) and conv1 (1x1, 256 -> 64), layer-3 conv2 (3x3, 256)
        n, h, w, c, k, r = {"l1c3x3_fwd": (64, 56, 56, 64, 256, 1),
                            "l1c1x3_fwd": (64, 56, 56, 256, 64, 1),
                            "l3c2x3_fwd": (64, 14, 14, 256, 256, 3)}[case]
        M = n * h * w
        hi, lo = T(M, c), T(M, c)
        w3 = T(k, r * r * 2 * c)
        y, y_lo = T(M, k), T(M, k)
        st = torch.empty(ops.stats_tiles(M), 2, k, device="cuda")
        xk = dict(x3=True, a_lo=lo, x3_pairs=True, aux_out=y_lo, ldaux_out=k)
        if r == 1:
            return 2 * M * k * c * 3, lambda: ops.gemm(M, k, 2 * c, hi, c, w3, 2 * c, y, k,
                                                       epilogue=L.EPI_F32_STATS, stats=st,
                                                       tile=tile, **xk)
        g3 = ops.ConvGeom(n, h, w, 2 * c, k, r, r, 1, 1)
        K3 = r * r * 2 * c
        return 2 * M * k * r * r * c * 3, lambda: ops.gemm(M, k, K3, hi, 0, w3, K3, y, k,
                                                           a_mode=L.OPND_CONV_FWD,
                                                           epilogue=L.EPI_F32_STATS, stats=st,
                                                           conv=g3, tile=tile, **xk)
    if case == "l1c3_fwd":
        M, N, K = 200704, 256, 64
        A, B, C = T(M, K), T(N, K), T(M, N)
        st = torch.empty(ops.stats_tiles(M), 2, N, device="cuda")
        return 2 * M * N * K, lambda: ops.gemm(M, N, K, A, K, B, K, C, N,
                                               epilogue=L.EPI_BF16_STATS, stats=st, tile=tile)
    raise SystemExit(f"unknown case {case}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("case")
    ap.add_argument("--tile", type=int, default=0)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--check", action="store_true", help="one launch checked against torch fp32")
    a = ap.parse_args()
    flops, fn = build(a.case, a.tile)
    fn()
    torch.cuda.synchronize()
    if a.check:
        if not CHECK:
            raise SystemExit(f"--check: no reference for {a.case}")
        got, ref = CHECK[0]()
        err = ((got - ref).abs().max() / ref.abs().max()).item()
        print(f"{a.case} tile {a.tile}: max rel err {err:.2e}")
        if not err < 1e-2:
            raise SystemExit(f"{a.case}: CHECK FAILED")
        return
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / a.iters
    print(f"{a.case} tile {a.tile}: {us:.1f} us  {flops / us / 1e6:.0f} TFLOP/s")


if __name__ == "__main__":
    main()
