"""Time the persistent 256x256 GEMM (tile 8) under a timing-ablation build of the library
(DFU_HIP_LIB=dfu_hip/libdfu_ablate_<mask>.so, tools/build_ablate.sh; results wrong by design):
what the K-loop's MFMAs, LDS reads, DMA, barrier and epilogue each cost on a square and the
ViT forward shapes.  One process per library ('zero': all-zero operands; a non-numeric tag is
an experiment build, whose results are checked against torch):
  for m in full 1 2 4 8 12 16; do python tools/gemm_ablate.py $m; done"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1] if len(sys.argv) > 1 else "full"
zero = len(sys.argv) > 2 and sys.argv[2] == "zero"  # zero operands: the clock the chip holds rises
if tag != "full":
    os.environ["DFU_HIP_LIB"] = os.path.join(ROOT, "dfu-multimodal_amd", "dfu_hip",
                                             f"libdfu_ablate_{tag}.so")
sys.path[:0] = [ROOT, os.path.join(ROOT, "dfu-multimodal_amd")]
import torch  # noqa: E402

from dfu_hip import _lib as L  # noqa: E402
from dfu_hip import ops  # noqa: E402


def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


out = []
for M, N, K in [(4096, 4096, 4096), (12608, 3072, 768), (12608, 768, 3072), (12608, 2304, 768)]:
    A = ((torch.rand(M, K, device="cuda") * 2 - 1) * (0 if zero else 1)).to(torch.bfloat16)
    B = ((torch.rand(N, K, device="cuda") * 2 - 1) * (0 if zero else 1)).to(torch.bfloat16)
    C = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    us = timeit(lambda: ops.gemm(M, N, K, A, K, B, K, C, N, epilogue=L.EPI_BF16, tile=8))
    if not tag.isdigit():  # an experiment build (not a timing ablation): check the result too
        ref = (A.float() @ B.float().t())
        err = ((C.float() - ref).abs().max() / ref.abs().max()).item()
        assert err < 1e-2, (tag, M, N, K, err)
    out.append(f"{M}x{N}x{K} {us:7.1f} us {2.0 * M * N * K / us / 1e6:6.0f} TF")
print(f"[{tag + (' zero' if zero else ''):>9s}] " + " | ".join(out), flush=True)
