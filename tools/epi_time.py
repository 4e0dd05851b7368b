"""Standalone time of the fp16 fc1 GEMM (12608 x 3072 x 768, persistent 256x256 tile) with its
epilogues: BF16 (one bf16 output), F16_DUAL (one fp16 output) and F16_GELU (fp16 + bf16 gelu and
bf16 gelu').  With DFU_HIP_LIB=<experiment build> (tools/build_exp.sh) the same cases run on a
variant library.  python tools/epi_time.py [tag]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dfu-multimodal_amd")]
import torch  # noqa: E402

from dfu_hip import _lib as L  # noqa: E402
from dfu_hip import ops  # noqa: E402


def timeit(fn, iters=30):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


torch.manual_seed(0)  # the same operands in every process: checksums compare across builds
M, N, K = 12608, 3072, 768
A = (torch.randn(M, K, device="cuda") * 0.5).half()
B = (torch.randn(N, K, device="cuda") * 0.05).half()
bias = torch.randn(N, device="cuda") * 0.1
C2 = torch.empty(M, 2 * N, dtype=torch.bfloat16, device="cuda")
C = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
D = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
f = 2.0 * M * N * K
res = {}
res["BF16 (bf16 operands)"] = timeit(lambda: ops.gemm(M, N, K, A.view(torch.bfloat16), K,
                                                      B.view(torch.bfloat16), K, C, N,
                                                      epilogue=L.EPI_BF16, bias=bias, tile=8))
res["F16_DUAL"] = timeit(lambda: ops.gemm(M, N, K, A, K, B, K, C, N, epilogue=L.EPI_F16_DUAL,
                                          bias=bias, tile=8, operand_type=1))
res["F16_GELU"] = timeit(lambda: ops.gemm(M, N, K, A, K, B, K, C2, 2 * N, epilogue=L.EPI_F16_GELU,
                                          bias=bias, aux_out=D, ldaux_out=N, tile=8,
                                          operand_type=1))
tag = sys.argv[1] if len(sys.argv) > 1 else "product"
print(tag, " ".join(f"{k}: {v:.1f} us ({f / v / 1e6:.0f} TF)" for k, v in res.items()))
ops.gemm(M, N, K, A, K, B, K, C2, 2 * N, epilogue=L.EPI_F16_GELU, bias=bias, aux_out=D,
         ldaux_out=N, tile=8, operand_type=1)
torch.cuda.synchronize()
print(tag, "F16_GELU output checksums (fp16 gelu | bf16 gelu | bf16 gelu'):",
      int(C2[:, :N].contiguous().view(torch.int16).long().sum()),
      int(C2[:, N:].contiguous().view(torch.int16).long().sum()),
      int(D.view(torch.int16).long().sum()))
