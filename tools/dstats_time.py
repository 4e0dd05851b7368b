"""Time one dgrad GEMM with the plain bf16 epilogue vs the BN-statistics (DSTATS) epilogue,
plus the separate dfu_bn_bwd_reduce pass it replaces (layer shapes of ResNet-50 at B=64)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dfu-multimodal_amd")]
import torch  # noqa: E402

from dfu_hip import _lib as L  # noqa: E402
from dfu_hip import ops  # noqa: E402

DEV = "cuda"


def timeit(fn, iters=30):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def case(name, M, C, K, conv=None, tile=0):
    dy = (torch.randn(M if conv is None else conv.n * conv.p * conv.q, K if conv is None else conv.k,
                      device=DEV) * 0.1).bfloat16()
    if conv is None:
        w = (torch.randn(K, C, device=DEV) * 0.05).bfloat16()
        kw = dict(b_mode=L.OPND_MNMAJOR)
        args = (M, C, K, dy, K, w, C)
    else:
        w = ops.pack_conv_weight(torch.randn(conv.k, conv.c, conv.r, conv.s, device=DEV) * 0.05)
        kw = dict(a_mode=L.OPND_CONV_DGRAD, b_mode=L.OPND_CONV_DGRAD_W, conv=conv)
        args = (M, C, conv.r * conv.s * conv.k, dy, 0, w, conv.r * conv.s * conv.c)
    y = torch.randn(M, C, device=DEV).bfloat16()
    coef = torch.rand(4, C, device=DEV) + 0.5
    dx = torch.empty(M, C, device=DEV, dtype=torch.bfloat16)
    st = torch.empty(ops.stats_tiles(M), 2, C, device=DEV)
    t_bf = timeit(lambda: ops.gemm(*args, dx, C, epilogue=L.EPI_BF16, tile=tile, **kw))
    t_ds = timeit(lambda: ops.gemm(*args, dx, C, epilogue=L.EPI_BF16_DSTATS, aux=y, ldaux=C,
                                   stats=st, bn_coef=coef, tile=tile, **kw))
    blocks = ops.lib().dfu_bn_bwd_blocks(M, C)
    part = torch.empty(blocks, 2, C, device=DEV)
    sc, sf, mu, iv = coef.unbind(0)
    t_red = timeit(lambda: ops.check(ops.lib().dfu_bn_bwd_reduce(
        ops.ptr(dx), ops.ptr(y), None, 2, ops.ptr(sc), ops.ptr(sf), ops.ptr(mu), ops.ptr(iv), M,
        C, ops.ptr(part), ops.stream_ptr()), "reduce"))
    print(f"{name:28s} tile {tile}: bf16 {t_bf:7.1f} us  dstats {t_ds:7.1f} us  "
          f"(+{t_ds - t_bf:5.1f})  separate reduce {t_red:6.1f} us")


def main():
    g1 = ops.ConvGeom(64, 56, 56, 64, 64, 3, 3, 1, 1)
    g3 = ops.ConvGeom(64, 14, 14, 256, 256, 3, 3, 1, 1)
    for t in (0, 1, 5, 6):
        case("l1 conv2 dgrad 200704x64", 200704, 64, 576, conv=g1, tile=t)
        case("l3 conv2 dgrad 12544x256", 12544, 256, 2304, conv=g3, tile=t)
        case("l1 conv3 dgrad 200704x64x256", 200704, 64, 256, tile=t)
        case("l3 conv3 dgrad 12544x256x1024", 12544, 256, 1024, tile=t)


if __name__ == "__main__":
    main()
