"""Time every GEMM mode of the DFU step at its real B=64 shapes (HIP events) -> TFLOP/s,
for the library's automatic plan and (with --sweep) each forced tile shape, which is the
data the cost model in csrc/gemm.hip is calibrated on.
Usage (GPU box): python tools/gemm_bench.py [filter] [--sweep]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dfu-multimodal_amd")]
import torch  # noqa: E402

from dfu_hip import _lib as L  # noqa: E402
from dfu_hip import ops  # noqa: E402

dev = "cuda"
bf = torch.bfloat16
TILE_NAMES = ["auto", "128x128", "256x128", "128x256", "256x256", "128x128o2", "128x128w4",
              "256x256p8", "256x256ps", "192x256ps", "256x64", "128x64o2"]


def T(*s, dtype=bf):
    return (torch.randn(*s, device=dev) * 0.1).to(dtype)


def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3  # us


cases = []  # (name, flops, fn(tile))


def case(name, flops, args, **kw):
    def fn(tile=0):
        ops.gemm(*args, tile=tile, **kw)
    cases.append((name, flops, fn))


def lin(name, M, N, K):
    A, Bw = T(M, K), T(N, K)
    C = torch.empty(M, N, dtype=bf, device=dev)
    fl = 2 * M * N * K
    case(f"fwd  {name} {M}x{N}x{K}", fl, (M, N, K, A, K, Bw, K, C, N), epilogue=L.EPI_BF16)
    dY = T(M, N)  # dgrad: dX[M,K] = dY[M,N] W[N,K]
    dX = torch.empty(M, K, dtype=bf, device=dev)
    case(f"dgrd {name} {M}x{K}x{N}", fl, (M, K, N, dY, N, Bw, K, dX, K), b_mode=L.OPND_MNMAJOR,
         epilogue=L.EPI_BF16)
    X = T(M, K)
    dW = torch.zeros(N, K, device=dev)
    case(f"wgrd {name} {N}x{K}x{M}", fl, (N, K, M, dY, N, X, K, dW, K), a_mode=L.OPND_MNMAJOR,
         b_mode=L.OPND_MNMAJOR, epilogue=L.EPI_F32_ACC)


def conv(name, B, H, C, K, R, stride):
    pad = R // 2
    g = ops.ConvGeom(B, H, H, C, K, R, R, stride, pad)
    x = T(B * H * H, C)
    w = T(K, R * R * C)
    M = B * g.p * g.q
    y = torch.empty(M, K, dtype=bf, device=dev)
    st = torch.empty(ops.stats_tiles(M), 2, K, device=dev)
    fl = 2 * M * K * R * R * C
    plain = R == 1 and stride == 1
    if plain:
        case(f"cfwd {name}", fl, (M, K, C, x, C, w, C, y, K), epilogue=L.EPI_BF16_STATS, stats=st)
    else:
        case(f"cfwd {name}", fl, (M, K, R * R * C, x, 0, w, R * R * C, y, K),
             a_mode=L.OPND_CONV_FWD, epilogue=L.EPI_BF16_STATS, stats=st, conv=g)
    dy = T(M, K)
    dx = torch.empty(B * H * H, C, dtype=bf, device=dev)
    if plain:
        case(f"cdgd {name}", fl, (B * H * H, C, K, dy, K, w, C, dx, C), b_mode=L.OPND_MNMAJOR,
             epilogue=L.EPI_BF16)
    else:
        case(f"cdgd {name}", fl, (B * H * H, C, R * R * K, dy, 0, w, R * R * C, dx, C),
             a_mode=L.OPND_CONV_DGRAD, b_mode=L.OPND_CONV_DGRAD_W, epilogue=L.EPI_BF16, conv=g)
    Nw = R * R * C
    dw = torch.zeros(K, Nw, device=dev)
    if plain:
        case(f"cwgd {name}", fl, (K, C, M, dy, K, x, C, dw, C), a_mode=L.OPND_MNMAJOR,
             b_mode=L.OPND_MNMAJOR, epilogue=L.EPI_F32_ACC)
    else:
        case(f"cwgd {name}", fl, (K, Nw, M, dy, K, x, 0, dw, Nw), a_mode=L.OPND_MNMAJOR,
             b_mode=L.OPND_CONV_WGRAD_X, epilogue=L.EPI_F32_ACC, conv=g)


def stem(name, M, N, K, epi=L.EPI_BF16_STATS):
    A, W = T(M, K), T(N, K)
    y = torch.empty(M, N, dtype=bf if epi == L.EPI_BF16_STATS else torch.float32, device=dev)
    st = torch.empty(ops.stats_tiles(M), 2, N, device=dev)
    case(f"cfwd {name} {M}x{N}x{K}", 2 * M * N * K, (M, N, K, A, K, W, K, y, N), epilogue=epi,
         stats=st)


TOK = 64 * 197
lin("qkv", TOK, 2304, 768)
lin("proj", TOK, 768, 768)
lin("fc1", TOK, 3072, 768)
lin("fc2", TOK, 768, 3072)
stem("stem im2col", 802816, 64, 160)
stem("x3 l1c1 1x1 256->64 56", 200704, 64, 768, L.EPI_F32_STATS)
conv("l1c1 1x1 256->64 56", 64, 56, 256, 64, 1, 1)
conv("l1c2 3x3 64 56", 64, 56, 64, 64, 3, 1)
conv("l1c3 1x1 64->256 56", 64, 56, 64, 256, 1, 1)
conv("l2c2 3x3 128 s2 56", 64, 56, 128, 128, 3, 2)
conv("l3c2 3x3 256 14", 64, 14, 256, 256, 3, 1)
conv("l3c3 1x1 256->1024 14", 64, 14, 256, 1024, 1, 1)
conv("l4c2 3x3 512 7", 64, 7, 512, 512, 3, 1)
conv("l4ds 1x1 1024->2048 s2 14", 64, 14, 1024, 2048, 1, 2)

args = [a for a in sys.argv[1:] if not a.startswith("--")]
flt = args[0] if args else ""
sweep = "--sweep" in sys.argv
ab = "--ab" in sys.argv  # persistent vs one-workgroup-per-unit schedule, auto plan
tiles = range(len(TILE_NAMES)) if sweep else [0]
for a in sys.argv[1:]:
    if a.startswith("--tiles="):  # e.g. --tiles=0,6,10,11
        tiles = [int(t) for t in a.split("=", 1)[1].split(",")]
print(f"{'case':42s} " + " ".join(f"{TILE_NAMES[t]:>16s}" for t in tiles) +
      (f" {'one-shot':>16s}" for _ in [0]).__next__() * ab)
tot_us = 0.0
for name, flops, fn in cases:
    if flt and flt not in name:
        continue
    cells = []
    for t in tiles:
        try:
            us = timeit(lambda: fn(t))
        except L.DfuError:
            cells.append(f"{'-':>16s}")
            continue
        if t == 0:
            tot_us += us
        cells.append(f"{us:7.1f}us {flops / us / 1e6:6.0f}T")
    if ab:
        old = ops.gemm_set_persistent(0)
        try:
            us = timeit(lambda: fn(0))
        finally:
            ops.gemm_set_persistent(old)
        cells.append(f"{us:7.1f}us {flops / us / 1e6:6.0f}T")
    print(f"{name:42s} " + " ".join(cells), flush=True)
print(f"total (auto) {tot_us:.1f} us")
