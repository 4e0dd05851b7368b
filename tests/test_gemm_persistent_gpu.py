"""The persistent GEMM schedule against one workgroup per work unit.

Under the persistent schedule (csrc/gemm_kernel.h) a workgroup walks several output tiles as
one continuous K-step stream: the next tile's operands are in flight during the current tile's
epilogue and the counted vmcnt waits of the K-loop count that epilogue's stores.  The tile's
accumulation order does not change, so every output must be BITWISE equal to the one-unit-per-
workgroup launch of the same plan.  Shapes are chosen so that each workgroup owns several units
(more tiles than CUs x occupancy), with K as short as one K-step per tile (an epilogue every
step: the hardest case for the wait counts), ragged M, and N with and without N % 4 == 0."""
import math

import pytest
import torch

from dfu_hip import _lib as L
from dfu_hip import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"
TILES = [1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11]


def drnd(*shape, scale=1.0, dtype=torch.bfloat16, seed=0):
    g = torch.Generator(device=DEV).manual_seed(seed)
    return (torch.randn(*shape, generator=g, device=DEV) * scale).to(dtype)


def gemm_t(*args, tile=0, **kw):
    try:
        ops.gemm(*args, tile=tile, **kw)
    except L.DfuError as e:
        if tile and e.code == L.DFU_E_UNSUPPORTED:
            pytest.skip(f"tile {tile} not instantiated for this combination")
        raise


def both_schedules(run):
    """[outputs under the persistent schedule, outputs with one workgroup per unit]."""
    res = []
    for pers in (ops.PERSISTENT_ALL, 0):
        old = ops.gemm_set_persistent(pers)
        try:
            res.append([t.clone() for t in run()])
        finally:
            ops.gemm_set_persistent(old)
    torch.cuda.synchronize()
    return res


def assert_bitwise(res, what):
    for a, b in zip(*res):
        assert torch.equal(a, b), f"{what}: persistent != one-shot " \
            f"(max diff {(a.float() - b.float()).abs().max().item():.3e})"


SHAPES = [(12608, 2304, 64), (12601, 200, 192), (6001, 198, 128)]
EPIS = ["bf16", "gelu", "f32", "resid", "dgelu", "add", "stats", "acc", "acc_split", "patch"]


@pytest.mark.parametrize("tile", TILES)
@pytest.mark.parametrize("epi", EPIS)
@pytest.mark.parametrize("M,N,K", SHAPES)
def test_gemm_persistent_bitwise(M, N, K, epi, tile):
    n8, m8 = (N + 7) // 8 * 8, (M + 7) // 8 * 8
    A = drnd(M, K, seed=1)
    B = drnd(N, K, seed=2)
    Bkn = drnd(K, n8, seed=3)
    bias = drnd(N, dtype=torch.float32, seed=4)
    h16 = drnd(M, N, seed=5)
    r32 = drnd(M, N, dtype=torch.float32, seed=6)

    def run():
        if epi == "bf16":
            C = torch.full((M, N), 7.0, dtype=torch.bfloat16, device=DEV)
            gemm_t(M, N, K, A, K, B, K, C, N, epilogue=L.EPI_BF16, bias=bias, tile=tile)
            return [C]
        if epi == "gelu":
            C = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
            pre = torch.empty_like(C)
            gemm_t(M, N, K, A, K, B, K, C, N, epilogue=L.EPI_BF16_GELU, bias=bias, aux_out=pre,
                   ldaux_out=N, tile=tile)
            return [C, pre]
        if epi == "f32":
            C = torch.empty(M, N, dtype=torch.float32, device=DEV)
            gemm_t(M, N, K, A, K, Bkn, n8, C, N, b_mode=L.OPND_MNMAJOR, epilogue=L.EPI_F32,
                   tile=tile)
            return [C]
        if epi == "resid":
            C = torch.empty(M, N, dtype=torch.float32, device=DEV)
            gemm_t(M, N, K, A, K, B, K, C, N, epilogue=L.EPI_F32_RESID, bias=bias, aux=r32,
                   ldaux=N, tile=tile)
            return [C]
        if epi in ("dgelu", "add"):
            C = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
            gemm_t(M, N, K, A, K, Bkn, n8, C, N, b_mode=L.OPND_MNMAJOR,
                   epilogue=L.EPI_BF16_DGELU if epi == "dgelu" else L.EPI_BF16_ADD, aux=h16,
                   ldaux=N, tile=tile)
            return [C]
        if epi == "stats":
            C = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
            st = torch.full((ops.stats_tiles(M), 2, N), -1.0, device=DEV)
            gemm_t(M, N, K, A, K, B, K, C, N, epilogue=L.EPI_BF16_STATS, stats=st, tile=tile)
            return [C, st]
        if epi in ("acc", "acc_split"):
            Akm = drnd(K, m8, seed=7)
            C = r32.clone()
            gemm_t(M, N, K, Akm, m8, Bkn, n8, C, N, a_mode=L.OPND_MNMAJOR, b_mode=L.OPND_MNMAJOR,
                   epilogue=L.EPI_F32_ACC, split_k=1 if epi == "acc" else 2, tile=tile)
            return [C]
        if epi == "patch":
            T = 196
            Bsz = M // T
            Mp = Bsz * T
            pos = drnd(T + 1, N, dtype=torch.float32, seed=8)
            X = torch.zeros(Bsz, T + 1, N, dtype=torch.float32, device=DEV)
            gemm_t(Mp, N, K, A, K, B, K, X, N, epilogue=L.EPI_PATCH, bias=bias, aux=pos, ldaux=N,
                   ep_tokens=T, tile=tile)
            return [X]
        raise AssertionError(epi)

    res = both_schedules(run)
    assert_bitwise(res, f"{epi} {M}x{N}x{K} tile {tile}")
    if epi == "bf16":  # and the common result is the product itself
        ref = A.float() @ B.float().t() + bias
        err = (res[0][0].float() - ref).abs()
        assert (err <= 3e-2 + 1e-2 * ref.abs()).all(), err.max().item()
    if epi == "acc":
        Akm = drnd(K, m8, seed=7)
        ref = r32 + Akm.float()[:, :M].t() @ Bkn.float()[:, :N]
        assert (res[0][0] - ref).abs().max().item() < 3e-3 * math.sqrt(K)


CONV = [  # N, H, W, C, K, R, S, stride, pad — ResNet-50 layers at B = 64
    (64, 56, 56, 64, 64, 3, 3, 1, 1),
    (64, 28, 28, 128, 128, 3, 3, 2, 1),
    (64, 14, 14, 1024, 2048, 1, 1, 2, 0),
]


@pytest.mark.parametrize("tile", TILES)
@pytest.mark.parametrize("case", CONV)
def test_conv_persistent_bitwise(case, tile):
    Nb, H, W, C, K, R, S, st, pad = case
    g = ops.ConvGeom(Nb, H, W, C, K, R, S, st, pad)
    x = drnd(Nb * H * W, C, seed=11)
    w = drnd(K, R * S * C, seed=12, scale=0.1)
    M = Nb * g.p * g.q
    dy = drnd(M, K, seed=13)
    base = drnd(Nb * H * W, C, seed=14)

    def run():
        y = torch.empty(M, K, dtype=torch.bfloat16, device=DEV)
        stt = torch.empty(ops.stats_tiles(M), 2, K, device=DEV)
        if R == 1 and st == 1:
            gemm_t(M, K, C, x, C, w, C, y, K, epilogue=L.EPI_BF16_STATS, stats=stt, tile=tile)
        else:
            gemm_t(M, K, R * S * C, x, 0, w, R * S * C, y, K, a_mode=L.OPND_CONV_FWD,
                   epilogue=L.EPI_BF16_STATS, stats=stt, conv=g, tile=tile)
        dx = torch.empty(Nb * H * W, C, dtype=torch.bfloat16, device=DEV)
        gemm_t(Nb * H * W, C, R * S * K, dy, 0, w, R * S * C, dx, C, a_mode=L.OPND_CONV_DGRAD,
               b_mode=L.OPND_CONV_DGRAD_W, epilogue=L.EPI_BF16_ADD, aux=base, ldaux=C, conv=g,
               tile=tile)
        acc = torch.zeros(K, R * S * C, device=DEV)
        gemm_t(K, R * S * C, M, dy, K, x, 0, acc, R * S * C, a_mode=L.OPND_MNMAJOR,
               b_mode=L.OPND_CONV_WGRAD_X, epilogue=L.EPI_F32_ACC, conv=g, tile=tile)
        return [y, stt, dx, acc]

    assert_bitwise(both_schedules(run), f"conv {case} tile {tile}")


@pytest.mark.parametrize("tile", TILES)
@pytest.mark.parametrize("M,N,K,split", [(768, 3072, 12608, 3), (2304, 768, 12608, 4),
                                         (64, 147, 802816 // 16, 0), (300, 200, 4000, 7)])
def test_gemm_splitk_inkernel_bitwise(M, N, K, split, tile):
    """Split-K slabs reduced by the last-arriving split inside the GEMM (tile counters) equal the
    separate reduce kernel bitwise (same summation order), under both schedules; the counters
    come back zeroed (graph replays and the next launch rely on it)."""
    m8, n8 = (M + 7) // 8 * 8, (N + 7) // 8 * 8
    Akm = drnd(K, m8, seed=21)
    Bkn = drnd(K, n8, seed=22)
    C0 = drnd(M, N, dtype=torch.float32, seed=23)
    res = []
    for ink in (1, 0):
        old = ops.gemm_set_inkernel_reduce(ink)
        try:
            C = C0.clone()
            gemm_t(M, N, K, Akm, m8, Bkn, n8, C, N, a_mode=L.OPND_MNMAJOR, b_mode=L.OPND_MNMAJOR,
                   epilogue=L.EPI_F32_ACC, split_k=split, tile=tile)
            C2 = C0.clone()  # twice: counters must have been left zeroed
            gemm_t(M, N, K, Akm, m8, Bkn, n8, C2, N, a_mode=L.OPND_MNMAJOR,
                   b_mode=L.OPND_MNMAJOR, epilogue=L.EPI_F32_ACC, split_k=split, tile=tile)
            res.append((C, C2))
        finally:
            ops.gemm_set_inkernel_reduce(old)
    torch.cuda.synchronize()
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])
    assert torch.equal(res[0][0], res[0][1])
    assert int(ops.tile_counters(C0.device).abs().sum().item()) == 0
    ref = C0 + Akm.float()[:, :M].t() @ Bkn.float()[:, :N]
    assert (res[0][0] - ref).abs().max().item() < 3e-3 * math.sqrt(K)


def both_tail(run):
    """[outputs with the tail split, the same again, outputs without it]."""
    res = []
    for tail in (1, 1, 0):
        old = ops.gemm_set_tail_split(tail)
        try:
            res.append([t.clone() for t in run()])
        finally:
            ops.gemm_set_tail_split(old)
    torch.cuda.synchronize()
    return res


@pytest.mark.parametrize("tile", [0, 1, 5])
@pytest.mark.parametrize("M,N,K,epi", [(12608, 768, 3072, "bf16"), (12608, 768, 2304, "resid"),
                                       (3136, 512, 2048, "stats"), (1000, 300, 4096, "dgelu"),
                                       (6001, 200, 2560, "gelu")])
def test_gemm_tail_split(M, N, K, epi, tile):
    """Tail split (the last partial round's tiles split along K, the last split to arrive sums
    the fp32 slabs in split order and runs the epilogue): deterministic run to run, equal to the
    unsplit launch up to fp32 summation order, the tile counters left zeroed."""
    n8 = (N + 7) // 8 * 8
    A = drnd(M, K, seed=31)
    B = drnd(N, K, seed=32)
    Bkn = drnd(K, n8, seed=33)
    bias = drnd(N, dtype=torch.float32, seed=34)
    h16 = drnd(M, N, seed=35)
    r32 = drnd(M, N, dtype=torch.float32, seed=36)

    def run():
        if epi == "bf16":
            C = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
            gemm_t(M, N, K, A, K, B, K, C, N, epilogue=L.EPI_BF16, bias=bias, tile=tile)
            return [C]
        if epi == "resid":
            C = torch.empty(M, N, dtype=torch.float32, device=DEV)
            gemm_t(M, N, K, A, K, B, K, C, N, epilogue=L.EPI_F32_RESID, bias=bias, aux=r32,
                   ldaux=N, tile=tile)
            return [C]
        if epi == "stats":
            C = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
            st = torch.empty(ops.stats_tiles(M), 2, N, device=DEV)
            gemm_t(M, N, K, A, K, B, K, C, N, epilogue=L.EPI_BF16_STATS, stats=st, tile=tile)
            return [C, st]
        if epi == "dgelu":
            C = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
            gemm_t(M, N, K, A, K, Bkn, n8, C, N, b_mode=L.OPND_MNMAJOR,
                   epilogue=L.EPI_BF16_DGELU, aux=h16, ldaux=N, tile=tile)
            return [C]
        C = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
        pre = torch.empty_like(C)
        gemm_t(M, N, K, A, K, B, K, C, N, epilogue=L.EPI_BF16_GELU, bias=bias, aux_out=pre,
               ldaux_out=N, tile=tile)
        return [C, pre]

    e = {"bf16": L.EPI_BF16, "resid": L.EPI_F32_RESID, "stats": L.EPI_BF16_STATS,
         "dgelu": L.EPI_BF16_DGELU, "gelu": L.EPI_BF16_GELU}[epi]
    bm = L.OPND_MNMAJOR if epi == "dgelu" else L.OPND_KMAJOR
    if tile:  # (the automatic plan may pick a tile without a tail round)
        assert ops.gemm_workspace_bytes(M, N, K, L.OPND_KMAJOR, bm, e, tile=tile) > 0, "no tail"
    on, again, off = both_tail(run)
    for a, b in zip(on, again):
        assert torch.equal(a, b), f"tail split not deterministic ({epi} {M}x{N}x{K} tile {tile})"
    for a, b in zip(on, off):
        a, b = a.float(), b.float()
        tol = 2e-2 if a.dtype == torch.bfloat16 or epi in ("bf16", "dgelu", "gelu", "stats") else 1e-3
        assert ((a - b).abs() <= tol * (1 + b.abs())).all(), (a - b).abs().max().item()
    assert int(ops.tile_counters(A.device).abs().sum().item()) == 0
    if epi == "bf16":
        ref = A.float() @ B.float().t() + bias
        err = (on[0].float() - ref).abs()
        assert (err <= 3e-2 + 1e-2 * ref.abs()).all(), err.max().item()


@pytest.mark.parametrize("case", [(64, 7, 7, 512, 512, 3, 3, 1, 1),
                                  (64, 28, 28, 128, 128, 3, 3, 2, 1)])
def test_conv_tail_split(case):
    """Implicit-GEMM conv fwd (STATS) and strided dgrad (per-phase launches) with and without
    the tail split."""
    Nb, H, W, C, K, R, S, st, pad = case
    g = ops.ConvGeom(Nb, H, W, C, K, R, S, st, pad)
    x = drnd(Nb * H * W, C, seed=41)
    w = drnd(K, R * S * C, seed=42, scale=0.05)
    M = Nb * g.p * g.q
    dy = drnd(M, K, seed=43)

    def run():
        y = torch.empty(M, K, dtype=torch.bfloat16, device=DEV)
        stt = torch.empty(ops.stats_tiles(M), 2, K, device=DEV)
        ops.gemm(M, K, R * S * C, x, 0, w, R * S * C, y, K, a_mode=L.OPND_CONV_FWD,
                 epilogue=L.EPI_BF16_STATS, stats=stt, conv=g)
        dx = torch.empty(Nb * H * W, C, dtype=torch.bfloat16, device=DEV)
        ops.gemm(Nb * H * W, C, R * S * K, dy, 0, w, R * S * C, dx, C, a_mode=L.OPND_CONV_DGRAD,
                 b_mode=L.OPND_CONV_DGRAD_W, epilogue=L.EPI_BF16, conv=g)
        return [y, stt, dx]

    on, again, off = both_tail(run)
    for a, b in zip(on, again):
        assert torch.equal(a, b)
    for a, b in zip(on, off):
        a, b = a.float(), b.float()
        assert ((a - b).abs() <= 2e-2 * (1 + b.abs())).all(), (a - b).abs().max().item()
    assert int(ops.tile_counters(x.device).abs().sum().item()) == 0


@pytest.mark.parametrize("M,N,K", [(12608, 3072, 768), (1000, 768, 256)])
def test_dgelu_column_sums(M, N, K):
    """dGELU epilogue with `stats` on the persistent 256x256 tile: besides C = bf16(acc * aux),
    fp32 column sums of the stored C over each 128-row half of every 256-row tile (the fc1 bias
    gradient's partials, ViTBlockFn.backward); other tiles refuse the request."""
    A = drnd(M, K, seed=70)
    B = drnd(N, K, seed=71)
    aux = drnd(M, N, seed=72)
    C = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    parts = torch.full((2 * ((M + 255) // 256), N), float("nan"), device=DEV)
    ops.gemm(M, N, K, A, K, B, K, C, N, epilogue=L.EPI_BF16_DGELU, aux=aux, ldaux=N,
             stats=parts, tile=8)
    ref = torch.empty_like(C)
    ops.gemm(M, N, K, A, K, B, K, ref, N, epilogue=L.EPI_BF16_DGELU, aux=aux, ldaux=N, tile=8)
    assert torch.equal(C, ref), "the column sums changed the stored output"
    # the halves: rows [256 t + 128 h + 64 w .. ] -- wave row w of tile t covers rows
    # 256 t + {0..63, 128..191} (w = 0) and {64..127, 192..255} (w = 1)
    Cf = torch.zeros(parts.shape[0] // 2 * 256, N, device=DEV)
    Cf[:M] = C.float()
    blk = Cf.view(-1, 2, 2, 64, N)  # [tile][h][w][64 rows][N]
    want = blk.sum(dim=(1, 3)).reshape(-1, N)  # [tile * 2 + w][N]
    torch.cuda.synchronize()
    assert not torch.isnan(parts).any()
    assert torch.allclose(parts, want, rtol=1e-5, atol=1e-3 * (1 + want.abs().max().item()) * 1e-2)
    assert torch.allclose(parts.sum(0), C.float().sum(0), rtol=1e-4, atol=1e-2)
    with pytest.raises(L.DfuError):
        ops.gemm(M, N, K, A, K, B, K, C, N, epilogue=L.EPI_BF16_DGELU, aux=aux, ldaux=N,
                 stats=parts, tile=1)
