"""Per-kernel numerics on the GPU: every libdfu_hip entry point against a plain PyTorch fp32
reference of the same op on the same (bf16-representable) inputs."""
import math

import pytest
import torch
import torch.nn.functional as F

from dfu_hip import _lib as L
from dfu_hip import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rnd(*shape, scale=1.0, dtype=torch.bfloat16, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(dtype).to(DEV)


def close(a, b, atol, rtol=0.0, what=""):
    a = a.float()
    b = b.float()
    err = (a - b).abs()
    tol = atol + rtol * b.abs()
    bad = (err > tol)
    assert not bad.any(), f"{what}: max err {err.max().item():.3e} (n_bad={bad.sum().item()})"


# ------------------------------------------------------------------------------ GEMM
TILES = [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11]  # auto, 128x128, 256x128, 128x256, 256x256,
# 128x128 @2/CU (8, 4 waves), phased 256x256, persistent phased 256x256 and 192x256, 4-wave
# 256x64 and 128x64 @2/CU


def gemm_t(*args, tile=0, **kw):
    """ops.gemm with a forced tile; skip the case when that tile has no such instantiation."""
    try:
        ops.gemm(*args, tile=tile, **kw)
    except L.DfuError as e:
        if tile and e.code == L.DFU_E_UNSUPPORTED:
            pytest.skip(f"tile {tile} not instantiated for this combination")
        raise


@pytest.mark.parametrize("tile", TILES)
@pytest.mark.parametrize("M,N,K", [(300, 200, 136), (128, 128, 64), (1000, 2304, 768), (64, 2, 512),
                                   (12608, 768, 768)])
def test_gemm_nt_f32(M, N, K, tile):
    A = rnd(M, K, seed=1)
    B = rnd(N, K, seed=2)
    C = torch.empty(M, N, dtype=torch.float32, device=DEV)
    gemm_t(M, N, K, A, K, B, K, C, N, epilogue=L.EPI_F32, tile=tile)
    ref = A.float() @ B.float().t()
    close(C, ref, atol=2e-3 * math.sqrt(K), what="nt_f32")


@pytest.mark.parametrize("tile", TILES)
@pytest.mark.parametrize("M,N,K", [(300, 200, 136), (777, 768, 3072)])
def test_gemm_nn_f32(M, N, K, tile):
    A = rnd(M, K, seed=3)
    Bkn = rnd(K, N, seed=4)
    C = torch.empty(M, N, dtype=torch.float32, device=DEV)
    gemm_t(M, N, K, A, K, Bkn, N, C, N, b_mode=L.OPND_MNMAJOR, epilogue=L.EPI_F32, tile=tile)
    close(C, A.float() @ Bkn.float(), atol=2e-3 * math.sqrt(K), what="nn_f32")


@pytest.mark.parametrize("tile", TILES)
@pytest.mark.parametrize("M,N,K,split", [(200, 136, 300, 1), (768, 2304, 12608, 4), (64, 147, 5000, 7),
                                         (768, 3072, 12608, 0), (296, 200, 4000, 0)])
def test_gemm_tn_acc(M, N, K, split, tile):
    Akm = rnd(K, M, seed=5)
    Bkn = rnd(K, (N + 7) // 8 * 8, seed=6)
    C = rnd(M, N, dtype=torch.float32, seed=7)
    ref = C + Akm.float().t() @ Bkn.float()[:, :N]
    gemm_t(M, N, K, Akm, M, Bkn, Bkn.shape[1], C, N, a_mode=L.OPND_MNMAJOR,
           b_mode=L.OPND_MNMAJOR, epilogue=L.EPI_F32_ACC, split_k=split, tile=tile)
    close(C, ref, atol=3e-3 * math.sqrt(K), what="tn_acc")


def test_gemm_split_slab_deterministic():
    """Split-K through fp32 slabs + reduce kernel is bitwise reproducible."""
    M, N, K = 768, 768, 12608
    Akm = rnd(K, M, seed=40)
    Bkn = rnd(K, N, seed=41)
    outs = []
    for _ in range(2):
        C = torch.zeros(M, N, dtype=torch.float32, device=DEV)
        ops.gemm(M, N, K, Akm, M, Bkn, N, C, N, a_mode=L.OPND_MNMAJOR, b_mode=L.OPND_MNMAJOR,
                 epilogue=L.EPI_F32_ACC, split_k=8)
        outs.append(C)
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("M,N,K,split", [(64, 64, 200704, 96), (64, 147, 65536, 64),
                                         (256, 128, 50176, 48), (64, 64, 4096, 8)])
def test_gemm_split_wide_reduce(M, N, K, split):
    """Small planes with many splits take the wave-split reduce (k_splitk_reduce_wide):
    vector and scalar (N = 147, the stem) forms against fp32, bitwise reproducible."""
    ldb = (N + 7) // 8 * 8  # MN-major operands need ld % 8 == 0 (the stem pads 147 -> 152)
    Akm = rnd(K, M, seed=42)
    Bkn = rnd(K, ldb, seed=43)
    ref = Akm.float().t() @ Bkn[:, :N].float()
    outs = []
    for _ in range(2):
        C = torch.full((M, N), 0.25, dtype=torch.float32, device=DEV)
        ops.gemm(M, N, K, Akm, M, Bkn, ldb, C, N, a_mode=L.OPND_MNMAJOR, b_mode=L.OPND_MNMAJOR,
                 epilogue=L.EPI_F32_ACC, split_k=split)
        outs.append(C)
    assert torch.equal(outs[0], outs[1])
    close(outs[0], ref + 0.25, atol=2e-3 * (K ** 0.5), rtol=1e-3, what="wide reduce")


def gemm_or_auto(*args, tile=0, **kw):
    """ops.gemm with a tile preference; falls back to auto where that tile is not built."""
    try:
        ops.gemm(*args, tile=tile, **kw)
    except L.DfuError as e:
        if not (tile and e.code == L.DFU_E_UNSUPPORTED):
            raise
        ops.gemm(*args, **kw)


@pytest.mark.parametrize("tile", TILES)
def test_gemm_epilogues(tile):
    def gemm(*a, **k):
        gemm_or_auto(*a, tile=tile, **k)

    M, N, K = 333, 256, 192
    A = rnd(M, K, seed=8)
    B = rnd(N, K, seed=9)
    bias = rnd(N, dtype=torch.float32, seed=10)
    acc = A.float() @ B.float().t()
    C = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    gemm(M, N, K, A, K, B, K, C, N, epilogue=L.EPI_BF16, bias=bias, alpha=0.5)
    close(C, acc * 0.5 + bias, atol=3e-2, rtol=1e-2, what="bf16 bias alpha")
    gemm(M, N, K, A, K, B, K, C, N, epilogue=L.EPI_BF16_RELU, bias=bias)
    close(C, torch.relu(acc + bias), atol=3e-2, rtol=1e-2, what="relu")
    pre = torch.empty_like(C)
    gemm(M, N, K, A, K, B, K, C, N, epilogue=L.EPI_BF16_GELU, bias=bias, aux_out=pre, ldaux_out=N)
    u = acc + bias  # aux_out carries gelu'(pre) (the DGELU epilogue's factor)
    dgu = 0.5 * (1 + torch.erf(u / math.sqrt(2))) + u * torch.exp(-0.5 * u * u) / math.sqrt(2 * math.pi)
    close(pre, dgu, atol=3e-2, rtol=1e-2, what="gelu derivative")
    close(C, F.gelu(u), atol=3e-2, rtol=1e-2, what="gelu")
    res = rnd(M, N, dtype=torch.float32, seed=11)
    Cf = torch.empty(M, N, dtype=torch.float32, device=DEV)
    gemm(M, N, K, A, K, B, K, Cf, N, epilogue=L.EPI_F32_RESID, bias=bias, aux=res, ldaux=N)
    close(Cf, res + acc + bias, atol=2e-3 * math.sqrt(K), what="resid")
    # dgrad-style epilogues (B as [K][N])
    Bkn = rnd(K, N, seed=12)
    acc2 = A.float() @ Bkn.float()
    h = rnd(M, N, seed=13)
    gemm(M, N, K, A, K, Bkn, N, C, N, b_mode=L.OPND_MNMAJOR, epilogue=L.EPI_BF16_DGELU, aux=h, ldaux=N)
    close(C, acc2 * h.float(), atol=5e-2, rtol=1e-2, what="dgelu")  # acc * aux (aux = gelu')
    gemm(M, N, K, A, K, Bkn, N, C, N, b_mode=L.OPND_MNMAJOR, epilogue=L.EPI_BF16_ADD, aux=h, ldaux=N)
    close(C, acc2 + h.float(), atol=5e-2, rtol=1e-2, what="add")


@pytest.mark.parametrize("tile", TILES)
@pytest.mark.parametrize("M", [1000, 1100, 1024])
def test_gemm_stats(M, tile):
    N, K = 192, 128
    A = rnd(M, K, seed=14)
    B = rnd(N, K, seed=15)
    C = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    tiles = ops.stats_tiles(M)
    stats = torch.empty(tiles, 2, N, dtype=torch.float32, device=DEV)
    gemm_t(M, N, K, A, K, B, K, C, N, epilogue=L.EPI_BF16_STATS, stats=stats, tile=tile)
    ref = A.float() @ B.float().t()
    close(C, ref, atol=5e-2, rtol=1e-2, what="stats store")
    Cf = C.float()
    for t in range(tiles):
        blk = Cf[t * 128:(t + 1) * 128]
        close(stats[t, 0], blk.sum(0), atol=1e-2, rtol=1e-4, what="tile sum")
        close(stats[t, 1], ((blk - blk.mean(0)) ** 2).sum(0), atol=1e-2, rtol=1e-3, what="tile M2")


def test_gemm_patch():
    Bsz, T, D = 3, 196, 768
    M, K = Bsz * T, 768
    A = rnd(M, K, seed=16)
    W = rnd(D, K, seed=17, scale=0.05)
    bias = rnd(D, dtype=torch.float32, seed=18)
    pos = rnd(T + 1, D, dtype=torch.float32, seed=19)
    X = torch.zeros(Bsz, T + 1, D, dtype=torch.float32, device=DEV)
    ops.gemm(M, D, K, A, K, W, K, X, D, epilogue=L.EPI_PATCH, bias=bias, aux=pos, ldaux=D, ep_tokens=T)
    ref = (A.float() @ W.float().t() + bias).view(Bsz, T, D) + pos[1:]
    close(X[:, 1:], ref, atol=1e-2, what="patch")
    assert X[:, 0].abs().max().item() == 0.0


# ------------------------------------------------------------------------------ implicit conv
CONV_CASES = [
    # N, H, W, C, K, R, S, stride, pad
    (2, 14, 14, 64, 128, 3, 3, 1, 1),
    (2, 15, 15, 64, 64, 3, 3, 2, 1),
    (3, 14, 14, 128, 256, 1, 1, 2, 0),
    (2, 7, 7, 512, 512, 3, 3, 1, 1),
    (2, 28, 28, 128, 128, 3, 3, 2, 1),   # ResNet layer2 first block conv2 (stride phases)
    (2, 14, 14, 256, 512, 1, 1, 2, 0),   # downsample 1x1/s2: 3 of 4 phases have no tap
]


def _nhwc(t):
    return t.permute(0, 2, 3, 1).contiguous()


@pytest.mark.parametrize("tile", TILES)
@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_fwd_dgrad_wgrad(case, tile):
    N, H, W, C, K, R, S, st, pad = case
    g = ops.ConvGeom(N, H, W, C, K, R, S, st, pad)
    x = rnd(N, C, H, W, seed=20)
    w = rnd(K, C, R, S, seed=21, scale=0.1)
    xf = x.float().requires_grad_(True)
    wf = w.float().requires_grad_(True)
    y_ref = F.conv2d(xf, wf, stride=st, padding=pad)
    dy = rnd(*y_ref.shape, seed=22)
    y_ref.backward(dy.float())
    x_nhwc = _nhwc(x)
    w_krsc = ops.pack_conv_weight(w.float())
    M = N * g.p * g.q
    Y = torch.empty(M, K, dtype=torch.bfloat16, device=DEV)
    stats = torch.empty(ops.stats_tiles(M), 2, K, dtype=torch.float32, device=DEV)
    if R == 1 and S == 1 and st == 1:
        gemm_or_auto(M, K, C, x_nhwc, C, w_krsc, C, Y, K, epilogue=L.EPI_BF16_STATS, stats=stats, tile=tile)
    else:
        gemm_or_auto(M, K, R * S * C, x_nhwc, 0, w_krsc, R * S * C, Y, K, a_mode=L.OPND_CONV_FWD,
                 epilogue=L.EPI_BF16_STATS, stats=stats, conv=g, tile=tile)
    close(Y.view(N, g.p, g.q, K), _nhwc(y_ref.detach()), atol=5e-2, rtol=1e-2, what="conv fwd")
    # dgrad
    dy_nhwc = _nhwc(dy)
    dX = torch.empty(N * H * W, C, dtype=torch.bfloat16, device=DEV)
    gemm_or_auto(N * H * W, C, R * S * K, dy_nhwc, 0, w_krsc, R * S * C, dX, C,
             a_mode=L.OPND_CONV_DGRAD, b_mode=L.OPND_CONV_DGRAD_W, epilogue=L.EPI_BF16, conv=g, tile=tile)
    close(dX.view(N, H, W, C), _nhwc(xf.grad), atol=5e-2, rtol=1e-2, what="conv dgrad")
    # dgrad + addend (the bottleneck's identity/downsample gradient), separate and in place
    base = rnd(N * H * W, C, seed=23)
    dXa = torch.empty_like(dX)
    gemm_or_auto(N * H * W, C, R * S * K, dy_nhwc, 0, w_krsc, R * S * C, dXa, C,
                 a_mode=L.OPND_CONV_DGRAD, b_mode=L.OPND_CONV_DGRAD_W, epilogue=L.EPI_BF16_ADD,
                 aux=base, ldaux=C, conv=g, tile=tile)
    ref_add = _nhwc(xf.grad).reshape(-1, C) + base.float()
    close(dXa, ref_add, atol=6e-2, rtol=1e-2, what="conv dgrad + add")
    dXi = base.clone()
    gemm_or_auto(N * H * W, C, R * S * K, dy_nhwc, 0, w_krsc, R * S * C, dXi, C,
                 a_mode=L.OPND_CONV_DGRAD, b_mode=L.OPND_CONV_DGRAD_W, epilogue=L.EPI_BF16_ADD,
                 aux=dXi, ldaux=C, conv=g, tile=tile)
    close(dXi, ref_add, atol=6e-2, rtol=1e-2, what="conv dgrad + add in place")
    # wgrad (OIHW fp32 accumulate)
    dW = torch.zeros(K, C, R, S, dtype=torch.float32, device=DEV)
    acc = torch.zeros(K, R * S * C, dtype=torch.float32, device=DEV)
    gemm_or_auto(K, R * S * C, M, dy_nhwc, K, x_nhwc, 0, acc, R * S * C, a_mode=L.OPND_MNMAJOR,
             b_mode=L.OPND_CONV_WGRAD_X, epilogue=L.EPI_F32_ACC, conv=g, tile=tile)
    ops.conv_grad_krsc_to_oihw(acc, dW)
    close(dW, wf.grad, atol=2e-2 * math.sqrt(M / 100), rtol=1e-2, what="conv wgrad")


# ------------------------------------------------------------------------------ attention
@pytest.mark.parametrize("B,N,H", [(2, 197, 12), (1, 40, 2), (3, 256, 1)])
def test_attention(B, N, H):
    dh = 64
    qkv = rnd(B * N, 3 * H * dh, seed=30)
    scale = dh ** -0.5
    o, lse = ops.attention_fwd(qkv, B, N, H, dh, scale)
    q, k, v = qkv.float().view(B, N, 3, H, dh).permute(2, 0, 3, 1, 4).unbind(0)
    q.requires_grad_(True); k.requires_grad_(True); v.requires_grad_(True)
    ref = F.scaled_dot_product_attention(q, k, v)
    ref_o = ref.permute(0, 2, 1, 3).reshape(B * N, H * dh)
    close(o, ref_o, atol=2e-2, what="attn fwd")
    s = (q @ k.transpose(-1, -2)) * scale
    close(lse.view(B, H, -1)[:, :, :N], torch.logsumexp(s, -1), atol=1e-3, what="lse")
    do = rnd(B * N, H * dh, seed=31)
    ref_o.backward(do.float())
    dqkv = ops.attention_bwd(qkv, o, do, lse, B, N, H, dh, scale)
    dq, dk, dv = dqkv.float().view(B, N, 3, H, dh).permute(2, 0, 3, 1, 4).unbind(0)
    close(dq, q.grad, atol=3e-2, what="dq")
    close(dk, k.grad, atol=3e-2, what="dk")
    close(dv, v.grad, atol=3e-2, what="dv")


# ------------------------------------------------------------------------------ norms
def test_batchnorm_train_fwd_bwd():
    M, C = 5000, 128
    y = rnd(M, C, seed=40, scale=2.0) + 0.5
    A = torch.eye(C, dtype=torch.bfloat16, device=DEV)
    # produce stats through the GEMM epilogue: y @ I
    Y = torch.empty(M, C, dtype=torch.bfloat16, device=DEV)
    stats = torch.empty(ops.stats_tiles(M), 2, C, dtype=torch.float32, device=DEV)
    ops.gemm(M, C, C, y, C, A, C, Y, C, epilogue=L.EPI_BF16_STATS, stats=stats)
    gamma = rnd(C, dtype=torch.float32, seed=41) * 0.5 + 1
    beta = rnd(C, dtype=torch.float32, seed=42)
    rm = torch.zeros(C, device=DEV)
    rv = torch.ones(C, device=DEV)
    nbt = torch.zeros((), dtype=torch.int64, device=DEV)
    mean, invstd, scale, shift = (torch.empty(C, device=DEV) for _ in range(4))
    ops.bn_finalize(stats, M, C, gamma, beta, 1e-5, 0.1, rm, rv, nbt, mean, invstd, scale, shift)
    res = rnd(M, C, seed=43)
    out = torch.empty_like(Y)
    ops.bn_apply(Y, scale, shift, res, True, out, M, C)
    yf = Y.float().requires_grad_(True)
    gf = gamma.clone().requires_grad_(True)
    bf = beta.clone().requires_grad_(True)
    rm2 = torch.zeros(C, device=DEV)
    rv2 = torch.ones(C, device=DEV)
    ref = torch.relu(F.batch_norm(yf, rm2, rv2, gf, bf, training=True, momentum=0.1, eps=1e-5) + res.float())
    close(out, ref, atol=3e-2, rtol=1e-2, what="bn fwd")
    close(rm, rm2, atol=1e-4, what="running mean")
    close(rv, rv2, atol=1e-3, rtol=1e-3, what="running var")
    assert nbt.item() == 1
    dout = rnd(M, C, seed=44)
    ref.backward(dout.float())
    dy = torch.empty_like(Y)
    dres = torch.empty_like(Y)
    dgamma = torch.zeros(C, device=DEV)
    dbeta = torch.zeros(C, device=DEV)
    ops.bn_bwd(dout, Y, out, True, mean, invstd, gamma, M, C, dy, dres, dgamma, dbeta)
    close(dy, yf.grad, atol=2e-2, rtol=2e-2, what="bn dx")
    close(dgamma, gf.grad, atol=0.5, rtol=1e-2, what="dgamma")
    close(dbeta, bf.grad, atol=0.5, rtol=1e-2, what="dbeta")


@pytest.mark.parametrize("M,C", [(5000, 128), (3136, 2048), (200704, 64)])
def test_batchnorm_bwd_mask_from_y_is_bitwise(M, C):
    """relu=2 (mask recomputed from y with the forward scale/shift, `out` not read) and relu=3
    (the bitmask bn_apply wrote beside its output) equal relu=1 (mask from the stored BN+ReLU
    output) bit for bit."""
    y = rnd(M, C, seed=50, scale=2.0)
    stats = torch.empty(ops.stats_tiles(M), 2, C, dtype=torch.float32, device=DEV)
    Y = torch.empty(M, C, dtype=torch.bfloat16, device=DEV)
    ops.gemm(M, C, C, y, C, torch.eye(C, dtype=torch.bfloat16, device=DEV), C, Y, C,
             epilogue=L.EPI_BF16_STATS, stats=stats)
    gamma = rnd(C, dtype=torch.float32, seed=51) * 0.5 + 1
    beta = rnd(C, dtype=torch.float32, seed=52)
    mean, invstd, scale, shift = (torch.empty(C, device=DEV) for _ in range(4))
    ops.bn_finalize(stats, M, C, gamma, beta, 1e-5, 0.1, None, None, None, mean, invstd, scale,
                    shift)
    out = torch.empty_like(Y)
    mask = torch.empty(M * C // 8, dtype=torch.uint8, device=DEV)
    ops.bn_apply(Y, scale, shift, None, True, out, M, C, mask=mask)
    bits = ((mask.view(-1, 1) >> torch.arange(8, device=DEV, dtype=torch.uint8)) & 1).view(M, C)
    assert torch.equal(bits.bool(), out.float() > 0), "bitmask != (out > 0)"
    dout = rnd(M, C, seed=53)
    res = []
    for mode, o in ((1, out), (2, None), (3, mask)):
        dy = torch.empty_like(Y)
        dg, db = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
        ops.bn_bwd(dout, Y, o, mode, mean, invstd, gamma, M, C, dy, None, dg, db,
                   scale=scale, shift=shift)
        res.append((dy, dg, db))
    for other in res[1:]:
        for a, b in zip(res[0], other):
            assert torch.equal(a, b)


@pytest.mark.parametrize("M,C,relu", [(5000, 128, 1), (200704, 64, 3), (3136, 2048, 0)])
def test_batchnorm_bwd_one_call_equals_three(M, C, relu):
    """dfu_bn_bwd (the step's path: one C call, one workspace) is bit for bit the three-call
    sequence reduce -> finalize -> apply it replaces (sliced finalize included: M = 200704)."""
    lib = L.load()
    y = rnd(M, C, seed=60, scale=2.0)
    stats = torch.empty(ops.stats_tiles(M), 2, C, dtype=torch.float32, device=DEV)
    Y = torch.empty(M, C, dtype=torch.bfloat16, device=DEV)
    ops.gemm(M, C, C, y, C, torch.eye(C, dtype=torch.bfloat16, device=DEV), C, Y, C,
             epilogue=L.EPI_BF16_STATS, stats=stats)
    gamma = rnd(C, dtype=torch.float32, seed=61) * 0.5 + 1
    beta = rnd(C, dtype=torch.float32, seed=62)
    mean, invstd, scale, shift = (torch.empty(C, device=DEV) for _ in range(4))
    ops.bn_finalize(stats, M, C, gamma, beta, 1e-5, 0.1, None, None, None, mean, invstd, scale,
                    shift)
    out = torch.empty_like(Y)
    mask = torch.empty(M * C // 8, dtype=torch.uint8, device=DEV)
    ops.bn_apply(Y, scale, shift, rnd(M, C, seed=63) if relu == 1 else None, relu != 0, out, M,
                 C, mask=mask)
    o = {0: None, 1: out, 3: mask}[relu]
    dout = rnd(M, C, seed=64)

    def grads():
        return (torch.empty_like(Y), torch.empty_like(Y), torch.full((C,), 0.25, device=DEV),
                torch.full((C,), -0.5, device=DEV))
    dy1, dr1, dg1, db1 = grads()
    ops.bn_bwd(dout, Y, o, relu, mean, invstd, gamma, M, C, dy1, dr1, dg1, db1)
    dy2, dr2, dg2, db2 = grads()
    s = ops.stream_ptr()
    blocks = lib.dfu_bn_bwd_blocks(M, C)
    partial = torch.empty(blocks, 2, C, dtype=torch.float32, device=DEV)
    P = lambda t: None if t is None else t.data_ptr()  # noqa: E731
    assert lib.dfu_bn_bwd_reduce(P(dout), P(Y), P(o), relu, None, None, P(mean), P(invstd), M, C,
                                 P(partial), s) == 0
    nb = lib.dfu_bn_bwd_finalize_ws_bytes(blocks, C)
    ws = torch.empty(max(nb, 8) // 8, dtype=torch.float64, device=DEV) if nb > 0 else None
    cnt = ops.tile_counters(torch.device(DEV)) if nb > 0 else None
    coef = torch.empty(C, 3, dtype=torch.float32, device=DEV)
    assert lib.dfu_bn_bwd_finalize(P(partial), blocks, M, C, P(gamma), P(invstd), 1, P(dg2),
                                   P(db2), P(coef), P(ws), P(cnt),
                                   0 if cnt is None else cnt.numel(), s) == 0
    assert lib.dfu_bn_bwd_apply(P(dout), P(Y), P(o), relu, None, None, P(mean), P(invstd),
                                P(coef), M, C, P(dy2), P(dr2), s) == 0
    torch.cuda.synchronize()
    for a, b, what in ((dy1, dy2, "dy"), (dr1, dr2, "dres"), (dg1, dg2, "dgamma"),
                       (db1, db2, "dbeta")):
        assert torch.equal(a, b), what
    # a workspace smaller than dfu_bn_bwd_ws_bytes is refused before any launch
    small = torch.empty(1, dtype=torch.float64, device=DEV)
    rc = lib.dfu_bn_bwd(P(dout), P(Y), P(o), relu, None, None, P(mean), P(invstd), P(gamma), M,
                        C, 1, None, None, P(dy1), None, P(small), 8, None, 0, s)
    assert rc == L.DFU_E_INVALID


def test_layernorm_fwd_bwd():
    rows, D = 1000, 768
    x = (torch.randn(rows, D, device=DEV) * 3 + 1).float()
    gamma = torch.randn(D, device=DEV)
    beta = torch.randn(D, device=DEV)
    out = torch.empty(rows, D, dtype=torch.bfloat16, device=DEV)
    mean = torch.empty(rows, device=DEV)
    rstd = torch.empty(rows, device=DEV)
    ops.layernorm_fwd(x, D, rows, D, gamma, beta, 1e-6, out, D, True, mean, rstd)
    xr = x.clone().requires_grad_(True)
    gr = gamma.clone().requires_grad_(True)
    br = beta.clone().requires_grad_(True)
    ref = F.layer_norm(xr, (D,), gr, br, 1e-6)
    close(out, ref, atol=3e-2, rtol=1e-2, what="ln fwd")
    dy = rnd(rows, D, seed=50)
    ref.backward(dy.float())
    gx = torch.randn(rows, D, device=DEV)
    gx0 = gx.clone()
    gxb = torch.empty(rows, D, dtype=torch.bfloat16, device=DEV)
    dgam = torch.zeros(D, device=DEV)
    dbet = torch.zeros(D, device=DEV)
    gsp = ops.layernorm_bwd(dy, D, True, x, D, mean, rstd, gamma, rows, D, gx, D, gxb, dgam, dbet,
                            gsum=True)
    close(gx, gx0 + xr.grad, atol=1e-3, rtol=1e-3, what="ln dx")
    gsum = torch.zeros(D, device=DEV)
    ops.reduce_partials_add(gsp, gsum)
    close(gsum, gx.sum(0), atol=1e-3, rtol=1e-4, what="ln updated-gradient column sums")
    close(gxb, gx, atol=2e-2, rtol=1e-2, what="ln dx bf16")
    close(dgam, gr.grad, atol=1e-2, rtol=1e-3, what="ln dgamma")
    close(dbet, br.grad, atol=1e-2, rtol=1e-3, what="ln dbeta")


# ------------------------------------------------------------------------------ misc
def test_pooling_and_layout():
    B, C, H, W = 2, 64, 112, 112
    x = rnd(B, C, H, W, seed=60)
    xn = _nhwc(x)
    y, am, P, Q = ops.maxpool_fwd(xn, B, H, W, C)
    xr = x.float().requires_grad_(True)
    ref = F.max_pool2d(xr, 3, 2, 1)
    close(y, _nhwc(ref.detach()), atol=0, what="maxpool fwd")
    dy = rnd(B, C, P, Q, seed=61)
    ref.backward(dy.float())
    dx = ops.maxpool_bwd(_nhwc(dy), am, B, H, W, C, P, Q)
    close(dx, _nhwc(xr.grad), atol=2e-2, rtol=1e-2, what="maxpool bwd")
    # the stem's fused bn1 + relu + maxpool == bn_apply(relu) then maxpool, bit for bit (odd
    # sizes too: windows clipped at both borders)
    for (Bb, Hh, Ww) in ((2, 112, 112), (3, 57, 61)):
        yb = rnd(Bb * Hh * Ww, C, seed=63)
        sc = torch.randn(C, device=DEV)
        sh = torch.randn(C, device=DEV)
        ab = torch.empty_like(yb)
        ops.bn_apply(yb, sc, sh, None, True, ab, Bb * Hh * Ww, C)
        y0, am0, P0, Q0 = ops.maxpool_fwd(ab, Bb, Hh, Ww, C)
        y1, am1, _, _ = ops.maxpool_fwd(yb, Bb, Hh, Ww, C, scale=sc, shift=sh)
        assert torch.equal(y0, y1) and torch.equal(am0, am1), "maxpool_bn_fwd"
        ref = F.max_pool2d(ab.view(Bb, Hh, Ww, C).permute(0, 3, 1, 2).float(), 3, 2, 1)
        close(y1, _nhwc(ref), atol=0, what="maxpool_bn_fwd vs torch")
        g = rnd(Bb, C, P0, Q0, seed=64)
        ar = ab.view(Bb, Hh, Ww, C).permute(0, 3, 1, 2).float().requires_grad_(True)
        F.max_pool2d(ar, 3, 2, 1).backward(g.float())
        dxo = ops.maxpool_bwd(_nhwc(g), am1, Bb, Hh, Ww, C, P0, Q0)
        close(dxo, _nhwc(ar.grad), atol=2e-2, rtol=1e-2, what="maxpool bwd (odd)")
    # avgpool
    x4 = rnd(B, 7, 7, 2048, seed=62)
    yf = ops.avgpool_fwd(x4, B, 49, 2048)
    close(yf, x4.float().mean((1, 2)), atol=1e-4, what="avgpool")
    g = torch.randn(B, 2048, device=DEV)
    dx4 = ops.avgpool_bwd(g, B, 49, 2048)
    close(dx4, (g / 49)[:, None, :].expand(B, 49, 2048), atol=1e-3, rtol=1e-2, what="avgpool bwd")
    # stem im2col and patchify vs unfold
    xi = torch.randn(2, 3, 224, 224, device=DEV)
    for xin in (xi, xi.contiguous(memory_format=torch.channels_last),
                torch.randn(3, 3, 57, 61, device=DEV)):
        col, P, Q = ops.im2col_f32(xin, 7, 7, 2, 3, 160)
        ref = F.unfold(xin, 7, padding=3, stride=2).transpose(1, 2).reshape(-1, 147)
        assert torch.equal(col[:, :147].float(), ref.to(torch.bfloat16).float()), "im2col"
        assert col[:, 147:].abs().max().item() == 0
        # the bf16x3 split pair: hi == the bf16 col, hi + lo == the fp32 unfold
        (c_hi, c_lo), _, _ = ops.im2col_f32_x3(xin, 7, 7, 2, 3, 160)
        assert torch.equal(c_hi, col), "im2col x3 hi"
        rec = c_hi[:, :147].float() + c_lo[:, :147].float()
        close(rec, ref, atol=1e-6, rtol=1e-5, what="im2col x3 hi + lo")
    pt = ops.patchify_f32(xi, 16)
    ref = F.unfold(xi, 16, stride=16).transpose(1, 2).reshape(-1, 768)
    close(pt, ref, atol=2e-2, rtol=1e-2, what="patchify")
    # weight packing
    w = torch.randn(64, 32, 3, 3, device=DEV)
    close(ops.pack_conv_weight(w), w.permute(0, 2, 3, 1), atol=2e-2, rtol=1e-2, what="pack")


def test_colsum_ce_adamw_dropout():
    x = rnd(12608, 768, seed=70)
    out = torch.ones(768, device=DEV)
    ops.colsum_add(x, out)
    close(out, 1 + x.float().sum(0), atol=1e-2, rtol=1e-4, what="colsum")
    logits = torch.randn(64, 2, device=DEV)
    labels = torch.randint(0, 2, (64,), device=DEV)
    w = torch.tensor([2.0, 3.0], device=DEV)
    loss = torch.empty(1, device=DEV)
    dl = torch.empty_like(logits)
    ops.ce_weighted_fwd(logits, labels, w, loss, dl)
    lr = logits.clone().requires_grad_(True)
    ref = F.cross_entropy(lr, labels, weight=w)
    ref.backward()
    close(loss, ref.detach().view(1), atol=1e-5, what="ce")
    close(dl, lr.grad, atol=1e-6, what="ce grad")
    # AdamW vs torch.optim.AdamW over 3 steps
    n = 10007
    p = torch.randn(n, device=DEV)
    pr = p.clone().requires_grad_(True)
    opt = torch.optim.AdamW([pr], lr=1e-3, weight_decay=1e-2)
    m = torch.zeros(n, device=DEV)
    v = torch.zeros(n, device=DEV)
    step = torch.zeros((), dtype=torch.int64, device=DEV)
    for i in range(3):
        g = torch.randn(n, device=DEV)
        pr.grad = g.clone()
        opt.step()
        ops.step_increment(step)
        ops.adamw_flat(p, g, m, v, 1e-3, 0.9, 0.999, 1e-8, 1e-2, step)
    close(p, pr.detach(), atol=1e-6, rtol=1e-5, what="adamw")
    # dropout statistics and backward consistency
    xd = torch.ones(1 << 20, device=DEV)
    off = torch.zeros((), dtype=torch.int64, device=DEV)
    yd, mask = ops.dropout_fwd(xd, 0.7, 1234, off)
    keep = mask.float().mean().item()
    assert abs(keep - 0.3) < 0.01
    close(yd, mask.float() / 0.3, atol=1e-5, what="dropout scale")
    assert off.item() == xd.numel()
    dx = ops.dropout_bwd(torch.ones_like(xd), mask, 0.7)
    close(dx, yd, atol=1e-6, what="dropout bwd")
