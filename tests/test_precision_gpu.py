"""bf16x3 ("split-bf16") forward kernels (csrc/precise.hip) against plain PyTorch fp32.

Each kernel of the fp32-accurate forward mode is checked against the fp32 op it replaces: the
split itself (hi + lo reconstructs x to 2^-17), GEMMs over triples (fp32-grade products), the
F32_STATS epilogue (fp32 output + the BN tile statistics), BN apply with both residual forms,
maxpool / avgpool, LayerNorm, exact GELU and fp32 softmax attention.
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ops():
    from dfu_hip import _lib as L
    from dfu_hip import ops
    return L, ops


def _trip(t3, C):
    """hi + lo of a pattern-0 triple [rows][3C] and its two hi copies."""
    t = t3.float()
    return t[:, :C] + t[:, C:2 * C], t[:, :C], t[:, 2 * C:]


def _pair(x):
    """Split pair of fp32 x: (hi, lo) bf16 with hi + lo = x to 2^-17."""
    hi = x.to(torch.bfloat16)
    return hi, (x - hi.float()).to(torch.bfloat16)


def test_split_x3_patterns_and_padding():
    L, ops = _ops()
    torch.manual_seed(0)
    x = torch.randn(37, 147, device=DEV) * 3.0
    a = ops.split_x3(x, ops.X3_A, seg=160)
    b = ops.split_x3(x, ops.X3_B, seg=160)
    assert a.shape == (37, 480) and b.shape == (37, 480)
    af, bf = a.float(), b.float()
    hi = x.to(torch.bfloat16).float()
    # pattern A: hi | lo | hi ; pattern B: hi | hi | lo ; columns 147..159 of each segment zero
    for seg in (af[:, 0:160], af[:, 320:480], bf[:, 0:160], bf[:, 160:320]):
        assert torch.equal(seg[:, :147], hi) and torch.all(seg[:, 147:] == 0)
    recon = af[:, :147] + af[:, 160:307]
    assert torch.equal(bf[:, 320:467], af[:, 160:307])
    assert ((recon - x).abs() <= x.abs() * 2.0 ** -16).all()


def test_pack_conv_weight_x3():
    L, ops = _ops()
    w = torch.randn(64, 32, 3, 3, device=DEV)
    p = ops.pack_conv_weight_x3(w).float()  # [K][R][S][3C]
    krsc = w.permute(0, 2, 3, 1)
    hi = krsc.to(torch.bfloat16).float()
    assert torch.equal(p[..., :32], hi) and torch.equal(p[..., 32:64], hi)
    assert ((p[..., :32] + p[..., 64:] - krsc).abs() <= krsc.abs() * 2.0 ** -16).all()


def test_interleaved_pair_layouts():
    """Pattern X3_PAIRS (dfu_gemm_desc.x3_pairs' B operand): per 32 columns [hi 32 | lo 32],
    zero-padded to the segment; the conv weight packing the same along each tap's channels."""
    L, ops = _ops()
    torch.manual_seed(12)
    x = torch.randn(37, 147, device=DEV) * 3.0
    p = ops.split_x3(x, ops.X3_PAIRS, seg=160).float()
    assert p.shape == (37, 320)
    g = p.view(37, 5, 2, 32)
    hi, lo = g[:, :, 0].reshape(37, 160), g[:, :, 1].reshape(37, 160)
    assert torch.equal(hi[:, :147], x.to(torch.bfloat16).float()) and torch.all(hi[:, 147:] == 0)
    assert torch.equal(lo[:, :147], (x - hi[:, :147]).to(torch.bfloat16).float())
    assert torch.all(lo[:, 147:] == 0)
    assert ops.split_x3(x[:, :64], ops.X3_PAIRS).shape == (37, 128)
    with pytest.raises(L.DfuError):  # pattern 2 needs whole 32-column groups
        ops.split_x3(x, ops.X3_PAIRS, seg=152)
    w = torch.randn(64, 96, 3, 3, device=DEV)
    q = ops.pack_conv_weight_x3(w, ops.X3_PAIRS).float().view(64, 3, 3, 3, 2, 32)
    krsc = w.permute(0, 2, 3, 1)
    assert torch.equal(q[..., 0, :].reshape(64, 3, 3, 96), krsc.to(torch.bfloat16).float())
    kh = krsc.to(torch.bfloat16).float()
    assert torch.equal(q[..., 1, :].reshape(64, 3, 3, 96), (krsc - kh).to(torch.bfloat16).float())
    with pytest.raises(L.DfuError):
        ops.pack_conv_weight_x3(torch.randn(8, 48, 3, 3, device=DEV), ops.X3_PAIRS)


@pytest.mark.parametrize("conv,C", [(False, 160), (True, 128), (True, 96)])
def test_x3_pairs_gemm_every_tile(conv, C):
    """The interleaved-pair bf16x3 kernels (three products per K-step from a hi and a lo tile)
    on every tile that instantiates them -- F32_STATS with the pair output on tiles 1, 2, 10,
    11 -- K-major and implicit-conv A, ragged M: fp32-accurate
    against fp64, and within fp32 summation order of the tripled-K kernels (which need the
    conv's C % 64 == 0: C = 96 runs the pair kernels only)."""
    L, ops = _ops()
    torch.manual_seed(13)
    if conv:
        Bn, H, Kout, R, st_ = 5, 13, 192, 3, 2
        g = ops.ConvGeom(Bn, H, H, C, Kout, R, R, st_, 1)
        M = Bn * g.p * g.q
        x = torch.randn(Bn, C, H, H, device=DEV)
        w = torch.randn(Kout, C, R, R, device=DEV) / math.sqrt(C * R * R)
        rows = x.permute(0, 2, 3, 1).reshape(-1, C).contiguous()
        ref = torch.nn.functional.conv2d(x.double(), w.double(), stride=st_, padding=1)
        ref = ref.permute(0, 2, 3, 1).reshape(-1, Kout)
        w2, w3 = ops.pack_conv_weight_x3(w, ops.X3_PAIRS), ops.pack_conv_weight_x3(w)
        K2, K3 = R * R * 2 * C, R * R * 3 * C
        kw2 = dict(a_mode=L.OPND_CONV_FWD, conv=ops.ConvGeom(Bn, H, H, 2 * C, Kout, R, R, st_, 1))
        kw3 = dict(a_mode=L.OPND_CONV_FWD, conv=ops.ConvGeom(Bn, H, H, 3 * C, Kout, R, R, st_, 1))
        lda = 0
    else:
        M, Kout = 1001, 192
        rows = torch.randn(M, C, device=DEV)
        w = torch.randn(Kout, C, device=DEV) / math.sqrt(C)
        ref = rows.double() @ w.double().T
        w2, w3 = ops.split_x3(w, ops.X3_PAIRS), ops.split_x3(w, ops.X3_B)
        K2, K3, kw2, kw3, lda = 2 * C, 3 * C, {}, {}, C
    hi, lo = _pair(rows)
    st3 = torch.empty(ops.stats_tiles(M), 2, Kout, device=DEV)
    y3 = None
    if not conv or C % 64 == 0:
        y3 = torch.empty(M, Kout, device=DEV)
        ops.gemm(M, Kout, K3, hi, lda, w3, K3, y3, Kout, epilogue=L.EPI_F32_STATS, stats=st3,
                 x3=True, a_lo=lo, tile=1, **kw3)
    for tile in (1, 2, 10, 11):
        y = torch.full((M, Kout), float("nan"), device=DEV)
        st = torch.empty_like(st3)
        ops.gemm(M, Kout, K2, hi, lda, w2, K2, y, Kout, epilogue=L.EPI_F32_STATS, stats=st,
                 x3=True, a_lo=lo, x3_pairs=True, tile=tile, **kw2)
        assert ((y.double() - ref).norm() / ref.norm()).item() < 2e-5, tile
        if y3 is None:
            y3, st3 = y.clone(), st.clone()  # C = 96: the tiles against each other
        assert ((y - y3).norm() / y3.norm()).item() < 2e-6, tile
        assert ((st - st3).norm() / st3.norm()).item() < 1e-5, tile
        # the pair output (aux_out): hi = bf16(y), lo = bf16(y - hi)
        yh = torch.empty(M, Kout, dtype=torch.bfloat16, device=DEV)
        yl = torch.empty_like(yh)
        ops.gemm(M, Kout, K2, hi, lda, w2, K2, yh, Kout, epilogue=L.EPI_F32_STATS, stats=st,
                 x3=True, a_lo=lo, x3_pairs=True, tile=tile, aux_out=yl, ldaux_out=Kout, **kw2)
        assert torch.equal(yh, y.to(torch.bfloat16)), tile
        assert torch.equal(yl, (y - yh.float()).to(torch.bfloat16)), tile
    with pytest.raises(L.DfuError):  # no interleaved-pair kernel on the persistent tiles
        ops.gemm(M, Kout, K2, hi, lda, w2, K2, y3, Kout, epilogue=L.EPI_F32_STATS, stats=st3,
                 x3=True, a_lo=lo, x3_pairs=True, tile=8, **kw2)


@pytest.mark.parametrize("M,N,K", [(2048, 768, 768), (1000, 384, 3072), (333, 200, 160)])
def test_gemm_over_triples_is_fp32_accurate(M, N, K):
    """A3 . B3^T on the bf16 MFMA GEMM equals fp32 A . B^T to ~1e-5 relative (bf16: ~4e-3)."""
    L, ops = _ops()
    torch.manual_seed(1)
    A = torch.randn(M, K, device=DEV)
    B = torch.randn(N, K, device=DEV)
    ref = (A.double() @ B.double().T)
    A3, B3 = ops.split_x3(A, ops.X3_A), ops.split_x3(B, ops.X3_B)
    C = torch.empty(M, N, device=DEV)
    ops.gemm(M, N, 3 * K, A3, 3 * K, B3, 3 * K, C, N, epilogue=L.EPI_F32)
    err = ((C.double() - ref).norm() / ref.norm()).item()
    Cb = torch.empty(M, N, device=DEV)
    ops.gemm(M, N, K, A.to(torch.bfloat16), K, B.to(torch.bfloat16), K, Cb, N, epilogue=L.EPI_F32)
    errb = ((Cb.double() - ref).norm() / ref.norm()).item()
    print(f"\n[x3 gemm {M}x{N}x{K}] rel err {err:.2e} (plain bf16 {errb:.2e})")
    assert err < 2e-5 and errb > 20 * err


@pytest.mark.parametrize("M,N,K", [(12608, 3072, 768), (1000, 520, 200), (257, 264, 64)])
def test_x3_gelu_and_f32_epilogues_on_persistent_tile(M, N, K):
    """The bf16x3 ViT forward's fc1 + GELU on the persistent 256x256 tile (DFU_EPI_X3_GELU):
    the triple [hi | lo | hi] of gelu(A.B^T + bias) to ~1e-5 of fp64, gelu'(pre) in bf16, and
    the same GEMM with the plain fp32 epilogue (qkv); ragged M and N edges included."""
    import math
    L, ops = _ops()
    torch.manual_seed(11)
    A = torch.randn(M, K, device=DEV) * 0.5
    B = torch.randn(N, K, device=DEV) * (1.0 / math.sqrt(K))
    bias = torch.randn(N, device=DEV)
    A3, B3 = ops.split_x3(A, ops.X3_A), ops.split_x3(B, ops.X3_B)
    pre = A.double() @ B.double().T + bias.double()
    C = torch.empty(M, N, device=DEV)
    ops.gemm(M, N, 3 * K, A3, 3 * K, B3, 3 * K, C, N, epilogue=L.EPI_F32, bias=bias, tile=8)
    assert ((C.double() - pre).norm() / pre.norm()).item() < 2e-5
    h3 = torch.full((M, 3 * N), float("nan"), device=DEV).to(torch.bfloat16)
    dg = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    ops.gemm(M, N, 3 * K, A3, 3 * K, B3, 3 * K, h3, 3 * N, epilogue=L.EPI_X3_GELU, bias=bias,
             aux_out=dg, ldaux_out=N, tile=8)
    g = torch.nn.functional.gelu(pre)
    v, hi0, hi2 = _trip(h3, N)
    err = (v.double() - g).abs().max().item()
    print(f"\n[x3 gelu {M}x{N}x{K}] max abs err {err:.2e} (max |gelu| {g.abs().max().item():.2f})")
    assert err < 2e-5 * max(1.0, g.abs().max().item())
    assert torch.equal(hi0, hi2)
    dref = 0.5 * torch.erfc(-pre / math.sqrt(2)) + pre * torch.exp(-0.5 * pre * pre) / math.sqrt(2 * math.pi)
    assert ((dg.double() - dref).abs() <= 2.0 ** -8 * dref.abs() + 1e-5).all()
    with pytest.raises(L.DfuError):  # the fused triple exists on the persistent tile only
        ops.gemm(M, N, 3 * K, A3, 3 * K, B3, 3 * K, h3, 3 * N, epilogue=L.EPI_X3_GELU,
                 bias=bias, aux_out=dg, ldaux_out=N, tile=1)


@pytest.mark.parametrize("tile", [1, 2])
def test_f32_stats_epilogue(tile):
    """fp32 output + per-128-row (sum, M2) of the unrounded accumulators, both tiles that
    instantiate it; an implicit-GEMM conv forward over a channel-tripled input too."""
    L, ops = _ops()
    torch.manual_seed(2)
    M, N, K = 1000, 256, 192
    A = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    B = torch.randn(N, K, device=DEV).to(torch.bfloat16)
    C = torch.empty(M, N, device=DEV)
    st = torch.empty(ops.stats_tiles(M), 2, N, device=DEV)
    ops.gemm(M, N, K, A, K, B, K, C, N, epilogue=L.EPI_F32_STATS, stats=st, tile=tile)
    ref = A.float() @ B.float().T
    assert torch.allclose(C, ref, rtol=1e-5, atol=1e-4)
    for t in range(ops.stats_tiles(M)):
        blk = C[t * 128:(t + 1) * 128].double()
        s = blk.sum(0)
        q = ((blk - blk.mean(0)) ** 2).sum(0)
        assert torch.allclose(st[t, 0].double(), s, rtol=1e-5, atol=1e-3)
        assert torch.allclose(st[t, 1].double(), q, rtol=1e-4, atol=1e-2)


@pytest.mark.parametrize("R,stride", [(3, 1), (3, 2), (1, 1), (1, 2)])
def test_conv_fwd_x3_matches_fp32_conv(R, stride):
    """Conv forward over a split pair against fp64 conv2d: the interleaved-pair kernels (the
    default) within fp32 summation order of the tripled-K ones (hi | lo | hi read from two
    buffers: K-major for the 1x1 stride-1 case, the implicit-GEMM loader otherwise), which are
    bit-identical to the same GEMM over the materialised triple."""
    from dfu_hip import functional as Fn
    L, ops = _ops()
    torch.manual_seed(3)
    Bn, C, H, W, Kout = 4, 64, 14, 14, 128
    x = torch.randn(Bn, C, H, W, device=DEV)
    w = torch.randn(Kout, C, R, R, device=DEV) * 0.05
    pad = R // 2
    g = ops.ConvGeom(Bn, H, W, C, Kout, R, R, stride, pad)
    rows = x.permute(0, 2, 3, 1).reshape(-1, C).contiguous()
    M = Bn * g.p * g.q
    ref = torch.nn.functional.conv2d(x.double(), w.double(), stride=stride, padding=pad)
    ref = ref.permute(0, 2, 3, 1).reshape(-1, Kout)
    old = Fn._X3_PAIRS
    ys = []
    try:
        for pairs in (True, False):
            Fn._X3_PAIRS = pairs
            w3 = Fn.conv_weight_x3(w)
            y = torch.empty(M, Kout, device=DEV)
            st = torch.empty(ops.stats_tiles(M), 2, Kout, device=DEV)
            Fn.conv_fwd_x3(_pair(rows), g, w3, y, st)
            err = ((y.double() - ref).norm() / ref.norm()).item()
            assert err < 2e-5, (R, stride, pairs, err)
            # the same conv writing its output as a split pair (F32_STATS with aux_out): hi =
            # bf16(y), lo = bf16(y - hi) of the very fp32 values above, the same statistics
            yh = torch.empty(y.shape, dtype=torch.bfloat16, device=DEV)
            yl = torch.empty_like(yh)
            st2 = torch.empty_like(st)
            Fn.conv_fwd_x3(_pair(rows), g, w3, yh, st2, y_lo=yl)
            assert torch.equal(yh, y.to(torch.bfloat16)) and torch.equal(st2, st)
            assert torch.equal(yl, (y - yh.float()).to(torch.bfloat16))
            ys.append(y)
    finally:
        Fn._X3_PAIRS = old
    assert ((ys[0] - ys[1]).norm() / ys[1].norm()).item() < 2e-6
    # the tripled-K contraction over the materialised triple [hi | lo | hi]: bit-identical
    x3 = ops.split_x3(rows, ops.X3_A)
    y3 = torch.empty_like(y)
    if R == 1 and stride == 1:
        ops.gemm(M, Kout, 3 * C, x3, 3 * C, w3, 3 * C, y3, Kout, epilogue=L.EPI_F32_STATS,
                 stats=st, x3=True)
    else:
        g3 = ops.ConvGeom(Bn, H, W, 3 * C, Kout, R, R, stride, pad)
        ops.gemm(M, Kout, R * R * 3 * C, x3, 0, w3, R * R * 3 * C, y3, Kout,
                 a_mode=L.OPND_CONV_FWD, epilogue=L.EPI_F32_STATS, stats=st, conv=g3, x3=True)
    assert torch.equal(ys[1], y3)


@pytest.mark.parametrize("R,stride,C,H", [(3, 1, 512, 7), (3, 2, 256, 28), (1, 1, 2048, 7)])
def test_conv_fwd_x3_long_k_few_tiles(R, stride, C, H):
    """The layer-3/4 shapes (few output tiles over a long K) on the pair kernels: the output
    pair and the BN tile statistics against fp64 conv2d / fp64 statistics of the fp32 output."""
    from dfu_hip import functional as Fn
    L, ops = _ops()
    torch.manual_seed(10)
    Bn, Kout = 64, 512 if C >= 512 else 256
    x = torch.randn(Bn, C, H, H, device=DEV)
    w = torch.randn(Kout, C, R, R, device=DEV) / math.sqrt(C * R * R)
    pad = R // 2
    g = ops.ConvGeom(Bn, H, H, C, Kout, R, R, stride, pad)
    M = Bn * g.p * g.q
    rows = x.permute(0, 2, 3, 1).reshape(-1, C).contiguous()
    yh = torch.empty(M, Kout, dtype=torch.bfloat16, device=DEV)
    yl = torch.empty_like(yh)
    st = torch.empty(ops.stats_tiles(M), 2, Kout, device=DEV)
    Fn.conv_fwd_x3(_pair(rows), g, Fn.conv_weight_x3(w), yh, st, y_lo=yl)
    y = yh.double() + yl.double()
    ref = torch.nn.functional.conv2d(x.double(), w.double(), stride=stride, padding=pad)
    ref = ref.permute(0, 2, 3, 1).reshape(-1, Kout)
    assert ((y - ref).norm() / ref.norm()).item() < 2e-5
    for t in range(ops.stats_tiles(M)):
        blk = y[t * 128:(t + 1) * 128]
        assert torch.allclose(st[t, 0].double(), blk.sum(0), rtol=1e-4, atol=1e-3)
        q = ((blk - blk.mean(0)) ** 2).sum(0)
        assert torch.allclose(st[t, 1].double(), q, rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("C", [192, 160, 96])
def test_split_pair_gemm_ragged_and_rejects_bad_pairs(C):
    """K-major split pair on a ragged M (the lo buffer's rows past M are never read), segments
    that are and are not K-step multiples (160: the stem's im2col rows; each lane's 16-B chunk
    picks its segment), bit-identical to the materialised triple, and the descriptor check:
    lda must equal the segment."""
    L, ops = _ops()
    torch.manual_seed(8)
    M, N = 1001, 256
    x = torch.randn(M, C, device=DEV)
    w = torch.randn(N, C, device=DEV) / math.sqrt(C)
    hi, lo = _pair(x)
    w3 = ops.split_x3(w, ops.X3_B)
    y = torch.empty(M, N, device=DEV)
    st = torch.empty(ops.stats_tiles(M), 2, N, device=DEV)
    for tile in (1, 11):
        ops.gemm(M, N, 3 * C, hi, C, w3, 3 * C, y, N, epilogue=L.EPI_F32_STATS, stats=st,
                 x3=True, a_lo=lo, tile=tile)
        ref = x.double() @ w.double().T
        assert ((y.double() - ref).norm() / ref.norm()).item() < 2e-5
        y3 = torch.empty_like(y)
        ops.gemm(M, N, 3 * C, ops.split_x3(x, ops.X3_A), 3 * C, w3, 3 * C, y3, N,
                 epilogue=L.EPI_F32_STATS, stats=st, x3=True, tile=tile)
        assert torch.equal(y, y3), tile
    with pytest.raises(L.DfuError):
        ops.gemm(M, N, 3 * C, hi, 2 * C, w3, 3 * C, y, N, epilogue=L.EPI_F32_STATS, stats=st,
                 x3=True, a_lo=lo)


def test_stem_im2col_pair():
    """The stem's fp32 im2col as a split pair: hi = bf16(col), hi + lo = col to 2^-17."""
    L, ops = _ops()
    torch.manual_seed(9)
    x = torch.randn(2, 3, 224, 224, device=DEV)
    (hi, lo), P, Q = ops.im2col_f32_x3(x, 7, 7, 2, 3, 160)
    col = torch.nn.functional.unfold(x, 7, padding=3, stride=2).transpose(1, 2).reshape(-1, 147)
    assert (P, Q) == (112, 112) and hi.shape == (2 * 112 * 112, 160)
    assert torch.equal(hi[:, :147], col.to(torch.bfloat16)) and torch.all(hi[:, 147:] == 0)
    v = hi[:, :147].float() + lo[:, :147].float()
    assert ((v - col).abs() <= col.abs() * 2.0 ** -16).all() and torch.all(lo[:, 147:] == 0)


def test_bn_apply_x3_residual_modes():
    L, ops = _ops()
    torch.manual_seed(4)
    M, C = 3000, 256
    y = torch.randn(M, C, device=DEV)
    sc = torch.rand(C, device=DEV) + 0.5
    sh = torch.randn(C, device=DEV)
    res = torch.randn(M, C, device=DEV)
    rhi, rlo = _pair(res)
    for mode, r, rl in ((0, None, None), (1, res, None), (2, rhi, rlo)):
        lo = torch.empty(M, C, dtype=torch.bfloat16, device=DEV)
        ob = torch.empty(M, C, dtype=torch.bfloat16, device=DEV)
        of = torch.empty(M, C, device=DEV)
        yb = torch.empty(M, C, dtype=torch.bfloat16, device=DEV)
        ops.bn_apply_x3(y, sc, sh, r, mode, True, M, C, out_lo=lo, out_bf16=ob, out_f32=of,
                        y_bf16=yb, residual_lo=rl)
        ref = y * sc + sh + (res if mode else 0)
        ref = ref.clamp_min(0)
        tol = 2e-6 if mode != 2 else 2e-5  # the pair residual carries 16 mantissa bits
        assert torch.allclose(of, ref, rtol=tol, atol=tol), mode
        assert ((ob.float() + lo.float() - of).abs() <= of.abs() * 2.0 ** -16).all()
        assert torch.equal(ob.float(), of.to(torch.bfloat16).float())
        assert torch.equal(yb, y.to(torch.bfloat16))
        # y as a split pair (the conv epilogue's form): the same output to the pair's 2^-17
        yh, yl = _pair(y)
        lo2, ob2 = torch.empty_like(lo), torch.empty_like(ob)
        mask = torch.empty(M * C // 8, dtype=torch.uint8, device=DEV)
        ops.bn_apply_x3(yh, sc, sh, r, mode, True, M, C, out_lo=lo2, out_bf16=ob2,
                        residual_lo=rl, y_lo=yl, relu_mask=mask)
        v2 = ob2.float() + lo2.float()
        assert torch.allclose(v2, ref, rtol=3e-5, atol=3e-5), mode
        # the ReLU bitmask: bit k of byte i = output element 8i + k > 0 (of the fp32 output)
        pos = ((ob2.float() + lo2.float()) > 0).view(-1, 8).to(torch.int32)
        want = (pos << torch.arange(8, device=DEV, dtype=torch.int32)).sum(1).to(torch.uint8)
        assert torch.equal(mask, want), mode
    with pytest.raises(L.DfuError):  # a pair residual needs its lo buffer
        ops.bn_apply_x3(y, sc, sh, rhi, 2, True, M, C, out_bf16=ob)


def test_maxpool_and_avgpool_x3():
    L, ops = _ops()
    torch.manual_seed(5)
    B, H, W, C = 2, 112, 112, 64
    x = torch.randn(B, H, W, C, device=DEV)
    ylo, yb, am, P, Q = ops.maxpool_fwd_x3(x.reshape(-1, C), B, H, W, C)
    ref = torch.nn.functional.max_pool2d(x.permute(0, 3, 1, 2), 3, 2, 1).permute(0, 2, 3, 1)
    v = yb.float().reshape(-1, C) + ylo.float()
    assert torch.allclose(v.view(B, P, Q, C), ref, rtol=2e-5, atol=0)
    assert torch.equal(yb.float(), ref.to(torch.bfloat16).float())
    # avgpool over a split pair
    t = torch.randn(B * 49, 2048, device=DEV)
    a = ops.avgpool_fwd_x3(*_pair(t), B, 49, 2048)
    assert torch.allclose(a, t.view(B, 49, 2048).mean(1), rtol=1e-5, atol=1e-6)


def test_layernorm_and_gelu_x3():
    L, ops = _ops()
    torch.manual_seed(6)
    rows, D = 1000, 768
    x = torch.randn(rows, D, device=DEV) * 2 + 0.5
    g = torch.randn(D, device=DEV)
    b = torch.randn(D, device=DEV)
    o3 = torch.empty(rows, 3 * D, dtype=torch.bfloat16, device=DEV)
    ob = torch.empty(rows, D, dtype=torch.bfloat16, device=DEV)
    mean = torch.empty(rows, device=DEV)
    rstd = torch.empty(rows, device=DEV)
    ops.layernorm_fwd_x3(x, D, rows, D, g, b, 1e-6, o3, ob, mean, rstd)
    ref = torch.nn.functional.layer_norm(x.double(), (D,), g.double(), b.double(), 1e-6)
    v, _, _ = _trip(o3, D)
    assert ((v.double() - ref).abs().max() / ref.abs().max()).item() < 2e-5
    h = torch.randn(rows, 3072, device=DEV) * 3
    h3, hb, hp = ops.gelu_x3(h)
    refg = torch.nn.functional.gelu(h.double())
    v, _, _ = _trip(h3, 3072)
    assert (v.double() - refg).abs().max().item() < 1e-5 * 9
    hd = h.double()
    dref = 0.5 * torch.erfc(-hd / math.sqrt(2)) + hd * torch.exp(-0.5 * hd * hd) / math.sqrt(2 * math.pi)
    assert ((hp.double() - dref).abs() <= 2.0 ** -8 * dref.abs() + 1e-6).all()  # bf16 gelu'(h)


@pytest.mark.parametrize("N", [197, 50, 1])
def test_attention_fwd_f32_matches_sdpa(N):
    """The bf16x3 MFMA attention (csrc/attn.hip k_attn_fwd_x3) against fp64 SDPA.  Each product
    keeps 16 mantissa bits (lo*lo and the split remainders dropped: ~2^-17 relative), so the
    bar is 2^-14 of max |o| -- bf16 operands miss it by ~30x."""
    L, ops = _ops()
    torch.manual_seed(7)
    B, H, dh = 3, 12, 64
    D = H * dh
    qkv = torch.randn(B * N, 3 * D, device=DEV) * 2
    qb = torch.empty(B * N, 3 * D, dtype=torch.bfloat16, device=DEV)
    o3, ob, lse = ops.attention_fwd_f32(qkv, B, N, H, dh, dh ** -0.5, qkv_bf16=qb)
    q, k, v = qkv.double().view(B, N, 3, H, dh).permute(2, 0, 3, 1, 4)
    s = (q @ k.transpose(-1, -2)) * dh ** -0.5
    ref = (s.softmax(-1) @ v).permute(0, 2, 1, 3).reshape(B * N, D)
    o, _, _ = _trip(o3, D)
    err = (o.double() - ref).abs().max().item()
    print(f"\n[attn x3 N={N}] max abs err {err:.2e} (max |o| {ref.abs().max().item():.2f})")
    assert err < 2.0 ** -14 * ref.abs().max().item()
    assert torch.equal(ob, o3[:, :D])  # the plain bf16 o is the triple's hi segment
    assert torch.equal(o3[:, 2 * D:], o3[:, :D])  # pattern 0: [hi | lo | hi]
    assert torch.equal(qb, qkv.to(torch.bfloat16))  # the backward's bf16 qkv, written in passing
    lref = torch.logsumexp(s, -1).reshape(B * H, N)
    assert torch.allclose(lse[:, :N].double(), lref, rtol=2.0 ** -14, atol=1e-5)


@pytest.mark.parametrize("H,W", [(112, 112), (15, 9)])
def test_maxpool_bn_fused_x3_equals_apply_then_pool(H, W):
    """The stem's fused bn1 + ReLU + maxpool over the conv output pair (dfu_maxpool_bn_fwd_x3)
    is bitwise dfu_bn_apply_x3 (fp32 out, ReLU bitmask) followed by dfu_maxpool_fwd_x3: pooled
    pair, argmax and the bitmask (each element written once, odd sizes included)."""
    L, ops = _ops()
    torch.manual_seed(6)
    B, C = 2, 64
    M = B * H * W
    yf = torch.randn(M, C, device=DEV)
    hi, lo = _pair(yf)
    sc = torch.rand(C, device=DEV) + 0.5
    sh = torch.randn(C, device=DEV) * 0.5
    af = torch.empty(M, C, device=DEV)
    mask_ref = torch.empty(M * C // 8, dtype=torch.uint8, device=DEV)
    ops.bn_apply_x3(hi, sc, sh, None, 0, True, M, C, out_f32=af, y_lo=lo, relu_mask=mask_ref)
    lo_r, out_r, am_r, P, Q = ops.maxpool_fwd_x3(af, B, H, W, C)
    mask = torch.full((M * C // 8,), 0xAA, dtype=torch.uint8, device=DEV)
    lo_f, out_f, am_f, P2, Q2 = ops.maxpool_bn_fwd_x3(hi, lo, sc, sh, B, H, W, C, relu_mask=mask)
    assert (P, Q) == (P2, Q2)
    assert torch.equal(out_f, out_r) and torch.equal(lo_f, lo_r) and torch.equal(am_f, am_r)
    assert torch.equal(mask, mask_ref)


@pytest.mark.parametrize("contig", [True, False])
def test_stem_conv_x3_fused_equals_pair_im2col_gemm(contig):
    """The fused stem conv (dfu_stem_conv_x3: input rows staged in LDS, A fragments split in
    registers) against the explicit path it replaces (pair im2col + interleaved-pair GEMM with
    the F32_STATS epilogue): the conv output pair and the hi im2col rows bitwise, the BN tile
    statistics to fp32 summation order; and the pair within split-bf16 accuracy of an fp64
    convolution."""
    L, ops = _ops()
    torch.manual_seed(8)
    B, H, W = 2, 224, 224
    xs = torch.randn(B, 3, H, W + (0 if contig else 5), device=DEV)
    x = xs[..., :W] if not contig else xs
    w = torch.randn(64, 3, 7, 7, device=DEV) * 0.05
    assert ops.stem_conv_x3_ok(x, w, 2, 3)
    y, ylo, st, col, P, Q = ops.stem_conv_x3(x, w)
    M = B * P * Q
    (chi, clo), P2, Q2 = ops.im2col_f32_x3(x, 7, 7, 2, 3, 160)
    w3 = ops.split_x3(w.reshape(64, -1), ops.X3_PAIRS, seg=160)
    y2 = torch.empty(M, 64, dtype=torch.bfloat16, device=DEV)
    y2lo = torch.empty_like(y2)
    st2 = torch.empty(M // 128, 2, 64, device=DEV)
    ops.gemm(M, 64, 320, chi, 160, w3, 320, y2, 64, epilogue=L.EPI_F32_STATS, stats=st2,
             x3=True, a_lo=clo, x3_pairs=True, aux_out=y2lo, ldaux_out=64)
    assert (P, Q) == (P2, Q2) == (112, 112)
    assert torch.equal(col, chi)
    assert torch.equal(y, y2) and torch.equal(ylo, y2lo)
    torch.testing.assert_close(st[:, 0], st2[:, 0], rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(st[:, 1], st2[:, 1], rtol=1e-4, atol=1e-3)
    ref = torch.nn.functional.conv2d(x.double(), w.double(), stride=2, padding=3)
    ref = ref.permute(0, 2, 3, 1).reshape(M, 64)
    v = y.double() + ylo.double()
    err = ((v - ref).abs().max() / ref.abs().max()).item()
    print(f"\n[stem x3 fused] rel err vs fp64 conv {err:.2e}")
    assert err < 2e-5


@pytest.mark.parametrize("contig", [True, False])
def test_stem_wgrad_x3_from_x_equals_im2col_gemm(contig):
    """The stem weight gradient straight from x (dfu_stem_wgrad_x3: no im2col rows) against the
    explicit MN x MN F32_ACC GEMM over the hi im2col rows it replaces: equal to fp32 summation
    order, accumulated onto what dw held, and within bf16-operand accuracy of an fp64 sum."""
    L, ops = _ops()
    torch.manual_seed(11)
    B, H, W = 2, 224, 224
    xs = torch.randn(B, 3, H, W + (0 if contig else 5), device=DEV)
    x = xs[..., :W] if not contig else xs
    M = B * 112 * 112
    dy = (torch.randn(M, 64, device=DEV) * 0.1).to(torch.bfloat16)
    col, P, Q = ops.im2col_f32(x, 7, 7, 2, 3, 160)
    d0 = torch.randn(64, 147, device=DEV)
    ref = d0.clone()
    ops.gemm(64, 147, M, dy, 64, col, 160, ref, 147, a_mode=L.OPND_MNMAJOR,
             b_mode=L.OPND_MNMAJOR, epilogue=L.EPI_F32_ACC)
    dw = d0.clone()
    ops.stem_wgrad_x3(x, dy, dw)
    torch.testing.assert_close(dw, ref, rtol=1e-4, atol=1e-3)
    exact = d0.double() + dy.double().t() @ col[:, :147].double()
    err = ((dw.double() - exact).abs().max() / (exact - d0.double()).abs().max()).item()
    print(f"\n[stem wgrad from x] rel err vs fp64 sum {err:.2e}")
    assert err < 1e-5
    dw2 = d0.clone()
    ops.stem_wgrad_x3(x, dy, dw2)
    assert torch.equal(dw, dw2)  # deterministic
