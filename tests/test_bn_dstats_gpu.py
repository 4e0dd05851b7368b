"""BatchNorm backward sums fused into the dgrad epilogue (DFU_EPI_BF16_DSTATS): the records
against an fp64 restatement of k_bn_bwd_reduce's relu-mode-2 sums (bn.hip), and the whole
Bottleneck backward with the fusion on vs off (the separate dfu_bn_bwd_reduce pass).
Reference ops: torchvision Bottleneck bn1/bn2 + ReLU backward (resnet.py), the autograd of
train_multimodal_fusion.py:375-379."""
import pytest
import torch

from dfu_hip import _lib as L
from dfu_hip import functional as Fn
from dfu_hip import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _coef4(C, seed):
    g = torch.Generator().manual_seed(seed)
    scale = torch.rand(C, generator=g) + 0.5
    shift = torch.rand(C, generator=g) - 0.5
    mean = torch.randn(C, generator=g) * 0.1
    invstd = torch.rand(C, generator=g) + 0.5
    return torch.stack([scale, shift, mean, invstd]).to(DEV)


def _ref_records(dx, y, coef, M, C):
    """fp64 per-128-row (sum g', sum g' xhat) with g' = bf16 dx masked by fma(y, s, b) > 0."""
    g = dx.double().cpu()
    yy = y.double().cpu()
    sc, sf, mu, iv = (coef[i].double().cpu() for i in range(4))
    pre = (y.float() * coef[0] + coef[1]).cpu()  # the kernel's fp32 fma mask
    gm = torch.where(pre > 0, g, torch.zeros_like(g))
    xh = (yy - mu) * iv
    T = (M + 127) // 128
    pad = T * 128 - M
    gm = torch.nn.functional.pad(gm, (0, 0, 0, pad)).view(T, 128, C)
    xh = torch.nn.functional.pad(xh, (0, 0, 0, pad)).view(T, 128, C)
    return torch.stack([gm.sum(1), (gm * xh).sum(1)], 1)


@pytest.mark.parametrize("case", ["1x1", "3x3"])
@pytest.mark.parametrize("tile", [0, 1, 5, 6])
def test_dstats_epilogue_records(case, tile):
    torch.manual_seed(3)
    if case == "1x1":  # conv3 dgrad of a layer2 block: dX[M, 128] = dY[M, 512] W
        M, C, K = 50176 // 4 + 37, 128, 512
        dy = (torch.randn(M, K, device=DEV) * 0.1).bfloat16()
        w = (torch.randn(K, C, device=DEV) * 0.05).bfloat16()  # [k][n] MN-major B
        y = torch.randn(M, C, device=DEV).bfloat16()
        coef = _coef4(C, 1)
        dx = torch.empty(M, C, device=DEV, dtype=torch.bfloat16)
        st = torch.empty(ops.stats_tiles(M), 2, C, device=DEV)
        ops.gemm(M, C, K, dy, K, w, C, dx, C, b_mode=L.OPND_MNMAJOR,
                 epilogue=L.EPI_BF16_DSTATS, aux=y, ldaux=C, stats=st, bn_coef=coef, tile=tile)
        ref_dx = torch.empty_like(dx)
        ops.gemm(M, C, K, dy, K, w, C, ref_dx, C, b_mode=L.OPND_MNMAJOR, epilogue=L.EPI_BF16,
                 tile=tile)
    else:  # conv2 (3x3, stride 1) dgrad of a layer1 block
        B, H, C, Ko = 4, 56, 64, 64
        g = ops.ConvGeom(B, H, H, C, Ko, 3, 3, 1, 1)
        M = B * H * H
        dy = (torch.randn(M, Ko, device=DEV) * 0.1).bfloat16()
        wf = torch.randn(Ko, C, 3, 3, device=DEV) * 0.05
        w = ops.pack_conv_weight(wf)
        y = torch.randn(M, C, device=DEV).bfloat16()
        coef = _coef4(C, 2)
        dx = torch.empty(M, C, device=DEV, dtype=torch.bfloat16)
        st = torch.empty(ops.stats_tiles(M), 2, C, device=DEV)
        ops.gemm(M, C, 9 * Ko, dy, 0, w, 9 * C, dx, C, a_mode=L.OPND_CONV_DGRAD,
                 b_mode=L.OPND_CONV_DGRAD_W, epilogue=L.EPI_BF16_DSTATS, aux=y, ldaux=C,
                 conv=g, stats=st, bn_coef=coef, tile=tile)
        ref_dx = torch.empty_like(dx)
        ops.gemm(M, C, 9 * Ko, dy, 0, w, 9 * C, ref_dx, C, a_mode=L.OPND_CONV_DGRAD,
                 b_mode=L.OPND_CONV_DGRAD_W, epilogue=L.EPI_BF16, conv=g, tile=tile)
    torch.cuda.synchronize()
    assert torch.equal(dx, ref_dx)  # the stored gradient is the plain bf16 dgrad, bitwise
    ref = _ref_records(dx, y, coef, M, C)
    got = st.double().cpu()
    scale = ref.abs().amax(dim=(0, 2), keepdim=True)
    err = ((got - ref).abs() / scale).max().item()
    print(f"\nDSTATS {case} tile {tile}: max rel record error {err:.2e}")
    assert err < 2e-5


def _bottleneck_grads(fuse, inpl, planes, stride, ds, H, B=4):
    from models.resnet import Bottleneck, conv1x1
    from dfu_hip import nn as hnn
    torch.manual_seed(0)
    dhip = None
    if ds:
        dhip = torch.nn.Sequential(conv1x1(inpl, planes * 4, stride), hnn.BatchNorm2d(planes * 4))
    m = Bottleneck(inpl, planes, stride, dhip).to(DEV)
    with torch.no_grad():
        for mod in m.modules():
            if isinstance(mod, torch.nn.BatchNorm2d):
                mod.weight.uniform_(0.5, 1.5)
                mod.bias.uniform_(-0.5, 0.5)
    x = torch.randn(B, inpl, H, H, device=DEV).bfloat16().contiguous(
        memory_format=torch.channels_last).requires_grad_(True)
    old = Fn.FUSE_BN_DSTATS, Fn.FUSE_BN_DSTATS_MIN_C
    Fn.FUSE_BN_DSTATS, Fn.FUSE_BN_DSTATS_MIN_C = fuse, 0
    try:
        out = m(x)
        g = torch.randn_like(out.float()).bfloat16().contiguous(memory_format=torch.channels_last)
        out.backward(g)
    finally:
        Fn.FUSE_BN_DSTATS, Fn.FUSE_BN_DSTATS_MIN_C = old
    torch.cuda.synchronize()
    return x.grad.float(), {n: p.grad.clone() for n, p in m.named_parameters()}


@pytest.mark.parametrize("inpl,planes,stride,ds,H", [(256, 64, 1, False, 56),
                                                     (256, 128, 2, True, 56),
                                                     (1024, 256, 1, False, 14)])
def test_bottleneck_fused_vs_separate_reduce(inpl, planes, stride, ds, H):
    dx0, g0 = _bottleneck_grads(False, inpl, planes, stride, ds, H)
    dx1, g1 = _bottleneck_grads(True, inpl, planes, stride, ds, H)
    # the two reductions sum in different orders (fp32 partials, fp64 totals): the BN
    # coefficients agree to ~1e-6 relative, so the bf16 gradients agree up to rare rounding flips
    e = ((dx1 - dx0).norm() / dx0.norm()).item()
    print(f"\nfused vs separate {inpl},{planes},s{stride}: dx {e:.2e}")
    assert e < 2e-3
    for n in g0:
        en = ((g1[n] - g0[n]).norm() / g0[n].norm().clamp(min=1e-12)).item()
        assert en < 2e-3, (n, en)
