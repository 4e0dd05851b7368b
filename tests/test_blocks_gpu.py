"""Block-level parity on the GPU: each fused autograd Function vs the matching oracle module
(fp32 CPU) on identical bf16-representable inputs, weights and upstream gradients."""
import pytest
import torch

from oracle import torch_ref as R

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True)
def _bf16_kernels():
    """These checks hold the bf16 kernels to the bf16-rounded oracle (same rounding sites): run
    the bf16 mode explicitly (the library default is "parity")."""
    from dfu_hip import functional as Fn
    with Fn.precision("bf16"):
        yield


def rel(a, b):
    a = a.detach().float().cpu()
    b = b.detach().float().cpu()
    return ((a - b).norm() / b.norm().clamp(min=1e-12)).item()


def bfr(t):
    """round to bf16-representable fp32"""
    return t.to(torch.bfloat16).float()


def _grad_report(hip_mod, ref_mod, tol, tag):
    rp = dict(ref_mod.named_parameters())
    bad = []
    for n, p in hip_mod.named_parameters():
        if rp[n].grad is None:
            continue
        e = rel(p.grad, rp[n].grad)
        print(f"{tag} grad {n}: {e:.3e}")
        if not e < tol:
            bad.append((n, e))
    assert not bad, bad


@pytest.mark.parametrize("inpl,planes,stride,ds,H", [(64, 64, 1, True, 56), (256, 64, 1, False, 56),
                                                     (256, 128, 2, True, 56), (1024, 512, 2, True, 14)])
def test_bottleneck(inpl, planes, stride, ds, H):
    from models.resnet import Bottleneck, conv1x1
    from dfu_hip import nn as hnn
    torch.manual_seed(0)
    B = 2
    dref = None
    if ds:
        dref = torch.nn.Sequential(torch.nn.Conv2d(inpl, planes * 4, 1, stride=stride, bias=False),
                                   torch.nn.BatchNorm2d(planes * 4))
    ref = R.Bottleneck(inpl, planes, stride, dref)
    with torch.no_grad():
        for m in ref.modules():
            if isinstance(m, torch.nn.BatchNorm2d):
                m.weight.uniform_(0.5, 1.5)
                m.bias.uniform_(-0.5, 0.5)
            if isinstance(m, torch.nn.Conv2d):
                m.weight.copy_(bfr(m.weight))
    dhip = None
    if ds:
        dhip = torch.nn.Sequential(conv1x1(inpl, planes * 4, stride), hnn.BatchNorm2d(planes * 4))
    hip = Bottleneck(inpl, planes, stride, dhip)
    hip.load_state_dict(ref.state_dict())
    hip = hip.to(DEV)
    x = bfr(torch.randn(B, inpl, H, H))
    xr = x.clone().requires_grad_(True)
    R.set_bf16_emulation(True)  # compare with the bf16-rounded oracle block (same rounding)
    try:
        out_r = ref(xr)
        g = bfr(torch.randn_like(out_r))
        out_r.backward(g)
    finally:
        R.set_bf16_emulation(False)
    xh = x.to(DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    out_h = hip(xh)
    out_h.backward(g.to(DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last))
    torch.cuda.synchronize()
    eo = rel(out_h, out_r)
    ex = rel(xh.grad, xr.grad)
    print(f"\nbottleneck {inpl},{planes},s{stride}: out {eo:.3e} dx {ex:.3e}")
    rb = dict(ref.named_buffers())
    for n, b in hip.named_buffers():
        if "running" in n:
            print(f"  buf {n}: {rel(b, rb[n]):.3e}")
    assert eo < 2e-2 and ex < 3e-2
    _grad_report(hip, ref, 3e-2, "  ")


def test_stem():
    from models.resnet import ResNet
    torch.manual_seed(0)
    ref = R.ResNet()
    hip = ResNet()
    hip.load_state_dict(ref.state_dict())
    hip = hip.to(DEV)
    B = 2
    rgb, _, _ = R.synthetic_batch(B)
    with torch.no_grad():
        ref.conv1.weight.copy_(bfr(ref.conv1.weight))
    hip.conv1.weight.data.copy_(ref.conv1.weight.to(DEV))
    rgb = bfr(rgb)
    R.set_bf16_emulation(True)
    try:
        a = ref.maxpool(R.rb(ref.relu(ref.bn1(R.rb(R.conv(rgb, ref.conv1.weight, 2, 3))))))
        g = bfr(torch.randn_like(a))
        a.backward(g)
    finally:
        R.set_bf16_emulation(False)
    from dfu_hip import functional as Fn
    ah = Fn.StemFn.apply(rgb.to(DEV), hip.conv1.weight, hip.bn1.weight, hip.bn1.bias, hip)
    ah.backward(g.to(DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last))
    torch.cuda.synchronize()
    print(f"\nstem out {rel(ah, a):.3e}")
    for n in ["conv1.weight", "bn1.weight", "bn1.bias"]:
        e = rel(dict(hip.named_parameters())[n].grad, dict(ref.named_parameters())[n].grad)
        print(f"  stem grad {n}: {e:.3e}")
        assert e < 3e-2
    assert rel(ah, a) < 2e-2


def test_vit_block_and_embed():
    from models.vit import VisionTransformer
    torch.manual_seed(0)
    ref = R.VisionTransformer(num_classes=0, depth=2)
    hip = VisionTransformer(num_classes=0, depth=2)
    hip.load_state_dict(ref.state_dict())
    hip = hip.to(DEV)
    B = 2
    _, th, _ = R.synthetic_batch(B)
    th = bfr(th)
    out_r = ref(th)
    g = torch.randn_like(out_r)
    out_r.backward(g)
    out_h = hip(th.to(DEV))
    out_h.backward(g.to(DEV))
    torch.cuda.synchronize()
    print(f"\nvit out {rel(out_h, out_r):.3e}")
    assert rel(out_h, out_r) < 2e-2
    _grad_report(hip, ref, 3e-2, "  vit")


def test_vit_block_output_hooks_see_true_gradient():
    """ViTBlockFn's backward updates the incoming residual-stream gradient in place;
    a retain_grad() / tensor hook on a block output must still hold the true gradient."""
    from models.vit import vit_base_patch16_224
    torch.manual_seed(0)
    vit = vit_base_patch16_224(num_classes=0).to(DEV).train()
    x0 = torch.randn(2, 197, 768, device=DEV)
    Rg = torch.randn(2, 197, 768, device=DEV)
    hooked = []
    out = vit.blocks[0](x0.requires_grad_(True))
    out.retain_grad()
    out.register_hook(lambda g: hooked.append(g))
    (vit.blocks[1](out) * Rg).sum().backward()
    # reference: the same gradient at a leaf (nothing downstream can touch a leaf's .grad)
    leaf = out.detach().clone().requires_grad_(True)
    (vit.blocks[1](leaf) * Rg).sum().backward()
    assert torch.equal(out.grad, leaf.grad)
    assert torch.equal(hooked[0], leaf.grad)


@pytest.mark.parametrize("shape", [(2304, 768), (768, 3072), (64, 8), (200, 136)])
def test_transpose_bf16(shape):
    from dfu_hip import ops
    x = torch.randn(*shape, device=DEV).to(torch.bfloat16)
    assert torch.equal(ops.transpose_bf16(x), x.t().contiguous())
    y = torch.randn(shape[1], shape[0], device=DEV).to(torch.bfloat16)
    outs = [torch.empty(shape[1], shape[0], dtype=torch.bfloat16, device=DEV),
            torch.empty(shape[0], shape[1], dtype=torch.bfloat16, device=DEV)]
    jobs = ops.TransposeJobs([(x, outs[0]), (y, outs[1])])  # one launch, two jobs
    jobs.launch()
    assert torch.equal(outs[0], x.t()) and torch.equal(outs[1], y.t())


def test_vit_dgrad_on_transposed_shadow_is_bitwise_equal(monkeypatch):
    """The ViT input-gradient GEMMs read the weight K-contiguous from the transposed bf16 shadow
    (FusedAdamW-managed weights, functional.weight_bf16_T) or MN-major from the shadow itself:
    the same products in the same K order, so every gradient is bitwise equal; after an
    optimizer step the batched transpose keeps the copy current."""
    from dfu_hip import functional as Fn
    # fc1.bias by the colsum pass on both sides (the dGELU epilogue sums exist on one tile only,
    # and the two operand layouts may be planned on different tiles)
    monkeypatch.setattr(Fn, "_DGELU_COLSUM", False)
    from models.vit import vit_base_patch16_224
    from dfu_hip.optim import FusedAdamW
    torch.manual_seed(0)
    a = vit_base_patch16_224(num_classes=0).to(DEV).train()
    b = vit_base_patch16_224(num_classes=0).to(DEV).train()
    b.load_state_dict(a.state_dict())
    blocks_a, blocks_b = a.blocks[:2], b.blocks[:2]
    opt = FusedAdamW(blocks_a.parameters(), lr=1e-3, weight_decay=1e-4)  # a: shadows + T copies
    x0 = torch.randn(4, 197, 768, device=DEV)
    Rg = torch.randn(4, 197, 768, device=DEV)
    for step in range(2):
        for blocks in (blocks_a, blocks_b):
            for p in blocks.parameters():
                p.grad = None if blocks is blocks_b else p.grad
            xa = x0.clone().requires_grad_(True)
            (blocks[1](blocks[0](xa)) * Rg).sum().backward()
            blocks.xgrad = xa.grad
        torch.cuda.synchronize()
        assert getattr(blocks_a[0].mlp.fc1.weight, "_dfu_shadow_T", None) is not None
        assert torch.equal(blocks_a.xgrad, blocks_b.xgrad), step
        for (n, pa), pb in zip(blocks_a.named_parameters(), blocks_b.parameters()):
            assert torch.equal(pa.grad, pb.grad), (step, n)
        # same update on both sides: the T copies must follow the new weights
        opt.step()
        opt.zero_grad()
        with torch.no_grad():
            for pa, pb in zip(blocks_a.parameters(), blocks_b.parameters()):
                pb.copy_(pa)
        w = blocks_a[1].attn.qkv.weight
        assert torch.equal(w._dfu_shadow_T, w._dfu_shadow.t())


def test_resnet_stage_with_channels_last_conv_weights_is_bitwise_equal(monkeypatch):
    """FusedAdamW stores the 3x3 conv weights channels-last (KRSC, optim.FlatParams): the
    forward reads the bf16 shadow as the GEMM operand and the weight-gradient GEMM accumulates
    straight into p.grad.  Against unmanaged weights (per-call OIHW -> KRSC packing, gradient
    permute-added from a scratch buffer) every gradient and output is bitwise equal, before and
    after an optimizer step (the stride-1 dgrads on their dgrad loaders here, as unmanaged
    weights run them: test_stride1_dgrad_on_flipped_weights covers the forward-conv form)."""
    from models.resnet import resnet50
    from dfu_hip import functional as Fn
    from dfu_hip.optim import FusedAdamW
    monkeypatch.setattr(Fn, "_DGRAD_FLIP", False)
    torch.manual_seed(0)
    a = resnet50(num_classes=0).to(DEV).train()
    b = resnet50(num_classes=0).to(DEV).train()
    b.load_state_dict(a.state_dict())
    sa, sb = a.layer2, b.layer2  # stride-2 3x3 conv, downsample, stride-1 3x3 convs
    opt = FusedAdamW(sa.parameters(), lr=1e-3, weight_decay=1e-4)
    w = sa[0].conv2.weight
    assert w.is_contiguous(memory_format=torch.channels_last) and not w.is_contiguous()
    x0 = torch.randn(4, 256, 56, 56, device=DEV).contiguous(memory_format=torch.channels_last)
    for step in range(2):
        outs = []
        for s in (sa, sb):
            if s is sb:
                for p in s.parameters():
                    p.grad = None
            y = s(x0)
            Rg = torch.randn(y.shape, device=DEV,
                             generator=torch.Generator(device=DEV).manual_seed(step))
            (y.float() * Rg).sum().backward()
            outs.append(y.detach().float())
        torch.cuda.synchronize()
        assert torch.equal(outs[0], outs[1]), step
        for (n, pa), pb in zip(sa.named_parameters(), sb.parameters()):
            assert torch.equal(pa.grad, pb.grad), (step, n)
        opt.step()
        opt.zero_grad()
        with torch.no_grad():
            for pa, pb in zip(sa.parameters(), sb.parameters()):
                pb.copy_(pa)
        for bn_a, bn_b in zip(sa.modules(), sb.modules()):
            if isinstance(bn_a, torch.nn.BatchNorm2d):
                bn_b.running_mean.copy_(bn_a.running_mean)
                bn_b.running_var.copy_(bn_a.running_var)


def test_stride1_dgrad_on_flipped_weights(monkeypatch):
    """The stride-1 3x3 conv input gradients of FusedAdamW-managed weights run as forward
    convolutions of dY with the flipped channel-transposed bf16 copy W'[c][r][s][k] =
    W[k][2-r][2-s][c] (optim.FlatParams.add_flipped, refreshed in the optimizer's batched
    transpose launch): the copy equals the flip of the shadow after each step; outputs are
    unchanged and every gradient matches the dgrad-loader form to fp32 summation-order rounding
    of the bf16 input gradients (relative L2 < 1e-2) and a torch fp32 conv2d_input (< 2e-2)."""
    from models.resnet import resnet50
    from dfu_hip import functional as Fn
    from dfu_hip.optim import FusedAdamW
    torch.manual_seed(0)
    net = resnet50(num_classes=0).to(DEV).train()
    stage = net.layer3  # 5 stride-1 3x3 convs, 14x14, 256 channels
    opt = FusedAdamW(stage.parameters(), lr=1e-3, weight_decay=1e-4)
    x0 = torch.randn(4, 512, 28, 28, device=DEV).contiguous(memory_format=torch.channels_last)
    for step in range(2):
        res = []
        for flip in (False, True):
            monkeypatch.setattr(Fn, "_DGRAD_FLIP", flip)
            opt.zero_grad()
            y = stage(x0)
            Rg = torch.randn(y.shape, device=DEV,
                             generator=torch.Generator(device=DEV).manual_seed(step))
            (y.float() * Rg).sum().backward()
            res.append((y.detach().float(), [p.grad.clone() for p in stage.parameters()]))
        torch.cuda.synchronize()
        assert torch.equal(res[0][0], res[1][0]), "forward changed"
        for (n, _), g0, g1 in zip(stage.named_parameters(), res[0][1], res[1][1]):
            assert rel(g1, g0) < 1e-2, (step, n, rel(g1, g0))
        w = stage[1].conv2.weight
        f = w._dfu_shadow_F.view(256, 3, 3, 256)
        kr = w._dfu_shadow.view(256, 3, 3, 256)  # [k][r][s][c]
        assert torch.equal(f, kr.flip(1, 2).permute(3, 1, 2, 0)), step
        opt.step()
    # the forward-conv form against torch on one conv
    w = stage[1].conv2.weight
    dy = torch.randn(4, 256, 14, 14, device=DEV).to(torch.bfloat16)
    g = Fn._geom(stage[1].conv2, 4, 14, 14)
    dx = torch.empty(4 * 14 * 14, 256, dtype=torch.bfloat16, device=DEV)
    Fn.conv_dgrad(Fn.rows_view(Fn.nhwc_bf16(dy)), g, None, dx,
                  w_flip=Fn.conv_weight_flipped(w))
    wb = Fn.weight_bf16_rows(w).view(256, 3, 3, 256).permute(0, 3, 1, 2).float()
    ref = torch.nn.grad.conv2d_input((4, 256, 14, 14), wb, dy.float(), padding=1)
    assert rel(dx.view(4, 14, 14, 256).permute(0, 3, 1, 2), ref) < 2e-2


def test_1x1_dgrad_on_transposed_weights(monkeypatch):
    """Layer 1's 1x1 input gradients to 64 channels (conv3 of every block, conv1 and the
    downsample of block 0: N = 64 GEMMs) run K-contiguous on the transposed bf16 shadow
    (functional.conv1x1_weight_T, kept current by the optimizer's batched transposes): outputs
    unchanged; every gradient matches the MN-major weight form to summation-order rounding of
    the bf16 input gradients (relative L2 < 1e-2), before and after optimizer steps; the
    transposed copy equals the shadow's transpose after each step; the ADD form against torch."""
    from models.resnet import resnet50
    from dfu_hip import functional as Fn
    from dfu_hip.optim import FusedAdamW
    torch.manual_seed(0)
    net = resnet50(num_classes=0).to(DEV).train()
    stage = net.layer1
    opt = FusedAdamW(stage.parameters(), lr=1e-3, weight_decay=1e-4)
    x0 = torch.randn(4, 64, 56, 56, device=DEV).contiguous(memory_format=torch.channels_last)
    x0.requires_grad_(True)
    for step in range(2):
        res = []
        for maxc in (0, 64):
            monkeypatch.setattr(Fn, "_DGRAD_T1X1_MAXC", maxc)
            opt.zero_grad()
            x0.grad = None
            y = stage(x0)
            Rg = torch.randn(y.shape, device=DEV,
                             generator=torch.Generator(device=DEV).manual_seed(step))
            (y.float() * Rg).sum().backward()
            res.append((y.detach().float(), x0.grad.float().clone(),
                        [p.grad.clone() for p in stage.parameters()]))
        torch.cuda.synchronize()
        assert torch.equal(res[0][0], res[1][0]), "forward changed"
        assert rel(res[1][1], res[0][1]) < 1e-2, (step, rel(res[1][1], res[0][1]))
        for (n, _), g0, g1 in zip(stage.named_parameters(), res[0][2], res[1][2]):
            assert rel(g1, g0) < 1e-2, (step, n, rel(g1, g0))
        for conv in (stage[0].conv1, stage[0].conv3, stage[0].downsample[0], stage[2].conv3):
            w = conv.weight
            assert torch.equal(w._dfu_shadow_T, w._dfu_shadow.t()), (step, tuple(w.shape))
        opt.step()
    # the ADD form (downsample dgrad added in place) against torch on one conv
    monkeypatch.setattr(Fn, "_DGRAD_T1X1_MAXC", 64)
    conv = stage[0].downsample[0]
    g = Fn._geom(conv, 4, 56, 56)
    dy = torch.randn(4 * 56 * 56, 256, device=DEV).to(torch.bfloat16)
    base = torch.randn(4 * 56 * 56, 64, device=DEV).to(torch.bfloat16)
    dx = base.clone()
    Fn.conv_dgrad(dy, g, None, dx, add=dx, w_t=Fn.conv1x1_weight_T(conv, g))
    wb = Fn.weight_bf16_rows(conv.weight).float()  # [256][64]
    ref = dy.float() @ wb + base.float()
    assert rel(dx, ref) < 1e-2
