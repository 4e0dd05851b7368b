"""FusedAdamW on the GPU: the flat update matches torch.optim.AdamW, and the bf16 weight shadow
the same kernel writes stays equal to bf16(param) — after optimizer steps and after the
parameters change outside the optimizer (load_state_dict bumps the version counter)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _model():
    from dfu_hip import nn as hnn
    torch.manual_seed(3)
    return torch.nn.Sequential(hnn.Linear(768, 512), hnn.ReLU(), hnn.Linear(512, 64)).to(DEV)


def test_adamw_matches_torch_and_shadow_tracks():
    from dfu_hip import functional as Fn
    from dfu_hip.optim import FusedAdamW
    m = _model()
    ref = [p.detach().clone() for p in m.parameters()]
    opt = FusedAdamW(m.parameters(), lr=1e-3, weight_decay=1e-2)
    ref_p = [torch.nn.Parameter(r) for r in ref]
    ref_opt = torch.optim.AdamW(ref_p, lr=1e-3, weight_decay=1e-2)
    g = torch.Generator(device="cpu").manual_seed(5)
    for _ in range(4):
        grads = [torch.randn(p.shape, generator=g).to(DEV) for p in ref_p]
        opt.zero_grad()
        for p, gr in zip(m.parameters(), grads):
            p.grad.copy_(gr)
        for p, gr in zip(ref_p, grads):
            p.grad = gr.clone()
        opt.step()
        ref_opt.step()
    for p, r in zip(m.parameters(), ref_p):
        torch.testing.assert_close(p.detach(), r.detach(), rtol=1e-5, atol=1e-6)
    # the shadow the forward GEMMs read is exactly bf16 of the updated fp32 weights
    for p in m.parameters():
        if p.dim() == 2:
            sh = Fn.weight_bf16_rows(p)
            assert sh.data_ptr() == p._dfu_shadow.data_ptr()
            assert torch.equal(sh, p.detach().to(torch.bfloat16))
    # a change outside the optimizer is picked up on the next use
    sd = {k: torch.randn_like(v) for k, v in m.state_dict().items()}
    m.load_state_dict(sd)
    # 6000 rows: the first Linear takes the bf16 GEMM path (reads the shadow); a stale shadow
    # would hold the old random weights and miss this reference completely
    x = torch.randn(6000, 768, device=DEV)
    with torch.no_grad():
        y = m(x)
    h = torch.relu(x.to(torch.bfloat16).float() @ sd["0.weight"].to(torch.bfloat16).float().t()
                   + sd["0.bias"])
    ref_y = h @ sd["2.weight"].t() + sd["2.bias"]
    err = (y.float() - ref_y).norm() / ref_y.norm()
    assert err < 2e-2, err.item()
    assert torch.equal(m[0].weight._dfu_shadow, sd["0.weight"].to(torch.bfloat16))


def test_early_adamw_on_side_stream_is_bitwise_equal():
    """In the two-stream fusion step the ViT branch's parameters get their AdamW update on the
    ViT side stream as soon as its backward is done (FusedAdamW.step early block), the rest
    after the join: parameters, moments, bf16 shadows and the ViT transposed
    shadows after three steps equal the single-launch update bit for bit."""
    import bench
    from dfu_hip import nn as hnn
    from dfu_hip.optim import FusedAdamW
    dev = torch.device("cuda", 0)
    res = []
    from models.fusion import MultimodalFusionModel
    for early in (False, True):
        torch.manual_seed(0)
        model = MultimodalFusionModel(num_classes=2, dropout=0.0).to(dev).train()
        fwd = lambda m, r, t: m(r, t)  # noqa: E731
        opt = FusedAdamW(model.parameters(), lr=1e-3, weight_decay=1e-4)
        opt.early_update = early
        crit = hnn.CrossEntropyLoss(weight=torch.tensor([2.0, 2.0], device=dev))
        rgb, th, y = bench.synthetic(4, dev, seed=3)
        for _ in range(3):
            opt.zero_grad()
            crit(fwd(model, rgb, th), y).backward()
            opt.step()
        torch.cuda.synchronize()
        if early:
            lo, hi = opt.last_early
            vit = [i for i, p in enumerate(opt.flat.params)
                   if any(p is q for q in model.vit.parameters())]
            assert opt.flat.offsets[vit[0]] == lo and hi - lo >= 85_000_000
            assert int(opt.step_dev) == 3
        else:
            assert opt.last_early is None
        tq = model.vit.blocks[0].mlp.fc1.weight
        res.append([opt.flat.data.clone(), opt.exp_avg.clone(), opt.exp_avg_sq.clone(),
                    opt.flat.shadow.clone(), getattr(tq, "_dfu_shadow_T").clone(),
                    opt.step_dev.clone()])
    for a, b in zip(*res):
        assert torch.equal(a, b)


def test_x3_pair_shadow_tracks_conv_weights():
    """The interleaved-pair bf16x3 shadow the AdamW kernel writes (FlatParams.enable_x3) equals
    the per-layer split (dfu_split_x3 / dfu_pack_conv_weight_x3 pattern 2) of the updated conv
    weights bitwise, for 1x1 and channels-last 3x3 weights, after steps and after an edit
    outside the optimizer; the stem-like 3-channel weight is left out."""
    from dfu_hip import functional as Fn
    from dfu_hip import ops
    from dfu_hip.optim import FusedAdamW
    torch.manual_seed(7)
    shapes = [(64, 3, 7, 7), (64,), (256, 64, 1, 1), (64, 64, 3, 3), (64,), (128, 256, 1, 1),
              (128, 128, 3, 3), (7,)]
    ps = [torch.nn.Parameter(torch.randn(s, device=DEV) * 0.05) for s in shapes]
    opt = FusedAdamW(ps, lr=1e-3, weight_decay=1e-2)

    def want(w):
        if w.shape[2] * w.shape[3] == 1:
            return ops.split_x3(w.detach().reshape(w.shape[0], -1), ops.X3_PAIRS)
        return ops.pack_conv_weight_x3(w.detach().contiguous(), ops.X3_PAIRS).view(w.shape[0], -1)
    convs = [p for p in ps if p.dim() == 4 and p.shape[1] % 32 == 0]
    for w in convs:  # first use enables the shadow (one split)
        assert torch.equal(Fn.conv_weight_x3(w), want(w))
    assert opt.flat.shadow_x3 is not None and ps[0].__dict__.get("_dfu_shadow_x3") is None
    g = torch.Generator(device="cpu").manual_seed(1)
    for _ in range(3):
        opt.zero_grad()
        for p in ps:
            p.grad.copy_(torch.randn(p.shape, generator=g).to(DEV))
        opt.step()
        for w in convs:
            assert torch.equal(Fn.conv_weight_x3(w), want(w))
    with torch.no_grad():  # an edit outside the optimizer bumps the version: re-split
        convs[1].mul_(0.5)
    assert torch.equal(Fn.conv_weight_x3(convs[1]), want(convs[1]))


def test_x3_span_holds_only_conv_weights_in_the_fusion_model():
    """the x3 shadow covers the flat span from the first to the last x3 conv
    weight.  In the fusion model that span holds the ResNet's BN vectors only (a few 10^4
    elements beside 23.5M); a model that registers a large parameter between its convs is
    reported."""
    import warnings
    from dfu_hip.optim import FusedAdamW
    from models.fusion import MultimodalFusionModel
    model = MultimodalFusionModel(num_classes=2, dropout=0.0).to(DEV)
    opt = FusedAdamW(model.parameters(), lr=1e-4, weight_decay=1e-4)
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        opt.flat.enable_x3()
    span = opt.flat.x3_hi - opt.flat.x3_lo
    print(f"\n[x3 span] {span} elements, {opt.flat.x3_extra} of them not x3 conv weights")
    assert 23_000_000 < span < 24_000_000 and opt.flat.x3_extra < 100_000
    ps = [torch.nn.Parameter(torch.randn(s, device=DEV)) for s in
          [(64, 64, 1, 1), (4096, 1024), (64, 64, 1, 1)]]
    opt2 = FusedAdamW(ps, lr=1e-4)
    with pytest.warns(UserWarning, match="x3 shadow"):
        opt2.flat.enable_x3()
