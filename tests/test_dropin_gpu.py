"""The reference scripts' own construct lines on the HIP encoders:
plain torch.nn heads and torch.optim.AdamW around models.encoders, exactly as written in

  * train_rgb_only.py:200-217      resnet50(); model.fc = nn.Sequential(nn.Dropout(0.5),
                                   nn.Linear(model.fc.in_features, 2))
  * train_thermal_only.py:188-205  vit_base_patch16_224(num_classes=2); model.head =
                                   nn.Sequential(nn.Dropout(0.5), nn.Linear(768, 2))
  * train_multimodal_fusion.py:285-326, 341-347  hub_load resnet50 with fc = Identity, timm ViT
                                   with num_classes=0, torch.cat, nn.Sequential(Linear(2816, 512),
                                   ReLU, Dropout, Linear(512, 256), ReLU, Dropout, Linear(256, 2)),
                                   nn.CrossEntropyLoss(weight), AdamW(lr 1e-4, wd 1e-4)

Each trains one step against the CPU oracle built the same way, with NO precision call (the
library default, "parity": logits within 1e-3; parameters after the AdamW step within one Adam
step), then two more steps stay finite; the fusion construct also at C3's B = 64 within the
5e-4 margin (what a drop-in caller gets).  Also:
gradients edited in place between backward and step (clip_grad_norm_) reach the optimizer --
the end-of-backward stream join and FusedAdamW's early-update guard."""
import copy

import pytest
import torch
import torch.nn as nn

from oracle import torch_ref as R

pytestmark = pytest.mark.gpu
DEV = "cuda"
BAR = 1e-3


def _maxd(a, b):
    return (a.detach().float().cpu() - b.detach().float().cpu()).abs().max().item()


def _train_step(model, opt, crit, inputs, y):
    opt.zero_grad()
    out = model(*inputs)
    loss = crit(out, y)
    loss.backward()
    opt.step()
    return out.detach(), loss.detach()


def _compare(name, hip, ref, make_inputs, B=8, steps_after=2, bar=BAR):
    from dfu_hip import functional as Fn
    assert Fn.get_precision() == "parity" == Fn.DEFAULT_PRECISION
    torch.manual_seed(3)
    rgb, th, y = R.synthetic_batch(B, seed=5)
    w = R.class_weights(y)
    hip.load_state_dict(ref.state_dict(), strict=True)
    hip = hip.to(DEV).train()
    m = copy.deepcopy(ref).train()
    opt_r = torch.optim.AdamW(m.parameters(), lr=1e-4, weight_decay=1e-4)
    out_r, loss_r = _train_step(m, opt_r, nn.CrossEntropyLoss(weight=w), make_inputs(rgb, th), y)
    opt_h = torch.optim.AdamW(hip.parameters(), lr=1e-4, weight_decay=1e-4)
    crit_h = nn.CrossEntropyLoss(weight=w.to(DEV))
    out_h, loss_h = _train_step(hip, opt_h, crit_h, make_inputs(rgb.to(DEV), th.to(DEV)), y.to(DEV))
    torch.cuda.synchronize()
    d = _maxd(out_h, out_r)
    p_r = dict(m.named_parameters())
    p_0 = dict(ref.named_parameters())
    worst, agree, total = 0.0, 0, 0
    for n, p in hip.named_parameters():
        a, b, z = p.detach().cpu(), p_r[n].detach(), p_0[n].detach()
        worst = max(worst, (a - b).abs().max().item())
        same = torch.sign(a - z) == torch.sign(b - z)
        agree += int(same.sum())
        total += same.numel()
    print(f"\n[{name} B={B}] default-mode logits vs fp32 oracle {d:.3e} (bar {bar}), loss "
          f"{abs(loss_h.item() - loss_r.item()):.2e}; after torch AdamW: max |p - p_oracle| "
          f"{worst:.2e}, update signs agree {agree / total:.4%}")
    assert d <= bar and abs(loss_h.item() - loss_r.item()) <= bar
    assert worst <= 2.05e-4 and agree / total > 0.97
    assert all(p.grad is not None for p in hip.parameters())
    for _ in range(steps_after):
        _, loss = _train_step(hip, opt_h, crit_h, make_inputs(rgb.to(DEV), th.to(DEV)), y.to(DEV))
        assert torch.isfinite(loss).item()
    torch.cuda.synchronize()
    assert all(torch.isfinite(p).all() for p in hip.parameters())


def test_rgb_only_construct_lines_torch_head_and_adamw():
    from models import encoders
    ref = R.ResNet()
    ref.fc = nn.Sequential(nn.Dropout(0.0), nn.Linear(ref.fc.in_features, 2))
    hip = encoders.resnet50(pretrained=False)
    hip.fc = nn.Sequential(nn.Dropout(0.0), nn.Linear(hip.fc.in_features, 2))
    _compare("train_rgb_only.py construct", hip, ref, lambda r, t: (r,))


def test_thermal_only_construct_lines_torch_head_and_adamw():
    from models import encoders
    ref = R.VisionTransformer(num_classes=2)
    ref.head = nn.Sequential(nn.Dropout(0.0), nn.Linear(768, 2))
    hip = encoders.create_model("vit_base_patch16_224", pretrained=False, num_classes=2)
    hip.head = nn.Sequential(nn.Dropout(0.0), nn.Linear(768, 2))
    _compare("train_thermal_only.py construct", hip, ref, lambda r, t: (t,))


class _ScriptFusion(nn.Module):
    """train_multimodal_fusion.py:285-326 verbatim in structure, on a given encoder pair."""

    def __init__(self, rgb_branch, thermal_branch, dropout=0.0, num_classes=2):
        super().__init__()
        self.rgb_branch = rgb_branch
        rgb_feat_dim = self.rgb_branch.fc.in_features
        self.rgb_branch.fc = nn.Identity()
        self.thermal_branch = thermal_branch
        self.fusion = nn.Sequential(nn.Linear(rgb_feat_dim + 768, 512), nn.ReLU(),
                                    nn.Dropout(dropout), nn.Linear(512, 256), nn.ReLU(),
                                    nn.Dropout(dropout), nn.Linear(256, num_classes))

    def forward(self, rgb, thermal):
        return self.fusion(torch.cat([self.rgb_branch(rgb), self.thermal_branch(thermal)], dim=1))


def test_fusion_script_construct_lines_torch_head_and_adamw():
    from models import encoders
    torch.manual_seed(0)
    ref = _ScriptFusion(R.ResNet(), R.VisionTransformer(num_classes=0))
    hip = _ScriptFusion(encoders.hub_load("pytorch/vision:v0.13.1", "resnet50", pretrained=False),
                        encoders.create_model("vit_base_patch16_224", pretrained=False,
                                              num_classes=0))
    _compare("train_multimodal_fusion.py construct", hip, ref, lambda r, t: (r, t))


def test_c3_fusion_construct_default_precision_b64():
    """INTEGRATION.md §1's switch of train_multimodal_fusion.py (hub_load + create_model, the
    script's own torch.nn 3-layer head, nn.CrossEntropyLoss, torch.optim.AdamW), no precision
    call anywhere, at C3's batch of 64: logits within the 5e-4 margin of the fp32 oracle."""
    from models import encoders
    torch.manual_seed(0)
    ref = _ScriptFusion(R.ResNet(), R.VisionTransformer(num_classes=0))
    hip = _ScriptFusion(encoders.hub_load("pytorch/vision:v0.13.1", "resnet50", pretrained=False),
                        encoders.create_model("vit_base_patch16_224", pretrained=False,
                                              num_classes=0))
    _compare("train_multimodal_fusion.py construct", hip, ref, lambda r, t: (r, t), B=64,
             steps_after=1, bar=5e-4)


class _EncoderHead(nn.Module):
    """A caller's own head on an encoder with no classifier: models/models.py:15-22's
    ThermalViTEncoder + a Linear, or notebooks/test_time_augmentation.py:99-104's
    ThermalOnlyModel (timm ViT with num_classes=0, then nn.Linear(768, 1))."""

    def __init__(self, vit, out):
        super().__init__()
        self.vit = vit
        self.classifier = nn.Linear(768, out)

    def forward(self, x):
        return self.classifier(self.vit(x))


class _RefViTEncoder(nn.Module):
    def __init__(self):
        super().__init__()
        self.vit = R.VisionTransformer(num_classes=0)

    def forward(self, x):
        return self.vit(x)


def test_thermal_vit_encoder_with_caller_head_b64():
    """ThermalViTEncoder() (head = Identity) followed by a caller's
    nn.Linear(768, 2) is NOT a diluted fusion feature extractor: the default parity mode must
    hold the 5e-4 margin at B = 64 (fp16 Blocks here gave 1.6e-3 before the policy inversion)."""
    from models import models as M
    torch.manual_seed(0)
    ref = _EncoderHead(_RefViTEncoder(), 2)
    hip = _EncoderHead(M.ThermalViTEncoder(pretrained=False), 2)
    assert not hip.vit.vit.dfu_feature_extractor
    _compare("ThermalViTEncoder + Linear(768, 2)", hip, ref, lambda r, t: (t,), B=64,
             steps_after=1, bar=5e-4)
    assert [b.dfu_parity_precision for b in hip.vit.vit.blocks] == ["bf16x3"] * 9 + ["fp16"] * 3


def test_tta_create_model_num_classes0_linear1_b64():
    """notebooks/test_time_augmentation.py:99-104: create_model(num_classes=0) then
    nn.Linear(768, 1), run in eval mode as the TTA script does; logits within the 5e-4 margin
    of the fp32 oracle at B = 64, no precision call."""
    from dfu_hip import functional as Fn
    from models import encoders
    assert Fn.get_precision() == "parity"
    torch.manual_seed(1)
    ref = _EncoderHead(R.VisionTransformer(num_classes=0), 1).eval()
    hip = _EncoderHead(encoders.create_model("vit_base_patch16_224", pretrained=False,
                                             num_classes=0), 1)
    hip.load_state_dict(ref.state_dict(), strict=True)
    hip = hip.to(DEV).eval()
    _, th, _ = R.synthetic_batch(64, seed=6)
    with torch.no_grad():
        out_r = ref(th)
        out_h = hip(th.to(DEV))
    torch.cuda.synchronize()
    d = _maxd(out_h, out_r)
    print(f"\n[TTA ViT num_classes=0 + Linear(768, 1), B=64] default-mode logits vs fp32 oracle "
          f"{d:.3e} (bar 5e-4)")
    assert d <= 5e-4


def test_feature_extractor_mark_and_user_override():
    """The fusion model marks its ViT (every Block fp16); the mark is an explicit opt-in for
    script-built fusions (models.precision.mark_feature_extractor); a per-Block override set
    by the user survives the policy."""
    from models import encoders
    from models import precision as P
    from models.fusion import MultimodalFusionModel
    m = MultimodalFusionModel(num_classes=2, dropout=0.0).to(DEV).train()
    assert m.vit.dfu_feature_extractor
    rgb, th, _ = R.synthetic_batch(2, seed=2)
    m(rgb.to(DEV), th.to(DEV))
    assert [b.dfu_parity_precision for b in m.vit.blocks] == ["fp16"] * 12
    v = encoders.create_model("vit_base_patch16_224", num_classes=0).to(DEV)
    v.blocks[10].dfu_parity_precision = "bf16x3"
    P.mark_feature_extractor(v)
    v(th.to(DEV))
    got = [b.dfu_parity_precision for b in v.blocks]
    assert got == ["fp16"] * 10 + ["bf16x3", "fp16"]
    P.mark_feature_extractor(v, on=False)
    v(th.to(DEV))
    assert [b.dfu_parity_precision for b in v.blocks] == ["bf16x3"] * 9 + ["fp16", "bf16x3",
                                                                          "fp16"]
    torch.cuda.synchronize()


def _fusion_step(clip, early):
    from dfu_hip import nn as hnn
    from dfu_hip.optim import FusedAdamW
    from models.fusion import MultimodalFusionModel
    torch.manual_seed(0)
    model = MultimodalFusionModel(num_classes=2, dropout=0.0).to(DEV).train()
    opt = FusedAdamW(model.parameters(), lr=1e-4, weight_decay=1e-4)
    opt.early_update = early
    rgb, th, y = R.synthetic_batch(8, seed=9)
    crit = hnn.CrossEntropyLoss(weight=R.class_weights(y).to(DEV))
    opt.zero_grad()
    loss = crit(model(rgb.to(DEV), th.to(DEV)), y.to(DEV))
    loss.backward()  # no explicit join: the backward's final callback joined the streams
    if clip:
        torch.nn.utils.clip_grad_norm_(model.parameters(), 1e-3)
    opt.step()
    torch.cuda.synchronize()
    return opt.flat.data.clone(), opt.last_early


def test_clip_grad_norm_before_fused_adamw_step():
    """the early AdamW update of the ViT block on its side stream must
    not read gradients that user code changed after backward.  Clipped: the early path is off
    and the result is bitwise the one-launch update; unclipped: the early path still runs and
    is bitwise equal to the one-launch update."""
    base, e0 = _fusion_step(clip=False, early=False)
    fast, e1 = _fusion_step(clip=False, early=True)
    assert e0 is None and e1 is not None, "the early update should run on untouched gradients"
    assert torch.equal(base, fast)
    clip_ref, _ = _fusion_step(clip=True, early=False)
    clip_got, e2 = _fusion_step(clip=True, early=True)
    assert e2 is None, "gradients edited in place: the early update must be skipped"
    assert torch.equal(clip_ref, clip_got)
    assert not torch.equal(clip_ref, base)  # the clip changed the update


def test_backward_joins_gradient_streams_for_user_code():
    """After loss.backward() every p.grad is complete on the calling stream, with no explicit
    join: a copy taken right after backward equals the gradients after a full synchronize."""
    from dfu_hip import functional as Fn
    from dfu_hip import nn as hnn
    from models.fusion import MultimodalFusionModel
    torch.manual_seed(0)
    model = MultimodalFusionModel(num_classes=2, dropout=0.0).to(DEV).train()
    rgb, th, y = R.synthetic_batch(8, seed=10)
    crit = hnn.CrossEntropyLoss(weight=R.class_weights(y).to(DEV))
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        loss = crit(model(rgb.to(DEV), th.to(DEV)), y.to(DEV))
        loss.backward()
        snap = [p.grad.clone() for p in model.parameters()]  # on s, immediately
    torch.cuda.synchronize()
    assert not Fn._join_armed[0]
    for p, g in zip(model.parameters(), snap):
        assert torch.equal(p.grad, g)
