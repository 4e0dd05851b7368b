"""ORACLE — test infrastructure only (imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py; never by the product path in dfu-multimodal_amd/).

A plain-PyTorch fp32 CPU restatement of the reference's hot path
(notebooks/train_multimodal_fusion.py:285-326, 341-347, 368-388):

  * RGB branch  — torchvision ``resnet50`` as loaded by
    ``torch.hub.load('pytorch/vision:v0.13.1', 'resnet50', ...)`` (:294-296).  torchvision is a
    third-party dependency absent from /root/reference and from this image; its published
    algorithm (torchvision/models/resnet.py @ v0.13.1: ResNet v1.5 Bottleneck with the stride on
    the 3x3, BatchNorm2d eps 1e-5 momentum 0.1, ReLU, maxpool 3/2/1, AdaptiveAvgPool(1),
    kaiming_normal(fan_out) conv init) is restated here with identical state_dict keys.
  * thermal branch — timm ``vit_base_patch16_224`` (timm>=0.9.2, requirements.txt:19;
    created at :299-302).  timm is absent too; restated from timm/models/vision_transformer.py
    0.9.x: PatchEmbed conv16/s16, class token + learned pos_embed, 12 pre-norm Blocks
    (LayerNorm eps 1e-6, qkv bias, 12 heads, F.scaled_dot_product_attention, Linear proj,
    Mlp 768->3072->768 with exact GELU), final norm, ``global_pool='token'``.
  * fusion head — MLPFusion, grad_cam_visualization.py:289-302 / extended_metrics.py:338-350
    (2816->512->ReLU->Dropout->2); pinned against the reference's own class source by the
    fixtures in tests/golden/ (oracle/gen_golden.py).
  * loss / optimizer — nn.CrossEntropyLoss(weight=total/count_c) (:341-346) and
    torch.optim.AdamW(lr=1e-4, weight_decay=1e-4) (:347).

Parity status: the fusion head and loss are pinned against the reference's own code (golden
fixtures); the encoders are pinned only against the published torchvision/timm algorithms
(no reference fixtures, checkpoints or tests exist for them: "parity unpinned" at that
boundary).
"""
import math

import torch
import torch.nn as nn
import torch.nn.functional as F

# ------------------------------------------------------------------ bf16 emulation
# When enabled, every tensor is rounded to bf16 at exactly the points where the MI355X path
# stores bf16 (GEMM operands and outputs, BN/LN outputs, attention probabilities, GELU input
# and output), while accumulation stays fp32.  This is the "bf16-rounded oracle" of SURVEY.md
# §7 (hard parts: report both the fp32-oracle and the bf16-rounded-oracle deltas).
_EMU = False
_EXACT_SITES = set()  # rounding sites left in fp32 (precision studies, tools/precision_study.py)
_EMU_DTYPE = [torch.bfloat16]  # the storage type emulated (fp16: tools/fp16_study.py)


def set_bf16_emulation(on, exact_sites=(), dtype=torch.bfloat16):
    global _EMU, _EXACT_SITES
    _EMU = bool(on)
    _EXACT_SITES = set(exact_sites)
    _EMU_DTYPE[0] = dtype


def rb(x, site=None):
    return x.to(_EMU_DTYPE[0]).float() if _EMU and site not in _EXACT_SITES else x


def conv(x, w, stride=1, padding=0):
    return F.conv2d(rb(x), rb(w), stride=stride, padding=padding)


def linear(x, lin, site=None):
    return F.linear(rb(x, site), rb(lin.weight, site and site + "_w"), lin.bias)


# ------------------------------------------------------------------ torchvision ResNet50
class Bottleneck(nn.Module):
    """torchvision.models.resnet.Bottleneck (v1.5)."""

    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride=stride, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = nn.Conv2d(planes, planes * 4, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        identity = x
        out = rb(self.relu(self.bn1(rb(conv(x, self.conv1.weight)))))
        out = rb(self.relu(self.bn2(rb(conv(out, self.conv2.weight, self.conv2.stride,
                                            self.conv2.padding)))))
        out = self.bn3(rb(conv(out, self.conv3.weight)))
        if self.downsample is not None:
            d = self.downsample
            identity = rb(d[1](rb(conv(x, d[0].weight, d[0].stride))))
        return rb(self.relu(out + identity))


class ResNet(nn.Module):
    """torchvision.models.resnet.ResNet(Bottleneck, [3, 4, 6, 3])."""

    def __init__(self, layers=(3, 4, 6, 3), num_classes=1000, zero_init_residual=False):
        super().__init__()
        self.inplanes = 64
        self.conv1 = nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, 2, 1)
        self.layer1 = self._make_layer(64, layers[0])
        self.layer2 = self._make_layer(128, layers[1], 2)
        self.layer3 = self._make_layer(256, layers[2], 2)
        self.layer4 = self._make_layer(512, layers[3], 2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(2048, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)
        if zero_init_residual:  # torchvision resnet.py option
            for m in self.modules():
                if isinstance(m, Bottleneck):
                    nn.init.constant_(m.bn3.weight, 0)

    def _make_layer(self, planes, blocks, stride=1):
        downsample = None
        if stride != 1 or self.inplanes != planes * 4:
            downsample = nn.Sequential(nn.Conv2d(self.inplanes, planes * 4, 1, stride=stride,
                                                 bias=False), nn.BatchNorm2d(planes * 4))
        layers = [Bottleneck(self.inplanes, planes, stride, downsample)]
        self.inplanes = planes * 4
        layers += [Bottleneck(self.inplanes, planes) for _ in range(1, blocks)]
        return nn.Sequential(*layers)

    def forward(self, x):
        x = self.maxpool(rb(self.relu(self.bn1(rb(conv(x, self.conv1.weight, 2, 3))))))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        x = torch.flatten(self.avgpool(x), 1)
        return self.fc(x)


# ------------------------------------------------------------------ timm ViT-B/16
class PatchEmbed(nn.Module):
    def __init__(self, patch=16, in_chans=3, dim=768):
        super().__init__()
        self.proj = nn.Conv2d(in_chans, dim, patch, stride=patch)
        self.norm = nn.Identity()

    def forward(self, x):
        y = F.conv2d(rb(x, "patch"), rb(self.proj.weight, "patch_w"), self.proj.bias,
                     stride=self.proj.stride)
        return self.norm(y.flatten(2).transpose(1, 2))


class _EmuAttention(torch.autograd.Function):
    """bf16-emulated SDPA with the MI355X kernels' rounding points (dfu-multimodal_amd/csrc/
    attn.hip): fp32 scores; forward P V with the unnormalised P rounded to bf16, output
    normalised then rounded; backward P recomputed from the log-sum-exp, delta = rowsum(dO * O)
    from the stored bf16 O, dV = bf16(P)^T dO, dS = P (dP - delta) rounded to bf16 before
    dQ = dS K * scale and dK = dS^T Q * scale."""

    @staticmethod
    def forward(ctx, q, k, v, scale):
        s = q @ k.transpose(-1, -2)
        mx = s.amax(-1, keepdim=True)
        p = torch.exp((s - mx) * scale)
        l = p.sum(-1, keepdim=True)
        o = rb((rb(p, "p") @ v) / l, "attn_out")
        lse = mx * scale + torch.log(l)
        ctx.save_for_backward(q, k, v, o, lse)
        ctx.scale = scale
        ctx.exact = None if _EMU else "all"  # rounding state captured at forward time
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        scale = ctx.scale

        def r(x, site):
            exact = ctx.exact == "all" or site in _EXACT_SITES
            return x if exact else x.to(_EMU_DTYPE[0]).float()
        p = torch.exp(q @ k.transpose(-1, -2) * scale - lse)
        delta = (do * o).sum(-1, keepdim=True)
        dv = r(p, "p").transpose(-1, -2) @ do
        ds = r(p * (do @ v.transpose(-1, -2) - delta), "ds")
        dq = (ds @ k) * scale
        dk = (ds.transpose(-1, -2) @ q) * scale
        return dq, dk, dv, None


class Attention(nn.Module):
    def __init__(self, dim, num_heads):
        super().__init__()
        self.num_heads = num_heads
        self.head_dim = dim // num_heads
        self.scale = self.head_dim ** -0.5
        self.qkv = nn.Linear(dim, dim * 3, bias=True)
        self.proj = nn.Linear(dim, dim)

    def forward(self, x):
        B, N, C = x.shape
        qkv = rb(linear(x, self.qkv, "ln1"), "qkv").reshape(B, N, 3, self.num_heads, self.head_dim)
        q, k, v = qkv.permute(2, 0, 3, 1, 4).unbind(0)
        if _EMU:
            x = _EmuAttention.apply(q, k, v, self.scale)
        else:
            x = F.scaled_dot_product_attention(q, k, v)
        return linear(x.transpose(1, 2).reshape(B, N, C), self.proj, "attn_out")


class Mlp(nn.Module):
    def __init__(self, dim, hidden):
        super().__init__()
        self.fc1 = nn.Linear(dim, hidden)
        self.act = nn.GELU()
        self.fc2 = nn.Linear(hidden, dim)

    def forward(self, x):
        return linear(rb(self.act(linear(x, self.fc1, "ln2")), "gelu"), self.fc2, "gelu")


class Block(nn.Module):
    def __init__(self, dim, num_heads):
        super().__init__()
        self.norm1 = nn.LayerNorm(dim, eps=1e-6)
        self.attn = Attention(dim, num_heads)
        self.norm2 = nn.LayerNorm(dim, eps=1e-6)
        self.mlp = Mlp(dim, dim * 4)

    def forward(self, x):
        x = x + self.attn(rb(self.norm1(x), "ln1"))
        return x + self.mlp(rb(self.norm2(x), "ln2"))


class VisionTransformer(nn.Module):
    def __init__(self, num_classes=1000, dim=768, depth=12, heads=12, patch=16, img=224):
        super().__init__()
        self.patch_embed = PatchEmbed(patch, 3, dim)
        n = (img // patch) ** 2
        self.cls_token = nn.Parameter(torch.zeros(1, 1, dim))
        self.pos_embed = nn.Parameter(torch.zeros(1, n + 1, dim))
        self.blocks = nn.Sequential(*[Block(dim, heads) for _ in range(depth)])
        self.norm = nn.LayerNorm(dim, eps=1e-6)
        self.head = nn.Linear(dim, num_classes) if num_classes > 0 else nn.Identity()
        nn.init.trunc_normal_(self.pos_embed, std=0.02, a=-2.0, b=2.0)
        nn.init.normal_(self.cls_token, std=1e-6)
        for m in self.modules():
            if isinstance(m, nn.Linear):
                nn.init.trunc_normal_(m.weight, std=0.02, a=-2.0, b=2.0)
                nn.init.zeros_(m.bias)

    def forward(self, x):
        x = self.patch_embed(x)
        x = torch.cat([self.cls_token.expand(x.shape[0], -1, -1), x], dim=1) + self.pos_embed
        x = self.norm(self.blocks(x))
        return self.head(x[:, 0])


# ------------------------------------------------------------------ fusion head / model
class MLPFusion(nn.Module):
    """grad_cam_visualization.py:289-302 (Dropout p configurable, 0.7 there);
    hidden_dims=(512, 256) gives the train-script head, train_multimodal_fusion.py:305-313."""

    def __init__(self, rgb_feat_dim=2048, thermal_feat_dim=768, hidden_dim=512, num_classes=2,
                 dropout=0.7, hidden_dims=None):
        super().__init__()
        dims = tuple(hidden_dims) if hidden_dims is not None else (hidden_dim,)
        layers, d = [], rgb_feat_dim + thermal_feat_dim
        for h in dims:
            layers += [nn.Linear(d, h), nn.ReLU(), nn.Dropout(dropout)]
            d = h
        layers.append(nn.Linear(d, num_classes))
        self.classifier = nn.Sequential(*layers)

    def forward(self, rgb_feat, thermal_feat):
        # the MI355X head runs in exact fp32 (dfu_gemm_f32): no bf16 rounding here
        return self.classifier(torch.cat([rgb_feat, thermal_feat], dim=1))


class MultimodalFusionModel(nn.Module):
    """grad_cam_visualization.py:305-320: attributes resnet / vit / fusion."""

    def __init__(self, num_classes=2, dropout=0.7, zero_init_residual=False):
        super().__init__()
        self.resnet = ResNet(zero_init_residual=zero_init_residual)
        self.resnet.fc = nn.Identity()
        self.vit = VisionTransformer(num_classes=0)
        self.fusion = MLPFusion(num_classes=num_classes, dropout=dropout)

    def forward(self, rgb, thermal):
        return self.fusion(self.resnet(rgb), self.vit(thermal))


# ------------------------------------------------------------------ synthetic batch / step
RGB_MEAN = (0.485, 0.456, 0.406)  # train_multimodal_fusion.py:181
RGB_STD = (0.229, 0.224, 0.225)


def synthetic_batch(B, seed=42, size=224):
    """uint8 images U{0..255}, normalised as the reference transforms
    (rgb ImageNet stats :181, thermal 0.5/0.5 :198); labels U{0,1}."""
    g = torch.Generator().manual_seed(seed)
    rgb_u8 = torch.randint(0, 256, (B, 3, size, size), generator=g, dtype=torch.uint8)
    th_u8 = torch.randint(0, 256, (B, 3, size, size), generator=g, dtype=torch.uint8)
    labels = torch.randint(0, 2, (B,), generator=g, dtype=torch.int64)
    mean = torch.tensor(RGB_MEAN).view(1, 3, 1, 1)
    std = torch.tensor(RGB_STD).view(1, 3, 1, 1)
    rgb = (rgb_u8.float() / 255.0 - mean) / std
    th = (th_u8.float() / 255.0 - 0.5) / 0.5
    return rgb, th, labels


def class_weights(labels, num_classes=2):
    """w_c = total / count_c (train_multimodal_fusion.py:341-345)."""
    counts = torch.bincount(labels, minlength=num_classes).float()
    total = counts.sum().clamp(min=1)
    return torch.where(counts > 0, total / counts.clamp(min=1), torch.zeros_like(counts))


def train_step(model, opt, criterion, rgb, th, labels):
    """One iteration of the reference hot loop (:374-380)."""
    opt.zero_grad()
    out = model(rgb, th)
    loss = criterion(out, labels)
    loss.backward()
    opt.step()
    return out.detach(), loss.detach()
