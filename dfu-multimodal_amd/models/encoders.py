"""Encoder factories replacing the reference's remote loaders:
  torch.hub.load('pytorch/vision:v0.13.1', 'resnet50', pretrained=...)  (train_multimodal_fusion.py:294)
  timm.create_model('vit_base_patch16_224', pretrained=..., num_classes=...) (:299-302)
and the library classes of models/models.py:6-22.

No network is available, so ``pretrained=True`` cannot download torchvision IMAGENET1K_V1 or
timm augreg weights; pass ``weights_path`` to a torchvision/timm state_dict saved with
torch.save (loaded with weights_only=True) instead.
"""
import warnings

import torch
import torch.nn as tnn

from .resnet import ResNet, resnet50 as _resnet50
from .vit import VisionTransformer, vit_base_patch16_224 as _vit_b16


def _load_weights(model, weights_path, strict=False):
    sd = torch.load(weights_path, map_location="cpu", weights_only=True)
    if isinstance(sd, dict) and "model_state_dict" in sd:
        sd = sd["model_state_dict"]
    missing, unexpected = model.load_state_dict(sd, strict=strict)
    return missing, unexpected


def _pretrained_note(pretrained, weights_path, what):
    if pretrained and weights_path is None:
        warnings.warn(f"{what}: pretrained weights cannot be fetched offline; using the "
                      f"reference's seeded initialisation (pass weights_path= to load a file)")


def resnet50(pretrained=False, weights=None, num_classes=1000, weights_path=None,
             zero_init_residual=False):
    model = _resnet50(num_classes=num_classes, zero_init_residual=zero_init_residual)
    _pretrained_note(pretrained or weights is not None, weights_path, "resnet50")
    if weights_path is not None:
        _load_weights(model, weights_path)
    return model


def vit_base_patch16_224(pretrained=False, num_classes=1000, weights_path=None, **kw):
    model = _vit_b16(num_classes=num_classes, **kw)
    _pretrained_note(pretrained, weights_path, "vit_base_patch16_224")
    if weights_path is not None:
        _load_weights(model, weights_path)
    return model


def create_model(name, pretrained=False, num_classes=1000, **kw):
    """timm.create_model subset: 'vit_base_patch16_224'."""
    if name != "vit_base_patch16_224":
        raise ValueError(f"create_model: only 'vit_base_patch16_224' is provided, got {name!r}")
    return vit_base_patch16_224(pretrained=pretrained, num_classes=num_classes, **kw)


def hub_load(repo, name, pretrained=False, **kw):
    """torch.hub.load('pytorch/vision:v0.13.1', 'resnet50', pretrained=...) subset."""
    if name != "resnet50":
        raise ValueError(f"hub_load: only 'resnet50' is provided, got {name!r}")
    return resnet50(pretrained=pretrained, **kw)


class RGBResNetEncoder(tnn.Module):
    """models/models.py:6-13 — ResNet50 with fc = Identity -> (B, 2048)."""

    def __init__(self, pretrained=False, weights_path=None):
        super().__init__()
        self.resnet = resnet50(pretrained=pretrained, weights_path=weights_path)
        self.resnet.fc = tnn.Identity()

    def forward(self, x):
        return self.resnet(x)


class ThermalViTEncoder(tnn.Module):
    """models/models.py:15-22 — ViT-B/16 with head = Identity -> (B, 768)."""

    def __init__(self, pretrained=False, weights_path=None):
        super().__init__()
        self.vit = vit_base_patch16_224(pretrained=pretrained, weights_path=weights_path)
        self.vit.head = tnn.Identity()

    def forward(self, x):
        return self.vit(x)


class EfficientNetEncoder(tnn.Module):
    """models/encoders.py:5-12 (early-era EfficientNet-B0). Out of scope for the MI355X path
    (SURVEY.md §2 row 6): the name is kept so imports resolve."""

    def __init__(self, *a, **k):
        super().__init__()
        raise NotImplementedError("EfficientNetEncoder is outside the fused DFU hot path")
