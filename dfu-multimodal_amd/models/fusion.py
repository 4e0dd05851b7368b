"""Late-fusion heads and the multimodal model.

North-star head (grad_cam_visualization.py:289-302, extended_metrics.py:338-350):
    cat([f_rgb (2048), f_th (768)]) -> Linear(2816, 512) -> ReLU -> Dropout(p) -> Linear(512, 2)
``hidden_dims=(512, 256)`` builds the train-script variant (train_multimodal_fusion.py:305-313).
"""
import os

import torch
import torch.nn as tnn

from dfu_hip import functional as Fn
from dfu_hip import nn as hnn
from dfu_hip import ops

from .encoders import resnet50, vit_base_patch16_224


def _mlp(in_dim, hidden_dims, num_classes, dropout):
    layers = []
    d = in_dim
    for h in hidden_dims:
        layers += [hnn.Linear(d, h), hnn.ReLU(), hnn.Dropout(dropout)]
        d = h
    layers.append(hnn.Linear(d, num_classes))
    return tnn.Sequential(*layers)


class MLPFusion(tnn.Module):
    """MLPFusion(rgb_feat_dim=2048, thermal_feat_dim=768, hidden_dim=512, num_classes=2):
    ``.classifier`` = Sequential(Linear, ReLU, Dropout(0.7), Linear)."""

    def __init__(self, rgb_feat_dim=2048, thermal_feat_dim=768, hidden_dim=512, num_classes=2,
                 dropout=0.7, hidden_dims=None):
        super().__init__()
        dims = tuple(hidden_dims) if hidden_dims is not None else (hidden_dim,)
        self.classifier = _mlp(rgb_feat_dim + thermal_feat_dim, dims, num_classes, dropout)

    def forward(self, rgb_feat, thermal_feat):
        fused = Fn.ConcatFn.apply(rgb_feat, thermal_feat)
        return self.classifier(fused)


# DFU_INTERLEAVE_ENCODERS=0: run the ViT's forward, then the ResNet's (A/B).  Interleaved, the
# host enqueues ViT and ResNet stages alternately, so both streams start at once, and the
# autograd engine -- which runs ready backward nodes latest-created first -- alternates between
# the branches in backward instead of enqueueing the whole ResNet backward before the ViT's
# (the critical path) gets its first kernel.
_INTERLEAVE = os.environ.get("DFU_INTERLEAVE_ENCODERS", "1") != "0"


def _stageable(net):
    """The encoder has forward_stages and no hook on a container forward_stages bypasses."""
    if not hasattr(net, "forward_stages"):
        return False
    return not any(m._forward_hooks or m._forward_pre_hooks for m in net.stage_containers())


def _interleave(rgen, vgen, side):
    """Advance the ResNet generator (current stream) and the ViT generator (side stream) one
    stage at a time, in proportion to their stage counts (18 and 14); returns both outputs."""
    out = [None, None]
    live = [True, True]
    credit = [0.0, 0.0]
    share = (18.0 / 14.0, 1.0)

    def advance(i):
        try:
            if i == 0:
                next(rgen)
            else:
                with ops.on_stream(side):
                    next(vgen)
        except StopIteration as e:
            out[i] = e.value
            live[i] = False

    while live[0] or live[1]:
        for i in (1, 0):  # the ViT (critical path) first
            if live[i]:
                credit[i] += share[i]
                while live[i] and credit[i] >= 1.0:
                    credit[i] -= 1.0
                    advance(i)
    return out[0], out[1]


class MultimodalFusionModel(tnn.Module):
    """ResNet50 (RGB) + ViT-B/16 (thermal) late fusion.

    layout='eval' (default): attributes ``resnet``, ``vit``, ``fusion`` (an MLPFusion) — the
    grad_cam_visualization.py:305-320 / extended_metrics.py:353-367 model, 2816->512->2.
    layout='train': attributes ``rgb_branch``, ``thermal_branch``, ``fusion`` (a Sequential
    with hidden_dims=(512, 256)) — train_multimodal_fusion.py:285-326 keys.
    hidden_dims=None selects each layout's reference head; any sequence (list or tuple) gives
    exactly those hidden widths.
    """

    def __init__(self, num_classes=2, dropout=0.7, hidden_dims=None, layout="eval",
                 pretrained=False, concurrent_branches=True):
        super().__init__()
        self.layout = layout
        self.concurrent_branches = concurrent_branches
        rgb = resnet50(pretrained=pretrained)
        rgb.fc = tnn.Identity()
        th = vit_base_patch16_224(pretrained=pretrained, num_classes=0)
        # the ViT's 768 features reach the logits only through the 2816-wide fusion head, whose
        # dilution keeps fp16 Blocks inside the parity margin (models/vit.py _parity_policy)
        th.dfu_feature_extractor = True
        if layout == "eval":
            self.resnet = rgb
            self.vit = th
            self.fusion = MLPFusion(2048, 768, num_classes=num_classes, dropout=dropout,
                                    hidden_dims=(512,) if hidden_dims is None else hidden_dims)
        elif layout == "train":
            self.rgb_branch = rgb
            self.thermal_branch = th
            self.fusion = _mlp(2048 + 768, (512, 256) if hidden_dims is None else tuple(hidden_dims),
                               num_classes, dropout)
        else:
            raise ValueError(f"layout must be 'eval' or 'train', got {layout!r}")

    def _encode(self, rgb_net, th_net, rgb, thermal):
        """Both encoders; on the GPU the thermal ViT runs on a side stream concurrently with the
        ResNet on the current stream (their kernels fill each other's idle CUs).  Backward ops
        run on their forward op's stream (autograd), and parameter-gradient producers are
        joined by FusedAdamW.step / GradAllReducer.finish (functional.join_grad_streams)."""
        if not (self.concurrent_branches and rgb.is_cuda):
            return rgb_net(rgb), th_net(thermal)
        main = ops.current_stream()
        side = Fn.side_stream(rgb.device)
        ops.stream_wait(side, main)
        with Fn.concurrent_encoders():
            thermal.record_stream(side)
            if _INTERLEAVE and _stageable(rgb_net) and _stageable(th_net):
                rgb_feat, th_feat = _interleave(rgb_net.forward_stages(rgb),
                                                th_net.forward_stages(thermal), side)
            else:
                with ops.on_stream(side):
                    th_feat = th_net(thermal)
                rgb_feat = rgb_net(rgb)
        ops.stream_wait(main, side)
        th_feat.record_stream(main)
        return rgb_feat, th_feat

    def forward(self, rgb, thermal):
        if self.layout == "eval":
            return self.fusion(*self._encode(self.resnet, self.vit, rgb, thermal))
        f = Fn.ConcatFn.apply(*self._encode(self.rgb_branch, self.thermal_branch, rgb, thermal))
        return self.fusion(f)


class GatedFusion(tnn.Module):
    """models/fusion.py:4-18 (early-era gated fusion; off the north-star path):
    g = sigmoid(MLP(cat)), fused = g*rgb + (1-g)*th."""

    def __init__(self, feat_dim=1280):
        super().__init__()
        self.gate = tnn.Sequential(hnn.Linear(feat_dim * 2, feat_dim), hnn.ReLU(),
                                   hnn.Linear(feat_dim, feat_dim), tnn.Sigmoid())

    def forward(self, rgb_feat, th_feat):
        g = self.gate(Fn.ConcatFn.apply(rgb_feat, th_feat))
        return g * rgb_feat + (1 - g) * th_feat
