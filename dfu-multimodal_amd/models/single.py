"""Single-modality classifiers of the reference's C1 / C2 scripts, on the HIP encoders.

  RGBOnlyModel      notebooks/train_rgb_only.py:200-217: ``self.backbone`` = torchvision
                    resnet50 with ``fc = Sequential(Dropout(DROP_RATE), Linear(2048, 2))``
  ThermalOnlyModel  notebooks/train_thermal_only.py:188-205: ``self.backbone`` = timm
                    vit_base_patch16_224(num_classes=2) with ``head = Sequential(Dropout,
                    Linear(768, 2))``
State-dict keys are the reference's (``backbone.*``); ``pretrained=True`` cannot download offline
(see models.encoders).  DROP_RATE = 0.5 in both scripts (:44 / :45).  layout="eval" builds the
evaluation scripts' twins instead (extended_metrics.py:307-335: the encoder as ``.resnet`` /
``.vit``), which load the training checkpoints through load_checkpoint_flexible's
``backbone.`` remap.
"""
import torch.nn as tnn

from dfu_hip import nn as hnn

from .encoders import resnet50, vit_base_patch16_224

DROP_RATE = 0.5


def _attr(layout, eval_name):
    if layout not in ("train", "eval"):
        raise ValueError(f"layout must be 'train' or 'eval', got {layout!r}")
    return "backbone" if layout == "train" else eval_name


class RGBOnlyModel(tnn.Module):
    def __init__(self, num_classes=2, pretrained=False, drop_rate=DROP_RATE, weights_path=None,
                 layout="train"):
        super().__init__()
        self._enc = _attr(layout, "resnet")
        net = resnet50(pretrained=pretrained, weights_path=weights_path)
        in_features = net.fc.in_features
        net.fc = tnn.Sequential(hnn.Dropout(p=drop_rate), hnn.Linear(in_features, num_classes))
        setattr(self, self._enc, net)

    def forward(self, x):
        return getattr(self, self._enc)(x)


class ThermalOnlyModel(tnn.Module):
    def __init__(self, num_classes=2, pretrained=False, drop_rate=DROP_RATE, weights_path=None,
                 layout="train"):
        super().__init__()
        self._enc = _attr(layout, "vit")
        net = vit_base_patch16_224(pretrained=pretrained, num_classes=num_classes,
                                   weights_path=weights_path)
        in_features = net.head.in_features
        net.head = tnn.Sequential(hnn.Dropout(p=drop_rate), hnn.Linear(in_features, num_classes))
        setattr(self, self._enc, net)

    def forward(self, x):
        return getattr(self, self._enc)(x)
