"""Reference library surface models/models.py:1-40 (RGBResNetEncoder, ThermalViTEncoder,
MultimodalFusion with its 1-logit sigmoid head)."""
import torch.nn as tnn

from dfu_hip import functional as Fn
from dfu_hip import nn as hnn

from .encoders import RGBResNetEncoder, ThermalViTEncoder  # noqa: F401


class MultimodalFusion(tnn.Module):
    """Late concatenation + MLP classifier: Linear->ReLU->Dropout(0.3)->Linear(.,1)->Sigmoid."""

    def __init__(self, rgb_dim=2048, thermal_dim=768, hidden_dim=512):
        super().__init__()
        self.classifier = tnn.Sequential(hnn.Linear(rgb_dim + thermal_dim, hidden_dim),
                                         hnn.ReLU(), hnn.Dropout(0.3),
                                         hnn.Linear(hidden_dim, 1), tnn.Sigmoid())

    def forward(self, rgb_feat, thermal_feat):
        return self.classifier(Fn.ConcatFn.apply(rgb_feat, thermal_feat))
