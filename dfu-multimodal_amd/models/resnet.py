"""ResNet-50 (torchvision v0.13.1 semantics, the hub tag at train_multimodal_fusion.py:294)
on MI355X kernels.

Attribute tree and state_dict keys are torchvision's (conv1, bn1, relu, maxpool,
layer1..layer4[i].{conv1,bn1,conv2,bn2,conv3,bn3,relu,downsample}, avgpool, fc), so
``.fc.in_features``, ``model.fc = nn.Identity()`` / ``nn.Sequential(Dropout, Linear)``
(train_rgb_only.py:211) and checkpoint loaders work unchanged.  Compute runs as fused
blocks (functional.StemFn / BottleneckFn) on NHWC bf16 activations with fp32 accumulation.
"""
import torch
import torch.nn as tnn

from dfu_hip import functional as Fn
from dfu_hip import nn as hnn
from dfu_hip.functional import module_param


def conv3x3(in_planes, out_planes, stride=1):
    return hnn.Conv2d(in_planes, out_planes, kernel_size=3, stride=stride, padding=1, bias=False)


def conv1x1(in_planes, out_planes, stride=1):
    return hnn.Conv2d(in_planes, out_planes, kernel_size=1, stride=stride, bias=False)


class Bottleneck(tnn.Module):
    """torchvision Bottleneck (ResNet v1.5: stride on the 3x3 conv)."""

    expansion = 4
    # forward precision under functional.precision("parity") (models/precision.py)
    dfu_parity_precision = "bf16x3"

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        width = planes
        self.conv1 = conv1x1(inplanes, width)
        self.bn1 = hnn.BatchNorm2d(width)
        self.conv2 = conv3x3(width, width, stride)
        self.bn2 = hnn.BatchNorm2d(width)
        self.conv3 = conv1x1(width, planes * self.expansion)
        self.bn3 = hnn.BatchNorm2d(planes * self.expansion)
        self.relu = hnn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def _params(self):
        # through the modules' dicts: nn.Module.__getattr__ is the slow path (~0.25 us an
        # attribute, 12-18 a block a step)
        m = self._modules
        ps = []
        for name in ("conv1", "bn1", "conv2", "bn2", "conv3", "bn3"):
            mod = m[name]
            ps.append(module_param(mod, "weight"))
            if name[0] == "b":
                ps.append(module_param(mod, "bias"))
        ds = m.get("downsample")
        if ds is not None:
            ps += [ds[0].weight, ds[1].weight, ds[1].bias]
        return ps

    def forward(self, x):
        hooked = bool(self.relu._forward_hooks or self.relu._forward_pre_hooks)
        self._probe = hooked and torch.is_grad_enabled()
        out = Fn.BottleneckFn.apply(x, *self._params(), self)
        if hooked:
            # Someone hooks `relu` (Grad-CAM target 'layer4.2.relu',
            # grad_cam_visualization.py:355-357, 389-392).  torchvision calls it three times per
            # block — after bn1, after bn2, after the residual add — and the reference's CAM
            # depends on that (its stored gradient is the first call's, its activation the
            # last's).  Replay the two inner calls to the forward hooks with probe leaves that
            # BottleneckFn.backward feeds their gradients to, then call the module on the
            # block output (already relu(...), so the idempotent ReLU is exact).
            for probe in self.__dict__.pop("_probes", ()):
                for hook in list(self.relu._forward_hooks.values()):
                    hook(self.relu, (probe,), probe)
            out = self.relu(out)
        return out


class ResNet(tnn.Module):
    def __init__(self, layers=(3, 4, 6, 3), num_classes=1000, zero_init_residual=False):
        super().__init__()
        self.inplanes = 64
        self.dilation = 1
        self.groups = 1
        self.base_width = 64
        self.conv1 = hnn.Conv2d(3, self.inplanes, kernel_size=7, stride=2, padding=3, bias=False)
        self.bn1 = hnn.BatchNorm2d(self.inplanes)
        self.relu = hnn.ReLU(inplace=True)
        self.maxpool = hnn.MaxPool2d(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._make_layer(64, layers[0])
        self.layer2 = self._make_layer(128, layers[1], stride=2)
        self.layer3 = self._make_layer(256, layers[2], stride=2)
        self.layer4 = self._make_layer(512, layers[3], stride=2)
        self.avgpool = hnn.AdaptiveAvgPool2d((1, 1))
        self.fc = hnn.Linear(512 * Bottleneck.expansion, num_classes)
        # torchvision resnet.py init: kaiming_normal_(fan_out, relu) convs, BN weight 1 bias 0
        for m in self.modules():
            if isinstance(m, tnn.Conv2d):
                tnn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, (tnn.BatchNorm2d, tnn.GroupNorm)):
                tnn.init.constant_(m.weight, 1)
                tnn.init.constant_(m.bias, 0)
        if zero_init_residual:  # torchvision option: each block starts as the identity
            for m in self.modules():
                if isinstance(m, Bottleneck):
                    tnn.init.constant_(m.bn3.weight, 0)

    def _make_layer(self, planes, blocks, stride=1):
        downsample = None
        if stride != 1 or self.inplanes != planes * Bottleneck.expansion:
            downsample = tnn.Sequential(
                conv1x1(self.inplanes, planes * Bottleneck.expansion, stride),
                hnn.BatchNorm2d(planes * Bottleneck.expansion),
            )
        layers = [Bottleneck(self.inplanes, planes, stride, downsample)]
        self.inplanes = planes * Bottleneck.expansion
        for _ in range(1, blocks):
            layers.append(Bottleneck(self.inplanes, planes))
        return tnn.Sequential(*layers)

    def forward_features(self, x):
        """conv1 .. layer4 -> bf16 channels_last (B, 2048, 7, 7)."""
        x = Fn.StemFn.apply(x, self.conv1.weight, self.bn1.weight, self.bn1.bias, self)
        x = self.layer1(x)
        x = self.layer2(x)
        x = self.layer3(x)
        x = self.layer4(x)
        return x

    def forward(self, x):
        x = self.forward_features(x)
        x = self.avgpool(x)
        x = torch.flatten(x, 1)
        return self.fc(x)

    def forward_stages(self, x):
        """forward() as a generator that yields after the stem and after every Bottleneck and
        returns the output (StopIteration.value): models.fusion interleaves the two encoders'
        stages so both streams get work early and their backward nodes alternate in the
        autograd engine's queue.  The same modules are called as in forward(); only the
        containers' own calls are skipped (fusion uses it when no hook sits on them)."""
        x = Fn.StemFn.apply(x, self.conv1.weight, self.bn1.weight, self.bn1.bias, self)
        yield
        for layer in (self.layer1, self.layer2, self.layer3, self.layer4):
            for blk in layer:
                x = blk(x)
                yield
        x = self.avgpool(x)
        x = torch.flatten(x, 1)
        return self.fc(x)

    def stage_containers(self):
        return (self, self.layer1, self.layer2, self.layer3, self.layer4)


def resnet50(num_classes=1000, zero_init_residual=False):
    return ResNet((3, 4, 6, 3), num_classes=num_classes, zero_init_residual=zero_init_residual)
