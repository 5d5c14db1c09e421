"""Local stand-in for the `torchvision.models` symbols the reference imports
(src/unet.py:4-5): `mobilenet_v2(weights=...)` and `MobileNet_V2_Weights`.

torchvision is not installed in this image.  This is a restatement of the
published MobileNetV2 (torchvision >= 0.13 module layout) used ONLY by
tests/golden/make_golden.py to import and run the reference's own
src/unet.py on CPU.  Self-check (test_oracle.py): 3,504,872 parameters and the
`features.N.conv.M.*` key layout, as documented for torchvision.
Pretrained weights are never fetched (no network): `weights` is ignored and
the caller re-initialises every tensor deterministically.
"""
from __future__ import annotations

import sys
import types

from torch import nn


def _make_divisible(v, divisor=8):
    new_v = max(divisor, int(v + divisor / 2) // divisor * divisor)
    if new_v < 0.9 * v:
        new_v += divisor
    return new_v


class Conv2dNormActivation(nn.Sequential):
    def __init__(self, cin, cout, kernel_size=3, stride=1, groups=1):
        super().__init__(nn.Conv2d(cin, cout, kernel_size, stride, (kernel_size - 1) // 2, groups=groups, bias=False),
                         nn.BatchNorm2d(cout), nn.ReLU6(inplace=True))


class InvertedResidual(nn.Module):
    def __init__(self, inp, oup, stride, expand_ratio):
        super().__init__()
        hidden = int(round(inp * expand_ratio))
        self.use_res_connect = stride == 1 and inp == oup
        layers = []
        if expand_ratio != 1:
            layers.append(Conv2dNormActivation(inp, hidden, kernel_size=1))
        layers += [Conv2dNormActivation(hidden, hidden, stride=stride, groups=hidden),
                   nn.Conv2d(hidden, oup, 1, 1, 0, bias=False), nn.BatchNorm2d(oup)]
        self.conv = nn.Sequential(*layers)

    def forward(self, x):
        return x + self.conv(x) if self.use_res_connect else self.conv(x)


class MobileNetV2(nn.Module):
    def __init__(self, num_classes=1000):
        super().__init__()
        setting = [[1, 16, 1, 1], [6, 24, 2, 2], [6, 32, 3, 2], [6, 64, 4, 2], [6, 96, 3, 1], [6, 160, 3, 2],
                   [6, 320, 1, 1]]
        cin = _make_divisible(32)
        last = _make_divisible(1280)
        feats = [Conv2dNormActivation(3, cin, stride=2)]
        for t, c, n, s in setting:
            for i in range(n):
                feats.append(InvertedResidual(cin, _make_divisible(c), s if i == 0 else 1, t))
                cin = _make_divisible(c)
        feats.append(Conv2dNormActivation(cin, last, kernel_size=1))
        self.features = nn.Sequential(*feats)
        self.classifier = nn.Sequential(nn.Dropout(0.2), nn.Linear(last, num_classes))

    def forward(self, x):
        x = self.features(x)
        x = nn.functional.adaptive_avg_pool2d(x, (1, 1)).flatten(1)
        return self.classifier(x)


class MobileNet_V2_Weights:  # noqa: N801 (torchvision's name)
    DEFAULT = "IMAGENET1K_V2"
    IMAGENET1K_V1 = "IMAGENET1K_V1"
    IMAGENET1K_V2 = "IMAGENET1K_V2"


def mobilenet_v2(weights=None, progress=True, **kwargs):
    return MobileNetV2(**kwargs)


def install():
    """Register `torchvision` and `torchvision.models` in sys.modules."""
    tv = types.ModuleType("torchvision")
    models = types.ModuleType("torchvision.models")
    models.mobilenet_v2 = mobilenet_v2
    models.MobileNet_V2_Weights = MobileNet_V2_Weights
    tv.models = models
    sys.modules["torchvision"] = tv
    sys.modules["torchvision.models"] = models
