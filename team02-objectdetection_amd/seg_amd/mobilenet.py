"""MobileNetV2 encoder containers with torchvision's parameter layout.

The reference builds its encoder with `torchvision.models.mobilenet_v2`
(src/unet.py:12) and slices `backbone.features` into down1..down5
(src/unet.py:15-19).  torchvision is a third-party dependency (unpinned,
requirements.txt:2) and is not installed here, so this module re-declares the
*parameter structure* of that network -- the published MobileNetV2 (Sandler et
al. 2018, torchvision v0.13+ module names) -- so that state_dict keys
(`backbone.features.N.conv.M.*`, `backbone.classifier.1.*`) match the
reference's checkpoints exactly.  These modules only hold parameters and
buffers; the computation is done by the HIP engine (seg_amd/engine.py).
"""
from __future__ import annotations

import torch
from torch import nn

# (expand ratio t, out channels c, repeats n, first stride s) -- MobileNetV2 Table 2
INVERTED_RESIDUAL_SETTING = ((1, 16, 1, 1), (6, 24, 2, 2), (6, 32, 3, 2), (6, 64, 4, 2),
                             (6, 96, 3, 1), (6, 160, 3, 2), (6, 320, 1, 1))


def make_divisible(v: float, divisor: int = 8) -> int:
    """Round channel counts to a multiple of 8 without dropping more than 10%."""
    new_v = max(divisor, int(v + divisor / 2) // divisor * divisor)
    if new_v < 0.9 * v:
        new_v += divisor
    return new_v


class ConvBNReLU6(nn.Sequential):
    """conv(k, stride, pad=(k-1)//2, groups, bias=False) -> BatchNorm2d -> ReLU6
    (torchvision's Conv2dNormActivation with its MobileNetV2 defaults)."""

    def __init__(self, cin: int, cout: int, kernel_size: int = 3, stride: int = 1, groups: int = 1):
        super().__init__(
            nn.Conv2d(cin, cout, kernel_size, stride, (kernel_size - 1) // 2, groups=groups, bias=False),
            nn.BatchNorm2d(cout),
            nn.ReLU6(inplace=True),
        )
        self.out_channels = cout


class InvertedResidual(nn.Module):
    """[1x1 expand + BN + ReLU6] -> dw3x3(stride) + BN + ReLU6 -> 1x1 project + BN (+x)."""

    def __init__(self, inp: int, oup: int, stride: int, expand_ratio: int):
        super().__init__()
        if stride not in (1, 2):
            raise ValueError(f"stride should be 1 or 2, got {stride}")
        self.stride = stride
        hidden = int(round(inp * expand_ratio))
        self.use_res_connect = stride == 1 and inp == oup
        layers = []
        if expand_ratio != 1:
            layers.append(ConvBNReLU6(inp, hidden, kernel_size=1))
        layers += [ConvBNReLU6(hidden, hidden, stride=stride, groups=hidden),
                   nn.Conv2d(hidden, oup, 1, 1, 0, bias=False),
                   nn.BatchNorm2d(oup)]
        self.conv = nn.Sequential(*layers)
        self.out_channels = oup
        self._is_cn = stride > 1


class MobileNetV2(nn.Module):
    """`features` (stem + 17 inverted residuals + 1x1 to 1280) and the (unused by
    the segmentation models) classifier."""

    def __init__(self, num_classes: int = 1000, width_mult: float = 1.0, dropout: float = 0.2):
        super().__init__()
        cin = make_divisible(32 * width_mult)
        self.last_channel = make_divisible(1280 * max(1.0, width_mult))
        feats = [ConvBNReLU6(3, cin, stride=2)]
        for t, c, n, s in INVERTED_RESIDUAL_SETTING:
            cout = make_divisible(c * width_mult)
            for i in range(n):
                feats.append(InvertedResidual(cin, cout, s if i == 0 else 1, t))
                cin = cout
        feats.append(ConvBNReLU6(cin, self.last_channel, kernel_size=1))
        self.features = nn.Sequential(*feats)
        self.classifier = nn.Sequential(nn.Dropout(p=dropout), nn.Linear(self.last_channel, num_classes))
        self.reset_parameters()

    def reset_parameters(self) -> None:
        # torchvision's MobileNetV2 init: kaiming-normal(fan_out) convs, unit BN, N(0, .01) linear
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out")
                if m.bias is not None:
                    nn.init.zeros_(m.bias)
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
            elif isinstance(m, nn.Linear):
                nn.init.normal_(m.weight, 0, 0.01)
                nn.init.zeros_(m.bias)

    def forward(self, x):  # pragma: no cover - the segmentation models never call it
        raise RuntimeError("MobileNetV2 is used as a parameter container; run MobileNetV2UNet instead")


def load_backbone_weights(backbone: MobileNetV2, path: str) -> None:
    """Load torchvision-format MobileNetV2 weights from a LOCAL file (the
    reference downloads MobileNet_V2_Weights.DEFAULT, src/unet.py:12; there is
    no network here).  Loaded with weights_only=True."""
    sd = torch.load(path, map_location="cpu", weights_only=True)
    backbone.load_state_dict(sd)
