"""Drop-in replacements for the reference's src/unet.py models.

Same class names, constructor arguments, sub-module attribute names and
state_dict keys as the reference (src/unet.py:7-171), so that
`MobileNetV2UNet(output_channels=10).to(device)` (main.py:98, inference.py:23),
`model.load_state_dict(torch.load(...))` (inference.py:24, convert.py:23) and
`torch.save(model.state_dict(), ...)` (src/train.py:77) work unchanged.

The modules hold parameters/buffers only.  `forward` runs the whole network
on the MI355X HIP kernels (seg_amd/engine.py) as one autograd node: NHWC
activations, fused BN/activation/residual, virtual skip-concat, and a backward
pass that is the engine's own reverse program.  GPU input never falls back to
anything else; CPU input (the reference's CPU device, main.py:13-21) runs the
reference composition in torch ops (seg_amd/export.py) for that device only.
"""
from __future__ import annotations

import torch
from torch import nn

from .mobilenet import MobileNetV2, load_backbone_weights


class double_conv(nn.Module):
    """(conv3x3(+bias) => BN => ReLU) * 2  -- src/unet.py:53-68"""

    def __init__(self, in_ch, out_ch):
        super().__init__()
        self.conv = nn.Sequential(
            nn.Conv2d(in_ch, out_ch, 3, padding=1), nn.BatchNorm2d(out_ch), nn.ReLU(inplace=True),
            nn.Conv2d(out_ch, out_ch, 3, padding=1), nn.BatchNorm2d(out_ch), nn.ReLU(inplace=True))


class inconv(nn.Module):
    """src/unet.py:71-77"""

    def __init__(self, in_ch, out_ch):
        super().__init__()
        self.conv = double_conv(in_ch, out_ch)


class down(nn.Module):
    """MaxPool2d(2) + double_conv -- src/unet.py:80-91"""

    def __init__(self, in_ch, out_ch):
        super().__init__()
        self.mpconv = nn.Sequential(nn.MaxPool2d(2), double_conv(in_ch, out_ch))


class up(nn.Module):
    """bilinear x2 (align_corners=False) of x1, cat([x2, x1]), double_conv -- src/unet.py:94-105"""

    def __init__(self, in_ch, out_ch):
        super().__init__()
        self.up = nn.Upsample(scale_factor=2, mode="bilinear")
        self.conv = double_conv(in_ch, out_ch)


class outconv(nn.Module):
    """1x1 -> BN -> ReLU -> 1x1 head -- src/unet.py:108-121"""

    def __init__(self, in_ch, out_ch):
        super().__init__()
        self.conv = nn.Sequential(
            nn.Conv2d(in_ch, in_ch // 2, 1), nn.BatchNorm2d(in_ch // 2), nn.ReLU(inplace=True),
            nn.Conv2d(in_ch // 2, out_ch, 1))


class _SegModel(nn.Module):
    """Shared forward.  A CUDA tensor runs through the HIP engine (and nothing else: a
    missing libsegamd.so raises).  A CPU tensor -- main.py:13-21 picks the CPU when no GPU
    is present, BASELINE configs[0] -- runs the reference's own composition in torch ops
    on this module's parameters (seg_amd.export.torch_forward), so train_model, Adam and
    state_dict work there too; the product never selects it for GPU input."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if x.device.type == "cpu":
            from .export import torch_forward
            return torch_forward(self, x)
        from .engine import run_logits
        return run_logits(self, x)

    def forward_loss(self, x: torch.Tensor, target: torch.Tensor, ignore_index: int = -100) -> torch.Tensor:
        """nn.CrossEntropyLoss()(self(x), target) (main.py:99, src/train.py:37) fused
        with the final upsample: the full-resolution logits are never stored."""
        if x.device.type == "cpu":
            return nn.functional.cross_entropy(self(x), target, ignore_index=ignore_index)
        from .engine import run_loss
        return run_loss(self, x, target, ignore_index)


class MobileNetV2UNet(_SegModel):
    """src/unet.py:7-51.  `backbone_weights`: optional LOCAL path to torchvision
    MobileNetV2 ImageNet weights (the reference downloads them, src/unet.py:12)."""

    def __init__(self, output_channels=1, backbone_weights: str | None = None):
        super().__init__()
        self.backbone = MobileNetV2()
        if backbone_weights:
            load_backbone_weights(self.backbone, backbone_weights)
        f = self.backbone.features
        self.down1 = f[:2]      # 16 ch, 1/2
        self.down2 = f[2:4]     # 24 ch, 1/4
        self.down3 = f[4:7]     # 32 ch, 1/8
        self.down4 = f[7:11]    # 64 ch, 1/16
        self.down5 = f[11:19]   # 1280 ch, 1/32
        self.up1 = up(1280 + 64, 256)
        self.up2 = up(256 + 32, 128)
        self.up3 = up(128 + 24, 64)
        self.up4 = up(64 + 16, 32)
        self.outc = outconv(32, output_channels)
        self.final_upsample = nn.Upsample(scale_factor=2, mode="bilinear", align_corners=True)


class UNet(_SegModel):
    """src/unet.py:124-147"""

    def __init__(self, output_channels=1, base_filters=64):
        super().__init__()
        b = base_filters
        self.inc = inconv(3, b)
        self.down1 = down(b, b * 2)
        self.down2 = down(b * 2, b * 4)
        self.down3 = down(b * 4, b * 4)
        self.up1 = up(b * 8, b * 2)
        self.up2 = up(b * 4, b)
        self.up3 = up(b * 2, b)
        self.sem_out = outconv(b, output_channels)


class LightUNet(_SegModel):
    """src/unet.py:149-171 (UNet with base 32 and one output channel)."""

    def __init__(self, base_filters=32):
        super().__init__()
        b = base_filters
        self.inc = inconv(3, b)
        self.down1 = down(b, b * 2)
        self.down2 = down(b * 2, b * 4)
        self.down3 = down(b * 4, b * 4)
        self.up1 = up(b * 8, b * 2)
        self.up2 = up(b * 4, b)
        self.up3 = up(b * 2, b)
        self.sem_out = outconv(b, 1)
