"""Traceable pure-PyTorch twins of the segamd models -- for ONNX export and CPU use.

The segamd models run their whole forward/backward as one HIP autograd node over
ctypes calls (seg_amd/engine.py), which torch.onnx.export / torch.jit.trace cannot see
through, and they refuse CPU input (there is no CPU execution path in the product).
The reference needs a traceable forward for convert.py:21-42 (torch.onnx.export,
opset 12, dynamic batch) and runs on the CPU when no GPU is present (main.py:13-21,
BASELINE configs[0]).  `traceable(model)` builds that module explicitly:

  * the same class layout, attribute names and state_dict keys (it IS the segamd
    model class with a torch-op forward), holding a CPU COPY of the model's state;
  * forward = the reference's own composition (src/unet.py:32-51, 94-121, 137-147 and
    torchvision's InvertedResidual) over nn.Conv2d / BatchNorm2d / ReLU(6) / Upsample /
    MaxPool2d modules, so tracing records standard aten ops;
  * it refuses CUDA input: on an MI355X the HIP model itself is the compute path, and
    nothing in the product ever routes a CUDA tensor here.

    model = MobileNetV2UNet(10).to("cuda"); ...            # train / infer on the HIP path
    torch.onnx.export(seg_amd.traceable(model), torch.randn(1, 3, 128, 256), path, ...)
"""
from __future__ import annotations

import torch
from torch import nn

from .mobilenet import ConvBNReLU6, InvertedResidual
from .unet import LightUNet, MobileNetV2UNet, UNet


def _block(m, x):
    if isinstance(m, InvertedResidual):
        out = m.conv(x)
        return x + out if m.use_res_connect else out
    if isinstance(m, ConvBNReLU6):
        return m(x)
    raise TypeError(f"unexpected encoder block {type(m).__name__}")


def _stage(seq, x):
    for m in seq:
        x = _block(m, x)
    return x


def _up(u, x1, x2):
    # src/unet.py:100-105: bilinear x2 (align_corners=False), cat([skip, up]), double_conv
    return u.conv.conv(torch.cat([x2, u.up(x1)], dim=1))


def _check(x):
    if x.device.type != "cpu":
        raise RuntimeError("seg_amd.traceable() modules are for export and CPU use; on the MI355X run the segamd "
                           "model itself (the HIP path)")


def mobilenet_unet_forward(m, x):
    """MobileNetV2UNet.forward (src/unet.py:32-51) over m's own modules, in torch ops."""
    x1 = _stage(m.down1, x)
    x2 = _stage(m.down2, x1)
    x3 = _stage(m.down3, x2)
    x4 = _stage(m.down4, x3)
    x5 = _stage(m.down5, x4)
    x = _up(m.up1, x5, x4)
    x = _up(m.up2, x, x3)
    x = _up(m.up3, x, x2)
    x = _up(m.up4, x, x1)
    return m.final_upsample(m.outc.conv(x))


def unet_forward(m, x):
    """UNet / LightUNet.forward (src/unet.py:137-147, :160-171) over m's own modules."""
    x1 = m.inc.conv.conv(x)
    x2 = m.down1.mpconv[1].conv(m.down1.mpconv[0](x1))
    x3 = m.down2.mpconv[1].conv(m.down2.mpconv[0](x2))
    x4 = m.down3.mpconv[1].conv(m.down3.mpconv[0](x3))
    x = _up(m.up1, x4, x3)
    x = _up(m.up2, x, x2)
    x = _up(m.up3, x, x1)
    return m.sem_out.conv(x)


def torch_forward(model, x):
    """The reference composition of `model` (a segamd model) in torch ops on its OWN
    parameters, under autograd.  Used for CPU tensors only (main.py:13-21's CPU device,
    BASELINE configs[0]); CUDA input always runs the HIP engine (unet._SegModel.forward)."""
    _check(x)
    return mobilenet_unet_forward(model, x) if isinstance(model, MobileNetV2UNet) else unet_forward(model, x)


class TorchMobileNetV2UNet(MobileNetV2UNet):
    def forward(self, x):
        return torch_forward(self, x)

    def forward_loss(self, x, target, ignore_index: int = -100):
        return nn.functional.cross_entropy(self(x), target, ignore_index=ignore_index)


class _TorchUNetMixin:
    def forward(self, x):
        return torch_forward(self, x)

    def forward_loss(self, x, target, ignore_index: int = -100):
        return nn.functional.cross_entropy(self(x), target, ignore_index=ignore_index)


class TorchUNet(_TorchUNetMixin, UNet):
    pass


class TorchLightUNet(_TorchUNetMixin, LightUNet):
    pass


@torch.no_grad()
def traceable(model: nn.Module) -> nn.Module:
    """A CPU, pure-torch copy of `model` (a segamd MobileNetV2UNet / UNet / LightUNet,
    or a DataParallel wrapper of one) with identical state_dict and train/eval mode."""
    model = getattr(model, "module", model)
    if isinstance(model, MobileNetV2UNet):
        twin = TorchMobileNetV2UNet(model.outc.conv[3].out_channels)
    elif isinstance(model, LightUNet):
        twin = TorchLightUNet(model.inc.conv.conv[0].out_channels)
    elif isinstance(model, UNet):
        twin = TorchUNet(model.sem_out.conv[3].out_channels, model.inc.conv.conv[0].out_channels)
    else:
        raise TypeError(f"no traceable twin for {type(model).__name__}")
    twin.load_state_dict({k: v.detach().cpu() for k, v in model.state_dict().items()})
    return twin.train(model.training)
