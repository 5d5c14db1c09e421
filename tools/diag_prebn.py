"""Diagnostics: magnitude of the pre-BatchNorm conv bias gradients (analytically zero:
BN removes the per-channel mean) in the HIP path vs the reference's fp32 / fp64 (golden
fixture), and their Adam update size.  python tools/diag_prebn.py"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "team02-objectdetection_amd"), REPO]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from seg_amd import MobileNetV2UNet, deterministic_init  # noqa: E402
from seg_amd.detinit import synthetic_scene  # noqa: E402
from oracle import segref  # noqa: E402

m = deterministic_init(MobileNetV2UNet(10), seed=3)
x, y = synthetic_scene(8, 128, 256, 10, seed=100)
p32 = segref.canonical_state(m.state_dict())
p64 = segref.canonical_state(m.state_dict(), torch.float64)
_, _, g32 = segref.forward_backward("MobileNetV2UNet", p32, x, y, True)
_, _, g64 = segref.forward_backward("MobileNetV2UNet", p64, x.double(), y, True)
mg = deterministic_init(MobileNetV2UNet(10), seed=3).cuda().train()
mg.forward_loss(x.cuda(), y.cuda()).backward()
gh = {k: p.grad.double().cpu() for k, p in mg.named_parameters() if p.grad is not None}
for k in g64:
    if k.startswith(("up", "outc.conv.0")) and k.endswith("bias") and ".conv.0." in k or ".conv.3.bias" in k:
        if k.startswith("outc.conv.3"):
            continue
        print(f"{k:28s} |g| hip {gh[k].abs().mean():.3e}  ref32 {g32[k].abs().mean():.3e}  ref64 "
              f"{g64[k].abs().mean():.3e}   (weight grad scale {g64[k.replace('bias', 'weight')].abs().mean():.3e})")
