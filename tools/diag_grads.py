"""Diagnostic (not a test): per-tensor gradient error of the HIP path vs the fp64
oracle, as a multiple of the SURVEY 4.4 tolerance.  Usage on the GPU box:
    python tests/diag_grads.py UNet 4 2 32 64
"""
import os
import sys

import torch

sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), p)
                for p in ("team02-objectdetection_amd", "")]
from oracle import segref  # noqa: E402
from seg_amd import LightUNet, MobileNetV2UNet, UNet  # noqa: E402
from seg_amd.detinit import deterministic_init, synthetic_batch  # noqa: E402

CT = {"MobileNetV2UNet": lambda c: MobileNetV2UNet(c), "UNet": lambda c: UNet(c, 64), "LightUNet": lambda c: LightUNet()}


def main(arch="UNet", classes=4, n=2, h=32, w=64, seed=3):
    classes, n, h, w, seed = int(classes), int(n), int(h), int(w), int(seed)
    mc = deterministic_init(CT[arch](classes), seed=seed)
    m = deterministic_init(CT[arch](classes), seed=seed).cuda().train()
    x, y = synthetic_batch(n, h, w, classes, seed=seed + 100)
    loss = m.forward_loss(x.cuda(), y.cuda())
    loss.backward()
    p32 = segref.canonical_state(mc.state_dict())
    p64 = segref.canonical_state(mc.state_dict(), torch.float64)
    l32, _, g32 = segref.forward_backward(arch, p32, x, y, True)
    l64, _, g64 = segref.forward_backward(arch, p64, x.double(), y, True)
    print("loss", loss.item(), float(l32), float(l64))
    G = float(torch.sqrt(sum((g ** 2).sum() for g in g64.values())))
    rows = []
    for k, prm in m.named_parameters():
        if k not in g64:
            continue
        g = prm.grad.double().cpu()
        d = float((g - g64[k]).norm())
        e32 = float((g32[k].double() - g64[k]).norm())
        tol = max(1e-3 * float(g64[k].norm()), 4 * e32, 1e-4 * G)
        rows.append((d / tol, k, d, e32, float(g64[k].norm())))
    rows.sort(reverse=True)
    for r in rows[:25]:
        print("%6.2f  %-45s d=%.3e eps32=%.3e |g64|=%.3e" % r)


if __name__ == "__main__":
    main(*sys.argv[1:])
