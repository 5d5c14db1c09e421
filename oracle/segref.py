"""CPU ORACLE -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module, and only as the checker / CPU baseline -- never as the product
path (the product, team02-objectdetection_amd/seg_amd, has no CPU path).

A functional, fp32-or-fp64 restatement on torch CPU (aten/oneDNN) of the
reference's hot path, written over a flat state_dict so it shares no code with
the product modules:
  * MobileNetV2UNet.forward            src/unet.py:32-51
  * torchvision mobilenet_v2 features  (third-party, unpinned in
    requirements.txt:2; restated from the published architecture: stem
    conv3x3 s2 + 17 InvertedResidual(t,c,n,s) blocks + 1x1 to 1280,
    ReLU6 everywhere, residual when stride 1 and cin == cout)
  * up / double_conv / outconv         src/unet.py:53-68, 94-121
  * UNet / LightUNet                   src/unet.py:124-171 (inconv :71-77, down :80-91)
  * nn.CrossEntropyLoss()              main.py:99, src/train.py:37
  * Adam(lr=1.5e-4) training step      main.py:100, src/train.py:35-39

Parity is PINNED by tests/golden/*.npz, produced by tests/golden/make_golden.py
from the reference's own src/unet.py (imported here, in the build container,
with a local torchvision stand-in); tests/test_oracle.py checks this module
against every fixture.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

MBV2_SETTING = ((1, 16, 1, 1), (6, 24, 2, 2), (6, 32, 3, 2), (6, 64, 4, 2),
                (6, 96, 3, 1), (6, 160, 3, 2), (6, 320, 1, 1))


def _bn(p, pre, x, training, momentum=0.1, eps=1e-5):
    # nn.BatchNorm2d: biased batch var for normalisation, unbiased for running_var
    return F.batch_norm(x, p[pre + "running_mean"], p[pre + "running_var"], p[pre + "weight"], p[pre + "bias"],
                        training, momentum, eps)


def _bump(p, pre, training):
    if training and (pre + "num_batches_tracked") in p:
        p[pre + "num_batches_tracked"] += 1


# Activation masks (tests only).  ReLU / ReLU6 gradients are discontinuous in the
# pre-activation z: an element within rounding distance of a threshold may pass the
# gradient in one valid fp32 implementation and block it in another.  MASK_OVERRIDE =
# {layer prefix: bool mask (NCHW)} makes the backward of that layer's activation use the
# given mask (the forward values are unchanged), so the oracle can be run with another
# implementation's masks (oracle/budget.py).  ACT_HI records each layer's upper
# threshold (6 for ReLU6, None for ReLU) as the forward passes it.
MASK_OVERRIDE = None
ACT_HI = {}


class _ActMasked(torch.autograd.Function):
    @staticmethod
    def forward(ctx, z, hi, mask):
        ctx.save_for_backward(mask)
        return z.clamp(0.0, hi) if hi is not None else z.clamp(min=0.0)

    @staticmethod
    def backward(ctx, g):
        (mask,) = ctx.saved_tensors
        return g * mask.to(g.dtype), None, None


# Max-pool window choices (tests only).  MaxPool2d's gradient is discontinuous in its input the same way: two
# elements of a 2x2 window within rounding distance of each other swap the window's argmax between two valid fp32
# implementations, and the whole window's gradient moves to the other element.  POOL_OVERRIDE = {pool name: window
# positions [N, C, H/2, W/2] (0..3, row-major in the window)} routes the backward through the given positions (the
# forward values are unchanged), so the oracle can be run with another implementation's choices (oracle/budget.py).
POOL_OVERRIDE = None


class _PoolChosen(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, pos):
        ctx.save_for_backward(pos)
        ctx.shape = x.shape
        return F.max_pool2d(x, 2)

    @staticmethod
    def backward(ctx, g):
        (pos,) = ctx.saved_tensors
        N, C, H, W = ctx.shape
        gx = torch.zeros(N, C, H // 2, W // 2, 4, dtype=g.dtype)
        gx.scatter_(4, pos.unsqueeze(-1), g.unsqueeze(-1))
        gx = gx.view(N, C, H // 2, W // 2, 2, 2).permute(0, 1, 2, 4, 3, 5).reshape(N, C, H, W)
        return gx, None


def pool_positions(a):
    """First-max position (0..3, row-major) of every 2x2 window of a [N, C, H, W] (aten's / the kernel's tie rule)."""
    N, C, H, W = a.shape
    w = a.reshape(N, C, H // 2, 2, W // 2, 2).permute(0, 1, 2, 4, 3, 5).reshape(N, C, H // 2, W // 2, 4)
    return w.argmax(-1)


def _pool(name, x):
    if POOL_OVERRIDE is not None and name in POOL_OVERRIDE:
        return _PoolChosen.apply(x, POOL_OVERRIDE[name])
    return F.max_pool2d(x, 2)


def act_mask(z, hi):
    """aten's gradient mask: hardtanh_backward passes 0 < z < 6 (strict), threshold_backward z > 0."""
    return (z > 0) & (z < hi) if hi is not None else z > 0


def _act(name, z, hi):
    ACT_HI[name] = hi
    if MASK_OVERRIDE is not None and name in MASK_OVERRIDE:
        return _ActMasked.apply(z, hi, MASK_OVERRIDE[name])
    return F.hardtanh(z, 0.0, 6.0) if hi is not None else F.relu(z)


def _cbr(p, pre_conv, pre_bn, x, training, stride=1, pad=0, groups=1, act="relu6", bias=None):
    y = F.conv2d(x, p[pre_conv + "weight"], p.get(pre_conv + "bias") if bias is None else bias,
                 stride=stride, padding=pad, groups=groups)
    _rec(pre_conv + "raw", y)
    y = _bn(p, pre_bn, y, training)
    _bump(p, pre_bn, training)
    if act == "relu6":
        return _rec(pre_conv + "out", _act(pre_conv, _rec(pre_conv + "z", y), 6.0))
    if act == "relu":
        return _rec(pre_conv + "out", _act(pre_conv, _rec(pre_conv + "z", y), None))
    return _rec(pre_conv + "out", y)


def preactivations(arch, p, x, training=True):
    """{conv layer prefix: its post-BN pre-activation z} of one forward (no grad)."""
    global RECORD
    saved, RECORD = RECORD, {}
    try:
        with torch.no_grad():
            FORWARDS[arch](p, x, training)
        return {k[:-1]: v for k, v in RECORD.items() if k.endswith(".z")}
    finally:
        RECORD = saved


def mobilenet_features(p, x, training, prefix="backbone.features."):
    """Returns the outputs after features[1], [3], [6], [10], [18]
    (= the reference's x1..x5, src/unet.py:34-38)."""
    taps = {}
    x = _cbr(p, prefix + "0.0.", prefix + "0.1.", x, training, stride=2, pad=1)
    idx, cin = 1, 32
    for t, c, n, s in MBV2_SETTING:
        for i in range(n):
            stride = s if i == 0 else 1
            pre = f"{prefix}{idx}.conv."
            hidden = int(round(cin * t))
            h, j = x, 0
            if t != 1:
                h = _cbr(p, pre + "0.0.", pre + "0.1.", h, training)
                j = 1
            h = _cbr(p, f"{pre}{j}.0.", f"{pre}{j}.1.", h, training, stride=stride, pad=1, groups=hidden)
            h = _cbr(p, f"{pre}{j + 1}.", f"{pre}{j + 2}.", h, training, act=None)
            x = x + h if (stride == 1 and cin == c) else h
            cin = c
            if idx in (1, 3, 6, 10):
                taps[idx] = x
            idx += 1
    x = _cbr(p, prefix + "18.0.", prefix + "18.1.", x, training)
    taps[18] = x
    return taps


def double_conv(p, pre, x, training):
    x = _cbr(p, pre + "conv.0.", pre + "conv.1.", x, training, pad=1, act="relu")
    return _cbr(p, pre + "conv.3.", pre + "conv.4.", x, training, pad=1, act="relu")


RECORD = None  # diagnostics: set to a dict to keep (and retain grads of) intermediates


def _rec(name, t):
    if RECORD is not None:
        if t.requires_grad:
            t.retain_grad()
        RECORD[name] = t
    return t


def up(p, pre, x1, x2, training):
    _rec(pre + "low", x1)
    x1 = F.interpolate(x1, scale_factor=2, mode="bilinear", align_corners=False)
    return double_conv(p, pre + "conv.", _rec(pre + "cat", torch.cat([x2, x1], dim=1)), training)


def outconv(p, pre, x, training):
    x = _cbr(p, pre + "conv.0.", pre + "conv.1.", x, training, act="relu")
    return F.conv2d(x, p[pre + "conv.3.weight"], p[pre + "conv.3.bias"])


def mobilenet_unet_forward(p, x, training):
    f = mobilenet_features(p, x, training)
    y = up(p, "up1.", f[18], f[10], training)
    y = up(p, "up2.", y, f[6], training)
    y = up(p, "up3.", y, f[3], training)
    y = up(p, "up4.", y, f[1], training)
    y = outconv(p, "outc.", y, training)
    return F.interpolate(y, scale_factor=2, mode="bilinear", align_corners=True)


def unet_forward(p, x, training):
    x1 = double_conv(p, "inc.conv.", x, training)
    x2 = double_conv(p, "down1.mpconv.1.", _pool("down1.", x1), training)
    x3 = double_conv(p, "down2.mpconv.1.", _pool("down2.", x2), training)
    x4 = double_conv(p, "down3.mpconv.1.", _pool("down3.", x3), training)
    y = up(p, "up1.", x4, x3, training)
    y = up(p, "up2.", y, x2, training)
    y = up(p, "up3.", y, x1, training)
    return outconv(p, "sem_out.", y, training)


FORWARDS = {"MobileNetV2UNet": mobilenet_unet_forward, "UNet": unet_forward, "LightUNet": unet_forward}


def canonical_state(state_dict, dtype=torch.float32):
    """Flat name -> tensor dict (aliases dropped: down1..5 of MobileNetV2UNet are
    views of backbone.features), float tensors cast to `dtype`, detached copies."""
    out = {}
    for k, v in state_dict.items():
        if any(k.startswith(f"down{i}.") for i in range(1, 6)) and "mpconv" not in k:
            continue
        t = v.detach().cpu().clone()
        if t.is_floating_point():
            t = t.to(dtype)
        out[k] = t
    return out


def trainable_names(p):
    return [k for k, v in p.items() if v.is_floating_point() and not k.endswith(("running_mean", "running_var"))
            and not k.startswith("backbone.classifier")]


def forward_backward(arch, p, x, y, training=True):
    """Loss, logits and per-parameter grads of CE(model(x), y)."""
    names = trainable_names(p)
    for k in names:
        p[k].requires_grad_(True)
        p[k].grad = None
    logits = FORWARDS[arch](p, x, training)
    loss = F.cross_entropy(logits, y)
    loss.backward()
    grads = {k: p[k].grad.detach().clone() for k in names}
    for k in names:
        p[k].requires_grad_(False)
    return loss.detach(), logits.detach(), grads


def adam_steps(arch, p, batches, lr=1.5e-4, betas=(0.9, 0.999), eps=1e-8):
    """Adam (torch.optim.Adam defaults, main.py:100) training steps; returns losses."""
    names = trainable_names(p)
    state = {k: (torch.zeros_like(p[k]), torch.zeros_like(p[k])) for k in names}
    losses = []
    for step, (x, y) in enumerate(batches, start=1):
        loss, _, grads = forward_backward(arch, p, x, y, True)
        losses.append(float(loss))
        with torch.no_grad():
            for k in names:
                m, v = state[k]
                g = grads[k]
                m.mul_(betas[0]).add_(g, alpha=1 - betas[0])
                v.mul_(betas[1]).addcmul_(g, g, value=1 - betas[1])
                bc1 = 1 - betas[0] ** step
                bc2 = 1 - betas[1] ** step
                denom = (v.sqrt() / (bc2 ** 0.5)).add_(eps)
                p[k].addcdiv_(m, denom, value=-lr / bc1)
    return losses


def miou(pred, target, classes):
    """Mean IoU over classes with a non-empty union (the build's definition;
    the reference has no metric code)."""
    pred = pred.reshape(-1).long()
    target = target.reshape(-1).long()
    cm = torch.bincount(target * classes + pred, minlength=classes * classes).reshape(classes, classes).double()
    tp = cm.diag()
    union = cm.sum(0) + cm.sum(1) - tp
    valid = union > 0
    return float((tp[valid] / union[valid]).mean()) if valid.any() else float("nan")


# ---------------------------------------------------------------- bf16 conv math
# The bf16 configurations (BASELINE configs[2]/[4]) have no code in the reference;
# their reference arithmetic is torch.autocast(dtype=torch.bfloat16) around the
# forward, whose convolutions (groups == 1: the dense 3x3 and the 1x1 convs; the
# depthwise convs stay in the product's fp32) take bf16 operands and accumulate in
# fp32.  `bf16_convs()` restates that on this oracle: inside it every non-grouped
# conv rounds its input and weight to bf16 (RNE) in the forward and its incoming
# gradient in the backward, then runs in the oracle's own precision (fp64 gives
# "exact products of bf16 operands").  Used only to size the bf16 tolerance budget
# (tests/test_gpu_bf16.py), like the fp32 ensemble does for the fp32 path.
class _Round(torch.autograd.Function):
    @staticmethod
    def forward(ctx, t, dtype):
        ctx.dtype = dtype
        return t.to(dtype).to(t.dtype)

    @staticmethod
    def backward(ctx, g):
        return g.to(ctx.dtype).to(g.dtype), None


class _F:
    def __init__(self, dtype):
        self.dtype = dtype

    def conv2d(self, x, w, b=None, stride=1, padding=0, dilation=1, groups=1):
        if groups == 1:
            x, w = _Round.apply(x, self.dtype), _Round.apply(w, self.dtype)
        return torch.nn.functional.conv2d(x, w, b, stride, padding, dilation, groups)

    def __getattr__(self, k):
        return getattr(torch.nn.functional, k)


class bf16_convs:
    """Context manager: this module's convolutions use bf16 operands (see above);
    dtype=torch.float16 gives the fp16 inference configuration (BASELINE configs[3])."""

    def __init__(self, dtype=torch.bfloat16):
        self.dtype = dtype

    def __enter__(self):
        global F
        self._saved, F = F, _F(self.dtype)
        return self

    def __exit__(self, *exc):
        global F
        F = self._saved
        return False
