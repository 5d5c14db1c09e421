"""Counter-based deterministic initialisation keyed by state_dict name.

Parity runs need identical weights in the reference (CPU), the oracle and the
HIP path without shipping a 31 MB checkpoint.  Every tensor is
drawn from numpy's PCG64 seeded with (seed, crc32(name)), so the values depend
only on the parameter's name and shape -- not on torch's RNG, module creation
order or device.  Scales follow the usual He init so activations stay O(1);
BN affine parameters and (optionally) running statistics are perturbed away
from 1/0 so that scale/shift mix-ups cannot cancel out in tests.
"""
from __future__ import annotations

import zlib

import numpy as np
import torch


def _rng(seed: int, name: str) -> np.random.Generator:
    return np.random.Generator(np.random.PCG64([seed, zlib.crc32(name.encode())]))


def tensor_for(name: str, shape, seed: int = 0, random_running_stats: bool = False) -> np.ndarray | None:
    """Deterministic value of the state_dict entry `name` (None = leave as is)."""
    g = _rng(seed, name)
    leaf = name.rsplit(".", 1)[-1]
    shape = tuple(shape)
    if leaf == "num_batches_tracked":
        return None
    if leaf == "running_mean":
        return (0.1 * g.standard_normal(shape)).astype(np.float32) if random_running_stats else np.zeros(shape, np.float32)
    if leaf == "running_var":
        return g.uniform(0.5, 1.5, shape).astype(np.float32) if random_running_stats else np.ones(shape, np.float32)
    if leaf == "weight" and len(shape) == 4:   # conv
        fan_in = shape[1] * shape[2] * shape[3]
        return (g.standard_normal(shape) * np.sqrt(2.0 / fan_in)).astype(np.float32)
    if leaf == "weight" and len(shape) == 2:   # linear (unused classifier)
        return (0.01 * g.standard_normal(shape)).astype(np.float32)
    if leaf == "weight" and len(shape) == 1:   # BN gamma
        return g.uniform(0.8, 1.2, shape).astype(np.float32)
    if leaf == "bias":
        return g.uniform(-0.1, 0.1, shape).astype(np.float32)
    raise KeyError(f"no deterministic init rule for {name} {shape}")


@torch.no_grad()
def deterministic_init(module: torch.nn.Module, seed: int = 0, random_running_stats: bool = False):
    """Overwrite every parameter and BN buffer of `module` in place."""
    seen = set()
    for name, t in list(module.named_parameters()) + list(module.named_buffers()):
        if id(t) in seen:
            continue
        seen.add(id(t))
        v = tensor_for(name, t.shape, seed, random_running_stats)
        if v is not None:
            t.copy_(torch.from_numpy(v).to(t.dtype))
    return module


def synthetic_batch(n: int, h: int, w: int, classes: int, seed: int = 0):
    """x ~ N(0,1) float32 [n,3,h,w] (the post-Normalize distribution,
    src/BDD100KDataset.py:44) and int64 labels in [0, classes) [n,h,w]."""
    g = np.random.Generator(np.random.PCG64(seed))
    x = g.standard_normal((n, 3, h, w)).astype(np.float32)
    y = g.integers(0, classes, (n, h, w)).astype(np.int64)
    return torch.from_numpy(x), torch.from_numpy(y)


# ImageNet normalisation of the readers (src/BDD100KDataset.py:44, inference.py:37-40)
IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def _palette(classes: int) -> np.ndarray:
    """Fixed, well-separated RGB colour per class in [0.1, 0.9]."""
    g = np.random.Generator(np.random.PCG64(12345))
    return g.uniform(0.1, 0.9, (classes, 3))


def synthetic_scene(n: int, h: int, w: int, classes: int, seed: int = 0, noise: float = 0.1):
    """A LEARNABLE synthetic road scene (SURVEY 8(d)'s mIoU workload; no dataset offline):
    piecewise-constant class regions shaped like BDD100K frames -- sky / background /
    road bands split at a random horizon, a few lane strips converging to a vanishing
    point, and random convex blobs (vehicles, signs) -- each class painted with a fixed
    colour plus N(0, noise) pixel noise, then ImageNet-normalised like the readers
    (src/BDD100KDataset.py:38-52).  Returns x float32 [n,3,h,w], y int64 [n,h,w] with
    labels in [0, classes)."""
    if classes < 4:
        raise ValueError("synthetic_scene needs >= 4 classes")
    g = np.random.Generator(np.random.PCG64([seed, 0x5CE4E]))
    rows = np.arange(h, dtype=np.float64)[:, None] + 0.5
    cols = np.arange(w, dtype=np.float64)[None, :] + 0.5
    y = np.empty((n, h, w), np.int64)
    for i in range(n):
        lab = np.empty((h, w), np.int64)
        horizon = h * g.uniform(0.3, 0.5)
        lab[:] = 0                                                   # sky
        lab[(rows > horizon * 0.7).repeat(w, 1)] = 1                 # buildings / background
        lab[(rows > horizon).repeat(w, 1)] = 2                       # road
        vx = w * g.uniform(0.35, 0.65)                               # vanishing point
        for _ in range(g.integers(2, 5)):                            # lane strips (class 3)
            xb = w * g.uniform(-0.2, 1.2)
            t = (rows - horizon) / max(h - horizon, 1.0)
            xc = vx + (xb - vx) * t
            half = np.maximum(0.6, 0.012 * w * t)
            lab[(rows > horizon) & (np.abs(cols - xc) < half)] = 3
        for _ in range(g.integers(3, 9)):                            # convex blobs, classes 4..C-1
            c = int(g.integers(4, classes)) if classes > 4 else 3
            cy, cx = g.uniform(horizon * 0.8, h), g.uniform(0, w)
            k = int(g.integers(3, 7))
            ang = np.sort(g.uniform(0, 2 * np.pi, k))
            rad = g.uniform(0.06, 0.2) * min(h, w) * g.uniform(0.6, 1.4, k) * (0.4 + cy / h)
            px, py = cx + rad * np.cos(ang), cy + rad * np.sin(ang)
            inside = np.ones((h, w), bool)
            for j in range(k):                                       # half-plane test per edge
                x0, y0, x1, y1 = px[j], py[j], px[(j + 1) % k], py[(j + 1) % k]
                inside &= (x1 - x0) * (rows - y0) - (y1 - y0) * (cols - x0) >= 0
            lab[inside] = c
        y[i] = lab
    rgb = _palette(classes)[y]                                       # [n,h,w,3]
    rgb = rgb + noise * g.standard_normal(rgb.shape)
    mean, std = np.array(IMAGENET_MEAN), np.array(IMAGENET_STD)
    x = ((rgb - mean) / std).transpose(0, 3, 1, 2).astype(np.float32)
    return torch.from_numpy(np.ascontiguousarray(x)), torch.from_numpy(y)


def miou(pred: torch.Tensor, target: torch.Tensor, classes: int) -> float:
    """Mean IoU over the classes with a non-empty union (confusion matrix of argmax
    predictions vs labels; IoU_c = TP / (TP + FP + FN)).  The reference has no metric
    code (src/train.py:46-76 is commented out); this is the definition SURVEY 8(d) fixes."""
    pred = pred.reshape(-1).long().cpu()
    target = target.reshape(-1).long().cpu()
    cm = torch.bincount(target * classes + pred, minlength=classes * classes).reshape(classes, classes).double()
    tp = cm.diag()
    union = cm.sum(0) + cm.sum(1) - tp
    valid = union > 0
    return float((tp[valid] / union[valid]).mean()) if valid.any() else float("nan")
