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
