"""CPU: seg_amd.Adam host logic -- the SegAdamTensor table layout it packs for
seg_adam_step (include/segamd.h) and its refusal of configurations the HIP step does
not implement (no silent fallback).  The step itself: tests/test_gpu_adam.py."""
import ctypes

import pytest
import torch

from seg_amd import Adam
from seg_amd.optim import _pack


class SegAdamTensor(ctypes.Structure):  # include/segamd.h
    _fields_ = [("p", ctypes.c_void_p), ("g", ctypes.c_void_p), ("m", ctypes.c_void_p), ("v", ctypes.c_void_p),
                ("n", ctypes.c_long), ("step_size", ctypes.c_float), ("bc2_sqrt", ctypes.c_float)]


def test_table_layout():
    rows = [(0x1000, 0x2000, 0x3000, 0x4000, 7, -1.5e-3, 0.031622776), (16, 32, 48, 64, 1 << 33, -2.0, 1.0)]
    t = _pack(rows)
    assert t.dtype == torch.int64 and t.shape == (2, 6) and t.is_contiguous()
    assert ctypes.sizeof(SegAdamTensor) == 6 * 8
    arr = (SegAdamTensor * 2).from_buffer_copy(t.numpy().tobytes())
    for r, e in zip(rows, arr):
        assert (e.p, e.g, e.m, e.v, e.n) == r[:5]
        assert e.step_size == pytest.approx(r[5], rel=1e-7) and e.bc2_sqrt == pytest.approx(r[6], rel=1e-7)


def test_refuses_unsupported():
    p = torch.nn.Parameter(torch.randn(4))
    p.grad = torch.randn(4)
    with pytest.raises(NotImplementedError):
        Adam([p], lr=1e-3).step()  # CPU tensors: the HIP step only
    for kw in ({"weight_decay": 1e-2}, {"amsgrad": True}, {"maximize": True}):
        with pytest.raises(NotImplementedError):
            Adam([p], lr=1e-3, **kw).step()
    q = torch.nn.Parameter(torch.randn(4))  # no gradient: skipped, nothing to do
    Adam([q], lr=1e-3).step()
    assert len(Adam([q]).state) == 0
