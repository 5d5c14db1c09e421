"""CPU: the training program's backward schedule decisions that need no GPU (seg_amd/engine.py).

Program.wgrad_defer (round 6): with bf16 storage the decoder's parameter gradients -- every op from the first
upsample (src/unet.py:97-103, the decoder's first `up`) on -- wait until the backward reaches the encoder's last op,
so they run beside the encoder's memory-bound BatchNorm / depthwise backward; fp32 keeps the per-layer fork
(measured: profiles/r06/ab_wgrad_defer.txt).  The deferral only moves launches between streams, never their
arithmetic (tests/test_gpu_bf16io.py checks the gradients with it on).
"""
import pytest

from seg_amd import MobileNetV2UNet, UNet
from seg_amd import engine as E


@pytest.mark.parametrize("model,first_up", [(MobileNetV2UNet, 52), (UNet, 11)])
def test_decoder_deferral_boundary(model, first_up):
    m = model(10)
    prog = E.build_program(m, 2, 64, 128, "bf16io")
    assert isinstance(prog.ops[first_up], E.UpsampleOp)
    assert not any(isinstance(op, E.UpsampleOp) for op in prog.ops[:first_up])
    assert prog.wgrad_defer() == (first_up, first_up - 1)
    assert E.build_program(m, 2, 64, 128, "f32").wgrad_defer() is None


def test_decoder_deferral_switch(monkeypatch):
    prog = E.build_program(MobileNetV2UNet(10), 2, 64, 128, "bf16io")
    monkeypatch.setattr(E, "DEFER_DECODER", False)
    assert prog.wgrad_defer() is None
    monkeypatch.setattr(E, "WGRAD_DEFER", (60, 55))
    assert prog.wgrad_defer() == (60, 55)
