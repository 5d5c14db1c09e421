"""CPU: seg_amd.traceable -- the pure-torch twin for convert.py:21-42's ONNX export and
CPU use (main.py:13-21, BASELINE configs[0]).  Same state_dict keys as the segamd model
(and the reference), forward equal to the oracle (pinned to the reference's fixtures),
traceable by torch.jit.trace; ONNX export itself needs the `onnx` package, which is not
installed here (the test skips that leg then).  The segamd model keeps refusing CPU input."""
import io

import pytest
import torch

from oracle import segref
from seg_amd import LightUNet, MobileNetV2UNet, UNet, deterministic_init, traceable
from seg_amd.detinit import synthetic_batch

CASES = [("MobileNetV2UNet", lambda: MobileNetV2UNet(10), 64, 128),
         ("UNet", lambda: UNet(4, 64), 32, 64),
         ("LightUNet", lambda: LightUNet(), 32, 32)]


@pytest.mark.parametrize("arch,ctor,h,w", CASES)
@pytest.mark.parametrize("training", [False, True])
def test_twin_matches_oracle(arch, ctor, h, w, training):
    m = deterministic_init(ctor(), seed=3, random_running_stats=True).train(training)
    t = traceable(m)
    assert list(t.state_dict().keys()) == list(m.state_dict().keys())
    assert t.training == training
    x, y = synthetic_batch(2, h, w, 10, seed=4)
    p = segref.canonical_state(m.state_dict())
    with torch.no_grad():
        ref = segref.FORWARDS[arch](p, x, training)
        out = t(x)
    assert out.shape == ref.shape
    assert float((out - ref).norm() / ref.norm()) < 1e-5


def test_twin_trains_on_cpu_like_main_py():
    """configs[0]: UNet 4-class 128x256 batch 4 on the CPU through the reference's loop."""
    from torch import nn
    from seg_amd import train_model
    m = traceable(deterministic_init(UNet(4, 64), seed=5))
    x, y = synthetic_batch(4, 128, 256, 4, seed=6)
    opt = torch.optim.Adam(m.parameters(), lr=1.5e-4)
    p = segref.canonical_state(m.state_dict())
    train_model(m, [(x, y)], nn.CrossEntropyLoss(), opt, "cpu", epochs=1, checkpoint_pattern=None, progress=False)
    losses = segref.adam_steps("UNet", p, [(x, y)])
    after = segref.canonical_state(m.state_dict())
    k = "up3.conv.conv.3.weight"
    assert float((after[k] - p[k]).norm() / p[k].norm()) < 1e-4, "one Adam step must match the oracle's"
    assert losses


def test_jit_trace_and_onnx_export():
    m = deterministic_init(MobileNetV2UNet(10), seed=1, random_running_stats=True).eval()
    t = traceable(m)
    x = torch.randn(1, 3, 128, 256, generator=torch.Generator().manual_seed(0))   # convert.py:26
    with torch.no_grad():
        ref = t(x)
        tr = torch.jit.trace(t, x)
        assert torch.equal(tr(x), ref)
        x2 = torch.randn(2, 3, 128, 256)  # dynamic batch (convert.py:38-41)
        assert torch.allclose(tr(x2), t(x2))
    pytest.importorskip("onnx")
    f = io.BytesIO()
    torch.onnx.export(t, x, f, export_params=True, opset_version=12, do_constant_folding=True,
                      input_names=["input"], output_names=["output"],
                      dynamic_axes={"input": {0: "batch_size"}, "output": {0: "batch_size"}}, dynamo=False)
    assert len(f.getvalue()) > 1 << 20


def test_segamd_model_on_cpu_runs_the_reference_composition():
    """main.py:13-21's CPU device: the segamd model itself runs the torch composition on
    its own parameters (configs[0]); same logits as its traceable twin, and gradients
    reach the model's own parameters."""
    m = deterministic_init(MobileNetV2UNet(10), seed=2).train()
    x = torch.randn(2, 3, 64, 64, generator=torch.Generator().manual_seed(0))
    out = m(x)
    twin = traceable(m)
    assert torch.equal(out, twin(x))
    out.sum().backward()
    assert m.up1.conv.conv[0].weight.grad is not None
