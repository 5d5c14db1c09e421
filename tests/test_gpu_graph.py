"""GPU: the HIP-graph captured training step (engine.set_step_graphs) against the eager
engine: identical kernels and reduction orders, so losses, gradients and parameters
after several Adam steps must be bitwise equal; gradient accumulation without
set_to_none, shape changes and a second forward before backward keep working."""
import pytest
import torch

from seg_amd import MobileNetV2UNet, UNet, engine
from seg_amd.detinit import deterministic_init, synthetic_batch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _train(ctor, math, graphs, batches, set_to_none=True, steps=None):
    model = deterministic_init(ctor(), seed=4).to(DEV).train()
    engine.set_conv_math(model, math)
    engine.set_step_graphs(model, graphs)
    opt = torch.optim.Adam(model.parameters(), lr=1.5e-3)
    losses = []
    for x, y in batches:
        opt.zero_grad(set_to_none=set_to_none)
        loss = model.forward_loss(x, y)
        loss.backward()
        opt.step()
        losses.append(loss.item())
    torch.cuda.synchronize()
    return losses, model


def _batches(n, N, H, W, seed=0):
    out = []
    for k in range(n):
        x, y = synthetic_batch(N, H, W, 10, seed=seed + k)
        out.append((x.to(DEV), y.to(DEV)))
    return out


@pytest.mark.parametrize("math", ["f32", "bf16io"])
@pytest.mark.parametrize("arch", ["MobileNetV2UNet", "UNet"])
def test_graph_step_bitwise_equals_eager(arch, math):
    ctor = (lambda: MobileNetV2UNet(10)) if arch == "MobileNetV2UNet" else (lambda: UNet(10, 16))
    batches = _batches(6, 2, 64, 64)
    le, me = _train(ctor, math, False, batches)
    lg, mg = _train(ctor, math, True, batches)
    assert le == lg, (le, lg)
    for (k, a), (_, b) in zip(me.state_dict().items(), mg.state_dict().items()):
        assert torch.equal(a, b), k
    assert mg.__dict__["_segamd_step_graphs"], "the step was captured"


def test_graph_accumulate_without_set_to_none():
    ctor = lambda: MobileNetV2UNet(10)  # noqa: E731
    batches = _batches(5, 2, 64, 64, seed=10)
    le, me = _train(ctor, "f32", False, batches, set_to_none=False)
    lg, mg = _train(ctor, "f32", True, batches, set_to_none=False)
    assert le == lg
    for (k, a), (_, b) in zip(me.state_dict().items(), mg.state_dict().items()):
        assert torch.equal(a, b), k


def test_graph_shape_change_and_double_forward():
    model = deterministic_init(MobileNetV2UNet(10), seed=4).to(DEV).train()
    ref = deterministic_init(MobileNetV2UNet(10), seed=4).to(DEV).train()
    engine.set_step_graphs(model, True)
    for shape in ((2, 64, 64), (2, 64, 64), (2, 64, 64), (1, 64, 128), (2, 64, 64), (1, 64, 128), (1, 64, 128),
                  (1, 64, 128)):
        x, y = synthetic_batch(*shape, 10, seed=sum(shape))
        x, y = x.to(DEV), y.to(DEV)
        a = model.forward_loss(x, y)
        b = model.forward_loss(x, y)  # second forward while the first awaits backward: eager
        (a + b).backward()
        c = ref.forward_loss(x, y)
        d = ref.forward_loss(x, y)
        (c + d).backward()
        assert a.item() == c.item() and b.item() == d.item()
        for p, q in zip(model.parameters(), ref.parameters()):
            if q.grad is not None:
                assert torch.equal(p.grad, q.grad)
        model.zero_grad(set_to_none=True)
        ref.zero_grad(set_to_none=True)
