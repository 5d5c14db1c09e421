"""CPU: BASELINE configs[0] -- vanilla UNet 4-class, 128x256, batch 4 on the CPU through
main.py's loop (main.py:13-21 selects the CPU when no GPU is present; src/train.py:31-42).

On a CPU device the segamd models run the reference composition in torch ops on their
own parameters (seg_amd/export.py torch_forward, under autograd), so the drop-in
train_model + torch.optim.Adam work unchanged.  One Adam step of UNet(4) at 4x128x256
through train_one_epoch is compared with the oracle's fp32 Adam step (oracle/segref.py)
from the same initial weights and batch: loss within 1e-5 relative, every parameter and
BN running statistic within 1e-3 relative L2 (north_star's fp32 bar), and the next
forward's logits within 1e-3.
"""
import torch
from torch import nn

from oracle import segref
from seg_amd import UNet, deterministic_init, synthetic_batch
from seg_amd.train import train_one_epoch


def _rel(a, b):
    a, b = a.detach().double(), b.detach().double()
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


def test_cfg0_unet4_cpu_adam_step_matches_oracle():
    torch.manual_seed(0)
    x, y = synthetic_batch(4, 128, 256, 4, seed=3)
    model = deterministic_init(UNet(4), seed=3).train()
    p = segref.canonical_state(deterministic_init(UNet(4), seed=3).state_dict())
    opt = torch.optim.Adam(model.parameters(), lr=1.5e-4)
    loss = train_one_epoch(model, [(x, y)], nn.CrossEntropyLoss(), opt, "cpu", progress=False)
    ref_losses = segref.adam_steps("UNet", p, [(x, y)], lr=1.5e-4)
    assert abs(loss - ref_losses[0]) <= 1e-5 * abs(ref_losses[0]), (loss, ref_losses)
    sd = model.state_dict()
    for k, v in p.items():
        if v.is_floating_point():
            assert _rel(sd[k], v) <= 1e-3, (k, _rel(sd[k], v))
        else:
            assert int(sd[k]) == int(v), k
    x2, _ = synthetic_batch(4, 128, 256, 4, seed=4)
    with torch.no_grad():
        got = model(x2)
        ref = segref.unet_forward(p, x2, True)
    assert got.shape == (4, 4, 128, 256)
    assert _rel(got, ref) <= 1e-3


def test_cpu_forward_loss_and_out_of_range_label():
    """forward_loss on the CPU is F.cross_entropy of the composition; an out-of-range
    label raises as nn.CrossEntropyLoss does."""
    model = deterministic_init(UNet(4, 8), seed=1).train()
    x, y = synthetic_batch(2, 32, 64, 4, seed=1)
    a = model.forward_loss(x, y)
    b = nn.CrossEntropyLoss()(model(x), y)
    assert torch.allclose(a, b, rtol=1e-6)
    y[0, 0, 0] = 7
    try:
        model.forward_loss(x, y)
    except (IndexError, RuntimeError):
        pass
    else:
        raise AssertionError("out-of-range label did not raise")
