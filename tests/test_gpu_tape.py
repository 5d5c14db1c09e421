"""GPU: the launch tape (csrc/tape.hip, seg_amd/tape.py, engine.Plan).  A training step
replayed from the recorded tapes must equal the immediate program walk (every launch a
ctypes call, the round-1 engine) bit for bit -- same kernels, same streams, same
reduction orders -- step after step with fresh input tensors, with the side stream on
and off, through the logits and the fused-loss modes, and when a second forward runs
before the first one's backward (a one-off plan keeps the first activations)."""
import pytest
import torch
from torch import nn

from seg_amd import MobileNetV2UNet, UNet, engine
from seg_amd.detinit import deterministic_init, synthetic_batch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def eager_step(model, x, y):
    """The immediate walk: Run without a recorder, every launch issued on the spot."""
    N, _, H, W = x.shape
    prog = engine.get_program(model, N, H, W)
    run = engine.Run(prog, x.contiguous(), True)
    run.forward()
    stats = engine._loss_forward(run, y, -100)
    engine._loss_backward(run, torch.ones(1, device=DEV), -100)
    grads = {k: run.grads[id(p)].clone() for k, p in model.named_parameters() if id(p) in run.grads}
    return stats[0].clone(), grads


def tape_step(model, x, y):
    model.zero_grad(set_to_none=True)
    loss = model.forward_loss(x, y)
    loss.backward()
    return loss.detach(), {k: p.grad.clone() for k, p in model.named_parameters() if p.grad is not None}


@pytest.mark.parametrize("overlap", [True, False])
@pytest.mark.parametrize("math", ["f32", "bf16io"])
def test_tape_replay_equals_immediate_walk(overlap, math):
    saved = engine.OVERLAP
    engine.OVERLAP = overlap
    try:
        model = deterministic_init(MobileNetV2UNet(10), seed=2).to(DEV).train()
        engine.set_conv_math(model, math)
        for step in range(3):  # record, then two replays with new input tensors
            x, y = synthetic_batch(2, 64, 128, 10, seed=50 + step)
            x, y = x.to(DEV), y.to(DEV)
            # same BN running-statistics state for both: snapshot, eager, restore, tape
            bufs = {k: b.clone() for k, b in model.named_buffers()}
            le, ge = eager_step(model, x, y)
            for k, b in model.named_buffers():
                b.copy_(bufs[k])
            lt, gt = tape_step(model, x, y)
            torch.cuda.synchronize()
            assert torch.equal(le, lt), (step, le.item(), lt.item())
            assert ge.keys() == gt.keys() and len(gt) == 194
            for k in ge:
                assert torch.equal(ge[k], gt[k]), (step, k)
    finally:
        engine.OVERLAP = saved


def test_logits_mode_and_second_forward_before_backward():
    model = deterministic_init(UNet(4, 16), seed=3).to(DEV).train()
    x1, y1 = synthetic_batch(2, 32, 64, 4, seed=1)
    x2, y2 = synthetic_batch(2, 32, 64, 4, seed=2)
    x1, y1, x2, y2 = x1.to(DEV), y1.to(DEV), x2.to(DEV), y2.to(DEV)
    crit = nn.CrossEntropyLoss()
    ref = []
    for x, y in ((x1, y1), (x2, y2)):
        model.zero_grad(set_to_none=True)
        bufs = {k: b.clone() for k, b in model.named_buffers()}
        crit(model(x), y).backward()
        ref.append({k: p.grad.clone() for k, p in model.named_parameters()})
        for k, b in model.named_buffers():
            b.copy_(bufs[k])
    # both forwards first, then both backwards: the second forward must not clobber the first
    model.zero_grad(set_to_none=True)
    l1 = crit(model(x1), y1)
    l2 = crit(model(x2), y2)
    l1.backward()
    g1 = {k: p.grad.clone() for k, p in model.named_parameters()}
    model.zero_grad(set_to_none=True)
    l2.backward()
    g2 = {k: p.grad.clone() for k, p in model.named_parameters()}
    for k in g1:
        assert torch.equal(g1[k], ref[0][k]), k
        assert torch.equal(g2[k], ref[1][k]), k


def test_kernel_timer_reads_tape_launches():
    model = deterministic_init(MobileNetV2UNet(10), seed=4).to(DEV).train()
    x, y = synthetic_batch(2, 64, 128, 10, seed=4)
    x, y = x.to(DEV), y.to(DEV)
    tape_step(model, x, y)  # record
    timer = engine.KernelTimer(kinds={"igemm3_fwd", "igemm3_dgrad", "wino3_fwd", "wino3_dgrad"})
    engine.TIMER = timer
    try:
        for _ in range(3):
            tape_step(model, x, y)
        torch.cuda.synchronize()
    finally:
        engine.TIMER = None
    rec = timer.elapsed()
    # per step: the 8 decoder 3x3 convs forward + data gradient and the stem forward
    assert len(rec) == 3 * 17, len(rec)
    assert all(s > 0 for _, _, s in rec)


def test_rebound_parameters_rerecord_the_tape():
    """the tapes hold raw parameter / BN-buffer pointers, so rebinding them
    (load_state_dict(assign=True)) must re-record instead of replaying into freed memory.
    After the rebind the step equals a fresh model's with the same state, bit for bit;
    the plan cache stays bounded (engine.MAX_PLANS) and release_plans() empties it."""
    x, y = synthetic_batch(2, 64, 128, 10, seed=61)
    x, y = x.to(DEV), y.to(DEV)
    model = deterministic_init(MobileNetV2UNet(10), seed=5).to(DEV).train()
    tape_step(model, x, y)
    tape_step(model, x, y)
    other = deterministic_init(MobileNetV2UNet(10), seed=6).to(DEV).train()
    sd = {k: v.clone() for k, v in other.state_dict().items()}
    model.load_state_dict({k: v.clone() for k, v in sd.items()}, assign=True)
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    l1, g1 = tape_step(model, x, y)
    fresh = deterministic_init(MobileNetV2UNet(10), seed=6).to(DEV).train()
    fresh.load_state_dict(sd)
    l2, g2 = tape_step(fresh, x, y)
    assert torch.equal(l1, l2)
    for k in g2:
        assert torch.equal(g1[k], g2[k]), k
    for hw in ((64, 64), (32, 64), (64, 96), (96, 64), (32, 32), (64, 128)):
        xs, ys = synthetic_batch(1, *hw, 10, seed=1)
        tape_step(model, xs.to(DEV), ys.to(DEV))
    assert len(model.__dict__["_segamd_plans"]) <= engine.MAX_PLANS
    engine.release_plans(model)
    assert "_segamd_plans" not in model.__dict__
    l3, g3 = tape_step(model, x, y)
    assert torch.isfinite(l3)
