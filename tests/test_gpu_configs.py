"""GPU: BASELINE configurations at their own shapes (VERDICT r2 "configs_untested").

configs[2] -- MobileNetV2UNet 10-class, 256x512, bs=32/GPU, bf16 (main.py:98-103's model
  and loop; the reference's equivalent of bf16 is torch.autocast around the forward).
  At the full per-GPU shape 32x256x512, for bf16 math and for bf16io (bf16 math + bf16
  activation storage):
    * loss and all 194 gradient tensors finite, bitwise reproducible step to step
      (fixed-order reductions);
    * the fused upsample + cross-entropy loss equals nn.CrossEntropyLoss on the model's
      own logits (src/train.py:37), within fp32 summation order;
    * the launch-tape replay equals the immediate program walk bit for bit.
  Its 2x256x512 slice is checked against the emulated-reference oracle budget in
  tests/test_gpu_bf16.py::test_model_bf16_vs_oracle.
configs[0] -- UNet 4-class, 128x256, bs=4 (main.py with UNet(4); the reference runs it on
  the CPU): the HIP f32 path at exactly 4x128x256 against the oracle, logits within 1e-3
  and every gradient inside oracle/budget.py's bound.  (The CPU leg itself --
  train_model on a CPU device -- is tests/test_cpu_train.py.)
"""
import pytest
import torch
from torch import nn

from oracle import budget, segref
from seg_amd import MobileNetV2UNet, UNet, engine
from seg_amd.detinit import deterministic_init, synthetic_batch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _eager_step(model, x, y):
    """The immediate walk (every launch issued on the spot, no tape)."""
    N, _, H, W = x.shape
    run = engine.Run(engine.get_program(model, N, H, W), x.contiguous(), True)
    run.forward()
    stats = engine._loss_forward(run, y, -100)
    engine._loss_backward(run, torch.ones(1, device=DEV), -100)
    grads = {k: run.grads[id(p)].clone() for k, p in model.named_parameters() if id(p) in run.grads}
    return stats[0].clone(), grads


def _tape_step(model, x, y):
    model.zero_grad(set_to_none=True)
    loss = model.forward_loss(x, y)
    loss.backward()
    return loss.detach().clone(), {k: p.grad.clone() for k, p in model.named_parameters() if p.grad is not None}


@pytest.mark.parametrize("math", ["bf16io", "bf16"])
def test_cfg2_bf16_full_size_properties(math, record):
    model = deterministic_init(MobileNetV2UNet(10), seed=23).to(DEV).train()
    engine.set_conv_math(model, math)
    x, y = synthetic_batch(32, 256, 512, 10, seed=23)
    x, y = x.to(DEV), y.to(DEV)
    bufs = {k: b.clone() for k, b in model.named_buffers()}
    steps = [_tape_step(model, x, y) for _ in range(3)]  # record, then two replays
    (l0, g0) = steps[1]
    for l, g in steps[2:]:
        assert torch.equal(l0, l), "fixed-order reductions must be bitwise reproducible"
        assert g.keys() == g0.keys()
        for k in g0:
            assert torch.equal(g0[k], g[k]), k
    assert torch.isfinite(l0)
    assert len(g0) == 194
    for k, t in g0.items():
        assert torch.isfinite(t).all(), k
    # the fused loss against nn.CrossEntropyLoss on the logits (same weights, BN in train mode)
    with torch.no_grad():
        logits = model(x)
        assert logits.shape == (32, 10, 256, 512) and logits.dtype == torch.float32
        l2 = nn.CrossEntropyLoss()(logits, y)
    assert abs(l2.item() - l0.item()) <= 1e-5 * abs(l0.item()), (l2.item(), l0.item())
    # tape == eager, from the same BN running statistics
    for k, b in model.named_buffers():
        b.copy_(bufs[k])
    le, ge = _eager_step(model, x, y)
    for k, b in model.named_buffers():
        b.copy_(bufs[k])
    lt, gt = _tape_step(model, x, y)
    torch.cuda.synchronize()
    assert torch.equal(le, lt), (le.item(), lt.item())
    assert ge.keys() == gt.keys()
    for k in ge:
        assert torch.equal(ge[k], gt[k]), k
    record(math=math, shape=[32, 256, 512], loss=l0.item(), loss_ce_on_logits=l2.item())


def test_cfg0_unet4_128x256_bs4_vs_oracle(record):
    """configs[0]'s workload on the HIP path: UNet(4), base 64, 4x128x256, f32."""
    x, y = synthetic_batch(4, 128, 256, 4, seed=17)
    model_cpu = deterministic_init(UNet(4), seed=17)
    model = deterministic_init(UNet(4), seed=17).to(DEV).train()
    engine.DEBUG_KEEP_RUN = True
    try:
        logits = model(x.to(DEV))
        loss = nn.CrossEntropyLoss()(logits, y.to(DEV))
        loss.backward()
        torch.cuda.synchronize()
        z = engine.debug_preactivations(model)
    finally:
        engine.DEBUG_KEEP_RUN, engine.LAST_RUN = False, None
    p64 = segref.canonical_state(model_cpu.state_dict(), torch.float64)
    with torch.no_grad():
        ref = segref.unet_forward(p64, x.double(), True)
    rel = float((logits.detach().double().cpu() - ref).norm() / ref.norm())
    grads = {k: p.grad for k, p in model.named_parameters() if p.grad is not None}
    rep = budget.check_hip("UNet", segref.canonical_state(model_cpu.state_dict()), x, y, grads, z)
    print(f"UNet(4) 4x128x256 f32: logits rel {rel:.2e}, worst grad {rep['worst']:.3f} of budget "
          f"({rep['worst_name']}), z {rep['z_worst']:.3f} of bound, {rep['n_flips']} mask flips")
    record(logits_rel=rel, worst=rep["worst"], worst_name=rep["worst_name"], z_worst=rep["z_worst"],
           n_flips=rep["n_flips"])
    assert logits.shape == (4, 4, 128, 256)
    assert rel < 1e-3, rel
    assert abs(loss.item() - rep["loss64"]) <= 1e-4 * abs(rep["loss64"])
    assert not rep["z_bad"] and not rep["missing_layers"], (rep["z_bad"][:3], rep["missing_layers"])
    assert not rep["bad"], rep["bad"][:8]
    assert len(grads) == len(list(model.parameters()))
