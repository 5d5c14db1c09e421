"""GPU: the full vanilla UNet (src/unet.py:124-147) at BASELINE configs[4]'s shape --
10 classes, 512x1024, bs=8/GPU, bf16 (here: the bf16io configuration) -- and an
oracle-checked slice that selects the same kernel kinds.

  * mid-size slice (2x128x256, f32): the Winograd forward / data-gradient, LDS-halo and
    implicit-GEMM choices per layer equal the full-size ones (tools: engine picks), and
    logits / loss / every gradient pass the oracle budget of tests/test_gpu_model.py;
  * full size (8x512x1024; bf16io and f32): finite, bitwise reproducible step to step
    (fixed-order reductions), the fused upsample+CE loss equals nn.CrossEntropyLoss on
    the model's logits, and the max-pool / concat / upsample launches at this size run.
"""
import pytest
import torch
from torch import nn

from oracle import budget, segref
from seg_amd import UNet, engine
from seg_amd.detinit import deterministic_init, synthetic_batch
from seg_amd.engine import query, r4

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _kinds(N, H, W, math):
    prog = engine.build_program(UNet(10), N, H, W, math)
    out = []
    for op in prog.ops:
        if isinstance(op, engine.ConvOp) and op.ks == 3:
            y = op.y
            wf = math == "f32" and bool(query("seg_conv_wino_pick", y.N, y.H, y.W, op.cin_pad, op.cout))
            wd = math == "f32" and not op.first and bool(query("seg_conv_wino_pick", y.N, y.H, y.W, r4(op.cout),
                                                                op.cin))
            hf = not wf and bool(query("seg_conv_halo_pick", y.N, y.H, y.W, op.cin_pad, op.cout))
            hd = not op.first and not wd and bool(query("seg_conv_halo_pick", y.N, y.H, y.W, r4(op.cout), op.cin))
            out.append(("wino" if wf else "halo" if hf else "igemm", "wino" if wd else "halo" if hd else "igemm"))
    return out


def test_mid_size_slice_selects_full_size_kernels():
    assert _kinds(2, 128, 256, "f32") == _kinds(8, 512, 1024, "f32")


def test_unet_mid_size_parity_vs_oracle():
    x, y = synthetic_batch(2, 128, 256, 10, seed=31)
    model_cpu = deterministic_init(UNet(10), seed=31)
    model = deterministic_init(UNet(10), seed=31).to(DEV).train()
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
    assert rel < 1e-3, rel
    grads = {k: p.grad for k, p in model.named_parameters() if p.grad is not None}
    rep = budget.check_hip("UNet", segref.canonical_state(model_cpu.state_dict()), x, y, grads, z)
    print(f"UNet 2x128x256 f32: logits rel {rel:.2e}, worst grad {rep['worst']:.3f} of budget "
          f"({rep['worst_name']}), z {rep['z_worst']:.3f} of bound, {rep['n_flips']} mask flips")
    assert abs(loss.item() - rep["loss64"]) <= 1e-4 * abs(rep["loss64"])
    assert not rep["z_bad"] and not rep["missing_layers"], (rep["z_bad"][:3], rep["missing_layers"])
    assert not rep["bad"], rep["bad"][:8]


@pytest.mark.parametrize("math", ["bf16io", "f32"])
def test_unet_cfg5_full_size_properties(math):
    model = deterministic_init(UNet(10), seed=41).to(DEV).train()
    engine.set_conv_math(model, math)
    x, y = synthetic_batch(8, 512, 1024, 10, seed=41)
    x, y = x.to(DEV), y.to(DEV)
    outs = []
    for _ in range(2):
        model.zero_grad(set_to_none=True)
        loss = model.forward_loss(x, y)
        loss.backward()
        outs.append((loss.detach().clone(), {k: p.grad.clone() for k, p in model.named_parameters()
                                              if p.grad is not None}))
    (l0, g0), (l1, g1) = outs
    assert torch.isfinite(l0)
    assert torch.equal(l0, l1), "fixed-order reductions must be bitwise reproducible"
    assert len(g0) == len(list(model.parameters()))
    for k in g0:
        assert torch.equal(g0[k], g1[k]), k
        assert torch.isfinite(g0[k]).all(), k
    with torch.no_grad():
        logits = model(x)
        assert logits.shape == (8, 10, 512, 1024)
        l2 = nn.CrossEntropyLoss()(logits, y)
    assert abs(l2.item() - l0.item()) <= 1e-5 * abs(l0.item()), (l2.item(), l0.item())
