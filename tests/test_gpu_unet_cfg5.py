"""GPU: the full vanilla UNet (src/unet.py:124-147) at BASELINE configs[4]'s shape --
10 classes, 512x1024, bs=8/GPU, bf16 (here: the bf16io configuration) -- and an
oracle-checked slice that selects the same kernel kinds.

  * mid-size slice (2x128x256, f32): the Winograd forward / data-gradient, LDS-halo and
    implicit-GEMM choices per layer equal the full-size ones (tools: engine picks), and
    logits / loss / every gradient pass the oracle budget of tests/test_gpu_model.py --
    with all Winograd transforms, with each group of them off and without Winograd, worst
    tensor recorded for each;
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


def _slice_run(x, y, state, side, fwd, dgrad, wgrad):
    """One f32 training step of the 2x128x256 slice with each Winograd transform on or off
    (fwd: F(2x2,3x3) forward, dgrad: F(2x2,3x3) data gradient, wgrad: F(3x3,2x2) weight
    gradient); returns the logits, loss, the oracle budget report (oracle side shared
    between the runs) and the Winograd launches per step."""
    saved = engine.WINOGRAD_FWD, engine.WINOGRAD_DGRAD, engine.WINOGRAD_WGRAD
    engine.WINOGRAD_FWD, engine.WINOGRAD_DGRAD, engine.WINOGRAD_WGRAD = fwd, dgrad, wgrad
    engine.DEBUG_KEEP_RUN = True
    try:
        model = deterministic_init(UNet(10), seed=31).to(DEV).train()
        logits = model(x.to(DEV))
        loss = nn.CrossEntropyLoss()(logits, y.to(DEV))
        loss.backward()
        torch.cuda.synchronize()
        z = engine.debug_preactivations(model)
        pools = engine.debug_pool_positions(model)
        prog = engine.get_program(model, *x.shape[:1], *x.shape[2:])
        n_wino = sum(op.wino_f + op.wino_d + bool(op.wino_w) for op in prog.ops if isinstance(op, engine.ConvOp))
    finally:
        engine.DEBUG_KEEP_RUN, engine.LAST_RUN = False, None
        engine.WINOGRAD_FWD, engine.WINOGRAD_DGRAD, engine.WINOGRAD_WGRAD = saved
    grads = {k: p.grad for k, p in model.named_parameters() if p.grad is not None}
    rep = budget.check_hip("UNet", state, x, y, grads, z, side=side, hip_pools=pools)
    return logits.detach().double().cpu(), loss.item(), rep, n_wino


# (tag, forward, data gradient, weight gradient) Winograd transforms on
SLICE_VARIANTS = (("winograd", True, True, True), ("winograd_fwd_dgrad_only", True, True, False),
                  ("winograd_fwd_only", True, False, False), ("winograd_dgrad_only", False, True, False),
                  ("no_winograd", False, False, False))


def test_unet_mid_size_parity_vs_oracle(record):
    """The slice against the oracle budget, run with the production kernel choice (Winograd
    F(2x2,3x3) forward / data gradient and F(3x3,2x2) weight gradient on the deep convs) and
    with the transforms switched off one group at a time, down to no Winograd at all (the
    same convs on the LDS-halo / implicit-GEMM kernels, exact fp32 products).  All must pass;
    the worst tensor of each is asserted below 1 and recorded, so the record shows which
    transform -- forward, data gradient or weight gradient -- drives the margin."""
    x, y = synthetic_batch(2, 128, 256, 10, seed=31)
    model_cpu = deterministic_init(UNet(10), seed=31)
    state = segref.canonical_state(model_cpu.state_dict())
    side = budget.oracle_side("UNet", state, x, y)
    p64 = segref.canonical_state(model_cpu.state_dict(), torch.float64)
    with torch.no_grad():
        ref = segref.unet_forward(p64, x.double(), True)
    res = {}
    for tag, fwd, dgrad, wgrad in SLICE_VARIANTS:
        logits, loss, rep, n_wino = _slice_run(x, y, state, side, fwd, dgrad, wgrad)
        rel = float((logits - ref).norm() / ref.norm())
        top = sorted(rep["ratios"].items(), key=lambda kv: -kv[1])[:3]
        print(f"UNet 2x128x256 f32 {tag} ({n_wino} Winograd launches/step): logits rel {rel:.2e}, worst grad "
              f"{rep['worst']:.3f} of budget ({rep['worst_name']}), next {top[1:]}, z {rep['z_worst']:.3f} of "
              f"bound, {rep['n_flips']} mask flips")
        record(kernels=tag, winograd_launches=n_wino, logits_rel=rel, worst=rep["worst"],
               worst_name=rep["worst_name"], top3=top, z_worst=rep["z_worst"], n_flips=rep["n_flips"])
        assert (n_wino > 0) == (fwd or dgrad or wgrad)
        assert rel < 1e-3, rel
        assert abs(loss - rep["loss64"]) <= 1e-4 * abs(rep["loss64"])
        assert not rep["z_bad"] and not rep["missing_layers"], (rep["z_bad"][:3], rep["missing_layers"])
        assert not rep["bad"], rep["bad"][:8]
        assert rep["worst"] < 1.0
        res[tag] = rep
    print("worst of budget: " + ", ".join(f"{t} {res[t]['worst']:.3f} ({res[t]['worst_name']})"
                                          for t, *_ in SLICE_VARIANTS))


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
