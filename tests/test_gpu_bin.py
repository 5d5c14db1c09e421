"""GPU: a depthwise conv's BatchNorm backward formed on load by its data and weight gradients (round 5, "BIN",
seg_dw_dgrad_bin / seg_dw_wgrad_bin, include/segamd.h) against the apply pass followed by the plain gradients.

dY = seg_bn_bwd_apply(dA, y; coefficients) is computed by the gradient kernels from dA and the conv's pre-BN output
on every load, rounded to the storage type as the apply pass stores it, so the data gradient and the weight-gradient
partials must be bitwise those of the two-pass path; a training step with BIN on equals the step with it off, bit
for bit (torchvision InvertedResidual's depthwise conv + BatchNorm + ReLU6, reached through src/unet.py:15-19)."""
import pytest
import torch

from seg_amd._lib import call, query

pytestmark = pytest.mark.gpu
DEV = "cuda"
BF = torch.bfloat16


def S():
    return torch.cuda.current_stream().cuda_stream


@pytest.mark.parametrize("math", ["f32", "bf16io"])
@pytest.mark.parametrize("N,H,W,C,stride,act", [(2, 16, 24, 96, 1, 2), (2, 17, 33, 144, 2, 2), (1, 8, 16, 384, 1, 0),
                                                (3, 12, 20, 32, 2, 1)])
@pytest.mark.parametrize("lazy", [False, True])
def test_dw_bin_equals_apply_then_gradients(math, N, H, W, C, stride, act, lazy):
    s = S()
    dt = BF if math == "bf16io" else torch.float32
    sfx = "_bf16io" if math == "bf16io" else ""
    g = torch.Generator().manual_seed(N * 131 + C + stride)
    Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
    Mo, Mi = N * Ho * Wo, N * H * W
    y = (torch.randn(Mo, C, generator=g) * 1.3 + 0.2).to(dt).to(DEV)
    da = torch.randn(Mo, C, generator=g).to(dt).to(DEV)
    x = torch.randn(Mi, C, generator=g).to(dt).to(DEV)
    mean = y.float().mean(0)
    invstd = 1.0 / (y.float().var(0, unbiased=False) + 1e-5).sqrt()
    gamma = (torch.rand(C, generator=g) + 0.5).to(DEV)
    beta = torch.randn(C, generator=g).to(DEV)
    scale, shift = gamma * invstd, beta - mean * gamma * invstd
    isc = (torch.rand(C, generator=g) + 0.5).to(DEV) if lazy else None
    ish = torch.randn(C, generator=g).to(DEV) if lazy else None
    xf = (isc.data_ptr(), ish.data_ptr(), 2) if lazy else (None, None, 0)
    wk = (torch.randn(9 * C, generator=g) * 0.2).to(DEV)
    coef = torch.empty(3 * C, device=DEV)
    dgam, dbet = torch.empty(C, device=DEV), torch.empty(C, device=DEV)
    work = torch.empty(query("seg_chan_workspace_floats", Mo, C), device=DEV)
    call("seg_bn_bwd_coef" + sfx, da.data_ptr(), C, y.data_ptr(), C, Mo, C, gamma.data_ptr(), mean.data_ptr(),
         invstd.data_ptr(), scale.data_ptr(), shift.data_ptr(), act, dgam.data_ptr(), dbet.data_ptr(), work.data_ptr(),
         coef.data_ptr(), s)
    # reference: the apply pass, then the plain gradients
    dy = torch.empty(Mo, C, device=DEV, dtype=dt)
    call("seg_bn_bwd_apply" + sfx, da.data_ptr(), C, y.data_ptr(), C, Mo, C, mean.data_ptr(), scale.data_ptr(),
         shift.data_ptr(), act, coef.data_ptr(), dy.data_ptr(), C, s)
    nblk = query("seg_dw_wgrad_blocks", N, Ho, Wo, C)
    outs = {}
    for tag in ("ref", "bin"):
        dx = torch.full((Mi, C), 0.25, device=DEV, dtype=dt)  # accumulate onto a known value
        part = torch.full((nblk * 9 * C,), float("nan"), device=DEV)
        if tag == "ref":
            call("seg_dw_dgrad" + sfx, dy.data_ptr(), C, N, Ho, Wo, C, wk.data_ptr(), dx.data_ptr(), C, H, W, stride, 1,
                 s)
            call("seg_dw_wgrad" + sfx, dy.data_ptr(), C, x.data_ptr(), C, N, H, W, C, *xf, Ho, Wo, stride,
                 part.data_ptr(), s)
        else:
            b = (y.data_ptr(), C, mean.data_ptr(), scale.data_ptr(), shift.data_ptr(), act, coef.data_ptr())
            call("seg_dw_dgrad_bin" + sfx, da.data_ptr(), C, N, Ho, Wo, C, wk.data_ptr(), dx.data_ptr(), C, H, W,
                 stride, 1, *b, s)
            call("seg_dw_wgrad_bin" + sfx, da.data_ptr(), C, x.data_ptr(), C, N, H, W, C, *xf, Ho, Wo, stride,
                 part.data_ptr(), *b, s)
        outs[tag] = (dx, part)
    torch.cuda.synchronize()
    assert torch.isfinite(outs["ref"][1]).all()
    assert torch.equal(outs["ref"][0], outs["bin"][0])
    assert torch.equal(outs["ref"][1], outs["bin"][1])


@pytest.mark.parametrize("math", ["f32", "bf16io"])
def test_bin_model_step_bitwise(math, monkeypatch):
    """MobileNetV2UNet training step with every depthwise BN backward formed on load (engine.BIN_DW) equals the step
    with the apply pass: loss, every gradient, BN running statistics, bit for bit."""
    from seg_amd import MobileNetV2UNet, engine
    from seg_amd.detinit import deterministic_init, synthetic_batch
    x, t = synthetic_batch(2, 64, 128, 10, seed=23)
    x, t = x.to(DEV), t.to(DEV)
    res = {}
    for on in (False, True):
        monkeypatch.setattr(engine, "BIN_DW", on)
        model = deterministic_init(MobileNetV2UNet(10), seed=23).to(DEV).train()
        engine.set_conv_math(model, math)
        loss = model.forward_loss(x, t)
        loss.backward()
        torch.cuda.synchronize()
        res[on] = (loss.detach().clone(), {k: p.grad.clone() for k, p in model.named_parameters() if p.grad is not None},
                   {k: b.clone() for k, b in model.named_buffers()})
    (l0, g0, b0), (l1, g1, b1) = res[False], res[True]
    assert torch.equal(l0, l1)
    assert set(g0) == set(g1) and len(g0) == 194
    for k in g0:
        assert torch.equal(g0[k], g1[k]), k
    for k in b0:
        assert torch.equal(b0[k], b1[k]), k
