"""GPU: lazy BatchNorm for 1x1 and 3x3 consumers -- seg_conv_igemm*_xf / seg_conv_halo*_xf /
seg_conv_wgrad*_xf (include/segamd.h) against a separate BN-apply pass followed by the plain conv.

The _xf kernels form x = act(y * scale + shift) (seg_bn_act4, the helper seg_bn_apply
uses) while staging the input operand, and round it to bf16 where the apply pass would
store bf16, so outputs, BN partial statistics and weight-gradient partials must be
bitwise those of the two-pass path.  Model-level parity with the lazy path on:
tests/test_gpu_model.py (the engine uses it for every inverted residual's project conv
and OutConv's last conv).
"""
import pytest
import torch

from seg_amd._lib import SegLibError, call, query

pytestmark = pytest.mark.gpu
DEV = "cuda"
BF = torch.bfloat16


def S():
    return torch.cuda.current_stream().cuda_stream


def _raw(M, ld, seed, dt):
    g = torch.Generator().manual_seed(seed)
    y = torch.randn(M, ld, generator=g) * 1.5 + 0.3
    y = y.to(BF).float()  # bf16-representable, so one buffer serves every storage type
    return y.to(DEV).to(dt)


MATHS = {  # math -> (storage dtype, apply, conv, conv xf, wgrad, wgrad xf)
    "f32": (torch.float32, "seg_bn_apply", "seg_conv_igemm", "seg_conv_igemm_xf", "seg_conv_wgrad",
            "seg_conv_wgrad_xf"),
    "bf16": (torch.float32, "seg_bn_apply", "seg_conv_igemm_bf16", "seg_conv_igemm_bf16_xf", "seg_conv_wgrad_bf16",
             "seg_conv_wgrad_bf16_xf"),
    "bf16io": (BF, "seg_bn_apply_bf16io", "seg_conv_igemm_bf16io", "seg_conv_igemm_bf16io_xf",
               "seg_conv_wgrad_bf16io", "seg_conv_wgrad_bf16io_xf"),
}


@pytest.mark.parametrize("math", list(MATHS))
@pytest.mark.parametrize("M,Cin,Cout,ld", [(4096, 144, 24, 144), (3001, 96, 24, 96), (517, 16, 10, 16),
                                           (2048, 320, 1280, 320), (1000, 32, 16, 40), (777, 960, 160, 960)])
@pytest.mark.parametrize("act", [1, 2])
def test_xf_matches_apply_then_conv(math, M, Cin, Cout, ld, act):
    s = S()
    dt, apply, conv, conv_xf, wgrad, wgrad_xf = MATHS[math]
    y = _raw(M, ld, 1, dt)
    g = torch.Generator().manual_seed(2)
    scale = (torch.rand(Cin, generator=g) + 0.5).to(DEV)
    shift = (torch.randn(Cin, generator=g)).to(DEV)
    w = (torch.randn(Cout, Cin, generator=g) * 0.1).to(DEV)
    b = torch.randn(Cout, generator=g).to(DEV)
    # two-pass reference: x = act(BN(y)) stored, then the plain conv
    x = torch.zeros(M, ld, device=DEV, dtype=dt)
    call(apply, y.data_ptr(), ld, M, Cin, scale.data_ptr(), shift.data_ptr(), act, None, 0, x.data_ptr(), ld, s)
    ntiles = query("seg_conv_igemm_row_tiles", M, Cout, None)
    outs = {}
    for tag, name, inp, xf in (("ref", conv, x, ()), ("xf", conv_xf, y, (scale.data_ptr(), shift.data_ptr(), act))):
        out = torch.full((M, Cout), 3.0, device=DEV, dtype=dt)
        st = torch.empty(ntiles * 2 * Cout, device=DEV)
        tail = (0, None, 1) if (math == "bf16" and not xf) else ()  # seg_conv_igemm_bf16: act, work, splits
        call(name, inp.data_ptr(), ld, 1, 1, M, Cin, w.data_ptr(), Cin, b.data_ptr(), out.data_ptr(), Cout, 1, M,
             Cout, 1, 1, 0, None, 0, st.data_ptr(), *tail, *xf, s)
        outs[tag] = (out, st)
    assert torch.equal(outs["ref"][0].float(), outs["xf"][0].float())
    assert torch.equal(outs["ref"][1], outs["xf"][1])
    # weight gradient (split-K partial slabs)
    lddy = (Cout + 3) & ~3
    dy = _raw(M, lddy, 3, dt)
    splits = query("seg_conv_wgrad_splits", M, Cout, Cin, 1)
    parts = {}
    for tag, name, inp, xf in (("ref", wgrad, x, ()), ("xf", wgrad_xf, y, (scale.data_ptr(), shift.data_ptr(), act))):
        part = torch.empty(splits * Cout * Cin, device=DEV)
        call(name, dy.data_ptr(), lddy, inp.data_ptr(), ld, 1, 1, M, Cin, 1, M, Cout, 1, 1, 0, part.data_ptr(), splits,
             *xf, s)
        parts[tag] = part
    assert torch.equal(parts["ref"], parts["xf"])


def test_xf_rejects_unsupported():
    """3x3 convs the uniform-tap loader does not take (Cin below the K chunk) and missing
    coefficients fail loudly (no silent untransformed path)."""
    s = S()
    M, C = 256, 32
    y = torch.zeros(M, C, device=DEV)
    sc = torch.ones(C, device=DEV)
    w = torch.zeros(C * 9 * C, device=DEV)
    out = torch.empty(M, C, device=DEV)
    with pytest.raises(SegLibError):  # Cin 8 < the 16-deep K chunk of K = 72
        call("seg_conv_igemm_xf", y.data_ptr(), 8, 1, 16, 16, 8, w.data_ptr(), 72, None, out.data_ptr(), C, 16, 16,
             C, 3, 1, 1, None, 0, None, sc.data_ptr(), sc.data_ptr(), 2, s)
    with pytest.raises(SegLibError):
        call("seg_conv_igemm_xf", y.data_ptr(), C, 1, 1, M, C, w.data_ptr(), C, None, out.data_ptr(), C, 1, M, C, 1, 1,
             0, None, 0, None, None, None, 2, s)
    part = torch.empty(C * C * 9, device=DEV)
    with pytest.raises(SegLibError):
        call("seg_conv_wgrad_xf", y.data_ptr(), C, y.data_ptr(), C, 1, 16, 16, C, 16, 16, C, 3, 1, 1, part.data_ptr(),
             1, sc.data_ptr(), None, 2, s)
    with pytest.raises(SegLibError):
        call("seg_conv_halo_xf", y.data_ptr(), C, 1, 4, 64, C, w.data_ptr(), 9 * C, None, out.data_ptr(), C, C,
             None, 0, None, sc.data_ptr(), None, 1, s)


# ---- 3x3 consumers (double_conv's second conv, src/unet.py:58-62): implicit GEMM, LDS halo, weight gradient

MATHS3 = {  # math -> (storage dtype, apply, [(conv, conv xf, bf16 weights)], wgrad, wgrad xf, halo, halo xf)
    "f32": (torch.float32, "seg_bn_apply", [("seg_conv_igemm", "seg_conv_igemm_xf", False)], "seg_conv_wgrad",
            "seg_conv_wgrad_xf", "seg_conv_halo", "seg_conv_halo_xf"),
    "bf16io": (BF, "seg_bn_apply_bf16io", [("seg_conv_igemm_bf16io", "seg_conv_igemm_bf16io_xf", False),
                                           ("seg_conv_igemm_bf16io_w16", "seg_conv_igemm_bf16io_xf_w16", True)],
               "seg_conv_wgrad_bf16io", "seg_conv_wgrad_bf16io_xf", "seg_conv_halo_bf16io", "seg_conv_halo_bf16io_xf"),
}


def _nhwc_case(N, H, W, Cin, Cout, ld, dt, act, seed=5):
    M = N * H * W
    y = _raw(M, ld, seed, dt)
    g = torch.Generator().manual_seed(seed + 1)
    scale = (torch.rand(Cin, generator=g) + 0.5).to(DEV)
    shift = torch.randn(Cin, generator=g).to(DEV)
    x = torch.zeros(M, ld, device=DEV, dtype=dt)
    call(MATHS3["f32" if dt == torch.float32 else "bf16io"][1], y.data_ptr(), ld, M, Cin, scale.data_ptr(),
         shift.data_ptr(), act, None, 0, x.data_ptr(), ld, S())
    wk = (torch.randn(Cout, 9 * Cin, generator=g) * 0.05).to(BF).float().to(DEV)  # [Cout][tap * Cin + ci]
    b = torch.randn(Cout, generator=g).to(DEV)
    return y, x, scale, shift, wk, b


@pytest.mark.parametrize("math", list(MATHS3))
@pytest.mark.parametrize("N,H,W,Cin,Cout,ld", [(2, 8, 64, 32, 32, 32), (1, 12, 128, 64, 64, 64), (2, 7, 9, 48, 40, 48),
                                               (1, 16, 24, 96, 128, 104), (2, 4, 64, 128, 64, 128)])
@pytest.mark.parametrize("act", [1, 2])
def test_xf3_matches_apply_then_conv(math, N, H, W, Cin, Cout, ld, act):
    """A 3x3 stride-1 conv on act(BN(y)) formed on load equals the BN-apply pass + the plain conv,
    bitwise: outputs, BN partials and weight-gradient slabs.  The padding taps must stay zero
    (a transform of the zero page would add act(shift) around the border)."""
    s = S()
    dt, apply, convs, wgrad, wgrad_xf, halo, halo_xf = MATHS3[math]
    M = N * H * W
    y, x, scale, shift, wk, b = _nhwc_case(N, H, W, Cin, Cout, ld, dt, act)
    xf_args = (scale.data_ptr(), shift.data_ptr(), act)
    ntiles = query("seg_conv_igemm_row_tiles", M, Cout, None)
    for conv, conv_xf, w16 in convs:
        w = wk.to(BF) if w16 else wk
        outs = {}
        for tag, name, inp, xf in (("ref", conv, x, ()), ("xf", conv_xf, y, xf_args)):
            out = torch.full((M, Cout), 3.0, device=DEV, dtype=dt)
            st = torch.empty(ntiles * 2 * Cout, device=DEV)
            call(name, inp.data_ptr(), ld, N, H, W, Cin, w.data_ptr(), 9 * Cin, b.data_ptr(), out.data_ptr(), Cout, H, W,
                 Cout, 3, 1, 1, None, 0, st.data_ptr(), *xf, s)
            outs[tag] = (out, st)
        assert torch.equal(outs["ref"][0].float(), outs["xf"][0].float()), conv
        assert torch.equal(outs["ref"][1], outs["xf"][1]), conv
    if query("seg_conv_halo_ok", N, H, W, Cin, Cout):
        for w16 in ((False, True) if dt == BF else (False,)):
            w = wk.to(BF) if w16 else wk
            sfx = "_w16" if w16 else ""
            ht = query("seg_conv_halo_row_tiles", N, H, W)
            outs = {}
            for tag, name, inp, xf in (("ref", halo + sfx, x, ()), ("xf", halo_xf + sfx, y, xf_args)):
                out = torch.full((M, Cout), 3.0, device=DEV, dtype=dt)
                st = torch.empty(ht * 2 * Cout, device=DEV)
                call(name, inp.data_ptr(), ld, N, H, W, Cin, w.data_ptr(), 9 * Cin, b.data_ptr(), out.data_ptr(), Cout,
                     Cout, None, 0, st.data_ptr(), *xf, s)
                outs[tag] = (out, st)
            assert torch.equal(outs["ref"][0].float(), outs["xf"][0].float()), halo + sfx
            assert torch.equal(outs["ref"][1], outs["xf"][1]), halo + sfx
    lddy = (Cout + 7) & ~7
    dy = _raw(M, lddy, 9, dt)
    splits = query("seg_conv_wgrad_splits", M, Cout, Cin, 3)
    parts = {}
    for tag, name, inp, xf in (("ref", wgrad, x, ()), ("xf", wgrad_xf, y, xf_args)):
        part = torch.empty(splits * Cout * 9 * Cin, device=DEV)
        call(name, dy.data_ptr(), lddy, inp.data_ptr(), ld, N, H, W, Cin, H, W, Cout, 3, 1, 1, part.data_ptr(), splits,
             *xf, s)
        parts[tag] = part
    assert torch.equal(parts["ref"], parts["xf"])


@pytest.mark.parametrize("arch", ["UNet", "MobileNetV2UNet"])
def test_lazy3_model_step_bitwise(arch, monkeypatch):
    """bf16io training step with double_conv's second conv applying the first one's BN + ReLU on load
    (engine.LAZY3) equals the step with the BN-apply pass, bitwise: loss, every gradient, BN running
    statistics.  (igemm2 and wgrad2 off in both runs: they take no input transform, so with LAZY3 the deep convs
    move to the implicit GEMM and a different K order; the default path is covered by the oracle-budget
    tests of test_gpu_model.py / test_gpu_configs.py.)"""
    from seg_amd import MobileNetV2UNet, UNet, engine
    from seg_amd.detinit import deterministic_init, synthetic_batch
    monkeypatch.setattr(engine, "IGEMM2", "0")
    monkeypatch.setattr(engine, "WGRAD2", False)  # takes no input transform either (another K order)
    N, H, W = (2, 64, 128) if arch == "UNet" else (2, 128, 256)
    x, t = synthetic_batch(N, H, W, 10 if arch == "UNet" else 3, seed=17)
    x, t = x.to(DEV), t.to(DEV)
    res, n_lazy3 = {}, {}
    for lazy in (False, True):
        monkeypatch.setattr(engine, "LAZY3", lazy)
        model = deterministic_init(UNet(10) if arch == "UNet" else MobileNetV2UNet(3), seed=17).to(DEV).train()
        engine.set_conv_math(model, "bf16io")
        loss = model.forward_loss(x, t)
        loss.backward()
        torch.cuda.synchronize()
        prog = engine.get_program(model, N, H, W)
        n_lazy3[lazy] = sum(1 for op in prog.ops if isinstance(op, engine.ConvOp) and op.ks == 3 and op.kind == "igemm"
                            and op.xform is not None)
        res[lazy] = (loss.detach().clone(), {k: p.grad.clone() for k, p in model.named_parameters()
                                             if p.grad is not None},
                     {k: b.clone() for k, b in model.named_buffers()})
    assert n_lazy3[False] == 0 and n_lazy3[True] >= (7 if arch == "UNet" else 4), n_lazy3
    (l0, g0, b0), (l1, g1, b1) = res[False], res[True]
    assert torch.equal(l0, l1)
    for k in g0:
        assert torch.equal(g0[k], g1[k]), k
    for k in b0:
        assert torch.equal(b0[k], b1[k]), k
