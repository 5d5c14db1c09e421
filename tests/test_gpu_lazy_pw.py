"""GPU: lazy BatchNorm for 1x1 consumers -- seg_conv_igemm*_xf / seg_conv_wgrad*_xf (include/segamd.h) against a separate BN-apply pass followed by the plain conv.

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
