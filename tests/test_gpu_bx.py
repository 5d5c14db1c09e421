"""GPU: 1x1 data gradients forming their BatchNorm-backward dY on load --
seg_bn_backward_coef + seg_conv_igemm_bx / seg_conv_igemm_bf16io_bx_w16 (include/segamd.h)
against seg_bn_backward (reduction + apply pass) followed by the plain 1x1 data gradient.

The BX loader computes dY with seg_bnbwd4 (the apply pass's arithmetic) and rounds it to
the storage type exactly where the pass stores it, so dX, the dY it writes back for the
parameter gradients and dgamma / dbeta must be bitwise those of the two-pass path.
Model-level parity with SEG_BX=1: tests/test_gpu_model.py runs every model path.
"""
import pytest
import torch

from seg_amd._lib import SegLibError, call, query

pytestmark = pytest.mark.gpu
DEV = "cuda"
BF = torch.bfloat16


def S():
    return torch.cuda.current_stream().cuda_stream


def _rand(shape, seed, scale=1.0, shift=0.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale + shift).to(BF).float()  # bf16-representable


MATHS = {  # math -> (storage, bn_backward, coef, plain dgrad, bx dgrad, weight element type, ldk multiple)
    "f32": (torch.float32, "seg_bn_backward", "seg_bn_backward_coef", "seg_conv_igemm", "seg_conv_igemm_bx",
            torch.float32, 4),
    "bf16io": (BF, "seg_bn_backward_bf16io", "seg_bn_backward_coef_bf16io", "seg_conv_igemm_bf16io_w16",
               "seg_conv_igemm_bf16io_bx_w16", BF, 8),
}


@pytest.mark.parametrize("math", list(MATHS))
@pytest.mark.parametrize("M,C,Cx,ld", [(4096, 144, 24, 144), (3001, 96, 16, 96), (16384, 24, 144, 24),
                                       (2048, 1280, 320, 1280), (777, 160, 960, 168), (1000, 16, 32, 16)])
@pytest.mark.parametrize("act", [0, 1, 2])
@pytest.mark.parametrize("accumulate", [False, True])
def test_bx_matches_bn_backward_then_dgrad(math, M, C, Cx, ld, act, accumulate):
    s = S()
    dt, bnb, coef_fn, dgrad, dgrad_bx, wt, q = MATHS[math]
    if (C % q) or (ld % q):
        pytest.skip("the BX loader needs 16-byte rows")
    da = _rand((M, ld), 1, 0.3).to(DEV).to(dt)
    y = _rand((M, ld), 2, 1.5, 0.4).to(DEV).to(dt)
    g = torch.Generator().manual_seed(3)
    gamma = (torch.rand(C, generator=g) + 0.5).to(DEV)
    mean = torch.randn(C, generator=g).to(DEV) * 0.2 + 0.4
    invstd = (torch.rand(C, generator=g) + 0.4).to(DEV)
    beta = torch.randn(C, generator=g).to(DEV)
    st = torch.cat([mean, invstd, gamma * invstd, beta - mean * gamma * invstd]).contiguous()
    C4 = C
    w = (torch.randn(C, Cx, generator=g) * 0.1).to(DEV)  # forward weight [C][Cx] (1x1): dgrad B = W^T
    ldk = (C + q - 1) // q * q
    wk = torch.zeros(Cx, ldk, device=DEV, dtype=wt)
    wk[:, :C] = w.t().to(wt)
    addend = _rand((M, Cx), 4).to(DEV).to(dt) if accumulate else None
    nws = query("seg_chan_workspace_floats", M, C)
    stp = st.data_ptr()
    ptrs = (stp, stp + 4 * C, stp + 8 * C, stp + 12 * C)
    # two-pass reference
    work = torch.zeros(nws + 3 * C, device=DEV)
    dgam, dbet = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
    dy = torch.zeros(M, ld, device=DEV, dtype=dt)
    call(bnb, da.data_ptr(), ld, y.data_ptr(), ld, M, C, gamma.data_ptr(), *ptrs, act, dgam.data_ptr(),
         dbet.data_ptr(), work.data_ptr(), dy.data_ptr(), ld, s)
    dx = addend.clone() if accumulate else torch.zeros(M, Cx, device=DEV, dtype=dt)
    call(dgrad, dy.data_ptr(), ld, 1, 1, M, C, wk.data_ptr(), ldk, None, dx.data_ptr(), Cx, 1, M, Cx, 1, 1, 0,
         dx.data_ptr() if accumulate else None, Cx if accumulate else 0, None, s)
    # BX
    work2 = torch.zeros(nws + 3 * C, device=DEV)
    dgam2, dbet2 = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
    call(coef_fn, da.data_ptr(), ld, y.data_ptr(), ld, M, C, gamma.data_ptr(), *ptrs, act, dgam2.data_ptr(),
         dbet2.data_ptr(), work2.data_ptr(), s)
    dy2 = torch.full((M, ld), 7.0, device=DEV, dtype=dt)
    dx2 = addend.clone() if accumulate else torch.zeros(M, Cx, device=DEV, dtype=dt)
    call(dgrad_bx, da.data_ptr(), ld, 1, 1, M, C, wk.data_ptr(), ldk, dx2.data_ptr(), Cx, Cx,
         dx2.data_ptr() if accumulate else None, Cx if accumulate else 0, y.data_ptr(), ld, st.data_ptr(),
         work2.data_ptr() + 4 * nws, act, dy2.data_ptr(), ld, s)
    torch.cuda.synchronize()
    assert torch.equal(dgam2, dgam) and torch.equal(dbet2, dbet)
    assert torch.equal(dy2[:, :C], dy[:, :C]), (dy2[:, :C] - dy[:, :C]).abs().max()
    if ld > C:  # padding columns beyond C are left alone
        assert bool((dy2[:, C:] == 7.0).all())
    assert torch.equal(dx2, dx), (dx2.float() - dx.float()).abs().max()


def test_bx_rejects_unaligned_rows():
    s = S()
    M, C, Cx = 256, 12, 16
    t = torch.zeros(M, 16, device=DEV, dtype=BF)
    st = torch.zeros(4 * 16, device=DEV)
    wk = torch.zeros(Cx, 16, device=DEV, dtype=BF)
    with pytest.raises(SegLibError):  # bf16: C % 8 != 0
        call("seg_conv_igemm_bf16io_bx_w16", t.data_ptr(), 16, 1, 1, M, C, wk.data_ptr(), 16, t.data_ptr(), 16, Cx,
             None, 0, t.data_ptr(), 16, st.data_ptr(), st.data_ptr(), 0, t.data_ptr(), 16, s)
