"""GPU: one-launch BatchNorm backward for small layers (seg_bn_backward_small, include/segamd.h)
against the three-launch seg_bn_backward and a float64 restatement of aten's
native_batch_norm_backward through the activation (src/unet.py:59-63; torchvision's
Conv2dNormActivation via src/unet.py:15-19).

The fused kernel sums the same terms over another row partition, so it is compared within
fp32 rounding (fp32 storage) / one bf16 rounding step (bf16io), and must be bitwise
reproducible call to call on the same workspace (its grid barrier re-arms itself); the
barrier's timeout word must stay zero.
"""
import pytest
import torch

from seg_amd._lib import SegLibError, call, query

pytestmark = pytest.mark.gpu
DEV = "cuda"
BF = torch.bfloat16


def S():
    return torch.cuda.current_stream().cuda_stream


def _ref64(da, y, gamma, mean, invstd, scale, shift, act):
    y, da = y.double(), da.double()
    z = y * scale.double() + shift.double()
    mask = torch.ones_like(z) if act == 0 else ((z > 0) if act == 1 else ((z > 0) & (z < 6))).double()
    dz = da * mask
    xhat = (y - mean.double()) * invstd.double()
    M = y.shape[0]
    k1 = gamma.double() * invstd.double()
    dy = k1 * (dz - dz.sum(0) / M - xhat * (dz * xhat).sum(0) / M)
    return dy, (dz * xhat).sum(0), dz.sum(0)


@pytest.mark.parametrize("io", [False, True])
@pytest.mark.parametrize("M,C,ld", [(4096, 1280, 1280), (4096, 160, 160), (16384, 384, 384), (16384, 96, 104),
                                    (65536, 192, 192), (65536, 32, 32), (1000, 24, 24), (37, 16, 16), (4096, 1024, 1032)])
@pytest.mark.parametrize("act", [0, 1, 2])
def test_small_matches_three_launch(io, M, C, ld, act):
    s = S()
    dt = BF if io else torch.float32
    sfx = "_bf16io" if io else ""
    g = torch.Generator().manual_seed(M + C + act)
    da = (torch.randn(M, ld, generator=g) * 0.3).to(BF).float().to(DEV).to(dt)
    y = (torch.randn(M, ld, generator=g) * 1.5 + 0.4).to(BF).float().to(DEV).to(dt)
    gamma = (torch.rand(C, generator=g) + 0.5).to(DEV)
    mean = (torch.randn(C, generator=g) * 0.2 + 0.4).to(DEV)
    invstd = (torch.rand(C, generator=g) + 0.4).to(DEV)
    beta = torch.randn(C, generator=g).to(DEV)
    st = torch.cat([mean, invstd, gamma * invstd, beta - mean * gamma * invstd]).contiguous()
    p = st.data_ptr()
    ptrs = (p, p + 4 * C, p + 8 * C, p + 12 * C)
    assert query("seg_bn_backward_small_blocks", M, C, 1 << 24) > 0
    work = torch.zeros(query("seg_chan_workspace_floats", M, C) + 3 * C, device=DEV)
    dg, db = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
    dy = torch.zeros(M, ld, device=DEV, dtype=dt)
    call("seg_bn_backward" + sfx, da.data_ptr(), ld, y.data_ptr(), ld, M, C, gamma.data_ptr(), *ptrs, act,
         dg.data_ptr(), db.data_ptr(), work.data_ptr(), dy.data_ptr(), ld, s)
    ws = torch.zeros(query("seg_bn_backward_small_floats", C), device=DEV)
    outs = []
    for rep in range(3):
        dg2, db2 = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
        dy2 = torch.full((M, ld), 7.0, device=DEV, dtype=dt)
        call("seg_bn_backward_small" + sfx, da.data_ptr(), ld, y.data_ptr(), ld, M, C, gamma.data_ptr(), *ptrs, act,
             dg2.data_ptr(), db2.data_ptr(), ws.data_ptr(), dy2.data_ptr(), ld, s)
        outs.append((dg2, db2, dy2))
    torch.cuda.synchronize()
    assert int(ws[:4].view(torch.int32)[2]) == 0, "grid barrier timed out"
    for o in outs[1:]:
        assert all(torch.equal(a, b) for a, b in zip(o, outs[0])), "not reproducible"
    dg2, db2, dy2 = outs[0]
    ref, rdg, rdb = _ref64(da[:, :C].float().cpu(), y[:, :C].float().cpu(), gamma.cpu(), mean.cpu(), invstd.cpu(),
                           (gamma * invstd).cpu(), (beta - mean * gamma * invstd).cpu(), act)
    assert torch.allclose(dg2.double().cpu(), rdg * invstd.double().cpu(), rtol=1e-4, atol=1e-3)
    assert torch.allclose(db2.double().cpu(), rdb, rtol=1e-4, atol=1e-3)
    assert torch.allclose(dg2, dg, rtol=1e-5, atol=1e-4) and torch.allclose(db2, db, rtol=1e-5, atol=1e-4)
    got, three = dy2[:, :C].float(), dy[:, :C].float()
    scale_ = three.abs().max().item()
    tol = (2.0 ** -7 if io else 1e-5) * scale_
    assert (got - three).abs().max().item() <= tol, ((got - three).abs().max().item(), tol)
    e = (got.double().cpu() - ref).norm() / ref.norm()
    assert e < (4e-3 if io else 1e-5), e
    if ld > C:
        assert bool((dy2[:, C:].float() == 7.0).all())


def test_small_rejects_large_layers_and_wide_unaligned_rows():
    assert query("seg_bn_backward_small_blocks", 1 << 20, 96, 1 << 24) == 0
    assert query("seg_bn_backward_small_blocks", 4096, 96, 0) == 0
    M, C = 256, 1028  # 4-channel lanes would need 257 > 256 lanes
    t = torch.zeros(M, C, device=DEV)
    st = torch.zeros(4 * C, device=DEV)
    ws = torch.zeros(query("seg_bn_backward_small_floats", C), device=DEV)
    with pytest.raises(SegLibError):
        call("seg_bn_backward_small", t.data_ptr(), C, t.data_ptr(), C, M, C, None, st.data_ptr(), st.data_ptr(),
             st.data_ptr(), st.data_ptr(), 0, None, None, ws.data_ptr(), t.data_ptr(), C, S())
