"""GPU: every C-ABI kernel against a plain PyTorch fp32 CPU reference of the
same op (forward and backward via torch.autograd), on odd shapes and edge cases.
All calls go through libsegamd.so (seg_amd._lib)."""
import ctypes

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from seg_amd._lib import call, query

pytestmark = pytest.mark.gpu
DEV = "cuda"


def r4(c):
    return (c + 3) & ~3


def S():
    return torch.cuda.current_stream().cuda_stream


def nhwc(t, ld=None):
    """NCHW CPU tensor -> [N*H*W, ld] CUDA rows (pad channels filled with NaN to
    prove they are never read as data)."""
    N, C, H, W = t.shape
    ld = ld or r4(C)
    out = torch.full((N * H * W, ld), float("nan"), dtype=torch.float32)
    out[:, :C] = t.permute(0, 2, 3, 1).reshape(-1, C)
    return out.to(DEV)


def from_nhwc(rows, N, C, H, W):
    return rows[:, :C].reshape(N, H, W, C).permute(0, 3, 1, 2).cpu()


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


def gen(*shape, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(*shape, generator=g)


@pytest.mark.parametrize("N,Cin,Cout,H,W,ks", [(2, 16, 96, 9, 13, 1), (1, 1344, 256, 4, 8, 3), (3, 80, 32, 7, 5, 3),
                                              (2, 152, 64, 6, 10, 3), (1, 16, 10, 5, 7, 1), (2, 24, 144, 8, 8, 1),
                                              (1, 320, 1280, 2, 4, 1), (2, 36, 200, 5, 6, 3)])
def test_conv_igemm_fwd_dgrad_wgrad(N, Cin, Cout, H, W, ks):
    pad = ks // 2
    x = gen(N, Cin, H, W, seed=1)
    w = gen(Cout, Cin, ks, ks, seed=2) * (2.0 / (Cin * ks * ks)) ** 0.5
    b = gen(Cout, seed=3)
    xr = x.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    y = F.conv2d(xr, wr, b, padding=pad)
    dy = gen(*y.shape, seed=4)
    y.backward(dy)
    s = S()
    # forward
    xg, wg, bg = nhwc(x), w.to(DEV), b.to(DEV)
    ldk = r4(ks * ks * Cin)
    wk = torch.empty(Cout * ldk, device=DEV)
    call("seg_pack_conv_weight", wg.data_ptr(), wk.data_ptr(), Cout, Cin, ks, ldk, 0, Cin, s)
    out = torch.full((N * H * W, r4(Cout)), float("nan"), device=DEV)
    call("seg_conv_igemm", xg.data_ptr(), xg.shape[1], N, H, W, Cin, wk.data_ptr(), ldk, bg.data_ptr(),
         out.data_ptr(), out.shape[1], H, W, Cout, ks, 1, pad, None, 0, None, s)
    assert rel(from_nhwc(out, N, Cout, H, W), y.detach()) < 1e-5
    # same conv with the BatchNorm statistics fused into the epilogue
    ntiles = query("seg_conv_igemm_row_tiles", N * H * W, Cout, None)
    tr = ctypes.c_int(0)
    query("seg_conv_igemm_row_tiles", N * H * W, Cout, ctypes.addressof(tr))
    stat = torch.empty(ntiles * 2 * Cout, device=DEV)
    out2 = torch.empty_like(out)
    call("seg_conv_igemm", xg.data_ptr(), xg.shape[1], N, H, W, Cin, wk.data_ptr(), ldk, bg.data_ptr(),
         out2.data_ptr(), out2.shape[1], H, W, Cout, ks, 1, pad, None, 0, stat.data_ptr(), s)
    assert torch.equal(out2[:, :Cout], out[:, :Cout])
    st = torch.empty(4 * Cout, device=DEV)
    rm, rv = torch.zeros(Cout, device=DEV), torch.ones(Cout, device=DEV)
    call("seg_bn_stats_tiles", stat.data_ptr(), ntiles, tr.value, N * H * W, Cout, None, None, 1e-5, 0.1,
         rm.data_ptr(), rv.data_ptr(), None, st[:Cout].data_ptr(), st[Cout:2 * Cout].data_ptr(),
         st[2 * Cout:3 * Cout].data_ptr(), st[3 * Cout:].data_ptr(), s)
    y64 = y.detach().double()
    mean64 = y64.mean((0, 2, 3))
    var64 = y64.var((0, 2, 3), unbiased=False)
    assert rel(st[:Cout], mean64) < 1e-5
    assert rel(st[Cout:2 * Cout], 1 / torch.sqrt(var64 + 1e-5)) < 1e-5
    assert rel(rv, 0.9 + 0.1 * y64.var((0, 2, 3), unbiased=True)) < 1e-5
    # data gradient (+ fused addend)
    dyg = nhwc(dy)
    if Cout % 4:
        dyg[:, Cout:] = 0.0  # the engine's contract: padded gradient channels are zero
    kin = r4(Cout)
    ldk2 = r4(ks * ks * kin)
    wkd = torch.empty(Cin * ldk2, device=DEV)
    call("seg_pack_conv_weight", wg.data_ptr(), wkd.data_ptr(), Cout, Cin, ks, ldk2, 1, kin, s)
    addend = gen(N, Cin, H, W, seed=5)
    addg = nhwc(addend)
    dx = torch.empty(N * H * W, r4(Cin), device=DEV)
    call("seg_conv_igemm", dyg.data_ptr(), dyg.shape[1], N, H, W, kin, wkd.data_ptr(), ldk2, None,
         dx.data_ptr(), dx.shape[1], H, W, Cin, ks, 1, pad, addg.data_ptr(), addg.shape[1], None, s)
    assert rel(from_nhwc(dx, N, Cin, H, W), xr.grad + addend) < 1e-5
    # weight gradient
    M = N * H * W
    splits = query("seg_conv_wgrad_splits", M, Cout, Cin, ks)
    part = torch.empty(splits * Cout * ks * ks * Cin, device=DEV)
    call("seg_conv_wgrad", dyg.data_ptr(), dyg.shape[1], xg.data_ptr(), xg.shape[1], N, H, W, Cin, H, W, Cout,
         ks, 1, pad, part.data_ptr(), splits, s)
    dw = torch.empty(Cout, Cin, ks, ks, device=DEV)
    call("seg_conv_wgrad_reduce", part.data_ptr(), splits, dw.data_ptr(), Cout, Cin, ks, 0, 0, s)
    assert rel(dw, wr.grad) < 1e-5


@pytest.mark.parametrize("lazy", [False, True])
@pytest.mark.parametrize("N,C,H,W,stride", [(2, 32, 9, 12, 1), (2, 96, 10, 14, 2), (1, 960, 4, 4, 1),
                                            (3, 144, 7, 9, 2), (1, 8, 1, 1, 1), (2, 24, 5, 19, 2),
                                            (1, 256, 3, 17, 1)])
def test_depthwise(N, C, H, W, stride, lazy):
    """Depthwise 3x3 fwd / dgrad / wgrad.  lazy: the kernels read the producer's raw
    conv output u and apply its BN affine + ReLU6 on load (x = relu6(u*sc + sh))."""
    u = gen(N, C, H, W, seed=1)
    if lazy:
        sc, sh = gen(C, seed=7) * 2.0, gen(C, seed=8) * 3.0
        x = torch.clamp(torch.addcmul(sh.view(1, C, 1, 1), u, sc.view(1, C, 1, 1)), 0.0, 6.0)
    else:
        x = u
    w = gen(C, 1, 3, 3, seed=2)
    xr, wr = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
    y = F.conv2d(xr, wr, None, stride=stride, padding=1, groups=C)
    Ho, Wo = y.shape[2], y.shape[3]
    dy = gen(*y.shape, seed=3)
    y.backward(dy)
    s = S()
    ug, wg = nhwc(u), w.to(DEV)
    scp = shp = None
    if lazy:
        scg, shg = sc.to(DEV), sh.to(DEV)
        scp, shp = scg.data_ptr(), shg.data_ptr()
    act = 2 if lazy else 0
    wk = torch.empty(9 * C, device=DEV)
    call("seg_pack_dw_weight", wg.data_ptr(), wk.data_ptr(), C, s)
    out = torch.empty(N * Ho * Wo, r4(C), device=DEV)
    call("seg_dw_fwd", ug.data_ptr(), ug.shape[1], N, H, W, C, scp, shp, act, wk.data_ptr(), out.data_ptr(),
         out.shape[1], Ho, Wo, stride, s)
    assert rel(from_nhwc(out, N, C, Ho, Wo), y.detach()) < 1e-5
    dyg = nhwc(dy)
    dx = nhwc(torch.ones(N, C, H, W))
    call("seg_dw_dgrad", dyg.data_ptr(), dyg.shape[1], N, Ho, Wo, C, wk.data_ptr(), dx.data_ptr(), dx.shape[1], H, W,
         stride, 1, s)  # accumulate onto ones
    assert rel(from_nhwc(dx, N, C, H, W), xr.grad + 1.0) < 1e-5
    dx0 = torch.empty(N * H * W, r4(C), device=DEV)
    call("seg_dw_dgrad", dyg.data_ptr(), dyg.shape[1], N, Ho, Wo, C, wk.data_ptr(), dx0.data_ptr(), dx0.shape[1], H,
         W, stride, 0, s)  # overwrite
    assert rel(from_nhwc(dx0, N, C, H, W), xr.grad) < 1e-5
    nblk = query("seg_dw_wgrad_blocks", N, Ho, Wo, C)
    part = torch.empty(nblk * 9 * C, device=DEV)
    call("seg_dw_wgrad", dyg.data_ptr(), dyg.shape[1], ug.data_ptr(), ug.shape[1], N, H, W, C, scp, shp, act, Ho, Wo,
         stride, part.data_ptr(), s)
    dw = torch.empty(C, 1, 3, 3, device=DEV)
    call("seg_conv_wgrad_reduce", part.data_ptr(), nblk, dw.data_ptr(), C, 1, 3, 1, 0, s)
    assert rel(dw, wr.grad) < 1e-5


@pytest.mark.parametrize("N,H,W,Cout,stride,bias", [(2, 16, 24, 32, 2, False), (1, 9, 14, 64, 1, True),
                                                    (2, 7, 11, 32, 1, True), (1, 13, 9, 64, 2, False)])
def test_first_conv_from_nchw_image(N, H, W, Cout, stride, bias):
    """Cin = 3 first conv (MobileNetV2 stem s2 / UNet inc s1): NCHW -> NHWC4, then the
    strided implicit GEMM with the 4th weight channel packed as zero."""
    x = gen(N, 3, H, W, seed=1)
    w = gen(Cout, 3, 3, 3, seed=2)
    b = gen(Cout, seed=3) if bias else None
    wr = w.clone().requires_grad_(True)
    y = F.conv2d(x, wr, b, stride=stride, padding=1)
    Ho, Wo = y.shape[2], y.shape[3]
    dy = gen(*y.shape, seed=4)
    y.backward(dy)
    s = S()
    xg, wg = x.to(DEV), w.to(DEV)
    bg = b.to(DEV) if bias else None
    x4 = torch.full((N * H * W, 4), float("nan"), device=DEV)
    call("seg_nchw_to_nhwc", xg.data_ptr(), N, 3, H, W, x4.data_ptr(), 4, s)
    assert torch.equal(x4[:, 3], torch.zeros_like(x4[:, 3]))
    assert torch.equal(from_nhwc(x4, N, 3, H, W), x)
    ldk = 36
    wk = torch.empty(Cout * ldk, device=DEV)
    call("seg_pack_conv_weight", wg.data_ptr(), wk.data_ptr(), Cout, 3, 3, ldk, 0, 4, s)
    out = torch.empty(N * Ho * Wo, Cout, device=DEV)
    call("seg_conv_igemm", x4.data_ptr(), 4, N, H, W, 4, wk.data_ptr(), ldk, bg.data_ptr() if bias else None,
         out.data_ptr(), Cout, Ho, Wo, Cout, 3, stride, 1, None, 0, None, s)
    assert rel(from_nhwc(out, N, Cout, Ho, Wo), y.detach()) < 1e-5
    dyg = nhwc(dy)
    splits = query("seg_conv_wgrad_splits", N * Ho * Wo, Cout, 4, 3)
    part = torch.empty(splits * Cout * 36, device=DEV)
    call("seg_conv_wgrad", dyg.data_ptr(), dyg.shape[1], x4.data_ptr(), 4, N, H, W, 4, Ho, Wo, Cout, 3, stride, 1,
         part.data_ptr(), splits, s)
    dw = torch.empty(Cout, 3, 3, 3, device=DEV)
    call("seg_conv_wgrad_reduce", part.data_ptr(), splits, dw.data_ptr(), Cout, 3, 3, 0, 0, s)
    assert rel(dw, wr.grad) < 1e-5


@pytest.mark.parametrize("act", [0, 1, 2])
@pytest.mark.parametrize("M,C,shift", [(1000, 96, 0.0), (4097, 1280, 5.0), (37, 16, 100.0)])
def test_batchnorm_train(act, M, C, shift):
    y = gen(M, C, seed=1) * 3 + shift
    gamma, beta = gen(C, seed=2) * 0.2 + 1, gen(C, seed=3) * 0.5
    rm, rv = gen(C, seed=4) * 0.1, torch.rand(C, generator=torch.Generator().manual_seed(5)) + 0.5
    res = gen(M, C, seed=6)
    da = gen(M, C, seed=7)
    # Elements whose pre-activation sits within rounding of a ReLU/ReLU6 threshold
    # take the mask of whichever fp32 rounding computed them; each such flip moves
    # one dy element by O(1).  Give them zero upstream gradient so the test checks
    # the arithmetic, not the coin flip.
    y64 = y.double()
    z64 = (y64 - y64.mean(0)) / torch.sqrt(y64.var(0, unbiased=False) + 1e-5) * gamma.double() + beta.double()
    da[(z64.abs() < 1e-4) | ((z64 - 6).abs() < 1e-4)] = 0.0
    yr = y.clone().requires_grad_(True)
    gr, br = gamma.clone().requires_grad_(True), beta.clone().requires_grad_(True)
    rm_ref, rv_ref = rm.clone(), rv.clone()
    z = F.batch_norm(yr.t().reshape(1, C, M), rm_ref, rv_ref, gr, br, True, 0.1, 1e-5).reshape(C, M).t()
    a = F.relu(z) if act == 1 else (F.hardtanh(z, 0, 6) if act == 2 else z)
    out_ref = a + res
    out_ref.backward(da)
    s = S()
    yg, gg, bgp = y.to(DEV), gamma.to(DEV), beta.to(DEV)
    rmg, rvg = rm.to(DEV), rv.to(DEV)
    nbt = torch.zeros(1, dtype=torch.int64, device=DEV)
    st = torch.empty(4 * C, device=DEV)
    work = torch.zeros(query("seg_chan_workspace_floats", M, C) + 3 * C, device=DEV)
    call("seg_bn_stats", yg.data_ptr(), C, M, C, gg.data_ptr(), bgp.data_ptr(), 1e-5, 0.1, rmg.data_ptr(),
         rvg.data_ptr(), nbt.data_ptr(), work.data_ptr(), st[0:C].data_ptr(), st[C:2 * C].data_ptr(),
         st[2 * C:3 * C].data_ptr(), st[3 * C:].data_ptr(), s)
    resg = res.to(DEV)
    out = torch.empty(M, C, device=DEV)
    call("seg_bn_apply", yg.data_ptr(), C, M, C, st[2 * C:3 * C].data_ptr(), st[3 * C:].data_ptr(), act,
         resg.data_ptr(), C, out.data_ptr(), C, s)
    assert rel(out, out_ref.detach()) < 1e-5
    assert rel(rmg, rm_ref) < 1e-5 and rel(rvg, rv_ref) < 1e-5 and int(nbt) == 1
    dag = da.to(DEV)
    dgam, dbet = torch.empty(C, device=DEV), torch.empty(C, device=DEV)
    dy = torch.empty(M, C, device=DEV)
    call("seg_bn_backward", dag.data_ptr(), C, yg.data_ptr(), C, M, C, gg.data_ptr(), st[0:C].data_ptr(),
         st[C:2 * C].data_ptr(), st[2 * C:3 * C].data_ptr(), st[3 * C:].data_ptr(), act, dgam.data_ptr(),
         dbet.data_ptr(), work.data_ptr(), dy.data_ptr(), C, s)
    assert rel(dy, yr.grad) < 1e-4
    assert rel(dgam, gr.grad) < 1e-4 and rel(dbet, br.grad) < 1e-4


@pytest.mark.parametrize("N,C,H,W,ac", [(2, 64, 5, 7, 0), (1, 1280, 2, 4, 0), (2, 12, 6, 9, 1), (1, 8, 1, 1, 0)])
def test_upsample(N, C, H, W, ac):
    x = gen(N, C, H, W, seed=1)
    xr = x.clone().requires_grad_(True)
    y = F.interpolate(xr, scale_factor=2, mode="bilinear", align_corners=bool(ac))
    Ho, Wo = 2 * H, 2 * W
    dy = gen(*y.shape, seed=2)
    y.backward(dy)
    s = S()
    xg = nhwc(x)
    # write into a channel slice of a wider (concat) buffer
    ld = r4(C) + 16
    cat = torch.full((N * Ho * Wo, ld), float("nan"), device=DEV)
    call("seg_upsample_fwd", xg.data_ptr(), xg.shape[1], N, H, W, C, cat.data_ptr() + 4 * 16, ld, Ho, Wo, ac, s)
    assert rel(from_nhwc(cat[:, 16:], N, C, Ho, Wo), y.detach()) < 1e-6
    dyg = torch.zeros(N * Ho * Wo, ld, device=DEV)
    dyg[:, 16:16 + C] = dy.permute(0, 2, 3, 1).reshape(-1, C).to(DEV)
    dx = torch.empty(N * H * W, r4(C), device=DEV)
    call("seg_upsample_bwd", dyg.data_ptr() + 4 * 16, ld, 0, N, Ho, Wo, C, dx.data_ptr(), dx.shape[1], H, W, ac, 0, s)
    assert rel(from_nhwc(dx, N, C, H, W), xr.grad) < 1e-6
    # NCHW gradient path + NCHW output path
    dyn = dy.contiguous().to(DEV)
    dx2 = torch.empty(N * H * W, r4(C), device=DEV)
    call("seg_upsample_bwd", dyn.data_ptr(), 0, 1, N, Ho, Wo, C, dx2.data_ptr(), dx2.shape[1], H, W, ac, 0, s)
    assert rel(from_nhwc(dx2, N, C, H, W), xr.grad) < 1e-6
    outn = torch.empty(N, C, Ho, Wo, device=DEV)
    call("seg_upsample_to_nchw", xg.data_ptr(), xg.shape[1], N, H, W, C, outn.data_ptr(), Ho, Wo, ac, s)
    assert rel(outn, y.detach()) < 1e-6


def test_maxpool_with_ties():
    N, C, H, W = 2, 8, 6, 10
    x = torch.randint(0, 3, (N, C, H, W)).float()  # many ties: first-max rule matters
    xr = x.clone().requires_grad_(True)
    y = F.max_pool2d(xr, 2)
    dy = gen(*y.shape, seed=1)
    y.backward(dy)
    s = S()
    xg = nhwc(x)
    out = torch.empty(N * (H // 2) * (W // 2), C, device=DEV)
    call("seg_maxpool2_fwd", xg.data_ptr(), C, N, H, W, C, out.data_ptr(), C, s)
    assert torch.equal(from_nhwc(out, N, C, H // 2, W // 2), y.detach())
    dyg = nhwc(dy)
    dx = nhwc(torch.full((N, C, H, W), 0.5))
    call("seg_maxpool2_bwd", xg.data_ptr(), C, dyg.data_ptr(), C, N, H, W, C, dx.data_ptr(), C, 1, s)
    assert torch.allclose(from_nhwc(dx, N, C, H, W), xr.grad + 0.5, atol=1e-6)


@pytest.mark.parametrize("N,C,H,W,ignore", [(2, 10, 8, 16, False), (1, 4, 5, 7, True), (2, 1, 4, 4, False),
                                            (1, 21, 3, 5, True)])
def test_ce_fused_upsample(N, C, H, W, ignore):
    low = gen(N, C, H, W, seed=1) * 2
    Ho, Wo = 2 * H, 2 * W
    g = torch.Generator().manual_seed(2)
    y = torch.randint(0, C, (N, Ho, Wo), generator=g)
    if ignore:
        y[0, :2] = -100
    lr = low.clone().requires_grad_(True)
    logits = F.interpolate(lr, scale_factor=2, mode="bilinear", align_corners=True)
    loss = F.cross_entropy(logits, y)
    loss.backward(torch.tensor(0.7))
    s = S()
    lg = nhwc(low)
    yg = y.to(DEV)
    stats = torch.empty(3, device=DEV)
    work = torch.empty(query("seg_ce_workspace_floats", N * Ho * Wo), device=DEV)
    call("seg_ce_upsample_loss", lg.data_ptr(), lg.shape[1], N, H, W, C, yg.data_ptr(), Ho, Wo, -100,
         work.data_ptr(), stats.data_ptr(), s)
    assert abs(stats[0].item() - loss.item()) <= 1e-5 * abs(loss.item()) + 1e-7
    assert stats[2].item() == 0
    gout = torch.tensor([0.7], device=DEV)
    ld = r4(C)
    dhigh = torch.empty(N * Ho * Wo * ld, device=DEV)
    call("seg_ce_upsample_grad", lg.data_ptr(), lg.shape[1], N, H, W, C, yg.data_ptr(), Ho, Wo, -100,
         gout.data_ptr(), stats.data_ptr(), dhigh.data_ptr(), ld, s)
    dlow = torch.empty(N * H * W, ld, device=DEV)
    call("seg_upsample_bwd", dhigh.data_ptr(), ld, 0, N, Ho, Wo, C, dlow.data_ptr(), ld, H, W, 1, 0, s)
    assert rel(from_nhwc(dlow, N, C, H, W), lr.grad) < 1e-5
    assert torch.all(dlow[:, C:] == 0)


@pytest.mark.parametrize("bad", [10, 255, -1])
def test_ce_target_out_of_bounds(bad):
    """A label outside [0, C) that is not ignore_index: nn.CrossEntropyLoss raises
    'Target out of bounds'; the fused kernels flag it (stats[2]), poison the loss and
    the gradient with NaN, and train_model / engine.check_targets raise."""
    N, C, H, W = 1, 10, 4, 6
    Ho, Wo = 2 * H, 2 * W
    low = gen(N, C, H, W, seed=1)
    y = torch.randint(0, C, (N, Ho, Wo), generator=torch.Generator().manual_seed(3))
    y[0, 1, 2] = bad
    with pytest.raises((IndexError, RuntimeError)):
        F.cross_entropy(F.interpolate(low, scale_factor=2, mode="bilinear", align_corners=True), y)
    s = S()
    lg, yg = nhwc(low), y.to(DEV)
    stats = torch.empty(3, device=DEV)
    work = torch.empty(query("seg_ce_workspace_floats", N * Ho * Wo), device=DEV)
    call("seg_ce_upsample_loss", lg.data_ptr(), lg.shape[1], N, H, W, C, yg.data_ptr(), Ho, Wo, -100,
         work.data_ptr(), stats.data_ptr(), s)
    assert stats[2].item() == 1 and torch.isnan(stats[0])
    dhigh = torch.empty(N * Ho * Wo * 12, device=DEV)
    call("seg_ce_upsample_grad", lg.data_ptr(), lg.shape[1], N, H, W, C, yg.data_ptr(), Ho, Wo, -100,
         torch.ones(1, device=DEV).data_ptr(), stats.data_ptr(), dhigh.data_ptr(), 12, s)
    assert torch.isnan(dhigh.view(-1, 12)[:, :C]).any()
    # through the model: the fused loss is NaN and check_targets raises like aten
    from seg_amd import MobileNetV2UNet, deterministic_init
    from seg_amd.engine import check_targets
    model = deterministic_init(MobileNetV2UNet(10), seed=1).to(DEV).train()
    x = torch.randn(1, 3, 64, 64, generator=torch.Generator().manual_seed(0)).to(DEV)
    t = torch.zeros(1, 64, 64, dtype=torch.int64, device=DEV)
    t[0, 5, 5] = bad
    loss = model.forward_loss(x, t)
    assert torch.isnan(loss)
    with pytest.raises(IndexError, match="Target out of bounds"):
        check_targets(model)
    t[0, 5, 5] = -100  # ignore_index is fine
    assert torch.isfinite(model.forward_loss(x, t))
    check_targets(model)
    # train_model raises BEFORE optimizer.step(): no NaN reaches the weights
    from torch import nn
    from seg_amd import train_model
    t[0, 5, 5] = bad
    before = {k: v.clone() for k, v in model.state_dict().items() if v.is_floating_point() and "running" not in k}
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    with pytest.raises(IndexError, match="Target out of bounds"):
        train_model(model, [(x, t)], nn.CrossEntropyLoss(), opt, DEV, epochs=1, checkpoint_pattern=None,
                    progress=False)
    for k, v in model.state_dict().items():
        if k in before:
            assert torch.equal(v, before[k]), k
    # seg_amd.Adam: the step is queued without a host wait and skips itself on the device;
    # the loop raises after loss.item() -- parameters and Adam moments unchanged
    from seg_amd import Adam
    sopt = Adam(model.parameters(), lr=1e-3)
    with pytest.raises(IndexError, match="Target out of bounds"):
        train_model(model, [(x, t)], nn.CrossEntropyLoss(), sopt, DEV, epochs=1, checkpoint_pattern=None,
                    progress=False)
    for k, v in model.state_dict().items():
        if k in before:
            assert torch.equal(v, before[k]), k
    for st in sopt.state.values():
        assert not st["exp_avg"].any() and not st["exp_avg_sq"].any()
        assert st["step"].item() == 0  # the skipped step's counter advance is taken back
    # and a clean batch after it takes the step -- bitwise the step of an optimizer that never saw the bad batch
    # (the reference never reaches optimizer.step() on it, so its first real step has t = 1)
    t[0, 5, 5] = 3
    twin = deterministic_init(MobileNetV2UNet(10), seed=1).to(DEV).train()
    twin.load_state_dict(model.state_dict())
    fresh = Adam(twin.parameters(), lr=1e-3)
    train_model(model, [(x, t)], nn.CrossEntropyLoss(), sopt, DEV, epochs=1, checkpoint_pattern=None, progress=False)
    train_model(twin, [(x, t)], nn.CrossEntropyLoss(), fresh, DEV, epochs=1, checkpoint_pattern=None, progress=False)
    assert any(not torch.equal(v, before[k]) for k, v in model.state_dict().items() if k in before)
    tw = twin.state_dict()
    for k, v in model.state_dict().items():
        assert torch.equal(v, tw[k]), k
    assert all(st["step"].item() == 1 for st in sopt.state.values())


def test_colsum_and_add():
    M, C = 3001, 10
    y = gen(M, r4(C), seed=1)
    s = S()
    yg = y.to(DEV)
    work = torch.zeros(query("seg_chan_workspace_floats", M, r4(C)), device=DEV)
    out = torch.empty(C, device=DEV)
    call("seg_colsum", yg.data_ptr(), r4(C), M, C, work.data_ptr(), out.data_ptr(), 0, s)
    assert rel(out, y[:, :C].sum(0)) < 1e-5
    a, b = gen(M, 16, seed=2).to(DEV), gen(M, 16, seed=3).to(DEV)
    o = torch.empty(M, 16, device=DEV)
    call("seg_add", a.data_ptr(), 16, b.data_ptr(), 16, M, 16, o.data_ptr(), 16, s)
    assert torch.equal(o, a + b)


@pytest.mark.parametrize("act", [0, 1, 2])
@pytest.mark.parametrize("N,Cin,Cout,H,W,ks,res", [(1, 1344, 256, 8, 16, 3, False), (1, 288, 128, 16, 32, 3, False),
                                                   (1, 960, 320, 8, 16, 1, False), (1, 96, 96, 4, 4, 1, True),
                                                   (2, 80, 32, 9, 11, 3, False)])
def test_conv_igemm_act_splitk(N, Cin, Cout, H, W, ks, res, act):
    """seg_conv_igemm_act: act(conv + bias + add), unsplit and split-K (the inference path)."""
    pad = ks // 2
    x = gen(N, Cin, H, W, seed=11)
    w = gen(Cout, Cin, ks, ks, seed=12) * (2.0 / (Cin * ks * ks)) ** 0.5
    b = gen(Cout, seed=13)
    add = gen(N, Cout, H, W, seed=14) if res else None
    z = F.conv2d(x, w, b, padding=pad) + (add if res else 0)
    ref = {0: z, 1: F.relu(z), 2: F.hardtanh(z, 0.0, 6.0)}[act]
    s = S()
    xg, wg, bg = nhwc(x), w.to(DEV), b.to(DEV)
    ldk = r4(ks * ks * Cin)
    wk = torch.empty(Cout * ldk, device=DEV)
    call("seg_pack_conv_weight", wg.data_ptr(), wk.data_ptr(), Cout, Cin, ks, ldk, 0, Cin, s)
    addg = nhwc(add) if res else None
    M = N * H * W
    auto = query("seg_conv_igemm_splits", M, Cout, Cin, ks)
    outs = []
    for splits in sorted({1, auto, 3}):
        out = torch.full((M, r4(Cout)), float("nan"), device=DEV)
        work = torch.empty(max(splits * M * Cout, 1), device=DEV)
        call("seg_conv_igemm_act", xg.data_ptr(), xg.shape[1], N, H, W, Cin, wk.data_ptr(), ldk, bg.data_ptr(),
             out.data_ptr(), out.shape[1], H, W, Cout, ks, 1, pad, addg.data_ptr() if res else None,
             addg.shape[1] if res else 0, None, act, work.data_ptr(), splits, s)
        assert rel(from_nhwc(out, N, Cout, H, W), ref) < 1e-5, splits
        outs.append(out)


@pytest.mark.parametrize("stride", [1, 2])
def test_dw_bias_act_and_bn_fold(stride):
    """seg_bn_fold_batch + seg_dw_fwd_bias_act == eval BN(dwconv) + ReLU6; igemm fold likewise."""
    import numpy as np
    N, C, H, W = 2, 96, 10, 14
    x = gen(N, C, H, W, seed=21)
    w = gen(C, 1, 3, 3, seed=22) * 0.3
    g, bta = gen(C, seed=23).abs() + 0.5, gen(C, seed=24)
    rm, rv = gen(C, seed=25) * 0.1, gen(C, seed=26).abs() + 0.5
    ref = F.hardtanh(F.batch_norm(F.conv2d(x, w, None, stride=stride, padding=1, groups=C), rm, rv, g, bta, False,
                                  0.1, 1e-5), 0.0, 6.0)
    wg, gg, bg, rmg, rvg = (t.to(DEV) for t in (w, g, bta, rm, rv))
    fk = torch.empty_like(wg)
    fb = torch.zeros(C, device=DEV)
    ft = np.dtype([("w", "<u8"), ("bias", "<u8"), ("gamma", "<u8"), ("beta", "<u8"), ("rm", "<u8"), ("rv", "<u8"),
                   ("w_out", "<u8"), ("b_out", "<u8"), ("cout", "<i4"), ("kper", "<i4"), ("eps", "<f4"),
                   ("pad", "<i4")])
    job = np.array([(wg.data_ptr(), 0, gg.data_ptr(), bg.data_ptr(), rmg.data_ptr(), rvg.data_ptr(), fk.data_ptr(),
                     fb.data_ptr(), C, 9, 1e-5, 0)], dtype=ft)
    jobs = torch.from_numpy(job.view(np.uint8).copy()).to(DEV)
    call("seg_bn_fold_batch", jobs.data_ptr(), 1, C * 9 + C, S())
    wk = torch.empty(9 * C, device=DEV)
    call("seg_pack_dw_weight", fk.data_ptr(), wk.data_ptr(), C, S())
    Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
    xg = nhwc(x)
    out = torch.full((N * Ho * Wo, C), float("nan"), device=DEV)
    call("seg_dw_fwd_bias_act", xg.data_ptr(), C, N, H, W, C, wk.data_ptr(), fb.data_ptr(), 2, out.data_ptr(), C,
         Ho, Wo, stride, S())
    assert rel(from_nhwc(out, N, C, Ho, Wo), ref) < 1e-5


def _pack_wino(w, mode, rows, ldk):
    import numpy as np
    Cout, Cin = w.shape[0], w.shape[1]
    from seg_amd.engine import pack_table
    wk = torch.full((16 * rows * ldk,), float("nan"), device=DEV)
    jobs, nj, nb = pack_table([(w.data_ptr(), wk.data_ptr(), Cout, Cin, 3, ldk, mode, ldk)], DEV)
    call("seg_pack_batch", jobs.data_ptr(), nj, nb, S())
    return wk


@pytest.mark.parametrize("fused", [False, True])
@pytest.mark.parametrize("N,Cin,Cout,H,W", [(2, 64, 32, 6, 10), (1, 1344, 256, 4, 8), (2, 152, 64, 8, 6),
                                           (3, 36, 200, 2, 4), (1, 288, 128, 10, 14), (2, 80, 32, 34, 18),
                                           (1, 12, 44, 130, 6)])
def test_conv_wino_fwd_stats_dgrad(N, Cin, Cout, H, W, fused):
    """Winograd F(2x2,3x3): forward (+bias, BN partials) and data gradient (+addend) vs torch; the two-launch
    form (seg_conv_wino: 16 GEMMs + output transform through an M workspace) and the fused one (seg_conv_wino_fused:
    M in registers; row tiles crossing blocks and partial last row tiles in the shapes above)."""
    def wino(*args, stat, work):
        if fused:
            call("seg_conv_wino_fused", *args, stat, S())
        else:
            call("seg_conv_wino", *args, stat, work, S())
    x = gen(N, Cin, H, W, seed=31)
    w = gen(Cout, Cin, 3, 3, seed=32) * (2.0 / (Cin * 9)) ** 0.5
    b = gen(Cout, seed=33)
    xr = x.clone().requires_grad_(True)
    y = F.conv2d(xr, w, b, padding=1)
    dy = gen(*y.shape, seed=34)
    y.backward(dy)
    wg = w.to(DEV)
    T = N * (H // 2) * (W // 2)
    work = torch.empty(16 * T * max(Cin, Cout), device=DEV)
    # forward + BN statistics
    cin4 = r4(Cin)
    U = _pack_wino(wg, 3, Cout, cin4)
    xg = nhwc(x)
    out = torch.full((N * H * W, r4(Cout)), float("nan"), device=DEV)
    nt = query("seg_conv_wino_row_tiles", N, H, W)
    stat = torch.empty(nt * 2 * Cout, device=DEV)
    wino(xg.data_ptr(), xg.shape[1], N, H, W, cin4, U.data_ptr(), cin4, b.to(DEV).data_ptr(), out.data_ptr(),
         out.shape[1], Cout, None, 0, stat=stat.data_ptr(), work=work.data_ptr())
    assert rel(from_nhwc(out, N, Cout, H, W), y.detach()) < 1e-5
    st = torch.empty(4 * Cout, device=DEV)
    rm, rv = torch.zeros(Cout, device=DEV), torch.ones(Cout, device=DEV)
    call("seg_bn_stats_tiles", stat.data_ptr(), nt, query("seg_conv_wino_tile_rows"), N * H * W, Cout, None, None,
         1e-5, 0.1, rm.data_ptr(), rv.data_ptr(), None, st[:Cout].data_ptr(), st[Cout:2 * Cout].data_ptr(),
         st[2 * Cout:3 * Cout].data_ptr(), st[3 * Cout:].data_ptr(), S())
    y64 = y.detach().double()
    assert rel(st[:Cout], y64.mean((0, 2, 3))) < 1e-5
    assert rel(st[Cout:2 * Cout], 1 / torch.sqrt(y64.var((0, 2, 3), unbiased=False) + 1e-5)) < 1e-5
    # data gradient with a fused addend
    kin = r4(Cout)
    Ud = _pack_wino(wg, 4, Cin, kin)
    dyg = nhwc(dy)
    if Cout % 4:
        dyg[:, Cout:] = 0.0
    addend = gen(N, Cin, H, W, seed=35)
    addg = nhwc(addend)
    dx = torch.full((N * H * W, r4(Cin)), float("nan"), device=DEV)
    wino(dyg.data_ptr(), dyg.shape[1], N, H, W, kin, Ud.data_ptr(), kin, None, dx.data_ptr(), dx.shape[1], Cin,
         addg.data_ptr(), addg.shape[1], stat=None, work=work.data_ptr())
    assert rel(from_nhwc(dx, N, Cin, H, W), xr.grad + addend) < 1e-5


@pytest.mark.parametrize("N,Cin,Cout,H,W", [(2, 64, 32, 6, 10), (1, 1344, 256, 4, 8), (2, 152, 64, 8, 6),
                                           (3, 36, 200, 2, 4), (2, 80, 32, 16, 12)])
def test_conv_wino_wgrad(N, Cin, Cout, H, W):
    """Winograd F(3x3,2x2) weight gradient (split-K slabs + G^T . G reduce) vs torch."""
    x = gen(N, Cin, H, W, seed=41)
    w = gen(Cout, Cin, 3, 3, seed=42) * 0.1
    wr = w.clone().requires_grad_(True)
    y = F.conv2d(x, wr, None, padding=1)
    dy = gen(*y.shape, seed=43)
    y.backward(dy)
    cin4 = r4(Cin)
    splits = query("seg_conv_wino_wgrad_splits", N, H, W, cin4, Cout)
    part = torch.empty(splits * 16 * Cout * cin4, device=DEV)
    xg, dyg = nhwc(x), nhwc(dy)
    if Cin % 4:
        xg[:, Cin:] = 0.0
    call("seg_conv_wino_wgrad", dyg.data_ptr(), dyg.shape[1], xg.data_ptr(), xg.shape[1], N, H, W, cin4, Cout,
         part.data_ptr(), splits, S())
    dw = torch.full((Cout, Cin, 3, 3), float("nan"), device=DEV)
    call("seg_conv_wino_wgrad_reduce", part.data_ptr(), splits, dw.data_ptr(), Cout, Cin, cin4, 0, S())
    assert rel(dw, wr.grad) < 1e-5
    for s2 in (1, 3):  # any split count gives the same sums up to rounding
        p2 = torch.empty(s2 * 16 * Cout * cin4, device=DEV)
        call("seg_conv_wino_wgrad", dyg.data_ptr(), dyg.shape[1], xg.data_ptr(), xg.shape[1], N, H, W, cin4, Cout,
             p2.data_ptr(), s2, S())
        dw2 = dw.clone()
        call("seg_conv_wino_wgrad_reduce", p2.data_ptr(), s2, dw2.data_ptr(), Cout, Cin, cin4, 1, S())
        assert rel(dw2, 2 * wr.grad) < 1e-5


@pytest.mark.parametrize("N,Cin,Cout,H,W", [(2, 64, 32, 6, 10), (1, 1344, 256, 4, 8), (2, 152, 64, 8, 6),
                                           (3, 36, 200, 2, 4), (2, 80, 32, 16, 12), (2, 128, 192, 10, 8),
                                           (1, 288, 128, 12, 14), (4, 32, 32, 2, 2)])
def test_conv_wino_wgrad16(N, Cin, Cout, H, W):
    """seg_conv_wino_wgrad16 (all 16 points per block): bitwise the per-point kernel's slabs at the same split
    count (up to the sign of zero), and dW vs torch."""
    x = gen(N, Cin, H, W, seed=44)
    w = gen(Cout, Cin, 3, 3, seed=45) * 0.1
    wr = w.clone().requires_grad_(True)
    y = F.conv2d(x, wr, None, padding=1)
    dy = gen(*y.shape, seed=46)
    y.backward(dy)
    cin4 = r4(Cin)
    xg, dyg = nhwc(x), nhwc(dy)
    if Cin % 4:
        xg[:, Cin:] = 0.0
    splits = query("seg_conv_wino_wgrad16_splits", N, H, W, cin4, Cout)
    for sp in sorted({splits, 1, 3, 40}):  # 40: the reduce folds runs of slabs in place first
        p16 = torch.full((sp * 16 * Cout * cin4,), float("nan"), device=DEV)
        ref = torch.full_like(p16, float("nan"))
        call("seg_conv_wino_wgrad16", dyg.data_ptr(), dyg.shape[1], xg.data_ptr(), xg.shape[1], N, H, W, cin4, Cout,
             p16.data_ptr(), sp, S())
        call("seg_conv_wino_wgrad", dyg.data_ptr(), dyg.shape[1], xg.data_ptr(), xg.shape[1], N, H, W, cin4, Cout,
             ref.data_ptr(), sp, S())
        assert torch.equal(p16, ref), (sp, (p16 - ref).abs().max().item())
        dw = torch.full((Cout, Cin, 3, 3), float("nan"), device=DEV)
        call("seg_conv_wino_wgrad_reduce", p16.data_ptr(), sp, dw.data_ptr(), Cout, Cin, cin4, 0, S())
        assert rel(dw, wr.grad) < 1e-5


@pytest.mark.parametrize("N,Cin,Cout,H,W,mode", [(2, 80, 32, 8, 64, 0), (1, 32, 32, 4, 128, 0),
                                                 (2, 152, 64, 4, 64, 0), (1, 64, 64, 12, 64, 0),
                                                 (2, 32, 80, 8, 64, 1), (1, 20, 96, 4, 128, 0)])
def test_conv_halo(N, Cin, Cout, H, W, mode):
    """seg_conv_halo == torch conv2d (forward + bias + BN partials, or data gradient + addend)."""
    x = gen(N, Cin, H, W, seed=71)
    w = gen(Cout, Cin, 3, 3, seed=72) * (2.0 / (Cin * 9)) ** 0.5
    b = gen(Cout, seed=73)
    s = S()
    wg = w.to(DEV)
    if mode == 0:
        ref = F.conv2d(x, w, b, padding=1)
        cin4 = r4(Cin)
        ldk = r4(9 * cin4)
        wk = torch.empty(Cout * ldk, device=DEV)
        call("seg_pack_conv_weight", wg.data_ptr(), wk.data_ptr(), Cout, Cin, 3, ldk, 0, cin4, s)
        xg = nhwc(x)
        if Cin % 4:
            xg[:, Cin:] = 0.0
        out = torch.full((N * H * W, r4(Cout)), float("nan"), device=DEV)
        nt = query("seg_conv_halo_row_tiles", N, H, W)
        stat = torch.empty(nt * 2 * Cout, device=DEV)
        call("seg_conv_halo", xg.data_ptr(), xg.shape[1], N, H, W, cin4, wk.data_ptr(), ldk, b.to(DEV).data_ptr(),
             out.data_ptr(), out.shape[1], Cout, None, 0, stat.data_ptr(), s)
        assert rel(from_nhwc(out, N, Cout, H, W), ref) < 1e-5
        st = torch.empty(4 * Cout, device=DEV)
        rm, rv = torch.zeros(Cout, device=DEV), torch.ones(Cout, device=DEV)
        call("seg_bn_stats_tiles", stat.data_ptr(), nt, 256, N * H * W, Cout, None, None, 1e-5, 0.1, rm.data_ptr(),
             rv.data_ptr(), None, st[:Cout].data_ptr(), st[Cout:2 * Cout].data_ptr(), st[2 * Cout:3 * Cout].data_ptr(),
             st[3 * Cout:].data_ptr(), s)
        assert rel(st[:Cout], ref.double().mean((0, 2, 3))) < 1e-5
    else:  # data gradient: dY has Cin channels here, dX has Cout
        xr = torch.zeros(N, Cout, H, W, requires_grad=True)
        wt = gen(Cin, Cout, 3, 3, seed=74) * 0.1   # forward conv Cout'=Cin <- Cin'=Cout
        y = F.conv2d(xr, wt, None, padding=1)
        dy = x
        y.backward(dy)
        kin = r4(Cin)
        ldk = r4(9 * kin)
        wkd = torch.empty(Cout * ldk, device=DEV)
        call("seg_pack_conv_weight", wt.to(DEV).data_ptr(), wkd.data_ptr(), Cin, Cout, 3, ldk, 1, kin, s)
        addend = gen(N, Cout, H, W, seed=75)
        addg = nhwc(addend)
        dx = torch.full((N * H * W, r4(Cout)), float("nan"), device=DEV)
        call("seg_conv_halo", nhwc(dy).data_ptr(), r4(Cin), N, H, W, kin, wkd.data_ptr(), ldk, None, dx.data_ptr(),
             dx.shape[1], Cout, addg.data_ptr(), addg.shape[1], None, s)
        assert rel(from_nhwc(dx, N, Cout, H, W), xr.grad + addend) < 1e-5


@pytest.mark.parametrize("mode,Cout,Cin,ks", [(0, 10, 32, 1), (0, 10, 30, 3), (1, 32, 1, 3)])
@pytest.mark.parametrize("splits", [17, 100, 257, 1024])
def test_wgrad_reduce_direct(mode, Cout, Cin, ks, splits):
    """seg_conv_wgrad_reduce on small slabs with many splits: the path that spreads the
    split dimension over up to 64 thread groups (E < 64) with a pairwise LDS tree.
    Against an fp64 sum of the slabs, and bitwise reproducible."""
    cp = r4(Cin) if mode == 0 else Cin
    taps = ks * ks
    g = torch.Generator().manual_seed(splits + Cout)
    if mode == 0:
        part = torch.randn(splits, Cout, taps, cp, generator=g)
        ref = part.double().sum(0)[..., :Cin].permute(0, 2, 1).reshape(Cout, Cin, ks, ks)
    else:
        part = torch.randn(splits, taps, Cout, generator=g)
        ref = part.double().sum(0).t().reshape(Cout, 1, ks, ks)
    s = S()
    pg = part.to(DEV)
    outs = []
    for acc in (0, 0, 1):
        out = torch.zeros(Cout, Cin, ks, ks, device=DEV) if acc == 0 else outs[0].clone()
        call("seg_conv_wgrad_reduce", pg.data_ptr(), splits, out.data_ptr(), Cout, Cin, ks, mode, acc, s)
        torch.cuda.synchronize()
        outs.append(out)
    assert torch.equal(outs[0], outs[1]), "fixed-order reduction must be bitwise reproducible"
    err = float((outs[0].double().cpu() - ref).abs().max())
    assert err <= 1e-5 * splits ** 0.5 * float(ref.abs().max() + 1), err
    assert torch.equal(outs[2], outs[0] + outs[0])


@pytest.mark.parametrize("M,C", [(262144, 96), (65536, 1280), (100, 12)])
def test_reduction_finalize_repeatable_under_load(M, C):
    """The channel reductions (fixed-order partials + one-round-trip fp64 finalize kernels):
    reusing one workspace call after call -- with a large GEMM running on another stream,
    so blocks run in uneven orders -- must give bitwise the same statistics, BN backward
    and column sums every time, and results equal to fp64 torch."""
    y = (gen(M, C, seed=11) * 2 + 1).to(DEV)
    da = gen(M, C, seed=12).to(DEV)
    gamma, beta = torch.ones(C, device=DEV), torch.zeros(C, device=DEV)
    work = torch.zeros(query("seg_chan_workspace_floats", M, C) + 3 * C, device=DEV)
    other = torch.cuda.Stream()
    big = torch.randn(4096, 4096, device=DEV)
    outs = []
    for rep in range(6):
        with torch.cuda.stream(other):
            if rep % 2:
                torch.mm(big, big)  # uneven load on part of the chip while the reduction runs
        s = S()
        st = torch.empty(4 * C, device=DEV)
        call("seg_bn_stats", y.data_ptr(), C, M, C, gamma.data_ptr(), beta.data_ptr(), 1e-5, 0.1, None, None, None,
             work.data_ptr(), st[0:C].data_ptr(), st[C:2 * C].data_ptr(), st[2 * C:3 * C].data_ptr(),
             st[3 * C:].data_ptr(), s)
        dg, db, dy = torch.empty(C, device=DEV), torch.empty(C, device=DEV), torch.empty(M, C, device=DEV)
        call("seg_bn_backward", da.data_ptr(), C, y.data_ptr(), C, M, C, gamma.data_ptr(), st[0:C].data_ptr(),
             st[C:2 * C].data_ptr(), st[2 * C:3 * C].data_ptr(), st[3 * C:].data_ptr(), 1, dg.data_ptr(),
             db.data_ptr(), work.data_ptr(), dy.data_ptr(), C, s)
        cs = torch.empty(C, device=DEV)
        call("seg_colsum", da.data_ptr(), C, M, C, work.data_ptr(), cs.data_ptr(), 0, s)
        torch.cuda.synchronize()
        outs.append((st.clone(), dg.clone(), db.clone(), dy.clone(), cs.clone()))
    for o in outs[1:]:
        for a, b in zip(outs[0], o):
            assert torch.equal(a, b)
    y64, d64 = y.double().cpu(), da.double().cpu()
    st, dg, db, dy, cs = outs[0]
    assert rel(st[:C], y64.mean(0)) < 1e-6
    assert rel(st[C:2 * C], 1 / torch.sqrt(y64.var(0, unbiased=False) + 1e-5)) < 1e-6
    assert rel(cs, d64.sum(0)) < 1e-5
    z = (y64 - y64.mean(0)) * (1 / torch.sqrt(y64.var(0, unbiased=False) + 1e-5))
    dz = d64 * (z > 0)
    assert rel(db, dz.sum(0)) < 1e-5 and rel(dg, (dz * z).sum(0)) < 1e-5


@pytest.mark.parametrize("M,tile_rows,C", [(1025 * 256, 256, 64), (4096 * 128 + 77, 128, 24), (20000 * 256 - 5, 256, 8),
                                           (1000 * 256, 256, 32)])
def test_bn_stats_tiles_merged(M, tile_rows, C):
    """seg_bn_stats_tiles_ws (many-tile layers: 16 tiles merged per row, then the per-channel finalize)
    against fp64 torch statistics of the same rows, and against the direct finalize; a short last tile
    and a short last super-tile included."""
    g = torch.Generator().manual_seed(M % 1000)
    y = (torch.randn(M, C, generator=g, dtype=torch.float64) * torch.linspace(0.5, 3, C, dtype=torch.float64)
         + torch.linspace(-2, 5, C, dtype=torch.float64))
    nt = (M + tile_rows - 1) // tile_rows
    pad = nt * tile_rows - M
    yt = torch.cat([y, torch.full((pad, C), float("nan"), dtype=torch.float64)]).view(nt, tile_rows, C)
    n = torch.full((nt, 1), float(tile_rows), dtype=torch.float64)
    n[-1] = tile_rows - pad
    valid = ~torch.isnan(yt)
    s = torch.where(valid, yt, 0.0).sum(1)
    m2 = torch.where(valid, (yt - (s / n)[:, None, :]) ** 2, 0.0).sum(1)
    part = torch.stack([s, m2], 1).float().to(DEV).contiguous()  # [nt][2][C]
    nw = query("seg_bn_stats_tiles_work_floats", nt, C)
    assert (nw > 0) == (nt > 1024)
    work = torch.empty(max(nw, 1), device=DEV)
    res = {}
    for name, extra in (("seg_bn_stats_tiles", ()), ("seg_bn_stats_tiles_ws", (work.data_ptr() if nw else None,))):
        st = torch.empty(4 * C, device=DEV)
        rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
        call(name, part.data_ptr(), nt, tile_rows, M, C, None, None, 1e-5, 0.1, rm.data_ptr(), rv.data_ptr(), None,
             st[:C].data_ptr(), st[C:2 * C].data_ptr(), st[2 * C:3 * C].data_ptr(), st[3 * C:].data_ptr(), *extra, S())
        res[name] = (st.double().cpu(), rm.double().cpu(), rv.double().cpu())
    mean, var = y.mean(0), y.var(0, unbiased=False)
    for name, (st, rm, rv) in res.items():
        assert rel(st[:C], mean) < 1e-6, name
        assert rel(st[C:2 * C], 1 / torch.sqrt(var + 1e-5)) < 1e-6, name
        assert rel(rv, 0.9 + 0.1 * y.var(0, unbiased=True)) < 1e-6, name
    a, b = res["seg_bn_stats_tiles"][0], res["seg_bn_stats_tiles_ws"][0]
    assert rel(a, b) < 1e-6
