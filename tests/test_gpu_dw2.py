"""GPU: seg_dw2_*_bf16io -- the LDS-DMA tile kernels for the depthwise 3x3 convs of the bf16io
configuration (csrc/dw2.hip; the groups=C Conv2d of torchvision's InvertedResidual, reached
through src/unet.py:15-19,34-38, and its convolution_backward).

  * forward without lazy BN and data gradient: equal, bit for bit, to dwconv.hip's strip
    kernels (seg_dw_fwd_bf16io / seg_dw_dgrad_bf16io: the same fp32 tap order), stride 1 and 2,
    accumulate on / off, ragged images (partial tiles), C not a multiple of the 64-channel slice,
    row strides wider than C (channel slices of a concat buffer);
  * forward with lazy BN: against float64 of the bf16-rounded transformed input;
  * BN tile partials of the forward: every tile's sum and M2 against float64 of the output
    tile, and the finalized mean / variance;
  * weight gradient: against float64 (fp32 accumulation) and against seg_dw_wgrad_bf16io;
    repeat launches bitwise equal (fixed-order slabs, no atomics);
  * seg_dw2_ok / seg_dw2_stat_tiles refuse what the kernels cannot do.
"""
import ctypes

import pytest
import torch
import torch.nn.functional as F

from seg_amd._lib import call, query

pytestmark = pytest.mark.gpu
DEV = "cuda"
BF = torch.bfloat16


def S():
    return torch.cuda.current_stream().cuda_stream


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


def outsz(H, s):
    return (H - 1) // s + 1


def rows(M, ld, seed, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(M, ld, generator=g) * scale).to(BF).to(DEV)


def packw(C, seed):
    g = torch.Generator().manual_seed(seed)
    w = (torch.randn(C, 1, 3, 3, generator=g) * 0.3).to(DEV)
    wk = torch.empty(9 * C, device=DEV)
    call("seg_pack_dw_weight", w.data_ptr(), wk.data_ptr(), C, S())
    return w, wk


def nchw(x, N, H, W, C, ld):
    return x.view(N, H, W, ld)[..., :C].permute(0, 3, 1, 2).double().cpu()


CASES = [  # N, C, H, W, stride, ld (>= C)
    (2, 64, 16, 64, 1, 64), (2, 64, 16, 64, 2, 64), (1, 72, 13, 40, 1, 80), (1, 72, 13, 40, 2, 72),
    (3, 8, 9, 33, 1, 16), (2, 136, 8, 32, 2, 136), (2, 144, 32, 64, 1, 144), (1, 960, 8, 16, 1, 960),
    (4, 192, 32, 64, 2, 192),
]


@pytest.mark.parametrize("N,C,H,W,s,ld", CASES)
def test_dw2_fwd_equals_strip_kernel(N, C, H, W, s, ld):
    Ho, Wo = outsz(H, s), outsz(W, s)
    x = rows(N * H * W, ld, N * H + C)
    _, wk = packw(C, C)
    outs = {}
    for name in ("seg_dw2_fwd_bf16io", "seg_dw_fwd_bf16io"):
        o = torch.full((N * Ho * Wo, ld), 5.0, device=DEV, dtype=BF)
        extra = (None,) if name.startswith("seg_dw2") else ()
        call(name, x.data_ptr(), ld, N, H, W, C, None, None, 0, wk.data_ptr(), o.data_ptr(), ld, Ho, Wo, s, *extra,
             S())
        outs[name] = o
    torch.cuda.synchronize()
    a, b = outs["seg_dw2_fwd_bf16io"], outs["seg_dw_fwd_bf16io"]
    assert torch.equal(a, b), f"max diff {(a.float() - b.float()).abs().max().item()}"
    if ld > C:
        assert bool((a[:, C:] == 5.0).all()), "channels beyond C untouched"


@pytest.mark.parametrize("N,C,H,W,s,ld", CASES[:6])
@pytest.mark.parametrize("acc", [0, 1])
def test_dw2_dgrad_equals_strip_kernel(N, C, H, W, s, ld, acc):
    Ho, Wo = outsz(H, s), outsz(W, s)
    dy = rows(N * Ho * Wo, ld, 3 * C + H)
    _, wk = packw(C, C + 1)
    base = rows(N * H * W, ld, 7 + W)
    outs = {}
    for name in ("seg_dw2_dgrad_bf16io", "seg_dw_dgrad_bf16io"):
        dx = base.clone()
        call(name, dy.data_ptr(), ld, N, Ho, Wo, C, wk.data_ptr(), dx.data_ptr(), ld, H, W, s, acc, S())
        outs[name] = dx
    torch.cuda.synchronize()
    a, b = outs["seg_dw2_dgrad_bf16io"], outs["seg_dw_dgrad_bf16io"]
    assert torch.equal(a, b), f"max diff {(a.float() - b.float()).abs().max().item()}"


def bn_xform(x, N, H, W, C, ld, sc, sh, act):
    v = nchw(x, N, H, W, C, ld) * sc.double().cpu().view(1, C, 1, 1) + sh.double().cpu().view(1, C, 1, 1)
    if act == 1:
        v = v.clamp(min=0)
    elif act == 2:
        v = v.clamp(0, 6)
    return v.float().to(BF).double()  # rounded to bf16 as the BN-apply pass stores it


@pytest.mark.parametrize("N,C,H,W,s,ld", [(2, 64, 16, 64, 1, 64), (2, 72, 13, 40, 2, 80), (2, 192, 32, 64, 2, 192)])
def test_dw2_fwd_lazy_bn_and_tile_stats(N, C, H, W, s, ld):
    Ho, Wo = outsz(H, s), outsz(W, s)
    x = rows(N * H * W, ld, 11 + C)
    w, wk = packw(C, 2 * C)
    g = torch.Generator().manual_seed(C)
    sc = (torch.rand(C, generator=g) + 0.5).to(DEV)
    sh = (torch.randn(C, generator=g) * 0.5).to(DEV)
    tr = ctypes.c_int(0)
    nt = query("seg_dw2_stat_tiles", N, Ho, Wo, s, ctypes.addressof(tr))
    stat = torch.full((max(nt, 1) * 2 * C,), float("nan"), device=DEV)
    o = torch.empty(N * Ho * Wo, ld, device=DEV, dtype=BF)
    call("seg_dw2_fwd_bf16io", x.data_ptr(), ld, N, H, W, C, sc.data_ptr(), sh.data_ptr(), 2, wk.data_ptr(),
         o.data_ptr(), ld, Ho, Wo, s, stat.data_ptr() if nt else None, S())
    torch.cuda.synchronize()
    ref = F.conv2d(bn_xform(x, N, H, W, C, ld, sc, sh, 2), w.double().cpu(), stride=s, padding=1, groups=C)
    got = nchw(o, N, Ho, Wo, C, ld)
    assert rel(got, ref) < 4e-3  # one bf16 rounding of the output
    assert float((got - ref).abs().max()) <= float(ref.abs().max()) * 2 ** -7
    if not nt:
        return
    tho, two = tr.value // 32, 32
    st = stat.view(nt, 2, C).double().cpu()
    tw, th = Wo // two, Ho // tho
    for t in range(nt):
        n, r = divmod(t, th * tw)
        hi, wi = divmod(r, tw)
        blk = ref[n, :, hi * tho:(hi + 1) * tho, wi * two:(wi + 1) * two].reshape(C, -1)
        sm = blk.sum(1)
        m2 = ((blk - sm[:, None] / blk.shape[1]) ** 2).sum(1)
        assert torch.allclose(st[t, 0], sm, rtol=1e-3, atol=1e-2 * float(blk.abs().mean()) + 1e-3), t
        assert torch.allclose(st[t, 1], m2, rtol=1e-3, atol=1e-3), t


@pytest.mark.parametrize("N,C,H,W,s,ld,lazy", [
    (2, 64, 16, 64, 1, 64, False), (2, 64, 16, 64, 2, 64, True), (1, 72, 13, 40, 1, 80, True),
    (1, 72, 13, 40, 2, 72, False), (3, 8, 9, 33, 1, 16, False), (8, 144, 64, 128, 1, 144, True),
    (8, 960, 8, 16, 1, 960, False), (8, 384, 16, 32, 2, 384, True),
])
def test_dw2_wgrad_vs_fp64_and_strip_kernel(N, C, H, W, s, ld, lazy):
    Ho, Wo = outsz(H, s), outsz(W, s)
    x = rows(N * H * W, ld, 5 + C + H)
    dy = rows(N * Ho * Wo, ld, 9 + C + W)
    g = torch.Generator().manual_seed(C + 1)
    sc = (torch.rand(C, generator=g) + 0.5).to(DEV)
    sh = (torch.randn(C, generator=g) * 0.5).to(DEV)
    xf = (sc.data_ptr(), sh.data_ptr(), 2) if lazy else (None, None, 0)
    blocks = query("seg_dw2_wgrad_blocks", N, Ho, Wo, C, s, 0)
    part = torch.full((blocks * 9 * C,), float("nan"), device=DEV)
    outs = []
    for _ in range(2):
        dw = torch.empty(C, 1, 3, 3, device=DEV)
        call("seg_dw2_wgrad_bf16io", dy.data_ptr(), ld, x.data_ptr(), ld, N, H, W, C, *xf, Ho, Wo, s, part.data_ptr(),
             S())
        call("seg_conv_wgrad_reduce", part.data_ptr(), blocks, dw.data_ptr(), C, 1, 3, 1, 0, S())
        outs.append(dw)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1]), "deterministic"
    xin = bn_xform(x, N, H, W, C, ld, sc, sh, 2) if lazy else nchw(x, N, H, W, C, ld)
    ref = torch.nn.grad.conv2d_weight(xin, (C, 1, 3, 3), nchw(dy, N, Ho, Wo, C, ld), stride=s, padding=1, groups=C)
    assert rel(outs[0], ref) < 1e-5
    if not lazy:  # dwconv.hip's strip kernel (its lazy path keeps the transformed input in fp32)
        nb = query("seg_dw_wgrad_blocks", N, Ho, Wo, C)
        p2 = torch.empty(nb * 9 * C, device=DEV)
        dw2 = torch.empty(C, 1, 3, 3, device=DEV)
        call("seg_dw_wgrad_bf16io", dy.data_ptr(), ld, x.data_ptr(), ld, N, H, W, C, None, None, 0, Ho, Wo, s,
             p2.data_ptr(), S())
        call("seg_conv_wgrad_reduce", p2.data_ptr(), nb, dw2.data_ptr(), C, 1, 3, 1, 0, S())
        torch.cuda.synchronize()
        assert rel(outs[0], dw2) < 1e-5


def test_dw2_refuses_what_it_cannot_do():
    assert query("seg_dw2_ok", 64, 1) == 1 and query("seg_dw2_ok", 64, 2) == 1
    assert query("seg_dw2_ok", 36, 1) == 0   # C % 8
    assert query("seg_dw2_ok", 64, 3) == 0   # stride
    tr = ctypes.c_int(0)
    assert query("seg_dw2_stat_tiles", 2, 64, 128, 1, ctypes.addressof(tr)) == 2 * 8 * 4 and tr.value == 256
    assert query("seg_dw2_stat_tiles", 2, 64, 128, 2, ctypes.addressof(tr)) == 2 * 16 * 4 and tr.value == 128
    assert query("seg_dw2_stat_tiles", 32, 8, 16, 1, None) == 0   # Wo % 32: statistics from seg_bn_stats
    x = torch.zeros(64, 64, device=DEV, dtype=BF)
    with pytest.raises(Exception):  # stat requested where the tiles do not divide the image
        call("seg_dw2_fwd_bf16io", x.data_ptr(), 64, 1, 8, 8, 64, None, None, 0, x.data_ptr(), x.data_ptr(), 64, 8, 8,
             1, x.data_ptr(), S())


# ---- the BatchNorm-backward fusions (seg_dw2_dgrad_bn_bf16io / seg_dw2_wgrad_bn_bf16io) ----

def bn_state(C, seed):
    """Per-channel (mean, invstd, scale, shift, gamma, coef[3][C]) of a plausible train-mode BN."""
    g = torch.Generator().manual_seed(seed)
    mean = torch.randn(C, generator=g) * 0.3
    invstd = torch.rand(C, generator=g) + 0.5
    gamma = torch.rand(C, generator=g) + 0.5
    beta = torch.randn(C, generator=g) * 0.2
    scale, shift = gamma * invstd, beta - mean * gamma * invstd
    coef = torch.cat([gamma * invstd, torch.randn(C, generator=g) * 0.05, torch.randn(C, generator=g) * 0.05])
    return [t.to(DEV) for t in (mean, invstd, scale, shift, gamma, coef)]


BN_CASES = [  # N, C, H, W, stride, ld
    (2, 64, 16, 64, 1, 64), (2, 64, 16, 64, 2, 64), (1, 72, 13, 40, 1, 80), (1, 72, 13, 40, 2, 72),
    (4, 192, 32, 64, 1, 192), (8, 960, 8, 16, 1, 960), (4, 144, 32, 64, 2, 144),
]


@pytest.mark.parametrize("N,C,H,W,s,ld", BN_CASES)
def test_dw2_dgrad_bin_equals_apply_then_dgrad(N, C, H, W, s, ld):
    """BIN: dY formed on load is bitwise the seg_bn_bwd_apply pass's stored dY."""
    Ho, Wo = outsz(H, s), outsz(W, s)
    da = rows(N * Ho * Wo, ld, 21 + C)
    y = rows(N * Ho * Wo, ld, 22 + C, 2.0)
    mean, invstd, scale, shift, gamma, coef = bn_state(C, C)
    _, wk = packw(C, C + 3)
    dy = torch.full((N * Ho * Wo, ld), 0.0, device=DEV, dtype=BF)
    call("seg_bn_bwd_apply_bf16io", da.data_ptr(), ld, y.data_ptr(), ld, N * Ho * Wo, C, mean.data_ptr(),
         scale.data_ptr(), shift.data_ptr(), 2, coef.data_ptr(), dy.data_ptr(), ld, S())
    ref = torch.zeros(N * H * W, ld, device=DEV, dtype=BF)
    call("seg_dw2_dgrad_bf16io", dy.data_ptr(), ld, N, Ho, Wo, C, wk.data_ptr(), ref.data_ptr(), ld, H, W, s, 0, S())
    got = torch.zeros(N * H * W, ld, device=DEV, dtype=BF)
    call("seg_dw2_dgrad_bn_bf16io", da.data_ptr(), ld, N, Ho, Wo, C, wk.data_ptr(), got.data_ptr(), ld, H, W, s, 0,
         y.data_ptr(), ld, scale.data_ptr(), shift.data_ptr(), mean.data_ptr(), coef.data_ptr(), 2,
         None, 0, None, None, None, None, None, 0, None, None, None, None, None, S())
    torch.cuda.synchronize()
    assert torch.equal(got, ref), f"max diff {(got.float() - ref.float()).abs().max().item()}"


@pytest.mark.parametrize("N,C,H,W,s,ld", BN_CASES)
def test_dw2_wgrad_bin_vs_apply_then_wgrad(N, C, H, W, s, ld):
    Ho, Wo = outsz(H, s), outsz(W, s)
    x = rows(N * H * W, ld, 31 + C)
    da = rows(N * Ho * Wo, ld, 32 + C)
    y = rows(N * Ho * Wo, ld, 33 + C, 2.0)
    mean, invstd, scale, shift, gamma, coef = bn_state(C, C + 5)
    dy = torch.zeros(N * Ho * Wo, ld, device=DEV, dtype=BF)
    call("seg_bn_bwd_apply_bf16io", da.data_ptr(), ld, y.data_ptr(), ld, N * Ho * Wo, C, mean.data_ptr(),
         scale.data_ptr(), shift.data_ptr(), 2, coef.data_ptr(), dy.data_ptr(), ld, S())
    outs = {}
    for bin_ in (0, 1):
        blocks = query("seg_dw2_wgrad_blocks", N, Ho, Wo, C, s, bin_)
        part = torch.full((blocks * 9 * C,), float("nan"), device=DEV)
        dw = torch.empty(C, 1, 3, 3, device=DEV)
        src = da if bin_ else dy
        b = (y.data_ptr(), ld, scale.data_ptr(), shift.data_ptr(), mean.data_ptr(), coef.data_ptr(), 2) if bin_ else \
            (None, 0, None, None, None, None, 0)
        call("seg_dw2_wgrad_bn_bf16io", src.data_ptr(), ld, x.data_ptr(), ld, N, H, W, C, None, None, 0, Ho, Wo, s,
             part.data_ptr(), *b, S())
        call("seg_conv_wgrad_reduce", part.data_ptr(), blocks, dw.data_ptr(), C, 1, 3, 1, 0, S())
        outs[bin_] = dw
    torch.cuda.synchronize()
    ref = torch.nn.grad.conv2d_weight(nchw(x, N, H, W, C, ld), (C, 1, 3, 3), nchw(dy, N, Ho, Wo, C, ld), stride=s,
                                      padding=1, groups=C)
    assert rel(outs[0], ref) < 1e-5 and rel(outs[1], ref) < 1e-5
    if s == 2:  # the same tiles with and without BIN: the same sums
        assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("N,C,H,W,s,ld", BN_CASES)
@pytest.mark.parametrize("bin_", [False, True])
def test_dw2_dgrad_bout_partials_and_finalize(N, C, H, W, s, ld, bin_):
    """BOUT: dX unchanged; the producer's BN-backward reduction from the epilogue matches
    seg_bn_bwd_coef_bf16io over the stored dX (fp32 partials, other grouping: rel 1e-5), repeat
    launches (re-armed counters) are bitwise equal."""
    Ho, Wo = outsz(H, s), outsz(W, s)
    dyin = rows(N * Ho * Wo, ld, 41 + C)
    yb = rows(N * Ho * Wo, ld, 42 + C, 2.0)
    oy = rows(N * H * W, ld, 43 + C, 2.0)
    _, wk = packw(C, C + 7)
    bm, _, bsc, bsh, _, bk = bn_state(C, C + 11)
    om, oinv, osc, osh, og, _ = bn_state(C, C + 13)
    b = (yb.data_ptr(), ld, bsc.data_ptr(), bsh.data_ptr(), bm.data_ptr(), bk.data_ptr(), 2) if bin_ else \
        (None, 0, None, None, None, None, 0)
    ref = torch.zeros(N * H * W, ld, device=DEV, dtype=BF)
    call("seg_dw2_dgrad_bn_bf16io", dyin.data_ptr(), ld, N, Ho, Wo, C, wk.data_ptr(), ref.data_ptr(), ld, H, W, s, 0,
         *b, None, 0, None, None, None, None, None, 0, None, None, None, None, None, S())
    tiles = query("seg_dw2_dgrad_tiles", N, H, W)
    part = torch.full((tiles * 2 * C,), float("nan"), device=DEV)
    cnt = torch.zeros((C + 63) // 64, device=DEV, dtype=torch.int32)
    res = []
    for _ in range(2):
        dx = torch.zeros(N * H * W, ld, device=DEV, dtype=BF)
        coef = torch.full((3 * C,), float("nan"), device=DEV)
        dg, db = torch.full((C,), float("nan"), device=DEV), torch.full((C,), float("nan"), device=DEV)
        call("seg_dw2_dgrad_bn_bf16io", dyin.data_ptr(), ld, N, Ho, Wo, C, wk.data_ptr(), dx.data_ptr(), ld, H, W, s,
             0, *b, oy.data_ptr(), ld, osc.data_ptr(), osh.data_ptr(), om.data_ptr(), og.data_ptr(), oinv.data_ptr(), 2,
             part.data_ptr(), dg.data_ptr(), db.data_ptr(), coef.data_ptr(), cnt.data_ptr(), S())
        res.append((dx, coef, dg, db))
    torch.cuda.synchronize()
    assert torch.equal(res[0][0], ref)
    for a, c in zip(res[0][1:], res[1][1:]):
        assert torch.equal(a, c), "deterministic"
    assert int(cnt.abs().sum()) == 0, "counters re-armed"
    work = torch.empty(query("seg_chan_workspace_floats", N * H * W, C), device=DEV)
    coef2 = torch.empty(3 * C, device=DEV)
    dg2, db2 = torch.empty(C, device=DEV), torch.empty(C, device=DEV)
    call("seg_bn_bwd_coef_bf16io", ref.data_ptr(), ld, oy.data_ptr(), ld, N * H * W, C, og.data_ptr(), om.data_ptr(),
         oinv.data_ptr(), osc.data_ptr(), osh.data_ptr(), 2, dg2.data_ptr(), db2.data_ptr(), work.data_ptr(),
         coef2.data_ptr(), S())
    torch.cuda.synchronize()
    _, coef, dg, db = res[0]
    assert rel(coef, coef2) < 1e-5 and rel(dg, dg2) < 1e-5 and rel(db, db2) < 1e-5
