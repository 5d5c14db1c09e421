"""GPU: BatchNorm backward formed on load ("bwx", include/segamd.h) -- every seg_*_bwx consumer against the
apply pass followed by the plain consumer.

The conv after which a train-mode BatchNorm sits needs dY = seg_bnbwd4(dA, y) for its data gradient and its
weight gradient (the backward of src/unet.py:57-63 / torchvision's Conv2dNormActivation via src/unet.py:15-19,
driven by loss.backward() at src/train.py:38).  The bwx entries form dY in their operand loaders from dA, the
raw conv output y and the layer's st[7][C] planes, rounding it to bf16 where the apply pass stores bf16, so
every output (data gradients, BN-backward tile partials, weight-gradient partial slabs) must be BITWISE the
apply-then-consumer result.  Model-level parity with bwx on: tests/test_gpu_model.py, test_gpu_bf16io.py.
"""
import pytest
import torch

from seg_amd._lib import call, query

pytestmark = pytest.mark.gpu
DEV = "cuda"
BF = torch.bfloat16


def S():
    return torch.cuda.current_stream().cuda_stream


def _t(rows, ld, seed, dt, scale=1.0, shift=0.0):
    g = torch.Generator().manual_seed(seed)
    x = (torch.randn(rows, ld, generator=g) * scale + shift).to(BF).float()  # bf16-representable
    return x.to(DEV).to(dt).contiguous()


def _layer(M, C, ldy, ldda, dt, seed):
    """(y, dA, st[7][C]) of a BN layer: raw output, upstream gradient, statistics + backward coefficients."""
    y = _t(M, ldy, seed, dt, 1.7, 0.4)
    dA = _t(M, ldda, seed + 1, dt)
    g = torch.Generator().manual_seed(seed + 2)
    mean = torch.randn(C, generator=g) * 0.3
    invstd = torch.rand(C, generator=g) + 0.5
    scale = torch.randn(C, generator=g) * invstd * 2.0  # some negative: both mask edges exercised
    shift = torch.randn(C, generator=g) * 2.0 + 1.0
    k = torch.randn(3, C, generator=g)
    st = torch.cat([mean, invstd, scale, shift, k.reshape(-1)]).to(DEV).float().contiguous()
    return y, dA, st


def _apply(y, dA, st, C, act, dt):
    """dY from the apply pass (seg_bn_bwd_apply*), [M][r4(C)]."""
    M = y.shape[0]
    b = st.data_ptr()
    dy = torch.zeros(M, C, device=DEV, dtype=dt)
    call("seg_bn_bwd_apply_bf16io" if dt == BF else "seg_bn_bwd_apply", dA.data_ptr(), dA.shape[1], y.data_ptr(),
         y.shape[1], M, C, b, b + 8 * C, b + 12 * C, act, b + 16 * C, dy.data_ptr(), C, S())
    return dy


MATHS = {"f32": torch.float32, "bf16io": BF}


@pytest.mark.parametrize("math", list(MATHS))
@pytest.mark.parametrize("act", [0, 1, 2])
@pytest.mark.parametrize("N,H,W,C,Cout,ks,pad_ld", [(2, 16, 24, 96, 16, 1, 0), (1, 9, 13, 144, 24, 1, 8),
                                                    (2, 8, 8, 1280, 320, 1, 0), (2, 12, 20, 64, 80, 3, 8),
                                                    (1, 7, 9, 32, 152, 3, 0), (2, 16, 16, 384, 64, 1, 16)])
@pytest.mark.parametrize("bnout", [False, True])
def test_igemm_dgrad_bwx(math, act, N, H, W, C, Cout, ks, pad_ld, bnout):
    dt = MATHS[math]
    if not query("seg_conv_igemm_bwx_ok", C, ks, int(dt == BF)):
        pytest.skip("not a uniform-tap data gradient")
    M = N * H * W
    s = S()
    y, dA, st = _layer(M, C, C + pad_ld, C + pad_ld, dt, 10)
    dy = _apply(y, dA, st, C, act, dt)
    K = ks * ks * C
    ldk = (K + 7) & ~7
    g = torch.Generator().manual_seed(5)
    wk = (torch.randn(Cout, ldk, generator=g) * 0.05).to(DEV)
    if dt == BF:
        wk = wk.to(BF)
    add = _t(M, Cout, 7, dt)
    # BN partials of the output (the producer layer's BN backward, seg_conv_igemm_bnout)
    by = _t(M, Cout, 8, dt, 1.3)
    gb = torch.Generator().manual_seed(9)
    bsc, bsh, bmu = [(torch.randn(Cout, generator=gb) + 0.5).to(DEV) for _ in range(3)]
    bact = 2
    ntiles = query("seg_conv_igemm_row_tiles", M, Cout, None)
    if bnout and not query("seg_conv_igemm_bnout_ok", M, Cout, int(dt == BF)):
        pytest.skip("no BN-partials epilogue for this tile")
    outs = {}
    for tag in ("ref", "bwx"):
        out = torch.full((M, Cout), 2.0, device=DEV, dtype=dt)
        part = torch.zeros(ntiles * 2 * Cout, device=DEV)
        bargs = (by.data_ptr(), Cout, bsc.data_ptr(), bsh.data_ptr(), bmu.data_ptr(), bact, part.data_ptr()) if bnout \
            else (None, 0, None, None, None, 0, None)
        if tag == "ref":
            if bnout:
                call("seg_conv_igemm_bnout_bf16io_w16" if dt == BF else "seg_conv_igemm_bnout", dy.data_ptr(), C, N, H,
                     W, C, wk.data_ptr(), ldk, out.data_ptr(), Cout, Cout, ks, add.data_ptr(), Cout, *bargs, s)
            else:
                call("seg_conv_igemm_bf16io_w16" if dt == BF else "seg_conv_igemm", dy.data_ptr(), C, N, H, W, C,
                     wk.data_ptr(), ldk, None, out.data_ptr(), Cout, H, W, Cout, ks, 1, ks // 2, add.data_ptr(), Cout,
                     None, s)
        else:
            call("seg_conv_igemm_bwx_bf16io_w16" if dt == BF else "seg_conv_igemm_bwx", dA.data_ptr(), dA.shape[1], N,
                 H, W, C, y.data_ptr(), y.shape[1], st.data_ptr(), act, wk.data_ptr(), ldk, out.data_ptr(), Cout, Cout,
                 ks, add.data_ptr(), Cout, *bargs, s)
        outs[tag] = (out, part)
    torch.cuda.synchronize()
    assert torch.equal(outs["ref"][0].float(), outs["bwx"][0].float())
    assert torch.equal(outs["ref"][1], outs["bwx"][1])


@pytest.mark.parametrize("math", list(MATHS))
@pytest.mark.parametrize("act", [0, 2])
@pytest.mark.parametrize("M,K,N,pad_ld", [(4096, 16, 32, 0), (3001, 24, 144, 8), (777, 32, 16, 0), (130, 16, 96, 16)])
def test_pw_dgrad_bwx(math, act, M, K, N, pad_ld):
    dt = MATHS[math]
    s = S()
    y, dA, st = _layer(M, K, K + pad_ld, K + pad_ld, dt, 20)
    dy = _apply(y, dA, st, K, act, dt)
    g = torch.Generator().manual_seed(21)
    wk = (torch.randn(N, K, generator=g) * 0.1).to(DEV).to(dt)
    add = _t(M, N, 22, dt)
    outs = []
    for bwx in (False, True):
        out = torch.full((M, N), 1.0, device=DEV, dtype=dt)
        if bwx:
            call("seg_conv_pw_bwx_bf16io" if dt == BF else "seg_conv_pw_bwx", dA.data_ptr(), dA.shape[1], y.data_ptr(),
                 y.shape[1], st.data_ptr(), act, M, K, wk.data_ptr(), K, out.data_ptr(), N, N, add.data_ptr(), N, s)
        else:
            call("seg_conv_pw_bf16io" if dt == BF else "seg_conv_pw", dy.data_ptr(), K, M, K, wk.data_ptr(), K, None,
                 out.data_ptr(), N, N, add.data_ptr(), N, None, None, None, 0, s)
        outs.append(out)
    torch.cuda.synchronize()
    assert torch.equal(outs[0].float(), outs[1].float())


@pytest.mark.parametrize("math", list(MATHS))
@pytest.mark.parametrize("stride", [1, 2])
@pytest.mark.parametrize("acc", [0, 1])
@pytest.mark.parametrize("N,H,W,C,pad_ld", [(2, 16, 22, 32, 0), (1, 9, 13, 96, 8), (2, 8, 8, 576, 0)])
def test_dw_dgrad_bwx(math, stride, acc, N, H, W, C, pad_ld):
    dt = MATHS[math]
    s = S()
    Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
    Mo = N * Ho * Wo
    y, dA, st = _layer(Mo, C, C + pad_ld, C + 2 * pad_ld, dt, 30)
    dy = _apply(y, dA, st, C, 2, dt)
    g = torch.Generator().manual_seed(31)
    wk = (torch.randn(9 * C, generator=g) * 0.3).to(DEV)
    base = _t(N * H * W, C, 32, dt)
    outs = []
    for bwx in (False, True):
        dx = base.clone()
        if bwx:
            call("seg_dw_dgrad_bwx_bf16io" if dt == BF else "seg_dw_dgrad_bwx", dA.data_ptr(), dA.shape[1],
                 y.data_ptr(), y.shape[1], st.data_ptr(), 2, N, Ho, Wo, C, wk.data_ptr(), dx.data_ptr(), C, H, W,
                 stride, acc, s)
        else:
            call("seg_dw_dgrad_bf16io" if dt == BF else "seg_dw_dgrad", dy.data_ptr(), C, N, Ho, Wo, C, wk.data_ptr(),
                 dx.data_ptr(), C, H, W, stride, acc, s)
        outs.append(dx)
    torch.cuda.synchronize()
    assert torch.equal(outs[0].float(), outs[1].float())


@pytest.mark.parametrize("math", list(MATHS))
@pytest.mark.parametrize("stride", [1, 2])
@pytest.mark.parametrize("lazy", [False, True])
@pytest.mark.parametrize("N,H,W,C", [(2, 16, 22, 32), (1, 9, 13, 96), (2, 8, 8, 960)])
def test_dw_wgrad_bwx(math, stride, lazy, N, H, W, C):
    dt = MATHS[math]
    s = S()
    Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
    Mo = N * Ho * Wo
    y, dA, st = _layer(Mo, C, C, C, dt, 40)
    dy = _apply(y, dA, st, C, 2, dt)
    x = _t(N * H * W, C, 41, dt)
    g = torch.Generator().manual_seed(42)
    sc, sh = (torch.rand(C, generator=g) + 0.5).to(DEV), torch.randn(C, generator=g).to(DEV)
    xf = (sc.data_ptr(), sh.data_ptr(), 2) if lazy else (None, None, 0)
    nblk = query("seg_dw_wgrad_blocks", N, Ho, Wo, C)
    parts = []
    for bwx in (False, True):
        part = torch.full((nblk * 9 * C,), 5.0, device=DEV)
        if bwx:
            call("seg_dw_wgrad_bwx_bf16io" if dt == BF else "seg_dw_wgrad_bwx", dA.data_ptr(), C, y.data_ptr(), C,
                 st.data_ptr(), 2, x.data_ptr(), C, N, H, W, C, *xf, Ho, Wo, stride, part.data_ptr(), s)
        else:
            call("seg_dw_wgrad_bf16io" if dt == BF else "seg_dw_wgrad", dy.data_ptr(), C, x.data_ptr(), C, N, H, W, C,
                 *xf, Ho, Wo, stride, part.data_ptr(), s)
        parts.append(part)
    torch.cuda.synchronize()
    assert torch.equal(parts[0], parts[1])


@pytest.mark.parametrize("math", list(MATHS))
@pytest.mark.parametrize("lazy", [False, True])
@pytest.mark.parametrize("N,H,W,Cin,Cout,ks,stride", [(2, 16, 24, 16, 96, 1, 1), (1, 9, 13, 144, 24, 1, 1),
                                                     (2, 8, 8, 320, 1280, 1, 1), (2, 12, 20, 80, 32, 3, 1),
                                                     (2, 16, 16, 4, 32, 3, 2), (1, 8, 12, 256, 256, 3, 1)])
def test_wgrad_bwx(math, lazy, N, H, W, Cin, Cout, ks, stride):
    dt = MATHS[math]
    s = S()
    pad = ks // 2
    Ho, Wo = (H + 2 * pad - ks) // stride + 1, (W + 2 * pad - ks) // stride + 1
    Mo = N * Ho * Wo
    y, dA, st = _layer(Mo, Cout, Cout, Cout, dt, 50)
    dy = _apply(y, dA, st, Cout, 2, dt)
    x = _t(N * H * W, Cin, 51, dt)
    g = torch.Generator().manual_seed(52)
    sc, sh = (torch.rand(Cin, generator=g) + 0.5).to(DEV), torch.randn(Cin, generator=g).to(DEV)
    xf = (sc.data_ptr(), sh.data_ptr(), 2) if lazy else (None, None, 0)
    splits = query("seg_conv_wgrad_splits_bf16" if dt == BF else "seg_conv_wgrad_splits", Mo, Cout, Cin, ks)
    parts = []
    for bwx in (False, True):
        part = torch.full((splits * Cout * ks * ks * Cin,), 5.0, device=DEV)
        if bwx:
            call("seg_conv_wgrad_bwx_bf16io" if dt == BF else "seg_conv_wgrad_bwx", dA.data_ptr(), Cout,
                 y.data_ptr(), Cout, st.data_ptr(), 2, x.data_ptr(), Cin, N, H, W, Cin, Ho, Wo, Cout, ks, stride, pad,
                 part.data_ptr(), splits, *xf, s)
        else:
            base = "seg_conv_wgrad_bf16io" if dt == BF else "seg_conv_wgrad"
            call(base + ("_xf" if lazy else ""), dy.data_ptr(), Cout, x.data_ptr(), Cin, N, H, W, Cin, Ho, Wo, Cout,
                 ks, stride, pad, part.data_ptr(), splits, *(xf if lazy else ()), s)
        parts.append(part)
    torch.cuda.synchronize()
    assert torch.equal(parts[0], parts[1])
