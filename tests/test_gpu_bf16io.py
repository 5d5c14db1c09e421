"""GPU: the `_bf16io` entry points (bf16 activation / gradient storage, engine math
"bf16io") against their fp32 namesakes.

Every bf16io kernel widens its bf16 inputs to fp32, runs the fp32 kernel's arithmetic
in the same order, and rounds its outputs to bf16 (RNE).  So on inputs that are exactly
representable in bf16, its output must equal the fp32 kernel's output rounded to bf16,
bit for bit -- which is what these tests check (pad channels and untouched rows too).
Model-level parity of the bf16io configuration: tests/test_gpu_bf16.py.
"""
import pytest
import torch
import torch.nn.functional as F

from seg_amd._lib import call, query

pytestmark = pytest.mark.gpu
DEV = "cuda"
BF = torch.bfloat16


def S():
    return torch.cuda.current_stream().cuda_stream


def r4(c):
    return (c + 3) & ~3


def rows(M, ld, seed, scale=1.0, shift=0.0):
    """bf16-representable fp32 rows and their bf16 twin."""
    g = torch.Generator().manual_seed(seed)
    x = (torch.randn(M, ld, generator=g) * scale + shift).to(BF)
    return x.float().to(DEV), x.to(DEV)


def same(b16, f32):
    """bf16 output == fp32 output rounded to bf16, bitwise."""
    ref = f32.to(BF)
    assert torch.equal(b16.view(torch.int16), ref.view(torch.int16)), \
        f"max diff {(b16.float() - ref.float()).abs().max().item()}"


def test_add_apply_stats_backward_colsum():
    s = S()
    M, C = 3001, 40
    y32, y16 = rows(M, C, 1, 2.0, 0.5)
    d32, d16 = rows(M, C, 2)
    r32, r16 = rows(M, C, 3)
    # add
    o32, o16 = torch.empty(M, C, device=DEV), torch.empty(M, C, device=DEV, dtype=BF)
    call("seg_add", y32.data_ptr(), C, r32.data_ptr(), C, M, C, o32.data_ptr(), C, s)
    call("seg_add_bf16io", y16.data_ptr(), C, r16.data_ptr(), C, M, C, o16.data_ptr(), C, s)
    same(o16, o32)
    # BN statistics (train) -> identical fp32 coefficients
    st = {}
    for tag, y, name in (("f", y32, "seg_bn_stats"), ("b", y16, "seg_bn_stats_bf16io")):
        out = torch.empty(4 * C, device=DEV)
        rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
        gamma, beta = torch.linspace(0.5, 1.5, C, device=DEV), torch.linspace(-1, 1, C, device=DEV)
        work = torch.zeros(query("seg_chan_workspace_floats", M, C), device=DEV)
        call(name, y.data_ptr(), C, M, C, gamma.data_ptr(), beta.data_ptr(), 1e-5, 0.1, rm.data_ptr(), rv.data_ptr(),
             None, work.data_ptr(), out[:C].data_ptr(), out[C:2 * C].data_ptr(), out[2 * C:3 * C].data_ptr(),
             out[3 * C:].data_ptr(), s)
        st[tag] = (out, rm, rv, gamma)
    assert torch.equal(st["f"][0], st["b"][0]) and torch.equal(st["f"][2], st["b"][2])
    out, _, _, gamma = st["f"]
    mean, invstd, scale, shift = out[:C], out[C:2 * C], out[2 * C:3 * C], out[3 * C:]
    for act in (0, 1, 2):
        # apply (+ residual)
        call("seg_bn_apply", y32.data_ptr(), C, M, C, scale.data_ptr(), shift.data_ptr(), act, r32.data_ptr(), C,
             o32.data_ptr(), C, s)
        call("seg_bn_apply_bf16io", y16.data_ptr(), C, M, C, scale.data_ptr(), shift.data_ptr(), act, r16.data_ptr(),
             C, o16.data_ptr(), C, s)
        same(o16, o32)
        # backward: fp32 dgamma/dbeta identical, dY rounded
        res = {}
        for tag, (d, y, name, dt) in {"f": (d32, y32, "seg_bn_backward", torch.float32),
                                      "b": (d16, y16, "seg_bn_backward_bf16io", BF)}.items():
            gw, gb = torch.empty(C, device=DEV), torch.empty(C, device=DEV)
            work = torch.zeros(query("seg_chan_workspace_floats", M, C) + 3 * C, device=DEV)
            dy = torch.empty(M, C, device=DEV, dtype=dt)
            call(name, d.data_ptr(), C, y.data_ptr(), C, M, C, gamma.data_ptr(), mean.data_ptr(), invstd.data_ptr(),
                 scale.data_ptr(), shift.data_ptr(), act, gw.data_ptr(), gb.data_ptr(), work.data_ptr(), dy.data_ptr(),
                 C, s)
            res[tag] = (gw, gb, dy)
        assert torch.equal(res["f"][0], res["b"][0]) and torch.equal(res["f"][1], res["b"][1])
        same(res["b"][2], res["f"][2])
    # colsum (bias gradient), C not a multiple of 4 in the data, ld padded
    cs = {}
    for tag, d, name in (("f", d32, "seg_colsum"), ("b", d16, "seg_colsum_bf16io")):
        o = torch.empty(C - 2, device=DEV)
        work = torch.zeros(query("seg_chan_workspace_floats", M, C), device=DEV)
        call(name, d.data_ptr(), C, M, C - 2, work.data_ptr(), o.data_ptr(), 0, s)
        cs[tag] = o
    assert torch.equal(cs["f"], cs["b"])


@pytest.mark.parametrize("M,C,ld,off", [(3001, 12, 16, 4), (517, 1280, 1280, 0), (33, 2064, 2064, 0),
                                         (1000, 40, 48, 8), (1, 8, 8, 0)])
def test_row_tiled_passes(M, C, ld, off):
    """The row-tiled BN apply / BN backward apply / add kernels over the layouts their
    launchers pick between: 8 bf16 channels per lane (C % 8 == 0, 16-byte aligned
    slices), the 4-channel fallback (C = 12; a channel slice at an 8-byte offset), more
    channel groups than lanes (C = 1280 fp32, C = 2064 bf16), row strides > C, M = 1.
    fp32 against the torch formula; bf16io bitwise against the fp32 kernel; in-place
    apply bitwise against out-of-place; channels outside the slice untouched."""
    s = S()
    y32, y16 = rows(M, ld, 11, 2.0, 0.5)
    d32, d16 = rows(M, ld, 12)
    r32, r16 = rows(M, ld, 13)
    g = torch.Generator().manual_seed(14)
    scale, shift, mean = (torch.randn(C, generator=g).to(DEV) for _ in range(3))
    sl = slice(off, off + C)

    def fresh(dt):
        return torch.full((M, ld), 7.0, device=DEV, dtype=dt)

    def p(t):
        return t[:, off:].data_ptr()

    yv, dv, rv = y32[:, sl], d32[:, sl], r32[:, sl]
    for act in (0, 1, 2):
        z = yv * scale + shift
        ref = z if act == 0 else (z.clamp(min=0) if act == 1 else z.clamp(0, 6))
        o32, o16 = fresh(torch.float32), fresh(BF)
        call("seg_bn_apply", p(y32), ld, M, C, scale.data_ptr(), shift.data_ptr(), act, p(r32), ld, p(o32), ld, s)
        call("seg_bn_apply_bf16io", p(y16), ld, M, C, scale.data_ptr(), shift.data_ptr(), act, p(r16), ld, p(o16), ld,
             s)
        torch.testing.assert_close(o32[:, sl], ref + rv, rtol=1e-6, atol=1e-6)
        same(o16, o32)
        inpl = y32.clone()
        call("seg_bn_apply", p(inpl), ld, M, C, scale.data_ptr(), shift.data_ptr(), act, p(r32), ld, p(inpl), ld, s)
        assert torch.equal(inpl[:, sl], o32[:, sl])
        # eval-mode BN backward (seg_bn_eval_backward): dY = scale * dA * act'(z)
        mask = torch.ones_like(z) if act == 0 else ((z > 0) if act == 1 else ((z > 0) & (z < 6))).float()
        dy = fresh(torch.float32)
        call("seg_bn_eval_backward", p(d32), ld, p(y32), ld, M, C, scale.data_ptr(), shift.data_ptr(), act, p(dy), ld,
             s)
        torch.testing.assert_close(dy[:, sl], scale * dv * mask, rtol=1e-6, atol=1e-6)
    # full BN backward (reduction + finalize + apply), fp32 vs bf16io twin, and vs its own coefficients
    gamma = torch.linspace(0.5, 1.5, C, device=DEV)
    invstd = scale.abs() + 0.5
    for act in (0, 2):
        res = {}
        for tag, d, y, name, dt in (("f", d32, y32, "seg_bn_backward", torch.float32),
                                    ("b", d16, y16, "seg_bn_backward_bf16io", BF)):
            gw, gb = torch.empty(C, device=DEV), torch.empty(C, device=DEV)
            work = torch.zeros(query("seg_chan_workspace_floats", M, C) + 3 * C, device=DEV)
            dy = fresh(dt)
            call(name, p(d), ld, p(y), ld, M, C, gamma.data_ptr(), mean.data_ptr(), invstd.data_ptr(),
                 scale.data_ptr(), shift.data_ptr(), act, gw.data_ptr(), gb.data_ptr(), work.data_ptr(), p(dy), ld, s)
            res[tag] = (gw, gb, dy)
        assert torch.equal(res["f"][0], res["b"][0]) and torch.equal(res["f"][1], res["b"][1])
        same(res["b"][2], res["f"][2])
        z = yv * scale + shift
        mask = torch.ones_like(z) if act == 0 else ((z > 0) & (z < 6)).float()
        dz = dv * mask
        xh = (yv - mean) * invstd
        dref = gamma * invstd * (dz - dz.mean(0) - xh * (dz * xh).mean(0))
        torch.testing.assert_close(res["f"][2][:, sl], dref, rtol=1e-4, atol=1e-4)
        assert torch.equal(res["f"][2][:, :off], fresh(torch.float32)[:, :off])
    # add (gradient fan-in), in place on the first operand too
    o32, o16 = fresh(torch.float32), fresh(BF)
    call("seg_add", p(y32), ld, p(r32), ld, M, C, p(o32), ld, s)
    call("seg_add_bf16io", p(y16), ld, p(r16), ld, M, C, p(o16), ld, s)
    assert torch.equal(o32[:, sl], yv + rv)
    same(o16, o32)
    a = y32.clone()
    call("seg_add", p(a), ld, p(r32), ld, M, C, p(a), ld, s)
    assert torch.equal(a[:, sl], yv + rv) and torch.equal(a[:, :off], y32[:, :off])


@pytest.mark.parametrize("stride", [1, 2])
@pytest.mark.parametrize("lazy", [False, True])
def test_depthwise(stride, lazy):
    s = S()
    N, C, H, W = 2, 24, 13, 18
    Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
    x32, x16 = rows(N * H * W, C, 4)
    g32, g16 = rows(N * Ho * Wo, C, 5)
    wk = torch.randn(9 * C, generator=torch.Generator().manual_seed(6)).to(DEV)
    sc = torch.linspace(0.5, 2, C, device=DEV) if lazy else None
    sh = torch.linspace(-1, 1, C, device=DEV) if lazy else None
    p = (lambda t: t.data_ptr() if t is not None else None)
    o32, o16 = torch.empty(N * Ho * Wo, C, device=DEV), torch.empty(N * Ho * Wo, C, device=DEV, dtype=BF)
    call("seg_dw_fwd", x32.data_ptr(), C, N, H, W, C, p(sc), p(sh), 2, wk.data_ptr(), o32.data_ptr(), C, Ho, Wo,
         stride, s)
    call("seg_dw_fwd_bf16io", x16.data_ptr(), C, N, H, W, C, p(sc), p(sh), 2, wk.data_ptr(), o16.data_ptr(), C, Ho,
         Wo, stride, s)
    same(o16, o32)
    for acc in (0, 1):
        a32, a16 = rows(N * H * W, C, 7)
        call("seg_dw_dgrad", g32.data_ptr(), C, N, Ho, Wo, C, wk.data_ptr(), a32.data_ptr(), C, H, W, stride, acc, s)
        call("seg_dw_dgrad_bf16io", g16.data_ptr(), C, N, Ho, Wo, C, wk.data_ptr(), a16.data_ptr(), C, H, W, stride,
             acc, s)
        same(a16, a32)  # accumulate: the old value widens exactly, one rounding of the fp32 sum
    nblk = query("seg_dw_wgrad_blocks", N, Ho, Wo, C)
    parts = []
    for name, dy, x in (("seg_dw_wgrad", g32, x32), ("seg_dw_wgrad_bf16io", g16, x16)):
        part = torch.empty(nblk * 9 * C, device=DEV)
        call(name, dy.data_ptr(), C, x.data_ptr(), C, N, H, W, C, p(sc), p(sh), 2, Ho, Wo, stride, part.data_ptr(), s)
        parts.append(part)
    assert torch.equal(parts[0], parts[1])


def test_resample_pool_layout():
    s = S()
    N, C, H, W = 2, 12, 7, 9
    x32, x16 = rows(N * H * W, C, 8)
    # x2 bilinear (align_corners False) into a strided concat slice, and its backward
    ld = 20
    o32, o16 = torch.zeros(N * 4 * H * W, ld, device=DEV), torch.zeros(N * 4 * H * W, ld, device=DEV, dtype=BF)
    call("seg_upsample_fwd", x32.data_ptr(), C, N, H, W, C, o32[:, 4:].data_ptr(), ld, 2 * H, 2 * W, 0, s)
    call("seg_upsample_fwd_bf16io", x16.data_ptr(), C, N, H, W, C, o16[:, 4:].data_ptr(), ld, 2 * H, 2 * W, 0, s)
    same(o16, o32)
    d32, d16 = rows(N * 4 * H * W, C, 9)
    for ac in (0, 1):
        for acc in (0,):
            i32, i16 = torch.empty(N * H * W, C, device=DEV), torch.empty(N * H * W, C, device=DEV, dtype=BF)
            call("seg_upsample_bwd", d32.data_ptr(), C, 0, N, 2 * H, 2 * W, C, i32.data_ptr(), C, H, W, ac, acc, s)
            call("seg_upsample_bwd_bf16io", d16.data_ptr(), C, 0, N, 2 * H, 2 * W, C, i16.data_ptr(), C, H, W, ac,
                 acc, s)
            same(i16, i32)
    # NCHW fp32 gradient of the returned logits -> bf16 NHWC
    gn = torch.randn(N, C, 2 * H, 2 * W, device=DEV)
    i32, i16 = torch.empty(N * H * W, C, device=DEV), torch.empty(N * H * W, C, device=DEV, dtype=BF)
    call("seg_upsample_bwd", gn.data_ptr(), 0, 1, N, 2 * H, 2 * W, C, i32.data_ptr(), C, H, W, 1, 0, s)
    call("seg_upsample_bwd_bf16io", gn.data_ptr(), 0, 1, N, 2 * H, 2 * W, C, i16.data_ptr(), C, H, W, 1, 0, s)
    same(i16, i32)
    # bf16 NHWC logits -> fp32 NCHW model output (identical fp32)
    n32, n16 = torch.empty(N, C, 2 * H, 2 * W, device=DEV), torch.empty(N, C, 2 * H, 2 * W, device=DEV)
    call("seg_upsample_to_nchw", x32.data_ptr(), C, N, H, W, C, n32.data_ptr(), 2 * H, 2 * W, 1, s)
    call("seg_upsample_to_nchw_bf16io", x16.data_ptr(), C, N, H, W, C, n16.data_ptr(), 2 * H, 2 * W, 1, s)
    # fp32 output: the two instantiations may contract the blend into FMAs differently
    torch.testing.assert_close(n16, n32, rtol=1e-6, atol=1e-6)
    # image NCHW fp32 -> NHWC4 rows
    img = torch.randn(N, 3, H, W, device=DEV)
    h32, h16 = torch.empty(N * H * W, 4, device=DEV), torch.empty(N * H * W, 4, device=DEV, dtype=BF)
    call("seg_nchw_to_nhwc", img.data_ptr(), N, 3, H, W, h32.data_ptr(), 4, s)
    call("seg_nchw_to_nhwc_bf16io", img.data_ptr(), N, 3, H, W, h16.data_ptr(), 4, s)
    same(h16, h32)
    # max pool 2x2 fwd / bwd (ties included: bf16 rounding makes many)
    He, We = 8, 10
    p32, p16 = rows(N * He * We, C, 10, 0.05)
    q32, q16 = torch.empty(N * He * We // 4, C, device=DEV), torch.empty(N * He * We // 4, C, device=DEV, dtype=BF)
    call("seg_maxpool2_fwd", p32.data_ptr(), C, N, He, We, C, q32.data_ptr(), C, s)
    call("seg_maxpool2_fwd_bf16io", p16.data_ptr(), C, N, He, We, C, q16.data_ptr(), C, s)
    same(q16, q32)
    gq32, gq16 = rows(N * He * We // 4, C, 11)
    b32, b16 = torch.empty(N * He * We, C, device=DEV), torch.empty(N * He * We, C, device=DEV, dtype=BF)
    call("seg_maxpool2_bwd", p32.data_ptr(), C, gq32.data_ptr(), C, N, He, We, C, b32.data_ptr(), C, 0, s)
    call("seg_maxpool2_bwd_bf16io", p16.data_ptr(), C, gq16.data_ptr(), C, N, He, We, C, b16.data_ptr(), C, 0, s)
    same(b16, b32)


def test_cross_entropy():
    s = S()
    N, C, H, W = 2, 10, 16, 32
    Ho, Wo = 2 * H, 2 * W
    lo32, lo16 = rows(N * H * W, 12, 12, 2.0)
    t = torch.randint(0, C, (N, Ho, Wo), generator=torch.Generator().manual_seed(13)).to(DEV)
    t[0, :3] = -100
    work = torch.empty(query("seg_ce_workspace_floats", N * Ho * Wo), device=DEV)
    st32, st16 = torch.empty(3, device=DEV), torch.empty(3, device=DEV)
    call("seg_ce_upsample_loss", lo32.data_ptr(), 12, N, H, W, C, t.data_ptr(), Ho, Wo, -100, work.data_ptr(),
         st32.data_ptr(), s)
    call("seg_ce_upsample_loss_bf16io", lo16.data_ptr(), 12, N, H, W, C, t.data_ptr(), Ho, Wo, -100, work.data_ptr(),
         st16.data_ptr(), s)
    assert torch.equal(st32, st16)
    g = torch.ones(1, device=DEV)
    d32, d16 = torch.empty(N * Ho * Wo, 12, device=DEV), torch.empty(N * Ho * Wo, 12, device=DEV, dtype=BF)
    call("seg_ce_upsample_grad", lo32.data_ptr(), 12, N, H, W, C, t.data_ptr(), Ho, Wo, -100, g.data_ptr(),
         st32.data_ptr(), d32.data_ptr(), 12, s)
    call("seg_ce_upsample_grad_bf16io", lo16.data_ptr(), 12, N, H, W, C, t.data_ptr(), Ho, Wo, -100, g.data_ptr(),
         st16.data_ptr(), d16.data_ptr(), 12, s)
    same(d16, d32)


@pytest.mark.parametrize("N,Cin,Cout,H,W,ks,stride", [(2, 16, 96, 9, 13, 1, 1), (1, 152, 64, 10, 12, 3, 1),
                                                     (2, 4, 32, 12, 17, 3, 2), (1, 320, 1280, 4, 6, 1, 1)])
def test_conv_bf16io(N, Cin, Cout, H, W, ks, stride):
    """seg_conv_igemm_bf16io / seg_conv_wgrad_bf16io == the bf16-math kernels on fp32
    storage fed the same (bf16-representable) values: identical LDS operands, identical
    fp32 accumulators, so the outputs are the fp32-storage results rounded once."""
    s = S()
    pad = ks // 2
    Ho, Wo = (H + 2 * pad - ks) // stride + 1, (W + 2 * pad - ks) // stride + 1
    x32, x16 = rows(N * H * W, Cin, 14)
    w = (torch.randn(Cout, Cin, ks, ks, generator=torch.Generator().manual_seed(15)) * 0.1).to(DEV)
    b = torch.randn(Cout, generator=torch.Generator().manual_seed(16)).to(DEV)
    ldk = r4(ks * ks * Cin)
    wk = torch.empty(Cout * ldk, device=DEV)
    call("seg_pack_conv_weight", w.data_ptr(), wk.data_ptr(), Cout, Cin, ks, ldk, 0, Cin, s)
    M = N * Ho * Wo
    ntiles = query("seg_conv_igemm_row_tiles", M, Cout, None)
    y32, y16 = torch.empty(M, Cout, device=DEV), torch.empty(M, Cout, device=DEV, dtype=BF)
    st32, st16 = torch.empty(ntiles * 2 * Cout, device=DEV), torch.empty(ntiles * 2 * Cout, device=DEV)
    call("seg_conv_igemm_bf16", x32.data_ptr(), Cin, N, H, W, Cin, wk.data_ptr(), ldk, b.data_ptr(), y32.data_ptr(),
         Cout, Ho, Wo, Cout, ks, stride, pad, None, 0, st32.data_ptr(), 0, None, 1, s)
    call("seg_conv_igemm_bf16io", x16.data_ptr(), Cin, N, H, W, Cin, wk.data_ptr(), ldk, b.data_ptr(), y16.data_ptr(),
         Cout, Ho, Wo, Cout, ks, stride, pad, None, 0, st16.data_ptr(), s)
    same(y16, y32)
    assert torch.equal(st32, st16)  # BN statistics from the fp32 accumulators
    if stride != 1:
        return
    # data gradient with an addend
    dy32, dy16 = rows(M, Cout, 17)
    a32, a16 = rows(N * H * W, Cin, 18)
    kin = r4(Cout)
    ldk2 = r4(ks * ks * kin)
    wkd = torch.empty(Cin * ldk2, device=DEV)
    call("seg_pack_conv_weight", w.data_ptr(), wkd.data_ptr(), Cout, Cin, ks, ldk2, 1, kin, s)
    dx32, dx16 = torch.empty(N * H * W, Cin, device=DEV), torch.empty(N * H * W, Cin, device=DEV, dtype=BF)
    call("seg_conv_igemm_bf16", dy32.data_ptr(), Cout, N, H, W, kin, wkd.data_ptr(), ldk2, None, dx32.data_ptr(), Cin,
         H, W, Cin, ks, 1, pad, a32.data_ptr(), Cin, None, 0, None, 1, s)
    call("seg_conv_igemm_bf16io", dy16.data_ptr(), Cout, N, H, W, kin, wkd.data_ptr(), ldk2, None, dx16.data_ptr(),
         Cin, H, W, Cin, ks, 1, pad, a16.data_ptr(), Cin, None, s)
    same(dx16, dx32)
    # weight gradient
    splits = query("seg_conv_wgrad_splits", M, Cout, Cin, ks)
    p32, p16 = (torch.empty(splits * Cout * ks * ks * Cin, device=DEV) for _ in range(2))
    call("seg_conv_wgrad_bf16", dy32.data_ptr(), Cout, x32.data_ptr(), Cin, N, H, W, Cin, H, W, Cout, ks, 1, pad,
         p32.data_ptr(), splits, s)
    call("seg_conv_wgrad_bf16io", dy16.data_ptr(), Cout, x16.data_ptr(), Cin, N, H, W, Cin, H, W, Cout, ks, 1, pad,
         p16.data_ptr(), splits, s)
    assert torch.equal(p32, p16)


@pytest.mark.parametrize("N,Cin,Cout,H,W", [(2, 80, 32, 8, 64), (1, 152, 64, 4, 128), (1, 32, 80, 8, 64),
                                            (1, 16, 64, 4, 64)])
def test_conv_halo_bf16io(N, Cin, Cout, H, W):
    """The bf16 LDS-halo direct conv (narrow 3x3 convs of the bf16io configuration)
    against a float64 conv of the same bf16 operands: the fp32 accumulation order differs
    from the implicit GEMM's, so the check is one bf16 rounding of the exact result;
    its BN-statistics partials (from the fp32 accumulators) to fp32 summation error."""
    s = S()
    x32, x16 = rows(N * H * W, Cin, 21)
    a32, a16 = rows(N * H * W, Cout, 22)
    w = (torch.randn(Cout, Cin, 3, 3, generator=torch.Generator().manual_seed(23)) * 0.1)
    b = torch.randn(Cout, generator=torch.Generator().manual_seed(24))
    ref = F.conv2d(x32.cpu().double().view(N, H, W, Cin).permute(0, 3, 1, 2),
                   w.to(BF).double(), b.double(), padding=1)
    ref = ref.permute(0, 2, 3, 1).reshape(-1, Cout) + a32.cpu().double()
    wg = w.to(DEV)
    ldk = r4(9 * Cin)
    wk = torch.empty(Cout * ldk, device=DEV)
    call("seg_pack_conv_weight", wg.data_ptr(), wk.data_ptr(), Cout, Cin, 3, ldk, 0, Cin, s)
    ntiles = query("seg_conv_halo_row_tiles", N, H, W)
    stat = torch.empty(ntiles * 2 * Cout, device=DEV)
    out = torch.empty(N * H * W, Cout, device=DEV, dtype=BF)
    call("seg_conv_halo_bf16io", x16.data_ptr(), Cin, N, H, W, Cin, wk.data_ptr(), ldk, b.to(DEV).data_ptr(),
         out.data_ptr(), Cout, Cout, a16.data_ptr(), Cout, stat.data_ptr(), s)
    got = out.double().cpu()
    err = (got - ref).abs()
    assert float(err.max()) <= float((ref.abs() * 2 ** -8 + 1e-6).max()) and \
        bool((err <= ref.abs() * 2 ** -8 + 1e-6).all())
    # tile sums are of acc + bias (before the addend), fp32
    pre = ref - a32.cpu().double()
    tile_sum = stat.view(ntiles, 2, Cout)[:, 0].sum(0).double().cpu()
    assert float((tile_sum - pre.sum(0)).norm() / pre.sum(0).norm()) < 1e-4
