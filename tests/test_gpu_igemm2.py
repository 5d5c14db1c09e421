"""GPU: seg_conv_igemm2_bf16io -- the LDS-DMA, 8-wave, split-K implicit GEMM for the deep
bf16io convs (csrc/igemm2.hip).

  * against a float64 conv of the same bf16 operands (rel-L2 1e-5: fp32 accumulation);
  * unsplit launches equal the 64x128 generic kernel (seg_conv_igemm_bf16io_w16) bit for
    bit -- both accumulate each output over k in the same 16-deep MFMA order -- which pins
    the swizzled LDS-DMA layout and the implicit-im2col tap handling exactly;
  * split-K launches (the last-arriving K slice combines the slices) are bitwise
    reproducible call after call on one workspace, and leave its tickets zero;
  * BatchNorm tile partials: the tile sums add up to the fp64 column sums, and each
    tile's M2 equals the fp64 M2 about that tile's mean;
  * the addend (data-gradient accumulation) and bias paths.
"""
import pytest
import torch
import torch.nn.functional as F

from seg_amd import engine
from seg_amd._lib import call, query

pytestmark = pytest.mark.gpu
DEV = "cuda"
BF = torch.bfloat16


def S():
    return torch.cuda.current_stream().cuda_stream


def r8(c):
    return (c + 7) & ~7


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


def plan(M, Cout, Cin, ks):
    import ctypes
    out = (ctypes.c_long * 4)()
    ok = query("seg_conv_igemm2_plan", M, Cout, Cin, ks, ctypes.addressof(out))
    return ok, list(out)


def pack16(w, Cout, Cin, ks):
    ldk = r8(ks * ks * Cin)
    wk = torch.full((Cout * ldk,), float("nan"), device=DEV).to(BF)
    table, n, blocks = engine.pack_table([(w.data_ptr(), wk.data_ptr(), Cout, Cin, ks, ldk, 16, Cin)], w.device)
    call("seg_pack_batch", table.data_ptr(), n, blocks, S())
    return wk, ldk


CASES = [  # (N, Cin, Cout, H, W, ks): split-K, dgrad-shaped, ragged M, taps spanning a K step, unsplit, 1x1
    (2, 1344, 256, 16, 32, 3), (8, 256, 1344, 8, 16, 3), (2, 128, 128, 33, 65, 3), (4, 288, 128, 64, 64, 3),
    (32, 128, 128, 32, 64, 3), (2, 960, 256, 16, 16, 1),
    # round 4: the 4-wave tiles -- the MobileNetV2 encoder's small-image 1x1 convs at bs=32 (M = 4k-65k rows),
    # K < one 64-deep step, ragged N, a 3x3 with 152 inputs
    (32, 960, 160, 8, 16, 1), (32, 96, 576, 16, 32, 1), (32, 32, 192, 32, 64, 1), (32, 144, 64, 32, 64, 1),
    (32, 320, 1280, 8, 16, 1), (32, 24, 144, 16, 32, 1), (8, 152, 64, 32, 64, 3)]


@pytest.mark.parametrize("N,Cin,Cout,H,W,ks", CASES)
def test_igemm2_vs_fp64_and_generic(N, Cin, Cout, H, W, ks):
    M = N * H * W
    ok, (tile_rows, ntiles, splits, work_floats) = plan(M, Cout, Cin, ks)
    assert ok, "the plan must apply to these shapes"
    g = torch.Generator().manual_seed(N * 1000 + Cin)
    x = (torch.randn(M, Cin, generator=g) * 1.3 + 0.2).to(BF)
    w = torch.randn(Cout, Cin, ks, ks, generator=g) * (2.0 / (Cin * ks * ks)) ** 0.5
    b = torch.randn(Cout, generator=g)
    add = (torch.randn(M, Cout, generator=g)).to(BF)
    xg, wg, bg, addg = x.to(DEV), w.to(DEV), b.to(DEV), add.to(DEV)
    wk, ldk = pack16(wg, Cout, Cin, ks)
    x64 = x.double().view(N, H, W, Cin).permute(0, 3, 1, 2)
    ref = F.conv2d(x64, w.to(BF).double(), b.double(), padding=ks // 2).permute(0, 2, 3, 1).reshape(M, Cout)
    work = torch.zeros(max(work_floats, 1), device=DEV)
    outs = []
    for rep in range(3):
        y = torch.full((M, Cout), 7.0, device=DEV).to(BF)
        st = torch.full((ntiles * 2 * Cout,), float("nan"), device=DEV)
        call("seg_conv_igemm2_bf16io", xg.data_ptr(), Cin, N, H, W, Cin, wk.data_ptr(), ldk, bg.data_ptr(),
             y.data_ptr(), Cout, Cout, ks, None, 0, st.data_ptr(), work.data_ptr(), S())
        outs.append((y, st))
    torch.cuda.synchronize()
    y, st = outs[0]
    for y2, st2 in outs[1:]:
        assert torch.equal(y, y2) and torch.equal(st, st2), "split-K combine must be deterministic"
    if splits > 1:  # (the first ntiles of the tiles' tickets)
        assert int(work[:ntiles].view(torch.int32).abs().sum()) == 0, "tickets re-armed"
    assert rel(y.float(), ref) < 4e-3  # the bf16 rounding of the stored output
    # statistics on the fp32 accumulator: tile sums and M2 about each tile's mean
    stv = st.view(ntiles, 2, Cout).double().cpu()
    assert rel(stv[:, 0].sum(0), ref.sum(0)) < 1e-5
    for t in (0, ntiles - 1):
        blk = ref[t * tile_rows:(t + 1) * tile_rows]
        m2 = ((blk - blk.mean(0)) ** 2).sum(0)
        assert rel(stv[t, 1], m2) < 1e-4, t
    # addend
    ya = torch.empty(M, Cout, device=DEV, dtype=BF)
    call("seg_conv_igemm2_bf16io", xg.data_ptr(), Cin, N, H, W, Cin, wk.data_ptr(), ldk, None, ya.data_ptr(), Cout,
         Cout, ks, addg.data_ptr(), Cout, None, work.data_ptr(), S())
    torch.cuda.synchronize()
    assert rel(ya.float(), ref - b.double() + add.double()) < 4e-3
    if splits == 1:  # same k order as the generic 16-bit kernel: bitwise equal
        y0 = torch.empty(M, Cout, device=DEV, dtype=BF)
        call("seg_conv_igemm_bf16io_w16", xg.data_ptr(), Cin, N, H, W, Cin, wk.data_ptr(), ldk, bg.data_ptr(),
             y0.data_ptr(), Cout, H, W, Cout, ks, 1, ks // 2, None, 0, None, S())
        torch.cuda.synchronize()
        assert torch.equal(y0, y)


def test_igemm2_plan_rejects_padding_heavy_shapes():
    assert plan(4096, 80, 32, 3)[0] == 0      # 3x3 with Cin < 64
    assert plan(4096, 10, 16, 1)[0] == 0      # 10 output channels: >= 40 % padded columns on every tile
    assert plan(4096, 16, 12, 1)[0] == 0      # Cin % 8
    assert plan(16384, 256, 1344, 3)[0] == 1
    assert plan(4096, 288, 128, 3)[0] == 1    # round 4: a 4-wave 128x64 / 64x64 tile (was rejected)


@pytest.mark.parametrize("tile", range(6))
def test_igemm2_every_tile(tile):
    """Each tile of the table, forced (seg_igemm2_force_tile), on one 3x3 and one 1x1 shape: unsplit
    launches bitwise equal to the generic kernel, split ones within the bf16 rounding of fp64."""
    try:
        query("seg_igemm2_force_tile", tile)
        for (N, Cin, Cout, H, W, ks) in ((2, 128, 96, 16, 40, 3), (4, 64, 200, 20, 24, 1)):
            M = N * H * W
            ok, (tile_rows, ntiles, splits, work_floats) = plan(M, Cout, Cin, ks)
            assert ok
            g = torch.Generator().manual_seed(tile * 7 + ks)
            x = (torch.randn(M, Cin, generator=g)).to(BF).to(DEV)
            w = (torch.randn(Cout, Cin, ks, ks, generator=g) * 0.1).to(DEV)
            b = torch.randn(Cout, generator=g).to(DEV)
            wk, ldk = pack16(w, Cout, Cin, ks)
            work = torch.zeros(max(work_floats, 1), device=DEV)
            y = torch.empty(M, Cout, device=DEV, dtype=BF)
            st = torch.empty(ntiles * 2 * Cout, device=DEV)
            call("seg_conv_igemm2_bf16io", x.data_ptr(), Cin, N, H, W, Cin, wk.data_ptr(), ldk, b.data_ptr(),
                 y.data_ptr(), Cout, Cout, ks, None, 0, st.data_ptr(), work.data_ptr(), S())
            y0 = torch.empty(M, Cout, device=DEV, dtype=BF)
            call("seg_conv_igemm_bf16io_w16", x.data_ptr(), Cin, N, H, W, Cin, wk.data_ptr(), ldk, b.data_ptr(),
                 y0.data_ptr(), Cout, H, W, Cout, ks, 1, ks // 2, None, 0, None, S())
            torch.cuda.synchronize()
            if splits == 1:
                assert torch.equal(y, y0), (tile, ks)
            else:
                assert rel(y.float(), y0.float()) < 4e-3, (tile, ks)
            stv = st.view(ntiles, 2, Cout).double().cpu()
            assert rel(stv[:, 0].sum(0), y0.double().cpu().sum(0)) < 1e-2
    finally:
        query("seg_igemm2_force_tile", -1)


def test_engine_routes_wide_convs_to_igemm2(monkeypatch):
    """UNet(10) bf16io at 8x512x1024 (configs[4]): past the 65k-row cap, the 3x3 convs whose GEMM N is a multiple
    of 128 take igemm2 (SEG_IGEMM2_WIDE), the others keep the implicit GEMM / LDS halo; off: none past the cap."""
    from seg_amd import UNet, deterministic_init
    m = deterministic_init(UNet(10), seed=0).to(DEV).train()
    engine.set_conv_math(m, "bf16io")
    for wide in (True, False):
        monkeypatch.setattr(engine, "IGEMM2_WIDE", wide)
        prog = engine.build_program(m, 8, 512, 1024, "bf16io")
        prog._build_pack([op for op in prog.ops if isinstance(op, engine.ConvOp)], None)
        big = [op for op in prog.ops if isinstance(op, engine.ConvOp) and op.ks == 3 and op.y.M > 65536]
        assert big
        for op in big:
            if wide and op.cout % 128 == 0 and op.cin_pad == op.cin and not op.halo_f:
                assert op.ig2_f is not None, (op.cin, op.cout, op.y.M)
            if op.cout % 128 or not wide:
                assert op.ig2_f is None, (op.cin, op.cout, op.y.M)
            if not op.first and (op.cin % 128 or not wide):
                assert op.ig2_d is None, (op.cin, op.cout, op.y.M)
        if wide:
            assert sum(op.ig2_f is not None for op in big) >= 4 and sum(op.ig2_d is not None for op in big) >= 4
