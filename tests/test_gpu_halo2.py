"""GPU: seg_conv_halo2_bf16io -- the persistent LDS-DMA halo kernel for the narrow 3x3 convs
of the bf16io configuration (csrc/halo2.hip; src/unet.py:58,61's up3 / up4 convs of
MobileNetV2UNet and their data gradients, UNet's 64-channel full-resolution levels).

  * equal, bit for bit, to the first-generation LDS-halo kernel (seg_conv_halo_bf16io_w16:
    the same chunk / tap / 16-deep MFMA accumulation order) -- outputs and BN tile partials,
    with bias, addend, forward (pack mode 16) and data-gradient (mode 17) weights;
  * against a float64 conv of the same bf16 operands (one bf16 rounding of the output);
  * the persistent tile walk: fewer tiles than CUs, several tiles per block, uneven splits,
    tiles crossing images, a half-empty last K chunk (Cin % 32 == 8 / 16);
  * deterministic (repeat launches bitwise equal); refuses shapes it cannot hold.
"""
import pytest
import torch
import torch.nn.functional as F

from seg_amd import engine
from seg_amd._lib import SegLibError, call, query

pytestmark = pytest.mark.gpu
DEV = "cuda"
BF = torch.bfloat16


def S():
    return torch.cuda.current_stream().cuda_stream


def r4(c):
    return (c + 3) & ~3


def r8(c):
    return (c + 7) & ~7


def rows(M, ld, seed, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(M, ld, generator=g) * scale + 0.1).to(BF).to(DEV)


def pack16(w, Cout, Cin, kin, mode):
    nrows = Cout if mode == 0 else Cin
    ld = r8(9 * kin)
    wk = torch.full((nrows * ld,), float("nan"), device=DEV).to(BF)
    table, n, blocks = engine.pack_table([(w.data_ptr(), wk.data_ptr(), Cout, Cin, 3, ld, mode | 16, kin)], w.device)
    call("seg_pack_batch", table.data_ptr(), n, blocks, S())
    return wk, ld


def run(name, x, ldx, N, H, W, cin_k, wk, ld, b, cout_k, add, stat):
    o = torch.full((N * H * W, cout_k), 3.0, device=DEV, dtype=BF)
    call(name, x.data_ptr(), ldx, N, H, W, cin_k, wk.data_ptr(), ld, b.data_ptr() if b is not None else None,
         o.data_ptr(), cout_k, cout_k, add.data_ptr() if add is not None else None, cout_k if add is not None else 0,
         stat.data_ptr() if stat is not None else None, S())
    return o


CASES = [  # N, Cin, Cout, H, W, mode (0 forward, 1 data gradient), bias, addend
    (2, 80, 32, 8, 64, 0, True, False),      # up4.0-like: half-empty last K chunk
    (1, 80, 32, 8, 128, 1, False, True),     # up4.0 data gradient: 80 outputs (3 column blocks), addend
    (3, 64, 64, 36, 192, 0, True, True),     # up3.3-like, 81 tiles (fewer than CUs), tiles cross images
    (4, 80, 32, 128, 256, 0, True, False),   # 512 tiles: two per block
    (3, 32, 32, 100, 256, 1, False, False),  # 300 tiles: uneven split over 256 blocks
    (1, 16, 16, 4, 64, 0, True, False),      # Cin = 16: one half-empty K chunk, a single tile
    (2, 40, 64, 12, 64, 0, True, True),      # nk = 2 with an 8-channel tail, addend
]


@pytest.mark.parametrize("N,Cin,Cout,H,W,mode,bias,addend", CASES)
def test_halo2_equals_halo_and_float64(N, Cin, Cout, H, W, mode, bias, addend):
    s = S()
    g = torch.Generator().manual_seed(N * 1000 + Cin * 10 + Cout)
    w = (torch.randn(Cout, Cin, 3, 3, generator=g) * 0.1).to(DEV)
    if mode == 0:
        cin_k, cout_k = Cin, Cout
    else:  # data gradient: dY (Cout channels) -> dX (Cin channels), transposed tap-flipped weights
        cin_k, cout_k = r4(Cout), Cin
    assert query("seg_conv_halo2_ok", N, H, W, cin_k, cout_k) == 1
    wk, ld = pack16(w, Cout, Cin, cin_k, mode)
    x = rows(N * H * W, cin_k, 3)
    b = torch.randn(cout_k, generator=g).to(DEV) if bias else None
    add = rows(N * H * W, cout_k, 4) if addend else None
    nt = query("seg_conv_halo2_row_tiles", N, H, W)
    assert nt == query("seg_conv_halo_row_tiles", N, H, W)
    st2, st1 = torch.empty(nt * 2 * cout_k, device=DEV), torch.empty(nt * 2 * cout_k, device=DEV)
    y2 = run("seg_conv_halo2_bf16io", x, cin_k, N, H, W, cin_k, wk, ld, b, cout_k, add, st2)
    y1 = run("seg_conv_halo_bf16io_w16", x, cin_k, N, H, W, cin_k, wk, ld, b, cout_k, add, st1)
    y2b = run("seg_conv_halo2_bf16io", x, cin_k, N, H, W, cin_k, wk, ld, b, cout_k, add, None)
    torch.cuda.synchronize()
    assert torch.equal(y2, y1), "same accumulation order as seg_conv_halo_bf16io_w16"
    assert torch.equal(st2, st1)
    assert torch.equal(y2, y2b), "deterministic"
    # float64 conv of the same bf16 operands
    xd = x.double().cpu().view(N, H, W, cin_k).permute(0, 3, 1, 2)
    wd = w.to(BF).double().cpu()
    if mode == 1:
        wd = wd.transpose(0, 1).flip(2, 3)  # [Cin][Cout][3][3]
        wd = F.pad(wd, (0, 0, 0, 0, 0, cin_k - Cout))
    ref = F.conv2d(xd, wd, padding=1).permute(0, 2, 3, 1).reshape(-1, cout_k)
    if b is not None:
        ref = ref + b.double().cpu()
    if add is not None:
        ref = ref + add.double().cpu()
    err = (y2.double().cpu() - ref).abs()
    assert float(err.max()) <= 2 ** -7 * float(ref.abs().max()), float(err.max())
    assert float((err.norm() / ref.norm())) < 4e-3
    # BN partials: per 256-pixel tile (4 rows x 64 columns) of the accumulators before the
    # addend, sum and M2 about the tile mean
    t = ref - add.double().cpu() if add is not None else ref
    t = t.view(N, H // 4, 4, W // 64, 64, cout_k).permute(0, 1, 3, 2, 4, 5).reshape(nt, 256, cout_k)
    sums = st2.view(nt, 2, cout_k)[:, 0].double().cpu()
    m2 = st2.view(nt, 2, cout_k)[:, 1].double().cpu()
    scale = float(t.abs().max())
    assert torch.allclose(sums, t.sum(1), rtol=1e-4, atol=1e-4 * 256 * scale)
    mu = t.mean(1, keepdim=True)
    assert torch.allclose(m2, ((t - mu) ** 2).sum(1), rtol=1e-3, atol=1e-4 * 256 * scale * scale)


def test_halo2_refuses_what_it_cannot_hold():
    assert query("seg_conv_halo2_ok", 1, 64, 128, 152, 64) == 0     # 9 x 64 x 160 weights exceed LDS
    assert query("seg_conv_halo2_ok", 1, 64, 128, 64, 128) == 0     # Cout > 96
    assert query("seg_conv_halo2_ok", 1, 62, 128, 64, 64) == 0      # H % 4
    assert query("seg_conv_halo2_ok", 1, 64, 96, 64, 64) == 0       # W % 64
    assert query("seg_conv_halo2_ok", 1, 64, 128, 20, 64) == 0      # Cin % 8
    x = rows(64 * 128, 152, 1)
    wk = torch.zeros(64 * r8(9 * 152), device=DEV, dtype=BF)
    out = torch.empty(64 * 128, 64, device=DEV, dtype=BF)
    with pytest.raises(SegLibError):
        call("seg_conv_halo2_bf16io", x.data_ptr(), 152, 1, 64, 128, 152, wk.data_ptr(), r8(9 * 152), None,
             out.data_ptr(), 64, 64, None, 0, None, S())


def test_engine_routes_narrow_convs_to_halo2(monkeypatch):
    """MobileNetV2UNet bf16io at bs=32 256x512 with SEG_HALO2=1 (default off since round 4): up4 / up3.3
    forward and data gradients on halo2."""
    from seg_amd import MobileNetV2UNet, deterministic_init
    monkeypatch.setattr(engine, "HALO2", True)
    m = deterministic_init(MobileNetV2UNet(10), seed=0).to(DEV).train()
    engine.set_conv_math(m, "bf16io")
    prog = engine.get_program(m, 32, 256, 512)
    prog._build_pack([op for op in prog.ops if isinstance(op, engine.ConvOp)], None)
    picked = {(op.cin, op.cout): (op.h2_f, op.h2_d) for op in prog.ops
              if isinstance(op, engine.ConvOp) and op.ks == 3 and not op.first}
    assert picked[(80, 32)] == (True, True)
    assert picked[(32, 32)] == (True, True)
    assert picked[(64, 64)] == (True, True)
    assert picked[(152, 64)] == (False, False)  # weights too large for LDS: implicit GEMM / halo
