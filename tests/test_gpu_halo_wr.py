"""GPU: the weight-resident persistent LDS-halo conv (csrc/halo.hip halo3x3_wr_kernel, round 6) is bitwise the
per-tile kernel (halo3x3_kernel) it replaces where the packed weights fit its LDS -- outputs, BN partials and the
addend -- for the bf16io (bf16 and fp32-packed weights) and fp32 kernels, ragged Cout, Cin that is not a whole number
of K chunks, and tile counts that do not divide over the XCDs; and both match a float64 conv of the same operand
rounding.  The narrow decoder convs of src/unet.py:58,61 (UNet 512x1024's 64-channel levels, MobileNetV2UNet up3/up4)."""
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


@pytest.mark.parametrize("kind", ["bf16io_w16", "bf16io", "f32"])
@pytest.mark.parametrize("N,H,W,Cin,Cout", [(8, 64, 256, 64, 64), (9, 64, 256, 32, 32), (8, 64, 256, 80, 32),
                                            (8, 64, 256, 64, 20), (2, 128, 512, 48, 60)])
def test_halo_wr_bitwise_per_tile_kernel(kind, N, H, W, Cin, Cout):
    if kind == "f32" and Cout > 32:
        pytest.skip("fp32: the weight-resident form takes Cout <= 32")
    bf = kind != "f32"
    g = torch.Generator().manual_seed(N * Cin + Cout)
    M = N * H * W
    x = torch.randn(M, Cin, generator=g)
    w = torch.randn(Cout, Cin, 3, 3, generator=g) / (9 * Cin) ** 0.5
    b = torch.randn(Cout, generator=g).to(DEV)
    ldo = Cout + 8 if Cout % 8 else Cout
    add = torch.randn(M, ldo, generator=g)
    wg = w.to(DEV)
    ldk = 9 * Cin
    if kind == "bf16io_w16":
        wk = torch.empty(Cout * ldk, device=DEV, dtype=BF)
        mode = 16
    else:
        wk = torch.empty(Cout * ldk, device=DEV)
        mode = 0
    table, n, blocks = engine.pack_table([(wg.data_ptr(), wk.data_ptr(), Cout, Cin, 3, ldk, mode, Cin)], wg.device)
    call("seg_pack_batch", table.data_ptr(), n, blocks, S())
    dt = BF if bf else torch.float32
    xg, ag = x.to(dt).to(DEV), add.to(dt).to(DEV)
    name = {"bf16io_w16": "seg_conv_halo_bf16io_w16", "bf16io": "seg_conv_halo_bf16io", "f32": "seg_conv_halo"}[kind]
    ntiles = query("seg_conv_halo_row_tiles", N, H, W)
    res = []
    old = query("seg_halo_wr", -1)
    try:
        for wr in (0, 1):
            query("seg_halo_wr", wr)
            out = torch.full((M, ldo), float("nan"), device=DEV, dtype=dt)
            stat = torch.full((ntiles * 2 * Cout,), float("nan"), device=DEV)
            call(name, xg.data_ptr(), Cin, N, H, W, Cin, wk.data_ptr(), ldk, b.data_ptr(), out.data_ptr(), ldo, Cout,
                 ag.data_ptr(), ldo, stat.data_ptr(), S())
            torch.cuda.synchronize()
            res.append((out, stat))
    finally:
        query("seg_halo_wr", old)
    (o0, s0), (o1, s1) = res
    assert not torch.isnan(o1[:, :Cout]).any() and not torch.isnan(s1).any()
    assert torch.equal(o0[:, :Cout], o1[:, :Cout]), "weight-resident kernel == per-tile kernel"
    assert torch.equal(s0, s1), "BN partials"
    if ldo > Cout:
        assert bool(o1[:, Cout:].isnan().all()), "nothing written beyond Cout"
    # float64 of the same operand rounding
    xr = x.to(dt).double() if bf else x.double()
    wr_ = w.to(BF).double() if bf else w.double()
    ref = F.conv2d(xr.view(N, H, W, Cin).permute(0, 3, 1, 2), wr_, padding=1) + b.double().cpu()[None, :, None, None]
    ref = ref.permute(0, 2, 3, 1).reshape(M, Cout) + add[:, :Cout].to(dt).double()
    got = o1[:, :Cout].double().cpu()
    tol = 1e-2 if bf else 1e-5  # bf16 output rounding
    assert float((got - ref).norm() / ref.norm()) < tol
