"""GPU: the bf16io implicit GEMM on bf16-packed weights (seg_pack_batch modes 16/17 +
seg_conv_igemm_bf16io_w16 / _xf_w16) is bitwise the fp32-weight launch: the pack rounds
each weight RNE once, exactly as the fp32-weight kernel rounds it on its way into LDS."""
import pytest
import torch

from seg_amd import engine
from seg_amd._lib import call, query

pytestmark = pytest.mark.gpu
DEV = "cuda"
BF = torch.bfloat16


def S():
    return torch.cuda.current_stream().cuda_stream


def r4(c):
    return (c + 3) & ~3


def r8(c):
    return (c + 7) & ~7


def rows(M, ld, seed):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(M, ld, generator=g) * 1.3 + 0.2).to(BF).to(DEV)


def packs(w, Cout, Cin, ks, kin, mode):
    """(fp32 pack [rows][r4], bf16 pack [rows][r8]) of one conv weight through seg_pack_batch."""
    nrows = Cout if mode == 0 else Cin
    ld4, ld8 = r4(ks * ks * kin), r8(ks * ks * kin)
    w32 = torch.full((nrows * ld4,), float("nan"), device=DEV)
    w16 = torch.full((nrows * ld8,), float("nan"), device=DEV).to(BF)
    jobs = [(w.data_ptr(), w32.data_ptr(), Cout, Cin, ks, ld4, mode, kin),
            (w.data_ptr(), w16.data_ptr(), Cout, Cin, ks, ld8, mode | 16, kin)]
    table, n, blocks = engine.pack_table(jobs, w.device)
    call("seg_pack_batch", table.data_ptr(), n, blocks, S())
    torch.cuda.synchronize()
    a = w32.view(nrows, ld4)
    b = w16.view(nrows, ld8)
    assert torch.equal(b[:, :ld4].float(), a.to(BF).float()), "bf16 pack != RNE of the fp32 pack"
    assert not b[:, ld4:].float().any(), "bf16 pack not zero beyond K"
    return w32, ld4, w16, ld8


@pytest.mark.parametrize("N,Cin,Cout,H,W,ks,stride", [(2, 16, 96, 9, 13, 1, 1), (1, 152, 64, 10, 12, 3, 1),
                                                     (2, 4, 32, 12, 17, 3, 2), (1, 320, 1280, 4, 6, 1, 1),
                                                     (1, 1344, 256, 4, 8, 3, 1), (2, 24, 144, 5, 7, 1, 1)])
def test_igemm_w16_equals_fp32_weights(N, Cin, Cout, H, W, ks, stride):
    s = S()
    pad = ks // 2
    Ho, Wo = (H + 2 * pad - ks) // stride + 1, (W + 2 * pad - ks) // stride + 1
    M = N * Ho * Wo
    x = rows(N * H * W, Cin, 1)
    w = (torch.randn(Cout, Cin, ks, ks, generator=torch.Generator().manual_seed(2)) * 0.1).to(DEV)
    b = torch.randn(Cout, generator=torch.Generator().manual_seed(3)).to(DEV)
    w32, ld4, w16, ld8 = packs(w, Cout, Cin, ks, Cin, 0)
    ntiles = query("seg_conv_igemm_row_tiles", M, Cout, None)
    outs = {}
    for tag, name, wk, ld in (("f", "seg_conv_igemm_bf16io", w32, ld4), ("h", "seg_conv_igemm_bf16io_w16", w16, ld8)):
        y = torch.full((M, Cout), 7.0, device=DEV).to(BF)
        st = torch.empty(ntiles * 2 * Cout, device=DEV)
        call(name, x.data_ptr(), Cin, N, H, W, Cin, wk.data_ptr(), ld, b.data_ptr(), y.data_ptr(), Cout, Ho, Wo, Cout,
             ks, stride, pad, None, 0, st.data_ptr(), s)
        outs[tag] = (y, st)
    torch.cuda.synchronize()
    assert torch.equal(outs["f"][0], outs["h"][0]) and torch.equal(outs["f"][1], outs["h"][1])
    if stride != 1:
        return
    # data gradient (mode 1 pack: transposed, tap-flipped) with an addend
    kin = r4(Cout)
    dy = rows(M, kin, 4)
    add = rows(N * H * W, Cin, 5)
    d32, dl4, d16, dl8 = packs(w, Cout, Cin, ks, kin, 1)
    dx = {}
    for tag, name, wk, ld in (("f", "seg_conv_igemm_bf16io", d32, dl4), ("h", "seg_conv_igemm_bf16io_w16", d16, dl8)):
        o = torch.empty(N * H * W, Cin, device=DEV, dtype=BF)
        call(name, dy.data_ptr(), kin, N, H, W, kin, wk.data_ptr(), ld, None, o.data_ptr(), Cin, H, W, Cin, ks, 1, pad,
             add.data_ptr(), Cin, None, s)
        dx[tag] = o
    torch.cuda.synchronize()
    assert torch.equal(dx["f"], dx["h"])


@pytest.mark.parametrize("M,Cin,Cout", [(4096, 144, 24), (517, 16, 16), (2048, 320, 1280), (777, 960, 160)])
def test_igemm_xf_w16_equals_fp32_weights(M, Cin, Cout):
    s = S()
    y = rows(M, Cin, 6)
    g = torch.Generator().manual_seed(7)
    scale = (torch.rand(Cin, generator=g) + 0.5).to(DEV)
    shift = torch.randn(Cin, generator=g).to(DEV)
    w = (torch.randn(Cout, Cin, 1, 1, generator=g) * 0.1).to(DEV)
    w32, ld4, w16, ld8 = packs(w, Cout, Cin, 1, Cin, 0)
    ntiles = query("seg_conv_igemm_row_tiles", M, Cout, None)
    outs = {}
    for tag, name, wk, ld in (("f", "seg_conv_igemm_bf16io_xf", w32, ld4),
                              ("h", "seg_conv_igemm_bf16io_xf_w16", w16, ld8)):
        o = torch.empty(M, Cout, device=DEV, dtype=BF)
        st = torch.empty(ntiles * 2 * Cout, device=DEV)
        call(name, y.data_ptr(), Cin, 1, 1, M, Cin, wk.data_ptr(), ld, None, o.data_ptr(), Cout, 1, M, Cout, 1, 1, 0,
             None, 0, st.data_ptr(), scale.data_ptr(), shift.data_ptr(), 2, s)
        outs[tag] = (o, st)
    torch.cuda.synchronize()
    assert torch.equal(outs["f"][0], outs["h"][0]) and torch.equal(outs["f"][1], outs["h"][1])


def test_w16_rejects_unaligned_ldk():
    """ldk must be a multiple of 8 (16-byte bf16 weight slots): fail loudly otherwise."""
    from seg_amd._lib import SegLibError
    s = S()
    x = rows(64, 16, 8)
    wk = torch.zeros(16 * 20, device=DEV, dtype=BF)
    out = torch.empty(64, 16, device=DEV, dtype=BF)
    with pytest.raises(SegLibError):
        call("seg_conv_igemm_bf16io_w16", x.data_ptr(), 16, 1, 8, 8, 16, wk.data_ptr(), 20, None, out.data_ptr(), 16,
             8, 8, 16, 1, 1, 0, None, 0, None, s)


@pytest.mark.parametrize("N,Cin,Cout,H,W,mode", [(2, 80, 32, 8, 64, 0), (1, 152, 64, 4, 128, 0), (1, 32, 80, 8, 64, 1),
                                                 (1, 64, 64, 4, 64, 1)])
def test_halo_w16_equals_fp32_weights(N, Cin, Cout, H, W, mode):
    """seg_conv_halo_bf16io_w16 == seg_conv_halo_bf16io (forward pack mode 0, data-gradient pack mode 1)."""
    s = S()
    w = (torch.randn(Cout, Cin, 3, 3, generator=torch.Generator().manual_seed(9)) * 0.1).to(DEV)
    if mode == 0:
        cin_k, cout_k, kin = Cin, Cout, Cin
    else:   # data gradient: dY (Cout channels) -> dX (Cin channels)
        cin_k, cout_k, kin = r4(Cout), Cin, r4(Cout)
    w32, ld4, w16, ld8 = packs(w, Cout, Cin, 3, kin, mode)
    x = rows(N * H * W, cin_k, 10)
    b = torch.randn(cout_k, generator=torch.Generator().manual_seed(11)).to(DEV) if mode == 0 else None
    ntiles = query("seg_conv_halo_row_tiles", N, H, W)
    outs = {}
    for tag, name, wk, ld in (("f", "seg_conv_halo_bf16io", w32, ld4), ("h", "seg_conv_halo_bf16io_w16", w16, ld8)):
        o = torch.empty(N * H * W, cout_k, device=DEV, dtype=BF)
        st = torch.empty(ntiles * 2 * cout_k, device=DEV)
        call(name, x.data_ptr(), cin_k, N, H, W, cin_k, wk.data_ptr(), ld, b.data_ptr() if b is not None else None,
             o.data_ptr(), cout_k, cout_k, None, 0, st.data_ptr(), s)
        outs[tag] = (o, st)
    torch.cuda.synchronize()
    assert torch.equal(outs["f"][0], outs["h"][0]) and torch.equal(outs["f"][1], outs["h"][1])
