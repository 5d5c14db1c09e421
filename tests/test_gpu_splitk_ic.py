"""GPU: seg_conv_igemm_{act,bf16,f16}_ic -- the implicit GEMM's split-K with the combine inside the
launch (the batch-1 convs of the folded inference forward, inference.py:162-163 through
src/unet.py:58-64,113-116): bitwise the two-launch split-K (same fixed-order sum and epilogue),
repeat launches equal, the tiles' epoch words advanced with no count or hand-off bit left over; the batch-1 plan's tiles (seg_conv_igemm_plan_b1) give
the two-launch result at the same split count."""
import ctypes

import pytest
import torch

from seg_amd._lib import call, query

pytestmark = pytest.mark.gpu
DEV = "cuda"


def S():
    return torch.cuda.current_stream().cuda_stream


def check_epoch_words(cnt, launches):
    """seg_tile_combine's per-tile 64-bit words after `launches` launches: arrival count and hand-off mask clear,
    the epoch advanced once per launch (or untouched when a launch fell back to the separate reduce)."""
    wv = cnt.view(-1, 4)
    assert int(wv[:, 0].abs().sum()) == 0 and int(wv[:, 2:].abs().sum()) == 0
    assert bool(((wv[:, 1] == 0) | (wv[:, 1] == launches << 6)).all())


CASES = [  # N, H, W, Cin, Cout, ks, act, addend -- decoder convs of a 128x256 frame, a head conv, ragged
    (1, 8, 16, 1344, 256, 3, 1, False), (1, 16, 32, 288, 128, 3, 1, False), (1, 32, 64, 152, 64, 3, 1, True),
    (1, 4, 8, 160, 960, 1, 2, False), (1, 5, 7, 64, 100, 3, 0, True),
]


@pytest.mark.parametrize("spin", [-1, 0])
@pytest.mark.parametrize("name", ["seg_conv_igemm_act", "seg_conv_igemm_bf16", "seg_conv_igemm_f16"])
@pytest.mark.parametrize("N,H,W,Cin,Cout,ks,act,addend", CASES)
def test_splitk_in_launch_equals_two_launch(name, N, H, W, Cin, Cout, ks, act, addend, spin):
    """spin 0 (seg_set_combine_spin): every block but a tile's last hands its share to the last arrival."""
    M = N * H * W
    splits = query("seg_conv_igemm_splits", M, Cout, Cin, ks)
    if splits == 1:
        pytest.skip("no split-K at this shape")
    g = torch.Generator().manual_seed(M + Cin)
    x = torch.randn(M, Cin, generator=g).to(DEV)
    ldk = ks * ks * Cin
    w = (torch.randn(Cout, ldk, generator=g) * 0.05).to(DEV)  # a packed [Cout][K] weight as is
    b = torch.randn(Cout, generator=g).to(DEV)
    add = torch.randn(M, Cout, generator=g).to(DEV) if addend else None
    work = torch.empty(splits * M * Cout, device=DEV)
    outs = []
    ref = torch.empty(M, Cout, device=DEV)
    call(name, x.data_ptr(), Cin, N, H, W, Cin, w.data_ptr(), ldk, b.data_ptr(), ref.data_ptr(), Cout, H, W, Cout, ks,
         1, ks // 2, add.data_ptr() if addend else None, Cout if addend else 0, None, act, work.data_ptr(), splits, S())
    cnt = torch.zeros(4 * query("seg_conv_igemm_tiles", M, Cout), device=DEV, dtype=torch.int32)
    work2 = torch.full_like(work, float("nan"))
    call("seg_set_combine_spin", spin)
    try:
        for _ in range(2):
            o = torch.full((M, Cout), float("nan"), device=DEV)
            call(name + "_ic", x.data_ptr(), Cin, N, H, W, Cin, w.data_ptr(), ldk, b.data_ptr(), o.data_ptr(), Cout, H,
                 W, Cout, ks, 1, ks // 2, add.data_ptr() if addend else None, Cout if addend else 0, act,
                 work2.data_ptr(), splits, -1, cnt.data_ptr(), S())
            outs.append(o)
        torch.cuda.synchronize()
    finally:
        call("seg_set_combine_spin", -1)
    assert torch.equal(outs[0], ref) and torch.equal(outs[1], ref)
    check_epoch_words(cnt, 2)


B1 = [  # the folded inference forward's decoder convs of a 128x256 frame (tools/icbench.py) + a 1x1 head conv
    (8, 16, 1344, 256, 3), (8, 16, 256, 256, 3), (16, 32, 288, 128, 3), (16, 32, 128, 128, 3), (32, 64, 152, 64, 3),
    (32, 64, 64, 64, 3), (64, 128, 80, 32, 3), (64, 128, 32, 32, 3), (4, 8, 320, 1280, 1), (5, 7, 64, 100, 3)]


def plan_b1(M, Cout, Cin, ks):
    out = (ctypes.c_int * 3)()
    assert query("seg_conv_igemm_plan_b1", M, Cout, Cin, ks, ctypes.addressof(out)) == 0
    return list(out)


@pytest.mark.parametrize("name", ["seg_conv_igemm_act", "seg_conv_igemm_f16"])
@pytest.mark.parametrize("H,W,Cin,Cout,ks", B1)
def test_plan_b1_equals_cost_model_tile(name, H, W, Cin, Cout, ks):
    """The plan's tile (8-wave 128x64 / 64x64) against the cost model's tile at the plan's split count:
    bitwise (tile choice keeps every output's K order); epoch words advanced, nothing left over."""
    M = H * W
    splits, tile, ntl = plan_b1(M, Cout, Cin, ks)
    assert tile in (-1, 3, 12) and splits >= 1 and ntl >= 1
    g = torch.Generator().manual_seed(M + Cout)
    x = torch.randn(M, Cin, generator=g).to(DEV)
    ldk = ks * ks * Cin
    w = (torch.randn(Cout, ldk, generator=g) * 0.05).to(DEV)
    b = torch.randn(Cout, generator=g).to(DEV)
    work = torch.empty(max(splits * M * Cout, 1), device=DEV)
    ref = torch.empty(M, Cout, device=DEV)
    call(name, x.data_ptr(), Cin, 1, H, W, Cin, w.data_ptr(), ldk, b.data_ptr(), ref.data_ptr(), Cout, H, W, Cout, ks,
         1, ks // 2, None, 0, None, 1, work.data_ptr() if splits > 1 else None, splits, S())
    cnt = torch.zeros(4 * ntl, device=DEV, dtype=torch.int32)
    work2 = torch.full_like(work, float("nan"))
    for _ in range(2):
        o = torch.full((M, Cout), float("nan"), device=DEV)
        call(name + "_ic", x.data_ptr(), Cin, 1, H, W, Cin, w.data_ptr(), ldk, b.data_ptr(), o.data_ptr(), Cout, H, W,
             Cout, ks, 1, ks // 2, None, 0, 1, work2.data_ptr(), splits, tile, cnt.data_ptr(), S())
        torch.cuda.synchronize()
        assert torch.equal(o, ref)
    check_epoch_words(cnt, 2)
