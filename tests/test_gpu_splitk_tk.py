"""GPU: split-K convs combined inside the launch (seg_conv_igemm_act_tk / _bf16_tk / _f16_tk,
include/segamd.h) -- the batch-1 inference convs -- against the two-launch path (raw partials
+ the fixed-order reduce pass of seg_conv_igemm_act / _bf16 / _f16).

The last-arriving K range sums the ranges of its tile in range order and applies the same
epilogue, so the outputs must be bitwise equal, the ticket words must be left zero, and a
second call (re-armed tickets) must reproduce the first.  Model level: tests/test_gpu_infer.py.
"""
import pytest
import torch

from seg_amd._lib import SegLibError, call, query

pytestmark = pytest.mark.gpu
DEV = "cuda"


def S():
    return torch.cuda.current_stream().cuda_stream


def r4(n):
    return (n + 3) // 4 * 4


@pytest.mark.parametrize("name", ["seg_conv_igemm_act", "seg_conv_igemm_bf16", "seg_conv_igemm_f16"])
@pytest.mark.parametrize("N,Cin,Cout,H,W,ks,res,act", [(1, 1344, 256, 8, 16, 3, False, 1), (1, 288, 128, 16, 32, 3, False, 2),
                                                       (1, 960, 320, 8, 16, 1, True, 0), (1, 320, 1280, 4, 8, 1, False, 2),
                                                       (2, 80, 32, 9, 11, 3, True, 1), (1, 152, 10, 16, 32, 1, False, 0)])
def test_tk_matches_reduce_pass(name, N, Cin, Cout, H, W, ks, res, act):
    s = S()
    g = torch.Generator().manual_seed(7)
    M = N * H * W
    pad = ks // 2
    x = torch.randn(M, Cin, generator=g).to(DEV)
    w = (torch.randn(Cout, Cin, ks, ks, generator=g) * (2.0 / (Cin * ks * ks)) ** 0.5).to(DEV)
    b = torch.randn(Cout, generator=g).to(DEV)
    add = torch.randn(M, r4(Cout), generator=g).to(DEV) if res else None
    ldk = r4(ks * ks * Cin)
    wk = torch.empty(Cout * ldk, device=DEV)
    call("seg_pack_conv_weight", w.data_ptr(), wk.data_ptr(), Cout, Cin, ks, ldk, 0, Cin, s)
    auto = query("seg_conv_igemm_splits", M, Cout, Cin, ks)
    nt = query("seg_conv_igemm_tickets", M, Cout)
    assert nt >= 1
    tickets = torch.zeros(nt + 16, device=DEV, dtype=torch.int32)
    common = (x.data_ptr(), Cin, N, H, W, Cin, wk.data_ptr(), ldk, b.data_ptr())
    tail = (H, W, Cout, ks, 1, pad, add.data_ptr() if res else None, add.shape[1] if res else 0)
    for splits in sorted({auto, 3, 7}):
        ref = torch.full((M, r4(Cout)), float("nan"), device=DEV)
        work = torch.empty(splits * M * Cout, device=DEV)
        call(name, *common, ref.data_ptr(), ref.shape[1], *tail, None, act, work.data_ptr(), splits, s)
        for rep in range(2):
            out = torch.full((M, r4(Cout)), float("nan"), device=DEV)
            work2 = torch.full((splits * M * Cout,), float("nan"), device=DEV)
            call(name + "_tk", *common, out.data_ptr(), out.shape[1], *tail, act, work2.data_ptr(), splits,
                 tickets.data_ptr(), s)
            torch.cuda.synchronize()
            assert torch.equal(out[:, :Cout], ref[:, :Cout]), (splits, rep, (out - ref)[:, :Cout].abs().max())
            assert int(tickets.abs().sum()) == 0, "tickets re-armed"


def test_tk_needs_tickets_when_split():
    s = S()
    x = torch.zeros(128, 1344, device=DEV)
    wk = torch.zeros(256 * 9 * 1344, device=DEV)
    out = torch.zeros(128, 256, device=DEV)
    work = torch.zeros(4 * 128 * 256, device=DEV)
    with pytest.raises(SegLibError):
        call("seg_conv_igemm_act_tk", x.data_ptr(), 1344, 1, 8, 16, 1344, wk.data_ptr(), 9 * 1344, None,
             out.data_ptr(), 256, 8, 16, 256, 3, 1, 1, None, 0, 0, work.data_ptr(), 4, None, s)
