"""GPU: seg_conv_igemm_{act,bf16,f16}_ic -- the implicit GEMM's split-K with the combine inside the
launch (the batch-1 convs of the folded inference forward, inference.py:162-163 through
src/unet.py:58-64,113-116): bitwise the two-launch split-K (same fixed-order sum and epilogue),
repeat launches equal, tile counters re-armed."""
import pytest
import torch

from seg_amd._lib import call, query

pytestmark = pytest.mark.gpu
DEV = "cuda"


def S():
    return torch.cuda.current_stream().cuda_stream


CASES = [  # N, H, W, Cin, Cout, ks, act, addend -- decoder convs of a 128x256 frame, a head conv, ragged
    (1, 8, 16, 1344, 256, 3, 1, False), (1, 16, 32, 288, 128, 3, 1, False), (1, 32, 64, 152, 64, 3, 1, True),
    (1, 4, 8, 160, 960, 1, 2, False), (1, 5, 7, 64, 100, 3, 0, True),
]


@pytest.mark.parametrize("name", ["seg_conv_igemm_act", "seg_conv_igemm_bf16", "seg_conv_igemm_f16"])
@pytest.mark.parametrize("N,H,W,Cin,Cout,ks,act,addend", CASES)
def test_splitk_in_launch_equals_two_launch(name, N, H, W, Cin, Cout, ks, act, addend):
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
    cnt = torch.zeros(2 * query("seg_conv_igemm_tiles", M, Cout), device=DEV, dtype=torch.int32)
    work2 = torch.full_like(work, float("nan"))
    for _ in range(2):
        o = torch.full((M, Cout), float("nan"), device=DEV)
        call(name + "_ic", x.data_ptr(), Cin, N, H, W, Cin, w.data_ptr(), ldk, b.data_ptr(), o.data_ptr(), Cout, H, W,
             Cout, ks, 1, ks // 2, add.data_ptr() if addend else None, Cout if addend else 0, act, work2.data_ptr(),
             splits, cnt.data_ptr(), S())
        outs.append(o)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], ref) and torch.equal(outs[1], ref)
    assert int(cnt.abs().sum()) == 0
