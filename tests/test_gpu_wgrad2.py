"""GPU: seg_conv_wgrad2_bf16io -- the persistent LDS-halo weight gradient of the narrow bf16io
3x3 convs (csrc/wgrad2.hip; aten's convolution_backward weight path of src/unet.py:58,61 at
MobileNetV2UNet up3 / up4 and UNet's 64-channel levels), reduced by seg_conv_wgrad_reduce.

  * against float64 (torch.nn.grad.conv2d_weight of the same bf16 operands): fp32 accumulation;
  * against the implicit-GEMM weight gradient (seg_conv_wgrad_bf16io) the engine used before;
  * one and two output blocks (Cout <= 32 / <= 64), channel groups walked more than once
    (Cin 152: five 32-channel chunks), Cout 16 (a partly empty block), tiles crossing images,
    fewer tiles than CUs; repeat launches bitwise equal (fixed-order slabs, no atomics).
"""
import pytest
import torch

from seg_amd._lib import call, query

pytestmark = pytest.mark.gpu
DEV = "cuda"
BF = torch.bfloat16


def S():
    return torch.cuda.current_stream().cuda_stream


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


CASES = [  # N, Cin, Cout, H, W
    (2, 80, 32, 8, 64), (1, 32, 32, 8, 128), (3, 64, 64, 36, 192), (4, 152, 64, 12, 64), (2, 40, 16, 4, 64),
    (8, 80, 32, 32, 256),
]


@pytest.mark.parametrize("N,Cin,Cout,H,W", CASES)
def test_wgrad2_vs_fp64_and_implicit_gemm(N, Cin, Cout, H, W):
    assert query("seg_conv_wgrad2_ok", N, H, W, Cin, Cout) == 1
    M = N * H * W
    g = torch.Generator().manual_seed(M + Cin)
    x = torch.randn(M, Cin, generator=g).to(BF)
    dy = torch.randn(M, Cout, generator=g).to(BF)
    xg, dyg = x.to(DEV), dy.to(DEV)
    blocks = query("seg_conv_wgrad2_blocks", N, H, W)
    part = torch.full((blocks * Cout * 9 * Cin,), float("nan"), device=DEV)
    outs = []
    for _ in range(2):
        dw = torch.empty(Cout, Cin, 3, 3, device=DEV)
        call("seg_conv_wgrad2_bf16io", dyg.data_ptr(), Cout, xg.data_ptr(), Cin, N, H, W, Cin, Cout, part.data_ptr(),
             S())
        call("seg_conv_wgrad_reduce", part.data_ptr(), blocks, dw.data_ptr(), Cout, Cin, 3, 0, 0, S())
        outs.append(dw)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1]), "deterministic"
    ref = torch.nn.grad.conv2d_weight(x.double().view(N, H, W, Cin).permute(0, 3, 1, 2), (Cout, Cin, 3, 3),
                                      dy.double().view(N, H, W, Cout).permute(0, 3, 1, 2), padding=1)
    assert rel(outs[0], ref) < 1e-5
    # the implicit-GEMM weight gradient on the same operands
    splits = query("seg_conv_wgrad_splits_bf16", M, Cout, Cin, 3)
    p2 = torch.empty(splits * Cout * 9 * Cin, device=DEV)
    dw2 = torch.empty(Cout, Cin, 3, 3, device=DEV)
    call("seg_conv_wgrad_bf16io", dyg.data_ptr(), Cout, xg.data_ptr(), Cin, N, H, W, Cin, H, W, Cout, 3, 1, 1,
         p2.data_ptr(), splits, S())
    call("seg_conv_wgrad_reduce", p2.data_ptr(), splits, dw2.data_ptr(), Cout, Cin, 3, 0, 0, S())
    torch.cuda.synchronize()
    assert rel(outs[0], dw2) < 1e-5


def test_wgrad2_refuses_what_it_cannot_hold():
    assert query("seg_conv_wgrad2_ok", 1, 64, 128, 64, 128) == 0   # Cout > 64
    assert query("seg_conv_wgrad2_ok", 1, 62, 128, 64, 64) == 0    # H % 4
    assert query("seg_conv_wgrad2_ok", 1, 64, 96, 64, 64) == 0     # W % 64
    assert query("seg_conv_wgrad2_ok", 1, 64, 128, 4, 32) == 0     # Cin % 8 (the stem)
