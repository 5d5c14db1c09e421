"""GPU: seg_conv_wgrad3_bf16io -- the LDS-DMA weight gradient of the wide bf16 3x3 / 1x1 convs (csrc/wgrad3.hip)
against a float64 weight gradient of the same bf16 operands and against the register-staged seg_conv_wgrad_bf16io.

dW[co][ci][ky][kx] = sum_p dY[p][co] X[p + (ky - 1, kx - 1)][ci] is the weight path of src/unet.py:58,61's
double_conv (loss.backward() at src/train.py:38).  Both kernels accumulate the same bf16 products in fp32 over
different split-K slices, so they agree to fp32 accumulation-order rounding, not bitwise; each is deterministic.
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
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


CASES = [  # N, H, W, Cin, Cout, ks: 128- and 64-channel output tiles, ragged n tiles, taps wrapping, 1x1
    (2, 8, 64, 128, 128, 3), (1, 4, 128, 64, 256, 3), (2, 6, 64, 256, 64, 3), (2, 4, 64, 256, 192, 1),
    (1, 16, 64, 64, 64, 3), (1, 2, 128, 512, 128, 3), (2, 5, 192, 96, 48, 3), (1, 3, 64, 1344, 256, 3),
    (4, 8, 64, 152, 64, 3), (2, 4, 64, 256, 256, 1)]


@pytest.mark.parametrize("N,H,W,Cin,Cout,ks", CASES)
def test_wgrad3_vs_fp64_and_wgrad(N, H, W, Cin, Cout, ks):
    splits = query("seg_conv_wgrad3_splits", N, H, W, Cin, Cout, ks)
    assert splits > 0, "the plan must apply to these shapes"
    M = N * H * W
    g = torch.Generator().manual_seed(N * 7 + Cin + Cout)
    ldx, lddy = Cin + 8, Cout
    x = (torch.randn(M, ldx, generator=g) * 1.2 + 0.1).to(BF)
    dy = (torch.randn(M, lddy, generator=g)).to(BF)
    xg, dyg = x.to(DEV), dy.to(DEV)
    # float64 reference on the same bf16 values
    x64 = x[:, :Cin].double().view(N, H, W, Cin).permute(0, 3, 1, 2)
    dy64 = dy[:, :Cout].double().view(N, H, W, Cout).permute(0, 3, 1, 2)
    ref = torch.nn.grad.conv2d_weight(x64, (Cout, Cin, ks, ks), dy64, padding=ks // 2)
    dws = []
    for rep in range(2):
        part = torch.full((splits * Cout * ks * ks * Cin,), float("nan"), device=DEV)
        call("seg_conv_wgrad3_bf16io", dyg.data_ptr(), lddy, xg.data_ptr(), ldx, N, H, W, Cin, Cout, ks,
             part.data_ptr(), S())
        dw = torch.empty(Cout, Cin, ks, ks, device=DEV)
        call("seg_conv_wgrad_reduce", part.data_ptr(), splits, dw.data_ptr(), Cout, Cin, ks, 0, 0, S())
        dws.append(dw)
    torch.cuda.synchronize()
    assert torch.equal(dws[0], dws[1]), "deterministic"
    assert rel(dws[0], ref) < 2e-5
    # the register-staged kernel on the same operands
    s2 = query("seg_conv_wgrad_splits_bf16", M, Cout, Cin, ks)
    part = torch.empty(s2 * Cout * ks * ks * Cin, device=DEV)
    call("seg_conv_wgrad_bf16io", dyg.data_ptr(), lddy, xg.data_ptr(), ldx, N, H, W, Cin, H, W, Cout, ks, 1, ks // 2,
         part.data_ptr(), s2, S())
    dw2 = torch.empty(Cout, Cin, ks, ks, device=DEV)
    call("seg_conv_wgrad_reduce", part.data_ptr(), s2, dw2.data_ptr(), Cout, Cin, ks, 0, 0, S())
    torch.cuda.synchronize()
    assert rel(dws[0], dw2) < 2e-5


def test_wgrad3_plan_rejects():
    assert query("seg_conv_wgrad3_splits", 2, 8, 32, 128, 128, 3) == 0    # W % 64
    assert query("seg_conv_wgrad3_splits", 2, 8, 64, 12, 128, 3) == 0     # Cin % 8
    assert query("seg_conv_wgrad3_splits", 2, 8, 64, 128, 16, 3) == 0     # Cout < 32
    assert query("seg_conv_wgrad3_splits", 8, 512, 1024, 64, 64, 3) > 0   # UNet's full-resolution 64 -> 64
