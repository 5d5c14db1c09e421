"""GPU: thin-K pointwise convs (seg_conv_pw / seg_conv_pw_bf16io, include/segamd.h) against a
float64 torch reference of the same (rounded) operands: the output, the fused addend, the BN
tile partials (tile sum and M2 about the tile mean of 128-row tiles, as seg_bn_stats_tiles
reads them) and the lazy-BN input transform.  Model level: every test_gpu_model / bf16io run
takes this kernel for the expand / head 1x1 convs and the thin project-conv data gradients.
"""
import pytest
import torch

from seg_amd._lib import SegLibError, call, query

pytestmark = pytest.mark.gpu
DEV = "cuda"
BF = torch.bfloat16


def S():
    return torch.cuda.current_stream().cuda_stream


@pytest.mark.parametrize("io", [False, True])
@pytest.mark.parametrize("M,K,N", [(5000, 16, 96), (20000, 24, 144), (4096, 32, 192), (777, 16, 10), (1024, 32, 16),
                                   (3000, 24, 32), (129, 8, 40)])
@pytest.mark.parametrize("mode", ["plain", "bias_stat", "add", "xf"])
def test_pw_matches_float64(io, M, K, N, mode):
    s = S()
    dt = BF if io else torch.float32
    v = 8 if io else 4
    ldin = (K + v - 1) // v * v
    ldo = (N + v - 1) // v * v
    g = torch.Generator().manual_seed(M + K + N)
    x = (torch.randn(M, ldin, generator=g) * 1.3 + 0.2).to(BF).float()
    w = (torch.randn(N, K, generator=g) * 0.2).to(BF).float()
    b = torch.randn(N, generator=g) if mode == "bias_stat" else None
    add = (torch.randn(M, ldo, generator=g)).to(BF).float() if mode == "add" else None
    xs = (torch.rand(K, generator=g) + 0.5) if mode == "xf" else None
    xb = torch.randn(K, generator=g) if mode == "xf" else None
    xg = x.to(DEV).to(dt)
    ldk = (K + v - 1) // v * v
    wk = torch.zeros(N, ldk, device=DEV, dtype=dt)
    wk[:, :K] = w.to(DEV).to(dt)
    out = torch.full((M, ldo), 5.0, device=DEV, dtype=dt)
    addg = add.to(DEV).to(dt) if add is not None else None
    if addg is not None:
        out.copy_(addg)
    tiles = query("seg_conv_pw_row_tiles", M)
    stat = torch.zeros(tiles * 2 * N, device=DEV) if mode == "bias_stat" else None
    xsg = xs.to(DEV) if xs is not None else None
    xbg = xb.to(DEV) if xb is not None else None
    call("seg_conv_pw_bf16io" if io else "seg_conv_pw", xg.data_ptr(), ldin, M, K, wk.data_ptr(), ldk,
         b.to(DEV).data_ptr() if b is not None else None, out.data_ptr(), ldo, N,
         out.data_ptr() if addg is not None else None, ldo if addg is not None else 0,
         stat.data_ptr() if stat is not None else None, xsg.data_ptr() if xsg is not None else None,
         xbg.data_ptr() if xbg is not None else None, 2 if mode == "xf" else 0, s)
    torch.cuda.synchronize()
    a = x[:, :K].double()
    if mode == "xf":
        a = torch.clamp(a * xs.double() + xb.double(), 0, 6)
        if io:
            a = a.float().to(BF).double()  # the apply pass would store bf16
        else:
            a = (x[:, :K] * xs + xb).clamp(0, 6).double()
    ref = a @ w.double().t()
    if b is not None:
        ref = ref + b.double()
    pre = ref.clone()
    if add is not None:
        ref = ref + add[:, :N].double()
    got = out[:, :N].double().cpu()
    tol = 2.0 ** -7 if io else 1e-5
    err = (got - ref).abs().max().item() / max(ref.abs().max().item(), 1e-6)
    assert err <= tol, err
    if ldo > N:
        pad = out[:, N:].float().cpu()
        exp = add[:, N:] if add is not None else torch.full_like(pad, 5.0)
        assert torch.equal(pad, exp.to(BF).float() if io else exp)
    if stat is not None:
        st = stat.view(tiles, 2, N).double().cpu()
        for t in range(tiles):
            blk = pre[t * 128:(t + 1) * 128]
            assert torch.allclose(st[t, 0], blk.sum(0), rtol=1e-4, atol=1e-3)
            m2 = ((blk - blk.mean(0)) ** 2).sum(0)
            assert torch.allclose(st[t, 1], m2, rtol=1e-3, atol=1e-3)


def test_pw_rejects_unsupported_shapes():
    t = torch.zeros(64, 64, device=DEV)
    with pytest.raises(SegLibError):  # K = 40 > 32
        call("seg_conv_pw", t.data_ptr(), 64, 64, 40, t.data_ptr(), 64, None, t.data_ptr(), 64, 16, None, 0, None,
             None, None, 0, S())
    with pytest.raises(SegLibError):  # K % 8 != 0
        call("seg_conv_pw", t.data_ptr(), 64, 64, 12, t.data_ptr(), 64, None, t.data_ptr(), 64, 16, None, 0, None,
             None, None, 0, S())
