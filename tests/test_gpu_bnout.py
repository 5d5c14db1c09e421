"""GPU: the BatchNorm-backward reduction from the epilogue of the implicit-GEMM data gradient
that completes a BN layer's dA (seg_conv_igemm_bnout*, csrc/igemm_impl.h; finalized by
seg_bn_bwd_finalize_tiles) -- in place of seg_bn_backward's reduction pass over dA (the
BN-backward chain of src/unet.py:59-63 and torchvision's BatchNorm via src/unet.py:15-19).

  * the conv output is bitwise that of the plain launch (same kernel body and store);
  * dgamma / dbeta / coef from the tile partials match seg_bn_bwd_coef over the stored output
    (fp32 partials in another grouping, fp64 finalize: rel 1e-5); f32, bf16io and bf16io with
    bf16 packed weights; 1x1 and 3x3; with a fused addend; ReLU6 / ReLU / no activation mask;
  * the whole MobileNetV2UNet / UNet f32 step with SEG_BNOUT on equals it off within fp32 reduction
    reordering; the oracle checks of test_gpu_model.py / test_gpu_bf16io.py run with it on (the
    default).
"""
import pytest
import torch

from seg_amd import engine
from seg_amd._lib import call, query

pytestmark = pytest.mark.gpu
DEV = "cuda"
BF = torch.bfloat16


def S():
    return torch.cuda.current_stream().cuda_stream


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


def r8(c):
    return (c + 7) & ~7


def pack(w, Cout, Cin, ks, w16):
    ldk = r8(ks * ks * Cin)
    wk = torch.zeros(Cout * ldk, device=DEV, dtype=BF if w16 else torch.float32)
    table, n, blocks = engine.pack_table([(w.data_ptr(), wk.data_ptr(), Cout, Cin, ks, ldk, 16 if w16 else 0, Cin)],
                                         w.device)
    call("seg_pack_batch", table.data_ptr(), n, blocks, S())
    return wk, ldk


CASES = [  # N, H, W, Cin, Cout (= the BN layer's channels), ks, act, addend
    (32, 16, 32, 64, 384, 1, 2, False), (32, 8, 16, 160, 960, 1, 2, True), (32, 32, 64, 192, 32, 1, 0, True),
    (8, 16, 32, 96, 64, 3, 1, False), (4, 32, 64, 144, 24, 1, 0, False), (2, 20, 30, 64, 128, 3, 2, True),
]


@pytest.mark.parametrize("math", ["f32", "bf16io", "bf16io_w16"])
@pytest.mark.parametrize("N,H,W,Cin,Cout,ks,act,addend", CASES)
def test_bnout_partials(math, N, H, W, Cin, Cout, ks, act, addend):
    io = math != "f32"
    dt = BF if io else torch.float32
    M = N * H * W
    if not query("seg_conv_igemm_bnout_ok", M, Cout, int(io)):
        pytest.skip("the picked tile has no per-lane column vector")
    g = torch.Generator().manual_seed(M + Cin + Cout)
    x = torch.randn(M, Cin, generator=g).to(dt).to(DEV)
    w = (torch.randn(Cout, Cin, ks, ks, generator=g) * 0.1).to(DEV)
    add = torch.randn(M, Cout, generator=g).to(dt).to(DEV) if addend else None
    y = (torch.randn(M, Cout, generator=g) * 2).to(dt).to(DEV)
    mean = (torch.randn(Cout, generator=g) * 0.3).to(DEV)
    invstd = (torch.rand(Cout, generator=g) + 0.5).to(DEV)
    gamma = (torch.rand(Cout, generator=g) + 0.5).to(DEV)
    scale = gamma * invstd
    shift = (torch.randn(Cout, generator=g) * 0.2).to(DEV) - mean * scale
    wk, ldk = pack(w, Cout, Cin, ks, math == "bf16io_w16")
    name = {"f32": "seg_conv_igemm", "bf16io": "seg_conv_igemm_bf16io", "bf16io_w16": "seg_conv_igemm_bf16io_w16"}[math]
    ref = torch.empty(M, Cout, device=DEV, dtype=dt)
    call(name, x.data_ptr(), Cin, N, H, W, Cin, wk.data_ptr(), ldk, None, ref.data_ptr(), Cout, H, W, Cout, ks, 1,
         ks // 2, add.data_ptr() if addend else None, Cout if addend else 0, None, S())
    tiles = query("seg_conv_igemm_row_tiles", M, Cout, None)
    part = torch.full((tiles * 2 * Cout,), float("nan"), device=DEV)
    out = torch.empty(M, Cout, device=DEV, dtype=dt)
    bname = name.replace("seg_conv_igemm", "seg_conv_igemm_bnout")
    call(bname, x.data_ptr(), Cin, N, H, W, Cin, wk.data_ptr(), ldk, out.data_ptr(), Cout, Cout, ks,
         add.data_ptr() if addend else None, Cout if addend else 0, y.data_ptr(), Cout, scale.data_ptr(),
         shift.data_ptr(), mean.data_ptr(), act, part.data_ptr(), S())
    coef, dg, db = (torch.full((n,), float("nan"), device=DEV) for n in (3 * Cout, Cout, Cout))
    call("seg_bn_bwd_finalize_tiles", part.data_ptr(), tiles, M, Cout, gamma.data_ptr(), invstd.data_ptr(),
         dg.data_ptr(), db.data_ptr(), coef.data_ptr(), S())
    work = torch.empty(query("seg_chan_workspace_floats", M, Cout), device=DEV)
    coef2, dg2, db2 = (torch.empty(n, device=DEV) for n in (3 * Cout, Cout, Cout))
    call("seg_bn_bwd_coef" + ("_bf16io" if io else ""), ref.data_ptr(), Cout, y.data_ptr(), Cout, M, Cout,
         gamma.data_ptr(), mean.data_ptr(), invstd.data_ptr(), scale.data_ptr(), shift.data_ptr(), act, dg2.data_ptr(),
         db2.data_ptr(), work.data_ptr(), coef2.data_ptr(), S())
    torch.cuda.synchronize()
    assert torch.equal(out, ref), "the conv output is the plain launch's"
    for a, b in ((coef, coef2), (dg, dg2), (db, db2)):
        assert rel(a, b) < 1e-5, rel(a, b)
    # a repeat launch is bitwise equal (no atomics)
    part2 = torch.full_like(part, float("nan"))
    call(bname, x.data_ptr(), Cin, N, H, W, Cin, wk.data_ptr(), ldk, out.data_ptr(), Cout, Cout, ks,
         add.data_ptr() if addend else None, Cout if addend else 0, y.data_ptr(), Cout, scale.data_ptr(),
         shift.data_ptr(), mean.data_ptr(), act, part2.data_ptr(), S())
    torch.cuda.synchronize()
    assert torch.equal(part, part2)


# (bf16io: one-ulp bf16 rounding flips of dY cascade through 50 layers, so a step-to-step comparison has no useful
# bound; its kernels are pinned above and the whole bf16io step against the oracle by tests/test_gpu_bf16io.py with
# the epilogue reduction on -- the default)
@pytest.mark.parametrize("arch,math,tol", [("MobileNetV2UNet", "f32", 1e-3), ("UNet", "f32", 1e-3)])
def test_bnout_step_equals_three_pass(arch, math, tol):
    from seg_amd import MobileNetV2UNet, UNet
    from seg_amd.detinit import deterministic_init, synthetic_batch
    x, y = synthetic_batch(4, 64, 128, 10, seed=5)
    x, y = x.to(DEV), y.to(DEV)
    res = {}
    saved = engine.BNOUT
    try:
        for flag in (False, True):
            engine.BNOUT = flag
            model = deterministic_init((MobileNetV2UNet if arch == "MobileNetV2UNet" else UNet)(10), seed=5).to(DEV)
            engine.set_conv_math(model, math)
            model.train()
            loss = model.forward_loss(x, y)
            loss.backward()
            torch.cuda.synchronize()
            res[flag] = (loss.item(), {k: p.grad.clone() for k, p in model.named_parameters() if p.grad is not None})
    finally:
        engine.BNOUT = saved
    assert res[True][0] == res[False][0]  # the forward is untouched
    # per tensor, relative to max(|g|, 1e-3 * the largest tensor norm): the project BNs' beta gradients are sums
    # that vanish in exact arithmetic (their dA is a column-centred BN-backward output times a 1x1 weight) and are
    # rounding noise either way
    g_max = max(float(g.double().norm()) for g in res[False][1].values())
    worst = max(float((res[True][1][k].double() - g.double()).norm()) / max(float(g.double().norm()), 1e-3 * g_max)
                for k, g in res[False][1].items())
    assert worst < tol, worst
