"""GPU: seg_mbconv_f16 -- one torchvision InvertedResidual of the BatchNorm-folded fp16 inference
forward in one launch (csrc/mbconv.hip; BASELINE configs[3], inference.py:162-163 through
src/unet.py:15-19).

  * against float64 of the same arithmetic (fp16-rounded 1x1 operands, fp32/fp64 depthwise):
    expand ratio 6 and 1, stride 1 (with the residual) and 2, split hidden ranges (the
    last-arrival combine) and one split, ragged tiles, every MobileNetV2 block shape at a
    128x256 frame;
  * repeat launches bitwise equal (fixed-order combine; the tiles' epoch words advance, nothing left over);
  * seg_pw2_f16 (the outconv head) against float64 of the same operand rounding;
  * seg_stem_pre_f16 (preprocess formed on load by the stem conv) against seg_preprocess_bgr + seg_conv_igemm_f16;
  * the fp16 Predictor with the fused blocks and head agrees with the one-launch-per-conv folded forward
    (SEG_MBCONV off) within fp16 operand-rounding noise, and its graph replay equals eager.
"""
import ctypes

import pytest
import torch
import torch.nn.functional as F

from seg_amd import MobileNetV2UNet, deterministic_init, engine
from seg_amd._lib import call, query

pytestmark = pytest.mark.gpu
DEV = "cuda"


def S():
    return torch.cuda.current_stream().cuda_stream


def h16(t):
    return t.to(torch.float16).double()


def reference(x, we, be, wd, bd, wp, bp, stride, res):
    """float64 NCHW of the block with the kernel's rounding points."""
    xx = x.double()
    if we is not None:
        h = F.conv2d(h16(xx), h16(we)[:, :, None, None]) + be.double()[None, :, None, None]
        h = h.clamp(0, 6).float().double()  # fp32 staging
    else:
        h = xx
    C = h.shape[1]
    d = F.conv2d(h, wd.double().view(C, 1, 3, 3), stride=stride, padding=1, groups=C) + bd.double()[None, :, None, None]
    d = d.clamp(0, 6)
    o = F.conv2d(h16(d), h16(wp)[:, :, None, None]) + bp.double()[None, :, None, None]
    if res is not None:
        o = o + res.double()
    return o


CASES = [  # N, H, W, Cin, t, Cout, stride, residual  (MobileNetV2 blocks at a 128x256 frame, plus ragged ones)
    (1, 64, 128, 32, 1, 16, 1, False), (1, 64, 128, 16, 6, 24, 2, False), (1, 32, 64, 24, 6, 24, 1, True),
    (1, 32, 64, 24, 6, 32, 2, False), (1, 16, 32, 32, 6, 32, 1, True), (1, 16, 32, 32, 6, 64, 2, False),
    (1, 8, 16, 64, 6, 64, 1, True), (1, 8, 16, 64, 6, 96, 1, False), (1, 8, 16, 96, 6, 96, 1, True),
    (1, 8, 16, 96, 6, 160, 2, False), (1, 4, 8, 160, 6, 160, 1, True), (1, 4, 8, 160, 6, 320, 1, False),
    (2, 13, 21, 24, 6, 24, 1, True), (1, 11, 19, 16, 6, 32, 2, False), (1, 9, 10, 40, 1, 24, 2, False),
]


@pytest.mark.parametrize("N,H,W,Cin,t,Cout,stride,res", CASES)
def test_mbconv_vs_fp64(N, H, W, Cin, t, Cout, stride, res):
    Ch = Cin * t
    assert query("seg_mbconv_ok", Cin, Ch, Cout, stride, int(t != 1)) == 1
    g = torch.Generator().manual_seed(N * H * W + Cin + Cout)
    x = torch.randn(N, Cin, H, W, generator=g)
    we = torch.randn(Ch, Cin, generator=g) / Cin ** 0.5 if t != 1 else None
    be = torch.randn(Ch, generator=g) * 0.1 + 0.5 if t != 1 else None
    wd = torch.randn(Ch, 9, generator=g) / 3
    bd = torch.randn(Ch, generator=g) * 0.1 + 0.2
    wp = torch.randn(Cout, Ch, generator=g) / Ch ** 0.5
    bp = torch.randn(Cout, generator=g) * 0.1
    Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
    r = torch.randn(N, Cout, Ho, Wo, generator=g) if res else None
    ref = reference(x, we, be, wd, bd, wp, bp, stride, r)
    rows = lambda t4: t4.permute(0, 2, 3, 1).reshape(-1, t4.shape[1]).contiguous().to(DEV)  # noqa: E731
    xg, rg = rows(x), rows(r) if res else None
    wdk = torch.empty(9 * Ch, device=DEV)
    call("seg_pack_dw_weight", wd.contiguous().to(DEV).data_ptr(), wdk.data_ptr(), Ch, S())
    weg, beg = (we.to(DEV), be.to(DEV)) if t != 1 else (None, None)
    wpg, bpg, bdg = wp.to(DEV), bp.to(DEV), bd.to(DEV)
    ncnt = ctypes.c_int(0)
    nw = query("seg_mbconv_work_floats", N, H, W, Ch, Cout, stride, ctypes.addressof(ncnt))
    work = torch.full((max(nw, 1),), float("nan"), device=DEV)
    cnt = torch.zeros(max(ncnt.value, 1), device=DEV, dtype=torch.int32)
    outs = []
    for _ in range(2):
        o = torch.full((N * Ho * Wo, Cout), float("nan"), device=DEV)
        call("seg_mbconv_f16", xg.data_ptr(), Cin, N, H, W, Cin, weg.data_ptr() if weg is not None else None,
             beg.data_ptr() if beg is not None else None, Ch, wdk.data_ptr(), bdg.data_ptr(), stride, wpg.data_ptr(),
             bpg.data_ptr(), Cout, rg.data_ptr() if res else None, Cout if res else 0, o.data_ptr(), Cout,
             work.data_ptr(), cnt.data_ptr(), S())
        outs.append(o)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1]), "deterministic"
    if cnt.numel() % 4:
        assert int(cnt.abs().sum()) == 0
    else:  # seg_tile_combine's epoch words: count and hand-off mask clear, epoch advanced per launch (or unused)
        wv = cnt.view(-1, 4)
        assert int(wv[:, 0].abs().sum()) == 0 and int(wv[:, 2:].abs().sum()) == 0
        assert bool(((wv[:, 1] == 0) | (wv[:, 1] == 2 << 6)).all())
    got = outs[0].double().cpu().view(N, Ho, Wo, Cout).permute(0, 3, 1, 2)
    rel = float((got - ref).norm() / ref.norm())
    assert rel < 1e-3, rel


def test_mbconv_refuses():
    assert query("seg_mbconv_ok", 320, 1920, 1280, 1, 1) == 0   # Cin > 160 with an expand
    assert query("seg_mbconv_ok", 32, 192, 640, 1, 1) == 0     # Cout > 320
    assert query("seg_mbconv_ok", 32, 192, 64, 3, 1) == 0      # stride 3
    assert query("seg_mbconv_ok", 32, 64, 16, 1, 0) == 0       # no expand: Ch == Cin


def test_predictor_fused_equals_unfused():
    from seg_amd.infer import Predictor
    import numpy as np
    model = deterministic_init(MobileNetV2UNet(10), seed=13, random_running_stats=True).to(DEV).eval()
    f = (np.random.default_rng(0).random((720, 1280, 3)) * 255).astype(np.uint8)
    saved = engine.MBCONV, engine.PW2, engine.STEM_PRE
    try:
        engine.MBCONV = engine.PW2 = engine.STEM_PRE = False
        p0 = Predictor(model, frame_hw=(720, 1280), graph=False, math="f16")
        p0(f)
        l0 = p0.logits()
        engine.MBCONV = engine.PW2 = engine.STEM_PRE = True
        p1 = Predictor(model, frame_hw=(720, 1280), graph=True, math="f16")
        assert p1.stem_pre is p1.prog.ops[0]  # preprocess + stem in one launch (seg_stem_pre_f16)
        assert len(p1.prog.mbconv_groups()) == 17  # every InvertedResidual of features[1..17]
        assert p1.prog.pw2_head() == len(p1.prog.ops) - 2  # outconv in one launch (seg_pw2_f16)
        m1 = p1(f).clone()
        l1 = p1.logits()
        p2 = Predictor(model, frame_hw=(720, 1280), graph=False, math="f16")
        m2 = p2(f).clone()
        assert torch.equal(m1, m2) and torch.equal(l1, p2.logits()), "graph replay == eager"
    finally:
        engine.MBCONV, engine.PW2, engine.STEM_PRE = saved
    # two valid fp16 forwards: the fp32 accumulation orders differ (split hidden ranges vs split-K), and an fp32
    # value one ulp either side of an fp16 rounding boundary moves that operand by an fp16 ulp (~5e-4); the oracle
    # bound of both is tests/test_gpu_infer.py::test_predictor_low_precision
    rel = float((l1 - l0).norm() / l0.norm())
    assert rel < 1e-2, rel
    agree = float((l1.argmax(1) == l0.argmax(1)).float().mean())
    # (0.99493 at round 6's fixed-fma upsample blend on this random-init model, whose logit margins are tiny: the
    # disagreement is the near-tie pixels, the fp16 rounding flips described above)
    assert agree >= 0.994, agree


@pytest.mark.parametrize("M,C2,act", [(8192, 10, 1), (1000, 3, 2), (255, 64, 1)])
def test_pw2_head_vs_fp64(M, C2, act):
    g = torch.Generator().manual_seed(M + C2)
    x = torch.randn(M, 32, generator=g)
    w1, b1 = torch.randn(16, 32, generator=g) / 32 ** 0.5, torch.randn(16, generator=g) * 0.1
    w2, b2 = torch.randn(C2, 16, generator=g) / 4, torch.randn(C2, generator=g) * 0.1
    h = (h16(x) @ h16(w1).T + b1.double())
    h = h.clamp(min=0) if act == 1 else h.clamp(0, 6)
    ref = h.float().to(torch.float16).double() @ h16(w2).T + b2.double()
    out = torch.full((M, C2 + 2), float("nan"), device=DEV)
    xg, w1g, b1g, w2g, b2g = (t.to(DEV) for t in (x, w1, b1, w2, b2))  # (kept alive across the launch)
    call("seg_pw2_f16", xg.data_ptr(), 32, M, 32, w1g.data_ptr(), b1g.data_ptr(), 16, act, w2g.data_ptr(),
         b2g.data_ptr(), C2, out.data_ptr(), C2 + 2, S())
    torch.cuda.synchronize()
    got = out[:, :C2].double().cpu()
    assert float((got - ref).norm() / ref.norm()) < 1e-4  # fp32 vs fp64 sums may move an fp16 rounding
    assert bool(out[:, C2:].isnan().all()), "nothing written beyond C2"


@pytest.mark.parametrize("fhw,hw", [((720, 1280), (128, 256)), ((90, 161), (64, 32))])
def test_stem_pre_equals_preprocess_then_conv(fhw, hw):
    import numpy as np
    from seg_amd.infer import MEAN, STD
    (Hf, Wf), (H, W) = fhw, hw
    frame = torch.from_numpy((np.random.default_rng(Hf).random((Hf, Wf, 3)) * 255).astype(np.uint8)).to(DEV)
    g = torch.Generator().manual_seed(Wf)
    wk = (torch.randn(32, 36, generator=g) * 0.3).to(DEV)
    wk.view(32, 9, 4)[:, :, 3] = 0.0  # the padded channel
    b = torch.randn(32, generator=g).to(DEV)
    img = torch.zeros(H * W, 4, device=DEV)
    call("seg_preprocess_bgr", frame.data_ptr(), 1, Hf, Wf, frame.stride(0), img.data_ptr(), 4, H, W, *MEAN, *STD, S())
    Ho, Wo = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    ref = torch.empty(Ho * Wo, 32, device=DEV)
    call("seg_conv_igemm_f16", img.data_ptr(), 4, 1, H, W, 4, wk.data_ptr(), 36, b.data_ptr(), ref.data_ptr(), 32, Ho,
         Wo, 32, 3, 2, 1, None, 0, None, 2, None, 1, S())
    out = torch.full((Ho * Wo, 36), float("nan"), device=DEV)
    call("seg_stem_pre_f16", frame.data_ptr(), Hf, Wf, frame.stride(0), H, W, *MEAN, *STD, wk.data_ptr(), 36,
         b.data_ptr(), 2, 32, out.data_ptr(), 36, S())
    torch.cuda.synchronize()
    assert float((out[:, :32] - ref).norm() / ref.norm()) < 1e-5
    assert bool(out[:, 32:].isnan().all())


@pytest.mark.parametrize("spin", [0, 1])
def test_predictor_combine_hand_off_bitwise(spin):
    """The in-launch split combines (seg_mbconv_f16, seg_conv_igemm_f16_ic) with the poll bound forced to 0 / 1
    (seg_set_combine_spin): every block but a tile's last hands its share over through the epoch word's mask --
    the path a block takes when a peer cannot become resident -- and the frame is bitwise the
    default's."""
    from seg_amd.infer import Predictor
    import numpy as np
    model = deterministic_init(MobileNetV2UNet(10), seed=13, random_running_stats=True).to(DEV).eval()
    f = (np.random.default_rng(1).random((720, 1280, 3)) * 255).astype(np.uint8)
    p = Predictor(model, frame_hw=(720, 1280), graph=False, math="f16")
    m0 = p(f).clone()
    l0 = p.logits().clone()
    try:
        call("seg_set_combine_spin", spin)
        for _ in range(2):  # the epoch words carry over between launches
            m1 = p(f).clone()
            assert torch.equal(m1, m0) and torch.equal(p.logits(), l0)
    finally:
        call("seg_set_combine_spin", -1)
    assert torch.equal(p(f), m0)

