"""GPU: the exact-zero gradient of conv biases in front of train-mode BatchNorm
(engine.ZERO_BN_BIAS, SEG_ZERO_BN_BIAS; INTEGRATION.md "Behavioural differences").

double_conv's convs carry a bias (src/unet.py:58,61) that the next BatchNorm's batch mean
removes again, so d loss / d bias = sum_p dY[p][c] = 0 exactly.  The reference computes that
sum in fp32 and gets rounding noise (~1e-9), which Adam (eps 1e-8) turns into steps of up to
lr, so its biases drift; its fp64 twin's noise is ~1e-17 and they stay put.  The build
writes zeros (default) or, with the switch off, reduces dY like the reference.

After 20 Adam(lr=1.5e-4) steps of MobileNetV2UNet at 2x64x128 (the reference's own
optimizer settings, main.py:100):
  * zeros on: the biases are bit-for-bit their initial values; eval logits within twice the
    reference's own fp32-vs-fp64 spread of the fp64 oracle run (and 1e-3), mIoU within 1e-3
    of the reference's fp32 / fp64 envelope -- the outputs are unaffected;
  * zeros off: the biases drift like the reference fp32 run's (same order of magnitude);
    the fp64 oracle's barely move.
"""
import numpy as np
import pytest
import torch

from oracle import segref
from seg_amd import MobileNetV2UNet, engine
from seg_amd.detinit import deterministic_init, synthetic_batch

pytestmark = pytest.mark.gpu
DEV = "cuda"
STEPS, LR, SEED = 20, 1.5e-4, 17


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / b.norm())


def _bias_names(sd):
    # the decoder's conv biases (double_conv's Conv2d at .0 and .3; .1 / .4 are its BatchNorms)
    return [k for k in sd if k.startswith("up") and k.endswith((".conv.conv.0.bias", ".conv.conv.3.bias"))]


def _batches():
    return [synthetic_batch(2, 64, 128, 10, seed=SEED + 100 + s) for s in range(STEPS)]


def _hip_run(zero):
    saved = engine.ZERO_BN_BIAS
    engine.ZERO_BN_BIAS = zero
    try:
        model = deterministic_init(MobileNetV2UNet(10), seed=SEED).to(DEV).train()
        opt = torch.optim.Adam(model.parameters(), lr=LR)
        for x, y in _batches():
            opt.zero_grad()
            model.forward_loss(x.to(DEV), y.to(DEV)).backward()
            opt.step()
        torch.cuda.synchronize()
    finally:
        engine.ZERO_BN_BIAS = saved
    return model


@pytest.fixture(scope="module")
def oracle_runs():
    init = deterministic_init(MobileNetV2UNet(10), seed=SEED).state_dict()
    out = {}
    for dt in (torch.float32, torch.float64):
        p = segref.canonical_state(init, dt)
        segref.adam_steps("MobileNetV2UNet", p, [(x.to(dt), y) for x, y in _batches()], lr=LR)
        out[dt] = p
    return segref.canonical_state(init), out


def _eval(model_or_p, x):
    with torch.no_grad():
        if isinstance(model_or_p, dict):
            return segref.FORWARDS["MobileNetV2UNet"](model_or_p, x.to(next(iter(model_or_p.values())).dtype), False)
        return model_or_p.eval()(x.to(DEV)).cpu()


def test_zero_bn_bias_outputs_track_the_reference(oracle_runs, record):
    init, ref = oracle_runs
    model = _hip_run(True)
    sd = model.state_dict()
    names = _bias_names(sd)
    assert len(names) == 8
    for k in names:  # never written by Adam: the gradient is exactly zero every step
        assert torch.equal(sd[k].cpu(), init[k]), k
    x, y = synthetic_batch(4, 64, 128, 10, seed=SEED + 999)
    hip = _eval(model, x)
    r32, r64 = _eval(ref[torch.float32], x), _eval(ref[torch.float64], x)
    spread, err = _rel(r32, r64), _rel(hip, r64)
    m_hip, m32, m64 = (segref.miou(t.argmax(1), y, 10) for t in (hip, r32, r64))
    drift32 = max(float((ref[torch.float32][k] - init[k]).abs().max()) for k in names)
    drift64 = max(float((ref[torch.float64][k] - init[k].double()).abs().max()) for k in names)
    print(f"{STEPS} Adam steps: eval logits vs fp64 oracle {err:.2e} (reference fp32 vs fp64 {spread:.2e}); "
          f"mIoU hip {m_hip:.5f} ref fp32 {m32:.5f} fp64 {m64:.5f}; pre-BN bias drift ref fp32 {drift32:.2e}, "
          f"fp64 {drift64:.2e}, hip 0")
    record(steps=STEPS, logits_rel_fp64=err, ref_spread=spread, miou_hip=m_hip, miou_ref32=m32, miou_ref64=m64,
           bias_drift_ref32=drift32, bias_drift_ref64=drift64)
    assert err <= max(1e-3, 2 * spread), (err, spread)
    assert min(m32, m64) - 1e-3 <= m_hip <= max(m32, m64) + 1e-3, (m_hip, m32, m64)
    # the reference's fp32 biases drift by Adam-normalised noise (up to ~lr per step); fp64's do not
    assert drift32 > 10 * drift64


def test_zero_bn_bias_off_reproduces_the_drift(oracle_runs):
    init, ref = oracle_runs
    model = _hip_run(False)
    sd = model.state_dict()
    names = _bias_names(sd)
    drift_hip = max(float((sd[k].cpu() - init[k]).abs().max()) for k in names)
    drift32 = max(float((ref[torch.float32][k] - init[k]).abs().max()) for k in names)
    print(f"SEG_ZERO_BN_BIAS=0: pre-BN bias drift hip {drift_hip:.2e}, reference fp32 {drift32:.2e}")
    # noise-driven, so only the scale is comparable: both within Adam's bound of lr per step
    assert 0 < drift_hip <= STEPS * LR * 1.01
    assert 0.05 * drift32 <= drift_hip <= 20 * drift32, (drift_hip, drift32)
    assert np.isfinite(drift_hip)
