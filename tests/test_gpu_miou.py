"""GPU: mIoU parity (BASELINE north_star "mIoU within 1e-3 of reference").

The reference has no metric code, so the build's definition (seg_amd.detinit.miou:
confusion matrix of argmax predictions, mean IoU over classes with a non-empty union)
is applied to a LEARNABLE synthetic road scene (seg_amd.detinit.synthetic_scene).
Fixture tests/golden/mnv2_miou_scene_150steps.npz was made by tests/golden/make_golden.py
from the reference's own MobileNetV2UNet trained by its own loop (src/train.py:35-39,
Adam lr 1.5e-4) for 150 batches of 8 at 128x256, then evaluated (model.eval()) on 32
held-out scenes -- three times: fp32 on 8 CPU threads, fp32 on 1 thread, fp64.

  1. identical weights: the HIP eval forward and the oracle's eval forward of the same
     (HIP-trained) weights give the same mIoU within 1e-4 on the held-out batch;
  2. after 150 identical training steps from identical init, through the drop-in
     train_model(): the HIP mIoU lies within 1e-3 of the reference's own run-to-run
     envelope [min, max] of its three runs.  A bare |mIoU_hip - mIoU_ref32| < 1e-3 is not
     a property even the reference has: its fp64 run lands 1.8e-3 from its fp32 run
     (0.49013 vs 0.48835; the 1-thread fp32 run 0.48864) -- training amplifies
     rounding differences chaotically; after 50 steps two fp32 thread counts already
     differed by 2.4e-3.  |mIoU_hip - mIoU_ref32| is printed beside it.
"""
import json
import os

import numpy as np
import pytest
import torch
from torch import nn

from oracle import segref
from seg_amd import MobileNetV2UNet, deterministic_init, train_model
from seg_amd.detinit import miou, synthetic_scene

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _eval_preds(model, xe):
    model.eval()
    with torch.no_grad():
        p = torch.cat([model(xe[i:i + 8].to(DEV)).argmax(1).cpu() for i in range(0, len(xe), 8)])
    model.train()
    return p


def test_miou_within_reference_envelope_after_150_steps(golden_dir, record):
    z = np.load(os.path.join(golden_dir, "mnv2_miou_scene_150steps.npz"), allow_pickle=False)
    c = json.loads(str(z["meta"]))
    xe, ye = synthetic_scene(c["heldout"], c["h"], c["w"], c["classes"], seed=c["heldout_seed"])
    assert np.array_equal(ye.numpy(), z["heldout_y"]), "scene generator drifted from the fixture"
    model = deterministic_init(MobileNetV2UNet(c["classes"]), seed=c["seed"]).to(DEV).train()
    p0 = _eval_preds(model, xe)
    m0 = miou(p0, ye, c["classes"])
    assert abs(m0 - float(z["miou_init32"])) < 1e-3, (m0, float(z["miou_init32"]))
    loader = [synthetic_scene(c["bs"], c["h"], c["w"], c["classes"], seed=c["batch_seed0"] + s)
              for s in range(c["steps"])]
    opt = torch.optim.Adam(model.parameters(), lr=c["lr"])
    train_model(model, loader, nn.CrossEntropyLoss(), opt, DEV, epochs=1, checkpoint_pattern=None, progress=False)
    p1 = _eval_preds(model, xe)
    m1 = miou(p1, ye, c["classes"])
    refs = [float(z["miou32"]), float(z["miou32t1"]), float(z["miou64"])]
    agree = float((p1.numpy() == z["pred32"]).mean())
    print(f"mIoU after {c['steps']} steps: HIP {m1:.5f}; reference fp32 {refs[0]:.5f}, fp32 1-thread {refs[1]:.5f}, "
          f"fp64 {refs[2]:.5f}; |HIP - ref fp32| = {abs(m1 - refs[0]):.2e}; pixel agreement with the reference "
          f"fp32 {agree:.4f}")
    record(steps=c["steps"], miou_hip=m1, miou_ref=refs, abs_diff_ref_fp32=abs(m1 - refs[0]), pixel_agreement=agree)
    assert m1 > 5 * m0, "the scene must be learnable (mIoU well above chance after training)"
    assert min(refs) - 1e-3 <= m1 <= max(refs) + 1e-3, (m1, refs)
    # identical weights: the oracle's eval forward of the trained HIP weights
    p = segref.canonical_state(model.state_dict())
    with torch.no_grad():
        po = torch.cat([segref.mobilenet_unet_forward(p, xe[i:i + 8], False).argmax(1) for i in range(0, len(xe), 8)])
    mo = miou(po, ye, c["classes"])
    print(f"identical weights: HIP {m1:.6f} vs oracle {mo:.6f}, {(po != p1).sum().item()} pixels differ")
    assert abs(m1 - mo) < 1e-4
