"""CPU: the oracle (oracle/segref.py) reproduces the reference's golden fixtures,
and the product's module surface matches the reference's state_dict layout."""
import json
import os

import numpy as np
import pytest
import torch

from oracle import segref
from seg_amd import LightUNet, MobileNetV2UNet, UNet
from seg_amd.detinit import deterministic_init, synthetic_batch

CTORS = {"MobileNetV2UNet": lambda c: MobileNetV2UNet(c), "UNet": lambda c: UNet(c, 64),
         "LightUNet": lambda c: LightUNet()}


def load(golden_dir, name):
    z = np.load(os.path.join(golden_dir, name + ".npz"), allow_pickle=False)
    return z, json.loads(str(z["meta"]))


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)


def oracle_params(meta, dtype=torch.float32):
    model = CTORS[meta["arch"]](meta["classes"])
    deterministic_init(model, seed=meta["seed"], random_running_stats=meta.get("random_running_stats", False))
    return segref.canonical_state(model.state_dict(), dtype)


@pytest.mark.parametrize("case", ["mnv2_train_2x64x128", "unet4_train_2x32x64"])
def test_oracle_train_matches_reference(golden_dir, case):
    z, meta = load(golden_dir, case)
    p = oracle_params(meta)
    x, y = synthetic_batch(meta["n"], meta["h"], meta["w"], meta["classes"], seed=meta["seed"] + 100)
    np.testing.assert_array_equal(x.numpy(), z["x"])
    np.testing.assert_array_equal(y.numpy(), z["y"])
    loss, logits, grads = segref.forward_backward(meta["arch"], p, x, y, True)
    assert rel(logits.numpy(), z["logits"]) < 1e-5
    assert abs(float(loss) - float(z["loss32"])) < 1e-5 * abs(float(z["loss32"]))
    n_checked = 0
    for k, g in grads.items():
        ref_norm = float(z[f"g32_norm/{k}"])
        # same aten ops in the same order: agreement far tighter than the reference's own fp32 error
        tol = max(1e-4 * ref_norm, 10 * float(z[f"gdiff/{k}"]), 1e-9)
        assert abs(float(g.double().norm()) - ref_norm) <= tol, k
        if f"g32_full/{k}" in z:
            d = np.linalg.norm(g.numpy().astype(np.float64) - z[f"g32_full/{k}"])
            assert d <= tol, (k, d, tol)
        n_checked += 1
    assert n_checked == len([k for k in z.files if k.startswith("g32_norm/")])
    for k in z.files:  # BN running statistics after the step
        if k.startswith("buf/"):
            name = k[4:]
            if name.endswith("num_batches_tracked"):
                assert int(p[name]) == int(z[k])
            else:
                assert rel(p[name].numpy(), z[k]) < 1e-5, name


@pytest.mark.parametrize("case", ["mnv2_eval_1x64x128", "lightunet_eval_1x32x32"])
def test_oracle_eval_matches_reference(golden_dir, case):
    z, meta = load(golden_dir, case)
    p = oracle_params(meta)
    x, _ = synthetic_batch(meta["n"], meta["h"], meta["w"], meta["classes"], seed=meta["seed"] + 100)
    with torch.no_grad():
        logits = segref.FORWARDS[meta["arch"]](p, x, False)
    assert rel(logits.numpy(), z["logits"]) < 1e-5


def test_oracle_adam_matches_reference(golden_dir):
    z, meta = load(golden_dir, "mnv2_adam3_2x64x64")
    p = oracle_params(meta)
    batches = [synthetic_batch(meta["n"], meta["h"], meta["w"], meta["classes"], seed=meta["seed"] + 1000 + s)
               for s in range(meta["steps"])]
    losses = segref.adam_steps(meta["arch"], p, batches, lr=meta["lr"])
    np.testing.assert_allclose(losses, z["losses"], rtol=1e-5)
    x, _ = synthetic_batch(meta["n"], meta["h"], meta["w"], meta["classes"], seed=meta["seed"] + 2000)
    with torch.no_grad():
        logits = segref.FORWARDS[meta["arch"]](p, x, False)
    # Adam normalises near-zero (noise) gradients, e.g. of the pre-BN conv biases, to
    # +-lr steps, so fp32 rounding differences grow to ~1e-4 after 3 steps: 1e-3 bar.
    assert rel(logits.numpy(), z["eval_logits"]) < 1e-3
    for k in z.files:
        if k.startswith("param_norm/") and not k.startswith("param_norm/backbone.classifier"):
            name = k[len("param_norm/"):]
            assert abs(float(p[name].double().norm()) - float(z[k])) <= 1e-4 * float(z[k]) + 1e-6, name


def test_state_dict_layout_matches_reference(golden_dir):
    with open(os.path.join(golden_dir, "state_dict_keys.json")) as f:
        ref = json.load(f)
    for arch, ctor in (("MobileNetV2UNet", lambda: MobileNetV2UNet(10)), ("UNet", lambda: UNet(10)),
                       ("LightUNet", lambda: LightUNet())):
        mine = [[k, list(v.shape)] for k, v in ctor().state_dict().items()]
        assert mine == ref[arch], arch
    assert len(ref["MobileNetV2UNet"]) == 691  # 691 keys incl. aliases


def test_torchvision_standin_param_count(golden_dir):
    with open(os.path.join(golden_dir, "state_dict_keys.json")) as f:
        ref = json.load(f)
    assert ref["_mobilenet_v2_param_count"] == 3_504_872  # torchvision's documented MobileNetV2 size
    from seg_amd.mobilenet import MobileNetV2
    assert sum(p.numel() for p in MobileNetV2().parameters()) == 3_504_872


def test_param_counts():
    m = MobileNetV2UNet(10)
    assert sum(p.numel() for p in m.parameters()) == 7_830_786
    assert sum(p.numel() for p in UNet(10).parameters()) == 3_364_586
    assert sum(p.numel() for p in LightUNet().parameters()) == 842_977


def test_miou_definition():
    pred = torch.tensor([0, 1, 1, 2, 2, 2])
    tgt = torch.tensor([0, 1, 2, 2, 2, 1])
    # class0 IoU 1; class1 tp1 fp1 fn1 -> 1/3; class2 tp2 fp1 fn1 -> 1/2
    assert abs(segref.miou(pred, tgt, 3) - (1 + 1 / 3 + 1 / 2) / 3) < 1e-12


def test_oracle_miou_scene_fixture(golden_dir):
    """The learnable scene is regenerated bit-exactly from its seed, and the oracle's Adam
    trajectory reproduces the reference's first training losses (fixture made from
    src/unet.py; the full 150-step mIoU is the GPU test's job)."""
    import json
    from seg_amd.detinit import miou, synthetic_scene
    z = np.load(os.path.join(golden_dir, "mnv2_miou_scene_150steps.npz"), allow_pickle=False)
    c = json.loads(str(z["meta"]))
    xe, ye = synthetic_scene(c["heldout"], c["h"], c["w"], c["classes"], seed=c["heldout_seed"])
    assert np.array_equal(ye.numpy(), z["heldout_y"])
    m = deterministic_init(MobileNetV2UNet(c["classes"]), seed=c["seed"])
    p = segref.canonical_state(m.state_dict())
    with torch.no_grad():
        pred = torch.cat([segref.mobilenet_unet_forward(p, xe[i:i + 8], False).argmax(1) for i in range(0, 32, 8)])
    assert abs(miou(pred, ye, c["classes"]) - float(z["miou_init32"])) < 1e-4
    batches = [synthetic_scene(c["bs"], c["h"], c["w"], c["classes"], seed=c["batch_seed0"] + s) for s in range(5)]
    losses = segref.adam_steps("MobileNetV2UNet", p, batches, lr=c["lr"])
    np.testing.assert_allclose(losses, z["losses32"][:5], rtol=1e-4)
