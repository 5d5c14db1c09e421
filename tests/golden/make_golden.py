"""Generate the golden fixtures in tests/golden/ from the REFERENCE implementation.

Run in the build container (needs /root/reference; never on the GPU box):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

The reference's own src/unet.py (MobileNetV2UNet, UNet, LightUNet) is imported
by file path with a local torchvision stand-in (tests/golden/tv_stub.py; the
real torchvision is not installed and ImageNet weights are never fetched).
Every weight comes from seg_amd.detinit.deterministic_init, every input from
seg_amd.detinit.synthetic_batch, so the oracle and the HIP path can
regenerate identical tensors from names and seeds alone.  The loss is the
reference's criterion nn.CrossEntropyLoss() (main.py:99) and the optimizer step
is optim.Adam(lr=1.5e-4) (main.py:100) driven like src/train.py:35-39.

Outputs: <case>.npz (inputs, logits, loss, per-parameter gradient statistics in
fp32 and fp64, BN running statistics; the mIoU case: held-out predictions and mIoU
before / after 150 training steps) and state_dict_keys.json.
    python tests/golden/make_golden.py [case ...]   # only the named cases
"""
from __future__ import annotations

import importlib.util
import json
import os
import sys

import numpy as np
import torch

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("SEG_REFERENCE", "/root/reference")
sys.path.insert(0, os.path.join(REPO, "team02-objectdetection_amd"))
sys.path.insert(0, HERE)

from seg_amd.detinit import deterministic_init, miou, synthetic_batch, synthetic_scene  # noqa: E402
import tv_stub  # noqa: E402

SMALL = 4096  # store full gradients of tensors up to this many elements


def load_reference_unet():
    tv_stub.install()
    spec = importlib.util.spec_from_file_location("reference_unet", os.path.join(REF, "src", "unet.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def grad_stats(model, prefix="g"):
    out = {}
    names = []
    seen = set()
    for name, p in model.named_parameters():
        if id(p) in seen or p.grad is None:
            continue
        seen.add(id(p))
        names.append(name)
        g = p.grad.detach().double()
        out[f"{prefix}_norm/{name}"] = np.array(g.norm().item())
        out[f"{prefix}_sum/{name}"] = np.array(g.sum().item())
        if g.numel() <= SMALL:
            out[f"{prefix}_full/{name}"] = g.float().numpy()
        else:
            out[f"{prefix}_head/{name}"] = g.flatten()[:64].float().numpy()
    return out, names


def run_case(ref, arch, ctor, n, h, w, classes, seed, training=True, backward=True, random_stats=False):
    torch.manual_seed(0)
    res = {}
    for dtype in (torch.float32, torch.float64):
        model = ctor()
        deterministic_init(model, seed=seed, random_running_stats=random_stats)
        model = model.to(dtype)
        model.train(training)
        x, y = synthetic_batch(n, h, w, classes, seed=seed + 100)
        x = x.to(dtype)
        model.zero_grad(set_to_none=True)
        with torch.set_grad_enabled(backward):
            logits = model(x)
            loss = torch.nn.CrossEntropyLoss()(logits, y)
            if backward:
                loss.backward()
        tag = "32" if dtype == torch.float32 else "64"
        res[f"loss{tag}"] = np.array(loss.item())
        if dtype == torch.float32:
            res["x"] = x.numpy()
            res["y"] = y.numpy()
            res["logits"] = logits.detach().numpy().astype(np.float32)
            seen = set()
            for bname, b in model.named_buffers():
                if id(b) in seen:
                    continue
                seen.add(id(b))
                if bname.endswith(("running_mean", "running_var")):
                    res[f"buf/{bname}"] = b.detach().numpy().astype(np.float32)
                elif bname.endswith("num_batches_tracked"):
                    res[f"buf/{bname}"] = b.detach().numpy()
        else:
            res["logits64_head"] = logits.detach().flatten()[:4096].numpy()
        if backward:
            st, names = grad_stats(model, "g" + tag)
            res.update(st)
            if dtype == torch.float32:
                g32 = {k: p.grad.detach().double().clone() for k, p in model.named_parameters() if p.grad is not None}
            else:
                for k, p in model.named_parameters():
                    if k in g32:
                        res[f"gdiff/{k}"] = np.array((g32[k] - p.grad.detach()).norm().item())
    res["meta"] = np.array(json.dumps({"arch": arch, "n": n, "h": h, "w": w, "classes": classes, "seed": seed,
                                       "training": training, "backward": backward,
                                       "random_running_stats": random_stats}))
    return res


def run_adam(ref, n, h, w, classes, seed, steps=3):
    model = ref.MobileNetV2UNet(output_channels=classes)
    deterministic_init(model, seed=seed)
    model.train()
    crit = torch.nn.CrossEntropyLoss()
    opt = torch.optim.Adam(model.parameters(), lr=1.5e-4)
    losses = []
    for s in range(steps):
        x, y = synthetic_batch(n, h, w, classes, seed=seed + 1000 + s)
        opt.zero_grad()
        loss = crit(model(x), y)
        loss.backward()
        opt.step()
        losses.append(loss.item())
    x, y = synthetic_batch(n, h, w, classes, seed=seed + 2000)
    with torch.no_grad():
        model.eval()
        logits = model(x)
    out = {"losses": np.array(losses), "eval_logits": logits.numpy().astype(np.float32),
           "eval_x": x.numpy(), "eval_y": y.numpy(),
           "meta": np.array(json.dumps({"arch": "MobileNetV2UNet", "n": n, "h": h, "w": w, "classes": classes,
                                        "seed": seed, "steps": steps, "lr": 1.5e-4}))}
    seen = set()
    for name, p in model.named_parameters():
        if id(p) in seen:
            continue
        seen.add(id(p))
        out[f"param_norm/{name}"] = np.array(p.detach().double().norm().item())
    return out


MIOU = {"seed": 3, "classes": 10, "h": 128, "w": 256, "bs": 8, "steps": 150, "lr": 1.5e-4, "heldout": 32,
        "heldout_seed": 999, "batch_seed0": 100}


def run_miou(ref):
    """SURVEY 8(d)'s mIoU parity case: the reference MobileNetV2UNet(10) trained by its own loop
    (src/train.py:35-39: zero_grad, CrossEntropyLoss, backward, Adam(lr=1.5e-4) step) for
    `steps` batches of the learnable synthetic scene (seg_amd.detinit.synthetic_scene), then
    evaluated (model.eval(), inference.py:25) on a held-out scene batch: argmax predictions
    and mIoU before and after training: fp32 on 8 threads (the reference as main.py runs it
    on this CPU), fp32 on 1 thread (another valid fp32 summation order) and fp64 -- the
    spread among the three is the reference's own run-to-run mIoU spread.  Measured:
    after 50 steps two fp32 thread counts differ by 2.4e-3 mIoU (97.8 % pixel agreement,
    the model is still uncertain), after 150 steps by <= 6.4e-4 (99.5 %), so 150 steps."""
    c = MIOU
    xe, ye = synthetic_scene(c["heldout"], c["h"], c["w"], c["classes"], seed=c["heldout_seed"])
    out = {"meta": np.array(json.dumps(c)), "heldout_y": ye.numpy().astype(np.uint8)}
    threads = torch.get_num_threads()
    for dtype, tag, nthr in ((torch.float32, "32", threads), (torch.float32, "32t1", 1), (torch.float64, "64", threads)):
        torch.set_num_threads(nthr)
        model = ref.MobileNetV2UNet(output_channels=c["classes"])
        deterministic_init(model, seed=c["seed"])
        model = model.to(dtype)
        crit = torch.nn.CrossEntropyLoss()
        opt = torch.optim.Adam(model.parameters(), lr=c["lr"])

        def evaluate():
            model.eval()
            with torch.no_grad():
                pred = torch.cat([model(xe[i:i + 8].to(dtype)).argmax(1) for i in range(0, len(xe), 8)])
            model.train()
            return pred

        p0 = evaluate()
        losses = []
        for s in range(c["steps"]):
            x, y = synthetic_scene(c["bs"], c["h"], c["w"], c["classes"], seed=c["batch_seed0"] + s)
            opt.zero_grad()
            loss = crit(model(x.to(dtype)), y)
            loss.backward()
            opt.step()
            losses.append(loss.item())
        p1 = evaluate()
        out[f"losses{tag}"] = np.array(losses)
        out[f"miou_init{tag}"] = np.array(miou(p0, ye, c["classes"]))
        out[f"miou{tag}"] = np.array(miou(p1, ye, c["classes"]))
        if tag == "32":
            out["pred_init32"] = p0.numpy().astype(np.uint8)
            out["pred32"] = p1.numpy().astype(np.uint8)
        print(f"  miou fp{tag}: init {float(out[f'miou_init{tag}']):.5f} after {c['steps']} steps "
              f"{float(out[f'miou{tag}']):.5f}, loss {losses[0]:.4f} -> {losses[-1]:.4f}")
    return out


def main():
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    ref = load_reference_unet()
    only = set(sys.argv[1:])
    cases = {
        "mnv2_train_2x64x128": lambda: run_case(ref, "MobileNetV2UNet", lambda: ref.MobileNetV2UNet(10),
                                                2, 64, 128, 10, seed=1),
        "mnv2_eval_1x64x128": lambda: run_case(ref, "MobileNetV2UNet", lambda: ref.MobileNetV2UNet(10),
                                               1, 64, 128, 10, seed=2, training=False, backward=False,
                                               random_stats=True),
        "unet4_train_2x32x64": lambda: run_case(ref, "UNet", lambda: ref.UNet(4, 64), 2, 32, 64, 4, seed=3),
        "lightunet_eval_1x32x32": lambda: run_case(ref, "LightUNet", lambda: ref.LightUNet(), 1, 32, 32, 1,
                                                   seed=4, training=False, backward=False, random_stats=True),
        "mnv2_adam3_2x64x64": lambda: run_adam(ref, 2, 64, 64, 10, seed=5),
        "mnv2_miou_scene_150steps": lambda: run_miou(ref),
    }
    for name, fn in cases.items():
        if only and name not in only:
            continue
        res = fn()
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **res)
        print(name, "loss32" in res and float(res["loss32"]), "written")
    if only:
        return
    keys = {}
    for arch, ctor in (("MobileNetV2UNet", lambda: ref.MobileNetV2UNet(10)), ("UNet", lambda: ref.UNet(10)),
                       ("LightUNet", lambda: ref.LightUNet())):
        m = ctor()
        keys[arch] = [[k, list(v.shape)] for k, v in m.state_dict().items()]
    bb = tv_stub.mobilenet_v2()
    keys["_mobilenet_v2_param_count"] = sum(p.numel() for p in bb.parameters())
    with open(os.path.join(HERE, "state_dict_keys.json"), "w") as f:
        json.dump(keys, f)
    print("state_dict_keys.json written")


if __name__ == "__main__":
    main()
