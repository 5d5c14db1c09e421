"""Diagnostic (not a test): compare the engine's concat activations and their
gradients with the oracle's, block by block (UNet / MobileNetV2UNet)."""
import os
import sys

import torch

sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), p)
                for p in ("team02-objectdetection_amd", "")]
from oracle import segref  # noqa: E402
from seg_amd import MobileNetV2UNet, UNet, engine  # noqa: E402
from seg_amd.detinit import deterministic_init, synthetic_batch  # noqa: E402


def rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm())


def main(arch="UNet", classes=4, n=2, h=32, w=64, seed=3):
    classes, n, h, w, seed = int(classes), int(n), int(h), int(w), int(seed)
    ctor = (lambda: UNet(classes, 64)) if arch == "UNet" else (lambda: MobileNetV2UNet(classes))
    mc = deterministic_init(ctor(), seed=seed)
    m = deterministic_init(ctor(), seed=seed).cuda().train()
    x, y = synthetic_batch(n, h, w, classes, seed=seed + 100)
    engine.DEBUG_KEEP_RUN = True
    loss = m.forward_loss(x.cuda(), y.cuda())
    loss.backward()
    torch.cuda.synchronize()
    run = engine.LAST_RUN
    for dt in (torch.float32, torch.float64):
        segref.RECORD = {}
        p = segref.canonical_state(mc.state_dict(), dt)
        segref.forward_backward(arch, p, x.to(dt), y, True)
        rec = segref.RECORD
        segref.RECORD = None
        print("== oracle", dt)
        for name, t in rec.items():
            if not name.endswith("cat"):
                continue
            blk = name.split(".")[0]
            cat_buf = {"UNet": {"up1": "cat1", "up2": "cat2", "up3": "cat3"},
                       "MobileNetV2UNet": {"up1": "cat1", "up2": "cat2", "up3": "cat3", "up4": "cat4"}}[arch][blk]
            N, C, H, W = t.shape
            ld = run.bufs[cat_buf].numel() // (N * H * W)
            act = run.bufs[cat_buf].view(N, H, W, ld)[..., :C].permute(0, 3, 1, 2).cpu()
            g = run.gbufs[cat_buf].view(N, H, W, ld)[..., :C].permute(0, 3, 1, 2).cpu()
            cs = C - rec[blk + ".low"].shape[1]
            print(f"{blk}: act rel {rel(act, t.detach()):.2e}  grad rel {rel(g, t.grad):.2e}  "
                  f"grad(skip) {rel(g[:, :cs], t.grad[:, :cs]):.2e}  grad(up) {rel(g[:, cs:], t.grad[:, cs:]):.2e}")
        ups = [op for op in run.prog.ops if isinstance(op, engine.UpsampleOp)]
        for k, op in enumerate(ups):
            lo = op.low
            t = rec[f"up{k + 1}.low"]
            g = run.gbufs[lo.buf].view(lo.M, -1)[:, lo.off:lo.off + lo.C].reshape(lo.N, lo.H, lo.W, lo.C)
            g = g.permute(0, 3, 1, 2).cpu()
            a = run.bufs[lo.buf].view(lo.M, -1)[:, lo.off:lo.off + lo.C].reshape(lo.N, lo.H, lo.W, lo.C)
            a = a.permute(0, 3, 1, 2).cpu()
            # recompute the upsample backward on CPU from the engine's own d(cat) to isolate the kernel
            cat = [o for o in run.prog.ops if isinstance(o, engine.UpsampleOp)][k].out
            dcat = run.gbufs[cat.buf].view(cat.M, -1)[:, cat.off:cat.off + cat.C]
            dcat = dcat.reshape(cat.N, cat.H, cat.W, cat.C).permute(0, 3, 1, 2).cpu().double()
            lo_t = torch.zeros(lo.N, lo.C, lo.H, lo.W, dtype=torch.float64, requires_grad=True)
            torch.nn.functional.interpolate(lo_t, scale_factor=2, mode="bilinear").backward(dcat)
            print(f"up{k + 1}.low {lo.buf}: act rel {rel(a, t.detach()):.2e}  grad rel {rel(g, t.grad):.2e}  "
                  f"kernel-vs-cpu-upsample-bwd {rel(g, lo_t.grad):.2e}")


if __name__ == "__main__" and (len(sys.argv) < 2 or sys.argv[1] not in ("layers", "stats")):
    main(*sys.argv[1:])


def layers(arch="UNet", classes=4, n=2, h=32, w=64, seed=3):
    """Per conv: engine raw output y, output activation and its gradient vs the oracle."""
    classes, n, h, w, seed = int(classes), int(n), int(h), int(w), int(seed)
    ctor = (lambda: UNet(classes, 64)) if arch == "UNet" else (lambda: MobileNetV2UNet(classes))
    mc = deterministic_init(ctor(), seed=seed)
    m = deterministic_init(ctor(), seed=seed).cuda().train()
    names = {id(mod): nm for nm, mod in m.named_modules()}
    x, y = synthetic_batch(n, h, w, classes, seed=seed + 100)
    engine.DEBUG_KEEP_RUN = True
    loss = m.forward_loss(x.cuda(), y.cuda())
    loss.backward()
    torch.cuda.synchronize()
    run = engine.LAST_RUN
    segref.RECORD = {}
    p = segref.canonical_state(mc.state_dict(), torch.float64)
    segref.forward_backward(arch, p, x.double(), y, True)
    rec = segref.RECORD
    segref.RECORD = None

    def get(bufs, a):
        t = bufs[a.buf].view(a.M, -1)[:, a.off:a.off + a.C].reshape(a.N, a.H, a.W, a.C)
        return t.permute(0, 3, 1, 2).cpu()

    for op in reversed(run.prog.ops):
        if not isinstance(op, engine.ConvOp):
            continue
        nm = names[id(op.conv)].replace("down1.", "backbone.features.", 0) + "."
        if nm + "out" not in rec:
            nm = nm.replace("down", "backbone.features.")
        r_out, r_raw = rec.get(nm + "out"), rec.get(nm + "raw")
        if r_out is None:
            print("?", nm)
            continue
        line = f"{nm:40s} out {rel(get(run.bufs, op.out), r_out.detach()):.1e}"
        if op.bn is not None:
            line += f" raw {rel(get(run.bufs, op.y), r_raw.detach()):.1e}"
        if r_out.grad is not None and op.out.buf in run.gbufs:
            line += f" dout {rel(get(run.gbufs, op.out), r_out.grad):.1e}"
        print(line)


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "layers":
    layers(*sys.argv[2:])


def stats(arch="UNet", classes=4, n=2, h=32, w=64, seed=3):
    """Do the saved BN statistics change between forward and backward?"""
    classes, n, h, w, seed = int(classes), int(n), int(h), int(w), int(seed)
    ctor = (lambda: UNet(classes, 64)) if arch == "UNet" else (lambda: MobileNetV2UNet(classes))
    m = deterministic_init(ctor(), seed=seed).cuda().train()
    names = {id(mod): nm for nm, mod in m.named_modules()}
    x, y = synthetic_batch(n, h, w, classes, seed=seed + 100)
    engine.DEBUG_KEEP_RUN = True
    loss = m.forward_loss(x.cuda(), y.cuda())
    torch.cuda.synchronize()
    run = engine.LAST_RUN
    snap = {k: v.clone() for k, v in run.saved.items()}
    ybufs = {k: v.clone() for k, v in run.bufs.items()}
    loss.backward()
    torch.cuda.synchronize()
    for op in run.prog.ops:
        if isinstance(op, engine.ConvOp) and id(op) in snap:
            d = (snap[id(op)] - run.saved[id(op)]).abs().max().item()
            if d != 0:
                print("STATS CHANGED", names[id(op.conv)], d)
    for k in ybufs:
        d = (ybufs[k] - run.bufs[k]).abs().max().item()
        if d != 0:
            print("BUFFER CHANGED", k, d)
    print("done")


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "stats":
    stats(*sys.argv[2:])
