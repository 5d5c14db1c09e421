"""Per-op timing of one MobileNetV2UNet (or UNet) training step on the GPU.

HIP events bracket every program op's forward and backward (all kernels of the
op, including its BatchNorm), median over R steps.  Each row shows the op's
algorithmic FLOPs and minimal HBM bytes (every tensor the op must touch, read
or written once) so the distance from the MFMA / HBM roofline is visible.

    python tools/opprof.py [--model MobileNetV2UNet] [--batch 32] [--steps 3] [--top 40]
"""
import argparse
import collections
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "team02-objectdetection_amd"), REPO]
from seg_amd import engine as E  # noqa: E402
import seg_amd as models  # noqa: E402
from seg_amd import deterministic_init, synthetic_batch  # noqa: E402

RECS = collections.defaultdict(list)
ACTIVE = [False]


def wrap(cls, phase):
    orig = getattr(cls, phase)

    def f(self, rt):
        if not ACTIVE[0]:
            return orig(self, rt)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        orig(self, rt)
        b.record()
        RECS[(id(self), phase)].append((a, b))
    setattr(cls, phase, f)


def op_cost(op, phase):
    """(flops, bytes) of the op's phase, fp32, minimal traffic model."""
    if isinstance(op, E.ConvOp):
        y, i = op.y, op.inp
        Mi, Mo, C = i.M, y.M, op.cout
        fl = op.flops()
        x_b, y_b = 4 * Mi * i.C, 4 * Mo * C
        bn = op.bn is not None
        if phase == "forward":
            b = x_b + y_b + (2 * y_b + (y_b if op.res is not None else 0) if bn else 0)
            return fl, b
        # backward: BN bwd (read dA, y twice, write dY), wgrad (read dY, x), dgrad (read dY, write dx)
        b = (5 * y_b if bn else 0) + (y_b + x_b) + (0 if op.first else y_b + x_b)
        return fl * (1 if op.first else 2), b
    if isinstance(op, E.UpsampleOp):
        return 0, 4 * (op.low.M * op.low.C + op.out.M * op.out.C)
    if isinstance(op, E.PoolOp):
        return 0, 4 * (op.inp.M * op.inp.C + op.out.M * op.out.C) * (1 if phase == "forward" else 2)
    return 0, 0


def label(op, k):
    if isinstance(op, E.ConvOp):
        return (f"{k:3d} {op.kind}{op.ks}{'s2' if op.stride == 2 else '  '} {op.cin:4d}->{op.cout:4d} "
                f"@{op.y.H}x{op.y.W}{' +res' if op.res is not None else ''}{' bn' if op.bn is not None else ''}")
    return f"{k:3d} {type(op).__name__} C={getattr(op, 'low', getattr(op, 'inp', None)).C}"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="MobileNetV2UNet")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--height", type=int, default=256)
    ap.add_argument("--width", type=int, default=512)
    ap.add_argument("--classes", type=int, default=10)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--top", type=int, default=45)
    a = ap.parse_args()
    for cls in (E.ConvOp, E.UpsampleOp, E.PoolOp):
        wrap(cls, "forward")
        wrap(cls, "backward")
    model = deterministic_init(getattr(models, a.model)(a.classes), seed=0).cuda().train()
    opt = torch.optim.Adam(model.parameters(), lr=1.5e-4)
    x, y = synthetic_batch(a.batch, a.height, a.width, a.classes, seed=1)
    x, y = x.cuda(), y.cuda()

    def step():
        opt.zero_grad(set_to_none=True)
        model.forward_loss(x, y).backward()
        opt.step()
    for _ in range(2):
        step()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ACTIVE[0] = True
    ev0.record()
    for _ in range(a.steps):
        step()
    ev1.record()
    torch.cuda.synchronize()
    ACTIVE[0] = False
    step_ms = ev0.elapsed_time(ev1) / a.steps
    prog = E.get_program(model, a.batch, a.height, a.width)
    rows, cat = [], collections.Counter()
    for k, op in enumerate(prog.ops):
        for ph in ("forward", "backward"):
            r = RECS.get((id(op), ph))
            if not r:
                continue
            t = statistics.median(s.elapsed_time(e) for s, e in r) * 1e-3
            fl, by = op_cost(op, ph)
            kind = (f"{op.kind}{op.ks}" if isinstance(op, E.ConvOp) else type(op).__name__) + "_" + ph[:3]
            cat[kind] += t
            rows.append((t, label(op, k), ph[:3], fl / t / 1e12 if fl else 0.0, by / t / 1e9))
    tot = sum(r[0] for r in rows)
    print(f"step {step_ms:.3f} ms (events), ops {tot * 1e3:.3f} ms, outside ops {step_ms - tot * 1e3:.3f} ms")
    print(f"{'ms':>7} {'op':44s} ph  {'TF/s':>6} {'GB/s':>7}")
    for t, lab, ph, tf, gbs in sorted(rows, reverse=True)[:a.top]:
        print(f"{t * 1e3:7.3f} {lab:44s} {ph} {tf:6.1f} {gbs:7.0f}")
    print("-- by kind")
    for k, v in cat.most_common():
        print(f"{v * 1e3:7.3f} {k}")


if __name__ == "__main__":
    main()
