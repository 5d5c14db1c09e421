"""Per-C-ABI-call timing of one training step: every libsegamd call the engine
makes is bracketed by HIP events and labelled with its program op, so each
kernel launch can be compared with the bytes / FLOPs of its layer.

    python tools/callprof.py [--batch 32] [--steps 3] [--top 60]
Columns: median ms, op label, phase, C-ABI function, y-tensor MB of the op
(conv output / upsample output), GB/s if the call streamed k*y bytes (k shown).
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
CUR = [None]
ACTIVE = [False]
_call = E.call


def timed(name, *args):
    if not ACTIVE[0]:
        return _call(name, *args)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    r = _call(name, *args)
    b.record()
    RECS[(CUR[0], name)].append((a, b))
    return r


def wrap(cls, phase):
    orig = getattr(cls, phase)

    def f(self, rt):
        CUR[0] = (id(self), phase[:3])
        try:
            return orig(self, rt)
        finally:
            CUR[0] = None
    setattr(cls, phase, f)


def label(op, k):
    if isinstance(op, E.ConvOp):
        return (f"{k:3d} {op.kind}{op.ks}{'s2' if op.stride == 2 else '  '} {op.cin:4d}->{op.cout:4d} "
                f"@{op.y.H}x{op.y.W}{' +res' if op.res is not None else ''}")
    return f"{k:3d} {type(op).__name__} C={getattr(op, 'low', getattr(op, 'inp', None)).C}"


def ybytes(op):
    if isinstance(op, E.ConvOp):
        return 4 * op.y.M * op.cout
    if isinstance(op, E.UpsampleOp):
        return 4 * op.out.M * op.out.C
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="MobileNetV2UNet")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--height", type=int, default=256)
    ap.add_argument("--width", type=int, default=512)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--top", type=int, default=60)
    a = ap.parse_args()
    E.call = timed
    E._timed_call = lambda kind, flops, name, *args: timed(name, *args)
    for cls in (E.ConvOp, E.UpsampleOp, E.PoolOp):
        wrap(cls, "forward")
        wrap(cls, "backward")
    model = deterministic_init(getattr(models, a.model)(10), seed=0).cuda().train()
    opt = torch.optim.Adam(model.parameters(), lr=1.5e-4)
    x, y = synthetic_batch(a.batch, a.height, a.width, 10, seed=1)
    x, y = x.cuda(), y.cuda()

    def step():
        opt.zero_grad(set_to_none=True)
        model.forward_loss(x, y).backward()
        opt.step()
    for _ in range(2):
        step()
    torch.cuda.synchronize()
    ACTIVE[0] = True
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.steps):
        step()
    e1.record()
    torch.cuda.synchronize()
    ACTIVE[0] = False
    prog = E.get_program(model, a.batch, a.height, a.width)
    ops = {id(op): (k, op) for k, op in enumerate(prog.ops)}
    rows, byfn = [], collections.Counter()
    for (cur, name), r in RECS.items():
        t = statistics.median(s.elapsed_time(e) for s, e in r) * 1e-3 * len(r) / a.steps
        if cur is None:
            lab, yb = "(outside ops)", 0
        else:
            k, op = ops[cur[0]]
            lab, yb = label(op, k) + " " + cur[1], ybytes(op)
        rows.append((t, lab, name, yb))
        byfn[name] += t
    step_ms = e0.elapsed_time(e1) / a.steps
    print(f"step {step_ms:.3f} ms (events), sum of calls {sum(r[0] for r in rows) * 1e3:.3f} ms")
    print(f"{'us':>8} {'op':48s} {'call':26s} {'yMB':>6} {'GB/s@1y':>8}")
    for t, lab, name, yb in sorted(rows, reverse=True)[:a.top]:
        print(f"{t * 1e6:8.1f} {lab:48s} {name:26s} {yb / 1e6:6.1f} {yb / t / 1e9 if yb else 0:8.0f}")
    print("-- by call")
    for k, v in byfn.most_common():
        print(f"{v * 1e3:8.3f} ms {k}")


if __name__ == "__main__":
    main()
