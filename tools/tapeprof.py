"""Per-launch timing of one training step replayed from the launch tape: every C-ABI
launch of the step bracketed by HIP events inside libsegamd (seg_tape_timing), median
over the profiled replays, grouped per program op and entry point, with the op's
shapes so HBM / MFMA rates can be read off.

    python tools/tapeprof.py [--math f32|bf16io] [--model MobileNetV2UNet] [--batch 32] [--steps 5]
"""
import argparse
import collections
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "team02-objectdetection_amd"), REPO]
import seg_amd  # noqa: E402
from seg_amd import engine as E  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--math", default="f32")
    ap.add_argument("--model", default="MobileNetV2UNet")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--height", type=int, default=256)
    ap.add_argument("--width", type=int, default=512)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--top", type=int, default=60)
    ap.add_argument("--csv", default=None, help="also write every launch (us, label, entry, kind, M, Cin, Cout) here")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    model = seg_amd.deterministic_init(getattr(seg_amd, a.model)(10), seed=0).to(dev).train()
    E.set_conv_math(model, a.math)
    opt = seg_amd.Adam(model.parameters(), lr=1.5e-4)
    x, y = seg_amd.synthetic_batch(a.batch, a.height, a.width, 10, seed=1)
    x, y = x.to(dev), y.to(dev)

    def step():
        opt.zero_grad(set_to_none=True)
        model.forward_loss(x, y).backward()
        opt.step()
    for _ in range(2):
        step()
    torch.cuda.synchronize()
    timer = E.KernelTimer(kinds=None, max_replays=a.steps)
    E.TIMER = timer
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    E.TIMER = None
    prog = E.get_program(model, a.batch, a.height, a.width)
    per = collections.defaultdict(list)
    for t in timer.tapes:
        for r, label, name, kind, flops, sec in t.elapsed(detail=True):
            per[(label, name)].append(sec)
    rows, csv_rows = [], []
    for (label, name), secs in per.items():
        k, phase = label.split(":") if label else ("-1", "")
        op = prog.ops[int(k)] if label else None
        desc = ""
        if isinstance(op, E.ConvOp):
            desc = f"{op.kind} k{op.ks}s{op.stride} {op.cin}->{op.cout} M={op.y.M}"
        elif op is not None:
            desc = type(op).__name__
        rows.append((statistics.median(secs) * 1e6, label, name, desc, len(secs)))
        if a.csv:
            shp = (op.kind, op.ks, op.stride, op.y.M, op.inp.M, op.cin, op.cout) if isinstance(op, E.ConvOp) else \
                (type(op).__name__, 0, 0, 0, 0, 0, 0)
            csv_rows.append((statistics.median(secs) * 1e6, label, name) + shp)
    total = sum(r[0] for r in rows)
    by_name = collections.Counter()
    for us, label, name, desc, n in rows:
        by_name[name] += us
    print(f"{a.model} {a.math} bs={a.batch} {a.height}x{a.width}: {len(rows)} launches, sum of medians {total / 1e3:.2f} ms "
          "(both streams)")
    for name, us in by_name.most_common():
        print(f"  {us / 1e3:7.3f} ms  {name}")
    print()
    for us, label, name, desc, n in sorted(rows, reverse=True)[:a.top]:
        print(f"{us:9.1f} us  {label:9s} {name:32s} {desc}")
    if a.csv:
        import csv
        with open(a.csv, "w", newline="") as fh:
            w = csv.writer(fh)
            w.writerow(["us", "label", "entry", "kind", "ks", "stride", "M_out", "M_in", "cin", "cout"])
            w.writerows(sorted(csv_rows, key=lambda r: r[1]))


if __name__ == "__main__":
    main()
