"""Host vs GPU timeline of one training step at the bench configuration: host time spent
in forward_loss / backward / opt.step, and how far the host runs ahead of the GPU (a HIP
event recorded when each phase returns, compared with the host clock).

    python tools/host_phases.py [--math f32|bf16io] [--steps 10]
"""
import argparse
import os
import statistics
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "team02-objectdetection_amd"), REPO]
import seg_amd  # noqa: E402
from seg_amd import engine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--math", default="f32")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--batch", type=int, default=32)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    model = seg_amd.deterministic_init(seg_amd.MobileNetV2UNet(10), seed=0).to(dev).train()
    engine.set_conv_math(model, a.math)
    opt = seg_amd.Adam(model.parameters(), lr=1.5e-4)
    x, y = seg_amd.synthetic_batch(a.batch, 256, 512, 10, seed=1)
    x, y = x.to(dev), y.to(dev)
    for _ in range(3):
        opt.zero_grad(set_to_none=True)
        model.forward_loss(x, y).backward()
        opt.step()
    torch.cuda.synchronize()
    rows = []
    for _ in range(a.steps):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        h = [time.perf_counter()]
        ev[0].record()
        opt.zero_grad(set_to_none=True)
        loss = model.forward_loss(x, y)
        h.append(time.perf_counter()); ev[1].record()
        loss.backward()
        h.append(time.perf_counter()); ev[2].record()
        opt.step()
        h.append(time.perf_counter()); ev[3].record()
        torch.cuda.synchronize()
        h.append(time.perf_counter())
        g = [0.0] + [ev[0].elapsed_time(e) for e in ev[1:]]
        rows.append(([1e3 * (t - h[0]) for t in h], g))
    med = lambda k, i: statistics.median(r[k][i] for r in rows)  # noqa: E731
    print(f"{a.math} bs={a.batch}: median over {a.steps} steps (ms from the step start)")
    for i, name in enumerate(["forward_loss", "backward", "opt.step"], start=1):
        print(f"  {name:13s} host returns {med(0, i):7.2f}   GPU reaches it {med(1, i):7.2f}")
    print(f"  host sync returns {med(0, 4):7.2f}")


if __name__ == "__main__":
    main()
