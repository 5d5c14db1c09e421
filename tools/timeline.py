"""Two-stream timeline of one training step from HIP events (no profiler): every launch of the replayed tape
bracketed by events on its own stream (side stream ON, as in the bench), then per tape and replay: when the main
stream's last kernel ends, when the side stream (weight gradients) ends, the main stream's idle time, and the
side-stream launches that end last -- the tail the weight gradients leave after the backward (DESIGN round 6).

    python tools/timeline.py [--math f32|bf16io] [--model MobileNetV2UNet] [--batch 32] [--steps 4]
(The event pairs add ~1-2 us per launch; compare the spans, not the absolute step time, with bench.py.)
"""
import argparse
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
    ap.add_argument("--math", default="bf16io")
    ap.add_argument("--model", default="MobileNetV2UNet")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--height", type=int, default=256)
    ap.add_argument("--width", type=int, default=512)
    ap.add_argument("--steps", type=int, default=4)
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
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    timer = E.KernelTimer(kinds=None, max_replays=a.steps)
    E.TIMER = timer
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    E.TIMER = None
    for tape in timer.tapes:
        lab = {t[0]: (t[3], t[4]) for t in tape.timers}
        rows = {k: [] for k in ("span", "main_end", "side_end", "tail", "main_busy", "side_busy", "main_idle")}
        for r in range(a.steps):
            tl = tape.timeline(r)
            main = sorted((s, e, i) for i, s, e in tl if tape.streams[i] == 0)
            side = sorted((s, e, i) for i, s, e in tl if tape.streams[i] == 1)
            if not main:
                continue
            main_end = max(e for s, e, i in main)
            side_end = max((e for s, e, i in side), default=0.0)
            idle, prev = 0.0, 0.0
            for s, e, i in main:
                idle += max(0.0, s - prev)
                prev = max(prev, e)
            rows["span"].append(max(main_end, side_end))
            rows["main_end"].append(main_end)
            rows["side_end"].append(side_end)
            rows["tail"].append(side_end - main_end)
            rows["main_busy"].append(sum(e - s for s, e, i in main))
            rows["side_busy"].append(sum(e - s for s, e, i in side))
            rows["main_idle"].append(idle)
            if r == a.steps - 1 and side:
                print(f"side-stream launches ending last (replay {r}): end ms, duration, op, entry")
                for s, e, i in sorted(side, key=lambda t: -t[1])[:12]:
                    print(f"   {e:7.3f} {1e3 * (e - s):7.1f} us  {lab[i][0]:9s} {lab[i][1]}")
                print(f"main-stream launches ending last (replay {r}):")
                for s, e, i in sorted(main, key=lambda t: -t[1])[:6]:
                    print(f"   {e:7.3f} {1e3 * (e - s):7.1f} us  {lab[i][0]:9s} {lab[i][1]}")
        print(f"tape of {tape.n} entries, {len(main)} main + {len(side)} side timed launches -- {a.model} {a.math} "
              f"bs={a.batch}: medians over {len(rows['span'])} replays (ms after the tape's first launch)")
        for k, v in rows.items():
            if v:
                print(f"  {k:10s} {statistics.median(v):8.3f}")


if __name__ == "__main__":
    main()
