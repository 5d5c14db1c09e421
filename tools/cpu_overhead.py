"""Host-side cost of one training step of the engine (Python + ctypes launches): the
step time at a tiny shape, where the GPU work is negligible, is the launch-bound floor.

    python tools/cpu_overhead.py [--math f32|bf16|bf16io]
"""
import argparse
import os
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
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    for (n, h, w) in ((1, 64, 128), (32, 256, 512)):
        model = seg_amd.deterministic_init(seg_amd.MobileNetV2UNet(10), seed=0).to(dev).train()
        engine.set_conv_math(model, a.math)
        opt = torch.optim.Adam(model.parameters(), lr=1.5e-4)
        x, y = seg_amd.synthetic_batch(n, h, w, 10, seed=1)
        x, y = x.to(dev), y.to(dev)

        def step():
            opt.zero_grad(set_to_none=True)
            loss = model.forward_loss(x, y)
            loss.backward()
            opt.step()
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            step()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"{a.math} bs={n} {h}x{w}: host enqueue {(t1 - t0) / 10 * 1e3:.2f} ms/step, "
              f"wall {(t2 - t0) / 10 * 1e3:.2f} ms/step", flush=True)


if __name__ == "__main__":
    main()
