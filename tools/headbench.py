"""Batch-1 fp16 inference frame time with outconv + mask in one launch (seg_head_argmax_f16) vs the two launches
(seg_pw2_f16 + seg_argmax_nearest): two captured Predictors, graph replays timed interleaved with HIP events.

    python tools/headbench.py [rounds] [frames]
"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "team02-objectdetection_amd"), REPO]
from seg_amd import MobileNetV2UNet, deterministic_init, engine  # noqa: E402
from seg_amd.infer import Predictor  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    frames = int(sys.argv[2]) if len(sys.argv) > 2 else 500
    model = deterministic_init(MobileNetV2UNet(10), seed=0).cuda().eval()
    f = (np.random.default_rng(0).random((720, 1280, 3)) * 255).astype(np.uint8)
    preds = {}
    for fused in (True, False):
        engine.HEAD_ARGMAX = fused
        p = Predictor(model, frame_hw=(720, 1280), graph=True, math="f16")
        p.set_frame(f)
        preds["fused" if fused else "two"] = p
    engine.HEAD_ARGMAX = True
    assert torch.equal(preds["fused"].step().clone(), preds["two"].step().clone())
    for r in range(rounds):
        for k, p in preds.items():
            for _ in range(20):
                p.step()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(frames):
                p.step()
            b.record()
            torch.cuda.synchronize()
            ms = a.elapsed_time(b) / frames
            print(f"{r} {k:6s} {1e3 / ms:8.1f} frames/s  {ms * 1e3:6.1f} us/frame", flush=True)


if __name__ == "__main__":
    main()
