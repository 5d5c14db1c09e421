"""Thin weight-gradient kernel vs the tiled kernel on the MobileNetV2UNet shapes it
serves (bs=32, 256x512): seg_conv_wgrad* + reduce, HIP-event medians.

    python tools/thinbench.py [--bf16io]
The tiled kernel is selected by passing a split count other than the thin plan's.
"""
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "team02-objectdetection_amd"))
from seg_amd._lib import call, query  # noqa: E402

SHAPES = [  # name, N, H, W (input), Cin (padded), Cout, ks, stride, xf
    ("stem", 32, 256, 512, 4, 32, 3, 2, False), ("f1.proj", 32, 128, 256, 32, 16, 1, 1, True),
    ("f2.exp", 32, 128, 256, 16, 96, 1, 1, False), ("f2.proj", 32, 64, 128, 96, 24, 1, 1, True),
    ("f3.exp", 32, 64, 128, 24, 144, 1, 1, False), ("f3.proj", 32, 64, 128, 144, 24, 1, 1, True),
    ("outc.0", 32, 128, 256, 32, 16, 1, 1, False), ("outc.3", 32, 128, 256, 16, 10, 1, 1, True)]


def timeit(fn, reps=15):
    fn()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return statistics.median(ts)


def main():
    bf = "--bf16io" in sys.argv
    dt = torch.bfloat16 if bf else torch.float32
    s = torch.cuda.current_stream().cuda_stream
    for name, N, H, W, Cin, Cout, ks, st, xf in SHAPES:
        pad = ks // 2
        Ho, Wo = (H + 2 * pad - ks) // st + 1, (W + 2 * pad - ks) // st + 1
        M = N * Ho * Wo
        ldy = (Cout + 3) & ~3
        x = torch.randn(N * H * W, Cin, device="cuda").to(dt)
        dy = torch.randn(M, ldy, device="cuda").to(dt)
        sc, sh = torch.rand(Cin, device="cuda"), torch.rand(Cin, device="cuda")
        fn = ("seg_conv_wgrad_bf16io" if bf else "seg_conv_wgrad") + ("_xf" if xf else "")
        extra = (sc.data_ptr(), sh.data_ptr(), 2) if xf else ()
        dw = torch.empty(Cout * Cin * ks * ks, device="cuda")
        res = []
        for splits in (query("seg_conv_wgrad_splits", M, Cout, Cin, ks), 1000):
            part = torch.empty(splits * Cout * Cin * ks * ks, device="cuda")

            def run():
                call(fn, dy.data_ptr(), ldy, x.data_ptr(), Cin, N, H, W, Cin, Ho, Wo, Cout, ks, st, pad,
                     part.data_ptr(), splits, *extra, s)
                call("seg_conv_wgrad_reduce", part.data_ptr(), splits, dw.data_ptr(), Cout, Cin, ks, 0, 0, s)
            res.append((splits, timeit(run)))
        (s1, t1), (s2, t2) = res
        print(f"{name:8s} {Cin:4d}->{Cout:4d} M={M:8d}: planned splits {s1:5d} {t1:7.1f} us | tiled 1000 splits {t2:7.1f} us")


if __name__ == "__main__":
    main()
