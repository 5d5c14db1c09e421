"""Per-launch timing of the bf16 3x3 / 1x1 weight gradients at the UNet 512x1024 bs 8 (BASELINE configs[4]) and
MobileNetV2UNet bs 32 decoder shapes: seg_conv_wgrad3_bf16io (csrc/wgrad3.hip) against the register-staged
seg_conv_wgrad_bf16io and, where it applies, the LDS-halo seg_conv_wgrad2_bf16io; slab reduce timed apart.
Median of R launches with HIP events, algorithmic TFLOP/s (2 M Cout 9 Cin).

    python tools/wg3bench.py [--set unet|mnv2] [--reps 10]

The LDS-DMA kernel it measures was removed after this measurement (DESIGN round 6, profiles/r06/wg3bench_*.txt):
run it on a checkout of commit a0c410c, where csrc/wgrad3.hip and its entry points still exist.
"""
import argparse
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "team02-objectdetection_amd"), REPO]
from seg_amd._lib import call, query  # noqa: E402

BF = torch.bfloat16
UNET = [("inc.3", 8, 512, 1024, 64, 64), ("d1.0", 8, 256, 512, 64, 128), ("d1.3", 8, 256, 512, 128, 128),
        ("d2.0", 8, 128, 256, 128, 256), ("d2.3", 8, 128, 256, 256, 256), ("d3.3", 8, 64, 128, 256, 256),
        ("u1.0", 8, 128, 256, 512, 128), ("u1.3", 8, 128, 256, 128, 128), ("u2.0", 8, 256, 512, 256, 64),
        ("u2.3", 8, 256, 512, 64, 64), ("u3.0", 8, 512, 1024, 128, 64), ("u3.3", 8, 512, 1024, 64, 64)]
MNV2 = [("up1.0", 32, 16, 32, 1344, 256), ("up1.3", 32, 16, 32, 256, 256), ("up2.0", 32, 32, 64, 288, 128),
        ("up2.3", 32, 32, 64, 128, 128), ("up3.0", 32, 64, 128, 152, 64), ("up3.3", 32, 64, 128, 64, 64)]


def timeit(fn, reps):
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--set", default="unet", choices=("unet", "mnv2"))
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    s = torch.cuda.current_stream().cuda_stream
    for name, N, H, W, Cin, Cout in (UNET if a.set == "unet" else MNV2):
        M = N * H * W
        x = torch.randn(M, Cin, device="cuda").to(BF)
        dy = torch.randn(M, Cout, device="cuda").to(BF)
        fl = 2.0 * M * Cout * 9 * Cin
        line = f"{name:6s} M={M:8d} {Cin:5d}->{Cout:4d}:"
        sp3 = query("seg_conv_wgrad3_splits", N, H, W, Cin, Cout, 3)
        if sp3:
            part = torch.empty(sp3 * Cout * 9 * Cin, device="cuda")
            us = timeit(lambda: call("seg_conv_wgrad3_bf16io", dy.data_ptr(), Cout, x.data_ptr(), Cin, N, H, W, Cin,
                                     Cout, 3, part.data_ptr(), s), a.reps)
            dw = torch.empty(Cout * Cin * 9, device="cuda")
            ur = timeit(lambda: call("seg_conv_wgrad_reduce", part.data_ptr(), sp3, dw.data_ptr(), Cout, Cin, 3, 0, 0, s),
                        a.reps)
            line += f" wg3 {us:7.1f} us {fl / us / 1e6:5.0f} TF/s (+reduce {ur:5.1f}, {sp3} slabs) |"
            del part
        sp = query("seg_conv_wgrad_splits_bf16", M, Cout, Cin, 3)
        part = torch.empty(sp * Cout * 9 * Cin, device="cuda")
        us = timeit(lambda: call("seg_conv_wgrad_bf16io", dy.data_ptr(), Cout, x.data_ptr(), Cin, N, H, W, Cin, H, W,
                                 Cout, 3, 1, 1, part.data_ptr(), sp, s), a.reps)
        dw = torch.empty(Cout * Cin * 9, device="cuda")
        ur = timeit(lambda: call("seg_conv_wgrad_reduce", part.data_ptr(), sp, dw.data_ptr(), Cout, Cin, 3, 0, 0, s),
                    a.reps)
        line += f" wg {us:7.1f} us {fl / us / 1e6:5.0f} TF/s (+reduce {ur:5.1f}, {sp}) |"
        del part
        if query("seg_conv_wgrad2_ok", N, H, W, Cin, Cout):
            nb = query("seg_conv_wgrad2_blocks", N, H, W)
            part = torch.empty(nb * Cout * 9 * Cin, device="cuda")
            us = timeit(lambda: call("seg_conv_wgrad2_bf16io", dy.data_ptr(), Cout, x.data_ptr(), Cin, N, H, W, Cin,
                                     Cout, part.data_ptr(), s), a.reps)
            line += f" wg2 {us:7.1f} us {fl / us / 1e6:5.0f} TF/s"
            del part
        print(line, flush=True)


if __name__ == "__main__":
    main()
