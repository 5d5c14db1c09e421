"""Microbenchmark of the bf16io deep-conv kernels at the MobileNetV2UNet (bs=32, 256x512)
shapes: seg_conv_igemm2_bf16io (csrc/igemm2.hip) against the generic 16-bit implicit GEMM
(seg_conv_igemm_bf16io_w16), forward and data-gradient shapes, median of R launches with
HIP events, in TFLOP/s.

    python tools/ig2bench.py [--only up1.0f,...] [--kernel ig2|gen|both] [--reps 20]
(--kernel ig2 with --only one shape is the form to run under rocprofv3 --pmc.)
"""
import argparse
import ctypes
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "team02-objectdetection_amd"), REPO]
from seg_amd import engine  # noqa: E402
from seg_amd._lib import call  # noqa: E402

BF = torch.bfloat16
SHAPES = [  # name, N, H, W, Cin, Cout (3x3, stride 1): forward shapes and data-gradient shapes
    ("up1.0f", 32, 16, 32, 1344, 256), ("up1.0d", 32, 16, 32, 256, 1344), ("up1.3", 32, 16, 32, 256, 256),
    ("up2.0f", 32, 32, 64, 288, 128), ("up2.3", 32, 32, 64, 128, 128),
    ("up3.3", 32, 64, 128, 64, 64), ("up4.0f", 32, 128, 256, 80, 32), ("up4.3", 32, 128, 256, 32, 32),
]
UNET = [  # UNet 10-class 512x1024 bs=8 (BASELINE configs[4]): forward shapes + data-gradient shapes (Cin <-> Cout)
    ("inc.3", 8, 512, 1024, 64, 64), ("d1.0f", 8, 256, 512, 64, 128), ("d1.0d", 8, 256, 512, 128, 64),
    ("d1.3", 8, 256, 512, 128, 128), ("d2.0f", 8, 128, 256, 128, 256), ("d2.0d", 8, 128, 256, 256, 128),
    ("d2.3", 8, 128, 256, 256, 256), ("d3.3", 8, 64, 128, 256, 256), ("u1.0f", 8, 128, 256, 512, 128),
    ("u1.0d", 8, 128, 256, 128, 512), ("u1.3", 8, 128, 256, 128, 128), ("u2.0f", 8, 256, 512, 256, 64),
    ("u2.0d", 8, 256, 512, 64, 256), ("u2.3", 8, 256, 512, 64, 64), ("u3.0f", 8, 512, 1024, 128, 64),
    ("u3.0d", 8, 512, 1024, 64, 128),
]


def timeit(fn, reps):
    fn()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e-3)
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="")
    ap.add_argument("--kernel", default="both", choices=("ig2", "gen", "both", "halo", "all"))
    ap.add_argument("--set", default="mnv2", choices=("mnv2", "unet"))
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    only = set(a.only.split(",")) if a.only else None
    s = torch.cuda.current_stream().cuda_stream
    g = torch.Generator().manual_seed(0)
    for name, N, H, W, Cin, Cout in (UNET if a.set == "unet" else SHAPES):
        if only and name not in only:
            continue
        M, ks = N * H * W, 3
        x = (torch.randn(M, Cin, generator=g)).to(BF).cuda()
        w = (torch.randn(Cout, Cin, 3, 3, generator=g) * 0.02).cuda()
        ldk = (9 * Cin + 7) & ~7
        wk = torch.empty(Cout * ldk, device="cuda", dtype=BF)
        table, n, blocks = engine.pack_table([(w.data_ptr(), wk.data_ptr(), Cout, Cin, 3, ldk, 16, Cin)], w.device)
        call("seg_pack_batch", table.data_ptr(), n, blocks, s)
        y = torch.empty(M, Cout, device="cuda", dtype=BF)
        plan = engine.igemm2_plan(M, Cout, Cin, ks)
        flops = 2.0 * M * Cout * Cin * 9
        res = []
        if plan and a.kernel in ("ig2", "both", "all"):
            work = torch.zeros(max(plan[3], 1), device="cuda")
            t = timeit(lambda: call("seg_conv_igemm2_bf16io", x.data_ptr(), Cin, N, H, W, Cin, wk.data_ptr(), ldk, None,
                                    y.data_ptr(), Cout, Cout, ks, None, 0, None, work.data_ptr(), s), a.reps)
            res.append(f"ig2 {t * 1e6:7.1f} us {flops / t / 1e12:6.0f} TF/s (tile rows {plan[0]}, splits {plan[2]})")
        if a.kernel in ("halo", "all") and engine.query("seg_conv_halo_pick", N, H, W, Cin, Cout):
            t = timeit(lambda: call("seg_conv_halo_bf16io_w16", x.data_ptr(), Cin, N, H, W, Cin, wk.data_ptr(),
                                    ldk, None, y.data_ptr(), Cout, Cout, None, 0, None, s), a.reps)
            res.append(f"halo {t * 1e6:7.1f} us {flops / t / 1e12:6.0f} TF/s")
        if a.kernel in ("gen", "both", "all"):
            t = timeit(lambda: call("seg_conv_igemm_bf16io_w16", x.data_ptr(), Cin, N, H, W, Cin, wk.data_ptr(), ldk,
                                    None, y.data_ptr(), Cout, H, W, Cout, 3, 1, 1, None, 0, None, s), a.reps)
            res.append(f"gen {t * 1e6:7.1f} us {flops / t / 1e12:6.0f} TF/s")
        print(f"{name:7s} M={M:6d} {Cin:5d}->{Cout:5d}: " + " | ".join(res), flush=True)


if __name__ == "__main__":
    main()
