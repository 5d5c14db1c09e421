"""Batch-1 decoder convs of the folded fp16 inference forward (configs[3], 128x256 frame):
seg_conv_igemm_f16_ic per launch over split counts and forced tiles, against the
engine's default (seg_conv_igemm_splits + the tile cost model).   python tools/icbench.py"""
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "team02-objectdetection_amd"), REPO]
from seg_amd._lib import call, query  # noqa: E402
from seg_amd import engine as E  # noqa: E402

SHAPES = [  # H, W, Cin, Cout, ks   (up1..up4 of MobileNetV2UNet at 1/16..1/2 of 128x256; features[18])
    (8, 16, 1344, 256, 3), (8, 16, 256, 256, 3), (16, 32, 288, 128, 3), (16, 32, 128, 128, 3),
    (32, 64, 152, 64, 3), (32, 64, 64, 64, 3), (64, 128, 80, 32, 3), (64, 128, 32, 32, 3), (4, 8, 320, 1280, 1)]
TILES = [-1, 0, 1, 2, 3, 6, 7, 12]


def timeit(fn, reps=40):
    for _ in range(5):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(reps):
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return statistics.median(ts)


def main():
    s = torch.cuda.current_stream().cuda_stream
    for H, W, Cin, Cout, ks in SHAPES:
        M = H * W
        x = torch.randn(M, Cin, device="cuda")
        K = ks * ks * Cin
        wk = torch.randn(Cout, K, device="cuda") * 0.02
        b = torch.randn(Cout, device="cuda")
        out = torch.empty(M, Cout, device="cuda")
        d = query("seg_conv_igemm_splits", M, Cout, Cin, ks)
        work = torch.empty(64 * M * Cout, device="cuda")
        cnt = torch.zeros(4 * 4096, device="cuda", dtype=torch.int32)
        res = {}
        for t in TILES:
            E.force_tiles(igemm=t)
            for sp in sorted({1, 2, 4, 8, 16, 32, 64, d}):
                if sp > 1 and sp != d and sp * 2 > K // 16:
                    continue

                def f():
                    call("seg_conv_igemm_f16_ic", x.data_ptr(), Cin, 1, H, W, Cin, wk.data_ptr(), K, b.data_ptr(),
                         out.data_ptr(), Cout, H, W, Cout, ks, 1, ks // 2, None, 0, 2, work.data_ptr(), sp,
                         cnt.data_ptr(), s)
                res[(t, sp)] = timeit(f)
        E.force_tiles(igemm=-1)
        best = min(res, key=res.get)
        flop = 2.0 * M * Cout * K
        print(f"H{H} W{W} {Cin}->{Cout} k{ks} M={M} K={K}: default (tile -1, {d} splits) {res[(-1, d)]:.1f} us; "
              f"best tile {best[0]} splits {best[1]} {res[best]:.1f} us ({flop / res[best] / 1e6:.0f} TF/s)", flush=True)
        row = " ".join(f"t{t}s{sp}:{v:.1f}" for (t, sp), v in sorted(res.items()))
        print("   ", row, flush=True)


if __name__ == "__main__":
    main()
