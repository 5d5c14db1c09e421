"""Isolated timing of the 1x1 (pointwise) conv launches of the bf16io / f32 step:
seg_conv_igemm(_bf16io) with and without the BN-statistics epilogue, against a plain
copy of the same bytes (the HBM floor).  python tools/pwbench.py [--io bf16|f32]"""
import argparse
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "team02-objectdetection_amd"), REPO]
from seg_amd._lib import call, query  # noqa: E402

SHAPES = [(1048576, 16, 96), (1048576, 96, 16), (1048576, 32, 16), (262144, 24, 144), (262144, 144, 24),
          (262144, 96, 24), (65536, 32, 192), (65536, 192, 32), (16384, 64, 384), (16384, 384, 64),
          (16384, 96, 576), (16384, 576, 96), (4096, 320, 1280)]


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--io", default="bf16")
    a = ap.parse_args()
    dt = torch.bfloat16 if a.io == "bf16" else torch.float32
    es = 2 if a.io == "bf16" else 4
    name = "seg_conv_igemm_bf16io" if a.io == "bf16" else "seg_conv_igemm"
    s = torch.cuda.current_stream().cuda_stream
    for M, cin, cout in SHAPES:
        x = torch.randn(M, cin, device="cuda").to(dt)
        w = torch.randn(cout, cin, device="cuda") * 0.1
        y = torch.empty(M, cout, device="cuda", dtype=dt)
        ntiles = query("seg_conv_igemm_row_tiles", M, cout, 0) if False else None
        import ctypes
        rows = ctypes.c_int(0)
        nt = query("seg_conv_igemm_row_tiles", M, cout, ctypes.addressof(rows))
        stat = torch.empty(nt * 2 * cout, device="cuda")
        f_stat = lambda: call(name, x.data_ptr(), cin, M, 1, 1, cin, w.data_ptr(), cin, None, y.data_ptr(), cout, 1, 1,
                              cout, 1, 1, 0, None, 0, stat.data_ptr(), s)
        f_nostat = lambda: call(name, x.data_ptr(), cin, M, 1, 1, cin, w.data_ptr(), cin, None, y.data_ptr(), cout, 1,
                                1, cout, 1, 1, 0, None, 0, None, s)
        src = torch.empty(M * (cin + cout) // 2, device="cuda", dtype=dt)
        dst = torch.empty_like(src)
        f_copy = lambda: dst.copy_(src)
        t1, t2, t3 = timeit(f_stat), timeit(f_nostat), timeit(f_copy)
        byts = M * (cin + cout) * es
        print(f"M={M:8d} {cin:4d}->{cout:4d}: stat {t1:7.1f} us ({byts / t1 / 1e3:5.0f} GB/s)  nostat {t2:7.1f} us  "
              f"copy-same-bytes {t3:6.1f} us ({byts / t3 / 1e3:5.0f} GB/s)  tile_rows {rows.value}", flush=True)


if __name__ == "__main__":
    main()
