"""seg_mbconv_f16 per launch for every InvertedResidual of a 128x256 frame (configs[3]) over the
split planner's block target (seg_mbconv_tune).   python tools/mbbench.py"""
import ctypes
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "team02-objectdetection_amd"), REPO]
from seg_amd._lib import call, query  # noqa: E402

BLOCKS = [  # H, W, Cin, t, Cout, stride  (features[1..17])
    (64, 128, 32, 1, 16, 1), (64, 128, 16, 6, 24, 2), (32, 64, 24, 6, 24, 1), (32, 64, 24, 6, 32, 2),
    (16, 32, 32, 6, 32, 1), (16, 32, 32, 6, 32, 1), (16, 32, 32, 6, 64, 2), (8, 16, 64, 6, 64, 1),
    (8, 16, 64, 6, 64, 1), (8, 16, 64, 6, 64, 1), (8, 16, 64, 6, 96, 1), (8, 16, 96, 6, 96, 1),
    (8, 16, 96, 6, 96, 1), (8, 16, 96, 6, 160, 2), (4, 8, 160, 6, 160, 1), (4, 8, 160, 6, 160, 1),
    (4, 8, 160, 6, 320, 1)]
CAPS = [128, 256, 384, 512, 768, 1024]


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
    tot = {c: 0.0 for c in CAPS}
    for H, W, Cin, t, Cout, st in BLOCKS:
        Ch = Cin * t
        x = torch.randn(H * W, Cin, device="cuda")
        we = torch.randn(Ch, Cin, device="cuda") / Cin ** 0.5 if t != 1 else None
        be = torch.randn(Ch, device="cuda") * 0.1 if t != 1 else None
        wd = torch.randn(9 * Ch, device="cuda") / 3
        bd = torch.randn(Ch, device="cuda") * 0.1
        wp = torch.randn(Cout, Ch, device="cuda") / Ch ** 0.5
        bp = torch.randn(Cout, device="cuda") * 0.1
        Ho, Wo = (H - 1) // st + 1, (W - 1) // st + 1
        res = torch.randn(Ho * Wo, Cout, device="cuda") if (st == 1 and Cin == Cout) else None
        out = torch.empty(Ho * Wo, Cout, device="cuda")
        row = []
        for cap in CAPS:
            query("seg_mbconv_tune", cap)
            ncnt = ctypes.c_int(0)
            nw = query("seg_mbconv_work_floats", 1, H, W, Ch, Cout, st, ctypes.addressof(ncnt))
            work = torch.empty(max(nw, 1), device="cuda")
            cnt = torch.zeros(max(ncnt.value, 1), device="cuda", dtype=torch.int32)

            def f():
                call("seg_mbconv_f16", x.data_ptr(), Cin, 1, H, W, Cin, we.data_ptr() if we is not None else None,
                     be.data_ptr() if be is not None else None, Ch, wd.data_ptr(), bd.data_ptr(), st, wp.data_ptr(),
                     bp.data_ptr(), Cout, res.data_ptr() if res is not None else None, Cout if res is not None else 0,
                     out.data_ptr(), Cout, work.data_ptr(), cnt.data_ptr(), s)
            v = timeit(f)
            tot[cap] += v
            row.append(f"cap{cap}:{v:.1f}(w{nw // max(Ho * Wo * Cout, 1)})")
        print(f"{H}x{W} {Cin}->{Ch}->{Cout} s{st}: " + " ".join(row), flush=True)
    query("seg_mbconv_tune", 256)
    print("sum:", {c: round(v, 1) for c, v in tot.items()})


if __name__ == "__main__":
    main()
