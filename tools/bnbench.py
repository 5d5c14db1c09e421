"""Isolated timing of the BatchNorm passes at the step's layer shapes: seg_bn_backward
(reduction + finalize + apply), seg_bn_stats and seg_bn_apply, bf16 and fp32 storage.
SEG_LIB_PATH selects a variant build (tools/variant.py).   python tools/bnbench.py"""
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "team02-objectdetection_amd"), REPO]
from seg_amd._lib import call, query  # noqa: E402

SHAPES = [(1048576, 96), (1048576, 32), (1048576, 16), (262144, 144), (262144, 24), (65536, 192), (16384, 384),
          (16384, 576), (4096, 1280)]
if os.environ.get("BNB_SHAPES") == "unet":  # UNet(10) at 8x512x1024 (configs[4])
    SHAPES = [(4194304, 64), (1048576, 64), (1048576, 128), (262144, 128), (262144, 256), (65536, 256),
              (65536, 512)]


def timeit(fn, reps=30):
    for _ in range(3):
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
    tot = {}
    for io, dt, suf in (("bf16", torch.bfloat16, "_bf16io"), ("f32", torch.float32, "")):
        es = 2 if io == "bf16" else 4
        for M, C in SHAPES:
            y = torch.randn(M, C, device="cuda").to(dt)
            da = torch.randn(M, C, device="cuda").to(dt)
            out = torch.empty_like(y)
            v = [torch.rand(C, device="cuda") + 0.5 for _ in range(6)]
            work = torch.zeros(query("seg_chan_workspace_floats", M, C) + 3 * C, device="cuda")
            bwd = lambda: call("seg_bn_backward" + suf, da.data_ptr(), C, y.data_ptr(), C, M, C, v[0].data_ptr(),
                               v[1].data_ptr(), v[2].data_ptr(), v[3].data_ptr(), v[4].data_ptr(), 2, v[5].data_ptr(),
                               v[5].data_ptr(), work.data_ptr(), out.data_ptr(), C, s)
            st = lambda: call("seg_bn_stats" + suf, y.data_ptr(), C, M, C, v[0].data_ptr(), v[1].data_ptr(), 1e-5,
                              0.1, None, None, None, work.data_ptr(), v[2].data_ptr(), v[3].data_ptr(),
                              v[4].data_ptr(), v[5].data_ptr(), s)
            ap = lambda: call("seg_bn_apply" + suf, y.data_ptr(), C, M, C, v[0].data_ptr(), v[1].data_ptr(), 2, None,
                              0, out.data_ptr(), C, s)
            tb, ts, ta = timeit(bwd), timeit(st), timeit(ap)
            gb = M * C * es
            tot[io] = tot.get(io, 0) + tb
            print(f"{io:4s} M={M:8d} C={C:5d}: bwd {tb:7.1f} us ({5 * gb / tb / 1e3:5.0f} GB/s)  stats {ts:6.1f} us "
                  f"({gb / ts / 1e3:5.0f} GB/s)  apply {ta:6.1f} us ({2 * gb / ta / 1e3:5.0f} GB/s)", flush=True)
    print("sum bwd:", {k: round(v, 1) for k, v in tot.items()})


if __name__ == "__main__":
    main()
