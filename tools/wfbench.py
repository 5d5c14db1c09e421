"""seg_conv_wino_fused per-launch timing on the decoder shapes (HIP-event medians); with SEG_LIB_PATH, a variant
library built by tools/variant.py (e.g. -DSEG_WF_EXP=1: timing experiments of csrc/wino.hip).

    python tools/wfbench.py [label]
"""
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "team02-objectdetection_amd"), REPO]
from seg_amd._lib import call  # noqa: E402

SHAPES = [("up1.0", 32, 16, 32, 1344, 256), ("up2.0", 32, 32, 64, 288, 128), ("up3.0", 32, 64, 128, 152, 64),
          ("up4.0", 32, 128, 256, 80, 32), ("up4.3", 32, 128, 256, 32, 32)]


def main():
    label = sys.argv[1] if len(sys.argv) > 1 else "base"
    s = torch.cuda.current_stream().cuda_stream
    for name, N, H, W, ci, co in SHAPES:
        x = torch.randn(N * H * W, ci, device="cuda")
        U = torch.randn(16 * co * ci, device="cuda") * 0.05
        y = torch.empty(N * H * W, co, device="cuda")

        def f():
            call("seg_conv_wino_fused", x.data_ptr(), ci, N, H, W, ci, U.data_ptr(), ci, None, y.data_ptr(), co, co,
                 None, 0, None, s)
        f()
        ts = []
        for _ in range(10):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            f()
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b) * 1e3)
        t = statistics.median(ts)
        macs = N * (H // 2) * (W // 2) * co * 16 * ci
        print(f"{label:8s} {name:6s} fused {t:8.1f} us  executed MFMA {2 * macs / t / 1e6:6.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
