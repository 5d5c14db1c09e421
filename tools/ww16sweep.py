"""seg_conv_wino_wgrad16 split sweep: kernel alone and reduce alone per split count (HIP-event medians), on the
MobileNetV2UNet decoder shapes (bs 32) or UNet 512x1024 (unet).

    python tools/ww16sweep.py [unet]
"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "team02-objectdetection_amd"), REPO, os.path.join(REPO, "tools")]
from seg_amd._lib import call, query  # noqa: E402
from ww16bench import MNV2, UNET, timeit  # noqa: E402


def main():
    shapes = UNET if sys.argv[1:] == ["unet"] else MNV2
    s = torch.cuda.current_stream().cuda_stream
    for name, N, H, W, Cin, Cout in shapes:
        fl = 2.0 * N * H * W * Cin * Cout * 9
        x = torch.randn(N * H * W, Cin, device="cuda")
        dy = torch.randn(N * H * W, Cout, device="cuda")
        dw = torch.empty(Cout, Cin, 3, 3, device="cuda")
        T = N * (H // 2) * (W // 2)
        d = query("seg_conv_wino_wgrad16_splits", N, H, W, Cin, Cout)
        line = f"{name:6s} default {d:4d}:"
        for k in (4, 8, 16, 32, 64, 128, 256, 512):
            if k > T // 64:
                break
            buf = torch.empty(k * 16 * Cout * Cin, device="cuda")
            tk = timeit(lambda: call("seg_conv_wino_wgrad16", dy.data_ptr(), Cout, x.data_ptr(), Cin, N, H, W, Cin,
                                     Cout, buf.data_ptr(), k, s))
            tr = timeit(lambda: call("seg_conv_wino_wgrad_reduce", buf.data_ptr(), k, dw.data_ptr(), Cout, Cin, Cin,
                                     0, s))
            del buf
            line += f"  [{k}] {tk * 1e6:6.1f}+{tr * 1e6:5.1f} ({fl / tk / 1e12:5.1f})"
        print(line, flush=True)


if __name__ == "__main__":
    main()
