"""Per-launch timing of the f32 3x3 weight gradient forms on the MobileNetV2UNet decoder (bs 32, 256x512) and
UNet 512x1024 (bs 8) shapes: the direct split-K kernel (seg_conv_wgrad), the per-point Winograd kernel
(seg_conv_wino_wgrad) and the all-points one (seg_conv_wino_wgrad16) at several split counts, each + its reduce,
HIP-event medians; TF/s are direct-conv-equivalent FLOPs.  Also checks that the two Winograd forms' slabs agree.

    python tools/ww16bench.py [unet]
"""
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "team02-objectdetection_amd"), REPO]
from seg_amd._lib import call, query  # noqa: E402

MNV2 = [("up1.0", 32, 16, 32, 1344, 256), ("up1.3", 32, 16, 32, 256, 256), ("up2.0", 32, 32, 64, 288, 128),
        ("up2.3", 32, 32, 64, 128, 128), ("up3.0", 32, 64, 128, 152, 64), ("up3.3", 32, 64, 128, 64, 64),
        ("up4.0", 32, 128, 256, 80, 32), ("up4.3", 32, 128, 256, 32, 32)]
UNET = [("inc.3", 8, 512, 1024, 64, 64), ("d1.0", 8, 256, 512, 64, 128), ("d1.3", 8, 256, 512, 128, 128),
        ("d2.0", 8, 128, 256, 128, 256), ("d2.3", 8, 128, 256, 256, 256), ("d3.0", 8, 64, 128, 256, 512),
        ("d3.3", 8, 64, 128, 512, 512), ("u1.0", 8, 128, 256, 512, 128), ("u2.0", 8, 256, 512, 256, 64),
        ("u2.3", 8, 256, 512, 64, 64), ("u3.0", 8, 512, 1024, 128, 64)]


def timeit(fn, reps=9):
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
    shapes = UNET if sys.argv[1:] == ["unet"] else MNV2
    s = torch.cuda.current_stream().cuda_stream
    for name, N, H, W, Cin, Cout in shapes:
        fl = 2.0 * N * H * W * Cin * Cout * 9
        x = torch.randn(N * H * W, Cin, device="cuda")
        dy = torch.randn(N * H * W, Cout, device="cuda")
        dw = torch.empty(Cout, Cin, 3, 3, device="cuda")
        M = N * H * W
        sp = query("seg_conv_wgrad_splits", M, Cout, Cin, 3)
        part = torch.empty(sp * Cout * 9 * Cin, device="cuda")

        def direct():
            call("seg_conv_wgrad", dy.data_ptr(), Cout, x.data_ptr(), Cin, N, H, W, Cin, H, W, Cout, 3, 1, 1,
                 part.data_ptr(), sp, s)
            call("seg_conv_wgrad_reduce", part.data_ptr(), sp, dw.data_ptr(), Cout, Cin, 3, 0, 0, s)
        t_d = timeit(direct)
        del part
        spw = query("seg_conv_wino_wgrad_splits", N, H, W, Cin, Cout)
        pw = torch.empty(spw * 16 * Cout * Cin, device="cuda")

        def wino(entry, k, buf):
            call(entry, dy.data_ptr(), Cout, x.data_ptr(), Cin, N, H, W, Cin, Cout, buf.data_ptr(), k, s)
            call("seg_conv_wino_wgrad_reduce", buf.data_ptr(), k, dw.data_ptr(), Cout, Cin, Cin, 0, s)
        call("seg_conv_wino_wgrad", dy.data_ptr(), Cout, x.data_ptr(), Cin, N, H, W, Cin, Cout, pw.data_ptr(), spw, s)
        ref = pw.clone()  # the slabs before a reduce (which folds them in place above 16 splits)
        t_w = timeit(lambda: wino("seg_conv_wino_wgrad", spw, pw))
        p16 = torch.empty_like(pw)
        call("seg_conv_wino_wgrad16", dy.data_ptr(), Cout, x.data_ptr(), Cin, N, H, W, Cin, Cout, p16.data_ptr(), spw, s)
        torch.cuda.synchronize()
        same = torch.equal(p16, ref)
        del pw, p16, ref
        line = (f"{name:6s} direct {t_d * 1e6:7.1f} us ({fl / t_d / 1e12:5.1f})  wino {t_w * 1e6:7.1f} "
                f"({fl / t_w / 1e12:5.1f}) sp {spw}  slabs-equal {same} |")
        s16 = query("seg_conv_wino_wgrad16_splits", N, H, W, Cin, Cout)
        best = None
        for k in sorted({s16, max(1, s16 // 2), 2 * s16}):
            buf = torch.empty(k * 16 * Cout * Cin, device="cuda")
            t = timeit(lambda: wino("seg_conv_wino_wgrad16", k, buf))
            del buf
            line += f" w16[{k}] {t * 1e6:7.1f}"
            if k == s16:
                best = t
        line += f"  -> default {fl / best / 1e12:5.1f} TF/s, {t_d / best:4.2f}x direct, {t_w / best:4.2f}x wino"
        print(line, flush=True)


if __name__ == "__main__":
    main()
