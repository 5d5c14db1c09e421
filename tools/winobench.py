"""Winograd F(2x2,3x3) (seg_conv_wino, and seg_conv_wino_fused) against the direct implicit GEMM
(seg_conv_igemm) on the MobileNetV2UNet / UNet decoder shapes, forward and data
gradient, HIP-event medians.  TF/s are direct-conv-equivalent FLOPs.

    python tools/winobench.py
"""
import os
import statistics
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "team02-objectdetection_amd"), REPO]
from seg_amd._lib import call, query  # noqa: E402

SHAPES = [("up1.0", 32, 16, 32, 1344, 256), ("up1.3", 32, 16, 32, 256, 256), ("up2.0", 32, 32, 64, 288, 128),
          ("up2.3", 32, 32, 64, 128, 128), ("up3.0", 32, 64, 128, 152, 64), ("up3.3", 32, 64, 128, 64, 64),
          ("up4.0", 32, 128, 256, 80, 32), ("up4.3", 32, 128, 256, 32, 32)]


SHAPES_UNET = [("u.d1a", 8, 256, 512, 64, 128), ("u.d1b", 8, 256, 512, 128, 128), ("u.d2b", 8, 128, 256, 128, 256), ("u.d2c", 8, 128, 256, 256, 256), ("u.d3", 8, 64, 128, 256, 256),
               ("u.up1a", 8, 128, 256, 512, 128), ("u.up1b", 8, 128, 256, 128, 128),
               ("u.up2a", 8, 256, 512, 256, 64), ("u.up2b", 8, 256, 512, 64, 64)]
if os.environ.get("WINOBENCH") == "unet":
    SHAPES = SHAPES_UNET


def timeit(fn, reps=10):
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


def pack(w, mode, rows, ldk, kin):
    from seg_amd.engine import pack_table
    n = (16 if mode >= 3 else 1) * rows * ldk
    wk = torch.empty(n, device="cuda")
    jobs, nj, nb = pack_table([(w.data_ptr(), wk.data_ptr(), w.shape[0], w.shape[1], 3, ldk, mode, kin)], "cuda")
    call("seg_pack_batch", jobs.data_ptr(), nj, nb, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return wk


def main():
    s = torch.cuda.current_stream().cuda_stream
    for name, N, H, W, Cin, Cout in SHAPES:
        fl = 2.0 * N * H * W * Cin * Cout * 9
        for d, (ci, co) in (("fwd", (Cin, Cout)), ("dgrad", (Cout, Cin))):
            x = torch.randn(N * H * W, ci, device="cuda")
            w = torch.randn(co, ci, 3, 3, device="cuda") * 0.05
            y = torch.empty(N * H * W, co, device="cuda")
            ldk = ((9 * ci + 3) // 4) * 4
            wk = pack(w, 0, co, ldk, ci)
            t_d = timeit(lambda: call("seg_conv_igemm", x.data_ptr(), ci, N, H, W, ci, wk.data_ptr(), ldk, None,
                                      y.data_ptr(), co, H, W, co, 3, 1, 1, None, 0, None, s))
            U = pack(w, 3, co, ci, ci)
            work = torch.empty(16 * N * (H // 2) * (W // 2) * co, device="cuda")
            t_w = timeit(lambda: call("seg_conv_wino", x.data_ptr(), ci, N, H, W, ci, U.data_ptr(), ci, None,
                                      y.data_ptr(), co, co, None, 0, None, work.data_ptr(), s))
            t_f = timeit(lambda: call("seg_conv_wino_fused", x.data_ptr(), ci, N, H, W, ci, U.data_ptr(), ci, None,
                                      y.data_ptr(), co, co, None, 0, None, s))
            pick = query("seg_conv_wino_pick", N, H, W, ci, co)
            if query("seg_conv_halo_ok", N, H, W, ci, co):
                t_h = timeit(lambda: call("seg_conv_halo", x.data_ptr(), ci, N, H, W, ci, wk.data_ptr(), ldk, None,
                                          y.data_ptr(), co, co, None, 0, None, s))
                print(f"{name:6s} {d:5s} halo {t_h * 1e6:7.1f} us ({fl / t_h / 1e12:5.1f} TF/s) vs direct "
                      f"{t_d * 1e6:7.1f}: speedup {t_d / t_h:4.2f}", flush=True)
            print(f"{name:6s} {d:5s} direct {t_d * 1e6:7.1f} us ({fl / t_d / 1e12:5.1f} TF/s)  wino {t_w * 1e6:7.1f} us "
                  f"({fl / t_w / 1e12:5.1f})  speedup {t_d / t_w:4.2f}  fused {t_f * 1e6:7.1f} us "
                  f"({fl / t_f / 1e12:5.1f})  speedup {t_d / t_f:4.2f}  pick={pick}", flush=True)
        # weight gradient: direct split-K wgrad + reduce vs Winograd wgrad + reduce
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
        spw = query("seg_conv_wino_wgrad_splits", N, H, W, Cin, Cout)
        pw = torch.empty(spw * 16 * Cout * Cin, device="cuda")

        def wino():
            call("seg_conv_wino_wgrad", dy.data_ptr(), Cout, x.data_ptr(), Cin, N, H, W, Cin, Cout, pw.data_ptr(),
                 spw, s)
            call("seg_conv_wino_wgrad_reduce", pw.data_ptr(), spw, dw.data_ptr(), Cout, Cin, Cin, 0, s)
        t_d, t_w = timeit(direct), timeit(wino)
        print(f"{name:6s} wgrad direct {t_d * 1e6:7.1f} us ({fl / t_d / 1e12:5.1f} TF/s)  wino {t_w * 1e6:7.1f} us "
              f"({fl / t_w / 1e12:5.1f})  speedup {t_d / t_w:4.2f}  splits {sp}/{spw}", flush=True)


if __name__ == "__main__":
    main()
