"""Microbenchmark of the depthwise 3x3 kernels on the MobileNetV2UNet (bs=32,
256x512) shapes: achieved GB/s of algorithmic traffic (input + output read or
written once; wgrad: dY + X) vs the ~6 TB/s achievable HBM rate.

    python tools/dwbench.py [--lazy] [--bf16io] [lib.so ...]
Several libraries can be given (A/B of kernel variants in one process).
"""
import ctypes
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "team02-objectdetection_amd"))
from seg_amd import _lib  # noqa: E402

LIB = None
SFX, DT, ES = "", torch.float32, 4  # entry-point suffix, storage dtype and bytes (--bf16io)


def load(path):
    h = ctypes.CDLL(path)
    for name, (res, args) in _lib.PROTOTYPES.items():
        if hasattr(h, name):
            f = getattr(h, name)
            f.restype, f.argtypes = res, args
    return h


def call(name, *args):
    rc = getattr(LIB, name)(*args)
    assert rc == 0, (name, rc)


def query(name, *args):
    return getattr(LIB, name)(*args)

SHAPES = [  # C, H, W (input), stride
    (32, 128, 256, 1), (96, 128, 256, 2), (144, 64, 128, 1), (144, 64, 128, 2), (192, 32, 64, 1),
    (192, 32, 64, 2), (384, 16, 32, 1), (576, 16, 32, 1), (576, 16, 32, 2), (960, 8, 16, 1)]
N = 32


def timeit(fn, reps=20):
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
    global LIB
    lazy = "--lazy" in sys.argv
    global SFX, DT, ES
    if "--bf16io" in sys.argv:
        SFX, DT, ES = "_bf16io", torch.bfloat16, 2
    paths = [a for a in sys.argv[1:] if not a.startswith("--")] or [_lib.LIB_PATH]
    _lib.lib()
    for p in paths:
        LIB = load(p)
        print("==", os.path.basename(p), "lazy" if lazy else "")
        run(lazy)


def run(lazy):
    s = torch.cuda.current_stream().cuda_stream
    tot = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0}
    for C, H, W, st in SHAPES:
        Ho, Wo = (H - 1) // st + 1, (W - 1) // st + 1
        x = torch.randn(N * H * W, C, device="cuda").to(DT)
        dy = torch.randn(N * Ho * Wo, C, device="cuda").to(DT)
        y = torch.empty(N * Ho * Wo, C, device="cuda", dtype=DT)
        dx = torch.empty(N * H * W, C, device="cuda", dtype=DT)
        wk = torch.randn(9 * C, device="cuda")
        sc, sh = torch.rand(C, device="cuda"), torch.rand(C, device="cuda")
        xf = (sc.data_ptr(), sh.data_ptr(), 2) if lazy else (None, None, 0)
        nblk = query("seg_dw_wgrad_blocks", N, Ho, Wo, C)
        part = torch.empty(nblk * 9 * C, device="cuda")
        dw = torch.empty(C * 9, device="cuda")
        bx, by = ES * N * H * W * C, ES * N * Ho * Wo * C
        tf = timeit(lambda: call("seg_dw_fwd" + SFX, x.data_ptr(), C, N, H, W, C, *xf, wk.data_ptr(), y.data_ptr(), C, Ho,
                                 Wo, st, s))
        td = timeit(lambda: call("seg_dw_dgrad" + SFX, dy.data_ptr(), C, N, Ho, Wo, C, wk.data_ptr(), dx.data_ptr(), C, H,
                                 W, st, 0, s))

        def wg():
            call("seg_dw_wgrad" + SFX, dy.data_ptr(), C, x.data_ptr(), C, N, H, W, C, *xf, Ho, Wo, st, part.data_ptr(), s)
            call("seg_conv_wgrad_reduce", part.data_ptr(), nblk, dw.data_ptr(), C, 1, 3, 1, 0, s)
        tw = timeit(wg)
        tot["fwd"] += tf
        tot["dgrad"] += td
        tot["wgrad"] += tw
        print(f"C={C:4d} {H:3d}x{W:3d} s{st}: fwd {tf * 1e6:7.1f} us {(bx + by) / tf / 1e9:6.0f} GB/s | "
              f"dgrad {td * 1e6:7.1f} us {(bx + by) / td / 1e9:6.0f} GB/s | wgrad {tw * 1e6:7.1f} us "
              f"{(bx + by) / tw / 1e9:6.0f} GB/s ({nblk} blk)")
    print("totals (ms):", {k: round(v * 1e3, 3) for k, v in tot.items()})


if __name__ == "__main__":
    main()
