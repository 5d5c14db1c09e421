"""Microbenchmark of the MFMA convolution kernels on the MobileNetV2UNet (bs=32,
256x512) dense-3x3 and largest 1x1 shapes: forward, data-gradient and
weight-gradient, timed with HIP events (median of R launches), in TFLOP/s.

    python tools/convbench.py [path/to/libsegamd.so ...]
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

SHAPES = [  # name, N, H, W (output = input spatial), Cin, Cout, ks
    ("stem", 32, 128, 256, 4, 32, 3),  # output spatial; stride 2 handled below
    ("up1.0", 32, 16, 32, 1344, 256, 3), ("up1.3", 32, 16, 32, 256, 256, 3),
    ("up2.0", 32, 32, 64, 288, 128, 3), ("up2.3", 32, 32, 64, 128, 128, 3),
    ("up3.0", 32, 64, 128, 152, 64, 3), ("up3.3", 32, 64, 128, 64, 64, 3),
    ("up4.0", 32, 128, 256, 80, 32, 3), ("up4.3", 32, 128, 256, 32, 32, 3),
    ("f2.exp", 32, 128, 256, 16, 96, 1), ("f18", 32, 8, 16, 320, 1280, 1),
]


def r4(c):
    return (c + 3) & ~3


def load(path):
    h = ctypes.CDLL(path)
    for name, (res, args) in _lib.PROTOTYPES.items():
        if hasattr(h, name):
            f = getattr(h, name)
            f.restype, f.argtypes = res, args
    return h


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


def bench(lib, only=None):
    s = torch.cuda.current_stream().cuda_stream
    out = {}
    for name, N, H, W, Cin, Cout, ks in SHAPES:
        if only and name not in only:
            continue
        stride = 2 if name == "stem" else 1
        pad = ks // 2
        Hi, Wi = H * stride, W * stride
        Ho, Wo = H, W
        M = N * Ho * Wo
        flops = 2.0 * M * Cout * Cin * ks * ks
        x = torch.randn(N * Hi * Wi, r4(Cin), device="cuda")
        w = torch.randn(Cout, Cin, ks, ks, device="cuda") * 0.05
        dy = torch.randn(M, r4(Cout), device="cuda")
        ldk = r4(ks * ks * Cin)
        wk = torch.empty(Cout * ldk, device="cuda")
        lib.seg_pack_conv_weight(w.data_ptr(), wk.data_ptr(), Cout, Cin, ks, ldk, 0, Cin, s)
        y = torch.empty(M, r4(Cout), device="cuda")
        t_f = timeit(lambda: lib.seg_conv_igemm(x.data_ptr(), r4(Cin), N, Hi, Wi, Cin, wk.data_ptr(), ldk, None,
                                                y.data_ptr(), r4(Cout), Ho, Wo, Cout, ks, stride, pad, None, 0, None, s))
        res = {"fwd": flops / t_f / 1e12}
        if stride == 1:
            kin = r4(Cout)
            ldk2 = r4(ks * ks * kin)
            wkd = torch.empty(Cin * ldk2, device="cuda")
            lib.seg_pack_conv_weight(w.data_ptr(), wkd.data_ptr(), Cout, Cin, ks, ldk2, 1, kin, s)
            dx = torch.empty(N * H * W, r4(Cin), device="cuda")
            t_d = timeit(lambda: lib.seg_conv_igemm(dy.data_ptr(), r4(Cout), N, H, W, kin, wkd.data_ptr(), ldk2,
                                                    None, dx.data_ptr(), r4(Cin), H, W, Cin, ks, 1, pad, None, 0, None, s))
            res["dgrad"] = flops / t_d / 1e12
        splits = lib.seg_conv_wgrad_splits(M, Cout, Cin, ks)
        part = torch.empty(splits * Cout * ks * ks * r4(Cin), device="cuda")
        dw = torch.empty(Cout, Cin, ks, ks, device="cuda")

        def wg():
            lib.seg_conv_wgrad(dy.data_ptr(), r4(Cout), x.data_ptr(), r4(Cin), N, Hi, Wi, Cin, Ho, Wo, Cout, ks,
                               stride, pad, part.data_ptr(), splits, s)
            lib.seg_conv_wgrad_reduce(part.data_ptr(), splits, dw.data_ptr(), Cout, Cin, ks, 0, 0, s)
        t_w = timeit(wg)
        res["wgrad"] = flops / t_w / 1e12
        res["ms"] = (t_f + t_w + (t_d if stride == 1 else 0)) * 1e3
        out[name] = res
    return out


def main():
    paths = sys.argv[1:] or [os.path.join(REPO, "team02-objectdetection_amd/seg_amd/_lib/libsegamd.so")]
    import seg_amd._lib  # noqa: F401  (torch first)
    libs = [(p, load(p)) for p in paths]
    only = os.environ.get("CONVBENCH_ONLY")
    only = set(only.split(",")) if only else None
    results = [(p, bench(lib, only)) for p, lib in libs]
    for p, res in results:
        print("==", p)
        tot = 0.0
        for name, r in res.items():
            tot += r["ms"]
            print(f"  {name:7s} fwd {r['fwd']:6.1f}  dgrad {r.get('dgrad', 0):6.1f}  wgrad {r['wgrad']:6.1f} TF/s"
                  f"   {r['ms']:.3f} ms")
        print(f"  total {tot:.3f} ms")


if __name__ == "__main__":
    main()
