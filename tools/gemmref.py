"""Reference point for the f32 MFMA kernels: our implicit-GEMM kernel run as a
plain GEMM (1x1 conv) vs torch.mm (hipBLASLt / rocBLAS f32) on the same shapes.

    python tools/gemmref.py
"""
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "team02-objectdetection_amd"))
from seg_amd import _lib  # noqa: E402
import ctypes  # noqa: E402


def load(path):
    h = ctypes.CDLL(path)
    for name, (res, args) in _lib.PROTOTYPES.items():
        if hasattr(h, name):
            f = getattr(h, name)
            f.restype, f.argtypes = res, args
    return h

SHAPES = [(4096, 4096, 4096), (65536, 256, 1024), (16384, 256, 12096), (65536, 128, 2592), (1048576, 32, 720)]


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
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
    _lib.lib()
    libs = [(os.path.basename(p), load(p)) for p in (sys.argv[1:] or [_lib.LIB_PATH])]
    torch.backends.cuda.matmul.allow_tf32 = False
    s = torch.cuda.current_stream().cuda_stream
    for M, N, K in SHAPES:
        a = torch.randn(M, K, device="cuda")
        w = torch.randn(N, K, device="cuda")
        out = torch.empty(M, N, device="cuda")
        fl = 2.0 * M * N * K
        t_ref = timeit(lambda: torch.mm(a, w.t(), out=out))
        res = []
        for name, lib in libs:
            t = timeit(lambda: lib.seg_conv_igemm(a.data_ptr(), K, 1, M, 1, K, w.data_ptr(), K, None,
                                                  out.data_ptr(), N, M, 1, N, 1, 1, 0, None, 0, None, s))
            res.append(f"{name} {fl / t / 1e12:6.1f}")
        print(f"M={M:8d} N={N:5d} K={K:6d}: torch.mm {fl / t_ref / 1e12:6.1f} TF/s | " + " | ".join(res), flush=True)


if __name__ == "__main__":
    main()
