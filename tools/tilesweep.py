"""Time every seg_conv_igemm tile configuration on every igemm launch shape of
a model's training step (forward and data gradient), to tune the cost model.

    python tools/tilesweep.py [--model MobileNetV2UNet] [--batch 32]
Prints per shape: the cost model's tile, the fastest tile, and both times.
"""
import argparse
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "team02-objectdetection_amd"), REPO]
import seg_amd  # noqa: E402
from seg_amd import engine as E  # noqa: E402
from seg_amd._lib import call, query, lib  # noqa: E402

TILES = ["128x128", "64x128", "128x64", "64x64", "128x96", "128x160", "256x32", "128x32",
         "8w128x128a", "8w128x128b", "8w256x128", "8w128x256", "8w128x64", "8w256x64", "8w64x128"]


def timeit(fn, reps=8):
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


def shapes(model, N, H, W):
    prog = E.build_program(model, N, H, W)
    out = []
    for op in prog.ops:
        if not isinstance(op, E.ConvOp) or op.kind != "igemm":
            continue
        i, y = op.inp, op.y
        out.append(("fwd", i.N, i.H, i.W, op.cin_pad, y.H, y.W, op.cout, op.ks, op.stride, op.pad))
        if not op.first:
            out.append(("dgrad", y.N, y.H, y.W, E.r4(op.cout), i.H, i.W, op.cin, op.ks, 1, op.pad))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="MobileNetV2UNet")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--height", type=int, default=256)
    ap.add_argument("--width", type=int, default=512)
    ap.add_argument("--math", choices=("f32", "bf16", "bf16io"), default="f32")
    a = ap.parse_args()
    lib()
    model = getattr(seg_amd, a.model)(10)
    s = torch.cuda.current_stream().cuda_stream
    seen, tot_auto, tot_best = set(), 0.0, 0.0
    for kind, N, H, W, Cin, Ho, Wo, Cout, ks, st, pad in shapes(model, a.batch, a.height, a.width):
        key = (N, H, W, Cin, Ho, Wo, Cout, ks, st)
        if key in seen:
            continue
        seen.add(key)
        io = a.math == "bf16io"
        if io and Cin % 8:
            continue  # (the image: the bf16io engine runs it on the 4-channel path)
        dt = torch.bfloat16 if io else torch.float32
        x = torch.randn(N * H * W, Cin, device="cuda").to(dt)
        ldk = E.r8(ks * ks * Cin) if io else E.r4(ks * ks * Cin)
        wk = (torch.randn(Cout * ldk, device="cuda") * 0.05).to(dt)  # bf16io: the bf16-packed weights
        y = torch.empty(N * Ho * Wo, E.r4(Cout), device="cuda", dtype=dt)

        def run():
            if io:
                call("seg_conv_igemm_bf16io_w16", x.data_ptr(), Cin, N, H, W, Cin, wk.data_ptr(), ldk, None,
                     y.data_ptr(), E.r4(Cout), Ho, Wo, Cout, ks, st, pad, None, 0, None, s)
            elif a.math == "bf16":
                call("seg_conv_igemm_bf16", x.data_ptr(), Cin, N, H, W, Cin, wk.data_ptr(), ldk, None, y.data_ptr(),
                     E.r4(Cout), Ho, Wo, Cout, ks, st, pad, None, 0, None, 0, None, 1, s)
            else:
                call("seg_conv_igemm", x.data_ptr(), Cin, N, H, W, Cin, wk.data_ptr(), ldk, None, y.data_ptr(),
                     E.r4(Cout), Ho, Wo, Cout, ks, st, pad, None, 0, None, s)
        times = []
        for t in range(len(TILES)):
            E.force_tiles(igemm=t)
            times.append(timeit(run))
        E.force_tiles(igemm=-1)
        auto_rows = query("seg_conv_igemm_row_tiles", N * Ho * Wo, Cout, None)
        t_auto = timeit(run)  # measured last: the first timings of a shape run slow
        best = min(range(len(TILES)), key=lambda t: times[t])
        fl = 2.0 * N * Ho * Wo * Cout * Cin * ks * ks
        tot_auto += t_auto
        tot_best += times[best]
        print(f"{kind:5s} M={N * Ho * Wo:8d} N={Cout:5d} K={ks * ks * Cin:6d}: auto {t_auto * 1e6:8.1f} us "
              f"({fl / t_auto / 1e12:5.1f} TF/s, {auto_rows} row tiles) | best {TILES[best]:8s} "
              f"{times[best] * 1e6:8.1f} us ({fl / times[best] / 1e12:5.1f}) | "
              + " ".join(f"{t * 1e6:.0f}" for t in times), flush=True)
    print(f"total auto {tot_auto * 1e3:.3f} ms, best {tot_best * 1e3:.3f} ms")


if __name__ == "__main__":
    main()
