"""Two-stream contention microbenchmark: a main-stream BatchNorm backward of a small layer
launched while a side-stream weight gradient of a deep layer runs, timed with HIP events on both streams, for
side grids of various sizes and stream priorities.

    python tools/contend.py
"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "team02-objectdetection_amd"), REPO]
from seg_amd._lib import call, query  # noqa: E402

BF = torch.bfloat16


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    g = torch.Generator(device="cpu").manual_seed(0)
    # side: the deep decoder conv's weight gradient (up1.0: 3x3, 1344 -> 256, 16x32 at bs 32 = 16384 rows)
    N, H, W, Cin, Cout = 32, 16, 32, 1344, 256
    M = N * H * W
    dy = torch.randn(M, Cout, generator=g).to(BF).to(dev)
    x = torch.randn(M, Cin, generator=g).to(BF).to(dev)
    # main: a 16k-row, 384-channel BN backward (three launches: reduction, finalize, apply)
    Mb, C = 16384, 384
    da = torch.randn(Mb, C, generator=g).to(BF).to(dev)
    yb = torch.randn(Mb, C, generator=g).to(BF).to(dev)
    st = [torch.rand(C, generator=g).to(dev) + 0.5 for _ in range(4)]
    gw, gb = torch.empty(C, device=dev), torch.empty(C, device=dev)
    work = torch.empty(query("seg_chan_workspace_floats", Mb, C) + 3 * C, device=dev)
    dyb = torch.empty(Mb, C, device=dev, dtype=BF)

    def bn(s):
        call("seg_bn_backward_bf16io", da.data_ptr(), C, yb.data_ptr(), C, Mb, C, st[0].data_ptr(), st[1].data_ptr(),
             st[2].data_ptr(), st[3].data_ptr(), st[0].data_ptr(), 2, gw.data_ptr(), gb.data_ptr(), work.data_ptr(),
             dyb.data_ptr(), C, s)

    base_splits = query("seg_conv_wgrad_splits_bf16", M, Cout, Cin, 3)
    print(f"side: wgrad 3x3 {Cin}->{Cout} M={M} (plan splits {base_splits}); main: BN backward {Mb}x{C}")
    for prio_main, prio_side in ((0, 0), (-1, 0)):
        sm = torch.cuda.Stream(dev, priority=prio_main)
        ss = torch.cuda.Stream(dev, priority=prio_side)
        for splits in (base_splits, max(base_splits // 2, 1), max(base_splits // 4, 1), 1):
            part = torch.empty(splits * Cout * 9 * Cin, device=dev)

            def wg(s):
                call("seg_conv_wgrad_bf16io", dy.data_ptr(), Cout, x.data_ptr(), Cin, N, H, W, Cin, H, W, Cout, 3, 1,
                     1, part.data_ptr(), splits, s)
            res = {}
            for mode in ("alone_bn", "alone_wg", "both"):
                tb, tw = [], []
                for rep in range(12):
                    e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
                    torch.cuda.synchronize()
                    if mode != "alone_bn":
                        e[2].record(ss)
                        wg(ss.cuda_stream)
                        e[3].record(ss)
                    if mode == "both":
                        with torch.cuda.stream(sm):
                            torch.cuda._sleep(40000)  # ~20 us: the weight gradient occupies the chip first
                    if mode != "alone_wg":
                        e[0].record(sm)
                        bn(sm.cuda_stream)
                        e[1].record(sm)
                    torch.cuda.synchronize()
                    if rep >= 2:
                        if mode != "alone_wg":
                            tb.append(e[0].elapsed_time(e[1]) * 1e3)
                        if mode != "alone_bn":
                            tw.append(e[2].elapsed_time(e[3]) * 1e3)
                res[mode] = (sorted(tb)[len(tb) // 2] if tb else 0.0, sorted(tw)[len(tw) // 2] if tw else 0.0)
            print(f"prio main {prio_main:2d} side {prio_side:2d}  splits {splits:4d}: BN alone {res['alone_bn'][0]:7.1f} us, "
                  f"wgrad alone {res['alone_wg'][1]:7.1f} us | together: BN {res['both'][0]:7.1f} us, "
                  f"wgrad {res['both'][1]:7.1f} us", flush=True)


if __name__ == "__main__":
    main()
