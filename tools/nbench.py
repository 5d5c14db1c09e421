"""Microbenchmark of the round-4 bf16io kernels against the ones they replace, at the
MobileNetV2UNet (bs=32, 256x512) launch shapes, median of R launches timed with HIP events
(same stream, back to back), with the algorithmic bytes / FLOPs of each launch:

  * narrow 3x3 convs (up3 / up4 and their data gradients): seg_conv_halo2_bf16io vs
    seg_conv_halo_bf16io_w16 vs seg_conv_igemm_bf16io_w16;
  * depthwise convs (forward with lazy BN + tile statistics, data gradient, weight gradient):
    seg_dw2_*_bf16io vs dwconv.hip's seg_dw_*_bf16io;
  * small-image 1x1 convs of the encoder: seg_conv_igemm2_bf16io (4-wave tiles; _xf for the
    lazy-BN project convs) vs seg_conv_igemm_bf16io_w16 (_xf_w16).

    python tools/nbench.py [--reps 30] [--only halo|pw|dw] [--csv out.csv]
"""
import argparse
import ctypes
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "team02-objectdetection_amd"), REPO]
from seg_amd import engine  # noqa: E402
from seg_amd._lib import call, query  # noqa: E402

BF = torch.bfloat16
HALO = [  # name, N, H, W, Cin, Cout (3x3 stride 1 as launched: dgrads as convs of dY)
    ("up4.0f", 32, 128, 256, 80, 32), ("up4.0d", 32, 128, 256, 32, 80), ("up4.3", 32, 128, 256, 32, 32),
    ("up3.0f", 32, 64, 128, 152, 64), ("up3.0d", 32, 64, 128, 64, 152), ("up3.3", 32, 64, 128, 64, 64),
    ("unet.inc3", 8, 512, 1024, 64, 64),
]
PW = [  # name, M, Cin, Cout, xf (lazy BN on the input: the project convs)
    ("16k 64->384", 16384, 64, 384, False), ("16k 384->64 xf", 16384, 384, 64, True),
    ("16k 96->576", 16384, 96, 576, False), ("16k 576->96 xf", 16384, 576, 96, True),
    ("16k 576->96 dg", 16384, 576, 96, False), ("4k 160->960", 4096, 160, 960, False),
    ("4k 960->160 xf", 4096, 960, 160, True), ("4k 960->160 dg", 4096, 960, 160, False),
    ("4k 960->320 xf", 4096, 960, 320, True), ("4k 320->1280", 4096, 320, 1280, False),
    ("4k 1280->320 dg", 4096, 1280, 320, False), ("65k 32->192", 65536, 32, 192, False),
    ("65k 192->32 xf", 65536, 192, 32, True), ("65k 144->32 dg", 65536, 144, 32, False),
]
DW = [  # name, N, H, W (input), C, stride -- MobileNetV2 features.1-17's depthwise convs
    ("f1 32 128x256", 32, 128, 256, 32, 1), ("f2 96 s2", 32, 128, 256, 96, 2), ("f3 144 64x128", 32, 64, 128, 144, 1),
    ("f4 144 s2", 32, 64, 128, 144, 2), ("f5 192 32x64", 32, 32, 64, 192, 1), ("f7 192 s2", 32, 32, 64, 192, 2),
    ("f8 384 16x32", 32, 16, 32, 384, 1), ("f12 576 16x32", 32, 16, 32, 576, 1), ("f14 576 s2", 32, 16, 32, 576, 2),
    ("f15 960 8x16", 32, 8, 16, 960, 1),
]


def S():
    return torch.cuda.current_stream().cuda_stream


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return statistics.median(a.elapsed_time(b) * 1e-3 for a, b in ev)


def pack16(w, Cout, Cin, ks):
    ldk = (ks * ks * Cin + 7) & ~7
    wk = torch.empty(Cout * ldk, device="cuda", dtype=BF)
    table, n, blocks = engine.pack_table([(w.data_ptr(), wk.data_ptr(), Cout, Cin, ks, ldk, 16, Cin)], w.device)
    call("seg_pack_batch", table.data_ptr(), n, blocks, S())
    return wk, ldk


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--only", default="")
    ap.add_argument("--csv", default=None)
    ap.add_argument("--ig2-tune", default="", help="target_blocks,min_steps of the igemm2 4-wave split-K")
    a = ap.parse_args()
    if a.ig2_tune:
        t, m = (int(v) for v in a.ig2_tune.split(","))
        query("seg_igemm2_tune", t, m)
    g = torch.Generator().manual_seed(0)
    rows = []
    if a.only in ("", "halo"):
        for name, N, H, W, Cin, Cout in HALO:
            M = N * H * W
            x = torch.randn(M, Cin, generator=g).to(BF).cuda()
            w = (torch.randn(Cout, Cin, 3, 3, generator=g) * 0.05).cuda()
            wk, ldk = pack16(w, Cout, Cin, 3)
            out = torch.empty(M, Cout, device="cuda", dtype=BF)
            nt = query("seg_conv_halo_row_tiles", N, H, W)
            st = torch.empty(nt * 2 * Cout, device="cuda")
            nbytes = 2 * M * (Cin + Cout)
            flops = 2 * M * Cout * Cin * 9
            res = {}
            if query("seg_conv_halo2_ok", N, H, W, Cin, Cout):
                res["halo2"] = timeit(lambda: call("seg_conv_halo2_bf16io", x.data_ptr(), Cin, N, H, W, Cin,
                                                   wk.data_ptr(), ldk, None, out.data_ptr(), Cout, Cout, None, 0,
                                                   st.data_ptr(), S()), a.reps)
            if query("seg_conv_halo_ok", N, H, W, Cin, Cout):
                res["halo"] = timeit(lambda: call("seg_conv_halo_bf16io_w16", x.data_ptr(), Cin, N, H, W, Cin,
                                                  wk.data_ptr(), ldk, None, out.data_ptr(), Cout, Cout, None, 0,
                                                  st.data_ptr(), S()), a.reps)
            ntg = query("seg_conv_igemm_row_tiles", M, Cout, None)
            stg = torch.empty(ntg * 2 * Cout, device="cuda")
            res["igemm"] = timeit(lambda: call("seg_conv_igemm_bf16io_w16", x.data_ptr(), Cin, N, H, W, Cin,
                                               wk.data_ptr(), ldk, None, out.data_ptr(), Cout, H, W, Cout, 3, 1, 1,
                                               None, 0, stg.data_ptr(), S()), a.reps)
            line = "  ".join(f"{k} {v * 1e6:7.1f} us {nbytes / v / 1e9:6.0f} GB/s {flops / v / 1e12:5.0f} TF"
                             for k, v in res.items())
            print(f"{name:10s} {line}", flush=True)
            rows += [(name, k, v * 1e6, nbytes / v / 1e9) for k, v in res.items()]
    if a.only in ("", "pw"):
        for name, M, Cin, Cout, xf in PW:
            x = (torch.randn(M, Cin, generator=g) * 0.5).to(BF).cuda()
            w = (torch.randn(Cout, Cin, 1, 1, generator=g) * 0.05).cuda()
            wk, ldk = pack16(w, Cout, Cin, 1)
            out = torch.empty(M, Cout, device="cuda", dtype=BF)
            sc = (torch.rand(Cin, generator=g) + 0.5).cuda()
            sh = torch.randn(Cin, generator=g).cuda()
            nbytes = 2 * M * (Cin + Cout)
            pl = (ctypes.c_long * 4)()
            res = {}
            if query("seg_conv_igemm2_plan", M, Cout, Cin, 1, ctypes.addressof(pl)):
                tr, ntl, sp, wf = list(pl)
                work = torch.zeros(max(wf, 1), device="cuda")
                st = torch.empty(ntl * 2 * Cout, device="cuda")
                xa = (sc.data_ptr(), sh.data_ptr(), 2) if xf else ()
                nm = "seg_conv_igemm2_bf16io" + ("_xf" if xf else "")
                res[f"ig2(s{sp},r{tr})"] = timeit(lambda: call(nm, x.data_ptr(), Cin, 1, 1, M, Cin, wk.data_ptr(), ldk,
                                                               None, out.data_ptr(), Cout, Cout, 1, None, 0,
                                                               st.data_ptr(), work.data_ptr(), *xa, S()), a.reps)
            ntg = query("seg_conv_igemm_row_tiles", M, Cout, None)
            stg = torch.empty(ntg * 2 * Cout, device="cuda")
            nm = "seg_conv_igemm_bf16io_xf_w16" if xf else "seg_conv_igemm_bf16io_w16"
            xa = (sc.data_ptr(), sh.data_ptr(), 2) if xf else ()
            res["igemm"] = timeit(lambda: call(nm, x.data_ptr(), Cin, 1, 1, M, Cin, wk.data_ptr(), ldk, None,
                                               out.data_ptr(), Cout, 1, M, Cout, 1, 1, 0, None, 0, stg.data_ptr(), *xa,
                                               S()), a.reps)
            line = "  ".join(f"{k} {v * 1e6:7.1f} us {nbytes / v / 1e9:6.0f} GB/s" for k, v in res.items())
            print(f"{name:16s} {line}", flush=True)
            rows += [(name, k, v * 1e6, nbytes / v / 1e9) for k, v in res.items()]
    if a.only in ("", "dw"):
        for name, N, H, W, C, s in DW:
            Ho, Wo = (H - 1) // s + 1, (W - 1) // s + 1
            x = torch.randn(N * H * W, C, generator=g).to(BF).cuda()
            dy = torch.randn(N * Ho * Wo, C, generator=g).to(BF).cuda()
            w = (torch.randn(C, 1, 3, 3, generator=g) * 0.3).cuda()
            wk = torch.empty(9 * C, device="cuda")
            call("seg_pack_dw_weight", w.data_ptr(), wk.data_ptr(), C, S())
            sc = (torch.rand(C, generator=g) + 0.5).cuda()
            sh = torch.randn(C, generator=g).cuda()
            o = torch.empty(N * Ho * Wo, C, device="cuda", dtype=BF)
            dx = torch.empty(N * H * W, C, device="cuda", dtype=BF)
            nbytes = 2 * C * (N * H * W + N * Ho * Wo)
            nt = query("seg_dw2_stat_tiles", N, Ho, Wo, s, None)
            st = torch.empty(max(nt, 1) * 2 * C, device="cuda")
            stp = st.data_ptr() if nt else None
            nb2 = query("seg_dw2_wgrad_blocks", N, Ho, Wo, C, s, 0)
            p2 = torch.empty(nb2 * 9 * C, device="cuda")
            nb1 = query("seg_dw_wgrad_blocks", N, Ho, Wo, C)
            p1 = torch.empty(nb1 * 9 * C, device="cuda")
            res = {
                "fwd2": timeit(lambda: call("seg_dw2_fwd_bf16io", x.data_ptr(), C, N, H, W, C, sc.data_ptr(),
                                            sh.data_ptr(), 2, wk.data_ptr(), o.data_ptr(), C, Ho, Wo, s, stp, S()), a.reps),
                "fwd1": timeit(lambda: call("seg_dw_fwd_bf16io", x.data_ptr(), C, N, H, W, C, sc.data_ptr(),
                                            sh.data_ptr(), 2, wk.data_ptr(), o.data_ptr(), C, Ho, Wo, s, S()), a.reps),
                "dg2": timeit(lambda: call("seg_dw2_dgrad_bf16io", dy.data_ptr(), C, N, Ho, Wo, C, wk.data_ptr(),
                                           dx.data_ptr(), C, H, W, s, 1, S()), a.reps),
                "dg1": timeit(lambda: call("seg_dw_dgrad_bf16io", dy.data_ptr(), C, N, Ho, Wo, C, wk.data_ptr(),
                                           dx.data_ptr(), C, H, W, s, 1, S()), a.reps),
                "wg2": timeit(lambda: call("seg_dw2_wgrad_bf16io", dy.data_ptr(), C, x.data_ptr(), C, N, H, W, C,
                                           sc.data_ptr(), sh.data_ptr(), 2, Ho, Wo, s, p2.data_ptr(), S()), a.reps),
                "wg1": timeit(lambda: call("seg_dw_wgrad_bf16io", dy.data_ptr(), C, x.data_ptr(), C, N, H, W, C,
                                           sc.data_ptr(), sh.data_ptr(), 2, Ho, Wo, s, p1.data_ptr(), S()), a.reps),
            }
            # dgrad with accumulate reads dX as well
            nb = {"fwd2": nbytes, "fwd1": nbytes, "dg2": nbytes + 2 * C * N * H * W, "dg1": nbytes + 2 * C * N * H * W,
                  "wg2": nbytes, "wg1": nbytes}
            line = "  ".join(f"{k} {v * 1e6:6.1f} us {nb[k] / v / 1e9:5.0f}" for k, v in res.items())
            print(f"{name:15s} {line}", flush=True)
            rows += [(name, k, v * 1e6, nb[k] / v / 1e9) for k, v in res.items()]
    if a.csv:
        with open(a.csv, "w") as fh:
            fh.write("shape,kernel,us,gbs\n")
            for r in rows:
                fh.write(",".join(str(v) for v in r) + "\n")


if __name__ == "__main__":
    main()
