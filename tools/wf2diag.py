"""why did the two-waves-per-SIMD fused Winograd kernel (wino_fused2_kernel, commit 152956a)
put the UNet 2x128x256 slice's weight gradients at 2.5x the oracle budget while its logits stayed at 3e-6?

    SEG_LIB_PATH=variants/wf2.so python tools/wf2diag.py
(variants/wf2.so: tools/variant.py wf2 --only wino.hip -DSEG_WF2_TEST=1 -- a test-only build; the product library
never contains the kernel.)  seg_wf2_mask(m): bit 0 routes the forward calls of seg_conv_wino_fused (bias / BN
partials given) to fused2, bit 1 the data-gradient calls; 0 = the product's one-wave kernel for both.

A: each form alone against a float64 direct convolution of the same operands, on the slice's fused shapes (down1.0
   forward 64 -> 128 at 64x128, up2.0 / up3.0 data gradients 64 -> 256 / 64 -> 128), with the data gradient's calling
   pattern (no bias, output rows wider than Cout, an addend), and a Cin % 8 == 4 case;
B: the slice test itself (tests/test_gpu_unet_cfg5.py::_slice_run, all Winograd transforms on) with fused2 on the
   forward only, the data gradient only, both, neither -- with the checker routing the fp64 oracle's max-pool gradients
   through the HIP forward's window choices (round 6), and the number of windows whose choice differs from fp64.
"""
import os
import sys

import torch
import torch.nn.functional as F

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "team02-objectdetection_amd"), REPO, os.path.join(REPO, "tests")]
from seg_amd import _lib, engine  # noqa: E402
from seg_amd._lib import call  # noqa: E402

DEV = "cuda"


def mask(m):
    rc = _lib.lib().seg_wf2_mask(m)
    assert rc == 0


def one(N, H, W, Cin, Cout, ldout, add, grad_like, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(N, H, W, Cin, generator=g)
    if grad_like:  # a data gradient's input: ReLU-masked, small, many exact zeros
        x = x * (torch.rand(N, H, W, Cin, generator=g) > 0.5) * 1e-4
    w = torch.randn(Cout, Cin, 3, 3, generator=g) / (9 * Cin) ** 0.5
    a = torch.randn(N * H * W, ldout, generator=g) * (1e-4 if grad_like else 1.0)
    ref = F.conv2d(x.permute(0, 3, 1, 2).double(), w.double(), padding=1).permute(0, 2, 3, 1).reshape(-1, Cout)
    if add:
        ref = ref + a[:, :Cout].double()
    xg, wg = x.reshape(-1, Cin).contiguous().to(DEV), w.to(DEV)
    u = torch.empty(16 * Cout * Cin, device=DEV)
    table, n, blocks = engine.pack_table([(wg.data_ptr(), u.data_ptr(), Cout, Cin, 3, Cin, 3, Cin)], wg.device)
    s = torch.cuda.current_stream().cuda_stream
    call("seg_pack_batch", table.data_ptr(), n, blocks, s)
    ag = a.to(DEV)
    res = {}
    for m in (0, 3):
        mask(m)
        out = torch.full((N * H * W, ldout), float("nan"), device=DEV)
        call("seg_conv_wino_fused", xg.data_ptr(), Cin, N, H, W, Cin, u.data_ptr(), Cin, None, out.data_ptr(), ldout,
             Cout, ag.data_ptr() if add else None, ldout, None, s)
        torch.cuda.synchronize()
        o = out[:, :Cout].double().cpu()
        err = (o - ref).norm() / ref.norm()
        mx = ((o - ref).abs().max() / ref.abs().max())
        beyond = bool(out[:, Cout:].isnan().all()) if ldout > Cout else True
        res[m] = (float(err), float(mx), beyond, int(torch.isnan(o).sum()))
    mask(0)
    return res


def main():
    print("A: seg_conv_wino_fused against float64 (rel L2, max rel, untouched beyond Cout, NaNs)")
    for (N, H, W, Cin, Cout, ldout, add) in [(2, 64, 128, 64, 128, 128, False), (2, 64, 128, 64, 256, 256, False),
                                             (2, 128, 256, 64, 128, 128, False), (2, 128, 256, 64, 128, 160, True),
                                             (2, 64, 128, 68, 128, 136, True), (1, 10, 14, 152, 64, 64, False)]:
        for gl in (False, True):
            r = one(N, H, W, Cin, Cout, ldout, add, gl, N * H + Cin + Cout)
            print(f"  N{N} {H}x{W} {Cin:4d}->{Cout:4d} ldout {ldout} add {int(add)} grad-like {int(gl)}: "
                  f"fused1 {r[0][0]:.2e} / {r[0][1]:.2e} {r[0][2]} {r[0][3]} | fused2 {r[3][0]:.2e} / {r[3][1]:.2e} "
                  f"{r[3][2]} {r[3][3]}", flush=True)
    print("B: UNet 2x128x256 slice (all Winograd transforms), worst gradient as a share of the oracle budget")
    import test_gpu_unet_cfg5 as t
    from oracle import budget, segref
    from seg_amd import UNet
    from seg_amd.detinit import deterministic_init, synthetic_batch
    x, y = synthetic_batch(2, 128, 256, 10, seed=31)
    model_cpu = deterministic_init(UNet(10), seed=31)
    state = segref.canonical_state(model_cpu.state_dict())
    side = budget.oracle_side("UNet", state, x, y)
    for m, tag in ((0, "fused1 everywhere"), (1, "fused2 forward only"), (2, "fused2 data gradient only"),
                   (3, "fused2 both")):
        mask(m)
        logits, loss, rep, n_wino = t._slice_run(x, y, state, side, True, True, True)
        top = sorted(rep["ratios"].items(), key=lambda kv: -kv[1])[:4]
        print(f"  {tag:26s}: worst {rep['worst']:.3f} ({rep['worst_name']}), next {top[1:]}, "
              f"{len(rep['bad'])} tensors over budget, z {rep['z_worst']:.3f}, ReLU mask flips {rep['n_flips']}, "
              f"max-pool window choices differing from fp64 {rep.get('pool_flips')}", flush=True)
    mask(0)


if __name__ == "__main__":
    main()
