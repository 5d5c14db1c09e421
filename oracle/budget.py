"""CPU ORACLE -- TEST INFRASTRUCTURE ONLY (tests/, __graft_entry__.smoke()).

Gradient parity of the fp32 HIP path against the fp64 oracle ("no worse
than the reference's own fp32 error"), with the ReLU/ReLU6 masks handled explicitly
instead of by a widened budget.

ReLU / ReLU6 gradients are discontinuous in the pre-activation z: an element within
rounding distance of a threshold passes its gradient in one valid fp32 implementation
and blocks it in another (a "mask flip"), and at test sizes one flip moves a weight
gradient by ~1e-3.  So the check has three parts, all sized from oracle runs only
(nothing depends on the HIP result except what is being checked):

 1. pre-activations: every activation layer's z from the HIP forward is within
    Z_FACTOR x the oracle's own fp32 error of z64 (max |z32 - z64| of that layer) --
    a per-layer forward check that also bounds where flips can occur;
 2. the fp64 oracle is re-run with the HIP path's own masks (segref.MASK_OVERRIDE):
    g64m = the exact gradient of the function the HIP path differentiated;
 3. per tensor  ||g_hip - g64m|| <= max(1e-3 ||g64m||, 4 eps_ref, 1e-4 ||G64||)
    with eps_ref = ||g32m - g64||, the oracle's fp32 accumulation error with the fp64
    masks forced (mask flips excluded from it too).

The number of flipped mask elements per layer is reported (they are legitimate only
because of 1.).
"""
from __future__ import annotations

import torch

from . import segref

Z_FACTOR = 16.0


def _cast(state, dtype):
    return {k: (v.to(dtype) if v.is_floating_point() else v.clone()) for k, v in state.items()}


def _grads(arch, state, x, y, dtype, masks=None, pools=None):
    p = _cast(state, dtype)
    segref.MASK_OVERRIDE, segref.POOL_OVERRIDE = masks, pools
    try:
        loss, _, g = segref.forward_backward(arch, p, x.to(dtype), y, True)
    finally:
        segref.MASK_OVERRIDE = segref.POOL_OVERRIDE = None
    return loss, g


def oracle_side(arch, state, x, y):
    """Everything that depends on the oracle only: z32 / z64 per layer, the fp64 masks,
    eps_ref per tensor.  state: segref.canonical_state(model.state_dict())."""
    z32 = segref.preactivations(arch, _cast(state, torch.float32), x.float())
    z64 = segref.preactivations(arch, _cast(state, torch.float64), x.double())
    hi = dict(segref.ACT_HI)
    m64 = {k: segref.act_mask(z, hi[k]) for k, z in z64.items()}
    loss64, g64 = _grads(arch, state, x, y, torch.float64)
    _, g32m = _grads(arch, state, x, y, torch.float32, m64)
    eps = {k: float((g32m[k].double() - g).norm()) for k, g in g64.items()}
    zerr = {k: float((z32[k].double() - z64[k]).abs().max()) for k in z64}
    return {"z64": z64, "hi": hi, "m64": m64, "loss64": loss64, "g64": g64, "eps": eps, "zerr": zerr}


def check_hip(arch, state, x, y, hip_grads, hip_z, side=None, hip_pools=None):
    """hip_z: {layer prefix: z (NCHW, any float dtype)} of the HIP forward; hip_grads:
    {name: grad}.  hip_pools (optional, UNet): {pool name: 2x2-window positions the HIP forward's max-pools chose}
    (engine.debug_pool_positions) -- the fp64 oracle then also routes its max-pool gradients through the HIP path's
    choices, as it takes its ReLU masks (round 6: a near-tie in a window is the same kind of discontinuity; VERDICT r5
    item 5).  Returns a report dict; report["ok"] is the verdict."""
    side = side or oracle_side(arch, state, x, y)
    z64, hi, m64 = side["z64"], side["hi"], side["m64"]
    missing = sorted(set(z64) - set(hip_z))
    zrep, masks, flips = {}, {}, {}
    zbad = []
    for k, z in z64.items():
        zh = hip_z[k].double().cpu()
        err = float((zh - z).abs().max())
        lim = Z_FACTOR * side["zerr"][k] + 1e-30
        zrep[k] = err / lim
        if err > lim:
            zbad.append((k, err, side["zerr"][k]))
        masks[k] = segref.act_mask(zh, hi[k])
        flips[k] = int((masks[k] != m64[k]).sum())
    pool_flips = {}
    if hip_pools:
        z64a = {k: segref.act_mask(z, None) * z for k, z in z64.items()}  # ReLU of the pool inputs (UNet: ReLU)
        src = {"down1.": "inc.conv.conv.3.", "down2.": "down1.mpconv.1.conv.3.", "down3.": "down2.mpconv.1.conv.3."}
        for k, pos in hip_pools.items():
            if src.get(k) in z64a:
                pool_flips[k] = int((segref.pool_positions(z64a[src[k]]) != pos).sum())
    _, g64m = _grads(arch, state, x, y, torch.float64, masks, hip_pools)
    g64 = side["g64"]
    gnorm = float(torch.sqrt(sum((g ** 2).sum() for g in g64.values())))
    worst, wname, bad, ratios = 0.0, None, [], {}
    for k, g in g64m.items():
        d = float((hip_grads[k].double().cpu() - g).norm())
        tol = max(1e-3 * float(g.norm()), 4 * side["eps"][k], 1e-4 * gnorm)
        r = d / tol
        ratios[k] = r
        if r > worst:
            worst, wname = r, k
        if d > tol:
            bad.append((k, d, tol))
    # the same tensor against the unmatched fp64 oracle, for the record
    d_unmatched = float((hip_grads[wname].double().cpu() - g64[wname]).norm()) if wname else 0.0
    return {"ok": not bad and not zbad and not missing, "worst": worst, "worst_name": wname, "bad": bad,
            "z_bad": zbad, "missing_layers": missing, "z_worst": max(zrep.values()) if zrep else 0.0,
            "flips": {k: v for k, v in flips.items() if v}, "n_flips": sum(flips.values()),
            "pool_flips": pool_flips,
            "worst_vs_unmatched_fp64": d_unmatched, "ratios": ratios, "loss64": float(side["loss64"])}
