"""CPU ORACLE -- TEST INFRASTRUCTURE ONLY (see oracle/segref.py's header).

numpy restatement of seg_amd/augment.py's kernels (csrc/augment.hip): the
readers' albumentations pipeline (src/BDD100KDataset.py:38-52) with the
arithmetic the GPU path defines -- cv2 INTER_LINEAR / INTER_NEAREST resize
(oracle/cvresize.py), class LUT, horizontal flip, ShiftScaleRotate as an inverse
affine warp (float32 bilinear, round half to even, BORDER_REFLECT_101; mask
nearest, round half up), albumentations' uint8 brightness/contrast LUT and
Normalize.  albumentations / cv2 are not installed: parity with them is
UNPINNED; these functions pin the kernels to this written-down arithmetic.
"""
from __future__ import annotations

import numpy as np

from . import cvresize


def _reflect101(i, n):
    i = np.asarray(i, np.int64).copy()
    if n == 1:
        return np.zeros_like(i)
    for _ in range(4):
        i = np.where(i < 0, -i, i)
        i = np.where(i >= n, 2 * n - 2 - i, i)
    return i


def augment(images, masks, params, H, W, lut, mean255, rstd255):
    """images uint8 [N,Hs,Ws,3], masks uint8 [N,Hs,Ws] -> (x float32 [N,3,H,W], y int64 [N,H,W])."""
    N = images.shape[0]
    xs = np.empty((N, 3, H, W), np.float32)
    ys = np.empty((N, H, W), np.int64)
    oy, ox = np.meshgrid(np.arange(H, dtype=np.float32), np.arange(W, dtype=np.float32), indexing="ij")
    for n in range(N):
        im = cvresize.resize_linear_u8(images[n], (W, H))
        mk = lut[cvresize.resize_nearest(masks[n], (W, H))]
        q = params[n]
        u, v = ox.copy(), oy.copy()
        if q["warp"]:
            m = q["m"].astype(np.float32)
            u = (m[0] * ox + m[1] * oy) + m[2]
            v = (m[3] * ox + m[4] * oy) + m[5]
        if q["flip"]:
            u = np.float32(W - 1) - u
        iu, iv = np.floor(u).astype(np.int64), np.floor(v).astype(np.int64)
        fu = (u - iu.astype(np.float32)).astype(np.float32)
        fv = (v - iv.astype(np.float32)).astype(np.float32)
        xa, xb = _reflect101(iu, W), _reflect101(iu + 1, W)
        ya, yb = _reflect101(iv, H), _reflect101(iv + 1, H)
        for c in range(3):
            ch = im[..., c].astype(np.float32)
            if q["warp"]:
                p00, p01, p10, p11 = ch[ya, xa], ch[ya, xb], ch[yb, xa], ch[yb, xb]
                top = p00 + (p01 - p00) * fu
                bot = p10 + (p11 - p10) * fu
                val = np.clip(np.rint(top + (bot - top) * fv), 0, 255).astype(np.float32)
            else:
                val = ch[ya, xa]
            if q["bc"]:
                t = val * np.float32(q["alpha"])
                t = t + np.float32(q["beta"]) * np.float32(255.0)
                val = np.trunc(np.clip(t, 0, 255)).astype(np.float32)
            xs[n, c] = (val - mean255[c]) * rstd255[c]
        nu = _reflect101(np.floor(u + np.float32(0.5)).astype(np.int64), W)
        nv = _reflect101(np.floor(v + np.float32(0.5)).astype(np.int64), H)
        ys[n] = mk[nv, nu]
    return xs, ys
