"""CPU: the oracle's restatement of cv2.resize (inference.py:30,68-70).

cv2 is not installed, so there are no golden vectors (parity with real cv2 is
unpinned).  These tests pin the restatement's internal consistency: the
vectorised numpy form equals a scalar per-pixel transcription of OpenCV's
loops, and it has the properties the published algorithm guarantees
(identity at scale 1, constants preserved, nearest == pure index selection).
"""
import math

import numpy as np
import pytest

from oracle import cvresize


def _scalar_linear(img, W, H):
    Hs, Ws, C = img.shape
    sxs, fxs = [], []
    for dx in range(W):
        fx = np.float32((dx + 0.5) * (1.0 / (W / Ws)) - 0.5)
        sx = math.floor(fx)
        fx = np.float32(fx - np.float32(sx))
        if sx < 0:
            sx, fx = 0, np.float32(0)
        if sx >= Ws - 1:
            sx, fx = Ws - 1, np.float32(0)
        sxs.append(sx)
        fxs.append((int(np.rint((np.float32(1) - fx) * np.float32(2048))),
                    int(np.rint(fx * np.float32(2048)))))
    out = np.zeros((H, W, C), np.uint8)
    for dy in range(H):
        fy = np.float32((dy + 0.5) * (1.0 / (H / Hs)) - 0.5)
        sy = math.floor(fy)
        fy = np.float32(fy - np.float32(sy))
        b0 = int(np.rint((np.float32(1) - fy) * np.float32(2048)))
        b1 = int(np.rint(fy * np.float32(2048)))
        r0 = min(max(sy, 0), Hs - 1)
        r1 = min(max(sy + 1, 0), Hs - 1)
        for dx in range(W):
            sx, (a0, a1) = sxs[dx], fxs[dx]
            sx1 = min(sx + 1, Ws - 1)
            for c in range(C):
                d0 = int(img[r0, sx, c]) * a0 + int(img[r0, sx1, c]) * a1
                d1 = int(img[r1, sx, c]) * a0 + int(img[r1, sx1, c]) * a1
                t = (((d0 >> 4) * b0) >> 16) + (((d1 >> 4) * b1) >> 16)
                out[dy, dx, c] = min(max((t + 2) >> 2, 0), 255)
    return out


@pytest.mark.parametrize("hs,ws,h,w", [(45, 80, 8, 16), (7, 9, 16, 20), (16, 16, 16, 16), (30, 50, 13, 7)])
def test_vectorised_equals_scalar(hs, ws, h, w):
    g = np.random.Generator(np.random.PCG64(hs * 100 + ws))
    img = g.integers(0, 256, (hs, ws, 3), dtype=np.uint8)
    np.testing.assert_array_equal(cvresize.resize_linear_u8(img, (w, h)), _scalar_linear(img, w, h))


def test_identity_and_constant():
    g = np.random.Generator(np.random.PCG64(1))
    img = g.integers(0, 256, (24, 40, 3), dtype=np.uint8)
    np.testing.assert_array_equal(cvresize.resize_linear_u8(img, (40, 24)), img)
    for v in (0, 1, 127, 254, 255):
        c = np.full((720, 1280, 3), v, np.uint8)
        assert np.all(cvresize.resize_linear_u8(c, (256, 128)) == v)


def test_nearest_and_preprocess_shapes():
    cls = np.arange(128 * 256, dtype=np.int64).reshape(128, 256) % 10
    m = cvresize.resize_nearest(cls.astype(np.uint8), (1280, 720))
    assert m.shape == (720, 1280)
    assert m[0, 0] == cls[0, 0] and m[719, 1279] == cls[127, 255]
    # x: 1280 -> 256 is an exact 5x: columns 5k..5k+4 read source column k
    assert np.array_equal(m[0, 5:10], np.full(5, cls[0, 1], np.uint8))
    f = np.zeros((720, 1280, 3), np.uint8)
    f[..., 2] = 255  # pure red in BGR
    x, rgb = cvresize.preprocess_image(f)
    assert x.shape == (1, 3, 128, 256) and x.dtype == np.float32
    assert np.all(rgb[..., 0] == 255) and np.all(rgb[..., 1:] == 0)
    np.testing.assert_allclose(x[0, 0], (1 - 0.485) / 0.229, rtol=1e-6)
