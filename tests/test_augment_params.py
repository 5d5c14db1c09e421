"""CPU: the host side of seg_amd.augment -- parameter distributions follow the
readers' albumentations arguments (src/BDD100KDataset.py:38-52), the BDD100K
class LUT restates src/BDD100KDataset.py:23-35,66-70, and the oracle's
restatement is self-consistent (identity pipeline = plain resize + normalise)."""
import math

import numpy as np

from oracle import augref, cvresize
from seg_amd.augment import BDD100K_CLASS_MAP, class_lut, draw_params, normalize_constants


def test_param_ranges_and_rates():
    rng = np.random.Generator(np.random.PCG64(0))
    p = draw_params(4000, 128, 256, rng)
    for k in ("flip", "warp", "bc"):
        assert abs(p[k].mean() - 0.5) < 0.05
    bc = p[p["bc"] == 1]
    assert np.all(np.abs(bc["alpha"] - 1) <= 0.2 + 1e-6) and np.all(np.abs(bc["beta"]) <= 0.2 + 1e-6)
    w = p[p["warp"] == 1]
    for m in w["m"]:  # inverse of scale*rotation: |det| = 1/scale^2 with scale in [0.95, 1.05]
        det = m[0] * m[4] - m[1] * m[3]
        assert 1 / 1.05 ** 2 - 1e-4 <= det <= 1 / 0.95 ** 2 + 1e-4
        ang = math.degrees(math.atan2(-m[3], m[0]))
        assert abs(ang) <= 10 + 1e-3
    off = p[(p["warp"] == 0)]
    assert np.all(off["m"] == 0)
    ev = draw_params(10, 128, 256, rng, is_train=False)
    assert not ev["flip"].any() and not ev["warp"].any() and not ev["bc"].any()


def test_class_lut():
    lut = class_lut(BDD100K_CLASS_MAP)
    assert lut[0] == 1 and lut[13] == 2 and lut[18] == 9 and lut[12] == 9
    assert lut[2] == 0 and lut[255] == 0 and lut[19] == 0


def test_identity_pipeline_is_resize_and_normalize():
    g = np.random.Generator(np.random.PCG64(1))
    imgs = g.integers(0, 256, (2, 50, 70, 3), dtype=np.uint8)
    masks = g.integers(0, 20, (2, 50, 70), dtype=np.uint8)
    params = draw_params(2, 20, 30, g, is_train=False)
    m, r = normalize_constants()
    x, y = augref.augment(imgs, masks, params, 20, 30, class_lut(BDD100K_CLASS_MAP), m, r)
    ref = (cvresize.resize_linear_u8(imgs[1], (30, 20)).astype(np.float32) - m) * r
    np.testing.assert_array_equal(x[1], ref.transpose(2, 0, 1))
    np.testing.assert_array_equal(y[0], class_lut(BDD100K_CLASS_MAP)[cvresize.resize_nearest(masks[0], (30, 20))])
