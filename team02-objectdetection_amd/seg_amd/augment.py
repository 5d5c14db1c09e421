"""GPU-side training augmentation.

The reference's readers run albumentations on the CPU per sample
(src/BDD100KDataset.py:38-52, src/CarlaDataset.py:40-47,
src/SEAMEDataset.py:55-62):
    A.Resize(height, width), A.HorizontalFlip(p=0.5),
    A.ShiftScaleRotate(shift_limit=0.05, scale_limit=0.05, rotate_limit=10, p=0.5),
    A.RandomBrightnessContrast(p=0.5), A.Normalize(ImageNet), ToTensorV2()
and remap BDD100K's class ids with a dict (src/BDD100KDataset.py:23-35, 66-70).
At >1k img/s per GPU that CPU work, not the decode, is what starves 8 GPUs.
`GpuAugment` takes a batch of decoded uint8 RGB images and raw uint8 masks on
the device and produces the model input (float NCHW) and int64 labels with two
kernels (seg_resize_u8 x2, seg_augment).  The random parameters follow
albumentations' distributions and are drawn on the host from a numpy Generator,
so a seed reproduces a batch exactly; the kernels' arithmetic is restated in
oracle/augref.py (albumentations / cv2 are not installed: parity with them is
unpinned).
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ._lib import call

# src/BDD100KDataset.py:23-35 (source id -> model class; everything else -> 0, :66-70)
BDD100K_CLASS_MAP = {0: 1, 13: 2, 6: 3, 7: 4, 11: 5, 1: 6, 14: 7, 15: 8, 17: 9, 18: 9, 12: 9}
MEAN = (0.485, 0.456, 0.406)
STD = (0.229, 0.224, 0.225)

PARAM_DTYPE = np.dtype([("m", "<f4", (6,)), ("alpha", "<f4"), ("beta", "<f4"), ("flip", "<i4"), ("warp", "<i4"),
                        ("bc", "<i4"), ("pad", "<i4")])
assert PARAM_DTYPE.itemsize == 48


def class_lut(class_map=None) -> np.ndarray:
    lut = np.zeros(256, np.uint8)
    if class_map is None:
        return np.arange(256, dtype=np.uint8)
    for s, t in class_map.items():
        lut[s] = t
    return lut


def normalize_constants(mean=MEAN, std=STD):
    """albumentations Normalize(max_pixel_value=255) in float32: (v - 255*mean) * (1/(255*std))."""
    m = np.asarray(mean, np.float32) * np.float32(255.0)
    r = np.reciprocal(np.asarray(std, np.float32) * np.float32(255.0))
    return m.astype(np.float32), r.astype(np.float32)


def draw_params(n, height, width, rng: np.random.Generator, is_train=True, p=0.5, shift_limit=0.05,
                scale_limit=0.05, rotate_limit=10.0, brightness_limit=0.2, contrast_limit=0.2) -> np.ndarray:
    """Per-sample parameters with albumentations' distributions (each transform applied
    with probability p): angle U(-10, 10) deg, scale U(0.95, 1.05), shift U(-0.05, 0.05)
    of the size, contrast alpha 1 + U(-0.2, 0.2), brightness beta U(-0.2, 0.2) (x 255)."""
    out = np.zeros(n, PARAM_DTYPE)
    out["alpha"] = 1.0
    if not is_train:
        return out
    cx, cy = (width - 1) * 0.5, (height - 1) * 0.5
    for k in range(n):
        out["flip"][k] = rng.random() < p
        if rng.random() < p:
            ang = rng.uniform(-rotate_limit, rotate_limit)
            sc = rng.uniform(1 - scale_limit, 1 + scale_limit)
            dx = rng.uniform(-shift_limit, shift_limit)
            dy = rng.uniform(-shift_limit, shift_limit)
            # cv2.getRotationMatrix2D(center, angle, scale) + shift; warpAffine samples M^-1
            a = sc * math.cos(math.radians(ang))
            b = sc * math.sin(math.radians(ang))
            M = np.array([[a, b, (1 - a) * cx - b * cy + dx * width],
                          [-b, a, b * cx + (1 - a) * cy + dy * height],
                          [0.0, 0.0, 1.0]])
            out["m"][k] = np.linalg.inv(M)[:2].reshape(-1).astype(np.float32)
            out["warp"][k] = 1
        if rng.random() < p:
            out["alpha"][k] = 1.0 + rng.uniform(-contrast_limit, contrast_limit)
            out["beta"][k] = rng.uniform(-brightness_limit, brightness_limit)
            out["bc"][k] = 1
    return out


class GpuAugment:
    """Batch version of the readers' albumentations pipeline on the MI355X.

    aug = GpuAugment(height=256, width=512, class_map=BDD100K_CLASS_MAP)
    x, y = aug(images, masks, rng)   # images uint8 [N,Hs,Ws,3] RGB, masks uint8 [N,Hs,Ws] (cuda)
    """

    def __init__(self, height=128, width=256, is_train=True, class_map=None, mean=MEAN, std=STD, **limits):
        self.H, self.W, self.is_train, self.limits = height, width, is_train, limits
        self.mean255, self.rstd255 = normalize_constants(mean, std)
        self._lut_host = class_lut(class_map)
        self._lut = {}

    def __call__(self, images: torch.Tensor, masks: torch.Tensor, rng: np.random.Generator | int = 0,
                 params: np.ndarray | None = None):
        if not images.is_cuda or images.dtype != torch.uint8 or images.dim() != 4 or images.shape[3] != 3:
            raise ValueError("images must be a cuda uint8 [N, Hs, Ws, 3] RGB tensor")
        N, Hs, Ws, _ = images.shape
        if tuple(masks.shape) != (N, Hs, Ws) or masks.dtype != torch.uint8 or not masks.is_cuda:
            raise ValueError("masks must be a cuda uint8 [N, Hs, Ws] tensor")
        dev = images.device
        if not isinstance(rng, np.random.Generator):
            rng = np.random.Generator(np.random.PCG64(rng))
        if params is None:
            params = draw_params(N, self.H, self.W, rng, self.is_train, **self.limits)
        images, masks = images.contiguous(), masks.contiguous()
        lut = self._lut.get(dev)
        if lut is None:
            lut = self._lut[dev] = torch.from_numpy(self._lut_host).to(dev)
        s = torch.cuda.current_stream(dev).cuda_stream
        H, W = self.H, self.W
        img_r = torch.empty((N, H, W, 3), device=dev, dtype=torch.uint8)
        msk_r = torch.empty((N, H, W), device=dev, dtype=torch.uint8)
        call("seg_resize_u8", images.data_ptr(), N, Hs, Ws, Ws * 3, img_r.data_ptr(), H, W, 3, None, s)
        call("seg_resize_u8", masks.data_ptr(), N, Hs, Ws, Ws, msk_r.data_ptr(), H, W, 1, lut.data_ptr(), s)
        prm = torch.from_numpy(np.ascontiguousarray(params).view(np.uint8).copy()).to(dev)
        x = torch.empty((N, 3, H, W), device=dev, dtype=torch.float32)
        y = torch.empty((N, H, W), device=dev, dtype=torch.int64)
        call("seg_augment", img_r.data_ptr(), msk_r.data_ptr(), N, H, W, prm.data_ptr(), *self.mean255.tolist(),
             *self.rstd255.tolist(), x.data_ptr(), y.data_ptr(), s)
        return x, y
