"""CPU ORACLE -- TEST INFRASTRUCTURE ONLY (see oracle/segref.py's header).

numpy restatement of the reference's inference-time image handling
(inference.py:28-46 preprocess_image, :64-70 argmax + mask resize), used only
by tests/ and bench.py's cpu_baseline leg as the checker.

OpenCV (cv2, unpinned in requirements.txt:7) is NOT installed in this image, so
the two resizes are restated from OpenCV's published imgproc/src/resize.cpp
(4.x) and their parity with real cv2 is UNPINNED:
  * cv2.resize(img, dsize) default INTER_LINEAR, 8-bit:
      x: fx = float32((dx + 0.5) * scale_x - 0.5); sx = floor(fx); fx -= sx;
         sx < 0 -> (0, 0.0); sx >= W-1 -> (W-1, 0.0)
         alpha = (cvRound((1-fx)*2048), cvRound(fx*2048))      (round half to even)
      y: the same without the clamp; rows clip(sy, 0, H-1), clip(sy+1, 0, H-1)
      horizontal (HResizeLinear, int32, exact):  D = S[sx]*a0 + S[sx+1]*a1
      vertical (VResizeLinearVec_32s8u, the SIMD path taken by every full row):
         out = sat_u8(((((D0 >> 4) * b0) >> 16) + (((D1 >> 4) * b1) >> 16) + 2) >> 2)
  * cv2.resize(..., INTER_NEAREST): sx = min(floor(x * (1 / (dst_w / src_w))), src_w - 1)
    in double precision (resizeNN).
The ToTensor / Normalize arithmetic is torchvision's: float32 x / 255, then
(x - mean) / std with float32 constants.
"""
from __future__ import annotations

import numpy as np

MEAN = (0.485, 0.456, 0.406)
STD = (0.229, 0.224, 0.225)


def _cv_round(x):
    return np.rint(x).astype(np.int64)  # half to even, like cvRound under the default FP mode


def resize_linear_u8(img: np.ndarray, dsize) -> np.ndarray:
    """cv2.resize(img, dsize=(W, H)) with INTER_LINEAR on a uint8 HxWxC image."""
    W, H = dsize
    Hs, Ws = img.shape[:2]
    scale_x = 1.0 / (W / Ws)
    scale_y = 1.0 / (H / Hs)
    dx = np.arange(W, dtype=np.float64)
    fx = ((dx + 0.5) * scale_x - 0.5).astype(np.float32)
    sx = np.floor(fx).astype(np.int64)
    fx = (fx - sx.astype(np.float32)).astype(np.float32)
    lo = sx < 0
    sx[lo], fx[lo] = 0, 0.0
    hi = sx >= Ws - 1
    sx[hi], fx[hi] = Ws - 1, 0.0
    a0 = _cv_round((np.float32(1.0) - fx) * np.float32(2048.0))
    a1 = _cv_round(fx * np.float32(2048.0))
    sx1 = np.minimum(sx + 1, Ws - 1)
    dy = np.arange(H, dtype=np.float64)
    fy = ((dy + 0.5) * scale_y - 0.5).astype(np.float32)
    sy = np.floor(fy).astype(np.int64)
    fy = (fy - sy.astype(np.float32)).astype(np.float32)
    b0 = _cv_round((np.float32(1.0) - fy) * np.float32(2048.0))
    b1 = _cv_round(fy * np.float32(2048.0))
    y0 = np.clip(sy, 0, Hs - 1)
    y1 = np.clip(sy + 1, 0, Hs - 1)
    S = img.astype(np.int64)
    # horizontal pass on every source row that is used
    D = S[:, sx, :] * a0[None, :, None] + S[:, sx1, :] * a1[None, :, None]   # [Hs, W, C]
    D0, D1 = D[y0], D[y1]                                                     # [H, W, C]
    t = (((D0 >> 4) * b0[:, None, None]) >> 16) + (((D1 >> 4) * b1[:, None, None]) >> 16)
    t = (t + 2) >> 2
    return np.clip(t, 0, 255).astype(np.uint8)


def resize_nearest(img: np.ndarray, dsize) -> np.ndarray:
    """cv2.resize(img, dsize=(W, H), interpolation=INTER_NEAREST) of a 2-D array."""
    W, H = dsize
    Hs, Ws = img.shape[:2]
    ifx = 1.0 / (W / Ws)
    ify = 1.0 / (H / Hs)
    xs = np.minimum(np.floor(np.arange(W, dtype=np.float64) * ifx).astype(np.int64), Ws - 1)
    ys = np.minimum(np.floor(np.arange(H, dtype=np.float64) * ify).astype(np.int64), Hs - 1)
    return img[ys][:, xs]


def preprocess_image(frame: np.ndarray, target_size=(256, 128)) -> tuple[np.ndarray, np.ndarray]:
    """inference.py:28-46: returns (float32 [1,3,H,W] normalised RGB, resized RGB uint8)."""
    img = resize_linear_u8(frame, target_size)
    img = img[:, :, ::-1]  # cv2.cvtColor(BGR2RGB)
    t = img.transpose(2, 0, 1).astype(np.float32) / np.float32(255.0)
    mean = np.asarray(MEAN, dtype=np.float32)[:, None, None]
    std = np.asarray(STD, dtype=np.float32)[:, None, None]
    t = (t - mean) / std
    return t[None].astype(np.float32), np.ascontiguousarray(img)


def class_mask(logits: np.ndarray, frame_hw) -> np.ndarray:
    """torch.max(logits, dim=1) (first maximum) -> uint8 -> INTER_NEAREST to the frame."""
    cls = np.argmax(logits[0], axis=0).astype(np.uint8)
    Hf, Wf = frame_hw
    return resize_nearest(cls, (Wf, Hf))
