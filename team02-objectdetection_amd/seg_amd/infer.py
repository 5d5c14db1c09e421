"""GPU replacement for the per-frame path of the reference's inference.py.

The reference loop (inference.py:150-170) does, per video frame:
    img_tensor, _ = preprocess_image(frame)            # :28-46  cv2.resize -> RGB -> ToTensor -> Normalize
    road_predictions = model(img_tensor)               # :162-163 eval forward under no_grad
    _, cls = torch.max(road_predictions, dim=1)        # :64     (inside overlay_predictions)
    cls = cv2.resize(cls.astype(uint8), (W, H), INTER_NEAREST)   # :68-70
and then OpenCV post-processing / display (out of scope, host GUI code).

`Predictor` runs all of that on the MI355X as four stages over static buffers,
captured once into a HIP graph (torch.cuda.CUDAGraph drives hipGraph on ROCm):
    seg_preprocess_bgr      uint8 BGR frame -> the model's NHWC4 input rows
    Run.forward_folded      eval forward, BatchNorm folded into every conv
                            (Program.fold: one seg_bn_fold_batch + one seg_pack_batch)
    seg_argmax_nearest      final align_corners=True upsample + argmax + nearest
                            resize to the frame -> uint8 class mask

`preprocess_image` mirrors inference.py's function of the same name (same
argument meaning and return values) for callers that still want the tensor.
"""
from __future__ import annotations

import numpy as np
import torch

from ._lib import call
from . import engine
from .engine import Run, get_program

MEAN = (0.485, 0.456, 0.406)   # inference.py:35
STD = (0.229, 0.224, 0.225)    # inference.py:36


def _frame_tensor(frame, device) -> torch.Tensor:
    if isinstance(frame, np.ndarray):
        if frame.dtype != np.uint8 or frame.ndim != 3 or frame.shape[2] != 3:
            raise ValueError(f"expected a uint8 HxWx3 BGR frame, got {frame.dtype} {frame.shape}")
        return torch.from_numpy(np.ascontiguousarray(frame)).to(device, non_blocking=False)
    if not torch.is_tensor(frame) or frame.dtype != torch.uint8 or frame.dim() != 3 or frame.shape[2] != 3:
        raise ValueError("expected a uint8 HxWx3 BGR frame (numpy array or tensor)")
    return frame.to(device).contiguous()


def preprocess_image(image, target_size=(256, 128), device="cuda"):
    """inference.py:28-46 on the GPU: returns (img_tensor [1,3,H,W] float32 on
    `device`, the resized RGB uint8 image is not materialised -> None)."""
    W, H = target_size  # cv2 dsize order (width, height)
    f = _frame_tensor(image, device)
    Hf, Wf = f.shape[0], f.shape[1]
    rows = torch.empty((H * W, 4), device=f.device, dtype=torch.float32)
    s = torch.cuda.current_stream(f.device).cuda_stream
    call("seg_preprocess_bgr", f.data_ptr(), 1, Hf, Wf, f.stride(0), rows.data_ptr(), 4, H, W, *MEAN, *STD, s)
    img = rows[:, :3].reshape(1, H, W, 3).permute(0, 3, 1, 2).contiguous()
    return img, None


class Predictor:
    """Frame -> class mask for a MobileNetV2UNet / UNet in eval mode.

    predictor = Predictor(model, frame_hw=(720, 1280))   # model already on cuda
    mask = predictor(frame)          # uint8 [720, 1280] class ids on the GPU
    logits = predictor.logits()      # [1, C, 128, 256] of the last frame (tests)

    math="f16" runs every folded conv on fp16 operands (BASELINE configs[3]).
    Weights are folded at construction; call `refresh()` after changing the
    model's parameters or running statistics (e.g. load_state_dict).
    """

    def __init__(self, model, frame_hw=(720, 1280), target_size=(256, 128), graph: bool = True, math: str = "f32"):
        p = next(model.parameters())
        if not p.is_cuda:
            raise RuntimeError("Predictor runs on the MI355X HIP path only; move the model to 'cuda' first")
        self.model = model.eval()
        self.device = p.device
        self.Hf, self.Wf = frame_hw
        self.W, self.H = target_size
        # math: conv arithmetic of the folded forward -- "f32" (the reference's), "f16"
        # (BASELINE configs[3]: fp16 operands, fp32 accumulation) or "bf16"
        if math not in ("f32", "f16", "bf16"):
            raise ValueError(f"Predictor math must be 'f32', 'f16' or 'bf16', got {math!r}")
        self.prog = get_program(model, 1, self.H, self.W, math)
        self.frame = torch.zeros((self.Hf, self.Wf, 3), device=self.device, dtype=torch.uint8)
        self.mask = torch.empty((self.Hf, self.Wf), device=self.device, dtype=torch.uint8)
        self.run = Run(self.prog, self.frame, training=False)
        self.classes = self.prog.logits.C
        self.graph = None
        self.refresh()
        self.stem_pre = self.prog.stem_pre() if (engine.STEM_PRE and math == "f16") else None
        if graph:
            self._capture()

    def refresh(self):
        """Re-fold BatchNorm into the conv weights (after weights/statistics change)."""
        with torch.no_grad():
            self.prog.fold(torch.cuda.current_stream(self.device).cuda_stream)

    def _launch(self):
        rt, prog = self.run, self.prog
        s = torch.cuda.current_stream(self.device).cuda_stream
        rt.stream = s
        img = prog.image
        if self.stem_pre is not None:  # preprocess formed on load by the stem conv (seg_stem_pre_f16)
            op, o = self.stem_pre, self.stem_pre.out
            call("seg_stem_pre_f16", self.frame.data_ptr(), self.Hf, self.Wf, self.frame.stride(0), self.H, self.W,
                 *MEAN, *STD, op.fk_pack.data_ptr(), op.ldk_f, op.fb.data_ptr(), op.act, op.cout, rt.ptr(o), o.ld, s)
            rt.forward_folded(start=1)
        else:
            call("seg_preprocess_bgr", self.frame.data_ptr(), 1, self.Hf, self.Wf, self.frame.stride(0), rt.ptr(img),
                 img.ld, self.H, self.W, *MEAN, *STD, s)
            rt.forward_folded()
        lo = prog.logits
        Ho, Wo = prog.out_hw
        call("seg_argmax_nearest", rt.ptr(lo), lo.ld, 1, lo.H, lo.W, lo.C, Ho, Wo, self.mask.data_ptr(), self.Hf,
             self.Wf, s)

    def _capture(self):
        side = torch.cuda.Stream(self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(side):
            self._launch()  # warm-up outside the capture (module load, first-launch setup)
        torch.cuda.current_stream(self.device).wait_stream(side)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self._launch()
        self.graph = g

    def set_frame(self, frame):
        """Copy a frame into the static input buffer (host numpy -> H2D, or device tensor)."""
        if isinstance(frame, np.ndarray):
            if frame.shape != (self.Hf, self.Wf, 3) or frame.dtype != np.uint8:
                raise ValueError(f"expected uint8 frame of shape {(self.Hf, self.Wf, 3)}, got {frame.dtype} "
                                 f"{frame.shape}")
            self.frame.copy_(torch.from_numpy(np.ascontiguousarray(frame)), non_blocking=False)
        else:
            if tuple(frame.shape) != (self.Hf, self.Wf, 3) or frame.dtype != torch.uint8:
                raise ValueError(f"expected uint8 frame of shape {(self.Hf, self.Wf, 3)}")
            self.frame.copy_(frame)

    def step(self):
        """Run the captured graph (or the eager launch sequence) on the current frame."""
        if self.graph is not None:
            self.graph.replay()
        else:
            self._launch()
        return self.mask

    def __call__(self, frame=None):
        if frame is not None:
            self.set_frame(frame)
        return self.step()

    def logits(self) -> torch.Tensor:
        """[1, C, H, W] logits of the last frame (the model's return value, src/unet.py:49)."""
        lo = self.prog.logits
        Ho, Wo = self.prog.out_hw
        out = torch.empty((1, lo.C, Ho, Wo), device=self.device, dtype=torch.float32)
        call("seg_upsample_to_nchw", self.run.ptr(lo), lo.ld, 1, lo.H, lo.W, lo.C, out.data_ptr(), Ho, Wo, 1,
             torch.cuda.current_stream(self.device).cuda_stream)
        return out
