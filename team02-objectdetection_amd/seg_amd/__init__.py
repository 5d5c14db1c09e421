"""seg_amd -- MI355X-native hot path for SEAME-pt/Team02-ObjectDetection's
segmentation models (MobileNetV2UNet / UNet / LightUNet).

Public surface (drop-in for the reference's src/unet.py and src/train.py):
    MobileNetV2UNet, UNet, LightUNet, double_conv, inconv, down, up, outconv
    train_model, train_one_epoch
    Adam                                  (main.py:100's optimizer, one-launch HIP step)
    traceable                             (pure-torch CPU twin for convert.py's ONNX export)
    Predictor, preprocess_image           (inference.py's per-frame path)
    CombinedLaneDataset, DistributedWeightedSampler, reference_sample_weights
                                          (main.py's data path, rank-aware)
All compute runs in libsegamd.so (HIP, gfx950); see include/segamd.h.
"""
from .unet import MobileNetV2UNet, UNet, LightUNet, double_conv, inconv, down, up, outconv  # noqa: F401
from .train import train_model, train_one_epoch  # noqa: F401
from .detinit import deterministic_init, synthetic_batch  # noqa: F401
from .data import CombinedLaneDataset, DistributedWeightedSampler, reference_sample_weights  # noqa: F401
from .infer import Predictor, preprocess_image  # noqa: F401
from .optim import Adam  # noqa: F401
from .export import traceable  # noqa: F401

__all__ = ["MobileNetV2UNet", "UNet", "LightUNet", "double_conv", "inconv", "down", "up", "outconv",
           "train_model", "train_one_epoch", "deterministic_init", "synthetic_batch",
           "CombinedLaneDataset", "DistributedWeightedSampler", "reference_sample_weights",
           "Predictor", "preprocess_image", "Adam", "traceable"]
