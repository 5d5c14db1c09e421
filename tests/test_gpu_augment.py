"""GPU: seg_amd.augment (the readers' albumentations pipeline on the device,
src/BDD100KDataset.py:38-52) against oracle/augref.py -- bit-exact on the same
per-sample parameters (images and labels), for train and eval pipelines, with
every transform forced on, off and mixed."""
import numpy as np
import pytest
import torch

from oracle import augref
from seg_amd.augment import BDD100K_CLASS_MAP, GpuAugment, class_lut, draw_params, normalize_constants

pytestmark = pytest.mark.gpu


def batch(n, hs, ws, seed):
    g = np.random.Generator(np.random.PCG64(seed))
    yy, xx = np.meshgrid(np.linspace(0, 5, hs), np.linspace(0, 7, ws), indexing="ij")
    base = 127.5 + 110 * np.sin(yy + xx)[None, ..., None] * np.cos(np.arange(3) + xx[None, ..., None])
    imgs = np.clip(base + g.normal(0, 20, (n, hs, ws, 3)), 0, 255).astype(np.uint8)
    masks = g.integers(0, 20, (n, hs, ws)).astype(np.uint8)
    masks[:, : hs // 3] = 0  # large constant regions, like real label maps
    return imgs, masks


@pytest.mark.parametrize("mode", ["random", "all_on", "all_off", "eval"])
@pytest.mark.parametrize("hs,ws,h,w", [(180, 320, 64, 128), (97, 131, 40, 56)])
def test_augment_matches_oracle(mode, hs, ws, h, w):
    n = 6
    imgs, masks = batch(n, hs, ws, seed=hs)
    rng = np.random.Generator(np.random.PCG64(7))
    params = draw_params(n, h, w, rng, is_train=mode != "eval", p={"random": 0.5, "all_on": 1.0}.get(mode, 0.0))
    aug = GpuAugment(h, w, is_train=mode != "eval", class_map=BDD100K_CLASS_MAP)
    x, y = aug(torch.from_numpy(imgs).cuda(), torch.from_numpy(masks).cuda(), params=params)
    m255, r255 = normalize_constants()
    xr, yr = augref.augment(imgs, masks, params, h, w, class_lut(BDD100K_CLASS_MAP), m255, r255)
    np.testing.assert_array_equal(y.cpu().numpy(), yr)
    np.testing.assert_array_equal(x.cpu().numpy(), xr)
    if mode == "all_on":
        assert params["warp"].all() and params["flip"].all() and params["bc"].all()
    assert set(np.unique(yr)) <= set(BDD100K_CLASS_MAP.values()) | {0}


def test_augment_throughput_smoke():
    """bs=32 BDD-sized frames (720x1280) -> 256x512: runs and reports img/s (printed)."""
    imgs, masks = batch(32, 720, 1280, seed=3)
    gi, gm = torch.from_numpy(imgs).cuda(), torch.from_numpy(masks).cuda()
    aug = GpuAugment(256, 512, class_map=BDD100K_CLASS_MAP)
    aug(gi, gm, 0)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for k in range(10):
        x, y = aug(gi, gm, k)
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / 10
    print(f"GPU augmentation bs=32 720x1280 -> 256x512: {ms:.3f} ms/batch = {32 / ms * 1e3:.0f} img/s")
    assert x.shape == (32, 3, 256, 512) and torch.isfinite(x).all()


def test_train_model_with_gpu_augment(tmp_path):
    """train_model(..., augment=GpuAugment) on decoded uint8 batches: the reference loop
    (src/train.py:31-42) with the readers' augmentation moved to the GPU."""
    from torch import nn
    from seg_amd import MobileNetV2UNet, deterministic_init, train_model
    imgs, masks = batch(4, 90, 160, seed=5)
    loader = [(torch.from_numpy(imgs[:2]), torch.from_numpy(masks[:2])),
              (torch.from_numpy(imgs[2:]), torch.from_numpy(masks[2:]))]
    model = deterministic_init(MobileNetV2UNet(10), seed=3).cuda()
    opt = torch.optim.Adam(model.parameters(), lr=1.5e-4)
    before = model.outc.conv[3].weight.detach().clone()
    train_model(model, loader, nn.CrossEntropyLoss(), opt, "cuda", epochs=1,
                checkpoint_pattern=str(tmp_path / "ep{epoch}.pth"), progress=False,
                augment=GpuAugment(64, 128, class_map=BDD100K_CLASS_MAP))
    assert (tmp_path / "ep1.pth").exists()
    assert not torch.equal(before, model.outc.conv[3].weight.detach())
