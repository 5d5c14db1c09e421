"""Drop-in training loop: `train_model(model, train_loader, criterion, optimizer,
device, epochs=10)` with the reference's signature and behaviour
(src/train.py:6-79): per epoch `model.train()`, for each batch `.to(device)`,
`optimizer.zero_grad()`, forward, `criterion`, `backward`, `optimizer.step()`,
running loss, a per-epoch "Training Loss" line and a state_dict checkpoint
`Models/obj/obj_MOB_1_epoch_{epoch}.pth` (src/train.py:77).

MI355X differences (results are the same):
  * when `criterion` is a plain `nn.CrossEntropyLoss()` (main.py:99) and the
    model is a seg_amd model, the loss is computed by the fused
    upsample+cross-entropy kernels (`model.forward_loss`), so the 168 MB of
    full-resolution logits per bs=32 batch are never written;
  * under torch.distributed the gradients are averaged across ranks by
    seg_amd.ddp (RCCL all-reduce overlapped with the backward) and only
    rank 0 prints and writes checkpoints.
"""
from __future__ import annotations

import os

import numpy as np
import torch
from torch import nn

try:
    from tqdm import tqdm
except ImportError:  # pragma: no cover
    tqdm = None


def _fusable_ce(criterion) -> bool:
    return (isinstance(criterion, nn.CrossEntropyLoss) and criterion.weight is None
            and criterion.reduction == "mean" and criterion.label_smoothing == 0.0)


def _is_rank0() -> bool:
    return not (torch.distributed.is_available() and torch.distributed.is_initialized()) or \
        torch.distributed.get_rank() == 0


def _check_labels(model, inputs):
    """Raise IndexError like nn.CrossEntropyLoss if the fused loss saw a label outside
    [0, C) (the kernels flag it; the loss and gradients are NaN).  Runs BEFORE
    optimizer.step(), so no NaN reaches the weights; under torch.distributed the count is
    summed over ranks first, so every rank raises together instead of one rank leaving
    the others in the next collective."""
    if not inputs.is_cuda:
        return  # the CPU composition's F.cross_entropy raises by itself
    from .engine import bad_label_count, bad_label_count_host, check_targets
    if torch.distributed.is_available() and torch.distributed.is_initialized() and hasattr(model, "module"):
        bad = bad_label_count(model)
        if bad is None:
            return
        torch.distributed.all_reduce(bad, group=getattr(model, "pg", None))
        check_targets(model, bad)
        return
    # one process: the count was copied to the host right after the loss kernel, so this waits
    # for the forward only and optimizer.step() is queued while the backward still runs
    n = bad_label_count_host(model)
    if n:
        check_targets(model, torch.tensor([float(n)]))


def compute_loss(model, criterion, inputs, targets):
    """criterion(model(inputs), targets), fused when the pair allows it."""
    core = getattr(model, "module", model)
    if hasattr(core, "forward_loss") and _fusable_ce(criterion):
        return model.forward_loss(inputs, targets, criterion.ignore_index)
    return criterion(model(inputs), targets)


def train_one_epoch(model, train_loader, criterion, optimizer, device, epoch: int = 0, epochs: int = 1,
                    progress: bool = True, augment=None) -> float:
    """One pass over `train_loader`; returns the mean batch loss (src/train.py:31-44).

    augment: optional seg_amd.augment.GpuAugment -- the loader then yields decoded
    uint8 batches (images [N,Hs,Ws,3] RGB, masks [N,Hs,Ws] raw class ids) and the
    readers' albumentations pipeline runs on the GPU."""
    model.train()
    train_loss = 0.0
    it = train_loader
    bar = None
    if progress and tqdm is not None and _is_rank0():
        bar = it = tqdm(train_loader, desc=f"Epoch {epoch + 1}/{epochs} [Train]", leave=True, position=0,
                        bar_format="{l_bar}{bar:20}{r_bar}{bar:-20b}")
    nb = 0
    for inputs, targets in it:
        inputs = inputs.to(device, non_blocking=True)
        targets = targets.to(device, non_blocking=True)
        if augment is not None:  # per-(rank, epoch, batch) parameter stream
            rank = torch.distributed.get_rank() if not _is_rank0() else 0
            rng = np.random.Generator(np.random.PCG64([rank, epoch, nb]))
            inputs, targets = augment(inputs, targets, rng=rng)
        optimizer.zero_grad()
        loss = compute_loss(model, criterion, inputs, targets)
        loss.backward()
        sync = getattr(model, "finish_gradient_sync", None)
        if sync is not None:
            sync()
        _check_labels(model, inputs)  # before the update, on every rank (nn.CrossEntropyLoss raises in the forward)
        optimizer.step()
        lv = loss.item()
        train_loss += lv
        nb += 1
        if bar is not None:
            bar.set_postfix(loss=f"{lv:.4f}")
    n = len(train_loader) if hasattr(train_loader, "__len__") else max(nb, 1)
    return train_loss / max(n, 1)


def train_model(model, train_loader, criterion, optimizer, device, epochs=10,
                checkpoint_pattern: str | None = "Models/obj/obj_MOB_1_epoch_{epoch}.pth", progress: bool = True,
                augment=None):
    """Train for `epochs` epochs (src/train.py:6-79)."""
    best_val_loss = float("inf")  # validation is disabled in the reference (src/train.py:46-76)
    for epoch in range(epochs):
        sampler = getattr(train_loader, "sampler", None)
        if hasattr(sampler, "set_epoch"):
            sampler.set_epoch(epoch)  # DistributedWeightedSampler: a new shared draw per epoch
        avg_train_loss = train_one_epoch(model, train_loader, criterion, optimizer, device, epoch, epochs, progress,
                                         augment)
        if _is_rank0():
            print(f"  Training Loss: {avg_train_loss:.4f}")
            if checkpoint_pattern:
                path = checkpoint_pattern.format(epoch=epoch + 1)
                os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
                core = getattr(model, "module", model)
                torch.save(core.state_dict(), path)
    if _is_rank0():
        print(f"Training completed. Best validation loss: {best_val_loss:.4f}")
