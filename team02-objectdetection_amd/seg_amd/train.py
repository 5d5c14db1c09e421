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


def _raise_bad_labels(n: float):
    if n:
        raise IndexError("Target out of bounds: label(s) outside [0, num_classes) that are not ignore_index "
                         "(nn.CrossEntropyLoss raises on these; the optimizer step was skipped)")


def _check_labels(model, inputs):
    """Raise IndexError like nn.CrossEntropyLoss if the fused loss saw a label outside
    [0, C) (the kernels flag it; the loss and gradients are NaN), BEFORE optimizer.step():
    the path for optimizers that cannot skip their step on the device.  Under
    seg_amd.ddp.DataParallel the count arrived with the last gradient bucket's all-reduce
    (every rank raises together, no extra collective).  When it did not (a no_sync step, or
    another wrapper under torch.distributed) the counts are summed over the ranks by an
    all-reduce of their own, so a peer never blocks in the next collective; in one
    process it was copied to the host right after the loss kernel, so this waits for the
    forward only."""
    if not inputs.is_cuda:
        return  # the CPU composition's F.cross_entropy raises by itself
    from .engine import bad_label_count, bad_label_count_host, label_flag
    if hasattr(model, "label_flag"):
        flag = label_flag(model)
        if flag is not None:
            _raise_bad_labels(float(flag.item()))
            return
    if torch.distributed.is_available() and torch.distributed.is_initialized():
        bad = bad_label_count(model)
        bad = torch.zeros(1, dtype=torch.float32, device=inputs.device) if bad is None else bad
        torch.distributed.all_reduce(bad)
        _raise_bad_labels(float(bad.item()))
        return
    n = bad_label_count_host(model)
    _raise_bad_labels(n or 0)


def _step_and_loss(model, inputs, optimizer, loss):
    """optimizer.step() and loss.item() (src/train.py:39-41) with the fused loss's label check.  With seg_amd.Adam
    the step is queued at once and skips itself on the device when the batch (on any rank) had an out-of-range
    label; the host reads the flag after loss.item(), whose wait covers it, and raises -- no host wait before the
    step and no extra collective.  Other optimizers: the check runs before the step."""
    from .optim import Adam
    from .engine import label_flag
    flag = label_flag(model) if inputs.is_cuda else None
    if flag is None or not isinstance(optimizer, Adam):
        _check_labels(model, inputs)
        optimizer.step()
        return loss.item()
    core = getattr(model, "module", model)
    host = core.__dict__.get("_segamd_flag_host")
    if host is None:
        host = core.__dict__["_segamd_flag_host"] = torch.zeros(1, dtype=torch.float32).pin_memory()
    host.copy_(flag, non_blocking=True)  # stream-ordered before the step and the loss copy below
    optimizer.step(skip_if_nonzero=flag)
    lv = loss.item()                     # waits for this stream: the flag copy has landed
    if float(host[0]):
        optimizer.undo_step_count()      # the device skipped the step: its counters go back too
        _raise_bad_labels(float(host[0]))
    return lv


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
        # the update never sees an out-of-range label's NaN gradients, on any rank (nn.CrossEntropyLoss raises in
        # the forward): seg_amd.Adam skips its step on the device, everything else is checked before the step
        lv = _step_and_loss(model, inputs, optimizer, loss)
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
