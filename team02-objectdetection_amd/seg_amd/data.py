"""Data-parallel data path of the reference's main.py.

The reference builds one `CombinedLaneDataset` over BDD100K / SEA / Carla
(src/CombinedDataset.py:8-205), weights its samples for a
`WeightedRandomSampler(weights, num_samples=len(weights), replacement=True)`
(main.py:62-87) and feeds a `DataLoader(batch_size=8, sampler=...)`
(main.py:90-95).  The per-dataset readers (cv2 decode + albumentations) are
host IO and out of scope; this module keeps everything between them and the
GPU step, made rank-aware:

  * `CombinedLaneDataset` -- the reference's index routing over any three
    map-style datasets, bit-for-bit: Python `random.seed(seed)` shuffles of the
    SEA, Carla and BDD100K index lists in that order, `int(size * val_split)`
    validation heads, train order BDD100K -> SEA -> Carla, validation order
    BDD100K -> SEA -> Carla.  The reference's training branch indexes
    `bdd100k_indices` (ALL BDD100K samples, src/CombinedDataset.py:181) rather
    than `bdd100k_train_indices`, so with val_split > 0 validation samples leak
    into training; that behaviour is kept (`fix_bdd_train_leak=True` opts out).
  * `reference_sample_weights` -- main.py:62-78's weights, including its quirk
    that Carla samples (indices past BDD100K + SEA) get the SEA weight.
  * `DistributedWeightedSampler` -- the global `torch.multinomial` draw of
    `WeightedRandomSampler` from a generator seeded identically on every rank
    (seed + epoch), then rank r keeps draws r, r+W, r+2W, ...  Step s of every
    rank's DataLoader together covers global draws [s*B*W, (s+1)*B*W): the
    union over ranks of one step is one contiguous global batch.  At W = 1 the
    index stream equals torch's WeightedRandomSampler with the same generator.
"""
from __future__ import annotations

import random

import numpy as np
import torch
from torch.utils.data import Dataset, Sampler


class CombinedLaneDataset(Dataset):
    """src/CombinedDataset.py:8-205 over already-constructed datasets."""

    def __init__(self, sea_dataset=None, carla_dataset=None, bdd100k_dataset=None, val_split: float = 0.2,
                 seed: int = 42, fix_bdd_train_leak: bool = False, verbose: bool = True):
        self.val_split = val_split
        self.seed = seed
        self.sea_dataset, self.carla_dataset, self.bdd100k_dataset = sea_dataset, carla_dataset, bdd100k_dataset
        self.fix_bdd_train_leak = fix_bdd_train_leak
        rng = random.Random(seed)  # == random.seed(seed) then the module-level shuffles (src/CombinedDataset.py:24,82-87)
        self.sea_size = len(sea_dataset) if sea_dataset is not None else 0
        self.carla_size = len(carla_dataset) if carla_dataset is not None else 0
        self.bdd100k_size = len(bdd100k_dataset) if bdd100k_dataset is not None else 0
        self.sea_indices = list(range(self.sea_size))
        self.carla_indices = list(range(self.carla_size))
        self.bdd100k_indices = list(range(self.bdd100k_size))
        if self.sea_size > 0:
            rng.shuffle(self.sea_indices)
        if self.carla_size > 0:
            rng.shuffle(self.carla_indices)
        if self.bdd100k_size > 0:
            rng.shuffle(self.bdd100k_indices)
        sv = int(self.sea_size * val_split)
        cv = int(self.carla_size * val_split)
        bv = int(self.bdd100k_size * val_split)
        self.sea_train_indices, self.sea_val_indices = self.sea_indices[sv:], self.sea_indices[:sv]
        self.carla_train_indices, self.carla_val_indices = self.carla_indices[cv:], self.carla_indices[:cv]
        self.bdd100k_train_indices, self.bdd100k_val_indices = self.bdd100k_indices[bv:], self.bdd100k_indices[:bv]
        self.sea_train_size, self.sea_val_size = len(self.sea_train_indices), len(self.sea_val_indices)
        self.carla_train_size, self.carla_val_size = len(self.carla_train_indices), len(self.carla_val_indices)
        self.bdd100k_train_size = len(self.bdd100k_train_indices)
        self.bdd100k_val_size = len(self.bdd100k_val_indices)
        self.train_size = self.bdd100k_train_size + self.sea_train_size + self.carla_train_size
        self.val_size = self.bdd100k_val_size + self.sea_val_size + self.carla_val_size
        self.total_size = self.train_size + self.val_size
        self.is_validation = False
        if verbose:
            print("Combined dataset created:")
            if self.sea_size > 0:
                print(f"SEA: {self.sea_train_size} train, {self.sea_val_size} validation")
            if self.carla_size > 0:
                print(f"Carla: {self.carla_train_size} train, {self.carla_val_size} validation")
            if self.bdd100k_size > 0:
                print(f"BDD100K: {self.bdd100k_train_size} train, {self.bdd100k_val_size} validation")
            print(f"Total: {self.train_size} train, {self.val_size} validation")

    def set_validation(self, is_validation: bool = True):
        self.is_validation = is_validation
        for d in (self.sea_dataset, self.carla_dataset, self.bdd100k_dataset):
            if d is not None and hasattr(d, "is_train"):
                d.is_train = not is_validation
        return self

    def __len__(self):
        return self.val_size if self.is_validation else self.train_size

    def route(self, idx: int):
        """(source name, index inside that source) of sample `idx` in the current mode."""
        if self.is_validation:
            b, s, c = self.bdd100k_val_size, self.sea_val_size, self.carla_val_size
            if idx < b:
                return "bdd100k", self.bdd100k_val_indices[idx]
            if idx < b + s:
                return "sea", self.sea_val_indices[idx - b]
            if idx < b + s + c:
                return "carla", self.carla_val_indices[idx - b - s]
            return "bdd100k", self.bdd100k_val_indices[idx - b - s - c]
        b, s, c = self.bdd100k_train_size, self.sea_train_size, self.carla_train_size
        if idx < b:
            src = self.bdd100k_train_indices if self.fix_bdd_train_leak else self.bdd100k_indices
            return "bdd100k", src[idx]
        if idx < b + s:
            return "sea", self.sea_train_indices[idx - b]
        if idx < b + s + c:
            return "carla", self.carla_train_indices[idx - b - s]
        return "bdd100k", self.bdd100k_train_indices[idx - b - s - c]

    def __getitem__(self, idx):
        name, i = self.route(idx)
        return {"bdd100k": self.bdd100k_dataset, "sea": self.sea_dataset, "carla": self.carla_dataset}[name][i]

    def get_train_dataset(self):
        return self.set_validation(False)

    def get_val_dataset(self):
        return self.set_validation(True)


def reference_sample_weights(train_dataset) -> np.ndarray:
    """main.py:62-78: 50 % BDD100K / 20 % SEA / 30 % Carla intent; as written, every
    sample past BDD100K (SEA and Carla alike) gets the SEA weight."""
    nb, ns, nc = train_dataset.bdd100k_train_size, train_dataset.sea_train_size, train_dataset.carla_train_size
    weights = np.zeros(train_dataset.train_size)
    total = nb + ns
    bdd_w = 0.5 / (nb / total) if nb > 0 else 0
    sea_w = 0.2 / (ns / total) if ns > 0 else 0
    weights[:nb] = bdd_w
    weights[nb:] = sea_w
    return weights


class DistributedWeightedSampler(Sampler):
    """Rank shard of one global WeightedRandomSampler draw (see the module docstring).

    weights, num_samples, replacement: as torch.utils.data.WeightedRandomSampler.
    seed: shared by every rank; the draw of epoch e uses torch.Generator seeded
    with seed + e (call set_epoch(e) each epoch, like DistributedSampler).
    """

    def __init__(self, weights, num_samples: int | None = None, replacement: bool = True, seed: int = 0,
                 rank: int | None = None, world_size: int | None = None):
        if rank is None or world_size is None:
            init = torch.distributed.is_available() and torch.distributed.is_initialized()
            rank = torch.distributed.get_rank() if init else 0
            world_size = torch.distributed.get_world_size() if init else 1
        if not 0 <= rank < world_size:
            raise ValueError(f"rank {rank} outside world of {world_size}")
        self.weights = torch.as_tensor(np.asarray(weights), dtype=torch.double)
        self.num_samples = int(num_samples if num_samples is not None else len(self.weights))
        if self.num_samples <= 0:
            raise ValueError("num_samples must be positive")
        self.replacement, self.seed, self.rank, self.world = replacement, seed, rank, world_size
        self.epoch = 0

    def set_epoch(self, epoch: int):
        self.epoch = epoch

    def global_indices(self) -> torch.Tensor:
        g = torch.Generator()
        g.manual_seed(self.seed + self.epoch)
        return torch.multinomial(self.weights, self.num_samples, self.replacement, generator=g)

    def __iter__(self):
        idx = self.global_indices()
        per = self.num_samples // self.world
        return iter(idx[self.rank:per * self.world:self.world].tolist())

    def __len__(self):
        return self.num_samples // self.world
