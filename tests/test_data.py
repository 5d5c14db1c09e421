"""CPU: the data-parallel data path (seg_amd/data.py, main.py:50-95).

  * CombinedLaneDataset routing == the reference's own src/CombinedDataset.py on
    every case of tests/golden/combined_dataset_routing.json (made by
    tests/golden/make_data_golden.py from the reference), including its
    BDD100K train/validation leak (src/CombinedDataset.py:181);
  * reference_sample_weights == main.py:62-78 as written (Carla gets the SEA weight);
  * DistributedWeightedSampler at world 1 == torch's WeightedRandomSampler with the
    same generator; at world W the ranks' streams interleave back into that one
    global draw (checked in-process and across 2 gloo processes).
"""
import json
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
from torch.utils.data import DataLoader, WeightedRandomSampler

from seg_amd.data import CombinedLaneDataset, DistributedWeightedSampler, reference_sample_weights

GOLD = os.path.join(os.path.dirname(__file__), "golden", "combined_dataset_routing.json")


class Src:
    def __init__(self, tag, n):
        self.tag, self.n, self.is_train = tag, n, True

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        return (self.tag, i)


def build(nb, ns, nc, vs, seed, **kw):
    return CombinedLaneDataset(sea_dataset=Src("sea", ns) if ns else None, carla_dataset=Src("carla", nc) if nc else None,
                               bdd100k_dataset=Src("bdd100k", nb) if nb else None, val_split=vs, seed=seed,
                               verbose=False, **kw)


@pytest.mark.parametrize("case", json.load(open(GOLD)), ids=lambda c: f"{c['bdd100k']}-{c['sea']}-{c['carla']}-{c['val_split']}")
def test_routing_matches_reference(case):
    ds = build(case["bdd100k"], case["sea"], case["carla"], case["val_split"], case["seed"])
    assert ds.train_size == case["train_size"] and ds.val_size == case["val_size"]
    tr = ds.get_train_dataset()
    assert [list(tr[i]) for i in range(len(tr))] == case["train"]
    va = ds.get_val_dataset()
    assert [list(va[i]) for i in range(len(va))] == case["val"]


def test_leak_fix_option():
    ds = build(7, 5, 3, 0.3, 42, fix_bdd_train_leak=True).get_train_dataset()
    bdd_train = {ds[i][1] for i in range(ds.bdd100k_train_size)}
    assert bdd_train == set(ds.bdd100k_train_indices)
    assert not bdd_train & set(ds.bdd100k_val_indices)


def test_reference_weights():
    ds = build(6, 3, 2, 0.0, 42).get_train_dataset()
    w = reference_sample_weights(ds)
    total = 6 + 3
    assert np.allclose(w[:6], 0.5 / (6 / total)) and np.allclose(w[6:], 0.2 / (3 / total))  # Carla: SEA weight
    assert len(w) == ds.train_size


def test_world1_equals_weighted_random_sampler():
    w = np.random.Generator(np.random.PCG64(0)).uniform(0.1, 2.0, 57)
    ours = DistributedWeightedSampler(w, seed=5, rank=0, world_size=1)
    g = torch.Generator()
    g.manual_seed(5)
    ref = list(WeightedRandomSampler(torch.as_tensor(w, dtype=torch.double), len(w), True, generator=g))
    assert list(ours) == ref
    ours.set_epoch(1)
    assert list(ours) != ref


@pytest.mark.parametrize("world", [2, 3, 8])
def test_shards_interleave_to_global_draw(world):
    w = np.linspace(0.1, 1.0, 101)
    global_idx = DistributedWeightedSampler(w, seed=3, rank=0, world_size=1).global_indices().tolist()
    shards = [list(DistributedWeightedSampler(w, seed=3, rank=r, world_size=world)) for r in range(world)]
    per = len(w) // world
    assert all(len(s) == per for s in shards)
    merged = [shards[i % world][i // world] for i in range(per * world)]
    assert merged == global_idx[:per * world]
    # one DataLoader step per rank (batch B) covers a contiguous block of the global draw
    B = 4
    step0 = sorted(sum((s[:B] for s in shards), []))
    assert step0 == sorted(global_idx[:B * world])


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ds = build(40, 25, 15, 0.2, 123).get_train_dataset()
    sampler = DistributedWeightedSampler(reference_sample_weights(ds), seed=11)
    loader = DataLoader(ds, batch_size=4, sampler=sampler, collate_fn=list)
    mine = [item for batch in loader for item in batch]
    gathered = [None] * world
    dist.all_gather_object(gathered, mine)
    if rank == 0:
        out.put(gathered)
    dist.destroy_process_group()


def test_gloo_two_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + os.getpid() % 1000
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    gathered = q.get(timeout=120)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    ds = build(40, 25, 15, 0.2, 123).get_train_dataset()
    ref = DistributedWeightedSampler(reference_sample_weights(ds), seed=11, rank=0, world_size=1).global_indices()
    per = ds.train_size // 2
    expect = [[tuple(ds[int(i)]) for i in ref[r:2 * per:2]] for r in range(2)]
    assert [[tuple(x) for x in g] for g in gathered] == expect
