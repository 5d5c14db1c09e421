"""GPU: two ranks of the REAL engine (tape replay, side-stream parameter gradients,
bucket all-reduces at host-callback stops, flat BN-buffer broadcast) on the box's one
MI355X.  RCCL needs a device per rank, so the ranks talk over gloo here (CUDA tensors);
the engine-side path is the same one the driver's 8-GPU RCCL run takes.  Each rank
trains on its own shard; after every step its gradients must equal, bit for bit, the
mean of the two shards' gradients computed by a plain single-process model
((g0 + g1) * 0.5, the same fp32 ops gloo's SUM and the 1/world scale perform), and
both ranks' parameters and BN buffers must stay identical."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _shards():
    from seg_amd.detinit import synthetic_batch
    return [synthetic_batch(2, 64, 128, 10, seed=70 + r) for r in range(2)]


def _worker(rank, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    try:
        torch.cuda.set_device(0)
        from seg_amd import MobileNetV2UNet, deterministic_init
        from seg_amd.ddp import DataParallel
        m = deterministic_init(MobileNetV2UNet(10), seed=8).cuda().train()
        dp = DataParallel(m, bucket_cap_mb=1.0)
        opt = torch.optim.SGD(m.parameters(), lr=0.01)
        x, y = _shards()[rank]
        x, y = x.cuda(), y.cuda()
        res = []
        for _ in range(2):
            opt.zero_grad(set_to_none=True)
            loss = dp.forward_loss(x, y)
            loss.backward()
            res.append({k: p.grad.cpu() for k, p in m.named_parameters() if p.grad is not None})
            opt.step()
        out[rank] = (res, {k: p.detach().cpu() for k, p in m.named_parameters()})
    finally:
        dist.destroy_process_group()


def test_two_ranks_real_engine_match_single_process_mean():
    ctx = mp.get_context("spawn")
    out = ctx.Manager().dict()
    mp.spawn(_worker, args=(_port(), out), nprocs=2, join=True)
    (g0, s0), (g1, s1) = out[0], out[1]
    for k in s0:  # parameters stay identical across ranks (BN buffers re-sync at the next forward)
        assert torch.equal(s0[k], s1[k]), k
    # single-process reference: per-shard gradients of two plain models stepped in lockstep
    from seg_amd import MobileNetV2UNet, deterministic_init
    ms = [deterministic_init(MobileNetV2UNet(10), seed=8).cuda().train() for _ in range(2)]
    opts = [torch.optim.SGD(m.parameters(), lr=0.01) for m in ms]
    shards = _shards()
    for step in range(2):
        gs = []
        for m, o, (x, y) in zip(ms, opts, shards):
            o.zero_grad(set_to_none=True)
            m.forward_loss(x.cuda(), y.cuda()).backward()
            gs.append({k: p.grad.clone() for k, p in m.named_parameters() if p.grad is not None})
        mean = {k: (gs[0][k] + gs[1][k]) * 0.5 for k in gs[0]}
        assert set(mean) == set(g0[step]) and len(mean) == 194
        for k in mean:
            assert torch.equal(g0[step][k], mean[k].cpu()), (step, k)
            assert torch.equal(g1[step][k], mean[k].cpu()), (step, k)
        for m in ms:  # both replicas take the averaged step, as the ranks did
            for k, p in m.named_parameters():
                if k in mean:
                    p.grad = mean[k].clone()
        for o in opts:
            o.step()
        # DDP broadcasts rank 0's BN buffers each step: replica 1 adopts replica 0's
        for b0, b1 in zip(ms[0].buffers(), ms[1].buffers()):
            b1.copy_(b0)


def _bad_label_worker(rank, port, out):
    """Rank 1's batch has an out-of-range label: both ranks must raise from train_model, with every parameter
    unchanged, and the step must issue only the gradient buckets' all-reduces (the label count rides in the last
    bucket)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    try:
        torch.cuda.set_device(0)
        from torch import nn
        from seg_amd import Adam, MobileNetV2UNet, deterministic_init, train_model
        from seg_amd.ddp import DataParallel
        m = deterministic_init(MobileNetV2UNet(10), seed=8).cuda().train()
        dp = DataParallel(m, bucket_cap_mb=1.0)
        opt = Adam(m.parameters(), lr=1e-3)
        x, y = _shards()[rank]
        x, y = x.cuda(), y.cuda()
        calls = {"all_reduce": 0}
        real = dist.all_reduce

        def counting(*a, **k):
            calls["all_reduce"] += 1
            return real(*a, **k)
        dist.all_reduce = counting
        train_model(dp, [(x, y)], nn.CrossEntropyLoss(), opt, "cuda", epochs=1, checkpoint_pattern=None,
                    progress=False)  # a clean step first
        per_step = calls["all_reduce"]
        before = {k: p.detach().clone() for k, p in m.named_parameters()}
        if rank == 1:
            y = y.clone()
            y[0, 3, 3] = 10
        raised = False
        try:
            train_model(dp, [(x, y)], nn.CrossEntropyLoss(), opt, "cuda", epochs=1, checkpoint_pattern=None,
                        progress=False)
        except IndexError:
            raised = True
        dist.all_reduce = real
        unchanged = all(torch.equal(p.detach(), before[k]) for k, p in m.named_parameters())
        out[rank] = (raised, unchanged, per_step, calls["all_reduce"] - per_step, len(dp._buckets))
    finally:
        dist.destroy_process_group()


def test_bad_label_on_one_rank_raises_on_both_without_update():
    ctx = mp.get_context("spawn")
    out = ctx.Manager().dict()
    mp.spawn(_bad_label_worker, args=(_port(), out), nprocs=2, join=True)
    for r in (0, 1):
        raised, unchanged, per_step, bad_step, nb = out[r]
        assert raised, f"rank {r} did not raise"
        assert unchanged, f"rank {r} changed its parameters"
        assert per_step == nb and bad_step == nb, (per_step, bad_step, nb)  # the buckets only: no extra collective
