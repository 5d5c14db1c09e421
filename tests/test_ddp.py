"""CPU, world_size 2 over gloo: the data-parallel gradient path (seg_amd/ddp.py).

The GPU engine cannot run here, so the test drives DataParallel exactly the way
the engine's backward does (Run.grad_param -> grad_storage, Run.params_done ->
on_ready, end of backward -> finish_gradient_sync) with rank-specific gradients,
and checks: initial parameter broadcast, bucket plan (every used parameter once,
in the engine's backward order, classifier excluded), asynchronous bucket
all-reduce launched as buckets fill, and the averaged result.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, results):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from seg_amd import MobileNetV2UNet
        from seg_amd.ddp import DataParallel
        from seg_amd.detinit import deterministic_init
        from seg_amd.engine import get_program

        model = deterministic_init(MobileNetV2UNet(10), seed=100 + rank)   # ranks start different
        dp = DataParallel(model, bucket_cap_mb=2.0)
        # 1. parameters and buffers now equal rank 0's
        ref = deterministic_init(MobileNetV2UNet(10), seed=100)
        for (k, a), b in zip(model.state_dict().items(), ref.state_dict().values()):
            assert torch.equal(a, b), k
        # 2. bucket plan follows the engine's backward order
        x = torch.zeros(2, 3, 64, 64)
        dp._ensure_plan(x)
        prog = get_program(model, 2, 64, 64)
        order = []
        for op in reversed(prog.ops):
            for p in op.params():
                if all(p is not q for q in order):
                    order.append(p)
        planned = [p for b in dp._buckets for p in b.params]
        assert len(planned) == len(order) == 194
        assert all(a is b for a, b in zip(planned, order))
        assert all(b.numel <= dp.bucket_cap or len(b.params) == 1 for b in dp._buckets)
        classifier = {id(p) for p in model.backbone.classifier.parameters()}
        assert not any(id(p) in classifier for p in planned)
        # 3. one simulated backward: write rank-specific grads, announce per layer
        dp._arm()
        launched_before_end = 0
        for op in reversed(prog.ops):
            ps = op.params()
            for p in ps:
                g = dp.grad_storage(p)
                g.copy_(torch.full_like(p, float(rank + 1)) * (1 + torch.arange(p.numel()).view_as(p) % 7))
            dp.on_ready(ps)
            launched_before_end = sum(b.handle is not None for b in dp._buckets)
        assert launched_before_end == len(dp._buckets)  # every bucket launched during the backward
        dp.finish_gradient_sync()
        dp.finish_gradient_sync()  # idempotent (train_model and the engine may both call it)
        ok = True
        for p in planned:
            g = dp.grad_storage(p)
            expect = torch.full_like(p, 1.5) * (1 + torch.arange(p.numel()).view_as(p) % 7)  # mean of 1 and 2
            ok &= torch.allclose(g, expect)
        # 4. autograd receives copies: no .grad may alias a bucket (gradient accumulation
        #    would otherwise add the next backward's bucket contents to themselves)
        ag = dp.autograd_grads(planned)
        for p, g in zip(planned, ag):
            ok &= torch.equal(g, dp.grad_storage(p))
            ok &= g.untyped_storage().data_ptr() != dp.grad_storage(p).untyped_storage().data_ptr()
        # 5. BN running statistics are views of one flat buffer: one broadcast per step
        flat = dp._bn_flat
        ok &= flat is not None
        for n, b in model.named_buffers():
            if b.is_floating_point():
                ok &= b.untyped_storage().data_ptr() == flat.untyped_storage().data_ptr()
        bn = model.up1.conv.conv[1]
        bn.running_mean.fill_(float(rank + 3))
        dp._broadcast_bn_buffers()
        ok &= torch.equal(bn.running_mean, torch.full_like(bn.running_mean, 3.0))  # rank 0's value
        # state_dict / load_state_dict keep working through the views
        sd = {k: v.clone() for k, v in model.state_dict().items()}
        sd["up1.conv.conv.1.running_var"].fill_(2.0)
        model.load_state_dict(sd)
        ok &= bool((model.up1.conv.conv[1].running_var == 2.0).all())
        ok &= model.up1.conv.conv[1].running_var.untyped_storage().data_ptr() == flat.untyped_storage().data_ptr()
        # 6. no_sync(): the engine sees no gradient-sync object inside the context
        with dp.no_sync():
            ok &= model.__dict__.get("_segamd_sync") is None
        ok &= model.__dict__.get("_segamd_sync") is dp
        results[rank] = bool(ok)
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_ddp_bucketed_allreduce_gloo():
    world = 2
    mgr = mp.Manager()
    results = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), results), nprocs=world, join=True)
    assert dict(results) == {0: True, 1: True}


def _train_worker(rank, world, port, results):
    """Real training steps of a CPU model under DataParallel (the torch-op composition;
    the reducer is DataParallel's post-accumulate-grad hooks): a step with one
    micro-batch under no_sync() followed by a synchronised one, then a plain step."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.set_num_threads(2)
        from seg_amd import UNet
        from seg_amd.ddp import DataParallel
        from seg_amd.detinit import deterministic_init, synthetic_batch
        model = deterministic_init(UNet(4, 8), seed=50 + rank)  # broadcast makes them equal
        dp = DataParallel(model, bucket_cap_mb=0.05)
        assert len(dp._buckets or []) == 0
        out = []
        xs = [synthetic_batch(2, 32, 64, 4, seed=10 * rank + k) for k in range(3)]
        model.zero_grad(set_to_none=True)
        with dp.no_sync():
            dp.forward_loss(*xs[0]).backward()
        dp.forward_loss(*xs[1]).backward()
        out.append({k: p.grad.clone() for k, p in model.named_parameters() if p.grad is not None})
        model.zero_grad(set_to_none=True)
        dp.forward_loss(*xs[2]).backward()
        out.append({k: p.grad.clone() for k, p in model.named_parameters() if p.grad is not None})
        results[rank] = (out, len(dp._buckets), {k: v.clone() for k, v in model.state_dict().items()})
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_ddp_cpu_no_sync_accumulation_gloo():
    """gradients accumulated under no_sync() must be averaged by the next
    synchronised backward -- .grad identical on both ranks and equal to the mean over
    ranks of each rank's (micro-batch 0 + micro-batch 1) gradients, as torch DDP."""
    world = 2
    mgr = mp.Manager()
    results = mgr.dict()
    mp.spawn(_train_worker, args=(world, _free_port(), results), nprocs=world, join=True)
    (o0, nb0, s0), (o1, nb1, s1) = results[0], results[1]
    assert nb0 == nb1 > 1
    from seg_amd import UNet
    from seg_amd.detinit import deterministic_init, synthetic_batch
    # single-process reference: each rank's local gradients from rank 0's initial weights
    local = []
    for r in range(world):
        m = deterministic_init(UNet(4, 8), seed=50)
        xs = [synthetic_batch(2, 32, 64, 4, seed=10 * r + k) for k in range(3)]
        m.zero_grad(set_to_none=True)
        m.forward_loss(*xs[0]).backward()
        m.forward_loss(*xs[1]).backward()
        acc = {k: p.grad.clone() for k, p in m.named_parameters() if p.grad is not None}
        m.zero_grad(set_to_none=True)
        m.forward_loss(*xs[2]).backward()
        local.append((acc, {k: p.grad.clone() for k, p in m.named_parameters() if p.grad is not None}))
    for step in range(2):
        g0, g1 = o0[step], o1[step]
        assert g0.keys() == g1.keys() == local[0][step].keys()
        for k in g0:
            assert torch.equal(g0[k], g1[k]), (step, k)
            mean = (local[0][step][k] + local[1][step][k]) * 0.5
            assert torch.allclose(g0[k], mean, rtol=1e-4, atol=1e-6), (step, k)
