"""GPU: the data-parallel path (seg_amd/ddp.py) on the real engine and RCCL, world size 1
(the multi-rank semantics are covered over gloo in tests/test_ddp.py; one GPU per box
here).  Bucket hooks fire from the side-stream weight gradients, all-reduces run on
RCCL's stream and the averaged gradients must equal the plain model's bitwise -- with
torch.optim.Adam and with seg_amd.Adam stepping the bucket-view gradients."""
import os
import socket

import pytest
import torch
import torch.distributed as dist

from seg_amd import Adam, MobileNetV2UNet, engine
from seg_amd.ddp import DataParallel
from seg_amd.detinit import deterministic_init, synthetic_batch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def pg():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1)
    yield
    dist.destroy_process_group()


@pytest.mark.parametrize("optim", ["torch", "seg"])
@pytest.mark.parametrize("math", ["f32", "bf16io"])
def test_ddp_world1_matches_plain(pg, math, optim):
    x, y = synthetic_batch(2, 64, 128, 10, seed=3)
    x, y = x.to(DEV), y.to(DEV)
    res = []
    for wrap in (False, True):
        m = deterministic_init(MobileNetV2UNet(10), seed=9).to(DEV).train()
        engine.set_conv_math(m, math)
        model = DataParallel(m, bucket_cap_mb=1.0) if wrap else m
        opt = (Adam if optim == "seg" else torch.optim.Adam)(model.parameters(), lr=1e-3)
        losses = []
        for _ in range(3):
            opt.zero_grad(set_to_none=True)
            loss = model.forward_loss(x, y)
            loss.backward()
            if wrap:
                model.finish_gradient_sync()
            opt.step()
            losses.append(loss.item())
        torch.cuda.synchronize()
        grads = {k: p.grad.clone() for k, p in m.named_parameters() if p.grad is not None}
        res.append((losses, grads, {k: v.clone() for k, v in m.state_dict().items()}))
    (l0, g0, s0), (l1, g1, s1) = res
    assert l0 == l1
    assert g0.keys() == g1.keys()
    for k in g0:
        assert torch.equal(g0[k], g1[k]), k
    for k in s0:
        assert torch.equal(s0[k], s1[k]), k


@pytest.mark.parametrize("set_to_none", [True, False])
def test_ddp_world1_grad_accumulation(pg, set_to_none):
    """Two micro-batches accumulated into .grad (and zero_grad(set_to_none=False)) must
    give g1 + g2 exactly as the plain model does: autograd never receives the bucket
    itself, so the second backward cannot overwrite an aliased .grad."""
    xs = [synthetic_batch(2, 64, 128, 10, seed=s) for s in (5, 6)]
    res = []
    for wrap in (False, True):
        m = deterministic_init(MobileNetV2UNet(10), seed=4).to(DEV).train()
        model = DataParallel(m, bucket_cap_mb=1.0) if wrap else m
        for step in range(2):
            model.zero_grad(set_to_none=set_to_none)
            for x, y in xs:
                model.forward_loss(x.to(DEV), y.to(DEV)).backward()
        torch.cuda.synchronize()
        res.append({k: p.grad.clone() for k, p in m.named_parameters() if p.grad is not None})
    g0, g1 = res
    assert g0.keys() == g1.keys() and len(g0) == 194
    for k in g0:
        assert torch.equal(g0[k], g1[k]), k


def test_ddp_world1_held_bias_grads_not_refolded(pg):
    """Conv biases in front of train-mode BatchNorm get an exact-zero gradient whose slot in
    the all-reduced bucket must be re-zeroed every step: a synchronised backward folds the
    .grad a rank still holds into the bucket, so a slot zeroed only once would keep that fold
    and double it on the next step.  Three backwards without zero_grad, each
    followed by an in-place change of every .grad (a manual L2 term), against the plain model."""
    x, y = synthetic_batch(2, 64, 128, 10, seed=12)
    x, y = x.to(DEV), y.to(DEV)
    res = []
    for wrap in (False, True):
        m = deterministic_init(MobileNetV2UNet(10), seed=13).to(DEV).train()
        model = DataParallel(m, bucket_cap_mb=1.0) if wrap else m
        for _ in range(3):
            model.forward_loss(x, y).backward()
            if wrap:
                model.finish_gradient_sync()
            with torch.no_grad():
                for p in m.parameters():
                    if p.grad is not None:
                        p.grad.add_(p.detach(), alpha=1e-3)
        torch.cuda.synchronize()
        res.append({k: p.grad.clone() for k, p in m.named_parameters() if p.grad is not None})
    g0, g1 = res
    biases = [k for k in g0 if k.startswith("up") and k.endswith("bias") and ".conv.conv." in k]
    assert biases, "the decoder's pre-BatchNorm conv biases"
    for k in g0:
        assert torch.equal(g0[k], g1[k]), k
