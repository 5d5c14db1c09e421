"""Data parallelism for the segamd models: one process per GPU, RCCL all-reduce
of the gradients over xGMI, overlapped with the backward.

The reference has no distributed code ("Parallelism strategies:
none"); BASELINE.json's north_star asks for data-parallel training that shards
the minibatch across the 8 GPUs of a node.  Semantics = PyTorch DDP without
SyncBN: BatchNorm statistics are per rank (bs=32 each), the all-reduced
gradient is the mean of the per-rank gradients, and (optionally) BN buffers
are broadcast from rank 0 so eval weights are rank-independent.

Mechanism (no autograd hooks needed -- the engine IS the backward):
  * gradients live in flat per-bucket buffers (about `bucket_cap_mb` each,
    ordered by when the reverse program produces them: decoder first);
    the engine's kernels write each parameter's gradient straight into its
    slot (Run.grad_param -> grad_storage);
  * after each layer's gradients are complete the engine calls `on_ready`;
    when a bucket is full it is all-reduced asynchronously
    (torch.distributed -> RCCL on its own stream, ordered after the producing
    kernels on the compute stream), so communication of the decoder's 3.1 M
    `up1.conv.0` weights overlaps the encoder's backward;
  * `finish_gradient_sync()` (called by train_model before optimizer.step)
    makes the compute stream wait for the outstanding all-reduces and scales
    by 1/world.
The unused `backbone.classifier` parameters never receive gradients (as in
the reference, where Adam skips them), so no find_unused_parameters dance.
"""
from __future__ import annotations

import torch
import torch.distributed as dist
from torch import nn


class _Bucket:
    __slots__ = ("params", "numel", "buf", "pending", "handle")

    def __init__(self):
        self.params, self.numel, self.buf, self.pending, self.handle = [], 0, None, 0, None


class DataParallel(nn.Module):
    def __init__(self, module: nn.Module, process_group=None, bucket_cap_mb: float = 8.0,
                 broadcast_buffers: bool = True, init_sync: bool = True):
        super().__init__()
        self.module = module
        self.pg = process_group
        self.world = dist.get_world_size(process_group)
        self.bucket_cap = int(bucket_cap_mb * (1 << 20) / 4)
        self.broadcast_buffers = broadcast_buffers
        self._buckets = None
        self._slot = {}      # id(param) -> (bucket, offset)
        self._order = None
        module.__dict__["_segamd_sync"] = self  # plain attribute: not a registered submodule
        if init_sync:
            self._broadcast_state()

    # ---------------------------------------------------------------- setup
    @torch.no_grad()
    def _broadcast_state(self):
        for t in list(self.module.parameters()) + list(self.module.buffers()):
            dist.broadcast(t.data, 0, group=self.pg)

    @torch.no_grad()
    def _broadcast_bn_buffers(self):
        bufs = [b for n, b in self.module.named_buffers() if b.is_floating_point()]
        if not bufs:
            return
        flat = torch.cat([b.reshape(-1) for b in bufs])
        dist.broadcast(flat, 0, group=self.pg)
        off = 0
        for b in bufs:
            b.copy_(flat[off:off + b.numel()].view_as(b))
            off += b.numel()

    def plan_buckets(self, ordered_params):
        """Group parameters (in gradient-ready order) into ~bucket_cap buckets."""
        buckets, cur = [], _Bucket()
        for p in ordered_params:
            if not p.requires_grad:
                continue
            if cur.params and cur.numel + p.numel() > self.bucket_cap:
                buckets.append(cur)
                cur = _Bucket()
            self._slot[id(p)] = (len(buckets), cur.numel)
            cur.params.append(p)
            cur.numel += p.numel()
        if cur.params:
            buckets.append(cur)
        dev = ordered_params[0].device
        for b in buckets:
            b.buf = torch.zeros(b.numel, device=dev, dtype=ordered_params[0].dtype)
        self._buckets = buckets

    def _ensure_plan(self, x):
        if self._buckets is not None:
            return
        from .engine import get_program
        N, _, H, W = x.shape
        prog = get_program(self.module, N, H, W)
        order, seen = [], set()
        for op in reversed(prog.ops):   # the engine's backward order
            for p in op.params():
                if id(p) not in seen:
                    seen.add(id(p))
                    order.append(p)
        self.plan_buckets(order)

    # -------------------------------------------------------------- engine hooks
    def grad_storage(self, p):
        slot = self._slot.get(id(p))
        if slot is None:
            return None
        b, off = slot
        return self._buckets[b].buf[off:off + p.numel()].view_as(p)

    def on_ready(self, params, run=None):
        for p in params:
            slot = self._slot.get(id(p))
            if slot is None:
                continue
            b = self._buckets[slot[0]]
            b.pending -= 1
            if b.pending == 0:
                b.handle = dist.all_reduce(b.buf, op=dist.ReduceOp.SUM, group=self.pg, async_op=True)

    def _arm(self):
        for b in self._buckets:
            b.pending = len(b.params)
            b.handle = None

    def finish_gradient_sync(self):
        """Wait (stream-ordered) for every bucket's all-reduce and average."""
        if self._buckets is None:
            return
        for b in self._buckets:
            if b.handle is None:
                # never launched (no gradient this step) or already finished
                if 0 < b.pending < len(b.params):
                    raise RuntimeError("segamd DDP: partially-ready gradient bucket")
                continue
            b.handle.wait()  # stream-ordered: the compute stream waits for RCCL, the host does not
            b.buf.mul_(1.0 / self.world)
            b.handle = None

    # --------------------------------------------------------------- forward
    def _pre(self, x):
        self._ensure_plan(x)
        self._arm()
        if self.broadcast_buffers and self.module.training:
            self._broadcast_bn_buffers()

    def forward(self, x):
        self._pre(x)
        return self.module(x)

    def forward_loss(self, x, target, ignore_index: int = -100):
        self._pre(x)
        return self.module.forward_loss(x, target, ignore_index)

    def state_dict(self, *args, **kwargs):
        return self.module.state_dict(*args, **kwargs)

    def load_state_dict(self, *args, **kwargs):
        return self.module.load_state_dict(*args, **kwargs)
