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
  * `finish_gradient_sync()` (called by the engine at the end of the backward)
    makes the compute stream wait for the outstanding all-reduces (RCCL
    averages in the reduction, ncclAvg); autograd receives views of a copy of
    each bucket (`autograd_grads`), never the bucket itself;
  * BN running statistics are views of one flat tensor: one broadcast per step;
  * the fused loss's out-of-range label count rides in one extra slot of the last
    bucket, so after the all-reduce every rank holds the mean count (non-zero iff
    any rank saw a bad label) with no collective of its own (label_flag).
The unused `backbone.classifier` parameters never receive gradients (as in
the reference, where Adam skips them), so no find_unused_parameters dance.
"""
from __future__ import annotations

import contextlib

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
        # RCCL averages inside the reduction (ncclAvg); gloo has no AVG: SUM, then one scale
        self._avg = dist.get_backend(process_group) == "nccl"
        self._buckets = None
        self._slot = {}      # id(param) -> (bucket, offset)
        self._order = None
        self._bn_flat = None
        self._replace_grads = False  # a bucket folded held .grad values in (see _launch)
        self._flag_sent = False      # this step's label count went out with the last bucket (label_flag)
        self._hooks = None           # CPU path: post-accumulate-grad hooks (_arm_cpu)
        self._cpu_armed = False
        module.__dict__["_segamd_sync"] = self  # plain attribute: not a registered submodule
        if init_sync:
            self._broadcast_state()
        if broadcast_buffers:
            self._flatten_buffers()

    # ---------------------------------------------------------------- setup
    @torch.no_grad()
    def _broadcast_state(self):
        for t in list(self.module.parameters()) + list(self.module.buffers()):
            dist.broadcast(t.data, 0, group=self.pg)

    @torch.no_grad()
    def _flatten_buffers(self):
        """Rebind every floating-point buffer (BN running statistics) as a view of one
        persistent flat tensor, so the per-step broadcast is a single collective with no
        gather / scatter copies.  load_state_dict copies in place, so the views survive."""
        mods = [(m, n, b) for m in self.module.modules() for n, b in m._buffers.items()
                if b is not None and b.is_floating_point()]
        if not mods:
            return
        dev, dt = mods[0][2].device, mods[0][2].dtype
        if any(b.device != dev or b.dtype != dt for _, _, b in mods):
            return  # mixed placement: keep the per-buffer tensors (broadcast falls back below)
        flat = torch.empty(sum(b.numel() for _, _, b in mods), device=dev, dtype=dt)
        off = 0
        for m, n, b in mods:
            v = flat[off:off + b.numel()].view_as(b)
            v.copy_(b)
            m._buffers[n] = v
            off += b.numel()
        self._bn_flat = flat

    @torch.no_grad()
    def _broadcast_bn_buffers(self):
        if self._bn_flat is not None:
            dist.broadcast(self._bn_flat, 0, group=self.pg)
            return
        for b in self.module.buffers():
            if b.is_floating_point():
                dist.broadcast(b, 0, group=self.pg)

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
        for b in buckets:  # the last bucket carries one more float: the batch's out-of-range label count
            b.buf = torch.zeros(b.numel + (b is buckets[-1]), device=dev, dtype=ordered_params[0].dtype)
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
                self._launch(b)

    # --- launch-tape form (engine recording): a host stop only where a bucket completes (the
    # world-1 RCCL block measured 62 stops per step at ~11 us of host time each, one per layer with parameters)
    def begin_record(self):
        """A backward is being recorded: restart the record-time count of each bucket's outstanding parameters."""
        self._shadow = [len(b.params) for b in self._buckets] if self._buckets is not None else None

    def plan_ready(self, params):
        """Record time: the buckets that `params` completes (indices), from the record-time counts; the engine
        records a tape stop only when this is non-empty and replays launch_ready(those) there."""
        if getattr(self, "_shadow", None) is None:
            self.begin_record()
        done = []
        for p in params:
            slot = self._slot.get(id(p))
            if slot is None:
                continue
            self._shadow[slot[0]] -= 1
            if self._shadow[slot[0]] == 0:
                done.append(slot[0])
        return done

    def launch_ready(self, idx):
        """Replay time: all-reduce the buckets a recorded readiness point completed."""
        for bi in idx:
            b = self._buckets[bi]
            b.pending = 0
            self._launch(b)

    def _launch(self, b):
        """All-reduce bucket `b` (asynchronous, on the current stream's RCCL queue).  Like
        torch DDP, what is reduced is the gradient .grad would hold after this backward's
        accumulation: the engine wrote this backward's gradients into the bucket, so any
        .grad already held (micro-batches under no_sync(), or no zero_grad between steps)
        is added in first; autograd_grads then REPLACES .grad with the average."""
        held = [(self.grad_storage(p), p.grad) for p in b.params if p.grad is not None]
        if held:
            torch._foreach_add_([v for v, _ in held], [g for _, g in held])
            self._replace_grads = True
        if b is self._buckets[-1]:
            # piggyback the fused loss's out-of-range label count (written by the forward's loss kernel, earlier on
            # this stream): averaged with the gradients, no collective of its own
            st = self.module.__dict__.get("_segamd_last_stats")
            if st is not None and st.device == b.buf.device:
                b.buf[-1:].copy_(st[2:3])
            else:
                b.buf[-1:].zero_()
            self._flag_sent = True
        op = dist.ReduceOp.AVG if self._avg else dist.ReduceOp.SUM
        b.handle = dist.all_reduce(b.buf, op=op, group=self.pg, async_op=True)

    def _arm(self):
        for b in self._buckets:
            b.pending = len(b.params)
            b.handle = None
        self._flag_sent = False

    def label_flag(self):
        """The out-of-range label count of this step's fused loss, averaged over the ranks (so non-zero on every
        rank iff any rank saw such a label): a [1] fp32 device view, valid in stream order after
        finish_gradient_sync(); None when this step's buckets did not go out (no_sync, unfused criterion path)."""
        if self._buckets is None or not self._flag_sent or self.module.__dict__.get("_segamd_last_stats") is None:
            return None
        return self._buckets[-1].buf[-1:]

    def finish_gradient_sync(self):
        """Wait (stream-ordered) for every bucket's all-reduce; the buckets then hold the mean."""
        if self._buckets is None:
            return
        for b in self._buckets:
            if b.handle is None:
                # never launched (no gradient this step) or already finished
                if 0 < b.pending < len(b.params):
                    raise RuntimeError("segamd DDP: partially-ready gradient bucket")
                continue
            b.handle.wait()  # stream-ordered: the compute stream waits for RCCL, the host does not
            if not self._avg:
                b.buf.mul_(1.0 / self.world)
            b.handle = None

    def autograd_grads(self, params):
        """The averaged gradients handed to autograd: views of a fresh copy of each bucket
        (one copy kernel per bucket, stream-ordered after the all-reduce).  A .grad must
        never alias a bucket -- the next backward writes the bucket before AccumulateGrad
        runs, so with gradient accumulation p.grad += g would add the new gradient to
        itself."""
        copies = {}
        out = []
        if self._replace_grads:  # the buckets already include the held .grad values
            for p in params:
                if id(p) in self._slot:
                    p.grad = None
            self._replace_grads = False
        for p in params:
            slot = self._slot.get(id(p))
            if slot is None:
                out.append(None)
                continue
            k, off = slot
            c = copies.get(k)
            if c is None:
                c = copies[k] = self._buckets[k].buf.clone()
            out.append(c[off:off + p.numel()].view_as(p))
        return out

    @contextlib.contextmanager
    def no_sync(self):
        """As torch DDP's no_sync(): backward passes inside the context keep their
        gradients local and accumulate them into .grad; the first synchronised backward
        after it all-reduces .grad + its own gradients (see _launch), so every rank ends
        with the average of the accumulated sums."""
        d = self.module.__dict__
        saved = d.pop("_segamd_sync", None)
        try:
            yield
        finally:
            if saved is not None:
                d["_segamd_sync"] = saved

    # ------------------------------------------------------ CPU (torch-op) forward
    def _cpu_hook(self, p):
        """Post-accumulate-grad hook of the CPU path (main.py's CPU device runs the torch
        composition, seg_amd/export.py): when a bucket's .grads are all accumulated, pack
        them, all-reduce (gloo) and write the average back -- torch DDP's reducer."""
        if not self._cpu_armed:
            return
        k, _ = self._slot[id(p)]
        b = self._buckets[k]
        b.pending -= 1
        if b.pending:
            return
        with torch.no_grad():
            for q in b.params:
                v = self.grad_storage(q)
                v.copy_(q.grad) if q.grad is not None else v.zero_()
            dist.all_reduce(b.buf, op=dist.ReduceOp.SUM, group=self.pg)
            b.buf.mul_(1.0 / self.world)
            for q in b.params:
                if q.grad is not None:
                    q.grad.copy_(self.grad_storage(q))

    def _arm_cpu(self):
        if self._hooks is None:
            self._hooks = [p.register_post_accumulate_grad_hook(self._cpu_hook)
                           for b in self._buckets for p in b.params]
        for b in self._buckets:
            b.pending = len(b.params)
        self._cpu_armed = True

    # --------------------------------------------------------------- forward
    def _pre(self, x):
        self._cpu_armed = False
        if self.module.__dict__.get("_segamd_sync") is self:
            self._ensure_plan(x)
            if x.device.type == "cpu":
                self._arm_cpu()
            else:
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
