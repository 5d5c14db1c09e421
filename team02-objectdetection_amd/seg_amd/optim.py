"""Adam with a one-launch HIP step (csrc/adam.hip, seg_adam_step).

Drop-in for the reference's `optim.Adam(model.parameters(), lr=1.5e-4)` (main.py:100),
stepped once per batch by train_model (src/train.py:39): same constructor, same
param_groups and state_dict layout (state 'step' as a CPU tensor, 'exp_avg',
'exp_avg_sq'), so checkpoints move between the two.  torch's foreach Adam issues ~8
multi-tensor launches per step, each streaming the 6.5 M parameters' p / g / m / v
again; seg_adam_step reads and writes each element once with the same fp32 operation
order (see adam.hip).  Supported: the reference's configuration (no weight decay, no
amsgrad, not maximize) on CUDA fp32 dense tensors; anything else raises -- there is no
silent fallback.
"""
from __future__ import annotations

import torch

from ._lib import call

_CHUNK = 4096  # elements per block


class Adam(torch.optim.Adam):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0, amsgrad=False, **kw):
        super().__init__(params, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=amsgrad, **kw)
        self._chunk_maps = {}
        self._last_steps = []  # the CPU step counters the last step() advanced (undo_step_count)

    def _chunks(self, sizes, device):
        key = (tuple(sizes), device)
        cm = self._chunk_maps.get(key)
        if cm is None:
            pairs = [(ti, s) for ti, n in enumerate(sizes) for s in range(0, n, _CHUNK)]
            cm = torch.tensor(pairs, dtype=torch.int64).reshape(-1, 2).to(device)
            self._chunk_maps[key] = cm
        return cm

    @torch.no_grad()
    def step(self, closure=None, *, skip_if_nonzero: torch.Tensor | None = None):
        """One Adam step.  skip_if_nonzero: a one-element fp32 device tensor; when it holds a non-zero value at the
        time the step runs on the GPU (stream order), the kernel leaves every parameter and moment unchanged --
        train_one_epoch passes the batch's out-of-range label count here so the step can be queued without a host
        wait; the CPU step counters advance at queue time, and the loop calls undo_step_count() before it raises, so
        a skipped step leaves 'step' where the reference's (which never reaches optimizer.step()) leaves it."""
        loss = None
        if skip_if_nonzero is not None and not (skip_if_nonzero.is_cuda and skip_if_nonzero.dtype == torch.float32
                                                and skip_if_nonzero.numel() >= 1):
            raise ValueError("skip_if_nonzero must be a float32 CUDA tensor")
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        self._last_steps = []
        for group in self.param_groups:
            if group["weight_decay"] != 0 or group["amsgrad"] or group["maximize"] or group.get("capturable") \
                    or group.get("differentiable") or group.get("decoupled_weight_decay"):
                raise NotImplementedError("seg_amd.Adam supports the reference's configuration only "
                                          "(weight_decay=0, amsgrad/maximize/capturable/differentiable off)")
            b1, b2 = group["betas"]
            lr, eps = float(group["lr"]), group["eps"]
            ps = [p for p in group["params"] if p.grad is not None]
            if not ps:
                continue
            for p in ps:
                g = p.grad
                if not (p.is_cuda and p.dtype == torch.float32 and g.dtype == torch.float32 and not g.is_sparse
                        and p.is_contiguous() and g.is_contiguous()):
                    raise NotImplementedError("seg_amd.Adam needs contiguous fp32 CUDA parameters and gradients")
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = torch.tensor(0.0)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            sts = [self.state[p] for p in ps]
            steps = [st["step"] for st in sts]
            torch._foreach_add_(steps, 1)  # CPU step counters, as torch's foreach Adam keeps them
            self._last_steps += steps
            rows = []
            for p, st, t in zip(ps, sts, torch.stack(steps).tolist()):
                bc1, bc2 = 1 - b1 ** t, 1 - b2 ** t
                rows.append((p.data_ptr(), p.grad.data_ptr(), st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr(),
                             p.numel(), -(lr / bc1), bc2 ** 0.5))
            device = ps[0].device
            table = _pack(rows).pin_memory().to(device, non_blocking=True)
            chunks = self._chunks([p.numel() for p in ps], device)
            call("seg_adam_step_skip", table.data_ptr(), chunks.data_ptr(), chunks.shape[0], _CHUNK, 1 - b1, b2, 1 - b2,
                 eps, skip_if_nonzero.data_ptr() if skip_if_nonzero is not None else None,
                 torch.cuda.current_stream(device).cuda_stream)
        return loss

    def undo_step_count(self):
        """Take back the step-counter advance of the last step() -- for a step the device skipped
        (skip_if_nonzero): the bias corrections of the next real step are then the reference's.  The
        moments need nothing: a skipped step leaves them as they were (zeros for a new parameter, as torch's Adam
        would create them on its first step)."""
        if self._last_steps:
            torch._foreach_sub_(self._last_steps, 1)
        self._last_steps = []


def _pack(rows):
    """SegAdamTensor[] (include/segamd.h) as int64 words: 4 pointers, n, (step_size, bc2_sqrt)."""
    f = torch.tensor([[r[5], r[6]] for r in rows], dtype=torch.float32)
    words = torch.tensor([r[:5] for r in rows], dtype=torch.int64)
    return torch.cat([words, f.view(torch.int64)], dim=1).contiguous()
