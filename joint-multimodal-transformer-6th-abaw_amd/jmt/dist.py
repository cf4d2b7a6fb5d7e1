"""One-process-per-GPU data parallelism (replaces nn.DataParallel, tools.py:16-21,
main.py:487-491): the batch is sharded contiguously over ranks, the CCC statistics are
all-gathered (8 doubles per rank and loss) so the loss is the global-batch CCC, and gradients are
all-reduced (SUM) over one flat fp32 buffer with RCCL over xGMI."""
from __future__ import annotations

from typing import Optional

import torch

_state = {"group": None}


def set_loss_group(group) -> None:
    """Register the process group over which CCC losses compute global statistics."""
    _state["group"] = group


def loss_group():
    return _state["group"]


def shard_range(global_batch: int, rank: int, world: int):
    """Contiguous split of the global batch (DataParallel scatter on dim 0)."""
    per = (global_batch + world - 1) // world
    lo = min(global_batch, rank * per)
    hi = min(global_batch, lo + per)
    return lo, hi


class FlatGrads:
    """Re-home the .grad of every trainable parameter into one flat fp32 buffer so that one
    RCCL all-reduce (bucketed) and one fused SGD launch cover them all."""

    def __init__(self, params, device, bucket_bytes: int = 64 << 20):
        self.params = [p for p in params if p.requires_grad]
        n = sum(p.numel() for p in self.params)
        self.flat = torch.zeros(n, dtype=torch.float32, device=device)
        self.views = []
        off = 0
        for p in self.params:
            v = self.flat[off:off + p.numel()].view_as(p)
            p.grad = v
            self.views.append(v)
            off += p.numel()
        self.numel = n
        self.bucket_elems = max(1, bucket_bytes // 4)

    def zero_(self):
        self.flat.zero_()
        for p, v in zip(self.params, self.views):
            if p.grad is None or p.grad.data_ptr() != v.data_ptr():
                p.grad = v

    def allreduce_(self, group=None):
        import torch.distributed as dist
        if not dist.is_initialized() or dist.get_world_size(group) == 1:
            return
        for off in range(0, self.numel, self.bucket_elems):
            dist.all_reduce(self.flat[off:off + self.bucket_elems], op=dist.ReduceOp.SUM,
                            group=group)
