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


def grad_write_profile(model_fn, params):
    """Run `model_fn()` (forward + backward) once with gradient-write notifications on: returns
    the parameters that received a gradient, ordered by when their LAST write was enqueued, and
    how many writes each gets per backward (the schedule GradBucketer counts down)."""
    from . import functional as F
    params = list(params)
    ids = {id(p): p for p in params}
    counts, last = {}, {}
    seq = [0]

    def hook(ps):
        for p in ps:
            if id(p) in ids:
                counts[id(p)] = counts.get(id(p), 0) + 1
                last[id(p)] = seq[0]
                seq[0] += 1

    handles = [p.register_post_accumulate_grad_hook(lambda p: hook([p])) for p in params]
    for p in params:
        p.grad = None
    prev, F._grad_hook = F._grad_hook, hook
    try:
        model_fn()
    finally:
        F._grad_hook = prev
        for h in handles:
            h.remove()
    used = [p for p in params if p.grad is not None]
    for p in params:
        p.grad = None
    missing = [p for p in used if id(p) not in counts]
    if missing:
        raise RuntimeError(f"{len(missing)} parameters got a gradient without a write "
                           "notification (jmt.functional._grad_done)")
    used.sort(key=lambda p: last[id(p)])
    return used, {id(p): counts[id(p)] for p in used}


class GradBucketer:
    """The gradient all-reduce overlapped with the backward (the reference's
    DataParallel reduces after its backward, main.py:487-491): the flat fp32 gradient buffer of
    FusedSGD — parameters laid out in the order their gradients complete (grad_write_profile) —
    is cut into contiguous buckets of >= bucket_bytes; each write notification counts its
    parameter down, and when every parameter of a bucket has had its last write enqueued, an
    event on the compute stream gates that bucket's SUM all-reduce on a communication stream
    (RCCL over xGMI with the nccl backend), so it runs under the rest of the backward.
    finish() issues any bucket still pending and joins the communication into the current
    stream before the optimizer step."""

    def __init__(self, opt, counts, bucket_bytes: int = 16 << 20, group=None):
        from . import functional as F
        self._F = F
        self.flat = opt.flat_g
        self.group = group
        self.expected = {}
        self.bucket_of = {}
        self.buckets = []          # (lo, hi, n_params)
        lo, cur, nbytes = 0, [], 0
        ends = [off + -(-p.numel() // 64) * 64 for p, off in zip(opt.params, opt.offsets)]
        for i, p in enumerate(opt.params):
            if id(p) not in counts:
                raise RuntimeError("GradBucketer: a parameter of the optimizer has no write "
                                   "profile")
            self.expected[id(p)] = counts[id(p)]
            cur.append(p)
            nbytes += p.numel() * 4
            if nbytes >= bucket_bytes or i == len(opt.params) - 1:
                for q in cur:
                    self.bucket_of[id(q)] = len(self.buckets)
                self.buckets.append((lo, ends[i], len(cur)))
                lo, cur, nbytes = ends[i], [], 0
        self.cuda = self.flat.is_cuda
        self.comm = torch.cuda.Stream(self.flat.device) if self.cuda else None
        self._hooks = [p.register_post_accumulate_grad_hook(lambda p: F._grad_done(p))
                       for p in opt.params]
        self.launch_log = []
        # collectives also at world size 1 (tests: RCCL inside a captured step on a 1-GPU box)
        self.world1 = False

    def begin(self):
        self._main = torch.cuda.current_stream() if self.cuda else None
        self.left = dict(self.expected)
        self.bucket_left = [b[2] for b in self.buckets]
        self.launched = [False] * len(self.buckets)
        # streams that enqueued a write of each bucket's parameters (the compute stream, the
        # weight-gradient side stream, the run_parallel branch streams, ...): the bucket's
        # all-reduce is ordered after ALL of them, not only after the stream of its last write
        self.writers = [[] for _ in self.buckets]
        self.works = []
        self.launch_log = []
        self._F._grad_hook = self._done

    def _done(self, ps):
        cur = torch.cuda.current_stream() if self.cuda else None
        for p in ps:
            k = id(p)
            if k not in self.left:
                continue
            b = self.bucket_of[k]
            if cur is not None and cur not in self.writers[b]:
                self.writers[b].append(cur)
            self.left[k] -= 1
            if self.left[k] == 0:
                self.bucket_left[b] -= 1
                if self.bucket_left[b] == 0:
                    self._launch(b)

    def _launch(self, b):
        import torch.distributed as dist
        if self.launched[b]:
            return
        self.launched[b] = True
        self.launch_log.append(b)
        lo, hi, _ = self.buckets[b]
        if not dist.is_initialized() or (dist.get_world_size(self.group) == 1 and
                                         not self.world1):
            return
        if self.cuda:
            from .graph import collective, segmented_capture_active
            if segmented_capture_active():
                # piecewise-captured step (jmt.graph.SegmentedStep): the bucket's all-reduce is
                # issued on the host between two segment replays, ordered after the segment
                # that wrote its gradients (the replay stream) and overlapping the next one
                def issue(lo=lo, hi=hi):
                    self.comm.wait_stream(torch.cuda.current_stream())
                    with torch.cuda.stream(self.comm):
                        self.works.append(dist.all_reduce(self.flat[lo:hi],
                                                          op=dist.ReduceOp.SUM,
                                                          group=self.group, async_op=True))
                collective(issue)
                return
            # every stream that wrote one of the bucket's gradients (recorded by _done), the
            # stream this last notification came from, the weight-gradient side stream
            # (jmt.streams.run_side) and the step's compute stream precede the all-reduce; a
            # wait is one event record + one stream wait, no host synchronisation
            from . import streams
            cur = torch.cuda.current_stream()
            waits = list(self.writers[b])
            for st in [cur] + streams.side_streams() + [self._main]:
                if st is not None and st.device == cur.device and st not in waits:
                    waits.append(st)
            for st in waits:
                self.comm.wait_stream(st)
            with torch.cuda.stream(self.comm):
                self.works.append(dist.all_reduce(self.flat[lo:hi], op=dist.ReduceOp.SUM,
                                                  group=self.group, async_op=True))
        else:
            self.works.append(dist.all_reduce(self.flat[lo:hi], op=dist.ReduceOp.SUM,
                                              group=self.group, async_op=True))

    def finish(self):
        self._F._grad_hook = None
        for b in range(len(self.buckets)):
            if not self.launched[b]:
                self._launch(b)

        def join():
            for w in self.works:
                w.wait()
            if self.cuda:
                torch.cuda.current_stream().wait_stream(self.comm)
            self.works = []
        if self.cuda:
            from .graph import collective
            collective(join)              # deferred to replay under a SegmentedStep capture
        else:
            join()

    def close(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []
