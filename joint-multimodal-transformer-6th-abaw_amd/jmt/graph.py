"""Whole-step HIP graph capture of the JMT training step.

One training step (zero_grad -> forward -> CCC losses -> backward -> fused SGD) is ~300 kernel
launches issued from Python (autograd + ctypes).  Replaying the captured hipGraph issues all of
them with one host call, so the step time is the GPU's time, not the host's issue rate.

Requirements the JMT path meets by construction:
  * static inputs: the caller keeps the input / label tensors alive and refills them in place;
  * no host synchronisation inside the step (the losses stay on device);
  * optimizer state lives in persistent buffers (jmt.optim.FusedSGD's flat buffers) and its
    first-step branch has been taken before capture (the warm-up steps run eagerly);
  * every launch goes to torch's current stream (jmt.ops) — under capture that is the capture
    stream; the concurrent branch streams (jmt.streams) fork from and join back into it.
"""
from __future__ import annotations

import os
from typing import Callable, List, Optional, Tuple

import torch


class GraphedStep:
    """`g = GraphedStep(step_fn).capture(warmup=3); out = g.replay()`.

    step_fn() enqueues one complete step on the current stream and returns a tensor (or tuple of
    tensors) that the caller reads after replay (e.g. the loss); those outputs are static."""

    def __init__(self, step_fn: Callable[[], object]):
        self.step_fn = step_fn
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.out = None

    def capture(self, warmup: int = 3):
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(max(warmup, 1)):   # eager steps on a side stream (torch's rule)
                self.step_fn()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        # JMT_COMPUTE_PRIO=1: capture on a high-priority stream, so the step's critical chain
        # outranks the weight-gradient side stream (jmt.streams, default priority) when both
        # have blocks waiting for CUs
        cap = torch.cuda.Stream(priority=-1) if os.environ.get("JMT_COMPUTE_PRIO") == "1" else None
        with torch.cuda.graph(self.graph, stream=cap):
            self.out = self.step_fn()
        torch.cuda.synchronize()
        return self

    def replay(self):
        if self.graph is None:
            raise RuntimeError("GraphedStep.replay() before capture()")
        self.graph.replay()
        return self.out


# ------------------------------------------------------------------ piecewise capture (N > 1)
_capturing: List["SegmentedStep"] = []


def segmented_capture_active() -> bool:
    return bool(_capturing)


def collective(op: Callable[[], object]):
    """Issue `op` (a collective: the CCC statistics all-gather, a gradient bucket's all-reduce,
    the join of the communication stream) now — or, while a SegmentedStep captures, end the
    current graph segment, record `op` to run on the host between that segment's replay and the
    next one's, and begin the next segment.  Returns op()'s result, or None when deferred."""
    if not _capturing:
        return op()
    _capturing[-1].cut(op)
    return None


class SegmentedStep:
    """The N > 1 training step as a sequence of hipGraph segments with the collectives between
    them issued eagerly: RCCL stays out of the graphs (the eager collectives
    the multi-rank tests run), and host issue per step is one graph launch per segment plus the
    collective calls instead of ~300 Python / ctypes launches (3.07 ms at c3, bench.py
    host_issue_ms_per_eager_step).  The segments are captured in one pass into one memory pool:
    a collective reached during capture (jmt.graph.collective — from the CCC loss and from
    jmt.dist.GradBucketer's bucket notifications inside the backward) ends the current segment
    after an empty marker kernel (no segment is empty), queues the collective, and starts the
    next segment; replay() runs segment, collective, segment, ... in capture order on the
    current stream, so each bucket's all-reduce still overlaps the rest of the backward.
    Requirements as GraphedStep, plus: no forked stream may be open across a collective (the
    weight-gradient side stream is turned off while capturing), and the caller holds no output
    of an earlier eager step (its autograd graph would keep the parameters' AccumulateGrad nodes,
    created on another stream, so their hooks — the bucket notifications — run on that stream)."""

    def __init__(self, step_fn: Callable[[], object]):
        self.step_fn = step_fn
        self.segments: List[Tuple[torch.cuda.CUDAGraph, Optional[Callable[[], object]]]] = []
        self.out = None
        self._g: Optional[torch.cuda.CUDAGraph] = None
        self._stream: Optional[torch.cuda.Stream] = None

    def capture(self, warmup: int = 3):
        from . import streams
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(max(warmup, 1)):
                self.step_fn()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        self.pool = torch.cuda.graph_pool_handle()
        self._stream = torch.cuda.Stream()
        self._stream.wait_stream(torch.cuda.current_stream())
        side_on = streams._enabled.get("side", True)
        streams.set_side_enabled(False)
        try:
            with torch.cuda.stream(self._stream):
                self._begin()
                _capturing.append(self)
                try:
                    self.out = self.step_fn()
                finally:
                    _capturing.pop()
                self._end(None)
        finally:
            streams.set_side_enabled(side_on)
        torch.cuda.current_stream().wait_stream(self._stream)
        torch.cuda.synchronize()
        return self

    def _begin(self):
        # relaxed: the bucket cuts come from autograd's device thread, and a thread-local (or
        # global) capture sequence may only be ended by the thread that began it
        # (hipErrorStreamCaptureWrongThread)
        self._g = torch.cuda.CUDAGraph()
        self._g.capture_begin(pool=self.pool, capture_error_mode="relaxed")

    def _end(self, op):
        from . import ops
        ops.noop()                       # a segment is never empty (empty graphs cannot replay)
        self._g.capture_end()
        self.segments.append((self._g, op))
        self._g = None

    def cut(self, op: Callable[[], object]):
        if torch.cuda.current_stream() != self._stream:
            # e.g. the post-accumulate hook of a parameter whose AccumulateGrad node was created
            # on another stream by an eager step whose outputs the caller still holds (their
            # autograd graph keeps the node alive): drop those outputs before capture()
            raise RuntimeError("SegmentedStep: a collective was reached on a forked stream (a "
                               "segment cannot end with unjoined work); release the outputs of "
                               "earlier eager steps before capture()")
        self._end(op)
        self._begin()

    def replay(self):
        if not self.segments:
            raise RuntimeError("SegmentedStep.replay() before capture()")
        for g, op in self.segments:
            g.replay()
            if op is not None:
                op()
        return self.out
