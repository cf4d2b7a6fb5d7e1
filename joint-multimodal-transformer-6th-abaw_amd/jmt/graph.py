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
from typing import Callable, Optional

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
