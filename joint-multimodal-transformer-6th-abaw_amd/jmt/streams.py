"""Concurrent execution of independent sub-graphs on separate HIP streams.

The JMT block has independent branches (the three encoders, mm_multi_transformers.py:132-136;
the six cross-attentions, :142-167).  Each branch alone launches GEMMs of 600-1800 tiles on a
512-slot machine (256 CUs x 2 resident blocks), so a lone launch ends with a partially idle
chip.  Running the branches on their own streams lets the hardware queues overlap one branch's
tail with the next branch's blocks; autograd replays every backward node on the stream of its
forward node, so the backward overlaps the same way."""
from __future__ import annotations

import os
from typing import Callable, List, Sequence

import torch

_pool: dict = {}
_enabled = {"on": True, "capture": os.environ.get("JMT_CAPTURE_STREAMS", "1") != "0"}


def set_enabled(on: bool) -> None:
    _enabled["on"] = bool(on)


def set_capture_enabled(on: bool) -> None:
    """Fork/join the branch streams inside a hipGraph capture too (jmt.graph): the captured
    graph then holds the branches as parallel nodes."""
    _enabled["capture"] = bool(on)


def _streams(device, n: int) -> List[torch.cuda.Stream]:
    key = (device.index if device.index is not None else torch.cuda.current_device(), n)
    if key not in _pool:
        _pool[key] = [torch.cuda.Stream(device=device) for _ in range(n)]
    return _pool[key]


_join = {"queued": False}


def join_after_backward() -> None:
    """Called by backward functions that write parameter gradients in place (wgrad / bias / LN
    grads return None to autograd).  Autograd joins a branch stream back into the caller's
    stream only through the gradients it hands on, so kernels that only update `param.grad` on
    a branch stream would stay unordered with the optimizer step (and leave an unjoined fork in
    a hipGraph capture).  The first such call of a backward pass queues one end-of-backward
    callback that makes the caller's current stream wait for every branch stream."""
    if _join["queued"] or not _pool:
        return
    cur = torch.cuda.current_stream()
    branches = [s for ss in _pool.values() for s in ss]
    if not any(cur == s for s in branches):
        return
    _join["queued"] = True

    def _cb():
        _join["queued"] = False
        main = torch.cuda.current_stream()    # the caller's stream (autograd restores it)
        for s in branches:
            if s.device == main.device:
                main.wait_stream(s)

    torch.autograd.Variable._execution_engine.queue_callback(_cb)


def run_parallel(fns: Sequence[Callable[[], object]], device) -> list:
    """Run each zero-argument callable on its own stream, then make the current stream wait for
    all of them.  Returns the callables' results (tensors are marked as used on the current
    stream so the caching allocator keeps them alive)."""
    if not _enabled["on"] or len(fns) <= 1 or \
            (torch.cuda.is_current_stream_capturing() and not _enabled["capture"]):
        return [f() for f in fns]
    main = torch.cuda.current_stream(device)
    side = _streams(device, len(fns))
    _join["queued"] = False
    outs = []
    for f, s in zip(fns, side):
        s.wait_stream(main)
        with torch.cuda.stream(s):
            outs.append(f())
    for s in side:
        main.wait_stream(s)

    def mark(x):
        if isinstance(x, torch.Tensor):
            x.record_stream(main)
        elif isinstance(x, (list, tuple)):
            for y in x:
                mark(y)

    for o in outs:
        mark(o)
    return outs
