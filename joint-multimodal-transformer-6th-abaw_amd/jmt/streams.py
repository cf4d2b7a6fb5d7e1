"""Concurrent execution of independent sub-graphs on separate HIP streams.

The JMT block has independent branches (the three encoders, mm_multi_transformers.py:132-136;
the six cross-attentions, :142-167).  Each branch alone launches GEMMs of 600-1800 tiles on a
512-slot machine (256 CUs x 2 resident blocks), so a lone launch ends with a partially idle
chip.  Running the branches on their own streams lets the hardware queues overlap one branch's
tail with the next branch's blocks; autograd replays every backward node on the stream of its
forward node, so the backward overlaps the same way."""
from __future__ import annotations

import os
from typing import Callable, List, Optional, Sequence

import torch

_pool: dict = {}
_enabled = {"on": True, "capture": os.environ.get("JMT_CAPTURE_STREAMS", "1") != "0",
            "side": os.environ.get("JMT_SIDE_STREAM", "0") == "1"}


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


# ------------------------------------------------------------------ weight-gradient side stream
# In a backward pass the input-gradient (dgrad) GEMMs form the critical chain; the weight- and
# bias-gradient launches of a layer only read that layer's output gradient and saved input and
# write parameter gradients.  They go to one side stream per device, forked from the compute
# stream right after the output gradient is enqueued, so their blocks fill the CUs the chain's
# launches leave idle (tile-quantised last rounds, epilogue bursts, latency-bound phases).
_side: dict = {}
_side_join = {"queued": None}    # graph task id whose end-of-backward join is queued


def set_side_enabled(on: bool) -> None:
    _enabled["side"] = bool(on)


def side_streams() -> List[torch.cuda.Stream]:
    """The side streams created so far (jmt.dist.GradBucketer gates its all-reduces on them)."""
    return list(_side.values())


def run_side(fn: Callable[[], object], reads: Sequence[Optional[torch.Tensor]] = ()):
    """Enqueue fn() on the current device's side stream after everything already queued on the
    current stream.  `reads`: tensors fn's kernels read that the caller may drop before they run
    (marked used on the side stream for the caching allocator).  Parameter-gradient writes of
    different streams must not target the same memory: callers move ALL writes of a gradient
    buffer to the side stream.  The caller's stream joins the side stream at the end of the
    backward pass (a queued autograd callback), before the optimizer reads the gradients."""
    if not (_enabled["on"] and _enabled["side"]) or \
            (torch.cuda.is_current_stream_capturing() and not _enabled["capture"]):
        return fn()
    main = torch.cuda.current_stream()
    dev = main.device.index if main.device.index is not None else torch.cuda.current_device()
    side = _side.get(dev)
    if side is None:
        side = _side[dev] = torch.cuda.Stream(device=main.device)
    side.wait_stream(main)
    with torch.cuda.stream(side):
        out = fn()
    for t in reads:
        if isinstance(t, torch.Tensor) and t.is_cuda:
            t.record_stream(side)
    # one join per backward pass, keyed on autograd's graph task (a backward that raised
    # before its final callbacks ran cannot leave a stale flag that skips later joins)
    task = torch._C._current_graph_task_id()
    if task < 0:                       # outside a backward: the caller joins (wait_side)
        return out
    if _side_join["queued"] != task:
        _side_join["queued"] = task

        def _cb():
            _side_join["queued"] = None
            cur = torch.cuda.current_stream()
            for st in _side.values():
                if st.device == cur.device:
                    cur.wait_stream(st)

        torch.autograd.Variable._execution_engine.queue_callback(_cb)
    return out


def wait_side() -> None:
    """Make the current stream wait for the work queued so far on its device's side stream (a
    kernel about to overwrite a buffer that side-stream work still reads)."""
    cur = torch.cuda.current_stream()
    for st in _side.values():
        if st.device == cur.device:
            cur.wait_stream(st)


def fork_side(fn: Callable[[], object], reads: Sequence[Optional[torch.Tensor]] = ()) -> bool:
    """Enqueue fn() on the side stream after the current stream's queued work, for the caller
    to overlap with its next launch and then join with wait_side().  Returns False (fn ran on
    the current stream) when side streams are off."""
    if not (_enabled["on"] and _enabled["side"]) or \
            (torch.cuda.is_current_stream_capturing() and not _enabled["capture"]):
        fn()
        return False
    main = torch.cuda.current_stream()
    dev = main.device.index if main.device.index is not None else torch.cuda.current_device()
    side = _side.get(dev)
    if side is None:
        side = _side[dev] = torch.cuda.Stream(device=main.device)
    side.wait_stream(main)
    with torch.cuda.stream(side):
        fn()
    for t in reads:
        if isinstance(t, torch.Tensor) and t.is_cuda:
            t.record_stream(side)
    return True
