"""Fused SGD over flat buffers (instantiator.py:32-38 semantics, config_file.json:73-80).

All trainable parameters are re-homed into ONE flat fp32 buffer, their gradients into another
(the buffer the RCCL all-reduce runs on), the momentum into a third; one jmt_sgd_step launch
updates everything and rewrites the bf16/f16 compute shadows of the weights in the same pass.
Parameters that never receive a gradient (the reference's unused `final_encoder`,
`gated_attention`) must not be passed: torch.optim.SGD skips them because their .grad is None,
so `used_parameters()` finds them with one probe backward."""
from __future__ import annotations

import os
from typing import Iterable, List, Optional

import torch

from . import _lib
from . import functional as F
from . import ops


def _bump_grad_gen(_p):
    F._grad_gen[0] += 1


class FusedSGD:
    def __init__(self, params: Iterable[torch.nn.Parameter], lr: float, momentum: float = 0.0,
                 dampening: float = 0.0, weight_decay: float = 0.0, nesterov: bool = False,
                 shadow_dtype: Optional[torch.dtype] = None, fuse_zero_grad: bool = False):
        """fuse_zero_grad: the step kernel zeroes each gradient after reading it (jmt_sgd_step_zero)
        and the next zero_grad() issues nothing while no gradient has been written since — the
        training step of train.py:96-315 without a fill launch.  Off by default: torch's
        optimizer.step() leaves .grad readable until zero_grad().

        Contract of the skipped fill: "written since" is known from functional._grad_gen, which
        the HIP gradient writers (functional._grad_buffer) and torch autograd's accumulation into
        .grad (post-accumulate hooks) bump.  Anything else that writes into a .grad in place
        (p.grad.add_/copy_ by hand, a helper writing into the flat views) is invisible to it and
        the next backward would add onto the stale values: call zero_grad(force=True) after such
        a write, or set JMT_CHECK_ZERO_GRAD=1 to have every skipped fill verify (one reduction +
        host sync) that the gradients are in fact zero."""
        self.params: List[torch.nn.Parameter] = list(params)
        assert self.params, "no parameters"
        dev = self.params[0].device
        # every parameter starts on a 256-B boundary (16-B aligned MFMA operand loads)
        offs = []
        n = 0
        for p in self.params:
            offs.append(n)
            n += -(-p.numel() // 64) * 64
        self.numel = n
        self.lr, self.momentum, self.dampening = lr, momentum, dampening
        self.weight_decay, self.nesterov = weight_decay, nesterov
        self.flat_p = torch.empty(n, dtype=torch.float32, device=dev)
        self.flat_g = torch.zeros(n, dtype=torch.float32, device=dev)
        self.buf = torch.zeros(n, dtype=torch.float32, device=dev) if momentum else None
        self.shadow = (torch.empty(n, dtype=shadow_dtype, device=dev)
                       if shadow_dtype not in (None, torch.float32) else None)
        self.flat_p.zero_()
        self.offsets = offs
        self._gviews = []
        with torch.no_grad():
            for p, off in zip(self.params, offs):
                k = p.numel()
                self.flat_p[off:off + k].copy_(p.detach().reshape(-1))
                p.data = self.flat_p[off:off + k].view_as(p)
                g = self.flat_g[off:off + k].view_as(p)
                p.grad = g
                self._gviews.append(g)
        if self.shadow is not None:
            ops.cast(self.flat_p, self.shadow.dtype, out=self.shadow)
        for p, off in zip(self.params, offs):
            F.register_shadow(p, self.shadow[off:off + p.numel()].view_as(p)
                              if self.shadow is not None else None)
        self.first = True
        self.fuse_zero_grad = bool(fuse_zero_grad)
        # the gradients are known to be zero while nothing has written one since the last fill /
        # zeroing step (functional._grad_gen counts the HIP writers; torch autograd accumulation
        # into .grad is caught by the post-accumulate hooks)
        self._clean_gen = F._grad_gen[0]
        self._hooks = [p.register_post_accumulate_grad_hook(_bump_grad_gen) for p in self.params]

    def close(self):
        """Remove the gradient-write hooks this optimizer put on its parameters (also on garbage
        collection); the parameters keep their flat-buffer storage."""
        for h in getattr(self, "_hooks", ()):
            h.remove()
        self._hooks = []

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def zero_grad(self, set_to_none: bool = False, force: bool = False):
        """optimizer.zero_grad().  With fuse_zero_grad the step kernel already zeroed the
        gradients, so after a step (and no gradient write since) this issues nothing; force=True
        fills regardless (after an in-place .grad write the write counter cannot see)."""
        for p, g in zip(self.params, self._gviews):
            if p.grad is None or p.grad.data_ptr() != g.data_ptr():
                p.grad = g
                self._clean_gen = None
        if force or not self.fuse_zero_grad or self._clean_gen != F._grad_gen[0]:
            self.flat_g.zero_()
            self._clean_gen = F._grad_gen[0]
        elif os.environ.get("JMT_CHECK_ZERO_GRAD", "0") == "1":
            nz = int(torch.count_nonzero(self.flat_g))
            if nz:
                raise RuntimeError(f"FusedSGD.zero_grad: {nz} gradient element(s) written outside "
                                   "the tracked writers since the fused zeroing step (see the "
                                   "fuse_zero_grad contract); call zero_grad(force=True)")

    @torch.no_grad()
    def step_amp(self, amp_state: torch.Tensor):
        """One step driven by a GradScaler's device state (unscale, skip on overflow).  Whether
        the momentum buffer is initialised is then decided on the device (steps_taken), so plain
        step() calls cannot follow scaled ones."""
        self._amp = True
        fn = "jmt_sgd_step_amp_zero" if self.fuse_zero_grad else "jmt_sgd_step_amp"
        _lib.call(fn, self.numel, self.flat_p.data_ptr(), self.flat_g.data_ptr(),
                  self.buf.data_ptr() if self.buf is not None else None, self.lr, self.momentum,
                  self.dampening, self.weight_decay, int(self.nesterov), int(self.first),
                  amp_state.data_ptr(),
                  self.shadow.data_ptr() if self.shadow is not None else None,
                  ops.dt(self.shadow) if self.shadow is not None else 1, ops.stream())
        self._clean_gen = F._grad_gen[0]

    @torch.no_grad()
    def step(self, grad_scale: float = 1.0):
        if getattr(self, "_amp", False):
            raise RuntimeError("FusedSGD: step() after GradScaler steps (first-step state is on "
                               "the device); keep using scaler.step(opt)")
        ops.sgd_step(self.flat_p, self.flat_g, self.buf, self.lr, self.momentum, self.dampening,
                     self.weight_decay, self.nesterov, self.first, grad_scale, self.shadow,
                     zero_grad=self.fuse_zero_grad)
        self.first = False
        self._clean_gen = F._grad_gen[0]


class GradScaler:
    """torch.cuda.amp.GradScaler semantics (train.py:89,314-316) for FusedSGD with the whole
    state on the device: `scaler.scale(loss).backward(); scaler.step(opt); scaler.update()` issue
    kernels only (no host synchronisation; the step stays capturable into a hipGraph)."""

    def __init__(self, init_scale: float = 2.0 ** 16, growth_factor: float = 2.0,
                 backoff_factor: float = 0.5, growth_interval: int = 2000, device=None):
        dev = torch.device(device) if device is not None else torch.device("cuda")
        self.growth_factor, self.backoff_factor = growth_factor, backoff_factor
        self.growth_interval = growth_interval
        self.state = torch.tensor([init_scale, 1.0 / init_scale, 0.0, 0.0, 0.0],
                                  dtype=torch.float32, device=dev)

    def scale(self, loss: torch.Tensor) -> torch.Tensor:
        return loss * self.state[0]

    def step(self, opt: "FusedSGD"):
        _lib.call("jmt_amp_check", opt.numel, opt.flat_g.data_ptr(), self.state.data_ptr(),
                  ops.stream())
        opt.step_amp(self.state)

    def update(self):
        _lib.call("jmt_amp_update", self.state.data_ptr(), self.growth_factor,
                  self.backoff_factor, self.growth_interval, ops.stream())

    def get_scale(self) -> float:
        return float(self.state[0])


def used_parameters(model_fn, params: Iterable[torch.nn.Parameter]):
    """Run `model_fn()` (forward + backward), return the parameters that received a gradient."""
    params = list(params)
    for p in params:
        p.grad = None
    model_fn()
    used = [p for p in params if p.grad is not None]
    for p in params:
        p.grad = None
    return used
