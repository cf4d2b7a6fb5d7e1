"""Intermediate-value taps for parity tests.

The golden generator records, with forward hooks on the reference's own submodules, each encoder
block's output, the cross-attention outputs in call order and the regressors' input, plus the
gradient of the loss with respect to each (tests/golden/make_golden.py).  The drop-in modules
call `record` at the same points; it does nothing unless a test has called `enable`.  Values are
kept in the canonical (B, T, F) layout; gradients arrive through tensor hooks on the tensor that
the rest of the graph consumes (a stacked group buffer is split per stream)."""
from __future__ import annotations

from typing import Optional, Sequence

import torch

_store: Optional[dict] = None


def enable(store: dict) -> None:
    global _store
    _store = store


def disable() -> None:
    global _store
    _store = None


def active() -> bool:
    return _store is not None


def _canon(t: torch.Tensor, seq_first: bool) -> torch.Tensor:
    return (t.permute(1, 0, 2) if seq_first else t).detach().clone()


def record(name: str, t: torch.Tensor, seq_first: bool = False) -> None:
    """One (B, T, F) tensor ((T, B, F) when seq_first)."""
    st = _store
    if st is None:
        return
    st[name] = {"val": _canon(t, seq_first)}
    if t.requires_grad:
        def hook(g, name=name):
            st[name]["grad"] = _canon(g, seq_first)
        t.register_hook(hook)


def record_stacked(names: Sequence[str], X: torch.Tensor) -> None:
    """X (G, B, T, F): stream g is `names[g]`."""
    st = _store
    if st is None:
        return
    for g, name in enumerate(names):
        st[name] = {"val": X[g].detach().clone()}
    if X.requires_grad:
        def hook(gX):
            for g, name in enumerate(names):
                st[name]["grad"] = gX[g].detach().clone()
        X.register_hook(hook)
