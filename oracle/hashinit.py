"""Counter-hash initialisation shared by the golden generator, the oracle tests and the GPU
parity tests.  TEST INFRASTRUCTURE ONLY — never imported by the product path.

Why: the reference has no fixtures, so parity is pinned by goldens we generate by
running the reference itself in the build container (tests/golden/make_golden.py).  To avoid
committing state_dicts and to be immune to RNG drift across torch versions, every tensor is a pure
function of (name, element index): splitmix64(fnv1a64(name) + i) -> U[0,1) -> scaled
(SURVEY.md §8c "Golden-vector plan").
"""
from __future__ import annotations

import numpy as np

_MASK = (1 << 64) - 1


def fnv1a64(name: str) -> int:
    h = 0xCBF29CE484222325
    for ch in name.encode("utf-8"):
        h ^= ch
        h = (h * 0x100000001B3) & _MASK
    return h


def _splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        x = x + np.uint64(0x9E3779B97F4A7C15)
        z = x
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def uniform01(name: str, n: int) -> np.ndarray:
    """n doubles in [0,1) from the stream keyed by `name`."""
    base = np.uint64(fnv1a64(name))
    with np.errstate(over="ignore"):
        idx = np.arange(n, dtype=np.uint64) + base
    z = _splitmix64(idx)
    return (z >> np.uint64(11)).astype(np.float64) * (1.0 / (1 << 53))


def uniform(name: str, shape, lo: float, hi: float) -> np.ndarray:
    n = int(np.prod(shape)) if len(shape) else 1
    return (lo + (hi - lo) * uniform01(name, n)).reshape(shape).astype(np.float32)


# Gains on the nn.Linear bound for selected 2-D weights (round 2).  With the plain bound the
# attention scores have std ~0.3, softmax is nearly flat over T keys, every attention output is
# ~the mean of V and the predictions are near-constant (spread 1e-3): a broken attention would
# not show.  x4 on the packed in_proj weights (scores x16: std ~5, peaked softmax) and x3 on the
# head / regressor output layers give predictions with O(0.3-1.6) spread on every golden case.
GAINS = (("in_proj_weight", 4.0), ("out_layer1.weight", 3.0), ("final_layer.weight", 3.0),
         ("regressor.3.weight", 3.0), ("mm_transformer.fc.weight", 3.0))


# Gains of the CONDITIONED cases (round 3, tests/golden/spec.py COND_CASES): x2 (x3 at T=300) on
# the packed in_proj weights only.  The CCC-trained GAINS cases above are ill-conditioned in 16
# bits — the reference's own fp32 gradients move by 8-20 % when its weights are rounded to bf16,
# and its own CPU autocast path is 7-90 % off (profiles/r03_parity_conditioning.txt) — so the
# tight 16-bit ceilings are asserted on these instead.
GAINS_COND = (("in_proj_weight", 2.0),)
GAINS_COND_T300 = (("in_proj_weight", 3.0),)


def gain(name: str, gains=None) -> float:
    for pat, g in (GAINS if gains is None else gains):
        if pat in name:
            return g
    return 1.0


def param_value(name: str, shape, gains=None) -> np.ndarray:
    """Deterministic value for a parameter of the given state_dict name and shape.

    * 2-D weights: U(-g/sqrt(fan_in), g/sqrt(fan_in)), fan_in = shape[1] (nn.Linear convention),
      g = gain(name, gains) (1 except the GAINS above, or the case's own `gains`).
    * LayerNorm weight ('layer_norm*.weight'): 1 + U(-0.1, 0.1) so the affine path is exercised.
    * any other 1-D tensor (biases, LN bias): U(-0.1, 0.1).
    """
    shape = tuple(int(s) for s in shape)
    if len(shape) == 2:
        b = gain(name, gains) / np.sqrt(shape[1])
        return uniform("w:" + name, shape, -b, b)
    if "layer_norm" in name and name.endswith("weight"):
        return (1.0 + uniform("w:" + name, shape, -0.1, 0.1)).astype(np.float32)
    return uniform("w:" + name, shape, -0.1, 0.1)


def init_module_(module, prefix: str = "", gains=None) -> None:
    """Overwrite every parameter of a torch module in place with param_value(prefix+name)."""
    import torch

    with torch.no_grad():
        for name, p in module.named_parameters():
            v = torch.from_numpy(param_value(prefix + name, p.shape, gains))
            p.copy_(v.to(dtype=p.dtype, device=p.device))


def state_dict_values(shapes: dict, prefix: str = "", gains=None) -> dict:
    return {k: param_value(prefix + k, s, gains) for k, s in shapes.items()}


def features(tag: str, shape) -> np.ndarray:
    """Synthetic backbone features ~ U(-1,1)."""
    return uniform("x:" + tag, shape, -1.0, 1.0)


def labels(tag: str, shape, ignore_frac: float = 0.0, ignore: float = -5.0) -> np.ndarray:
    """Labels ~ U(-1,1) with a fraction set to the `ignore` value (CCCLoss.py:15)."""
    y = uniform("y:" + tag, shape, -1.0, 1.0)
    if ignore_frac > 0:
        m = uniform01("m:" + tag, y.size).reshape(y.shape) < ignore_frac
        y = np.where(m, np.float32(ignore), y).astype(np.float32)
    return y


def proj_weights(tag: str, shape) -> np.ndarray:
    """Per-element weights of the conditioned cases' loss, mean(w * prediction), in [0.5, 1.5]:
    a smooth, non-cancelling objective (every window contributes with one sign), so each
    parameter gradient is a well-conditioned sum (tests/golden/spec.py COND_CASES)."""
    return (1.0 + 0.5 * features(tag, shape)).astype(np.float32)
