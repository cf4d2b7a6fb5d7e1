"""Golden vectors for the validation-metric row, produced by importing the
reference's own EvaluationMetrics/cccmetric.py (numpy only) from /root/reference.  Run in the
build container:  python tests/golden/make_golden_valpost.py  -> tests/golden/valpost.npz
(inputs + the reference's ccc outputs; nothing from the reference is copied)."""
import importlib.util
import os
import sys

import numpy as np

sys.dont_write_bytecode = True
REF = "/root/reference/EvaluationMetrics/cccmetric.py"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "valpost.npz")


def main():
    spec = importlib.util.spec_from_file_location("ref_cccmetric", REF)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    rng = np.random.default_rng(20261016)
    data = {}
    cases = {
        "rand": (rng.normal(0.1, 0.4, 5000), rng.uniform(-1, 1, 5000)),
        "corr": None,
        "f32": (rng.normal(0, 0.3, 777).astype(np.float32),
                rng.uniform(-1, 1, 777).astype(np.float32)),
        "smallvar": (0.5 + 1e-3 * rng.normal(size=300), rng.uniform(-1, 1, 300)),
        "n2": (np.array([0.25, -0.5]), np.array([0.1, 0.3])),
    }
    y = rng.uniform(-1, 1, 4000)
    cases["corr"] = (0.8 * y + 0.1 * rng.normal(size=4000) + 0.05, y)
    for tag, (x, t) in cases.items():
        data[f"{tag}/x"] = x
        data[f"{tag}/y"] = t
        data[f"{tag}/ccc"] = np.float64(mod.ccc(x, t))
    # cccva on (N, 2) pairs (the module's own __main__ pattern, cccmetric.py:24-38)
    yt = rng.uniform(-1, 1, (600, 2))
    yp = yt + rng.normal(0, 0.2, (600, 2))
    data["va/true"], data["va/pred"] = yt, yp
    data["va/ccc"] = np.array(mod.cccva(yt, yp), dtype=np.float64)
    np.savez(OUT, **data)
    print("wrote", OUT, len(data), "arrays")


if __name__ == "__main__":
    main()
