"""Parity report: HIP drop-in modules vs the reference goldens in fp32 / bf16 / fp16 compute.
Prints one JSON line per (case, dtype) with every error the tests bound (tests/parity.py).
Needs a GPU.  Usage: python scripts/parity_report.py [--full]"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "joint-multimodal-transformer-6th-abaw_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from tests.golden import spec  # noqa: E402
from tests.parity import measure  # noqa: E402


def main():
    full = "--full" in sys.argv
    with np.load(os.path.join(REPO, "tests", "golden", "golden.npz")) as z:
        gold = {k: z[k] for k in z.files}
    for c in spec.TT_CASES:
        for cd in (torch.float32, torch.bfloat16, torch.float16):
            r = measure(gold, c, cd)
            if not full:
                r.pop("pgrad", None)
                r.pop("inter", None)
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
