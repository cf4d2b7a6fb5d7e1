"""Parity report: HIP drop-in modules vs the reference goldens in fp32 / bf16 / fp16 compute.
Prints one line per (case, dtype): max abs / relative error of V/A predictions, loss errors.
Needs a GPU.  Usage: python scripts/parity_report.py"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "joint-multimodal-transformer-6th-abaw_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from tests.golden import spec  # noqa: E402
from tests.test_gpu_models import _run_tt  # noqa: E402


def main():
    with np.load(os.path.join(REPO, "tests", "golden", "golden.npz")) as z:
        gold = {k: z[k] for k in z.files}
    rows = []
    for c in spec.TT_CASES:
        for name, cd in (("fp32", torch.float32), ("bf16", torch.bfloat16),
                         ("fp16", torch.float16)):
            vo, ao, l1, l2, _ = _run_tt(c, cd)
            t = c["tag"]
            r = {"case": t, "dtype": name}
            for k, o in (("vouts", vo), ("aouts", ao)):
                a = o.detach().float().cpu().numpy()
                b = gold[f"{t}/{k}"]
                r[k + "_abs"] = float(np.abs(a - b).max())
                r[k + "_rel"] = float(np.abs(a - b).max() / np.abs(b).max())
                r[k + "_spread"] = float(b.max() - b.min())
            r["v_loss_err"] = abs(l1 - float(gold[f"{t}/v_loss"]))
            r["a_loss_err"] = abs(l2 - float(gold[f"{t}/a_loss"]))
            rows.append(r)
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
