"""Diagnostic: encoder-output gradient errors of the tr_fc_t300 golden case vs the backward's
loss scale, fp16 and bf16 (underflow vs rounding)."""
import json, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "joint-multimodal-transformer-6th-abaw_amd")]
import numpy as np, torch
from tests.golden import spec
from tests.parity import run_tt, errors
with np.load(os.path.join(REPO, "tests", "golden", "golden.npz")) as z:
    gold = {k: z[k] for k in z.files}
for tag in ("tr_fc_t300", "tr_fc"):
    c = [c for c in spec.TT_CASES if c["tag"] == tag][0]
    for cd in (torch.float16, torch.bfloat16):
        for ls in (1.0, 1024.0, 32768.0):
            r = errors(gold, c, *run_tt(c, cd, record=True, loss_scale=ls))
            print(json.dumps({"case": tag, "dtype": str(cd), "scale": ls,
                              **{k: round(v, 5) for k, v in r["inter"].items() if "enc" in k or k.startswith("ca.0")},
                              "pgrad_max": round(r["pgrad_max"], 4)}), flush=True)
