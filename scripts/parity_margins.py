"""Margins of the strict 16-bit suite from a parity_report.py --dump file (GPU and emulated
errors of every quantity, and the mutated runs), under the bounds tests/parity.py applies now:
one line per (case, dtype) with the smallest margins (bound / GPU error) and the GPU / emulated
ratios, then one line per mutation with the quantities it breaks.

    python scripts/parity_margins.py gpurun_out/r03/parity/strict_full.json > profiles/r03_parity_error_model.jsonl"""
import json
import math
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "joint-multimodal-transformer-6th-abaw_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from tests import parity as P  # noqa: E402

DT = {"bfloat16": torch.bfloat16, "float16": torch.float16}


def main():
    src = sys.argv[1]
    d = json.load(open(src))
    for case, v in d["strict"].items():
        tag, dt = case.split("/")
        gpu, emu = v["gpu"], v["emulated"]
        bnd = P.strict_bounds(emu, DT[dt])
        margin = {k: (bnd[k] / gpu[k] if gpu[k] > 0 else math.inf) for k in bnd}
        ratio = [gpu[k] / emu[k] for k in bnd if emu[k] > 0 and math.isfinite(gpu[k])]
        worst = sorted(margin, key=margin.get)[:5]
        print(json.dumps({
            "suite": "strict", "case": tag, "dtype": dt, "k_strict": P.K_STRICT,
            "n_quantities": len(bnd), "violations": sum(1 for k in bnd if not gpu[k] <= bnd[k]),
            "min_margin": round(margin[worst[0]], 3),
            "n_margin_below_1_5": sum(1 for k in bnd if margin[k] < 1.5),
            "min_margin_values": round(min(margin[k] for k in bnd if P._is_value(k)), 3),
            "worst": [{"q": k, "gpu": round(gpu[k], 6), "emulated": round(emu[k], 6),
                       "bound": round(bnd[k], 6), "margin": round(margin[k], 3)} for k in worst],
            "gpu_over_emulated": {"median": round(float(np.median(ratio)), 3),
                                  "p90": round(float(np.percentile(ratio, 90)), 3),
                                  "max": round(float(max(ratio)), 3)}}))
    base = d["strict"]["cond_tr_fc/bfloat16"]
    bnd = P.strict_bounds(base["emulated"], torch.bfloat16)
    for name, g in d.get("mutations", {}).items():
        bad = sorted(((g[k] / bnd[k], k) for k in bnd if not g[k] <= bnd[k]), reverse=True)
        print(json.dumps({"suite": "mutation", "case": "cond_tr_fc", "dtype": "bfloat16",
                          "mutation": name, "detected": bool(bad), "n_violations": len(bad),
                          "largest": [{"q": k, "gpu": round(g[k], 6),
                                       "unmutated_gpu": round(base["gpu"][k], 6),
                                       "bound": round(bnd[k], 6), "over": round(r, 3)}
                                      for r, k in bad[:4]]}))


if __name__ == "__main__":
    main()
