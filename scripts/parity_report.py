"""Parity report (needs a GPU): every error the 16-bit tests bound, with its bound and margin.

* strict suite (spec.COND_CASES, tests/parity.py check16_strict): per (case, dtype) the GPU error,
  the rounding-emulating oracle's error and the bound min(ceiling, K_STRICT x emulated) of every
  quantity; the line lists the smallest margins (bound / GPU error) and the GPU / emulated ratios.
* reference-relative suite (spec.TT_CASES, check_vs_ref16): GPU vs the reference's own autocast
  and the emulating oracle on prediction / loss / median and max parameter-gradient error.

    python scripts/parity_report.py [--dump DIR] > gpurun_out/parity_report.jsonl

--dump DIR also writes every quantity's GPU and emulated error per (case, dtype) and, for the
mutations of tests/test_gpu_models.py, the mutated GPU errors (DIR/strict_full.json)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "joint-multimodal-transformer-6th-abaw_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from tests.golden import spec  # noqa: E402
from tests import parity as P  # noqa: E402


def main():
    dump = sys.argv[sys.argv.index("--dump") + 1] if "--dump" in sys.argv else None
    full = {"strict": {}, "mutations": {}}
    with np.load(os.path.join(REPO, "tests", "golden", "golden.npz")) as z:
        gold = {k: z[k] for k in z.files}
    for c in spec.COND_CASES:
        for cd in (torch.bfloat16, torch.float16):
            gpu = P.measure_strict(gold, c, cd)
            emu = P.emulated_strict(gold, c, cd)
            full["strict"][f"{c['tag']}/{str(cd)[6:]}"] = {"gpu": gpu, "emulated": emu}
            bnd = P.strict_bounds(emu, cd)
            margin = {k: (bnd[k] / gpu[k] if gpu[k] > 0 else float("inf")) for k in bnd}
            ratio = [gpu[k] / emu[k] for k in bnd if emu[k] > 0]
            worst = sorted(margin, key=margin.get)[:5]
            kinds = {}
            for k in gpu:
                kind = k.split(":")[0]
                kinds.setdefault(kind, []).append(gpu[k])
            print(json.dumps({
                "suite": "strict", "case": c["tag"], "dtype": str(cd)[6:],
                "n_quantities": len(bnd), "violations": len(P.check16_strict(gpu, emu, cd)),
                "score_path_rows_bounded": sorted(k for k in bnd if k.endswith("[qk]")),
                "min_margin": round(margin[worst[0]], 3),
                "worst": [{"q": k, "gpu": round(gpu[k], 6), "emulated": round(emu[k], 6),
                           "bound": round(bnd[k], 6), "margin": round(margin[k], 3)}
                          for k in worst],
                "max_err_by_kind": {k: round(max(v), 6) for k, v in kinds.items()},
                "gpu_over_emulated": {"median": round(float(np.median(ratio)), 3),
                                      "p90": round(float(np.percentile(ratio, 90)), 3),
                                      "max": round(float(max(ratio)), 3)}}), flush=True)
    if dump:
        from tests import test_gpu_models as TM
        c = [c for c in spec.COND_CASES if c["tag"] == "cond_tr_fc"][0]
        for name, mut in TM.MUTATIONS.items():
            full["mutations"][name] = TM._mutated_errors(gold, c, torch.bfloat16, mut)
        os.makedirs(dump, exist_ok=True)
        with open(os.path.join(dump, "strict_full.json"), "w") as f:
            json.dump(full, f)
    for c in spec.TT_CASES:
        for cd in (torch.bfloat16, torch.float16):
            gpu = P.run_stats(P.measure(gold, c, cd))
            emu = P.run_stats(P.emulated(gold, c, cd))
            ref = P.ref16_stats(gold, c["tag"], cd)
            print(json.dumps({
                "suite": "vs_reference_autocast", "case": c["tag"], "dtype": str(cd)[6:],
                "gpu": {k: round(v, 6) for k, v in gpu.items()},
                "reference_autocast": {k: round(v, 6) for k, v in ref.items()},
                "emulated": {k: round(v, 6) for k, v in emu.items()}}), flush=True)


if __name__ == "__main__":
    main()
