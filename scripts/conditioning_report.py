"""Conditioning of the golden cases in 16 bits (CPU; reads tests/golden/golden.npz).

For every Two_transformers golden case: (1) the reference's OWN 16-bit error — its CPU autocast
bf16 / fp16 run vs its fp32 run, stored in the goldens by tests/golden/make_golden.py
(ref16_errors); (2) the oracle's exact fp32 gradients after ONLY the weights are rounded to the
16-bit type (what any 16-bit MFMA implementation must do first) vs the fp32 gradients; (3) the
rounding-emulating oracle.  Parameter-gradient errors are relative L2 norms, median / max.

    python scripts/conditioning_report.py > profiles/r03_parity_conditioning.txt"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "joint-multimodal-transformer-6th-abaw_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import jmt_ref as R  # noqa: E402
from tests.golden import spec  # noqa: E402
from tests.oracle_cases import case_losses  # noqa: E402


def grads(c, wdt=None, emulate=None):
    shapes = R.two_transformers_shapes(c["L"], c["jm"], c["fmt"], c["vin"])
    p = R.hash_params(shapes, "", c.get("gains"))
    fcp = R.hash_params({"fc_layer.weight": (512, 1024), "fc_layer.bias": (512,)}, "fc.",
                        c.get("gains"))
    allp = dict(p, **{"fc." + k: v for k, v in fcp.items()})
    with torch.no_grad():
        if wdt is not None:
            for t in allp.values():
                t.copy_(t.to(wdt).float())
    for t in allp.values():
        t.requires_grad_(True)
    a, v, lv, la = spec.tt_inputs(c["tag"], c["B"], c["T"], c["vin"])
    with R.emulate_storage(emulate):
        aud = R.linear(torch.from_numpy(a), fcp["fc_layer.weight"], fcp["fc_layer.bias"])
        vo, ao = R.two_transformers_forward(aud, torch.from_numpy(v), p, c["H"], c["L"], c["jm"],
                                            c["fmt"], c["vin"])
        l1, l2 = case_losses(c, vo, ao, torch.from_numpy(lv), torch.from_numpy(la), R.ccc_loss)
        scale = 1024.0 if emulate == torch.float16 else 1.0
        ((l1 + l2) * scale).backward()
    return {k: t.grad.double() / scale for k, t in allp.items() if t.grad is not None}


def stats(g, ref):
    e = [float((g[k] - ref[k]).norm() / ref[k].norm()) for k in ref if float(ref[k].norm()) > 0]
    return f"median {np.median(e):.4f} max {max(e):.4f}"


def main():
    torch.set_num_threads(8)
    with np.load(os.path.join(REPO, "tests", "golden", "golden.npz")) as z:
        gold = {k: z[k] for k in z.files}
    print(__doc__.strip().splitlines()[0])
    print("parameter-gradient relative L2 errors vs the fp32 reference, per case and 16-bit type\n")
    for c in spec.ALL_TT_CASES:
        ref = grads(c)
        for dt, key in ((torch.bfloat16, "bf16"), (torch.float16, "fp16")):
            pg = gold[f"{c['tag']}/ref16_{key}/pgrad"]
            print(f"{c['tag']:18s} {key}  reference autocast: median {np.median(pg):.4f} "
                  f"max {pg.max():.4f} | fp32 with {key}-rounded weights: "
                  f"{stats(grads(c, wdt=dt), ref)} | emulating oracle: "
                  f"{stats(grads(c, emulate=dt), ref)}", flush=True)


if __name__ == "__main__":
    main()
