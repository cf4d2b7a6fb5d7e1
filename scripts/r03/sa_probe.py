"""Which quantities of the SELF_ATTEN conditioned case deviate more on the GPU (bf16) than under
the rounding-emulating oracle (diagnostic for the strict parity suite)."""
import os, sys, numpy as np, torch
sys.path[:0] = ['.', 'joint-multimodal-transformer-6th-abaw_amd']
from tests.golden import spec
from tests import parity as P
with np.load('tests/golden/golden.npz') as z:
    gold = {k: z[k] for k in z.files}
c = [c for c in spec.COND_CASES if c['tag'] == 'cond_tr_sa'][0]
for cd in (torch.bfloat16, torch.float16):
    g = P.measure_strict(gold, c, cd)
    e = P.emulated_strict(gold, c, cd)
    keys = sorted(g, key=lambda k: -g[k] / max(e[k], 1e-9))
    print(str(cd), 'ratio-worst', [(k, round(g[k], 4), round(e[k], 4)) for k in keys[:8]], flush=True)
    print(str(cd), 'vals', [(k, round(g[k], 4), round(e[k], 4)) for k in g if k.endswith(':val') or k.startswith('out:')], flush=True)
