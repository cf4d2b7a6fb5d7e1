"""SELF_ATTEN conditioned case, bf16: where the GPU's head gradient differs from the fp32
oracle (per row / per column), vs the rounding-emulating oracle (diagnostic)."""
import sys, numpy as np, torch
sys.path[:0] = ['.', 'joint-multimodal-transformer-6th-abaw_amd']
from tests.golden import spec
from tests import parity as P
from tests.oracle_cases import oracle_tt
c = [c for c in spec.COND_CASES if c['tag'] == 'cond_tr_sa'][0]
torch.set_num_threads(16)
ref = oracle_tt(c)
emu = oracle_tt(c, torch.bfloat16)
res = P.run_tt(c, torch.bfloat16, record=True)
store = res[5]
for name in ('head', 'ca.0'):
    g = store[name]['grad'].double().cpu().reshape(-1, 512)
    r = ref['taps'][name]['grad'].double().reshape(-1, 512)
    e = emu['taps'][name]['grad'].double().reshape(-1, 512)
    print(name, 'gpu', float((g - r).norm() / r.norm()), 'emu', float((e - r).norm() / r.norm()),
          'gpu-emu', float((g - e).norm() / r.norm()))
    rows = ((g - r).norm(dim=1) / r.norm(dim=1)).numpy()
    print(' per-row gpu err', np.round(rows[:16], 4), 'emu', np.round(((e - r).norm(dim=1) / r.norm(dim=1)).numpy()[:16], 4))
    d = (g - r)
    print(' mean err / mean |r|', float(d.mean() / r.abs().mean()), 'corr(err, r)', float((d * r).sum() / (d.norm() * r.norm())))
vo, ao = res[0].float().cpu(), res[1].float().cpu()
print('vouts err mean', float((vo - torch.from_numpy(ref['vouts'])).mean()), 'emu', float((torch.from_numpy(emu['vouts']) - torch.from_numpy(ref['vouts'])).mean()))
print('aouts err mean', float((ao - torch.from_numpy(ref['aouts'])).mean()), 'emu', float((torch.from_numpy(emu['aouts']) - torch.from_numpy(ref['aouts'])).mean()))
print('aouts ref mean', float(np.mean(ref['aouts'])), 'std', float(np.std(ref['aouts'])))
