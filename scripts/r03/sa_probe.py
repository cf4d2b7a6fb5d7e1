import os, sys, json, numpy as np, torch
sys.path[:0]=['/root/repo','/root/repo/joint-multimodal-transformer-6th-abaw_amd']
from tests.golden import spec
from tests import parity as P
from jmt import functional as JF
with np.load('tests/golden/golden.npz') as z: gold={k:z[k] for k in z.files}
c=[c for c in spec.COND_CASES if c['tag']=='cond_tr_sa'][0]
for pair in (True, False):
    JF.set_pair_mlps(pair)
    for cd in (torch.bfloat16,):
        g=P.measure_strict(gold,c,cd)
        w=sorted(g,key=g.get,reverse=True)[:6]
        print('pair',pair, [(k,round(g[k],4)) for k in w], 'head', round(g['inter:head:grad'],4), flush=True)
JF.set_pair_mlps(True)
from jmt import streams
streams.set_side_enabled(False)
g=P.measure_strict(gold,c,torch.bfloat16); print('noside head', round(g['inter:head:grad'],4), round(g['inter:ca.0:grad'],4))
