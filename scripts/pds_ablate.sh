#!/bin/bash
# Ablations of the 128-row P / dS attention backward kernel (diagnostic build, JMT_ATTN_PDS_DBG
# bits: 1 no next-item row loads, 2 no MFMAs, 4 no P / dS stores, 8 no K / V DMA; results wrong,
# timing only) at the c3 cross-attention launch.  Usage: scripts/pds_ablate.sh OUT
OUT=${1:-gpurun_out/r06/pds_ablate.txt}
for d in ${DBGS:-0 1 2 4 8 6 3 7 15}; do
  JMT_LIB=joint-multimodal-transformer-6th-abaw_amd/jmt/libjmt_hip_diag.so JMT_ATTN_PDS_DBG=$d \
    timeout -k 10 60 python -u - <<'PY' >> "$OUT" 2>&1 || exit 1
import math, os, sys, statistics, torch
sys.path[:0] = ["joint-multimodal-transformer-6th-abaw_amd"]
from jmt import ops
N, L, E = 384, 300, 512
cd = torch.bfloat16; dt = ops.dt(cd)
g = torch.Generator(device="cuda").manual_seed(0)
qkv = torch.randn(N, L, 3 * E, device="cuda", generator=g).to(cd).permute(1, 0, 2)
q, k, v = qkv[..., :E], qkv[..., E:2 * E], qkv[..., 2 * E:]
st = (qkv.stride(0), qkv.stride(1))
o = torch.empty(N, L, E, device="cuda", dtype=cd).permute(1, 0, 2); so = (o.stride(0), o.stride(1))
if os.environ.get("ALIAS_ALL"):     # every sequence reads sequence 0's rows: all L2-resident
    st = (qkv.stride(0), 0); so = (o.stride(0), 0)
lse = torch.empty(N * L, device="cuda")
go = torch.randn(N, L, E, device="cuda", generator=g).to(cd).permute(1, 0, 2)
ldp = ops.attn_dkdv_ldp(L)
P = torch.zeros(N * L * ldp, device="cuda", dtype=cd); dS = torch.zeros_like(P)
ops.attn_fwd(dt, N, 1, L, L, E, q.data_ptr(), st, k.data_ptr(), st, v.data_ptr(), st, o.data_ptr(), so, 1 / math.sqrt(E), lse)
f = lambda: ops.attn_bwd(dt, N, 1, L, L, E, go.data_ptr(), so, o.data_ptr(), so, q.data_ptr(), st, k.data_ptr(), st, v.data_ptr(), st, lse, P, dS, ldp, None, st, 1 / math.sqrt(E))
for _ in range(3): f()
torch.cuda.synchronize()
ts = []
for _ in range(5):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(10): f()
    e.record(); torch.cuda.synchronize(); ts.append(s.elapsed_time(e) * 100)
print(f"dbg {os.environ['JMT_ATTN_PDS_DBG']:>2}: {statistics.median(ts):7.1f} us  (N {N} L {L}"
      f"{' alias_all' if os.environ.get('ALIAS_ALL') else ''})", flush=True)
PY
done
