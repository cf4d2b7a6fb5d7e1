"""Phase stamps of the 128-row P / dS attention backward kernel (diagnostic build: make diag,
JMT_ATTN_PDS_DBG=64): s_memtime of block gridDim / 2, waves 0 and 4, at the phase boundaries of
its first 31 tiles, printed as mean cycles per phase at the c3 cross-attention launch.
    JMT_LIB=.../libjmt_hip_diag.so JMT_ATTN_PDS_DBG=64 python scripts/pds_stamps.py [N L]"""
import ctypes
import math
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "joint-multimodal-transformer-6th-abaw_amd")]
import torch  # noqa: E402
from jmt import ops, _lib  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 384
L = int(sys.argv[2]) if len(sys.argv) > 2 else 300
E = 512
cd = torch.bfloat16
dt = ops.dt(cd)
g = torch.Generator(device="cuda").manual_seed(0)
qkv = torch.randn(N, L, 3 * E, device="cuda", generator=g).to(cd).permute(1, 0, 2)
q, k, v = qkv[..., :E], qkv[..., E:2 * E], qkv[..., 2 * E:]
st = (qkv.stride(0), qkv.stride(1))
o = torch.empty(N, L, E, device="cuda", dtype=cd).permute(1, 0, 2)
so = (o.stride(0), o.stride(1))
lse = torch.empty(N * L, device="cuda")
go = torch.randn(N, L, E, device="cuda", generator=g).to(cd).permute(1, 0, 2)
ldp = ops.attn_dkdv_ldp(L)
P = torch.zeros(N * L * ldp, device="cuda", dtype=cd)
dS = torch.zeros_like(P)
ops.attn_fwd(dt, N, 1, L, L, E, q.data_ptr(), st, k.data_ptr(), st, v.data_ptr(), st,
             o.data_ptr(), so, 1 / math.sqrt(E), lse)
stamps = torch.zeros(2 * 256 * 64, dtype=torch.int64, device="cuda")
lib = _lib.load()
lib.jmt_attn_set_stamps.argtypes = [ctypes.c_void_p]
assert lib.jmt_attn_set_stamps(ctypes.c_void_p(stamps.data_ptr())) == 0
for _ in range(3):
    ops.attn_bwd(dt, N, 1, L, L, E, go.data_ptr(), so, o.data_ptr(), so, q.data_ptr(), st,
                 k.data_ptr(), st, v.data_ptr(), st, lse, P, dS, ldp, None, st, 1 / math.sqrt(E))
torch.cuda.synchronize()
lib.jmt_attn_set_stamps(None)
t = stamps.view(2, 256, 64)[:, :, 0].cpu().tolist()        # lane 0 of waves 0 and 4
names = ["DMA issue", "MFMA (S, dP)", "softmax + stores", "end wait", "barrier", "-> next"]
for wv in range(2):
    acc = [[] for _ in names]
    for tt in range(30):
        b = 8 * tt
        ph = [t[wv][b + i] for i in range(6)] + [t[wv][b + 8]]
        if not all(ph[:4]) or not ph[6]:
            continue
        for i in range(6):
            if ph[i + 1] and ph[i] and (i < 3 or (ph[4] and ph[5])):
                acc[i].append(ph[i + 1] - ph[i])
    print(f"wave {4 * wv}: " + ", ".join(
        f"{n} {sum(a) / len(a):.0f}" for n, a in zip(names, acc) if a) + "  (cycles, mean)")
