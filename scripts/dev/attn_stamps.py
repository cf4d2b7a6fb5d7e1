"""Diagnostic: per-phase cycle breakdown of the 8-wave 16x16 attention forward (phase stamps of
one block in the middle of the grid, waves 0 and 4), at the cross-attention launch of the bench
(N = 384, L = 300).  Phases per 64-key tile: S MFMAs | wait V DMA | barrier 1 | softmax |
P V MFMAs | wait K DMA | barrier 2."""
import ctypes, math, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "joint-multimodal-transformer-6th-abaw_amd")]
import torch
from jmt import ops, _lib

N, L, E = int(sys.argv[1]) if len(sys.argv) > 1 else 384, 300, 512
cd = torch.bfloat16
lib = _lib.load()
lib.jmt_attn_set_stamps.argtypes = [ctypes.c_void_p]
buf = torch.zeros(2 * 256 * 64, dtype=torch.int64, device="cuda")
qkv = torch.randn(N, L, 3 * E, device="cuda").to(cd).permute(1, 0, 2)
st = (qkv.stride(0), qkv.stride(1))
o = torch.empty(N, L, E, device="cuda", dtype=cd).permute(1, 0, 2)
lse = torch.empty(N * L, device="cuda")
run = lambda: ops.attn_fwd(ops.dt(cd), N, 1, L, L, E, qkv[..., :E].data_ptr(), st,
                           qkv[..., E:2 * E].data_ptr(), st, qkv[..., 2 * E:].data_ptr(), st,
                           o.data_ptr(), (o.stride(0), o.stride(1)), 1 / math.sqrt(E), lse)
run(); torch.cuda.synchronize()
lib.jmt_attn_set_stamps(buf.data_ptr())
for _ in range(3):
    run()
torch.cuda.synchronize()
lib.jmt_attn_set_stamps(None)
b = buf.view(2, 256, 64)[:, :, 0].cpu().tolist()
names = ["S mfma", "wait V", "barrier1", "softmax", "PV mfma", "wait K", "barrier2"]
for wv in range(2):
    t0, tend = b[wv][255], b[wv][254]
    print(f"wave {4 * wv}: total {tend - t0} cycles, prologue {b[wv][0] - t0}")
    tot = [0] * 7
    for j in range(5):
        st_ = [b[wv][8 * j + k] for k in range(7)]
        nxt = b[wv][8 * (j + 1)] if j < 4 else tend
        seq = st_ + [nxt]
        d = [seq[k + 1] - seq[k] for k in range(7)] if j < 4 else \
            [seq[1] - seq[0], seq[2] - seq[1], seq[3] - seq[2], seq[4] - seq[3], seq[5] - seq[4], 0, tend - seq[5]]
        tot = [a + c for a, c in zip(tot, d)]
        print("  tile", j, " ".join(f"{n}={x}" for n, x in zip(names, d)))
    print("  sum  ", " ".join(f"{n}={x}" for n, x in zip(names, tot)))
