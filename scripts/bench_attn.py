"""Attention-kernel micro-benchmark at the bench workload's cross-attention launch (N = 6 pairs x
64 windows = 384 sequences, L = 300, head_dim 512, bf16) and the c4 long window (N = 6 x 16,
L = 1024): jmt_attn_fwd and jmt_attn_bwd launched back to back, HIP events on the launch stream.
Algorithmic FLOP: fwd 4 N L^2 d; bwd (P recompute, dP, dQ) 6 N L^2 d.
    python scripts/bench_attn.py [N L reps]"""
import json
import math
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "joint-multimodal-transformer-6th-abaw_amd")]

import torch  # noqa: E402

from jmt import ops  # noqa: E402

PEAK = 2516.6


def timeit(fn, reps):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def run(N, L, reps, alias=False):
    E = 512
    cd = torch.bfloat16
    dt = ops.dt(cd)
    g = torch.Generator(device="cuda").manual_seed(0)
    qkv = torch.randn(N, L, 3 * E, device="cuda", generator=g).to(cd).permute(1, 0, 2)
    q, k, v = qkv[..., :E], qkv[..., E:2 * E], qkv[..., 2 * E:]
    st = (qkv.stride(0), qkv.stride(1))
    skv = (qkv.stride(0), 0) if alias else st      # ablation: every sequence reads window 0's K/V
    o = torch.empty(N, L, E, device="cuda", dtype=cd).permute(1, 0, 2)
    so = (o.stride(0), o.stride(1))
    lse = torch.empty(N * L, device="cuda")
    go = torch.randn(N, L, E, device="cuda", generator=g).to(cd).permute(1, 0, 2)
    ldp = -(-L // 8) * 8
    P = torch.empty(N * L * ldp, device="cuda", dtype=cd)
    dS = torch.empty_like(P)
    dq = torch.empty_like(o)
    scale = 1.0 / math.sqrt(E)
    fwd = lambda: ops.attn_fwd(dt, N, 1, L, L, E, q.data_ptr(), st, k.data_ptr(), skv,
                               v.data_ptr(), skv, o.data_ptr(), so, scale, lse)
    bwd = lambda: ops.attn_bwd(dt, N, 1, L, L, E, go.data_ptr(), so, o.data_ptr(), so,
                               q.data_ptr(), st, k.data_ptr(), skv, v.data_ptr(), skv, lse, P, dS,
                               ldp, dq.data_ptr(), so, scale)
    fwd()
    tf = timeit(fwd, reps)
    tb = timeit(bwd, reps)
    u = 2.0 * N * L * L * E
    r = {"N": N, "L": L, "alias_kv": alias, "fwd_us": round(tf, 1), "fwd_frac": round(2 * u / tf / 1e6 / PEAK, 4),
         "bwd_us": round(tb, 1), "bwd_frac_3products": round(3 * u / tb / 1e6 / PEAK, 4)}
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 2:
        run(int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]) if len(sys.argv) > 3 else 20,
            len(sys.argv) > 4 and sys.argv[4] == "alias")
    else:
        run(384, 300, 20)
        run(96, 1024, 10)
