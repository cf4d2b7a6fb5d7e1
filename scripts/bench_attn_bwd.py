"""Attention backward A/B at the bench workload's launches: the round-5 pair (jmt_attn_bwd with dQ,
64 rows per block + jmt_attn_dkdv dK / dV) against the round-6 pair (jmt_attn_bwd with dq = NULL:
128-row P / dS kernel + jmt_attn_dkdv with dQ as its third product), same operands, interleaved,
median of `rounds` rounds of `reps` launches each (HIP events on the launch stream).
Shapes: c3 cross-attention (N = 6 x 64 = 384, L = 300), c3 encoders (N = 3 x 64 = 192), c4
cross-attention (N = 6 x 16 = 96, L = 1024); head_dim 512, bf16.
FLOP per launch pair: 5 products (S recompute, dP, dQ, dK, dV) x 2 N L^2 d; the old bwd kernel
does S, dP, dQ, the new one S, dP (its frac is over those products).
    python scripts/bench_attn_bwd.py [N L]"""
import json
import math
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "joint-multimodal-transformer-6th-abaw_amd")]

import torch  # noqa: E402

from jmt import ops  # noqa: E402

PEAK = 2516.6


def timeit(fn, reps):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def run(N, L, reps=10, rounds=5, alias=False):
    E = 512
    cd = torch.bfloat16
    dt = ops.dt(cd)
    g = torch.Generator(device="cuda").manual_seed(0)
    qkv = torch.randn(N, L, 3 * E, device="cuda", generator=g).to(cd).permute(1, 0, 2)
    q, k, v = qkv[..., :E], qkv[..., E:2 * E], qkv[..., 2 * E:]
    st = (qkv.stride(0), qkv.stride(1))
    # ablation: every sequence reads sequence 0's K / V (L2-resident), Q / dO unchanged
    skv = (qkv.stride(0), 0) if alias else st
    o = torch.empty(N, L, E, device="cuda", dtype=cd).permute(1, 0, 2)
    so = (o.stride(0), o.stride(1))
    lse = torch.empty(N * L, device="cuda")
    go = torch.randn(N, L, E, device="cuda", generator=g).to(cd).permute(1, 0, 2)
    ldp = ops.attn_dkdv_ldp(L)
    P = torch.zeros(N * L * ldp, device="cuda", dtype=cd)
    dS = torch.zeros_like(P)
    dqkv = torch.empty(N, L, 3 * E, device="cuda", dtype=cd).permute(1, 0, 2)
    dq, dk, dv = dqkv[..., :E], dqkv[..., E:2 * E], dqkv[..., 2 * E:]
    sd = (dqkv.stride(0), dqkv.stride(1))
    scale = 1.0 / math.sqrt(E)
    ops.attn_fwd(dt, N, 1, L, L, E, q.data_ptr(), st, k.data_ptr(), skv, v.data_ptr(), skv,
                 o.data_ptr(), so, scale, lse)

    def bwd(with_dq):
        return lambda: ops.attn_bwd(dt, N, 1, L, L, E, go.data_ptr(), so, o.data_ptr(), so,
                                    q.data_ptr(), st, k.data_ptr(), skv, v.data_ptr(), skv, lse, P,
                                    dS, ldp, dq.data_ptr() if with_dq else None, sd, scale)

    def dkdv(with_dq):
        extra = (k.data_ptr(), skv, dq.data_ptr(), sd) if with_dq else ()
        return lambda: ops.attn_dkdv(dt, N, 1, L, L, E, P, dS, ldp, go.data_ptr(), so,
                                     q.data_ptr(), st, dk.data_ptr(), sd, dv.data_ptr(), sd,
                                     *extra)

    cases = {"bwd_old": bwd(True), "dkdv_old": dkdv(False), "bwd_new": bwd(False),
             "dkdv_new": dkdv(True)}
    cases["pair_old"] = lambda: (cases["bwd_old"](), cases["dkdv_old"]())
    cases["pair_new"] = lambda: (cases["bwd_new"](), cases["dkdv_new"]())
    for f in cases.values():
        f()
    torch.cuda.synchronize()
    t = {n: [] for n in cases}
    for _ in range(rounds):
        for n, f in cases.items():
            t[n].append(timeit(f, reps))
    m = {n: round(statistics.median(v), 1) for n, v in t.items()}
    u = 2.0 * N * L * L * E           # one product
    r = {"N": N, "L": L, "alias_kv": alias, "us": m,
         "frac": {"bwd_old(S,dP,dQ)": round(3 * u / m["bwd_old"] / 1e6 / PEAK, 4),
                  "bwd_new(S,dP)": round(2 * u / m["bwd_new"] / 1e6 / PEAK, 4),
                  "dkdv_old(dK,dV)": round(2 * u / m["dkdv_old"] / 1e6 / PEAK, 4),
                  "dkdv_new(dK,dV,dQ)": round(3 * u / m["dkdv_new"] / 1e6 / PEAK, 4),
                  "pair_old(5)": round(5 * u / m["pair_old"] / 1e6 / PEAK, 4),
                  "pair_new(5)": round(5 * u / m["pair_new"] / 1e6 / PEAK, 4)}}
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 2:
        run(int(sys.argv[1]), int(sys.argv[2]), alias=len(sys.argv) > 3 and sys.argv[3] == "alias")
    else:
        run(384, 300)
        run(192, 300)
        run(96, 1024, reps=5)
