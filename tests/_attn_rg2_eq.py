"""The 32-rows-per-wave attention backward (JMT_ATTN_BWD_RG2=1, csrc/attn_bwd2.hip) against the
default 8-wave kernel on the same inputs: P, dS and dQ saved by one process and compared bit for
bit by another (the switch is read once per process).
    python tests/_attn_rg2_eq.py save|cmp FILE     (used by test_gpu_kernels.py)"""
import math
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "joint-multimodal-transformer-6th-abaw_amd")]
import torch  # noqa: E402
from jmt import ops  # noqa: E402

if __name__ != "__main__":
    raise ImportError("script, run as a child process")


def run():
    outs = {}
    E = 512
    for (N, Lq, Lk) in [(3, 300, 300), (2, 70, 129), (1, 1024, 1024), (300, 129, 1)]:
        g = torch.Generator(device="cuda").manual_seed(41)
        qkv = torch.randn(N, Lq, 3 * E, device="cuda", generator=g).bfloat16().permute(1, 0, 2)
        kv = torch.randn(N, Lk, 2 * E, device="cuda", generator=g).bfloat16().permute(1, 0, 2)
        qp, kp, vp = qkv[..., :E], kv[..., :E], kv[..., E:]
        scale = 1.0 / math.sqrt(E)
        dt = ops.dt(qkv)
        o = torch.empty(Lq, N, E, device="cuda", dtype=torch.bfloat16)
        lse = torch.empty(N * Lq, device="cuda")
        st = lambda t: (t.stride(0), t.stride(1))
        ops.attn_fwd(dt, N, 1, Lq, Lk, E, qp.data_ptr(), st(qkv), kp.data_ptr(), st(kv),
                     vp.data_ptr(), st(kv), o.data_ptr(), st(o), scale, lse)
        go = torch.randn(Lq, N, E, device="cuda", generator=g).bfloat16()
        ldp = ops.attn_dkdv_ldp(Lk)
        P = torch.zeros(N * Lq * ldp, device="cuda", dtype=torch.bfloat16)
        dS = torch.zeros_like(P)
        dq = torch.zeros(N, Lq, 3 * E, device="cuda", dtype=torch.bfloat16).permute(1, 0, 2)
        ops.attn_bwd(dt, N, 1, Lq, Lk, E, go.data_ptr(), st(go), o.data_ptr(), st(o),
                     qp.data_ptr(), st(qkv), kp.data_ptr(), st(kv), vp.data_ptr(), st(kv), lse,
                     P, dS, ldp, dq[..., E:2 * E].data_ptr(), st(dq), scale)
        torch.cuda.synchronize()
        key = f"{N}_{Lq}_{Lk}"
        outs[key + "_P"], outs[key + "_dS"], outs[key + "_dq"] = P.cpu(), dS.cpu(), dq.cpu()
    return outs


mode, path = sys.argv[1], sys.argv[2]
o = run()
if mode == "save":
    torch.save(o, path)
    print("saved", len(o))
else:
    ref = torch.load(path, weights_only=True)
    bad = [k for k in ref if not torch.equal(ref[k], o[k])]
    print("compared", len(ref), "mismatch", bad)
    sys.exit(1 if bad else 0)
