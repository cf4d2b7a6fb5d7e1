"""jmt_attn_dkdv vs the two batched TN GEMMs it replaces (dK = dS^T Q, dV = P^T dO), same
operands, interleaved in one process.   python scripts/bench_dkdv.py [--reps 30]"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "joint-multimodal-transformer-6th-abaw_amd")]

import torch  # noqa: E402

from jmt import ops  # noqa: E402
from jmt._lib import BF16  # noqa: E402

SHAPES = [(384, 300), (192, 300), (32, 1024), (16, 1024)]   # (N*H sequences, L)


def time_us(fn, reps):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(reps):
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) * 1e3)
    ts.sort()
    return ts[len(ts) // 2], ts[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--shapes", type=int, nargs="*", help="indices into SHAPES")
    ap.add_argument("--only", choices=["dkdv", "gemm"], help="time one implementation")
    args = ap.parse_args()
    dev = "cuda"
    E = 512
    for i, (N, L) in enumerate(SHAPES):
        if args.shapes and i not in args.shapes:
            continue
        g = torch.Generator(device=dev).manual_seed(1)
        ldp = ops.attn_dkdv_ldp(L)
        P = (torch.rand(N, L, ldp, device=dev, generator=g)).bfloat16()
        dS = (torch.randn(N, L, ldp, device=dev, generator=g) * 0.1).bfloat16()
        qkv = torch.randn(N, L, 3 * E, device=dev, generator=g).bfloat16().permute(1, 0, 2)
        go = torch.randn(N, L, E, device=dev, generator=g).bfloat16().permute(1, 0, 2)
        out = torch.empty(N, L, 3 * E, device=dev).bfloat16().permute(1, 0, 2)
        st = lambda t: (t.stride(0), t.stride(1))

        def fused():
            ops.attn_dkdv(BF16, N, 1, L, L, E, P, dS, ldp, go.data_ptr(), st(go),
                          qkv.data_ptr(), st(qkv), out[..., E:].data_ptr(), st(out),
                          out[..., 2 * E:].data_ptr(), st(out))

        def gemms():
            for A, B, c0 in ((dS, qkv, E), (P, go, 2 * E)):
                ops.gemm(M=L, N=E, K=L, ab_dtype=BF16, c_dtype=BF16, a=[A.data_ptr()], lda=ldp,
                         a_kmajor=False, sA=(L * ldp, L * ldp), b=[B.data_ptr()],
                         ldb=B.stride(0), b_kmajor=False, sB=(B.stride(1), E),
                         c=[out[..., c0:].data_ptr()], ldc=out.stride(0),
                         sC=(out.stride(1), E), batch0=N, batch1=1, device=dev)
        for f in (fused, gemms):
            f()
        torch.cuda.synchronize()
        res = {}
        for r in range(2):
            for name, f in (("dkdv", fused), ("gemm", gemms)):
                if args.only and name != args.only:
                    continue
                med, mn = time_us(f, args.reps)
                res.setdefault(name, []).append(med)
        flops = 4.0 * N * L * L * E
        nbytes = N * (2 * L * ldp * 2 + 2 * L * E * 2 + 2 * L * E * 2)
        line = {"shape": f"N*H={N} L={L}", "flops": flops, "bytes": nbytes}
        for k, v in res.items():
            m = min(v)
            line[k] = {"us": round(m, 2), "tflops": round(flops / m / 1e6, 1),
                       "gbs": round(nbytes / m / 1e3, 1)}
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
