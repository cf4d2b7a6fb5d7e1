"""Row-kernel micro-benchmark at the c3 step's shapes (bf16, R = B*T = 19200 rows): bias-gradient
column sums (jmt_colsum / _grouped) and LayerNorm forward / backward (single and grouped), timed
in isolation with events on the launching stream.
    python scripts/bench_rowops.py [--reps 50] [--out file.jsonl]
Prints per case: us/launch pair and algorithmic GB/s (bytes each kernel must move once)."""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "joint-multimodal-transformer-6th-abaw_amd")]

import torch  # noqa: E402

from jmt import _lib, ops  # noqa: E402

R = 19200
DEV = "cuda"


def timeit(fn, reps):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    _lib.load()
    res = []

    def rec(name, us, nbytes):
        d = {"case": name, "us": round(us, 2), "gbs": round(nbytes / us / 1e3, 1)}
        res.append(d)
        print(json.dumps(d), flush=True)

    bf = torch.bfloat16
    for N in (128, 512, 1024, 1536, 2048):
        dy = torch.randn(R, N, device=DEV).to(bf)
        db = torch.zeros(N, device=DEV)
        rec(f"colsum {R}x{N}", timeit(lambda: ops.colsum(dy, N, R, N, db, True), args.reps),
            R * N * 2.0)
    for G, N in ((3, 512), (3, 2048), (6, 512)):
        dy = torch.randn(G, R, N, device=DEV).to(bf)
        dbs = [torch.zeros(N, device=DEV) for _ in range(G)]
        rec(f"colsum_grouped G{G} {R}x{N}",
            timeit(lambda: ops.colsum_grouped(dy.data_ptr(), _lib.BF16, G, N, R * N, R, N, dbs,
                                              True, DEV), args.reps), G * R * N * 2.0)
    for G, D in ((1, 512), (3, 512), (6, 512), (1, 1024)):
        X = torch.randn(G, R, D, device=DEV).to(bf)
        Rr = torch.randn(G, R, D, device=DEV).to(bf)
        dY = torch.randn(G, R, D, device=DEV).to(bf)
        Y = torch.empty_like(X)
        dX = torch.empty_like(X)
        mean = torch.empty(G * R, device=DEV)
        rstd = torch.empty(G * R, device=DEV)
        gam = [torch.randn(D, device=DEV) for _ in range(G)]
        bet = [torch.randn(D, device=DEV) for _ in range(G)]
        dg = [torch.zeros(D, device=DEV) for _ in range(G)]
        db = [torch.zeros(D, device=DEV) for _ in range(G)]
        ds = [torch.zeros(D, device=DEV) for _ in range(G)]

        def fwd_loop():
            for i in range(G):
                ops.layernorm_fwd(X[i], D, Rr[i], D, gam[i], bet[i], 1e-5, Y[i], D,
                                  mean[i * R:], rstd[i * R:], R, D)

        def bwd_loop():
            for i in range(G):
                ops.layernorm_bwd_dsum(X[i], D, Rr[i], D, dY[i], D, mean[i * R:], rstd[i * R:],
                                       gam[i], dX[i], D, dg[i], db[i], ds[i], True, R, D)

        fb = G * R * D * 2.0 * 3          # x, r read; y written
        bb = G * R * D * 2.0 * 4          # x, r, dy read; dx written
        rec(f"ln_fwd loop G{G} {R}x{D}", timeit(fwd_loop, args.reps), fb)
        rec(f"ln_bwd_dsum loop G{G} {R}x{D}", timeit(bwd_loop, args.reps), bb)
        if G > 1:
            rec(f"ln_fwd grouped G{G} {R}x{D}",
                timeit(lambda: ops.layernorm_fwd_grouped(X, Rr, gam, bet, 1e-5, Y, mean, rstd),
                       args.reps), fb)
            rec(f"ln_bwd_dsum grouped G{G} {R}x{D}",
                timeit(lambda: ops.layernorm_bwd_grouped(X, Rr, dY, mean, rstd, gam, dX, dg, db,
                                                         ds, True), args.reps), bb)
    if args.out:
        with open(args.out, "w") as f:
            for d in res:
                f.write(json.dumps(d) + "\n")


if __name__ == "__main__":
    main()
