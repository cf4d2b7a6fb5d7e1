"""GEMM micro-benchmark on the JMT step's shapes (bf16), with optional ablations:
    python scripts/bench_gemm.py [--dbg 0|1|2|3] [--reps 50] [--cfg 0 43 44] [--only a,b]
(JMT_GEMM_PPSPLIT=0 in the environment: the weight-gradient shapes take the one-block split-K
plan instead of the split-K ping-pong kernel, cfg 44)
Prints per shape: µs/launch, TFLOP/s, and the algorithmic-bytes GB/s."""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "joint-multimodal-transformer-6th-abaw_amd")]

import torch  # noqa: E402

from jmt import _lib, ops  # noqa: E402
from jmt._lib import BF16, F32  # noqa: E402

# (name, M, N, K, a_kmajor, b_kmajor, batch, c_dtype, splits)
SHAPES = [
    ("fwd 19200x512x512 NT", 19200, 512, 512, True, True, 1, BF16, 1),
    ("fwd qkv 19200x1536x512 NT", 19200, 1536, 512, True, True, 1, BF16, 1),
    ("fwd b3 19200x512x512 NT", 19200, 512, 512, True, True, 3, BF16, 1),
    ("fwd b6 19200x512x512 NT", 19200, 512, 512, True, True, 6, BF16, 1),
    ("fwd 19200x1024x512 NT", 19200, 1024, 512, True, True, 1, BF16, 1),
    ("fwd out1 19200x1024x3072 NT", 19200, 1024, 3072, True, True, 1, BF16, 1),
    ("dgrad 19200x512x512 NN", 19200, 512, 512, True, False, 1, BF16, 1),
    ("dgrad b3 19200x512x512 NN", 19200, 512, 512, True, False, 3, BF16, 1),
    ("fwd b6 19200x1024x512 NT", 19200, 1024, 512, True, True, 6, BF16, 1),
    ("dgrad b6 19200x512x1024 NN", 19200, 512, 1024, True, False, 6, BF16, 1),
    ("dgrad out1 19200x3072x1024 NN", 19200, 3072, 1024, True, False, 1, BF16, 1),
    ("wgrad out1 1024x3072x19200 TN", 1024, 3072, 19200, False, False, 1, F32, None),
    ("wgrad 512x512x19200 TN", 512, 512, 19200, False, False, 1, F32, None),
    ("wgrad b3 512x512x19200 TN", 512, 512, 19200, False, False, 3, F32, None),
    ("wgrad b3 1024x512x19200 TN", 1024, 512, 19200, False, False, 3, F32, None),
    ("wgrad b6 1024x512x19200 TN", 1024, 512, 19200, False, False, 6, F32, None),
    ("wgrad b3 1536x512x19200 TN", 1536, 512, 19200, False, False, 3, F32, None),
    ("wgrad 512x2048x19200 TN", 512, 2048, 19200, False, False, 1, F32, None),
    ("attn S 300x300x512 b64 NT", 300, 300, 512, True, True, 64, F32, 1),
    ("attn PV 300x512x300 b64 NN", 300, 512, 300, True, False, 64, BF16, 1),
    ("attn dK 300x512x300 b64 TN", 300, 512, 300, False, False, 64, BF16, 1),
]


def run(reps, dbg, cfg=0):
    lib = _lib.load()
    lib.jmt_gemm_set_debug(dbg | (cfg << 8))
    dev = "cuda"
    out = []
    for name, M, N, K, ak, bk, batch, cdt, splits in SHAPES:
        a = torch.randn(batch, M * K, device=dev).bfloat16()
        b = torch.randn(batch, N * K, device=dev).bfloat16()
        c = torch.empty(batch, M * N, device=dev,
                        dtype=torch.float32 if cdt == F32 else torch.bfloat16)
        r8 = lambda v: -(-v // 8) * 8
        lda = r8(K) if ak else r8(M)
        ldb = r8(K) if bk else r8(N)
        a = torch.randn(batch, (M if ak else K) * lda, device=dev).bfloat16()
        b = torch.randn(batch, (N if bk else K) * ldb, device=dev).bfloat16()
        kw = dict(M=M, N=N, K=K, ab_dtype=BF16, c_dtype=cdt, a=[a.data_ptr()], lda=lda,
                  a_kmajor=ak, b=[b.data_ptr()], ldb=ldb, b_kmajor=bk, c=[c.data_ptr()], ldc=N,
                  batch0=batch, sA=(a.shape[1], 0), sB=(b.shape[1], 0), sC=(M * N, 0), splits=splits,
                  device=dev)
        for _ in range(3):
            ops.gemm(**kw)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            ops.gemm(**kw)
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) / reps * 1e3
        fl = 2.0 * M * N * K * batch
        by = (M * K + N * K) * 2 * batch + M * N * c.element_size() * batch
        r = {"shape": name, "dbg": dbg, "cfg": cfg, "us": round(us, 2), "tflops": round(fl / us / 1e6, 1),
             "gbs": round(by / us / 1e3, 1)}
        out.append(r)
        print(json.dumps(r), flush=True)
    lib.jmt_gemm_set_debug(0)
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--dbg", type=int, nargs="*", default=[0])
    ap.add_argument("--only", default="", help="substring filter on shape names")
    ap.add_argument("--cfg", type=int, nargs="*", default=[0])
    ap.add_argument("--copy", action="store_true", help="also time torch copy/fill of C-sized buffers")
    args = ap.parse_args()
    if args.copy:
        for mb in (19.6, 39.3, 78.6):
            n = int(mb * 1e6 / 2)
            x = torch.empty(n, dtype=torch.bfloat16, device="cuda")
            y = torch.empty_like(x)
            for name, fn, by in (("fill", lambda: y.fill_(1.0), n * 2), ("copy", lambda: y.copy_(x), n * 4)):
                for _ in range(3):
                    fn()
                torch.cuda.synchronize()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(50):
                    fn()
                e.record()
                torch.cuda.synchronize()
                us = s.elapsed_time(e) / 50 * 1e3
                print(json.dumps({"op": name, "MB": mb, "us": round(us, 2), "gbs": round(by / us / 1e3, 1)}))
    if args.only:
        keys = args.only.split(",")
        SHAPES[:] = [s for s in SHAPES if any(k in s[0] for k in keys)]
    for c in args.cfg:
        for d in args.dbg:
            run(args.reps, d, c)
