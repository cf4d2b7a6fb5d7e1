"""GEMM micro-benchmark on the grouped JMT step's launch shapes (bf16), as the model issues them
(pointer-table weights, beta=1 accumulate, ReLU-mask aux, K-concat):
    python scripts/bench_gemm_step.py [--cfg 0 1 5] [--only substr] [--reps 30]
Prints per shape: us/launch, TFLOP/s, algorithmic GB/s."""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "joint-multimodal-transformer-6th-abaw_amd")]

import torch  # noqa: E402

from jmt import _lib, ops  # noqa: E402
from jmt._lib import BF16, F32  # noqa: E402

R = 19200
# name, M, N, K, a_kmajor, b_kmajor, batch, c_dtype, extra
def make_shapes(R):
    return [
        ("enc b3 fwd NT 512x512", R, 512, 512, True, True, 3, BF16, {}),
        ("enc b3 qkv NT 1536x512", R, 1536, 512, True, True, 3, BF16, {}),
        ("enc b3 dgrad NN 512x512", R, 512, 512, True, False, 3, BF16, {}),
        ("enc b3 dgrad NN beta", R, 512, 512, True, False, 3, BF16, {"beta": 1.0}),
        ("enc b3 dgrad NN aux", R, 512, 512, True, False, 3, BF16, {"aux": True}),
        ("enc b3 dgrad NN K1536 beta", R, 512, 1536, True, False, 3, BF16, {"beta": 1.0}),
        ("ca b6 dgrad NN 512x512", R, 512, 512, True, False, 6, BF16, {}),
        ("stack b2 dgrad NN 512x512 beta", R, 512, 512, True, False, 2, BF16, {"beta": 1.0}),
        ("ca b6 dgrad NN 512x1024", R, 512, 1024, True, False, 6, BF16, {}),
        ("ca b6 kv NT 1024x512", R, 1024, 512, True, True, 6, BF16, {}),
        ("stream dgrad kcat6 NN 512x3072", R, 512, 3072, True, False, 1, BF16, {"kcat": 6}),
        ("head dgrad b6 NN 512x1024", R, 512, 1024, True, False, 6, BF16, {"sA0": True}),
        ("head fwd kcat6 NT 1024x3072", R, 1024, 3072, True, True, 1, BF16, {"kcat": 6}),
        ("wgrad b3 TN 512x512xR", 512, 512, R, False, False, 3, F32, {"beta": 1.0}),
        ("wgrad b3 TN 1536x512xR", 1536, 512, R, False, False, 3, F32, {"beta": 1.0}),
        ("attn dKdV b384 TN 300x512x300", 300, 512, 300, False, False, 384, BF16, {}),
        ("regressor dgrad NN 1024x128", R, 1024, 128, True, False, 1, BF16, {}),
        ("regressor dgrad NN 1024x128 beta", R, 1024, 128, True, False, 1, BF16, {"beta": 1.0}),
        ("regressor fwd pair NT 128x1024 relu", R, 128, 1024, True, True, 2, BF16, {"sA0": True}),
        ("attn dKdV b384 TN 300x512x320 (K padded)", 300, 512, 320, False, False, 384, BF16, {}),
        # round 3: P^T / dS^T handed over key-major (K-major A), so the 160-row tile applies
        ("attn dKdV b384 NN 300x512x300 (dS^T K-major)", 300, 512, 300, True, False, 384, BF16, {}),
        ("attn dKdV b192 NN 300x512x300 (dS^T K-major)", 300, 512, 300, True, False, 192, BF16, {}),
        ("attn dKdV b192 TN 300x512x300", 300, 512, 300, False, False, 192, BF16, {}),
        ("attn dKdV b384 TN 320x512x320 (M, K padded)", 320, 512, 320, False, False, 384, BF16, {}),
        ("attn dKdV b768 TN 300x512x300 (dK + dV)", 300, 512, 300, False, False, 768, BF16, {}),
        ("attn dKdV b768 TN 300x512x320 (dK + dV, K padded)", 300, 512, 320, False, False, 768, BF16, {}),
        ("ca wgrad b6 TN 1024x512xR", 1024, 512, R, False, False, 6, F32, {"beta": 1.0}),
        ("ca wgrad b6 TN 512x512xR", 512, 512, R, False, False, 6, F32, {"beta": 1.0}),
        ("enc wgrad b3 TN 512x1536xR", 512, 1536, R, False, False, 3, F32, {"beta": 1.0}),
        # round 3: the same weight gradients with their bias gradients as A row sums (dbias_tab)
        ("wgrad b3 TN 512x512xR +dbias", 512, 512, R, False, False, 3, F32, {"beta": 1.0, "dbias": True}),
        ("wgrad b3 TN 1536x512xR +dbias", 1536, 512, R, False, False, 3, F32, {"beta": 1.0, "dbias": True}),
        ("ca wgrad b6 TN 1024x512xR +dbias", 1024, 512, R, False, False, 6, F32, {"beta": 1.0, "dbias": True}),
        ("ca wgrad b6 TN 512x512xR +dbias", 512, 512, R, False, False, 6, F32, {"beta": 1.0, "dbias": True}),
        ("enc wgrad b3 TN 512x1536xR +dbias", 512, 1536, R, False, False, 3, F32, {"beta": 1.0, "dbias": True}),
        ("video linear fwd NT 512x2048", R, 512, 2048, True, True, 1, BF16, {}),
        ("fc fwd NT 512x1024", R, 512, 1024, True, True, 1, BF16, {}),
        ("pv dgrad NN 1024x512 b1", R, 1024, 512, True, False, 1, BF16, {}),
        ("head dgrad NN 512x1024 b1", R, 512, 1024, True, False, 1, BF16, {}),
    ]


SHAPES = make_shapes(R)


def run(reps, cfg, dbg=0, splits=None):
    lib = _lib.load()
    lib.jmt_gemm_set_debug(dbg | (cfg << 8))
    dev = "cuda"
    for name, M, N, K, ak, bk, batch, cdt, ex in SHAPES:
        r8 = lambda v: -(-v // 8) * 8
        kc = ex.get("kcat", 0)
        lda = r8(K // kc if kc else K) if ak else r8(M)
        ldb = r8(K // kc if kc else K) if bk else r8(N)
        arows = (M if ak else (K // kc if kc else K))
        brows = (N if bk else (K // kc if kc else K))
        nseg = kc if kc else 1
        A = [torch.randn(batch, arows * lda, device=dev).bfloat16() for _ in range(nseg)]
        Bt = [torch.randn(batch, brows * ldb, device=dev).bfloat16() for _ in range(max(nseg, 1))]
        c = torch.zeros(batch, M * N, device=dev, dtype=torch.float32 if cdt == F32 else torch.bfloat16)
        aux = torch.randn(batch, M * N, device=dev).bfloat16() if ex.get("aux") else None
        kw = dict(M=M, N=N, K=K, ab_dtype=BF16, c_dtype=cdt, lda=lda, a_kmajor=ak, ldb=ldb,
                  b_kmajor=bk, c=[c.data_ptr()], ldc=N, batch0=batch, sC=(M * N, 0),
                  beta=ex.get("beta", 0.0), aux=aux, ldaux=N if aux is not None else 0, device=dev,
                  splits=splits)
        if kc:
            kw.update(a=[a.data_ptr() for a in A], a_mode=2, a_kseg=K // kc,
                      b=[b.data_ptr() for b in Bt], b_mode=2, b_kseg=K // kc)
        else:
            kw.update(a=[A[0].data_ptr()], sA=(0 if ex.get("sA0") else A[0].shape[1], 0))
            if batch > 1 and batch <= 8:   # weights as a pointer table, as the model issues them
                kw.update(b=[Bt[0][i].data_ptr() for i in range(batch)], b_mode=1)
            else:
                kw.update(b=[Bt[0].data_ptr()], sB=(Bt[0].shape[1], 0))
        if ex.get("dbias"):
            kw.update(dbias_tab=[torch.zeros(M, device=dev) for _ in range(batch)])
        for _ in range(3):
            ws = ops.gemm(**kw)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            ws = ops.gemm(**kw)
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) / reps * 1e3
        fl = 2.0 * M * N * K * batch
        by = (M * K + N * K) * 2 * batch + M * N * c.element_size() * batch
        splits_used = splits or ops.auto_splits(M, N, K, batch, BF16)
        print(json.dumps({"shape": name, "cfg": cfg, "dbg": dbg, "splits": splits_used, "us": round(us, 2),
                          "tflops": round(fl / us / 1e6, 1), "gbs": round(by / us / 1e3, 1)}),
              flush=True)
        del ws
    lib.jmt_gemm_set_debug(0)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--cfg", type=int, nargs="*", default=[0])
    ap.add_argument("--only", default="")
    ap.add_argument("--dbg", type=int, nargs="*", default=[0])
    ap.add_argument("--rows", type=int, default=R, help="tokens per stream (realdata: 1024)")
    ap.add_argument("--splits", type=int, nargs="*", default=[0], help="forced split-K (0: planner)")
    args = ap.parse_args()
    SHAPES[:] = make_shapes(args.rows)
    if args.only:
        SHAPES[:] = [s for s in SHAPES if args.only in s[0]]
    for c in args.cfg:
        for d in args.dbg:
            for sp in args.splits:
                run(args.reps, c, d, sp or None)
