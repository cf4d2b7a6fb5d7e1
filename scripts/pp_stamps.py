"""Segment timeline of the ping-pong persistent GEMM (gemm_persist.hip cfg 43, dbg 8): one launch
of a step shape with s_memtime stamps of block 0's waves, printed as per-segment cycle counts
(median over the K-tiles 2..23, then the first K-tiles raw).

    python scripts/pp_stamps.py [--shape NT_b6_1024] [--dbg-extra 0]
Stamps per (wave, K-tile, phase): 0 load-segment start, 6 epilogue half done, 7 stream K-tile
step done, 1 LDS reads issued, 2 DMA issued, 3 deadline wait done, 4 after the barrier (MFMA
segment start), 5 MFMAs issued (+ deadline).  Per-K-tile rows list, per phase: [epilogue, step,
reads, dma, deadline, barrier1, mfma, barrier2]."""
import argparse
import ctypes as C
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "joint-multimodal-transformer-6th-abaw_amd")]

import torch  # noqa: E402

from jmt import _lib, ops  # noqa: E402
from jmt._lib import BF16  # noqa: E402

SHAPES = {"NT_b6_1024": (19200, 1024, 512, True, True, 6),
          "NT_b3_512": (19200, 512, 512, True, True, 3),
          "NN_b6_1024": (19200, 512, 1024, True, False, 6)}
PP_STK = 24


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="NT_b6_1024", choices=sorted(SHAPES))
    ap.add_argument("--dbg-extra", type=int, default=0)
    args = ap.parse_args()
    M, N, K, ak, bk, b = SHAPES[args.shape]
    lib = _lib.load()
    dev = "cuda"
    a = (torch.rand(b, M * K, device=dev) * 2 - 1).bfloat16()
    w = (torch.rand(b, N * K, device=dev) * 2 - 1).bfloat16()
    c = torch.empty(b, M * N, device=dev, dtype=torch.bfloat16)
    kw = dict(M=M, N=N, K=K, ab_dtype=BF16, c_dtype=BF16, a=[a.data_ptr()], lda=K,
              a_kmajor=ak, b=[w.data_ptr()], ldb=K if bk else N, b_kmajor=bk, c=[c.data_ptr()],
              ldc=N, batch0=b, sA=(M * K, 0), sB=(N * K, 0), sC=(M * N, 0), splits=1, device=dev)
    for dbg in (0, 8 | args.dbg_extra):
        lib.jmt_gemm_set_debug((43 << 8) | dbg)
        for _ in range(3):
            ops.gemm(**kw)
        torch.cuda.synchronize()
    lib.jmt_gemm_set_debug(0)
    n = 8 * PP_STK * 4 * 8
    buf = (C.c_uint64 * n)()
    fn = lib.jmt_gemm_pp_stamps_read
    fn.restype = C.c_int
    fn.argtypes = [C.c_void_p, C.c_int]
    assert fn(buf, n) == n
    st = [[[[buf[((w * PP_STK + t) * 4 + p) * 8 + e] for e in range(8)] for p in range(4)]
           for t in range(PP_STK)] for w in range(8)]
    names = ["reads", "dma", "deadline", "barrier1", "mfma", "barrier2"]
    for w in (0, 4):
        seg = {k: [] for k in names}
        for t in range(2, PP_STK):
            for p in range(4):
                s = st[w][t][p]
                nxt = st[w][t][p + 1][0] if p < 3 else (st[w][t + 1][0][0] if t + 1 < PP_STK else None)
                d = [s[1] - s[0], s[2] - s[1], s[3] - s[2], s[4] - s[3], s[5] - s[4]]
                d.append(nxt - s[5] if nxt else None)
                for k, v in zip(names, d):
                    if v is not None and 0 <= v < 10 ** 7:
                        seg[k].append(v)
        kt = [st[w][t + 1][0][0] - st[w][t][0][0] for t in range(2, PP_STK - 1)]
        for t in range(4, 11):
            row = []
            for p in range(4):
                s = st[w][t][p]
                nxt = st[w][t][p + 1][0] if p < 3 else st[w][t + 1][0][0]
                row.append([s[6] - s[0], s[7] - s[6], s[1] - s[7], s[2] - s[1], s[3] - s[2],
                            s[4] - s[3], s[5] - s[4], nxt - s[5]])
            print(json.dumps({"wave": w, "ktile": t, "segs": row}))
        print(json.dumps({"shape": args.shape, "wave": w,
                          "median_cycles": {k: statistics.median(v) for k, v in seg.items() if v},
                          "ktile_cycles_median": statistics.median(kt),
                          "ktile_cycles": kt[:12]}))


if __name__ == "__main__":
    main()
