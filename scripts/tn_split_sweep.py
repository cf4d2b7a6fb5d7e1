"""Split-count sweep of the weight-gradient GEMMs under 24 tiles (the 128 x 128 split-K plan):
    python scripts/tn_split_sweep.py
Prints per (shape, splits): us per launch (the GEMM + its reduce launch), beta = 1 into fp32."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "joint-multimodal-transformer-6th-abaw_amd")]

import torch  # noqa: E402

from jmt import ops  # noqa: E402
from jmt._lib import BF16, F32  # noqa: E402

SHAPES = [(512, 512, 19200, 3), (512, 512, 19200, 2), (512, 2048, 19200, 1),
          (512, 1024, 19200, 1), (128, 1024, 19200, 2)]
for M, N, K, nb in SHAPES:
    dy = torch.randn(nb, K, M, device="cuda").bfloat16()
    x = torch.randn(nb, K, N, device="cuda").bfloat16()
    c = torch.zeros(nb, M, N, device="cuda")
    auto = ops.auto_splits(M, N, K, nb, BF16)
    for s in sorted({auto, 2, 4, 6, 8, 10, 12, 16, 20, 24, 32}):
        kw = dict(M=M, N=N, K=K, ab_dtype=BF16, c_dtype=F32, a=[dy.data_ptr()], lda=M,
                  a_kmajor=False, sA=(K * M, 0), b=[x.data_ptr()], ldb=N, b_kmajor=False,
                  sB=(K * N, 0), c=[c.data_ptr()], ldc=N, sC=(M * N, 0), batch0=nb, beta=1.0,
                  splits=s, device="cuda")
        for _ in range(3):
            ops.gemm(**kw)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(30):
            ops.gemm(**kw)
        e1.record()
        torch.cuda.synchronize()
        print(json.dumps({"shape": [M, N, K, nb], "splits": s, "auto": s == auto,
                          "us": round(e0.elapsed_time(e1) / 30 * 1e3, 2)}), flush=True)
