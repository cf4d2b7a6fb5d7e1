"""Cross-check of HIP-event kernel timing against rocprofv3 (run under rocprofv3 --kernel-trace):
one NT GEMM shape of the step (3 x 19200x512x512, pointer-table weights) launched 40 times,
timed (a) by an event pair around each launch, (b) by one pair around all 40 and (c) by the host
clock; prints the three averages (us per launch) for comparison with the trace durations."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "joint-multimodal-transformer-6th-abaw_amd")]
import torch  # noqa: E402
from jmt import ops  # noqa: E402
from jmt._lib import BF16  # noqa: E402

M, N, K, batch, reps = 19200, 512, 512, 3, 40
A = torch.randn(batch, M * K, device="cuda").bfloat16()
W = torch.randn(batch, N * K, device="cuda").bfloat16()
C = torch.zeros(batch, M * N, device="cuda", dtype=torch.bfloat16)
kw = dict(M=M, N=N, K=K, ab_dtype=BF16, c_dtype=BF16, lda=K, a_kmajor=True, ldb=K, b_kmajor=True,
          c=[C.data_ptr()], ldc=N, batch0=batch, sC=(M * N, 0), a=[A.data_ptr()], sA=(M * K, 0),
          b=[W[i].data_ptr() for i in range(batch)], b_mode=1, device="cuda")
for _ in range(5):
    ops.gemm(**kw)
torch.cuda.synchronize()
pairs = []
for _ in range(reps):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    ops.gemm(**kw)
    e.record()
    pairs.append((s, e))
torch.cuda.synchronize()
per = sum(s.elapsed_time(e) for s, e in pairs) / reps * 1e3
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
t0 = time.perf_counter()
s.record()
for _ in range(reps):
    ops.gemm(**kw)
e.record()
torch.cuda.synchronize()
wall = (time.perf_counter() - t0) / reps * 1e6
print(json.dumps({"per_launch_events_us": round(per, 2),
                  "bracket_events_us": round(s.elapsed_time(e) / reps * 1e3, 2),
                  "host_wall_us": round(wall, 2)}))
