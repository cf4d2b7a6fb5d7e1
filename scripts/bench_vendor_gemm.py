"""Reference point only (not used by the product path): the vendor BLAS (torch.matmul ->
hipBLASLt / rocBLAS) on the step's GEMM shapes, bf16, to size the headroom of gemm.hip."""
import json
import torch

R = 19200
SHAPES = [("fwd 19200x512x512", 1, R, 512, 512), ("fwd b3 19200x512x512", 3, R, 512, 512),
          ("qkv b3 19200x1536x512", 3, R, 1536, 512), ("kv b6 19200x1024x512", 6, R, 1024, 512),
          ("head 19200x1024x3072", 1, R, 1024, 3072), ("wgrad b3 512x512x19200", 3, 512, 512, R)]
for name, b, M, N, K in SHAPES:
    a = torch.randn(b, M, K, device="cuda").bfloat16()
    w = torch.randn(b, N, K, device="cuda").bfloat16()
    f = lambda: torch.bmm(a, w.transpose(1, 2))
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20):
        f()
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) / 20 * 1e3
    print(json.dumps({"shape": name, "us": round(us, 1), "tflops": round(2 * b * M * N * K / us / 1e6, 1)}))
