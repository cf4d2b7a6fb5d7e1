"""hipBLASLt (torch.matmul) on the JMT step's GEMM shapes: what the vendor library reaches."""
import torch
dev = "cuda"
R = 19200
def bench(name, fn, flops, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) / reps * 1e3
    print(f"{name:40s} {us:8.2f} us  {flops / us / 1e6:7.1f} TF/s", flush=True)
bf = torch.bfloat16
for (M, N, K, b) in [(R, 512, 512, 3), (R, 1536, 512, 3), (R, 1024, 512, 6), (R, 512, 1024, 6), (R, 1024, 3072, 1), (R, 512, 3072, 1)]:
    A = torch.randn(b, M, K, device=dev, dtype=bf)
    W = torch.randn(b, N, K, device=dev, dtype=bf)
    bench(f"NT b{b} {M}x{N}x{K}", lambda: torch.bmm(A, W.transpose(1, 2)), 2.0 * M * N * K * b)
    Wn = torch.randn(b, K, N, device=dev, dtype=bf)
    bench(f"NN b{b} {M}x{N}x{K}", lambda: torch.bmm(A, Wn), 2.0 * M * N * K * b)
for (M, N, K, b) in [(512, 512, R, 3), (1536, 512, R, 3), (512, 1024, R, 6)]:
    G = torch.randn(b, K, M, device=dev, dtype=bf)
    X = torch.randn(b, K, N, device=dev, dtype=bf)
    bench(f"TN b{b} {M}x{N}x{K}", lambda: torch.bmm(G.transpose(1, 2), X), 2.0 * M * N * K * b)
