"""Which multi-stream capture pattern crashes hipGraph capture on this stack?  One case per run:
    python scripts/dev/capture_probe.py <case>"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "joint-multimodal-transformer-6th-abaw_amd")]
import torch

case = sys.argv[1]
dev = torch.device("cuda")
x = torch.randn(256, 256, device=dev)
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def fork_join(fn):
    main = torch.cuda.current_stream()
    outs = []
    for s in (s1, s2):
        s.wait_stream(main)
        with torch.cuda.stream(s):
            outs.append(fn())
    for s in (s1, s2):
        main.wait_stream(s)
    return outs


def body():
    if case == "torch_fork":
        a, b = fork_join(lambda: x @ x)
        return a + b
    if case == "torch_fork_record":
        a, b = fork_join(lambda: x @ x)
        a.record_stream(torch.cuda.current_stream())
        b.record_stream(torch.cuda.current_stream())
        return a + b
    if case == "torch_autograd":
        w = W
        a, b = fork_join(lambda: (x @ w).relu())
        l = (a + b).sum()
        l.backward()
        return l
    if case == "jmt_linear":
        from jmt import functional as F
        a, b = fork_join(lambda: F.linear(xb, Wj, bj))
        return a.float().sum() + b.float().sum()
    if case == "jmt_linear_bwd":
        from jmt import functional as F
        a, b = fork_join(lambda: F.linear(xb, Wj, bj))
        l = a.float().sum() + b.float().sum()
        l.backward()
        return l
    raise SystemExit("unknown case")


W = torch.randn(256, 256, device=dev, requires_grad=True)
xb = torch.randn(64, 300, 512, device=dev, requires_grad=True)
Wj = torch.nn.Parameter(torch.randn(512, 512, device=dev) * 0.02)
bj = torch.nn.Parameter(torch.zeros(512, device=dev))
side = torch.cuda.Stream()
side.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(side):
    for _ in range(2):
        body()
torch.cuda.current_stream().wait_stream(side)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    out = body()
torch.cuda.synchronize()
g.replay()
torch.cuda.synchronize()
print(case, "OK", float(out.float().sum()), flush=True)
