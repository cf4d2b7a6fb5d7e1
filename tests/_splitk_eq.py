"""Split-K reduced inside the GEMM launch (JMT_SPLITK_FUSED=1, gemm.hip splitk_fixup) vs the
separate reduce launch (default): split-K GEMMs of the step's kinds (TN weight gradients with
A row sums and beta = 1, 16-bit C with bias / ReLU / aux mask, fp32 operands, repeated launches
on one workspace), outputs saved by one process and compared bit for bit by another.
    python tests/_splitk_eq.py save|cmp FILE     (used by test_gpu_kernels.py)"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "joint-multimodal-transformer-6th-abaw_amd")]
import torch  # noqa: E402
from jmt import ops  # noqa: E402
from jmt._lib import BF16, F32  # noqa: E402

dev = "cuda"


def run():
    outs = {}
    g = torch.Generator(device=dev).manual_seed(3)
    r = lambda *s: (torch.rand(*s, device=dev, generator=g) * 2 - 1)
    # TN wgrad with row sums (fp32 C, accumulate), b3 512x512x19200 and ragged
    for (b, M, N, K, sp) in [(3, 512, 512, 19200, 8), (2, 200, 136, 3000, 5), (1, 384, 256, 1024, 4)]:
        a = r(b, K, M).bfloat16(); w = r(b, K, N).bfloat16()
        c = r(b, M, N)
        db = [r(M) for _ in range(b)]
        ops.gemm(M=M, N=N, K=K, ab_dtype=BF16, c_dtype=F32, a=[a.data_ptr()], lda=M, a_kmajor=False,
                 b=[w.data_ptr()], ldb=N, b_kmajor=False, c=[c.data_ptr()], ldc=N, batch0=b,
                 sA=(K * M, 0), sB=(K * N, 0), sC=(M * N, 0), beta=1.0, splits=sp,
                 dbias_tab=db, device=dev)
        outs[f"tn{b}_{M}_{N}_{K}"] = c.clone()
        for i, t in enumerate(db):
            outs[f"tn{b}_{M}_{N}_{K}_db{i}"] = t.clone()
    # NT 16-bit out with bias + relu + aux, split 3
    for (M, N, K, sp) in [(1000, 512, 2048, 3), (256, 260, 1536, 6)]:
        a = r(M, K).bfloat16(); w = r(N, K).bfloat16(); bias = r(N)
        aux = r(M, N).bfloat16()
        c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        ops.gemm(M=M, N=N, K=K, ab_dtype=BF16, c_dtype=BF16, a=[a.data_ptr()], lda=K, a_kmajor=True,
                 b=[w.data_ptr()], ldb=K, b_kmajor=True, c=[c.data_ptr()], ldc=N, bias=bias,
                 relu=True, aux=aux, ldaux=N, splits=sp, device=dev)
        outs[f"nt_{M}_{N}_{K}"] = c.clone()
    # fp32 operands split
    a = r(300, 900); w = r(900, 200)
    c = torch.empty(300, 200, device=dev)
    ops.gemm(M=300, N=200, K=900, ab_dtype=F32, c_dtype=F32, a=[a.data_ptr()], lda=900,
             a_kmajor=True, b=[w.data_ptr()], ldb=200, b_kmajor=False, c=[c.data_ptr()], ldc=200,
             alpha=0.5, splits=4, device=dev)
    outs["f32"] = c.clone()
    # repeated launches on one workspace (counters re-zeroed each launch)
    a = r(2, 4096, 256).bfloat16(); w = r(2, 4096, 384).bfloat16()
    c = torch.zeros(2, 256, 384, device=dev)
    for _ in range(5):
        ops.gemm(M=256, N=384, K=4096, ab_dtype=BF16, c_dtype=F32, a=[a.data_ptr()], lda=256,
                 a_kmajor=False, b=[w.data_ptr()], ldb=384, b_kmajor=False, c=[c.data_ptr()],
                 ldc=384, batch0=2, sA=(4096 * 256, 0), sB=(4096 * 384, 0), sC=(256 * 384, 0),
                 beta=1.0, splits=8, device=dev)
    outs["rep"] = c.clone()
    torch.cuda.synchronize()
    ref = torch.bmm(a.float().transpose(1, 2), w.float()) * 5
    print("rep max err vs fp32 bmm", (c - ref).abs().max().item())
    return outs


if __name__ != "__main__":
    raise ImportError("script, run as a child process")
mode, path = sys.argv[1], sys.argv[2]
o = run()
if mode == "save":
    torch.save({k: v.cpu() for k, v in o.items()}, path)
    print("saved", len(o))
else:
    ref = torch.load(path, weights_only=True)
    bad = [k for k in ref if not torch.equal(ref[k], o[k].cpu())]
    print("compared", len(ref), "mismatch", bad)
    sys.exit(1 if bad else 0)
