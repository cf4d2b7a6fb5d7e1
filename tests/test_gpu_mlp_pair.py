"""MLPPairFn (the V / A regressors of two_transformers.py:104-114,125-126 as one function) against
the two separate MLPFn calls it replaces, on a seq-first (T, B, E) input as the model feeds it:
fp32 bit-exact forward and input gradient (same per-element arithmetic, the two input gradients
summed by the same add autograd uses), weight / bias gradients within fp32 summation-order noise
(the grouped weight-gradient launch may pick another split-K); 16-bit: both paths against the fp32
result, the pair (csrc/head.hip output layers, one K-concatenated input-gradient GEMM) at least as
accurate as the separate path."""
import pytest
import torch

from jmt import functional as JF
from jmt.nn import MLP

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _run(pair, cd, x0, va, aa, k):
    JF.set_pair_mlps(pair)
    x = x0.clone().requires_grad_(True)
    for m in (va, aa):
        for p in m.parameters():
            p.grad = None
    with JF.compute_mode(cd):
        if pair:
            v, a = JF.mlp_pair(x, va, aa, out_dtype=torch.float32)
        else:
            v = va(x, out_dtype=torch.float32)
            a = aa(x, out_dtype=torch.float32)
        gv = torch.linspace(-1, 1, v.numel(), device=DEV).view_as(v)
        ga = torch.cos(torch.arange(a.numel(), device=DEV, dtype=torch.float32)).view_as(a)
        ((v * gv).sum() + (a * ga).sum()).backward()
    torch.cuda.synchronize()
    grads = [p.grad.clone() for m in (va, aa) for p in m.parameters()]
    return v.detach(), a.detach(), x.grad.detach().float(), grads


@pytest.mark.parametrize("cd", [torch.float32, torch.bfloat16, torch.float16],
                         ids=["fp32", "bf16", "fp16"])
@pytest.mark.parametrize("k", [1, 20], ids=["regressor", "digitized20"])
def test_mlp_pair_matches_two_mlps(cd, k):
    torch.manual_seed(7)
    T, B, E = 37, 6, 1024
    va = MLP(E, 128, k, dropout=0.0).to(DEV)
    aa = MLP(E, 128, k, dropout=0.0).to(DEV)
    x0 = torch.randn(B, T, E, device=DEV).permute(1, 0, 2)       # seq-first view, as in the model
    try:
        ref = _run(False, cd, x0, va, aa, k)
        got = _run(True, cd, x0, va, aa, k)
    finally:
        JF.set_pair_mlps(True)
    if cd == torch.float32:
        for r, g in zip(ref[:3], got[:3]):
            assert r.shape == g.shape and torch.equal(r, g)
        for r, g in zip(ref[3], got[3]):
            scale = max(1.0, float(r.abs().max()))
            assert float((r - g).abs().max()) <= 1e-5 * scale, float((r - g).abs().max())
        return
    # 16-bit: the pair's output layers run as csrc/head.hip row kernels from the fp32 loss
    # gradient and its input gradient is one K-concatenated GEMM (fewer roundings than the two
    # MLPFn calls): both paths against the fp32 result, the pair at least as accurate (x1.5)
    try:
        ref32 = _run(False, torch.float32, x0, va, aa, k)
    finally:
        JF.set_pair_mlps(True)
    u = 2 ** -8 if cd == torch.bfloat16 else 2 ** -11
    for r32, r, g in zip(list(ref32[:3]) + ref32[3], list(ref[:3]) + ref[3],
                         list(got[:3]) + got[3]):
        assert r.shape == g.shape
        # (the V head's output-bias gradient is sum(linspace(-1, 1)) = 0: absolute floor)
        den = max(float(r32.norm()), 1e-2)
        e_sep = float((r.float() - r32).norm()) / den
        e_pair = float((g.float() - r32).norm()) / den
        assert e_pair <= 1.5 * max(e_sep, u), (e_pair, e_sep)


def test_two_transformers_uses_the_pair():
    """The model routes its regressors through MLPPairFn (and back through MLPFn with it off)."""
    from models.two_transformers import Two_transformers
    m = Two_transformers(0.0, 0.0, 1, 1, "TRANSFORMER", "FC", 2048).to(DEV)
    a = torch.randn(2, 8, 512, device=DEV)
    v = torch.randn(2, 8, 2048, device=DEV)
    seen = []
    orig = JF.MLPPairFn.apply

    def spy(*args):
        seen.append(1)
        return orig(*args)

    JF.MLPPairFn.apply = spy
    try:
        vo, ao = m(a, v)
        JF.set_pair_mlps(False)
        vo2, ao2 = m(a, v)
    finally:
        JF.MLPPairFn.apply = orig
        JF.set_pair_mlps(True)
    assert seen == [1]
    assert torch.equal(vo, vo2) and torch.equal(ao, ao2)
