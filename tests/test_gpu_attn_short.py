"""jmt_attn_short_{fwd,bwd} (csrc/attn_short.hip): the one-block-per-sequence fused attention for
Lq, Lk <= 32 whose backward computes dQ, dK and dV in one kernel (the
batch-axis attention of mm_transformers.py:119-146 at B = 32, the T = 16 real-data windows of
config_file.json).  Checked against
  * a torch fp32 reference from the same rounded inputs (dq, dk, dv, o, lse);
  * the long-sequence path on the same inputs: the forward bit for bit (same tile arithmetic),
    dQ bit for bit in bf16, dK / dV against the path's P / dS hand-off within output rounding;
  * the model-level dispatch (AttnCoreFn routes 8 < L <= 32 here, 2 launches instead of 4)."""
import math

import pytest
import torch

from jmt import functional as JF
from jmt import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"
E = 512

SHAPES = [(32, 32, 300), (16, 16, 192), (9, 17, 5), (32, 1, 7), (1, 32, 3), (13, 29, 40),
          (32, 32, 1), (24, 32, 600)]


def _inputs(cd, Lq, Lk, N, H=1, seed=41):
    """Packed self-attention style layouts: q from a (Lq, N, 3E') buffer, k / v from a
    (Lk, N, 2E') one (E' = H * 512), dO contiguous."""
    Eh = E * H
    g = torch.Generator(device=DEV).manual_seed(seed)
    qkv = torch.randn(N, Lq, 3 * Eh, device=DEV, generator=g).to(cd).permute(1, 0, 2)
    kv = torch.randn(N, Lk, 2 * Eh, device=DEV, generator=g).to(cd).permute(1, 0, 2)
    go = torch.randn(Lq, N, Eh, device=DEV, generator=g).to(cd)
    return qkv, kv, go


def _st(t):
    return (t.stride(0), t.stride(1))


def _fwd(fn, cd, qkv, kv, Lq, Lk, N, H):
    Eh = E * H
    qp, kp, vp = qkv[..., :Eh], kv[..., :Eh], kv[..., Eh:]
    o = torch.full((Lq, N, Eh), float("nan"), device=DEV, dtype=cd)
    lse = torch.full((N * H * Lq,), float("nan"), device=DEV)
    fn(ops.dt(qkv), N, H, Lq, Lk, E, qp.data_ptr(), _st(qkv), kp.data_ptr(), _st(kv),
       vp.data_ptr(), _st(kv), o.data_ptr(), _st(o), 1.0 / math.sqrt(E), lse)
    return o, lse


def _ref(qkv, kv, go, o, H):
    """fp32 reference per head: P, dP, Delta (from the 16-bit O as the kernels), dS, dQ, dK, dV."""
    Eh = E * H
    outs = []
    for h in range(H):
        sl = slice(h * E, (h + 1) * E)
        q = qkv[..., :Eh][..., sl].float()
        k = kv[..., :Eh][..., sl].float()
        v = kv[..., Eh:][..., sl].float()
        d = go[..., sl].float()
        scale = 1.0 / math.sqrt(E)
        s = torch.einsum("lnd,knd->nlk", q, k) * scale
        p = torch.softmax(s, -1)
        dp = torch.einsum("lnd,knd->nlk", d, v)
        delta = (d * o[..., sl].float()).sum(-1).t().unsqueeze(-1)
        ds = p * (dp - delta) * scale
        outs.append(dict(o=torch.einsum("nlk,knd->lnd", p, v), lse=torch.logsumexp(s, -1),
                         dq=torch.einsum("nlk,knd->lnd", ds, k),
                         dk=torch.einsum("nlk,lnd->knd", ds, q),
                         dv=torch.einsum("nlk,lnd->knd", p, d), dpmax=dp.abs().max().item()))
    return outs


@pytest.mark.parametrize("cd", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("Lq,Lk,N", SHAPES)
def test_short_fwd_equals_long_kernel_and_fp32(cd, Lq, Lk, N):
    qkv, kv, _ = _inputs(cd, Lq, Lk, N)
    o, lse = _fwd(ops.attn_short_fwd, cd, qkv, kv, Lq, Lk, N, 1)
    o2, lse2 = _fwd(ops.attn_fwd, cd, qkv, kv, Lq, Lk, N, 1)
    torch.cuda.synchronize()
    assert torch.equal(o, o2), (o.float() - o2.float()).abs().max().item()
    assert torch.equal(lse, lse2)
    r = _ref(qkv, kv, qkv[..., :E], o, 1)[0]
    tol = (1e-2 if cd == torch.bfloat16 else 2e-3) * max(r["o"].abs().max().item(), 1.0)
    assert (o.float() - r["o"]).abs().max().item() <= tol
    assert (lse - r["lse"].reshape(-1)).abs().max().item() <= 1e-3 * max(
        r["lse"].abs().max().item(), 1.0)


def _bwd_short(cd, qkv, kv, go, o, lse, Lq, Lk, N, H):
    """dq written into the q slot of a NaN-poisoned packed (Lq, N, 3E') buffer, dk / dv into the
    k / v slots of a packed (Lk, N, 2E') one (as the grouped model's packed gradients)."""
    Eh = E * H
    dqkv = torch.full((N, Lq, 3 * Eh), float("nan"), device=DEV, dtype=cd).permute(1, 0, 2)
    dkv = torch.full((N, Lk, 2 * Eh), float("nan"), device=DEV, dtype=cd).permute(1, 0, 2)
    ops.attn_short_bwd(ops.dt(qkv), N, H, Lq, Lk, E, go.data_ptr(), _st(go), o.data_ptr(), _st(o),
                       qkv[..., :Eh].data_ptr(), _st(qkv), kv[..., :Eh].data_ptr(), _st(kv),
                       kv[..., Eh:].data_ptr(), _st(kv), lse, dqkv[..., Eh:2 * Eh].data_ptr(),
                       _st(dqkv), dkv[..., :Eh].data_ptr(), _st(dkv), dkv[..., Eh:].data_ptr(),
                       _st(dkv), 1.0 / math.sqrt(E))
    torch.cuda.synchronize()
    assert torch.isnan(dqkv[..., :Eh].float()).all() and torch.isnan(dqkv[..., 2 * Eh:].float()).all()
    return dqkv[..., Eh:2 * Eh], dkv[..., :Eh], dkv[..., Eh:]


@pytest.mark.parametrize("cd", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("Lq,Lk,N", SHAPES)
def test_short_bwd_vs_fp32_and_long_path(cd, Lq, Lk, N):
    qkv, kv, go = _inputs(cd, Lq, Lk, N)
    o, lse = _fwd(ops.attn_short_fwd, cd, qkv, kv, Lq, Lk, N, 1)
    dq, dk, dv = _bwd_short(cd, qkv, kv, go, o, lse, Lq, Lk, N, 1)
    for t in (dq, dk, dv):
        assert torch.isfinite(t.float()).all()
    r = _ref(qkv, kv, go, o, 1)[0]
    u = 2.0 ** -8 if cd == torch.bfloat16 else 2.0 ** -11
    floor = 4 * u * (1.0 / math.sqrt(E)) * r["dpmax"]
    qmax = qkv[..., :E].float().abs().max().item()
    kmax = kv[..., :E].float().abs().max().item()
    # dS / P rounded to the compute dtype before the products (as the long path's hand-off)
    assert (dq.float() - r["dq"]).abs().max().item() <= 16 * u * r["dq"].abs().max().item() + floor * kmax
    assert (dk.float() - r["dk"]).abs().max().item() <= 16 * u * r["dk"].abs().max().item() + floor * qmax
    assert (dv.float() - r["dv"]).abs().max().item() <= 8 * u * r["dv"].abs().max().item()
    # the long path on the same inputs: dQ bit for bit; dK / dV from its P / dS hand-off
    ldp = -(-Lk // 8) * 8
    P = torch.empty(N * Lq * ldp, device=DEV, dtype=cd)
    dS = torch.empty_like(P)
    dq2 = torch.empty(Lq, N, E, device=DEV, dtype=cd)
    ops.attn_bwd(ops.dt(qkv), N, 1, Lq, Lk, E, go.data_ptr(), _st(go), o.data_ptr(), _st(o),
                 qkv[..., :E].data_ptr(), _st(qkv), kv[..., :E].data_ptr(), _st(kv),
                 kv[..., E:].data_ptr(), _st(kv), lse, P, dS, ldp, dq2.data_ptr(), _st(dq2),
                 1.0 / math.sqrt(E))
    torch.cuda.synchronize()
    if cd == torch.bfloat16:
        assert torch.equal(dq.contiguous(), dq2), (dq.float() - dq2.float()).abs().max().item()
    else:
        # fp16: hipcc may contract Delta's products into v_dot2 (a different rounding) in one
        # kernel and not the other, so dQ agrees to output rounding only
        assert (dq.float() - dq2.float()).abs().max().item() <= 2 * u * dq2.float().abs().max().item()
    Pf = P.view(N, Lq, ldp)[..., :Lk].float()
    dSf = dS.view(N, Lq, ldp)[..., :Lk].float()
    dk2 = torch.einsum("nlk,lnd->knd", dSf, qkv[..., :E].float())
    dv2 = torch.einsum("nlk,lnd->knd", Pf, go.float())
    # absolute floor: fp16's subnormal spacing (dK at Lk = 1 is a cancellation residue ~1e-6)
    tiny = 2.0 ** -24 if cd == torch.float16 else 1e-30
    assert (dk.float() - dk2).abs().max().item() <= 2 * u * dk2.abs().max().item() + tiny
    assert (dv.float() - dv2).abs().max().item() <= 2 * u * dv2.abs().max().item() + tiny


def test_short_two_heads():
    """H = 2 heads of 512 (E' = 1024): head h at column h * 512 of every row."""
    cd, Lq, Lk, N, H = torch.bfloat16, 20, 27, 11, 2
    qkv, kv, go = _inputs(cd, Lq, Lk, N, H=H, seed=43)
    o, lse = _fwd(ops.attn_short_fwd, cd, qkv, kv, Lq, Lk, N, H)
    dq, dk, dv = _bwd_short(cd, qkv, kv, go, o, lse, Lq, Lk, N, H)
    u = 2.0 ** -8
    for h, r in enumerate(_ref(qkv, kv, go, o, H)):
        sl = slice(h * E, (h + 1) * E)
        assert (o[..., sl].float() - r["o"]).abs().max().item() <= 1e-2 * max(r["o"].abs().max().item(), 1.0)
        floor = 4 * u * r["dpmax"] / math.sqrt(E) * 5.0
        for name, t in (("dq", dq), ("dk", dk), ("dv", dv)):
            ref = r[name]
            assert (t[..., sl].float() - ref).abs().max().item() <= 16 * u * ref.abs().max().item() + floor, name


def test_short_rejects_unsupported():
    from jmt._lib import JMTError
    cd = torch.bfloat16
    x = torch.zeros(40, 4, 3 * E, dtype=cd, device=DEV)
    lse = torch.empty(4 * 40, device=DEV)
    st = (x.stride(0), x.stride(1))
    a = (x.data_ptr(), st)
    with pytest.raises(JMTError):                 # Lk = 33 > 32
        ops.attn_short_fwd(ops.dt(x), 4, 1, 8, 33, E, *a, *a, *a, *a, 1.0, lse)
    with pytest.raises(JMTError):                 # head dim 256
        ops.attn_short_fwd(ops.dt(x), 4, 1, 8, 8, 256, *a, *a, *a, *a, 1.0, lse)
    with pytest.raises(JMTError):                 # misaligned row start
        ops.attn_short_fwd(ops.dt(x), 4, 1, 8, 8, E, x.data_ptr() + 2, st, *a, *a, *a, 1.0, lse)


@pytest.mark.parametrize("cd", [torch.bfloat16, torch.float16])
def test_short_dispatch_matches_long_path(cd):
    """AttnCoreFn routes 8 < L <= 32 to the short kernels (one forward, one backward launch;
    the long path needs the attention backward plus two dK / dV GEMMs) and matches the long
    path (JMT_ATTN_SHORT=0) on a packed self-attention (B = 32 batch-axis shape)."""
    fams = []
    ops.set_launch_hook(lambda info, launch: (fams.append(info.get("family")), launch())[1])
    g = torch.Generator(device=DEV).manual_seed(7)
    N, L = 300, 32
    x = torch.randn(N, L, 3 * E, device=DEV, generator=g).to(cd).permute(1, 0, 2)
    w = torch.randn(L, N, E, device=DEV, generator=g)
    outs = []
    try:
        for short in (True, False):
            ops._attn_short["on"] = short
            fams.clear()
            xx = x.detach().clone().requires_grad_(True)
            with JF.compute_mode(cd):
                o = JF.AttnCoreFn.apply(xx, xx, xx, E, 1, 0, E, 2 * E)
            (o.float() * w).sum().backward()
            torch.cuda.synchronize()
            outs.append((o.float(), xx.grad.float()))
            if short:
                assert fams.count("attn_short_fwd") == 1 and fams.count("attn_short_bwd") == 1
                assert "attn_bwd" not in fams and not any(f and f.startswith("gemm") for f in fams)
            else:
                assert "attn_short_fwd" not in fams and "attn_bwd" in fams
    finally:
        ops._attn_short["on"] = True
        ops.set_launch_hook(None)
    (o1, g1), (o2, g2) = outs
    assert torch.equal(o1, o2)
    u = 2.0 ** -8 if cd == torch.bfloat16 else 2.0 ** -11
    assert (g1 - g2).abs().max().item() <= 4 * u * g2.abs().max().item()
