"""Grouped execution of the JMT block's parallel branches (MultimodalTransformer_w_JR,
mm_multi_transformers.py:118-214): the three encoders and the six cross-attentions run as
batched launches instead of 3 / 6 separate ones.

The reference applies three same-shaped TransformerEncoderLayers to v, a and the joint
representation (:132-136), then three nn.MultiheadAttention modules twice each (:142-167), then
`out_layer1` to the concatenation of the six outputs (:201-211).  Here the three encoder inputs
live in ONE stacked buffer X (3, B, T, E); every GEMM of the three encoders is one launch whose
per-batch operands come from pointer tables (weights, biases, gradient buffers: each module keeps
its own nn.Parameters, so state_dict keys are untouched), the attention core runs over 3B
sequences in one launch, and the six cross-attentions likewise over 6 stacked (query, key) pairs.
The backward of each group is written out explicitly: gradients that the reference's autograd
would sum from several uses (a stream's encoder output feeds 4 projections) are produced by ONE
K-concatenated dgrad GEMM per stream (K = 6E), and weight gradients are accumulated in place
(beta = 1) by batched wgrad GEMMs — no autograd adds, no cross-stream synchronisation, and a
single HIP stream that captures into a hipGraph (jmt/graph.py).

Stacked layouts (compute dtype, row-major, rows in (b, t) order per group):
  X, Y   (G, B, T, E)     encoder group input / output            G = 3
  QKV    (G', B, T, 3E)   packed in-projection outputs            G' = 3 (encoders), 6 (pairs)
  O      (G', B, T, E)    attention outputs (before out_proj)
"""
from __future__ import annotations

import os
from typing import List, Sequence

import torch
from torch.autograd import Function

from . import ops, streams
from .functional import (_dc, _grad_buffer, _grad_done, _ptr, attn_backward, attn_forward,
                         compute_dtype, weight_as)

_enabled = {"on": os.environ.get("JMT_GROUPED", "1") != "0"}
# the cross-attention backward's three stream-gradient GEMMs on branch streams: measured
# 1.6 % slower per step (profiles/r02_par_stream_dgrad.txt), off unless JMT_PAR_STREAM_DGRAD=1
_PAR_STREAM_DGRAD = os.environ.get("JMT_PAR_STREAM_DGRAD", "0") == "1"

# the six cross-attentions in the reference's order (mm_multi_transformers.py:142-167), which is
# also the order of torch.cat in the FC head (:201-211): (module, query stream, key/value stream)
# with module 0 = cross_attention_v, 1 = cross_attention_p, 2 = cross_attention_pv and stream
# 0 = visual, 1 = physiological (audio), 2 = joint representation.
CROSS_PAIRS = ((0, 0, 1), (1, 1, 0), (2, 2, 0), (0, 0, 2), (2, 2, 1), (1, 1, 2))


def enabled() -> bool:
    return _enabled["on"]


def set_enabled(on: bool) -> None:
    _enabled["on"] = bool(on)


# ------------------------------------------------------------------------- grouped GEMMs
def _gemm_fwd(a_ptrs: Sequence[int], lda: int, sA: int, rows: int, K: int, Ws, r0: int, n: int,
              bs, c_ptr: int, ldc: int, sC: int, c_dt: int, cd, dev, relu: bool = False):
    """C[g] = A[g] (rows x K) . W_g[r0:r0+n]^T + b_g[r0:r0+n]  for g < len(Ws), one launch.
    A is strided (a_ptrs = [base], sA) or a per-group pointer table (len(a_ptrs) == len(Ws))."""
    Wc = [weight_as(W, cd) for W in Ws]
    Kin = Wc[0].shape[1]
    table = len(a_ptrs) > 1
    ops.gemm(M=rows, N=n, K=K, ab_dtype=_dc(cd), c_dtype=c_dt,
             a=list(a_ptrs), lda=lda, a_kmajor=True, a_mode=1 if table else 0,
             sA=(0 if table else sA, 0),
             b=[_ptr(w, r0 * Kin) for w in Wc], ldb=Kin, b_kmajor=True, b_mode=1,
             c=[c_ptr], ldc=ldc, sC=(sC, 0), batch0=len(Ws),
             bias_tab=[b[r0:r0 + n] for b in bs] if bs is not None else None, bias_mode=1,
             relu=relu, device=dev)


def _gemm_dgrad(dy_ptr: int, ldy: int, sdy: int, rows: int, n: int, Ws, r0: int, c_ptr: int,
                ldc: int, sC: int, c_dt: int, cd, dev, beta: float = 0.0, aux=None,
                ldaux: int = 0):
    """dX[g] (+)= dY[g] (rows x n) . W_g[r0:r0+n, :]  (masked by aux > 0: ReLU backward)."""
    Wc = [weight_as(W, cd) for W in Ws]
    Kin = Wc[0].shape[1]
    ops.gemm(M=rows, N=Kin, K=n, ab_dtype=_dc(cd), c_dtype=c_dt,
             a=[dy_ptr], lda=ldy, a_kmajor=True, sA=(sdy, 0),
             b=[_ptr(w, r0 * Kin) for w in Wc], ldb=Kin, b_kmajor=False, b_mode=1,
             c=[c_ptr], ldc=ldc, sC=(sC, 0), batch0=len(Ws), beta=beta,
             aux=aux, ldaux=ldaux, device=dev)


def _gemm_wgrad(dy_ptrs: Sequence[int], ldy: int, sdy: int, x_ptrs: Sequence[int], ldx: int,
                sx: int, rows: int, n: int, Ws, r0: int, cd, dev, bs=None) -> bool:
    """W_g.grad[r0:r0+n] += dY[g]^T X[g]  (fp32, split-K over the rows).  dY / X are strided
    ([base], stride) or per-group pointer tables.  The Ws of one launch must be distinct
    parameters (their gradient regions are written concurrently).  With `bs` (distinct bias
    parameters), also b_g.grad[r0:r0+n] += the column sums of dY[g], taken inside the same GEMM
    (functional.fused_bgrad_ok); returns True when the bias gradients were written."""
    from .functional import fused_bgrad_ok
    grads = []
    for W in Ws:
        g = _grad_buffer(W)
        grads.append(g if g is not None else torch.zeros_like(W))
    dbt = None
    if bs is not None and n > 1 and fused_bgrad_ok(cd):
        dbt = []
        for b in bs:
            gb = _grad_buffer(b)
            dbt.append(gb[r0:r0 + n] if gb is not None else
                       torch.empty(n, dtype=torch.float32, device=dev))
    Kin = Ws[0].shape[1]
    ta, tb = len(dy_ptrs) > 1, len(x_ptrs) > 1
    ops.gemm(M=n, N=Kin, K=rows, ab_dtype=_dc(cd), c_dtype=ops.F32,
             a=list(dy_ptrs), lda=ldy, a_kmajor=False, a_mode=1 if ta else 0,
             sA=(0 if ta else sdy, 0),
             b=list(x_ptrs), ldb=ldx, b_kmajor=False, b_mode=1 if tb else 0,
             sB=(0 if tb else sx, 0),
             c=[_ptr(g, r0 * Kin) for g in grads], ldc=Kin, c_mode=1, batch0=len(Ws),
             beta=1.0, dbias_tab=dbt, device=dev)
    _grad_done(*Ws)
    if dbt is not None:
        _grad_done(*bs)
    return dbt is not None


def _kcat_ok(rows: int, n_ptrs: int, cd) -> bool:
    """Whether a per-batch K-concatenated wgrad (jmt_gemm operand mode 3) applies: the segment
    length (rows) a multiple of the 128-B K-tile and the pointer table within 8 entries."""
    return (_merge_wgrads["on"] and cd != torch.float32 and rows % 64 == 0 and n_ptrs <= 8)


# one weight-gradient launch for the two uses of each cross-attention module (K-concatenated
# pairs) and for the encoders' W1 / W2 (JMT_WGRAD_MERGE=0: the round-5 launches, A/B switch)
_merge_wgrads = {"on": os.environ.get("JMT_WGRAD_MERGE", "1") != "0"}


def _gemm_wgrad_kcat(dy_segs, ldy: int, x_segs, ldx: int, rows: int, n: int, Ws, r0: int, cd,
                     dev, bs=None) -> bool:
    """W_g.grad[r0:r0+n] += sum_s dY[g][s]^T X[g][s]: each weight's uses as the K-segments of ONE
    batch entry (jmt_gemm operand mode 3, K = len(segments) x rows), so the two uses of a module
    are one (256 x 256 tile, K = 2 rows) item set of the split-K ping-pong kernel instead of two
    12-tile launches on the 128 x 128 split plan.  With `bs`, b_g.grad += the column sums of all
    of dY[g]'s segments (the row sums of A over the whole K).  Returns as _gemm_wgrad."""
    from .functional import fused_bgrad_ok
    nseg = len(dy_segs[0])
    assert all(len(d) == nseg for d in dy_segs) and all(len(x) == nseg for x in x_segs)
    grads = []
    for W in Ws:
        g = _grad_buffer(W)
        grads.append(g if g is not None else torch.zeros_like(W))
    dbt = None
    if bs is not None and n > 1 and fused_bgrad_ok(cd):
        dbt = []
        for b in bs:
            gb = _grad_buffer(b)
            dbt.append(gb[r0:r0 + n] if gb is not None else
                       torch.empty(n, dtype=torch.float32, device=dev))
    Kin = Ws[0].shape[1]
    ops.gemm(M=n, N=Kin, K=nseg * rows, ab_dtype=_dc(cd), c_dtype=ops.F32,
             a=[p for d in dy_segs for p in d], lda=ldy, a_kmajor=False, a_mode=3, a_kseg=rows,
             b=[p for x in x_segs for p in x], ldb=ldx, b_kmajor=False, b_mode=3, b_kseg=rows,
             c=[_ptr(g, r0 * Kin) for g in grads], ldc=Kin, c_mode=1, batch0=len(Ws),
             beta=1.0, dbias_tab=dbt, device=dev)
    _grad_done(*Ws)
    if dbt is not None:
        _grad_done(*bs)
    return dbt is not None


def _bias_grad(dy2: torch.Tensor, ld: int, rows: int, n: int, b, r0: int):
    gb = _grad_buffer(b)
    if gb is not None:
        ops.colsum(dy2, ld, rows, n, gb[r0:r0 + n], beta_acc=True)
        _grad_done(b)


def _bias_grad_grouped(dy_ptr: int, G: int, ld: int, sdy: int, rows: int, n: int, bs, r0: int,
                       cd, dev):
    """b_g.grad[r0:r0+n] += column sums of the g-th (rows x n) block at dy_ptr + g*sdy (one
    grouped colsum launch pair; the bs must be distinct parameters)."""
    dbs = []
    for b in bs:
        gb = _grad_buffer(b)
        dbs.append(gb[r0:r0 + n] if gb is not None else
                   torch.empty(n, dtype=torch.float32, device=dev))
    ops.colsum_grouped(dy_ptr, _dc(cd), G, ld, sdy, rows, n, dbs, beta_acc=True, device=dev)
    _grad_done(*bs)


def _contig(t: torch.Tensor, cd) -> torch.Tensor:
    if t.dtype != cd:
        t = ops.cast(t.contiguous(), cd)
    return t if t.is_contiguous() else t.contiguous()


# ------------------------------------------------------------------------- stacking
class StackGroupsFn(Function):
    """X = stack(xs) -> (G, B, T, E) in the compute dtype (one strided copy per stream); the
    backward hands out views of the incoming gradient."""

    @staticmethod
    def forward(ctx, *xs):
        cd = compute_dtype()
        x0 = xs[0]
        B, T, E = x0.shape
        X = torch.empty(len(xs), B, T, E, dtype=cd, device=x0.device)
        for g, x in enumerate(xs):
            assert tuple(x.shape) == (B, T, E), "StackGroupsFn: streams must share (B, T, E)"
            if x.stride(-1) != 1 or x.stride(1) != E * x.stride(2) or x.stride(0) != T * x.stride(1):
                x = x.contiguous()
            ops.copy2d(x.data_ptr(), ops.dt(x), X[g].data_ptr(), ops.dt(X), B * T, E,
                       x.stride(1), 1, E, 1)
        return X

    @staticmethod
    def backward(ctx, dX):
        return tuple(dX[g] for g in range(dX.shape[0]))


def stack_groups(*xs) -> torch.Tensor:
    return StackGroupsFn.apply(*xs)


class StackJointFn(Function):
    """X = stack(v, p, cat(v, p) W^T + b) -> (3, B, T, E): the two streams and the joint
    representation of out_layer_pv (mm_multi_transformers.py:120-124) in one stacked buffer;
    the K-concatenated GEMM writes the third slot directly.  The backward adds out_layer_pv's
    input gradients into the first two slots of the incoming dX with the dgrad GEMM's beta = 1
    epilogue, so the two uses of v and p need no separate gradient sum."""

    @staticmethod
    def forward(ctx, v, p, W, b):
        from .functional import _linear_fwd
        cd = compute_dtype()
        B, T, E = v.shape
        assert tuple(p.shape) == (B, T, E) and W.shape == (E, 2 * E), (v.shape, p.shape, W.shape)
        X = torch.empty(3, B, T, E, dtype=cd, device=v.device)
        for g, x in enumerate((v, p)):
            if x.stride(-1) != 1 or x.stride(1) != E * x.stride(2) or \
                    x.stride(0) != T * x.stride(1):
                x = x.contiguous()
            ops.copy2d(x.data_ptr(), ops.dt(x), X[g].data_ptr(), ops.dt(X), B * T, E,
                       x.stride(1), 1, E, 1)
        _linear_fwd([X[0], X[1]], E, B * T, E, W, 0, E, b, X[2], E, cd)
        ctx.save_for_backward(X, W, b)
        ctx.meta = (cd, v.dtype, p.dtype)
        return X

    @staticmethod
    def backward(ctx, dX):
        from .functional import Rows, _bgrad, _cast_keep_layout, _dgrad, _wgrad
        X, W, b = ctx.saved_tensors
        cd, vdt, pdt = ctx.meta
        G3, B, T, E = X.shape
        # the incoming gradient is this Function's alone (the stacked X feeds the encoder group
        # only): its first two slots receive out_layer_pv's input gradients in place
        dX = _contig(dX, cd)
        G = Rows(dX[2])
        _dgrad(G, E, W, 0, cd, [dX[0], dX[1]], E, 2, E, beta=1.0)
        if not _wgrad(G, E, [X[0], X[1]], E, E, W, 0, cd, b):
            _bgrad(G, E, b, 0)
        dv = dX[0] if vdt == cd else _cast_keep_layout(dX[0], vdt)
        dp = dX[1] if pdt == cd else _cast_keep_layout(dX[1], pdt)
        return dv, dp, None, None


def stack_joint(v, p, W, b) -> torch.Tensor:
    return StackJointFn.apply(v, p, W, b)


class StackTokensFn(Function):
    """The SELF_ATTEN head's token stack (mm_multi_transformers.py:171-178) from the stacked
    cross-attention outputs O6 (S, B, T, E): a (B, T, S, E) buffer filled by S strided copies,
    returned as its seq-first (S, B*T, E) view.  The backward writes dO6 (S, B, T, E) with S
    strided copies — one gradient buffer, no per-slice zero-fill / copy / sum as the autograd of
    S separate selections of O6 would run."""

    @staticmethod
    def forward(ctx, X):
        cd = compute_dtype()
        X = _contig(X, cd)
        S, B, T, E = X.shape
        buf = torch.empty(B, T, S, E, dtype=cd, device=X.device)
        for s in range(S):
            ops.copy2d(X[s].data_ptr(), ops.dt(X), _ptr(buf, s * E), ops.dt(buf), B * T, E, E, 1,
                       S * E, 1)
        ctx.meta = (S, B, T, E, cd)
        return buf.view(B * T, S, E).permute(1, 0, 2)

    @staticmethod
    def backward(ctx, g):
        S, B, T, E, cd = ctx.meta
        gb = g.permute(1, 0, 2)                      # (B*T, S, E) logical
        if gb.dtype != cd or gb.stride(2) != 1 or gb.stride(1) != E or gb.stride(0) != S * E:
            gb = gb.to(cd).contiguous()
        dX = torch.empty(S, B, T, E, dtype=cd, device=g.device)
        for s in range(S):
            ops.copy2d(_ptr(gb, s * E), ops.dt(gb), dX[s].data_ptr(), ops.dt(dX), B * T, E, S * E,
                       1, E, 1)
        return dX


def stack_tokens(X) -> torch.Tensor:
    return StackTokensFn.apply(X)


class LastQueryMHAFn(Function):
    """nn.MultiheadAttention(last, enc, enc) with last = enc[-1:] (the SELF_ATTEN head's final
    attention, mm_multi_transformers.py:186-193: only the last query row is kept): q from the
    last token's rows, packed k|v from all tokens, attention core, out_proj; returns (N, E).
    The backward adds the query path's input gradient into the last token's rows of the key /
    value path's input gradient with a beta = 1 GEMM epilogue — no zero-filled slice gradient
    and no gradient sum."""

    @staticmethod
    def forward(ctx, enc, Win, bin_, Wout, bout, H):
        from .functional import Rows, _ld, _linear_fwd
        cd = compute_dtype()
        L, N, E = enc.shape
        X = Rows(enc, cd)                              # rows in enc's memory order
        kv = X.like(2 * E, cd)
        _linear_fwd([X.t], X.ld, X.rows, E, Win, E, 2 * E, bin_, kv, _ld(kv, X.perm), cd)
        xl = X.t[-1:]
        XL = Rows(xl)
        q = XL.like(E, cd)
        _linear_fwd([XL.t], XL.ld, XL.rows, E, Win, 0, E, bin_, q, _ld(q, XL.perm), cd)
        o, asaved = attn_forward(q, kv, kv, E, H, 0, 0, E)
        O = Rows(o)
        y = O.like(E, cd)
        _linear_fwd([O.t], O.ld, O.rows, E, Wout, 0, E, bout, y, _ld(y, O.perm), cd)
        ctx.save_for_backward(X.t, q, kv, o, Win, bin_, Wout, bout)
        ctx.asaved = asaved
        ctx.meta = (cd, enc.dtype, X.perm, XL.perm, O.perm)
        return y[0]

    @staticmethod
    def backward(ctx, gy):
        from .functional import (Rows, _bgrad, _cast_keep_layout, _dgrad, _ld, _match, _wgrad)
        x, q, kv, o, Win, bin_, Wout, bout = ctx.saved_tensors
        cd, xdt, xperm, xlperm, operm = ctx.meta
        L, N, E = x.shape
        O = Rows(o)
        G = _match(gy.unsqueeze(0), Rows(O.like(E, cd)), cd)          # (1, N, E) in o's order
        do = O.like(E, cd)
        _dgrad(G, E, Wout, 0, cd, [do], _ld(do, O.perm), 1, E)
        if not _wgrad(G, E, [O.t], O.ld, E, Wout, 0, cd, bout):
            _bgrad(G, E, bout, 0)
        X = Rows(x)
        dkv = X.like(2 * E, cd)
        dq = Rows(q).like(E, cd)
        attn_backward(ctx.asaved, do, dq, dkv, dkv)
        DKV = Rows(dkv)
        dx = X.like(E, cd)
        _dgrad(DKV, 2 * E, Win, E, cd, [dx], _ld(dx, X.perm), 1, E)
        if not _wgrad(DKV, 2 * E, [X.t], X.ld, E, Win, E, cd, bin_):
            _bgrad(DKV, 2 * E, bin_, E)
        DQ = Rows(dq)
        XL = Rows(x[-1:])
        dxl = dx[-1:]
        _dgrad(DQ, E, Win, 0, cd, [dxl], _ld(dxl, XL.perm), 1, E, beta=1.0)
        if not _wgrad(DQ, E, [XL.t], XL.ld, E, Win, 0, cd, bin_):
            _bgrad(DQ, E, bin_, 0)
        if xdt != cd:
            dx = _cast_keep_layout(dx, xdt)
        ctx.asaved = None
        return dx, None, None, None, None, None


def last_query_mha(enc, mha) -> torch.Tensor:
    return LastQueryMHAFn.apply(enc, mha.in_proj_weight, mha.in_proj_bias, mha.out_proj.weight,
                                mha.out_proj.bias, mha.num_heads)


# ------------------------------------------------------------------------- encoder group
def encoder_layer_params(layer) -> List[torch.Tensor]:
    """The 12 parameters of one TransformerEncoderLayer (mm_multi_transformers.py:48-70)."""
    a, ff = layer.attention, layer.feed_forward
    return [a.in_proj_weight, a.in_proj_bias, a.out_proj.weight, a.out_proj.bias,
            ff[0].weight, ff[0].bias, ff[len(ff) - 1].weight, ff[len(ff) - 1].bias,
            layer.layer_norm1.weight, layer.layer_norm1.bias,
            layer.layer_norm2.weight, layer.layer_norm2.bias]


class EncoderGroupFn(Function):
    """G post-LN encoder layers (mm_multi_transformers.py:61-70, one per stream, same shapes,
    own weights) on the stacked seq-first input X (G, B, T, E):
        Y_g = LN2(H_g + W2 relu(W1 H_g + b1) + b2),  H_g = LN1(X_g + MHA_g(X_g, X_g, X_g)).
    params: 12 per group (encoder_layer_params).
    batch_axis: the self-attention runs over the B axis of each group (sequences of length B,
    one per t) — MultimodalTransformer_wo_JR feeds its encoders batch-first tensors
    (mm_transformers.py:119-122); the attention core is then one launch per group (a group's
    (B, T) rows are a (seq, batch)-strided layout, the G groups together are not), every GEMM,
    LayerNorm and bias reduction stays one grouped launch."""

    @staticmethod
    def forward(ctx, X, meta, *params):
        H, eps1, eps2, batch_axis = meta
        cd = compute_dtype()
        X = _contig(X, cd)
        G, B, T, E = X.shape
        R = B * T
        dev = X.device
        P = [params[12 * g:12 * g + 12] for g in range(G)]
        hid = P[0][4].shape[0]
        cdt = _dc(cd)
        # packed in-projection (3 groups, one launch)
        QKV = torch.empty(G, B, T, 3 * E, dtype=cd, device=dev)
        _gemm_fwd([X.data_ptr()], E, R * E, R, E, [p[0] for p in P], 0, 3 * E,
                  [p[1] for p in P], QKV.data_ptr(), 3 * E, R * 3 * E, cdt, cd, dev)
        if batch_axis:
            # QKV[g] (B, T, 3E) read as seq-first (L = B, N = T): attention over the batch axis
            outs = [attn_forward(QKV[g], QKV[g], QKV[g], E, H, 0, E, 2 * E) for g in range(G)]
            O = [o for o, _ in outs]                           # G x (B, T, E)
            asaved = [sv for _, sv in outs]
            o_ptrs = [o.data_ptr() for o in O]
        else:
            sf = QKV.view(G * B, T, 3 * E).permute(1, 0, 2)      # (T, G*B, 3E) seq-first
            o, asaved = attn_forward(sf, sf, sf, E, H, 0, E, 2 * E)  # memory (G*B, T, E)
            O = o.permute(1, 0, 2)
            o_ptrs = [O.data_ptr()]
        A1 = torch.empty(G, B, T, E, dtype=cd, device=dev)
        _gemm_fwd(o_ptrs, E, R * E if len(o_ptrs) == 1 else 0, R, E, [p[2] for p in P], 0, E,
                  [p[3] for p in P], A1.data_ptr(), E, R * E, cdt, cd, dev)
        H1 = torch.empty_like(A1)
        st1 = torch.empty(2, G * R, dtype=torch.float32, device=dev)
        if not ops.layernorm_fwd_grouped(X, A1, [p[8] for p in P], [p[9] for p in P], eps1, H1,
                                         st1[0], st1[1]):
            for g in range(G):
                ops.layernorm_fwd(X[g], E, A1[g], E, P[g][8], P[g][9], eps1, H1[g], E,
                                  st1[0, g * R:], st1[1, g * R:], R, E)
        F1 = torch.empty(G, B, T, hid, dtype=cd, device=dev)
        _gemm_fwd([H1.data_ptr()], E, R * E, R, E, [p[4] for p in P], 0, hid,
                  [p[5] for p in P], F1.data_ptr(), hid, R * hid, cdt, cd, dev, relu=True)
        F2 = torch.empty(G, B, T, E, dtype=cd, device=dev)
        _gemm_fwd([F1.data_ptr()], hid, R * hid, R, hid, [p[6] for p in P], 0, E,
                  [p[7] for p in P], F2.data_ptr(), E, R * E, cdt, cd, dev)
        Y = torch.empty_like(A1)
        st2 = torch.empty(2, G * R, dtype=torch.float32, device=dev)
        if not ops.layernorm_fwd_grouped(H1, F2, [p[10] for p in P], [p[11] for p in P], eps2, Y,
                                         st2[0], st2[1]):
            for g in range(G):
                ops.layernorm_fwd(H1[g], E, F2[g], E, P[g][10], P[g][11], eps2, Y[g], E,
                                  st2[0, g * R:], st2[1, g * R:], R, E)
        ctx.params = params
        ctx.state = (X, QKV, asaved, O, A1, H1, st1, F1, F2, st2)
        ctx.meta = (G, B, T, E, hid, cd, batch_axis)
        return Y

    @staticmethod
    def backward(ctx, dY):
        G, B, T, E, hid, cd, batch_axis = ctx.meta
        X, QKV, asaved, O, A1, H1, st1, F1, F2, st2 = ctx.state
        o_ptrs = [o.data_ptr() for o in O] if batch_axis else [O.data_ptr()]
        o_reads = tuple(O) if batch_axis else (O,)
        params = ctx.params
        P = [params[12 * g:12 * g + 12] for g in range(G)]
        R = B * T
        dev = X.device
        cdt = _dc(cd)
        dY = _contig(dY, cd)

        def ln_bwd(x, r, dy, st, gamma, beta, dx, bias=None):
            """LayerNorm backward per group; with `bias` (the biases of the linears whose
            outputs r entered the residual sums) their gradients — the column sums of dx — are
            reduced in the same launch pair.  Returns whether they were.
            The fused bias sum reduces the fp32 dx before it is rounded to the compute dtype;
            the fallback column sum (_bias_grad) reads the rounded dx — the same quantity, one
            rounding apart.  The kernels take one accumulate flag for all their outputs, so when
            any of the gradient buffers is missing (a frozen parameter) every output goes to a
            scratch block and the present buffers accumulate it afterwards."""
            fused = bias is not None
            # all G groups in one launch pair when every gradient buffer exists
            gb = [_grad_buffer(t) for t in gamma]
            bb = [_grad_buffer(t) for t in beta]
            sb = [_grad_buffer(t) for t in bias] if fused else []
            if all(t is not None for t in gb + bb + sb) and ops.layernorm_bwd_grouped(
                    x, r, dy, st[0], st[1], gamma, dx, gb, bb, sb if fused else None,
                    True) is not None:
                for g in range(G):
                    _grad_done(gamma[g], beta[g], *([bias[g]] if fused else []))
                return fused
            for g in range(G):
                bufs = [_grad_buffer(gamma[g]), _grad_buffer(beta[g])]
                if fused:
                    bufs.append(_grad_buffer(bias[g]))
                tmp = None
                if any(b is None for b in bufs):
                    tmp = torch.zeros(3, E, dtype=torch.float32, device=dev)
                outs = bufs if tmp is None else [tmp[0], tmp[1], tmp[2]]
                args = (x[g], E, r[g], E, dy[g], E, st[0, g * R:], st[1, g * R:], gamma[g], dx[g],
                        E, outs[0], outs[1])
                done = fused and ops.layernorm_bwd_dsum(
                    *args, outs[2] if tmp is None else tmp[2], tmp is None, R, E) is not None
                if not done:
                    ops.layernorm_bwd(*args, tmp is None, R, E)
                if tmp is not None:
                    for b, t in zip(bufs[:3 if done else 2], tmp):
                        if b is not None:
                            b.add_(t)
                if done:
                    _grad_done(gamma[g], beta[g], bias[g])
                    continue
                _grad_done(gamma[g], beta[g])
                if fused:        # shape not covered by the fused form: this group's bias apart
                    _bias_grad(dx[g].view(R, E), E, R, E, bias[g], 0)
            return fused

        # LN2: dS2 = d(H1 + F2)
        dS = torch.empty(G, B, T, E, dtype=cd, device=dev)
        b2_done = ln_bwd(H1, F2, dY, st2, [p[10] for p in P], [p[11] for p in P], dS,
                         bias=[p[7] for p in P])
        # FFN (the ReLU mask is fused into the W2 dgrad epilogue)
        dF1 = torch.empty(G, B, T, hid, dtype=cd, device=dev)
        _gemm_dgrad(dS.data_ptr(), E, R * E, R, E, [p[6] for p in P], 0, dF1.data_ptr(), hid,
                    R * hid, cdt, cd, dev, aux=F1, ldaux=hid)
        # (W2's weight gradient stays on the compute stream: on the side stream the in-place
        # dH1 below would have to wait for it, which measured slower, profiles/r02_side_stream.txt)
        # With hid == E, W1's weight gradient (dF1 and H1 are ready here) goes in the same launch:
        # 2 G entries of 512 x 512 over the B T rows (24 tiles at G = 3: the split-K ping-pong
        # kernel) instead of two 12-tile launches on the 128 x 128 split plan
        merged = _merge_wgrads["on"] and hid == E and 2 * G <= 8 and cd != torch.float32
        if merged:
            ws = [p[6] for p in P] + [p[4] for p in P]
            bsw = ([] if b2_done else [p[7] for p in P]) + [p[5] for p in P]
            fused = _gemm_wgrad([dS[g].data_ptr() for g in range(G)] +
                                [dF1[g].data_ptr() for g in range(G)], E, 0,
                                [F1[g].data_ptr() for g in range(G)] +
                                [H1[g].data_ptr() for g in range(G)], E, 0, R, E, ws, 0, cd, dev,
                                bs=None if b2_done else bsw)
            if not fused:
                if not b2_done:
                    _bias_grad_grouped(dS.data_ptr(), G, E, R * E, R, E, [p[7] for p in P], 0,
                                       cd, dev)
                _bias_grad_grouped(dF1.data_ptr(), G, hid, R * hid, R, hid, [p[5] for p in P], 0,
                                   cd, dev)
            b2_done = True
        else:
            b2_done = _gemm_wgrad([dS.data_ptr()], E, R * E, [F1.data_ptr()], hid, R * hid, R, E,
                                  [p[6] for p in P], 0, cd, dev,
                                  bs=None if b2_done else [p[7] for p in P]) or b2_done
        if not b2_done:
            _bias_grad_grouped(dS.data_ptr(), G, E, R * E, R, E, [p[7] for p in P], 0, cd, dev)
        # dH1 = dS2 + dF1 . W1  (in place on dS: beta = 1)
        _gemm_dgrad(dF1.data_ptr(), hid, R * hid, R, hid, [p[4] for p in P], 0, dS.data_ptr(),
                    E, R * E, cdt, cd, dev, beta=1.0)

        def w1_grads():         # side stream: dF1 and H1 are not written again
            if not _gemm_wgrad([dF1.data_ptr()], hid, R * hid, [H1.data_ptr()], E, R * E, R,
                               hid, [p[4] for p in P], 0, cd, dev, bs=[p[5] for p in P]):
                _bias_grad_grouped(dF1.data_ptr(), G, hid, R * hid, R, hid, [p[5] for p in P], 0,
                                   cd, dev)

        if not merged:
            streams.run_side(w1_grads, reads=(dF1, H1))
        # LN1: dS1 = d(X + A1)
        dS1 = torch.empty_like(dS)
        bo_done = ln_bwd(X, A1, dS, st1, [p[8] for p in P], [p[9] for p in P], dS1,
                         bias=[p[3] for p in P])
        # out_proj
        dO = dS     # reuse: dS is dead
        _gemm_dgrad(dS1.data_ptr(), E, R * E, R, E, [p[2] for p in P], 0, dO.data_ptr(), E,
                    R * E, cdt, cd, dev)

        def out_proj_grads():   # side stream, under the attention backward
            done = _gemm_wgrad([dS1.data_ptr()], E, R * E, o_ptrs, E,
                               R * E if len(o_ptrs) == 1 else 0, R, E, [p[2] for p in P], 0, cd,
                               dev, bs=None if bo_done else [p[3] for p in P])
            if not (bo_done or done):
                _bias_grad_grouped(dS1.data_ptr(), G, E, R * E, R, E, [p[3] for p in P], 0, cd,
                                   dev)

        streams.run_side(out_proj_grads, reads=(dS1,) + o_reads)
        # attention core -> packed dQKV
        dQKV = torch.empty(G, B, T, 3 * E, dtype=cd, device=dev)
        if batch_axis:
            for g in range(G):
                attn_backward(asaved[g], dO[g], dQKV[g], dQKV[g], dQKV[g])
        else:
            dsf = dQKV.view(G * B, T, 3 * E).permute(1, 0, 2)
            attn_backward(asaved, dO.view(G * B, T, E).permute(1, 0, 2), dsf, dsf, dsf)
        # in_proj: dX = dS1 + dQKV . W_in  (in place on dS1, once the side stream has read it)
        streams.wait_side()
        _gemm_dgrad(dQKV.data_ptr(), 3 * E, R * 3 * E, R, 3 * E, [p[0] for p in P], 0,
                    dS1.data_ptr(), E, R * E, cdt, cd, dev, beta=1.0)

        def in_proj_grads():    # side stream: dQKV and X are not written again
            if not _gemm_wgrad([dQKV.data_ptr()], 3 * E, R * 3 * E, [X.data_ptr()], E, R * E, R,
                               3 * E, [p[0] for p in P], 0, cd, dev, bs=[p[1] for p in P]):
                _bias_grad_grouped(dQKV.data_ptr(), G, 3 * E, R * 3 * E, R, 3 * E,
                                   [p[1] for p in P], 0, cd, dev)

        streams.run_side(in_proj_grads, reads=(dQKV, X))
        ctx.state = None
        return (dS1, None) + (None,) * len(params)


def encoder_group(X, layers, num_heads: int, batch_axis: bool = False):
    """Apply `layers` (one TransformerEncoderLayer per stream) to the stacked X (attention over
    T, or over B with batch_axis)."""
    params = [p for layer in layers for p in encoder_layer_params(layer)]
    meta = (num_heads, layers[0].layer_norm1.eps, layers[0].layer_norm2.eps, bool(batch_axis))
    return EncoderGroupFn.apply(X, meta, *params)


# the wo_JR model's two cross-attentions (mm_transformers.py:125-135): (module, query, key/value)
# with module 0 = cross_attention_v, 1 = cross_attention_p, stream 0 = visual, 1 = physiological
CROSS_PAIRS_WO_JR = ((0, 0, 1), (1, 1, 0))


# ------------------------------------------------------------------------- cross attentions
def mha_params(mha) -> List[torch.Tensor]:
    return [mha.in_proj_weight, mha.in_proj_bias, mha.out_proj.weight, mha.out_proj.bias]


class CrossAttention6Fn(Function):
    """The six key-is-value cross-attentions of mm_multi_transformers.py:142-167 on the stacked
    encoder outputs Y (3, B, T, E) -> O6 (6, B, T, E) in the reference's concatenation order
    (CROSS_PAIRS).  params: 4 per module (mha_params) for cross_attention_v / _p / _pv."""

    @staticmethod
    def forward(ctx, Y, meta, *params):
        H, pairs = meta
        cd = compute_dtype()
        Y = _contig(Y, cd)
        S, B, T, E = Y.shape
        R = B * T
        dev = Y.device
        cdt = _dc(cd)
        M = [params[4 * m:4 * m + 4] for m in range(len(params) // 4)]
        NP = len(pairs)
        QKV = torch.empty(NP, B, T, 3 * E, dtype=cd, device=dev)
        in_w = [M[m][0] for m, _, _ in pairs]
        in_b = [M[m][1] for m, _, _ in pairs]
        # queries (each module's query projection is evaluated for both of its calls, exactly as
        # the reference does) and packed key/values, one launch each
        _gemm_fwd([Y[q].data_ptr() for _, q, _ in pairs], E, 0, R, E, in_w, 0, E, in_b,
                  QKV.data_ptr(), 3 * E, R * 3 * E, cdt, cd, dev)
        _gemm_fwd([Y[k].data_ptr() for _, _, k in pairs], E, 0, R, E, in_w, E, 2 * E, in_b,
                  _ptr(QKV, E), 3 * E, R * 3 * E, cdt, cd, dev)
        sf = QKV.view(NP * B, T, 3 * E).permute(1, 0, 2)
        o, asaved = attn_forward(sf, sf, sf, E, H, 0, E, 2 * E)
        O = o.permute(1, 0, 2)                                   # (NP*B, T, E) memory
        O6 = torch.empty(NP, B, T, E, dtype=cd, device=dev)
        _gemm_fwd([O.data_ptr()], E, R * E, R, E, [M[m][2] for m, _, _ in pairs], 0, E,
                  [M[m][3] for m, _, _ in pairs], O6.data_ptr(), E, R * E, cdt, cd, dev)
        ctx.params = params
        ctx.state = (Y, QKV, asaved, O)
        ctx.meta = (pairs, S, B, T, E, cd)
        return O6

    @staticmethod
    def backward(ctx, dO6):
        pairs, S, B, T, E, cd = ctx.meta
        Y, QKV, asaved, O = ctx.state
        params = ctx.params
        M = [params[4 * m:4 * m + 4] for m in range(len(params) // 4)]
        NP = len(pairs)
        R = B * T
        dev = Y.device
        cdt = _dc(cd)
        dO6 = _contig(dO6, cd)
        # launches of the batched wgrads: each launch holds distinct modules
        halves, seen = [[]], [set()]
        for i, (m, _, _) in enumerate(pairs):
            if m in seen[-1]:
                halves.append([])
                seen.append(set())
            halves[-1].append(i)
            seen[-1].add(m)
        # out_proj: input gradient on the compute stream, weight / bias gradients on the side
        # stream (jmt.streams.run_side) overlapping the attention backward
        dO = torch.empty(NP, B, T, E, dtype=cd, device=dev)
        _gemm_dgrad(dO6.data_ptr(), E, R * E, R, E, [M[m][2] for m, _, _ in pairs], 0,
                    dO.data_ptr(), E, R * E, cdt, cd, dev)

        # the two uses of each module (one per half) as the K-segments of one batch entry:
        # h0[u] and h1[u] are the pairs of module ms[u]
        kcat = (len(halves) == 2 and len(halves[0]) == len(halves[1]) and
                sorted(pairs[i][0] for i in halves[0]) ==
                sorted(pairs[i][0] for i in halves[1]) and
                _kcat_ok(R, 2 * len(halves[0]), cd))
        if kcat:
            h0 = list(halves[0])
            ms = [pairs[i][0] for i in h0]
            h1 = [next(j for j in halves[1] if pairs[j][0] == m) for m in ms]

        def out_proj_grads():
            if kcat:
                if _gemm_wgrad_kcat([[_ptr(dO6, i * R * E), _ptr(dO6, j * R * E)]
                                     for i, j in zip(h0, h1)], E,
                                    [[O[i * B].data_ptr(), O[j * B].data_ptr()]
                                     for i, j in zip(h0, h1)], E, R, E, [M[m][2] for m in ms],
                                    0, cd, dev, bs=[M[m][3] for m in ms]):
                    return
                for m, i, j in zip(ms, h0, h1):
                    _bias_grad(dO6[i], E, R, E, M[m][3], 0)
                    _bias_grad(dO6[j], E, R, E, M[m][3], 0)
                return
            rest = []
            for h in halves:
                if not _gemm_wgrad([_ptr(dO6, i * R * E) for i in h], E, 0,
                                   [O[i * B].data_ptr() for i in h], E, 0, R, E,
                                   [M[pairs[i][0]][2] for i in h], 0, cd, dev,
                                   bs=[M[pairs[i][0]][3] for i in h]):
                    rest.append(h)
            for h in rest:
                if _consecutive(h):
                    _bias_grad_grouped(_ptr(dO6, h[0] * R * E), len(h), E, R * E, R, E,
                                       [M[pairs[i][0]][3] for i in h], 0, cd, dev)
                else:
                    for i in h:
                        _bias_grad(dO6[i], E, R, E, M[pairs[i][0]][3], 0)

        streams.run_side(out_proj_grads, reads=(dO6, O))
        # attention core -> packed dQKV (NP, B, T, 3E)
        dQKV = torch.empty(NP, B, T, 3 * E, dtype=cd, device=dev)
        dsf = dQKV.view(NP * B, T, 3 * E).permute(1, 0, 2)
        attn_backward(asaved, dO.view(NP * B, T, E).permute(1, 0, 2), dsf, dsf, dsf)

        # in_proj weight gradients (side stream, overlapping the stream dgrads): query rows
        # [0, E) from the query stream, key/value rows [E, 3E) from the key stream
        def in_proj_grads():
            if kcat:
                ws = [M[m][0] for m in ms]
                bs = [M[m][1] for m in ms]
                seg = lambda off: [[_ptr(dQKV, i * R * 3 * E + off), _ptr(dQKV, j * R * 3 * E + off)]
                                   for i, j in zip(h0, h1)]
                fq = _gemm_wgrad_kcat(seg(0), 3 * E,
                                      [[Y[pairs[i][1]].data_ptr(), Y[pairs[j][1]].data_ptr()]
                                       for i, j in zip(h0, h1)], E, R, E, ws, 0, cd, dev, bs=bs)
                fkv = _gemm_wgrad_kcat(seg(E), 3 * E,
                                       [[Y[pairs[i][2]].data_ptr(), Y[pairs[j][2]].data_ptr()]
                                        for i, j in zip(h0, h1)], E, R, 2 * E, ws, E, cd, dev,
                                       bs=bs if fq else None)
                if not (fq and fkv):
                    assert not fq, "query-row bias sums fused without the key / value rows"
                    for m, i, j in zip(ms, h0, h1):
                        _bias_grad(dQKV[i], 3 * E, R, 3 * E, M[m][1], 0)
                        _bias_grad(dQKV[j], 3 * E, R, 3 * E, M[m][1], 0)
                return
            rest = []
            for h in halves:
                ws = [M[pairs[i][0]][0] for i in h]
                bs = [M[pairs[i][0]][1] for i in h]
                fq = _gemm_wgrad([_ptr(dQKV, i * R * 3 * E) for i in h], 3 * E, 0,
                                 [Y[pairs[i][1]].data_ptr() for i in h], E, 0, R, E, ws, 0, cd,
                                 dev, bs=bs)
                fkv = _gemm_wgrad([_ptr(dQKV, i * R * 3 * E + E) for i in h], 3 * E, 0,
                                  [Y[pairs[i][2]].data_ptr() for i in h], E, 0, R, 2 * E, ws, E,
                                  cd, dev, bs=bs if fq else None)
                if not (fq and fkv):
                    assert not fq, "query-row bias sums fused without the key / value rows"
                    rest.append(h)
            for h in rest:
                if _consecutive(h):
                    _bias_grad_grouped(_ptr(dQKV, h[0] * R * 3 * E), len(h), 3 * E, R * 3 * E,
                                       R, 3 * E, [M[pairs[i][0]][1] for i in h], 0, cd, dev)
                else:
                    for i in h:
                        _bias_grad(dQKV[i], 3 * E, R, 3 * E, M[pairs[i][0]][1], 0)

        streams.run_side(in_proj_grads, reads=(dQKV, Y))
        # stream gradients: every use of stream s (as a query: rows [0,E) of W_in; as a key /
        # value: rows [E,2E) and [2E,3E)) is one K-segment of ONE dgrad GEMM (K = nseg * E)
        dY = torch.zeros(S, B, T, E, dtype=cd, device=dev) if any(
            not any(q == s or k == s for _, q, k in pairs) for s in range(S)) else \
            torch.empty(S, B, T, E, dtype=cd, device=dev)
        keep = []     # the 16-bit weight copies must outlive the launches that read them
        launches = []
        for s in range(S):
            a_ptrs, b_ptrs = [], []
            for i, (m, q, k) in enumerate(pairs):
                Wc = weight_as(M[m][0], cd)
                keep.append(Wc)
                if q == s:
                    a_ptrs.append(_ptr(dQKV, i * R * 3 * E))
                    b_ptrs.append(_ptr(Wc, 0))
                if k == s:
                    a_ptrs += [_ptr(dQKV, i * R * 3 * E + E), _ptr(dQKV, i * R * 3 * E + 2 * E)]
                    b_ptrs += [_ptr(Wc, E * E), _ptr(Wc, 2 * E * E)]
            def stream_dgrad(a_ptrs=a_ptrs, b_ptrs=b_ptrs, c_ptr=dY[s].data_ptr()):
                for c0 in range(0, len(a_ptrs), 8):   # at most 8 K-segments per launch
                    ap, bp = a_ptrs[c0:c0 + 8], b_ptrs[c0:c0 + 8]
                    ops.gemm(M=R, N=E, K=len(ap) * E, ab_dtype=cdt, c_dtype=cdt,
                             a=ap, lda=3 * E, a_kmajor=True, a_mode=2, a_kseg=E,
                             b=bp, ldb=E, b_kmajor=False, b_mode=2, b_kseg=E,
                             c=[c_ptr], ldc=E, beta=1.0 if c0 else 0.0, device=dev)
            if a_ptrs:
                launches.append(stream_dgrad)
        # one launch per stream (600 128x128 tiles each, under one round of the chip's resident
        # slots): on their own streams the three overlap each other's last-round tails
        if _PAR_STREAM_DGRAD:
            streams.run_parallel(launches, dev)
        else:
            for f in launches:
                f()
        ctx.state = None
        return (dY, None) + (None,) * len(params)


def _consecutive(h) -> bool:
    return all(b == a + 1 for a, b in zip(h[:-1], h[1:]))


def cross_attention6(Y, modules, num_heads: int, pairs=CROSS_PAIRS):
    params = [p for mod in modules for p in mha_params(mod)]
    return CrossAttention6Fn.apply(Y, (num_heads, pairs), *params)


# ------------------------------------------------------------------------- concat head
class ConcatLinearFn(Function):
    """y = cat(X[0], ..., X[S-1], dim=-1) . W^T + b for a stacked X (S, B, T, E): the FC head's
    torch.cat + out_layer1 (mm_multi_transformers.py:201-211) as one K-concatenated GEMM; the
    backward writes the stacked dX in one batched dgrad launch and W.grad in one batched wgrad."""

    @staticmethod
    def forward(ctx, X, W, b):
        cd = compute_dtype()
        X = _contig(X, cd)
        S, B, T, E = X.shape
        R = B * T
        N = W.shape[0]
        assert W.shape[1] == S * E
        dev = X.device
        Wc = weight_as(W, cd)
        y = torch.empty(B, T, N, dtype=cd, device=dev)
        ops.gemm(M=R, N=N, K=S * E, ab_dtype=_dc(cd), c_dtype=_dc(cd),
                 a=[X[s].data_ptr() for s in range(S)], lda=E, a_kmajor=True, a_mode=2,
                 a_kseg=E, b=[Wc.data_ptr()], ldb=S * E, b_kmajor=True,
                 c=[y.data_ptr()], ldc=N, bias=b, bias_mode=1, device=dev)
        ctx.save_for_backward(X, W, b)
        ctx.meta = cd
        return y

    @staticmethod
    def backward(ctx, dy):
        X, W, b = ctx.saved_tensors
        cd = ctx.meta
        S, B, T, E = X.shape
        R = B * T
        N = W.shape[0]
        dev = X.device
        dy = _contig(dy, cd)
        Wc = weight_as(W, cd)
        dX = torch.empty_like(X)
        ops.gemm(M=R, N=E, K=N, ab_dtype=_dc(cd), c_dtype=_dc(cd),
                 a=[dy.data_ptr()], lda=N, a_kmajor=True, sA=(0, 0),
                 b=[Wc.data_ptr()], ldb=S * E, b_kmajor=False, sB=(E, 0),
                 c=[dX.data_ptr()], ldc=E, sC=(R * E, 0), batch0=S, device=dev)

        def param_grads():      # side stream: overlaps the dgrads of the cross-attentions
            from .functional import fused_bgrad_ok
            gW = _grad_buffer(W)
            gb = _grad_buffer(b)
            fuse = gW is not None and gb is not None and N > 1 and fused_bgrad_ok(cd)
            if gW is not None:
                # the S K-segments share dY: segment 0 also takes its row sums (the bias grad)
                ops.gemm(M=N, N=E, K=R, ab_dtype=_dc(cd), c_dtype=ops.F32,
                         a=[dy.data_ptr()], lda=N, a_kmajor=False, sA=(0, 0),
                         b=[X.data_ptr()], ldb=E, b_kmajor=False, sB=(R * E, 0),
                         c=[gW.data_ptr()], ldc=S * E, sC=(E, 0), batch0=S, beta=1.0,
                         dbias_tab=[gb] + [None] * (S - 1) if fuse else None, device=dev)
                _grad_done(W)
            if b is not None:
                if fuse:
                    _grad_done(b)
                else:
                    _bias_grad(dy, N, R, N, b, 0)

        streams.run_side(param_grads, reads=(dy, X))
        return dX, None, None


def concat_linear(X, W, b):
    return ConcatLinearFn.apply(X, W, b)
