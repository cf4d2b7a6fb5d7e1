"""Thin, typed wrappers over the C-ABI: torch tensors in, kernel launches on the current HIP
stream out.  No math happens here — every op is one (or a few) libjmt_hip.so launches."""
from __future__ import annotations

import ctypes as C
import math
import os
from typing import Optional, Sequence

import torch

from . import _lib
from ._lib import BF16, F16, F32, GemmDesc

_DT = {torch.float32: F32, torch.bfloat16: BF16, torch.float16: F16}


def dt(t_or_dtype) -> int:
    d = t_or_dtype if isinstance(t_or_dtype, torch.dtype) else t_or_dtype.dtype
    try:
        return _DT[d]
    except KeyError:
        raise _lib.JMTError(f"unsupported dtype {d}") from None


def stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _require_cuda(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise _lib.JMTError("JMT HIP ops need device tensors (there is no CPU path)")


def workspace(nbytes: int, device) -> torch.Tensor:
    return torch.empty(max(int(nbytes), 16), dtype=torch.uint8, device=device)


# ------------------------------------------------------------------------------------ GEMM
_launch_hook = None


def set_launch_hook(hook) -> None:
    """hook(info: dict, launch: callable) -> result; used by bench.py to bracket launches of one
    GEMM instance with HIP events on the launch stream.  None disables."""
    global _launch_hook
    _launch_hook = hook


def auto_splits(M: int, N: int, K: int, batch: int, ab_dtype: int) -> int:
    """Split-K factor from the library's GEMM planner (jmt_gemm_plan_splits)."""
    return int(_lib.load().jmt_gemm_plan_splits(ab_dtype, M, N, K, batch))


def gemm(*, M: int, N: int, K: int, ab_dtype: int, c_dtype: int,
         a: Sequence[int], lda: int, a_kmajor: bool,
         b: Sequence[int], ldb: int, b_kmajor: bool,
         c: Sequence[int], ldc: int,
         a_mode: int = 0, b_mode: int = 0, c_mode: int = 0, a_kseg: int = 0, b_kseg: int = 0,
         batch0: int = 1, batch1: int = 1, sA=(0, 0), sB=(0, 0), sC=(0, 0),
         alpha: float = 1.0, beta: float = 0.0, bias: Optional[torch.Tensor] = None,
         bias_mode: int = 1, relu: bool = False, aux: Optional[torch.Tensor] = None,
         ldaux: int = 0, splits: Optional[int] = None, bias_tab=None, dbias_tab=None,
         dbias_acc: bool = True, device=None) -> None:
    """dbias_tab: per-b0 fp32 outputs (None: skip that entry) that receive (dbias_acc: += ) the
    row sums of A — a weight-gradient GEMM's bias gradient (jmt_gemm_desc ABI 4)."""
    d = GemmDesc()
    d.ab_dtype, d.c_dtype = ab_dtype, c_dtype
    d.aux_dtype = dt(aux) if aux is not None else c_dtype
    d.M, d.N, d.K = M, N, K
    for i, p in enumerate(a):
        d.a[i] = p
    for i, p in enumerate(b):
        d.b[i] = p
    for i, p in enumerate(c):
        d.c[i] = p
    d.n_a, d.n_b, d.n_c = len(a), len(b), len(c)
    d.a_mode, d.b_mode, d.c_mode = a_mode, b_mode, c_mode
    d.a_kseg, d.b_kseg = a_kseg, b_kseg
    d.a_kmajor, d.b_kmajor = int(a_kmajor), int(b_kmajor)
    d.lda, d.ldb, d.ldc, d.ldaux = lda, ldb, ldc, ldaux
    d.batch0, d.batch1 = batch0, batch1
    d.sA0, d.sA1 = sA
    d.sB0, d.sB1 = sB
    d.sC0, d.sC1 = sC
    d.alpha, d.beta = alpha, beta
    d.bias = bias.data_ptr() if bias is not None else None
    d.bias_mode = bias_mode if (bias is not None or bias_tab) else 0
    if bias_tab:
        for i, t in enumerate(bias_tab):
            d.bias_tab[i] = t.data_ptr()
        d.n_bias = len(bias_tab)
    d.relu = int(relu)
    d.aux = aux.data_ptr() if aux is not None else None
    if splits is None:
        splits = auto_splits(M, N, K, batch0 * batch1, ab_dtype)
    d.splits = splits
    ws = None
    if dbias_tab:
        for i, t in enumerate(dbias_tab):
            d.dbias_tab[i] = t.data_ptr() if t is not None else None
        d.n_dbias = len(dbias_tab)
        d.dbias_acc = int(dbias_acc)
    if splits > 1:
        nbytes = _lib.load().jmt_gemm_workspace_bytes(M, N, batch0 * batch1, splits)
        if dbias_tab:
            # the A row sums' split partials after the slabs (16-B aligned: the slab bytes are)
            dbytes = splits * batch0 * M * 4
            ws = workspace(nbytes + dbytes, device)
            d.dbias_ws = ws.data_ptr() + nbytes
            d.dbias_ws_bytes = dbytes
        else:
            ws = workspace(nbytes, device)
        d.workspace = ws.data_ptr()
        d.ws_bytes = nbytes
    launch = lambda: _lib.check(_lib.load().jmt_gemm(C.byref(d), stream()), "jmt_gemm")
    if _launch_hook is not None:
        fam = {(True, True): "gemm_NT", (True, False): "gemm_NN", (False, False): "gemm_TN",
               (False, True): "gemm_TT"}[(bool(a_kmajor), bool(b_kmajor))]
        _launch_hook({"family": fam, "ab_dtype": ab_dtype, "c_dtype": c_dtype,
                      "a_kmajor": bool(a_kmajor), "b_kmajor": bool(b_kmajor), "M": M, "N": N,
                      "K": K, "batch": batch0 * batch1, "beta": beta,
                      "dbias": bool(dbias_tab),
                      "flops": 2.0 * M * N * K * batch0 * batch1,
                      "bytes": batch0 * batch1 * ((M + N) * K * (4 if ab_dtype == F32 else 2) +
                                                  M * N * (4 if c_dtype == F32 else 2)),
                      "inplace": any(p in list(c) for p in list(a) + list(b))}, launch)
    else:
        launch()
    return ws   # keep alive until the launch is ordered (caching allocator is stream-ordered)


# ------------------------------------------------------------------------------------ rows

def l2norm_fwd(x2: torch.Tensor, ldx: int, rows: int, D: int, y2: torch.Tensor, ldy: int,
               inv_norm: torch.Tensor, eps: float):
    _require_cuda(x2, y2)
    _lib.call("jmt_l2norm_fwd", dt(x2), dt(y2), rows, D, x2.data_ptr(), ldx, y2.data_ptr(), ldy,
              inv_norm.data_ptr(), eps, stream())


def l2norm_bwd(x2, ldx, dy2, lddy, inv_norm, eps, dx2, lddx, rows, D):
    _lib.call("jmt_l2norm_bwd", dt(x2), dt(dy2), dt(dx2), rows, D, x2.data_ptr(), ldx,
              dy2.data_ptr(), lddy, inv_norm.data_ptr(), eps, dx2.data_ptr(), lddx, stream())


def layernorm_fwd(x, ldx, r, ldr, gamma, beta, eps, y, ldy, mean, rstd, rows, D):
    _lib.call("jmt_layernorm_fwd", dt(x), dt(y), rows, D, x.data_ptr(), ldx,
              r.data_ptr() if r is not None else None, ldr, gamma.data_ptr(), beta.data_ptr(),
              eps, y.data_ptr(), ldy, mean.data_ptr(), rstd.data_ptr(), stream())


def layernorm_bwd(x, ldx, r, ldr, dy, lddy, mean, rstd, gamma, dx, lddx, dgamma, dbeta,
                  beta_acc, rows, D):
    nblk = _lib.load().jmt_layernorm_bwd_blocks(rows)
    part = torch.empty(max(nblk, 1) * 2 * D, dtype=torch.float32, device=x.device)
    _lib.call("jmt_layernorm_bwd", dt(x), dt(dy), dt(dx), rows, D, x.data_ptr(), ldx,
              r.data_ptr() if r is not None else None, ldr, dy.data_ptr(), lddy,
              mean.data_ptr(), rstd.data_ptr(), gamma.data_ptr(), dx.data_ptr(), lddx,
              dgamma.data_ptr(), dbeta.data_ptr(), int(beta_acc), part.data_ptr(), stream())
    return part


def layernorm_bwd_dsum(x, ldx, r, ldr, dy, lddy, mean, rstd, gamma, dx, lddx, dgamma, dbeta,
                       dsum, beta_acc, rows, D):
    """layernorm_bwd plus dsum (+)= column sums of dx; returns the partials buffer, or None when
    the shape is not covered (nothing written: the caller reduces dsum itself)."""
    nblk = _lib.load().jmt_layernorm_bwd_blocks(rows)
    part = torch.empty(max(nblk, 1) * 3 * D, dtype=torch.float32, device=x.device)
    rc = _lib.load().jmt_layernorm_bwd_dsum(
        dt(x), dt(dy), dt(dx), rows, D, x.data_ptr(), ldx,
        r.data_ptr() if r is not None else None, ldr, dy.data_ptr(), lddy, mean.data_ptr(),
        rstd.data_ptr(), gamma.data_ptr(), dx.data_ptr(), lddx, dgamma.data_ptr(),
        dbeta.data_ptr(), dsum.data_ptr(), int(beta_acc), part.data_ptr(), stream())
    if rc == _lib.ERR_UNSUPPORTED:
        return None
    _lib.check(rc, "jmt_layernorm_bwd_dsum")
    return part


def _ptr_array(ts):
    arr = (C.c_void_p * len(ts))(*[t.data_ptr() if t is not None else None for t in ts])
    return arr


def layernorm_fwd_grouped(X, R, gammas, betas, eps, Y, mean, rstd):
    """Y[g] = LayerNorm(X[g] (+ R[g])) with (gammas[g], betas[g]) for the G groups of the stacked
    (G, rows, D) tensors in one launch; mean / rstd (G * rows).  False when the shape is not
    covered (nothing written: the caller runs the groups one by one)."""
    G, D = X.shape[0], X.shape[-1]
    rows = X[0].numel() // D
    ga, be = _ptr_array(gammas), _ptr_array(betas)
    rc = _lib.load().jmt_layernorm_fwd_grouped(
        dt(X), dt(Y), G, rows, D, X.data_ptr(), D, X[0].numel(),
        R.data_ptr() if R is not None else None, D, R[0].numel() if R is not None else 0,
        ga, be, eps, Y.data_ptr(), D, Y[0].numel(), mean.data_ptr(), rstd.data_ptr(), stream())
    if rc == _lib.ERR_UNSUPPORTED:
        return False
    _lib.check(rc, "jmt_layernorm_fwd_grouped")
    return True


def layernorm_bwd_grouped(X, R, dY, mean, rstd, gammas, dX, dgammas, dbetas, dsums, beta_acc):
    """Grouped jmt_layernorm_bwd(_dsum) over the stacked (G, rows, D) tensors: one launch + one
    reduce; dsums None or a list of column-sum outputs.  Returns the partials buffer (keep it
    alive until the launches are ordered) or None when the shape is not covered."""
    G, D = X.shape[0], X.shape[-1]
    rows = X[0].numel() // D
    nblk = _lib.load().jmt_layernorm_bwd_grouped_blocks(rows)
    ns = 3 if dsums is not None else 2
    part = torch.empty(max(nblk, 1) * ns * D * G, dtype=torch.float32, device=X.device)
    rc = _lib.load().jmt_layernorm_bwd_grouped(
        dt(X), dt(dY), dt(dX), G, rows, D, X.data_ptr(), D, X[0].numel(),
        R.data_ptr() if R is not None else None, D, R[0].numel() if R is not None else 0,
        dY.data_ptr(), D, dY[0].numel(), mean.data_ptr(), rstd.data_ptr(), _ptr_array(gammas),
        dX.data_ptr(), D, dX[0].numel(), _ptr_array(dgammas), _ptr_array(dbetas),
        _ptr_array(dsums) if dsums is not None else None, int(beta_acc), part.data_ptr(),
        stream())
    if rc == _lib.ERR_UNSUPPORTED:
        return None
    _lib.check(rc, "jmt_layernorm_bwd_grouped")
    return part


def softmax_fwd(s, lds, rows, n, scale, p, ldp):
    _lib.call("jmt_softmax_fwd", dt(p), rows, n, s.data_ptr(), lds, scale, p.data_ptr(), ldp,
              stream())


def softmax_bwd(p, ldp, dp, lddp, rows, n, scale, ds, ldds):
    _lib.call("jmt_softmax_bwd", dt(p), dt(ds), rows, n, p.data_ptr(), ldp, dp.data_ptr(), lddp,
              scale, ds.data_ptr(), ldds, stream())


_attn_fused = {"on": os.environ.get("JMT_ATTN_FUSED", "1") != "0"}


def attn_supported(dtype: int, dh: int) -> bool:
    return _attn_fused["on"] and bool(_lib.load().jmt_attn_supported(dtype, dh))


def _hooked(info, launch):
    if _launch_hook is not None:
        return _launch_hook(info, launch)
    return launch()


def noop():
    _lib.call("jmt_noop", stream())


def attn_fwd(dtype, N, H, Lq, Lk, dh, q_ptr, sq, k_ptr, sk, v_ptr, sv, o_ptr, so, scale, lse):
    """Fused softmax(scale Q K^T) V + lse; sq/sk/sv/so = (row stride, batch stride) in
    elements."""
    launch = lambda: _lib.call("jmt_attn_fwd", dtype, N, H, Lq, Lk, dh, q_ptr, sq[0], sq[1],
                               k_ptr, sk[0], sk[1], v_ptr, sv[0], sv[1], o_ptr, so[0], so[1],
                               scale, lse.data_ptr() if lse is not None else None, stream())
    es = 4 if dtype == F32 else 2
    _hooked({"family": "attn_fwd", "flops": 4.0 * N * H * Lq * Lk * dh,
             "bytes": float(N * H) * ((2 * Lq + 2 * Lk) * dh * es + 4 * Lq)}, launch)


def attn_bwd(dtype, N, H, Lq, Lk, dh, go_ptr, sgo, o_ptr, so, q_ptr, sq, k_ptr, sk, v_ptr, sv,
             lse, p, ds, ldp, dq_ptr, sdq, scale):
    """P = exp(scale Q K^T - lse) and dS = scale P o (dO V^T - rowsum(dO o O)) written to p / ds
    (ldp), dQ = dS K; dq_ptr None: P and dS only (the 128-row kernel; dQ from attn_dkdv)."""
    launch = lambda: _lib.call("jmt_attn_bwd", dtype, N, H, Lq, Lk, dh, go_ptr, sgo[0], sgo[1],
                               o_ptr, so[0], so[1], q_ptr, sq[0], sq[1], k_ptr, sk[0], sk[1],
                               v_ptr, sv[0], sv[1], lse.data_ptr(), p.data_ptr(), ds.data_ptr(),
                               ldp, dq_ptr, sdq[0], sdq[1], scale, stream())
    # algorithmic: two products per launch — dP and dQ, or (dq_ptr None) the S recompute and dP
    # (cdna_hip_programming.md counts the recompute as one of the backward's five products);
    # bytes: dO, O, Q, K, V, (dQ,) lse and the P / dS rows handed to attn_dkdv
    es = 4 if dtype == F32 else 2
    nrow = 3 if dq_ptr is None else 4
    lw = -(-Lk // 32) * 32 if dq_ptr is None else ldp     # P / dS columns written
    _hooked({"family": "attn_bwd", "flops": 4.0 * N * H * Lq * Lk * dh,
             "bytes": float(N * H) * ((nrow * Lq + 2 * Lk) * dh * es + 4 * Lq +
                                      2 * Lq * lw * es)}, launch)


_attn_dkdv = {"on": os.environ.get("JMT_ATTN_DKDV", "1") != "0"}
# the 128-row P / dS backward kernel with dQ as jmt_attn_dkdv's third product (round 6);
# JMT_ATTN_PDS=0 keeps dQ in the 64-row backward kernel (A/B switch)
_attn_pds = {"on": os.environ.get("JMT_ATTN_PDS", "1") != "0"}


def attn_pds_ok(Lq, Lk, sdq_l, sk_l, H) -> bool:
    """Host-side mirror of the dq = NULL checks of jmt_attn_bwd and the dQ checks of
    jmt_attn_dkdv: P / dS rows of attn_dkdv_ldp(Lk) with 32-bit offsets over Lq + 128 rows, a
    128-row dQ tile and Lk K rows within 32-bit byte offsets."""
    ldp = attn_dkdv_ldp(Lk)
    lim = 1 << 31
    return ((Lq + 128) * ldp * 2 < lim // 2 and sdq_l >= H * 512 and 128 * sdq_l * 2 < lim
            and Lk * sk_l * 2 < lim)


def attn_dkdv_ldp(Lk: int) -> int:
    """P / dS row stride jmt_attn_dkdv reads (whole 128-key tiles)."""
    return (Lk + 127) // 128 * 128


def attn_dkdv_ok(N, H, Lq, Lk, dh, sgo_l, sq_l, sdk_l, sdv_l) -> bool:
    """Host-side mirror of jmt_attn_dkdv's range checks (csrc/attn_dkdv.hip): 512-wide heads,
    32-bit row offsets of dO / Q / P (Lq rows < 2 GiB) and of a 128-row dK / dV tile, and the
    item count.  The caller takes the batched-GEMM dK / dV path when this says no."""
    ldp = attn_dkdv_ldp(Lk)
    lim = 1 << 31
    return (dh == 512 and sdk_l >= H * dh and sdv_l >= H * dh
            and 128 * sdk_l * 2 < lim and 128 * sdv_l * 2 < lim
            and N * H * 2 * (ldp // 128) < lim
            and Lq * sgo_l * 2 < lim and Lq * sq_l * 2 < lim and Lq * ldp * 2 < lim)


def attn_dkdv(dtype, N, H, Lq, Lk, dh, p, ds, ldp, go_ptr, sgo, q_ptr, sq, dk_ptr, sdk, dv_ptr,
              sdv, k_ptr=None, sk=(0, 0), dq_ptr=None, sdq=(0, 0)):
    """dV = P^T dO and dK = dS^T Q per (n, h) from attn_bwd's P / dS (ldp >= attn_dkdv_ldp(Lk));
    with dq_ptr also dQ = dS K (k_ptr: the attention's K operand); one persistent kernel in place
    of two (three) batched GEMMs (off with JMT_ATTN_DKDV=0)."""
    launch = lambda: _lib.call("jmt_attn_dkdv", dtype, N, H, Lq, Lk, dh, p.data_ptr(),
                               ds.data_ptr(), ldp, go_ptr, sgo[0], sgo[1], q_ptr, sq[0], sq[1],
                               k_ptr, sk[0], sk[1], dk_ptr, sdk[0], sdk[1], dv_ptr, sdv[0],
                               sdv[1], dq_ptr, sdq[0], sdq[1], stream())
    # algorithmic: the two (three) products; bytes: P, dS (128-key tiles), dO and Q read once per
    # head, dK and dV written (+ K read per 128-query tile, dS again (32-key chunks), dQ written)
    es = 4 if dtype == F32 else 2
    nprod = 2 if dq_ptr is None else 3
    extra = 0.0 if dq_ptr is None else (Lk + Lq) * dh * es + Lq * (-(-Lk // 32) * 32) * es
    _hooked({"family": "attn_dkdv", "flops": 2.0 * nprod * N * H * Lq * Lk * dh,
             "bytes": float(N * H) * ((2 * Lq + 2 * Lk) * dh * es +
                                      2 * Lq * attn_dkdv_ldp(Lk) * es + extra)}, launch)


def attn_short_ok(dtype: int, dh: int, Lq: int, Lk: int) -> bool:
    """Shapes the one-block-per-sequence fused kernels cover (jmt_attn_short_*: 16-bit, dh = 512,
    Lq, Lk <= 32); off with JMT_ATTN_FUSED=0 or JMT_ATTN_SHORT=0 (A/B switch)."""
    return (_attn_fused["on"] and _attn_short["on"] and
            bool(_lib.load().jmt_attn_short_supported(dtype, dh, Lq, Lk)))


_attn_short = {"on": os.environ.get("JMT_ATTN_SHORT", "1") != "0"}


def attn_short_fwd(dtype, N, H, Lq, Lk, dh, q_ptr, sq, k_ptr, sk, v_ptr, sv, o_ptr, so, scale,
                   lse):
    """jmt_attn_fwd's result (o, lse) for Lq, Lk <= 32: one block per (n, h)."""
    launch = lambda: _lib.call("jmt_attn_short_fwd", dtype, N, H, Lq, Lk, dh, q_ptr, sq[0], sq[1],
                               k_ptr, sk[0], sk[1], v_ptr, sv[0], sv[1], o_ptr, so[0], so[1],
                               scale, lse.data_ptr(), stream())
    es = 4 if dtype == F32 else 2
    _hooked({"family": "attn_short_fwd", "flops": 4.0 * N * H * Lq * Lk * dh,
             "bytes": float(N * H) * ((2 * Lq + 2 * Lk) * dh * es + 4 * Lq)}, launch)


def attn_short_bwd(dtype, N, H, Lq, Lk, dh, go_ptr, sgo, o_ptr, so, q_ptr, sq, k_ptr, sk, v_ptr,
                   sv, lse, dq_ptr, sdq, dk_ptr, sdk, dv_ptr, sdv, scale):
    """dQ, dK, dV of attn_short_fwd in one kernel (P recomputed from lse; no P / dS in HBM)."""
    launch = lambda: _lib.call("jmt_attn_short_bwd", dtype, N, H, Lq, Lk, dh, go_ptr, sgo[0],
                               sgo[1], o_ptr, so[0], so[1], q_ptr, sq[0], sq[1], k_ptr, sk[0],
                               sk[1], v_ptr, sv[0], sv[1], lse.data_ptr(), dq_ptr, sdq[0], sdq[1],
                               dk_ptr, sdk[0], sdk[1], dv_ptr, sdv[0], sdv[1], scale, stream())
    # algorithmic: dP, dQ, dK, dV (the P recompute is not counted); bytes: q, o, dO, k, v, lse
    # read, dq, dk, dv written
    es = 4 if dtype == F32 else 2
    _hooked({"family": "attn_short_bwd", "flops": 8.0 * N * H * Lq * Lk * dh,
             "bytes": float(N * H) * ((4 * Lq + 4 * Lk) * dh * es + 4 * Lq)}, launch)


SMALL_ATTN_MAX_L = 8


def small_attn_ok(E: int, H: int, Lq: int, Lk: int) -> bool:
    """Shapes jmt_small_attn_* cover (include/jmt.h): E = 512, E/8/H a power of two, L <= 8
    (off with the fused kernels: JMT_ATTN_FUSED=0 selects the GEMM + softmax path)."""
    g = E // 8 // H if H > 0 and E % (8 * H) == 0 else 0
    return (_attn_fused["on"] and E == 512 and g > 0 and (g & (g - 1)) == 0 and 1 <= Lq <= SMALL_ATTN_MAX_L
            and 1 <= Lk <= SMALL_ATTN_MAX_L)


def small_attn_fwd(dtype, N, H, Lq, Lk, E, q_ptr, sq, k_ptr, sk, v_ptr, sv, o_ptr, so, scale,
                   p):
    """O = softmax(scale Q K^T) V for Lq, Lk <= 8, one wave per sequence; p (fp32,
    N*H*Lq*Lk) keeps the probabilities for small_attn_bwd."""
    launch = lambda: _lib.call("jmt_small_attn_fwd", dtype, N, H, Lq, Lk, E, q_ptr, sq[0],
                               sq[1], k_ptr, sk[0], sk[1], v_ptr, sv[0], sv[1], o_ptr, so[0],
                               so[1], scale, p.data_ptr() if p is not None else None, stream())
    es = 4 if dtype == F32 else 2
    nbytes = float(N) * (2 * Lq + 2 * Lk) * E * es + (4.0 * N * H * Lq * Lk if p is not None
                                                       else 0.0)
    _hooked({"family": "small_attn_fwd", "flops": 4.0 * N * Lq * Lk * E, "bytes": nbytes},
            launch)


def small_attn_bwd(dtype, N, H, Lq, Lk, E, go_ptr, sgo, q_ptr, sq, k_ptr, sk, v_ptr, sv, p,
                   dq_ptr, sdq, dk_ptr, sdk, dv_ptr, sdv, scale):
    """dQ, dK, dV of small_attn_fwd from the kept P (no score recompute)."""
    launch = lambda: _lib.call("jmt_small_attn_bwd", dtype, N, H, Lq, Lk, E, go_ptr, sgo[0],
                               sgo[1], q_ptr, sq[0], sq[1], k_ptr, sk[0], sk[1], v_ptr, sv[0],
                               sv[1], p.data_ptr(), dq_ptr, sdq[0], sdq[1], dk_ptr, sdk[0],
                               sdk[1], dv_ptr, sdv[0], sdv[1], scale, stream())
    es = 4 if dtype == F32 else 2
    nbytes = float(N) * (3 * Lq + 4 * Lk) * E * es + 4.0 * N * H * Lq * Lk
    _hooked({"family": "small_attn_bwd", "flops": 8.0 * N * Lq * Lk * E, "bytes": nbytes},
            launch)


def colsum(dy, ld, rows, N, db, beta_acc=False):
    nblk = _lib.load().jmt_colsum_blocks(rows)
    part = torch.empty(max(nblk, 1) * N, dtype=torch.float32, device=dy.device)
    _lib.call("jmt_colsum", dt(dy), rows, N, dy.data_ptr(), ld, db.data_ptr(), int(beta_acc),
              part.data_ptr(), stream())
    return part


def colsum_grouped(dy_ptr: int, dtype: int, G: int, ld: int, sdy: int, rows: int, N: int,
                   dbs, beta_acc=True, device=None):
    """db_g (+)= column sums of the g-th (rows x N) block at dy_ptr + g*sdy, one launch pair."""
    nblk = _lib.load().jmt_colsum_blocks(rows)
    part = torch.empty(max(nblk, 1) * N * G, dtype=torch.float32, device=device)
    tab = (C.c_void_p * 8)(*[d.data_ptr() for d in dbs])
    _lib.call("jmt_colsum_grouped", dtype, G, rows, N, dy_ptr, ld, sdy, tab, int(beta_acc),
              part.data_ptr(), stream())
    return part


def copy2d(src_ptr, src_dt, dst_ptr, dst_dt, rows, cols, src_rs, src_cs, dst_rs, dst_cs,
           accumulate=False):
    _lib.call("jmt_copy2d", src_dt, dst_dt, rows, cols, src_ptr, src_rs, src_cs, dst_ptr, dst_rs,
              dst_cs, int(accumulate), stream())


def cast(src: torch.Tensor, dtype: torch.dtype, out: Optional[torch.Tensor] = None):
    """Contiguous dtype conversion through jmt_copy2d (weight shadows, label upcasts)."""
    _require_cuda(src)
    src = src if src.is_contiguous() else src.contiguous()
    if out is None:
        out = torch.empty(src.shape, dtype=dtype, device=src.device)
    n = src.numel()
    copy2d(src.data_ptr(), dt(src), out.data_ptr(), dt(out), 1, n, n, 1, n, 1)
    return out


# ------------------------------------------------------------------------------------ CCC

def ccc_stats(kind, pred, label, k, ignore, lo, hi, stats):
    n = label.numel()
    _lib.call("jmt_ccc_stats", kind, dt(pred), n, k, pred.data_ptr(), label.data_ptr(), ignore,
              lo, hi, stats.data_ptr(), stream())


def ccc_finish(kind, world, stats_all, bs, eps, loss, coef, add=None):
    """add (fp32 scalar tensor or None): loss = add + this loss, in the same kernel."""
    if add is None:
        _lib.call("jmt_ccc_finish", kind, world, stats_all.data_ptr(), bs, eps, loss.data_ptr(),
                  coef.data_ptr(), stream())
    else:
        _lib.call("jmt_ccc_finish_add", kind, world, stats_all.data_ptr(), bs, eps,
                  add.data_ptr(), loss.data_ptr(), coef.data_ptr(), stream())


HEAD_HID, HEAD_KMAX = 128, 24      # csrc/head.hip


def head_fwd(h, ldh, rows, k, w2, b2, ys, ldy):
    """Both regressors' output layers (csrc/head.hip jmt_head_fwd)."""
    p = lambda t: t.data_ptr() if t is not None else None
    _lib.call("jmt_head_fwd", dt(h), dt(ys[0]), rows, HEAD_HID, k, h.data_ptr(), ldh,
              w2[0].data_ptr(), w2[1].data_ptr(), p(b2[0]), p(b2[1]), ys[0].data_ptr(),
              ys[1].data_ptr(), ldy, stream())


def head_bwd(h, ldh, rows, k, w2, gys, ldgy, dh, lddh, dw2, db2):
    """dh (ReLU-masked) and += weight / bias gradients of both output layers (jmt_head_bwd)."""
    p = lambda t: t.data_ptr() if t is not None else None
    nbytes = _lib.load().jmt_head_bwd_workspace_bytes(rows)
    ws = torch.empty(max(1, nbytes // 4), dtype=torch.float32, device=h.device)
    _lib.call("jmt_head_bwd", dt(h), dt(gys[0]), rows, HEAD_HID, k, h.data_ptr(), ldh,
              w2[0].data_ptr(), w2[1].data_ptr(), gys[0].data_ptr(), gys[1].data_ptr(), ldgy,
              dh.data_ptr(), lddh, p(dw2[0]), p(dw2[1]), p(db2[0]), p(db2[1]), ws.data_ptr(),
              stream())


def ce_stats(x, label, k, lo, hi, weights, stats):
    n = x.numel() // k
    _lib.call("jmt_ce_stats", dt(x), n, k, x.data_ptr(), label.data_ptr(), lo, hi,
              weights.data_ptr() if weights is not None else None, stats.data_ptr(), stream())


def ce_finish(world, stats_all, loss, coef):
    _lib.call("jmt_ce_finish", world, stats_all.data_ptr(), loss.data_ptr(), coef.data_ptr(),
              stream())


def ce_bwd(x, label, k, lo, hi, weights, coef, grad_loss, dx):
    n = x.numel() // k
    _lib.call("jmt_ce_bwd", dt(x), n, k, x.data_ptr(), label.data_ptr(), lo, hi,
              weights.data_ptr() if weights is not None else None, coef.data_ptr(),
              grad_loss.data_ptr() if grad_loss is not None else None, dx.data_ptr(), stream())


def ce_labels(label, k, lo, hi):
    out = torch.empty(label.numel(), dtype=torch.int64, device=label.device)
    _lib.call("jmt_ce_labels", label.numel(), k, label.data_ptr(), lo, hi, out.data_ptr(),
              stream())
    return out


def ccc_bwd(kind, pred, label, k, ignore, lo, hi, coef, grad_loss, dpred):
    n = label.numel()
    _lib.call("jmt_ccc_bwd", kind, dt(pred), n, k, pred.data_ptr(), label.data_ptr(), ignore, lo,
              hi, coef.data_ptr(), grad_loss.data_ptr() if grad_loss is not None else None,
              dpred.data_ptr(), stream())


def mask_indices(label: torch.Tensor, ignore: float):
    n = label.numel()
    idx = torch.empty(max(n, 1), dtype=torch.int64, device=label.device)
    cnt = torch.empty(1, dtype=torch.int64, device=label.device)
    _lib.call("jmt_mask_indices", n, label.data_ptr(), ignore, idx.data_ptr(), cnt.data_ptr(),
              stream())
    return idx, cnt


# ------------------------------------------------------------------------------------ SGD

def sgd_step(param, grad, buf, lr, momentum, dampening, weight_decay, nesterov, first,
             grad_scale=1.0, shadow=None, zero_grad=False):
    """zero_grad: grad is zeroed by the same kernel after it is read (jmt_sgd_step_zero)."""
    _lib.call("jmt_sgd_step_zero" if zero_grad else "jmt_sgd_step", param.numel(),
              param.data_ptr(), grad.data_ptr(),
              buf.data_ptr() if buf is not None else None, lr, momentum, dampening, weight_decay,
              int(nesterov), int(first), grad_scale,
              shadow.data_ptr() if shadow is not None else None,
              dt(shadow) if shadow is not None else BF16, stream())
