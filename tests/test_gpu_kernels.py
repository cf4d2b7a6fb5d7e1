"""Kernel-level numerics on the MI355X: every HIP kernel vs a plain PyTorch fp32 reference of the
same op (computed from the same, already-rounded inputs), through the C-ABI."""
import math
import os

import pytest
import torch

from jmt import functional as JF
from jmt import ops
from jmt._lib import BF16, F16, F32

pytestmark = pytest.mark.gpu
DEV = "cuda"
TD = {F32: torch.float32, BF16: torch.bfloat16, F16: torch.float16}


def _rup(a, b):
    return -(-a // b) * b


def _tol(dt, K):
    # fp32: exact-f32 MFMA chain; 16-bit: inputs exact, fp32 accumulate -> only order effects
    return 2e-5 * math.sqrt(max(K, 1)) if dt == F32 else 2e-4 * math.sqrt(max(K, 1))


def _operand(rows, cols, kmajor_rows, dt, batch=1, gen=None):
    """Logical X[b] (rows x cols) stored row-major with padded ld if kmajor_rows, else stored
    transposed (cols x rows) with padded ld.  Returns (storage, logical_fp32, ld, batch_stride)."""
    t = TD[dt]
    if kmajor_rows:
        ld = _rup(cols, 8) + 8
        st = torch.randn(batch, rows, ld, device=DEV, generator=gen).to(t)
        logical = st[:, :, :cols].float()
    else:
        ld = _rup(rows, 8) + 8
        st = torch.randn(batch, cols, ld, device=DEV, generator=gen).to(t)
        logical = st[:, :, :rows].float().transpose(1, 2)
    return st, logical, ld, st.stride(0)


SHAPES = [(128, 128, 64), (300, 300, 512), (37, 53, 300), (19, 1, 128), (1, 128, 37),
          (200, 72, 130), (256, 512, 1024)]


@pytest.mark.parametrize("dt", [F32, BF16, F16])
@pytest.mark.parametrize("ak", [True, False])
@pytest.mark.parametrize("bk", [True, False])
def test_gemm_layouts_dtypes(dt, ak, bk):
    g = torch.Generator(device=DEV).manual_seed(1)
    for (M, N, K) in SHAPES:
        A, Al, lda, sa = _operand(M, K, ak, dt, gen=g)
        # B logical K x N; "b_kmajor" = stored [N][K]
        Bs, Bl_t, ldb, sb = _operand(N, K, bk, dt, gen=g)
        Bl = Bl_t.transpose(1, 2)
        C = torch.full((M, N + 3), float("nan"), device=DEV)
        ops.gemm(M=M, N=N, K=K, ab_dtype=dt, c_dtype=F32, a=[A.data_ptr()], lda=lda, a_kmajor=ak,
                 b=[Bs.data_ptr()], ldb=ldb, b_kmajor=bk, c=[C.data_ptr()], ldc=N + 3,
                 splits=1, device=DEV)
        ref = Al[0] @ Bl[0]
        err = (C[:, :N] - ref).abs().max().item()
        assert err <= _tol(dt, K) * max(1.0, ref.abs().max().item()), (M, N, K, err)
        assert torch.isnan(C[:, N:]).all(), "wrote outside N"


@pytest.mark.parametrize("cfg", [1, 5, 10, 11, 20, 21, 32])
@pytest.mark.parametrize("ak,bk", [(True, True), (True, False), (False, True), (False, False)])
def test_gemm_forced_configs(cfg, ak, bk):
    """Every tile configuration of the planner forced on every operand layout (bf16), on ragged
    shapes (partial tiles, trailing partial K-tile), a K-concatenated A and a pointer-table
    batch: the interleaved-DMA configs (20, 21) keep three K-tiles in flight."""
    from jmt import _lib
    lib = _lib.load()
    dt = BF16
    g = torch.Generator(device=DEV).manual_seed(5)
    lib.jmt_gemm_set_debug(cfg << 8)
    try:
        for (M, N, K) in [(300, 520, 512), (257, 129, 320), (64, 64, 1000), (1, 300, 96)]:
            A, Al, lda, sa = _operand(M, K, ak, dt, batch=2, gen=g)
            Bs, Bl_t, ldb, sb = _operand(N, K, bk, dt, batch=2, gen=g)
            Bl = Bl_t.transpose(1, 2)
            C = torch.full((2, M, N + 3), float("nan"), device=DEV)
            ops.gemm(M=M, N=N, K=K, ab_dtype=dt, c_dtype=F32, a=[A.data_ptr()], lda=lda,
                     a_kmajor=ak, sA=(sa, 0), b=[Bs[i].data_ptr() for i in range(2)], ldb=ldb,
                     b_kmajor=bk, b_mode=1, c=[C.data_ptr()], ldc=N + 3, sC=(M * (N + 3), 0),
                     batch0=2, splits=1, device=DEV)
            for i in range(2):
                ref = Al[i] @ Bl[i]
                err = (C[i, :, :N] - ref).abs().max().item()
                assert err <= _tol(dt, K) * max(1.0, ref.abs().max().item()), (cfg, M, N, K, err)
            assert torch.isnan(C[:, :, N:]).all(), "wrote outside N"
        if ak:   # K-concat A (3 segments of 128) x K-major / MN-major B, bf16 out
            M, N, seg = 333, 256, 128
            As = [torch.randn(M, seg, device=DEV, generator=g).bfloat16() for _ in range(3)]
            Bs2, Bl_t2, ldb2, _ = _operand(N, 3 * seg, bk, dt, gen=g)
            C = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
            ops.gemm(M=M, N=N, K=3 * seg, ab_dtype=dt, c_dtype=dt, a=[a.data_ptr() for a in As],
                     lda=seg, a_kmajor=True, a_mode=2, a_kseg=seg, b=[Bs2.data_ptr()], ldb=ldb2,
                     b_kmajor=bk, c=[C.data_ptr()], ldc=N, splits=1, device=DEV)
            ref = torch.cat([a.float() for a in As], 1) @ Bl_t2.transpose(1, 2)[0]
            err = (C.float() - ref).abs().max().item()
            assert err <= 1e-2 * ref.abs().max().item(), (cfg, "kcat", err)
    finally:
        lib.jmt_gemm_set_debug(0)


@pytest.mark.parametrize("dt", [F32, BF16])
def test_gemm_epilogues_and_splitk(dt):
    g = torch.Generator(device=DEV).manual_seed(2)
    M, N, K = 333, 200, 1000
    A, Al, lda, _ = _operand(M, K, True, dt, gen=g)
    Bs, Bl_t, ldb, _ = _operand(N, K, True, dt, gen=g)
    Bl = Bl_t.transpose(1, 2)[0]
    base = Al[0] @ Bl
    bias = torch.randn(N, device=DEV, generator=g)
    biasr = torch.randn(M, device=DEV, generator=g)
    for splits in (1, 4):
        # bias per column + relu, out in the ab dtype
        C = torch.empty(M, N, device=DEV, dtype=TD[dt])
        ops.gemm(M=M, N=N, K=K, ab_dtype=dt, c_dtype=dt, a=[A.data_ptr()], lda=lda, a_kmajor=True,
                 b=[Bs.data_ptr()], ldb=ldb, b_kmajor=True, c=[C.data_ptr()], ldc=N,
                 bias=bias, bias_mode=1, relu=True, splits=splits, device=DEV)
        ref = torch.relu(base + bias)
        tol = _tol(dt, K) * ref.abs().max().item() + (0 if dt == F32 else 8e-3 * ref.abs().max().item())
        assert (C.float() - ref).abs().max().item() <= tol
        # alpha, row bias, beta accumulate into fp32
        C0 = torch.randn(M, N, device=DEV, generator=g)
        C = C0.clone()
        ops.gemm(M=M, N=N, K=K, ab_dtype=dt, c_dtype=F32, a=[A.data_ptr()], lda=lda, a_kmajor=True,
                 b=[Bs.data_ptr()], ldb=ldb, b_kmajor=True, c=[C.data_ptr()], ldc=N,
                 alpha=0.5, beta=1.0, bias=biasr, bias_mode=2, splits=splits, device=DEV)
        ref = 0.5 * base + biasr[:, None] + C0
        assert (C - ref).abs().max().item() <= _tol(dt, K) * ref.abs().max().item()
        # aux mask (ReLU backward): zero where aux <= 0
        aux = torch.randn(M, N, device=DEV, generator=g)      # the mask has the output dtype
        C = torch.empty(M, N, device=DEV)
        ops.gemm(M=M, N=N, K=K, ab_dtype=dt, c_dtype=F32, a=[A.data_ptr()], lda=lda, a_kmajor=True,
                 b=[Bs.data_ptr()], ldb=ldb, b_kmajor=True, c=[C.data_ptr()], ldc=N, aux=aux,
                 ldaux=N, splits=splits, device=DEV)
        ref = torch.where(aux > 0, base, torch.zeros_like(base))
        assert (C - ref).abs().max().item() <= _tol(dt, K) * base.abs().max().item()


@pytest.mark.parametrize("dt", [F32, BF16])
def test_gemm_batched_two_level_strides(dt):
    """attention-shaped: S[n,h] = Q[n,h] K[n,h]^T on seq-first (L, N, H*dh) packed buffers."""
    g = torch.Generator(device=DEV).manual_seed(3)
    L, Nb, H, dh = 45, 3, 4, 64
    t = TD[dt]
    qkv = torch.randn(Nb, L, 3 * H * dh, device=DEV, generator=g).to(t)   # (N, L, 3E) memory
    E = H * dh
    S = torch.empty(Nb, H, L, 48, device=DEV)
    ops.gemm(M=L, N=L, K=dh, ab_dtype=dt, c_dtype=F32,
             a=[qkv.data_ptr()], lda=3 * E, a_kmajor=True, sA=(L * 3 * E, dh),
             b=[qkv.data_ptr() + E * qkv.element_size()], ldb=3 * E, b_kmajor=True,
             sB=(L * 3 * E, dh), c=[S.data_ptr()], ldc=48, sC=(H * L * 48, L * 48),
             batch0=Nb, batch1=H, device=DEV)
    q = qkv[..., :E].float().view(Nb, L, H, dh).permute(0, 2, 1, 3)
    k = qkv[..., E:2 * E].float().view(Nb, L, H, dh).permute(0, 2, 1, 3)
    ref = q @ k.transpose(-1, -2)
    assert (S[..., :L] - ref).abs().max().item() <= _tol(dt, dh) * ref.abs().max().item()


@pytest.mark.parametrize("dt", [F32, BF16])
def test_gemm_kconcat_and_pointer_tables(dt):
    g = torch.Generator(device=DEV).manual_seed(4)
    t = TD[dt]
    M, seg, nseg, N = 150, 64 if dt == BF16 else 32, 6, 96
    xs = [torch.randn(M, seg, device=DEV, generator=g).to(t) for _ in range(nseg)]
    W = torch.randn(N, seg * nseg, device=DEV, generator=g).to(t)
    C = torch.empty(M, N, device=DEV)
    ops.gemm(M=M, N=N, K=seg * nseg, ab_dtype=dt, c_dtype=F32, a=[x.data_ptr() for x in xs],
             lda=seg, a_kmajor=True, a_mode=2, a_kseg=seg, b=[W.data_ptr()], ldb=seg * nseg,
             b_kmajor=True, c=[C.data_ptr()], ldc=N, device=DEV)
    ref = torch.cat([x.float() for x in xs], 1) @ W.float().t()
    assert (C - ref).abs().max().item() <= _tol(dt, seg * nseg) * ref.abs().max().item()
    # dgrad-style: outs[s] = dY @ W[:, s] with a C pointer table and B batch stride
    dY = torch.randn(M, N, device=DEV, generator=g).to(t)
    outs = [torch.empty(M, seg, device=DEV) for _ in range(nseg)]
    ops.gemm(M=M, N=seg, K=N, ab_dtype=dt, c_dtype=F32, a=[dY.data_ptr()], lda=N, a_kmajor=True,
             b=[W.data_ptr()], ldb=seg * nseg, b_kmajor=False, c=[o.data_ptr() for o in outs],
             ldc=seg, c_mode=1, batch0=nseg, sB=(seg, 0), device=DEV)
    full = dY.float() @ W.float()
    for s in range(nseg):
        r = full[:, s * seg:(s + 1) * seg]
        assert (outs[s] - r).abs().max().item() <= _tol(dt, N) * full.abs().max().item()
    # wgrad-style: dW[:, s] += dY^T X_s with a B pointer table, split-K over M
    dW = torch.randn(N, seg * nseg, device=DEV, generator=g)
    dW0 = dW.clone()
    ops.gemm(M=N, N=seg, K=M, ab_dtype=dt, c_dtype=F32, a=[dY.data_ptr()], lda=N, a_kmajor=False,
             b=[x.data_ptr() for x in xs], ldb=seg, b_kmajor=False, b_mode=1,
             c=[dW.data_ptr()], ldc=seg * nseg, batch0=nseg, sC=(seg, 0), beta=1.0, splits=3,
             device=DEV)
    ref = dW0 + dY.float().t() @ torch.cat([x.float() for x in xs], 1)
    assert (dW - ref).abs().max().item() <= _tol(dt, M) * ref.abs().max().item()


def _kernel_names(fn):
    """Names of the device kernels fn() launches (torch.profiler; None if it records none)."""
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        fn()
        torch.cuda.synchronize()
    names = [e.name for e in prof.events() if e.device_type == torch.autograd.DeviceType.CUDA]
    return names or None


@pytest.mark.parametrize("ak,bk", [(True, True), (True, False), (False, True), (False, False)])
def test_gemm_pp_partial_row_panel(ak, bk):
    """cfg 45 (ping-pong persistent GEMM) with M % 256 != 0 (round 6: c2's 9,600 rows): the last
    row panel's A rows are clamped and its stores go through a buffer resource ending at row M.
    vs torch fp32 for the plain / bias-table + ReLU / beta * C / ReLU-mask epilogues, batched with
    guard rows between the entries' C blocks that must stay untouched, dbg 32 bit-identical, and
    the default plan takes the ping-pong kernel for such a shape (kernel name via torch.profiler)."""
    from jmt import _lib
    lib = _lib.load()
    g = torch.Generator(device=DEV).manual_seed(45)
    bf = torch.bfloat16
    GUARD = 40                           # rows of sentinel after each entry's M rows
    for (M, N, K, nb) in [(9600, 512, 512, 2), (1000, 768, 256, 3), (264, 256, 128, 1)]:
        A, Al, lda, sa = _operand(M, K, ak, BF16, batch=nb, gen=g)
        Bs, Bl_t, ldb, sb = _operand(N, K, bk, BF16, batch=nb, gen=g)
        Bl = Bl_t.transpose(1, 2)
        bias = [torch.randn(N, device=DEV, generator=g) for _ in range(nb)]
        C0 = torch.randn(nb, M + GUARD, N, device=DEV, generator=g).to(bf)
        aux = torch.randn(nb, M + GUARD, N, device=DEV, generator=g).to(bf)
        for form in ("bias_relu", "beta", "mask"):
            kw = dict(M=M, N=N, K=K, ab_dtype=BF16, c_dtype=BF16, a=[A.data_ptr()], lda=lda,
                      a_kmajor=ak, sA=(sa, 0), b=[Bs.data_ptr()], ldb=ldb, b_kmajor=bk,
                      sB=(sb, 0), ldc=N, sC=((M + GUARD) * N, 0), batch0=nb, splits=1,
                      device=DEV)
            if form == "bias_relu":
                kw.update(alpha=0.75, bias_tab=bias, bias_mode=1, relu=True)
            elif form == "beta":
                kw.update(beta=0.5)
            else:
                kw.update(aux=aux, ldaux=N)
            outs = []
            for dbg in (0, 32):
                C = C0.clone()
                lib.jmt_gemm_set_debug((45 << 8) | dbg)
                try:
                    ops.gemm(c=[C.data_ptr()], **kw)
                finally:
                    lib.jmt_gemm_set_debug(0)
                outs.append(C)
            assert torch.equal(outs[0], outs[1]), (M, form, "dbg 32 changed the result")
            C = outs[0]
            assert torch.equal(C[:, M:], C0[:, M:]), (M, form, "stores past row M")
            for i in range(nb):
                ref = Al[i] @ Bl[i]
                if form == "bias_relu":
                    ref = torch.relu(0.75 * ref + bias[i])
                elif form == "beta":
                    ref = ref + 0.5 * C0[i, :M].float()
                else:
                    ref = torch.where(aux[i, :M].float() > 0, ref, torch.zeros_like(ref))
                err = (C[i, :M].float() - ref).abs().max().item()
                assert err <= 1e-2 * ref.abs().max().item(), (M, N, K, form, i, err)
    # the default plan: a 9,600-row launch of >= 128 tiles runs on the ping-pong kernel
    M, N, K, nb = 9600, 512, 512, 2
    A, Al, lda, sa = _operand(M, K, ak, BF16, batch=nb, gen=g)
    Bs, Bl_t, ldb, sb = _operand(N, K, bk, BF16, batch=nb, gen=g)
    Bl = Bl_t.transpose(1, 2)
    C = torch.empty(nb, M, N, device=DEV, dtype=bf)
    names = _kernel_names(lambda: ops.gemm(
        M=M, N=N, K=K, ab_dtype=BF16, c_dtype=BF16, a=[A.data_ptr()], lda=lda, a_kmajor=ak,
        sA=(sa, 0), b=[Bs.data_ptr()], ldb=ldb, b_kmajor=bk, sB=(sb, 0), c=[C.data_ptr()],
        ldc=N, sC=(M * N, 0), batch0=nb, device=DEV))
    if names is not None:
        assert any("gemm_pp2_kernel" in n for n in names), names
    ref = torch.bmm(Al, Bl.contiguous())
    assert (C.float() - ref).abs().max().item() <= 1e-2 * ref.abs().max().item()


@pytest.mark.parametrize("cfg", [40, 43, 45])
@pytest.mark.parametrize("ak,bk", [(True, True), (True, False), (False, True), (False, False)])
def test_gemm_persistent(cfg, ak, bk):
    """gemm_persist_kernel (csrc/gemm_persist.hip: one block per CU walks whole 256x256 tiles
    with one LDS-DMA pipeline across tile boundaries, stores drained under the next tile's
    MFMAs) vs torch fp32: more tiles than CUs (2-4 tiles per block, uneven), batched with bias
    tables, a K-concatenated A, C pointer tables, ReLU / alpha / per-column bias, K down to two
    K-tiles (the store window then spans a whole tile); and dbg 32 (every wait also drains the
    last epilogue's stores) bit-identical."""
    from jmt import _lib
    lib = _lib.load()
    g = torch.Generator(device=DEV).manual_seed(40)
    bf = torch.bfloat16

    def run(**kw):
        out = []
        for dbg in (0, 32):
            lib.jmt_gemm_set_debug((cfg << 8) | dbg)
            try:
                ops.gemm(device=DEV, **{k: v for k, v in kw.items() if k != "c"},
                         c=[t.data_ptr() for t in kw["c"]])
            finally:
                lib.jmt_gemm_set_debug(0)
            out.append([t.clone() for t in kw["c"]])
        for a, b in zip(*out):
            assert torch.equal(a, b), "dbg 32 (stores drained at every wait) changed the result"
        return out[0]

    for (M, N, K, nb) in [(10240, 512, 256, 4), (512, 1536, 128, 3), (2304, 256, 512, 1)]:
        A, Al, lda, sa = _operand(M, K, ak, BF16, batch=nb, gen=g)
        Bs, Bl_t, ldb, sb = _operand(N, K, bk, BF16, batch=nb, gen=g)
        Bl = Bl_t.transpose(1, 2)
        bias = [torch.randn(N, device=DEV, generator=g) for _ in range(nb)]
        C = torch.empty(nb, M, N, device=DEV, dtype=bf)
        (C2,) = run(M=M, N=N, K=K, ab_dtype=BF16, c_dtype=BF16, a=[A.data_ptr()], lda=lda,
                    a_kmajor=ak, sA=(sa, 0), b=[Bs.data_ptr()], ldb=ldb, b_kmajor=bk,
                    sB=(sb, 0), c=[C], ldc=N, sC=(M * N, 0), batch0=nb, alpha=0.75,
                    bias_tab=bias, bias_mode=1, relu=True, splits=1)
        for i in range(nb):
            ref = torch.relu(0.75 * (Al[i] @ Bl[i]) + bias[i])
            err = (C2[i].float() - ref).abs().max().item()
            assert err <= 1e-2 * ref.abs().max().item(), (cfg, M, N, K, i, err)
    # beta * C and the ReLU-backward mask (aux > 0) epilogue forms (the stacked-stream / FFN
    # dgrads): C accumulates, the mask zeroes
    M, N, K, nb = 4608, 512, 256, 3
    A, Al, lda, sa = _operand(M, K, ak, BF16, batch=nb, gen=g)
    Bs, Bl_t, ldb, sb = _operand(N, K, bk, BF16, batch=nb, gen=g)
    Bl = Bl_t.transpose(1, 2)
    C0 = torch.randn(nb, M, N, device=DEV, generator=g).to(bf)
    aux = torch.randn(nb, M, N, device=DEV, generator=g).to(bf)
    for beta, use_aux in ((1.0, False), (0.0, True), (0.5, True)):
        C = C0.clone()
        outs = []                    # (beta accumulates: each execution starts from C0)
        for dbg in (0, 32):
            C.copy_(C0)
            lib.jmt_gemm_set_debug((cfg << 8) | dbg)
            try:
                ops.gemm(M=M, N=N, K=K, ab_dtype=BF16, c_dtype=BF16, a=[A.data_ptr()], lda=lda,
                         a_kmajor=ak, sA=(sa, 0), b=[Bs.data_ptr()], ldb=ldb, b_kmajor=bk,
                         sB=(sb, 0), c=[C.data_ptr()], ldc=N, sC=(M * N, 0), batch0=nb,
                         beta=beta, aux=aux if use_aux else None, ldaux=N, splits=1, device=DEV)
            finally:
                lib.jmt_gemm_set_debug(0)
            outs.append(C.clone())
        assert torch.equal(outs[0], outs[1])
        for i in range(nb):
            ref = Al[i] @ Bl[i] + beta * C0[i].float()
            if use_aux:
                ref = torch.where(aux[i].float() > 0, ref, torch.zeros_like(ref))
            err = (outs[0][i].float() - ref).abs().max().item()
            assert err <= 1e-2 * ref.abs().max().item(), (cfg, beta, use_aux, i, err)
    if ak:
        # K-concat A (4 segments of 128) x (K-major | MN-major) B into a C pointer table of two
        # (batch1-strided) outputs, one bias for every batch entry
        M, N, seg = 1536, 512, 128
        As = [torch.randn(M, seg, device=DEV, generator=g).to(bf) for _ in range(4)]
        Bs2, Bl_t2, ldb2, sb2 = _operand(N, 4 * seg, bk, BF16, batch=2, gen=g)
        bias = torch.randn(N, device=DEV, generator=g)
        outs = [torch.empty(M, N, device=DEV, dtype=bf) for _ in range(2)]
        res = run(M=M, N=N, K=4 * seg, ab_dtype=BF16, c_dtype=BF16, a=[a.data_ptr() for a in As],
                  lda=seg, a_kmajor=True, a_mode=2, a_kseg=seg, b=[Bs2.data_ptr()], ldb=ldb2,
                  b_kmajor=bk, sB=(sb2, 0), c=outs, c_mode=1, ldc=N, batch0=2, bias=bias,
                  bias_mode=1, splits=1)
        Acat = torch.cat([a.float() for a in As], 1)
        for i in range(2):
            ref = Acat @ Bl_t2.transpose(1, 2)[i] + bias
            err = (res[i].float() - ref).abs().max().item()
            assert err <= 1e-2 * ref.abs().max().item(), (cfg, "kcat", i, err)


@pytest.mark.parametrize("ak,bk", [(True, True), (True, False), (False, True), (False, False)])
def test_gemm_pingpong_bit_identical_to_persistent(ak, bk):
    """The ping-pong persistent kernel (cfg 43: two wave groups one barrier apart, LDS-DMA
    pieces on a counted-vmcnt schedule, the epilogue in two halves) accumulates every output in
    the same k order as cfg 40: bit-identical C on step shapes with several items per block
    (item boundaries inside the DMA stream), beta * C, the ReLU mask, bias tables — repeated
    launches (a missed wait shows as a difference that comes and goes).  Also cfg 45, the same
    schedule with one 32-MFMA phase per k-half (half the barriers per K-tile)."""
    from jmt import _lib
    lib = _lib.load()
    g = torch.Generator(device=DEV).manual_seed(43)
    bf = torch.bfloat16
    for (M, N, K, nb, beta, use_aux) in [(19200, 1024, 512, 2, 0.0, False),
                                         (19200, 512, 1024, 2, 1.0, False),
                                         (7680, 768, 192, 3, 0.0, True),
                                         (4096, 512, 128, 5, 0.5, True)]:
        A, Al, lda, sa = _operand(M, K, ak, BF16, batch=nb, gen=g)
        Bs, Bl_t, ldb, sb = _operand(N, K, bk, BF16, batch=nb, gen=g)
        bias = [torch.randn(N, device=DEV, generator=g) for _ in range(nb)]
        C0 = torch.randn(nb, M, N, device=DEV, generator=g).to(bf)
        aux = torch.randn(nb, M, N, device=DEV, generator=g).to(bf) if use_aux else None
        outs = {}
        for cfg in (40, 43, 43, 43, 45, 45, 45):
            C = C0.clone()
            lib.jmt_gemm_set_debug(cfg << 8)
            try:
                ops.gemm(M=M, N=N, K=K, ab_dtype=BF16, c_dtype=BF16, a=[A.data_ptr()], lda=lda,
                         a_kmajor=ak, sA=(sa, 0), b=[Bs.data_ptr()], ldb=ldb, b_kmajor=bk,
                         sB=(sb, 0), c=[C.data_ptr()], ldc=N, sC=(M * N, 0), batch0=nb,
                         bias_tab=bias, bias_mode=1, beta=beta, aux=aux, ldaux=N, splits=1,
                         device=DEV)
            finally:
                lib.jmt_gemm_set_debug(0)
            outs.setdefault(cfg, []).append(C)
        for cfg in (43, 45):
            for C in outs[cfg]:
                assert torch.equal(C, outs[40][0]), (cfg, M, N, K, nb, beta, use_aux,
                                                     int((C != outs[40][0]).sum()))
        ref = (Al[0] @ Bl_t.transpose(1, 2)[0]) + bias[0] + beta * C0[0].float()
        if use_aux:
            ref = torch.where(aux[0].float() > 0, ref, torch.zeros_like(ref))
        err = (outs[43][0][0].float() - ref).abs().max().item()
        assert err <= 1e-2 * ref.abs().max().item(), (M, N, K, err)


def test_gemm_large_bf16_linear_shape():
    """The benchmark's dominant shape: (19200 x 1024) @ (1024 x 512)^T in bf16."""
    g = torch.Generator(device=DEV).manual_seed(5)
    X = torch.randn(19200, 1024, device=DEV, generator=g).bfloat16()
    W = torch.randn(512, 1024, device=DEV, generator=g).bfloat16()
    Y = torch.empty(19200, 512, device=DEV, dtype=torch.bfloat16)
    ops.gemm(M=19200, N=512, K=1024, ab_dtype=BF16, c_dtype=BF16, a=[X.data_ptr()], lda=1024,
             a_kmajor=True, b=[W.data_ptr()], ldb=1024, b_kmajor=True, c=[Y.data_ptr()], ldc=512,
             device=DEV)
    ref = X.float() @ W.float().t()
    rel = ((Y.float() - ref).abs().max() / ref.abs().max()).item()
    assert rel < 1e-2


@pytest.mark.parametrize("cd", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("D", [2048, 512, 768])      # vector kernels (NV 8, 2) and the loop form
def test_l2norm_fwd_bwd(cd, D):
    g = torch.Generator(device=DEV).manual_seed(6)
    x = torch.randn(5, 37, D, device=DEV, generator=g)
    x[0, 0] = 0.0                                      # the eps-clamped branch
    x.requires_grad_(True)
    with JF.compute_mode(cd):
        y = JF.l2_normalize(x)
        gy = torch.randn(y.shape, device=DEV, generator=g).to(cd)
        y.backward(gy)
    xr = x.detach().clone().requires_grad_(True)
    yr = torch.nn.functional.normalize(xr, dim=-1)
    yr.backward(gy.float())
    tol = 1e-6 if cd == torch.float32 else 1e-2
    assert (y.float() - yr).abs().max().item() <= tol * yr.abs().max().item() + 1e-7
    assert (x.grad - xr.grad).abs().max().item() <= tol * xr.grad.abs().max().item() + 1e-7


@pytest.mark.parametrize("cd", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("D", [512, 768])
def test_add_layernorm_fwd_bwd(cd, D):
    g = torch.Generator(device=DEV).manual_seed(7)
    x = (torch.randn(300, 7, D, device=DEV, generator=g) * 3 + 1).to(cd).requires_grad_(True)
    r = torch.randn(300, 7, D, device=DEV, generator=g).to(cd).requires_grad_(True)
    gam = torch.nn.Parameter(1 + 0.1 * torch.randn(D, device=DEV, generator=g))
    bet = torch.nn.Parameter(0.1 * torch.randn(D, device=DEV, generator=g))
    with JF.compute_mode(cd):
        y = JF.add_layer_norm(x, r, gam, bet, 1e-5)
    gy = torch.randn(y.shape, device=DEV, generator=g).to(cd)
    y.backward(gy)
    xr = x.detach().float().requires_grad_(True)
    rr = r.detach().float().requires_grad_(True)
    g2 = gam.detach().clone().requires_grad_(True)
    b2 = bet.detach().clone().requires_grad_(True)
    yr = torch.nn.functional.layer_norm(xr + rr, (D,), g2, b2, 1e-5)
    yr.backward(gy.float())
    tol = 2e-5 if cd == torch.float32 else 2e-2
    assert (y.float() - yr).abs().max().item() <= tol * yr.abs().max().item()
    assert (x.grad.float() - xr.grad).abs().max().item() <= tol * xr.grad.abs().max().item()
    assert (r.grad.float() - rr.grad).abs().max().item() <= tol * rr.grad.abs().max().item()
    assert (gam.grad - g2.grad).abs().max().item() <= tol * g2.grad.abs().max().item()
    assert (bet.grad - b2.grad).abs().max().item() <= tol * b2.grad.abs().max().item()


@pytest.mark.parametrize("cd", [torch.bfloat16, torch.float16])
def test_layernorm_bwd_16b_rows_match_8b_rows(cd):
    """Round 6: at D = 512 with 16-bit operands and 16-B aligned rows the LayerNorm backward
    maps 8 consecutive elements to a lane (one 16-B access per row and operand); rows whose
    stride is only a multiple of 4 (here 516) keep the 8-B mapping.  Same data through both:
    dgamma / dbeta bit-identical (same row order per element), dx within one rounding of the
    compute dtype (the row sums s1, s2 reassociate), both vs torch fp32."""
    g = torch.Generator(device=DEV).manual_seed(11)
    rows, D = 1000, 512
    X = (torch.randn(rows, D, device=DEV, generator=g) * 2 + 0.5).to(cd)
    R = torch.randn(rows, D, device=DEV, generator=g).to(cd)
    dY = torch.randn(rows, D, device=DEV, generator=g).to(cd)
    gam = 1 + 0.1 * torch.randn(D, device=DEV, generator=g)
    bet = 0.1 * torch.randn(D, device=DEV, generator=g)

    def padded(t):
        b = torch.zeros(rows, D + 4, device=DEV, dtype=t.dtype)
        b[:, :D] = t
        return b

    Y = torch.empty_like(X)
    st = torch.empty(2, rows, device=DEV)
    ops.layernorm_fwd(X, D, R, D, gam, bet, 1e-5, Y, D, st[0], st[1], rows, D)
    outs = []
    for pad in (False, True):
        x, r, dy = (padded(t) if pad else t for t in (X, R, dY))
        ld = D + 4 if pad else D
        dx = torch.zeros(rows, ld, device=DEV, dtype=cd)
        dg = torch.zeros(D, device=DEV)
        db = torch.zeros(D, device=DEV)
        ops.layernorm_bwd(x, ld, r, ld, dy, ld, st[0], st[1], gam, dx, ld, dg, db, True, rows, D)
        torch.cuda.synchronize()
        outs.append((dx[:, :D].clone(), dg, db))
    (a, b) = outs
    assert torch.equal(a[1], b[1]) and torch.equal(a[2], b[2])
    xr = (X.float() + R.float()).requires_grad_(True)
    g2 = gam.clone().requires_grad_(True)
    b2 = bet.clone().requires_grad_(True)
    torch.nn.functional.layer_norm(xr, (D,), g2, b2, 1e-5).backward(dY.float())
    scale = xr.grad.abs().max().item()
    for dx, dg, _ in outs:
        assert (dx.float() - xr.grad).abs().max().item() <= 2e-2 * scale
        assert (dg - g2.grad).abs().max().item() <= 2e-2 * g2.grad.abs().max().item()
    assert (a[0].float() - b[0].float()).abs().max().item() <= 1e-2 * scale


@pytest.mark.parametrize("cd", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("H,Lq,Lk,N", [(1, 300, 300, 3), (8, 37, 37, 2), (1, 1, 6, 40),
                                       (4, 64, 17, 5)])
def test_attention_core_fwd_bwd(cd, H, Lq, Lk, N):
    """q/k/v as slices of packed projections in a (N, L, *) memory layout (seq-first views)."""
    g = torch.Generator(device=DEV).manual_seed(8)
    E = 512 if H in (1, 4) else 256
    qsrc = torch.randn(N, Lq, E, device=DEV, generator=g).to(cd).permute(1, 0, 2)
    kv = torch.randn(N, Lk, 2 * E, device=DEV, generator=g).to(cd).permute(1, 0, 2)
    qsrc.requires_grad_(True)
    kv.requires_grad_(True)
    with JF.compute_mode(cd):
        o = JF.AttnCoreFn.apply(qsrc, kv, kv, E, H, 0, 0, E)
    go = torch.randn(o.shape, device=DEV, generator=g).to(cd)
    o.backward(go)
    dh = E // H
    qr = qsrc.detach().float().requires_grad_(True)
    kvr = kv.detach().float().requires_grad_(True)
    q = qr.reshape(Lq, N * H, dh).transpose(0, 1) / math.sqrt(dh)
    k = kvr[..., :E].reshape(Lk, N * H, dh).transpose(0, 1)
    v = kvr[..., E:].reshape(Lk, N * H, dh).transpose(0, 1)
    ref = (torch.softmax(q @ k.transpose(1, 2), -1) @ v).transpose(0, 1).reshape(Lq, N, E)
    ref.backward(go.float())
    tol = 5e-5 if cd == torch.float32 else 3e-2
    assert (o.float() - ref).abs().max().item() <= tol * ref.abs().max().item()
    assert (qsrc.grad.float() - qr.grad).abs().max().item() <= tol * qr.grad.abs().max().item()
    assert (kv.grad.float() - kvr.grad).abs().max().item() <= tol * kvr.grad.abs().max().item()


@pytest.mark.parametrize("cd", [torch.float32, torch.bfloat16])
def test_linear_mlp_autograd(cd):
    """Fused MLP fwd/bwd vs a torch reference that rounds the same intermediates to the compute
    dtype (x, W, h and dh are stored in `cd` by the HIP path; accumulation is fp32)."""
    g = torch.Generator(device=DEV).manual_seed(9)
    x = torch.randn(40, 3, 1024, device=DEV, generator=g).permute(1, 0, 2).requires_grad_(True)
    W1 = torch.nn.Parameter(torch.randn(128, 1024, device=DEV, generator=g) * 0.03)
    b1 = torch.nn.Parameter(torch.randn(128, device=DEV, generator=g) * 0.1)
    W2 = torch.nn.Parameter(torch.randn(1, 128, device=DEV, generator=g) * 0.1)
    b2 = torch.nn.Parameter(torch.randn(1, device=DEV, generator=g) * 0.1)
    with JF.compute_mode(cd):
        y = JF.mlp(x, W1, b1, W2, b2, out_dtype=torch.float32)
    gy = torch.randn(y.shape, device=DEV, generator=g)
    y.backward(gy)
    r = lambda t: t.to(cd).float()
    xr, W1r, W2r = r(x.detach()), r(W1.detach()), r(W2.detach())
    h = r(torch.relu(xr @ W1r.t() + b1.detach()))
    yr = h @ W2r.t() + b2.detach()
    gyr = r(gy)
    dh = r((gyr @ W2r) * (h > 0))
    ref = {"y": yr, "x": dh @ W1r, "W1": (dh.reshape(-1, 128).t() @ xr.reshape(-1, 1024)),
           "b1": dh.reshape(-1, 128).sum(0), "W2": gyr.reshape(-1, 1).t() @ h.reshape(-1, 128),
           "b2": gyr.reshape(-1).sum().reshape(1)}
    got = {"y": y, "x": x.grad, "W1": W1.grad, "b1": b1.grad, "W2": W2.grad, "b2": b2.grad}
    tol = 3e-5 if cd == torch.float32 else 1e-2     # bf16: the final dx rounding (2^-8)
    assert y.shape == yr.shape
    for k in ref:
        err = (got[k].float() - ref[k]).abs().max().item()
        assert err <= tol * ref[k].abs().max().item() + 1e-6, (k, err)


def test_softmax_rows_and_padding():
    g = torch.Generator(device=DEV).manual_seed(10)
    S = torch.randn(50, 304, device=DEV, generator=g) * 4
    P = torch.full((50, 304), 7.0, device=DEV, dtype=torch.bfloat16)
    ops.softmax_fwd(S, 304, 50, 300, 0.5, P, 304)
    ref = torch.softmax(S[:, :300] * 0.5, -1)
    assert (P[:, :300].float() - ref).abs().max().item() < 4e-3
    assert (P[:, 300:] == 0).all()


def test_colsum_and_copy2d():
    g = torch.Generator(device=DEV).manual_seed(11)
    dy = torch.randn(19201, 96, device=DEV, generator=g).bfloat16()
    db = torch.ones(96, device=DEV)
    ops.colsum(dy, 96, 19201, 96, db, beta_acc=True)
    ref = 1 + dy.float().sum(0)
    assert (db - ref).abs().max().item() < 1e-3
    x = torch.randn(37, 5, device=DEV, generator=g)
    y = torch.empty(5, 37, device=DEV, dtype=torch.bfloat16)
    ops.copy2d(x.data_ptr(), F32, y.data_ptr(), BF16, 37, 5, 5, 1, 1, 37)
    assert (y.float() - x.t().bfloat16().float()).abs().max().item() == 0


@pytest.mark.parametrize("N,ld", [(1, 1), (3, 5), (64, 64)])
def test_colsum_narrow(N, ld):
    """Narrow column sums (the regressor output biases): small-N kernel, ragged row count."""
    g = torch.Generator(device=DEV).manual_seed(13)
    dy = torch.randn(19201, ld, device=DEV, generator=g).bfloat16()
    db = torch.zeros(N, device=DEV)
    ops.colsum(dy, ld, 19201, N, db, beta_acc=False)
    ref = dy[:, :N].float().sum(0)
    assert (db - ref).abs().max().item() < 1e-3


def test_sgd_matches_torch_nesterov():
    g = torch.Generator(device=DEV).manual_seed(12)
    p = torch.randn(10007, device=DEV, generator=g)
    p_ref = p.clone().requires_grad_(True)
    opt = torch.optim.SGD([p_ref], lr=1e-2, momentum=0.9, dampening=0.0, weight_decay=1e-4,
                          nesterov=True)
    buf = torch.zeros_like(p)
    shadow = torch.empty(10007, device=DEV, dtype=torch.bfloat16)
    for step in range(3):
        gr = torch.randn(10007, device=DEV, generator=g)
        ops.sgd_step(p, gr * 2.0, buf, 1e-2, 0.9, 0.0, 1e-4, True, step == 0, 0.5, shadow)
        p_ref.grad = gr.clone()
        opt.step()
    assert (p - p_ref.detach()).abs().max().item() < 1e-6
    assert (shadow.float() - p.bfloat16().float()).abs().max().item() == 0


@pytest.mark.parametrize("cd", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("Lq,Lk,N", [(300, 300, 3), (1, 6, 40), (6, 6, 17), (70, 129, 2),
                                     (64, 64, 1), (129, 1, 2), (1024, 1024, 2),
                                     # more (n, q-tile) items than CUs: the persistent grid
                                     (300, 300, 64), (70, 129, 200), (129, 1, 300)])
def test_fused_attention_fwd_vs_fp32(cd, Lq, Lk, N):
    """jmt_attn_fwd (attn.hip) on packed self/cross-attention layouts vs softmax(QK^T/sqrt(d))V
    in fp32 from the same rounded inputs; the log-sum-exp against torch.logsumexp."""
    E = H_DIM = 512
    if not ops.attn_supported(ops.dt(torch.empty(0, dtype=cd)), H_DIM):
        pytest.skip("fused attention not built for this dtype")
    g = torch.Generator(device=DEV).manual_seed(21)
    q = torch.randn(N, Lq, 3 * E, device=DEV, generator=g).to(cd).permute(1, 0, 2)   # (Lq,N,3E)
    kv = torch.randn(N, Lk, 2 * E, device=DEV, generator=g).to(cd).permute(1, 0, 2)
    o = torch.full((Lq, N, E), float("nan"), device=DEV, dtype=cd)
    lse = torch.empty(N * Lq, device=DEV, dtype=torch.float32)
    scale = 1.0 / math.sqrt(E)
    qp, kp, vp = q[..., E:2 * E], kv[..., :E], kv[..., E:]
    ops.attn_fwd(ops.dt(q), N, 1, Lq, Lk, E, qp.data_ptr(), (q.stride(0), q.stride(1)),
                 kp.data_ptr(), (kv.stride(0), kv.stride(1)), vp.data_ptr(),
                 (kv.stride(0), kv.stride(1)), o.data_ptr(), (o.stride(0), o.stride(1)), scale,
                 lse)
    torch.cuda.synchronize()
    s = torch.einsum("lnd,knd->nlk", qp.float(), kp.float()) * scale
    ref = torch.einsum("nlk,knd->lnd", torch.softmax(s, -1), vp.float())
    err = (o.float() - ref).abs().max().item()
    assert torch.isfinite(o.float()).all()
    # P is rounded to the compute dtype before the PV product (as torch's 16-bit attention)
    tol = (1e-2 if cd == torch.bfloat16 else 2e-3) * max(ref.abs().max().item(), 1.0)
    assert err <= tol, err
    lref = torch.logsumexp(s, -1).reshape(-1)
    assert (lse - lref).abs().max().item() <= 1e-3 * max(lref.abs().max().item(), 1.0)


@pytest.mark.parametrize("pds", [False, True])
@pytest.mark.parametrize("cd", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("Lq,Lk,N", [(300, 300, 3), (1, 6, 40), (70, 129, 2), (129, 1, 2),
                                     (1024, 1024, 1), (257, 33, 3),
                                     # more (n, q-tile) items than CUs: the persistent grid
                                     (300, 300, 64), (70, 129, 200), (129, 1, 300)])
def test_fused_attention_bwd_vs_fp32(cd, Lq, Lk, N, pds):
    """jmt_attn_bwd (attn.hip): P recomputed from the forward's lse, dS and dQ vs an fp32
    reference from the same rounded inputs (P and dS are stored in the compute dtype; the
    padding columns [Lk, ldp) of P and dS must be written as zeros).  pds: dq = NULL, the
    128-row P / dS kernel (round 6): the padding columns up to the 32-key tile are zeros, the
    rest of the row and the dq buffer stay untouched."""
    E = 512
    g = torch.Generator(device=DEV).manual_seed(23)
    qkv = torch.randn(N, Lq, 3 * E, device=DEV, generator=g).to(cd).permute(1, 0, 2)
    kv = torch.randn(N, Lk, 2 * E, device=DEV, generator=g).to(cd).permute(1, 0, 2)
    qp, kp, vp = qkv[..., :E], kv[..., :E], kv[..., E:]
    scale = 1.0 / math.sqrt(E)
    dt = ops.dt(qkv)
    o = torch.empty(Lq, N, E, device=DEV, dtype=cd)
    lse = torch.empty(N * Lq, device=DEV, dtype=torch.float32)
    ops.attn_fwd(dt, N, 1, Lq, Lk, E, qp.data_ptr(), (qkv.stride(0), qkv.stride(1)),
                 kp.data_ptr(), (kv.stride(0), kv.stride(1)), vp.data_ptr(),
                 (kv.stride(0), kv.stride(1)), o.data_ptr(), (o.stride(0), o.stride(1)), scale,
                 lse)
    go = torch.randn(Lq, N, E, device=DEV, generator=g).to(cd)
    ldp = ops.attn_dkdv_ldp(Lk) if pds else -(-Lk // 8) * 8
    P = torch.full((N * Lq * ldp,), float("nan"), device=DEV, dtype=cd)
    dS = torch.full((N * Lq * ldp,), float("nan"), device=DEV, dtype=cd)
    dq = torch.full((N, Lq, 3 * E), float("nan"), device=DEV, dtype=cd).permute(1, 0, 2)
    ops.attn_bwd(dt, N, 1, Lq, Lk, E, go.data_ptr(), (go.stride(0), go.stride(1)), o.data_ptr(),
                 (o.stride(0), o.stride(1)), qp.data_ptr(), (qkv.stride(0), qkv.stride(1)),
                 kp.data_ptr(), (kv.stride(0), kv.stride(1)), vp.data_ptr(),
                 (kv.stride(0), kv.stride(1)), lse, P, dS, ldp,
                 None if pds else dq[..., E:2 * E].data_ptr(), (dq.stride(0), dq.stride(1)),
                 scale)
    torch.cuda.synchronize()
    s = torch.einsum("lnd,knd->nlk", qp.float(), kp.float()) * scale
    pr = torch.softmax(s, -1)
    dp = torch.einsum("lnd,knd->nlk", go.float(), vp.float())
    delta = (go.float() * o.float()).sum(-1).t().unsqueeze(-1)           # (N, Lq, 1)
    dsr = pr * (dp - delta) * scale
    dqr = torch.einsum("nlk,knd->lnd", dsr, kp.float())
    if pds:     # tile-major hand-off: (n, key tile, query, 32 keys) -> (n, query, key)
        Pg = P.view(N, ldp // 32, Lq, 32).permute(0, 2, 1, 3).reshape(N, Lq, ldp)
        dSg = dS.view(N, ldp // 32, Lq, 32).permute(0, 2, 1, 3).reshape(N, Lq, ldp)
    else:
        Pg = P.view(N, Lq, ldp)
        dSg = dS.view(N, Lq, ldp)
    lw = -(-Lk // 32) * 32 if pds else ldp        # columns the kernel writes
    assert torch.isfinite(Pg[..., :lw].float()).all() and torch.isfinite(dSg[..., :lw].float()).all()
    assert (Pg[..., Lk:lw] == 0).all() and (dSg[..., Lk:lw] == 0).all()
    assert torch.isnan(Pg[..., lw:].float()).all() and torch.isnan(dSg[..., lw:].float()).all()
    u = 2.0 ** -8 if cd == torch.bfloat16 else 2.0 ** -11
    assert (Pg[..., :Lk].float() - pr).abs().max().item() <= 2 * u
    # dS error floor: Delta = rowsum(dO o O) from the 16-bit O (the cancellation dP - Delta is
    # exact zero at Lk = 1)
    floor = 4 * u * scale * dp.abs().max().item()
    e_ds = (dSg[..., :Lk].float() - dsr).abs().max().item()
    assert e_ds <= 8 * u * dsr.abs().max().item() + floor, e_ds
    if pds:
        assert torch.isnan(dq.float()).all()
        return
    e_dq = (dq[..., E:2 * E].float() - dqr).abs().max().item()
    assert e_dq <= 16 * u * dqr.abs().max().item() + floor * kp.float().abs().max().item(), e_dq
    assert torch.isnan(dq[..., :E].float()).all() and torch.isnan(dq[..., 2 * E:].float()).all()


@pytest.mark.parametrize("with_dq", [False, True])
@pytest.mark.parametrize("cd", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("Lq,Lk,N,H", [(300, 300, 3, 1), (1024, 1024, 1, 1), (77, 130, 2, 2),
                                       (33, 20, 3, 1), (1, 65, 2, 1), (129, 1, 2, 1),
                                       (300, 45, 2, 1),
                                       # more (n, h, key-tile) items than CUs: persistent grid
                                       (300, 300, 64, 2), (40, 200, 100, 1)])
def test_attn_dkdv_vs_fp32(cd, Lq, Lk, N, H, with_dq):
    """jmt_attn_dkdv (attn_dkdv.hip): dV = P^T dO and dK = dS^T Q per (n, h) vs fp32 products of
    the same 16-bit inputs.  P / dS columns past Lk hold NaN (they may feed only keys that are
    not stored), outputs land in a packed (Lk, N, 3 E) buffer whose other columns must stay
    untouched, and the ragged query / key tails cover the clamped rows and the dropped stores.
    with_dq (ABI 7): also dQ = dS K (its third product: 128-query items, 32-key chunks, NaN in
    the dS columns past Lk masked) into the first columns of a packed (Lq, N, 3 E) buffer."""
    E = 512 * H
    g = torch.Generator(device=DEV).manual_seed(31)
    ldp = ops.attn_dkdv_ldp(Lk)
    P = torch.full((N * H, Lq, ldp), float("nan"), device=DEV, dtype=cd)
    dS = torch.full((N * H, Lq, ldp), float("nan"), device=DEV, dtype=cd)
    P[..., :Lk] = torch.rand(N * H, Lq, Lk, device=DEV, generator=g).to(cd)
    dS[..., :Lk] = (torch.randn(N * H, Lq, Lk, device=DEV, generator=g) * 0.1).to(cd)
    qkv = torch.randn(N, Lq, 3 * E, device=DEV, generator=g).to(cd).permute(1, 0, 2)
    go = torch.randn(Lq, N, E, device=DEV, generator=g).to(cd)
    qv = qkv[..., :E]
    out = torch.full((N, Lk, 3 * E), 7.0, device=DEV, dtype=cd).permute(1, 0, 2)
    dk, dv = out[..., E:2 * E], out[..., 2 * E:]
    kk = torch.randn(N, Lk, 2 * E, device=DEV, generator=g).to(cd).permute(1, 0, 2)
    kv_ = kk[..., E:]
    dqo = torch.full((N, Lq, 3 * E), 7.0, device=DEV, dtype=cd).permute(1, 0, 2)
    dq = dqo[..., :E]
    st = lambda t: (t.stride(0), t.stride(1))
    # with dq: the tile-major P / dS layout of jmt_attn_bwd(dq = NULL)
    tiled = lambda t: t.view(N * H, Lq, ldp // 32, 32).permute(0, 2, 1, 3).contiguous()
    ops.attn_dkdv(ops.dt(qkv), N, H, Lq, Lk, 512, tiled(P) if with_dq else P,
                  tiled(dS) if with_dq else dS, ldp, go.data_ptr(), st(go),
                  qv.data_ptr(), st(qkv), dk.data_ptr(), st(out), dv.data_ptr(), st(out),
                  *((kv_.data_ptr(), st(kk), dq.data_ptr(), st(dqo)) if with_dq else ()))
    torch.cuda.synchronize()
    Pr = P[..., :Lk].float().view(N, H, Lq, Lk)
    dSr = dS[..., :Lk].float().view(N, H, Lq, Lk)
    gor = go.float().view(Lq, N, H, 512)
    qr = qv.float().reshape(Lq, N, H, 512)
    dvr = torch.einsum("nhqk,qnhd->knhd", Pr, gor).reshape(Lk, N, E)
    dkr = torch.einsum("nhqk,qnhd->knhd", dSr, qr).reshape(Lk, N, E)
    u = 2.0 ** -8 if cd == torch.bfloat16 else 2.0 ** -11
    for got, ref in ((dv, dvr), (dk, dkr)):
        assert torch.isfinite(got.float()).all()
        err = (got.float() - ref).abs().max().item()
        # fp32 accumulation of Lq products; the result rounded once to 16 bits
        assert err <= 2 * u * ref.abs().max().item() + 1e-6 * Lq, (err, ref.abs().max().item())
    assert (out[..., :E].float() == 7.0).all()
    if with_dq:
        kr = kv_.float().reshape(Lk, N, H, 512)
        dqr = torch.einsum("nhqk,knhd->qnhd", dSr, kr).reshape(Lq, N, E)
        assert torch.isfinite(dq.float()).all()
        err = (dq.float() - dqr).abs().max().item()
        assert err <= 2 * u * dqr.abs().max().item() + 1e-6 * Lk, (err, dqr.abs().max().item())
        assert (dqo[..., E:].float() == 7.0).all()
    else:
        assert (dqo.float() == 7.0).all()


@pytest.mark.parametrize("Lq,Lk,N", [(300, 300, 4), (70, 129, 3)])
def test_attention_backward_dkdv_matches_gemm_path(Lq, Lk, N):
    """functional.attn_backward: the jmt_attn_dkdv path (default) and the two-GEMM path
    (JMT_ATTN_DKDV=0) give the same dQ and agree on dK / dV within fp32-accumulation noise
    (the same rounded P / dS feed both)."""
    from jmt import functional as F
    cd = torch.bfloat16
    E, H = 512, 1
    g = torch.Generator(device=DEV).manual_seed(32)
    qkv = torch.randn(N, Lq, 3 * E, device=DEV, generator=g).to(cd).permute(1, 0, 2)
    kv = torch.randn(N, Lk, 2 * E, device=DEV, generator=g).to(cd).permute(1, 0, 2)
    F.set_compute_dtype(cd)
    try:
        o, saved = F.attn_forward(qkv, kv, kv, E, H, 0, 0, E)
    finally:
        F.set_compute_dtype(None)
    go = torch.randn(Lq, N, E, device=DEV, generator=g).to(cd)
    res = []
    for on, pds in ((True, False), (False, False), (True, True)):
        ops._attn_dkdv["on"] = on
        ops._attn_pds["on"] = pds
        try:
            dq = torch.zeros(N, Lq, 3 * E, device=DEV, dtype=cd).permute(1, 0, 2)
            dkv = torch.zeros(N, Lk, 2 * E, device=DEV, dtype=cd).permute(1, 0, 2)
            F.attn_backward(saved, go, dq, dkv, dkv)
            torch.cuda.synchronize()
            res.append((dq.float().clone(), dkv.float().clone()))
        finally:
            ops._attn_dkdv["on"] = True
            ops._attn_pds["on"] = True
    assert torch.equal(res[0][0], res[1][0])
    ref = res[1][1]
    err = (res[0][1] - ref).abs().max().item()
    assert err <= 2 * 2.0 ** -8 * ref.abs().max().item(), err
    # the 128-row P / dS kernel + dQ in attn_dkdv (default): its P / dS sum Delta and the scores
    # in another order, so dQ / dK / dV agree within the 16-bit rounding of P and dS
    for a, b in ((res[2][0], res[1][0]), (res[2][1], res[1][1])):
        err = (a - b).abs().max().item()
        assert err <= 4 * 2.0 ** -8 * b.abs().max().item(), err


def test_attention_backward_dkdv_out_of_range_stride_takes_gemm_path():
    """a dK / dV row stride beyond jmt_attn_dkdv's 32-bit tile offsets (128 rows x
    stride x 2 B >= 2 GiB) is caught by ops.attn_dkdv_ok and the backward takes the batched-GEMM
    dK / dV path (bit-identical to JMT_ATTN_DKDV=0) instead of raising."""
    from jmt import functional as F
    cd = torch.bfloat16
    E, H, N, Lq, Lk = 512, 1, 1, 70, 129
    sl = (1 << 23) + 1024                       # 128 * sl * 2 B > 2 GiB
    assert not ops.attn_dkdv_ok(N, H, Lq, Lk, E, 3 * E, 3 * E, sl, sl)
    assert ops.attn_dkdv_ok(N, H, Lq, Lk, E, 3 * E, 3 * E, 2 * E, 2 * E)
    g = torch.Generator(device=DEV).manual_seed(33)
    qkv = torch.randn(N, Lq, 3 * E, device=DEV, generator=g).to(cd).permute(1, 0, 2)
    kv = torch.randn(N, Lk, 2 * E, device=DEV, generator=g).to(cd).permute(1, 0, 2)
    F.set_compute_dtype(cd)
    try:
        o, saved = F.attn_forward(qkv, kv, kv, E, H, 0, 0, E)
    finally:
        F.set_compute_dtype(None)
    go = torch.randn(Lq, N, E, device=DEV, generator=g).to(cd)
    big = torch.zeros((Lk - 1) * sl + 2 * E, device=DEV, dtype=cd)
    res = []
    for on in (True, False):
        ops._attn_dkdv["on"] = on
        try:
            dq = torch.zeros(N, Lq, 3 * E, device=DEV, dtype=cd).permute(1, 0, 2)
            big.zero_()
            dkv = big.as_strided((Lk, N, 2 * E), (sl, sl * Lk, 1))
            F.attn_backward(saved, go, dq, dkv, dkv)
            torch.cuda.synchronize()
            res.append((dq.float().clone(), dkv.float().clone()))
        finally:
            ops._attn_dkdv["on"] = True
    del big
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])
    assert res[0][1].abs().max().item() > 0


def test_fused_attention_forced_rescale():
    """The lazy-rescale branch of the forward (a row max rising > 8 log2 units after the first
    tile) must be exact: one key in the third 64-key tile is spiked to dominate one query row
    (cdna_hip_programming.md §5.4 rule 26)."""
    cd = torch.bfloat16
    E, L, N = 512, 300, 2
    g = torch.Generator(device=DEV).manual_seed(24)
    q = torch.randn(N, L, E, device=DEV, generator=g) * 0.3
    k = torch.randn(N, L, E, device=DEV, generator=g) * 0.3
    v = torch.randn(N, L, E, device=DEV, generator=g)
    k[0, 150] = q[0, 7] * 8.0           # tile 2 of row 7: score jump >> 8 (log2 units)
    k[1, 299] = q[1, 63] * 8.0          # last (partial) tile
    q, k, v = (t.to(cd).permute(1, 0, 2).contiguous() for t in (q, k, v))
    o = torch.empty(L, N, E, device=DEV, dtype=cd)
    lse = torch.empty(N * L, device=DEV, dtype=torch.float32)
    scale = 1.0 / math.sqrt(E)
    ops.attn_fwd(ops.dt(q), N, 1, L, L, E, q.data_ptr(), (q.stride(0), q.stride(1)),
                 k.data_ptr(), (k.stride(0), k.stride(1)), v.data_ptr(), (v.stride(0), v.stride(1)),
                 o.data_ptr(), (o.stride(0), o.stride(1)), scale, lse)
    torch.cuda.synchronize()
    s = torch.einsum("lnd,knd->nlk", q.float(), k.float()) * scale
    ref = torch.einsum("nlk,knd->lnd", torch.softmax(s, -1), v.float())
    assert (o.float() - ref).abs().max().item() <= 2e-2 * ref.abs().max().item()
    assert (o[7, 0].float() - v[150, 0].float()).abs().max().item() <= 2e-2
    lref = torch.logsumexp(s, -1).reshape(-1)
    assert (lse - lref).abs().max().item() <= 1e-3 * lref.abs().max().item()


def test_fused_attention_matches_unfused_path():
    """AttnCoreFn with the fused kernel vs the GEMM + softmax path (JMT_ATTN_FUSED=0)."""
    cd = torch.bfloat16
    g = torch.Generator(device=DEV).manual_seed(22)
    N, L, E = 4, 300, 512
    x = torch.randn(N, L, 3 * E, device=DEV, generator=g).to(cd).permute(1, 0, 2)
    outs = []
    for fused in (True, False):
        ops._attn_fused["on"] = fused
        try:
            xx = x.detach().clone().requires_grad_(True)
            with JF.compute_mode(cd):
                o = JF.AttnCoreFn.apply(xx, xx, xx, E, 1, 0, E, 2 * E)
            o.backward(torch.ones_like(o))
            outs.append((o.float(), xx.grad.float()))
        finally:
            ops._attn_fused["on"] = True
    (o1, g1), (o2, g2) = outs
    assert (o1 - o2).abs().max().item() <= 1e-2 * o2.abs().max().item()
    assert (g1 - g2).abs().max().item() <= 2e-2 * g2.abs().max().item()


@pytest.mark.parametrize("splits", [1, 3])
def test_gemm_grouped_bias_table_16bit_beta_aux(splits):
    """Grouped launch (jmt/grouped.py): per-batch weight pointers + per-batch bias table, a 16-bit
    output with beta=1 accumulate and the ReLU-backward aux mask (vector epilogue loads)."""
    g = torch.Generator(device=DEV).manual_seed(21)
    G, M, N, K = 3, 301, 136, 192
    A = torch.randn(G, M, K, device=DEV, generator=g).bfloat16()
    Ws = [torch.randn(N, K, device=DEV, generator=g).bfloat16() for _ in range(G)]
    bs = [torch.randn(N, device=DEV, generator=g) for _ in range(G)]
    C0 = torch.randn(G, M, N, device=DEV, generator=g).bfloat16()
    aux = torch.randn(G, M, N, device=DEV, generator=g).bfloat16()
    C = C0.clone()
    ops.gemm(M=M, N=N, K=K, ab_dtype=BF16, c_dtype=BF16, a=[A.data_ptr()], lda=K, a_kmajor=True,
             sA=(M * K, 0), b=[w.data_ptr() for w in Ws], ldb=K, b_kmajor=True, b_mode=1,
             c=[C.data_ptr()], ldc=N, sC=(M * N, 0), batch0=G, beta=1.0, bias_tab=bs,
             bias_mode=1, aux=aux, ldaux=N, splits=splits, device=DEV)
    for i in range(G):
        base = A[i].float() @ Ws[i].float().t() + bs[i] + C0[i].float()
        ref = torch.where(aux[i].float() > 0, base, torch.zeros_like(base))
        err = (C[i].float() - ref).abs().max().item()
        assert err <= 2e-2 * max(1.0, ref.abs().max().item()), (i, err)


def test_colsum_grouped():
    g = torch.Generator(device=DEV).manual_seed(12)
    G, R, N = 3, 19201, 96
    dy = torch.randn(G, R, N, device=DEV, generator=g).bfloat16()
    dbs = [torch.full((N,), float(i), device=DEV) for i in range(G)]
    ops.colsum_grouped(dy.data_ptr(), BF16, G, N, R * N, R, N, dbs, beta_acc=True, device=DEV)
    torch.cuda.synchronize()
    for i in range(G):
        ref = i + dy[i].float().sum(0)
        assert (dbs[i] - ref).abs().max().item() < 1e-3


def _small_ref(q, k, v, H, scale):
    """fp32 softmax(scale Q K^T) V over (L, N, E) views; returns O (Lq, N, E) and P (N,H,Lq,Lk)."""
    Lq, N, E = q.shape
    Lk = k.shape[0]
    dh = E // H
    qh = q.reshape(Lq, N * H, dh).transpose(0, 1)
    kh = k.reshape(Lk, N * H, dh).transpose(0, 1)
    vh = v.reshape(Lk, N * H, dh).transpose(0, 1)
    p = torch.softmax(scale * qh @ kh.transpose(1, 2), -1)
    return (p @ vh).transpose(0, 1).reshape(Lq, N, E), p.reshape(N, H, Lq, Lk)


@pytest.mark.parametrize("dt", [F32, BF16, F16])
@pytest.mark.parametrize("H,Lq,Lk,N", [(1, 6, 6, 300), (1, 1, 6, 1000), (1, 2, 2, 77),
                                       (1, 1, 2, 50), (8, 8, 8, 33), (8, 3, 5, 10), (1, 1, 1, 5),
                                       (64, 4, 7, 9)])
def test_small_attn_kernels_vs_fp32(dt, H, Lq, Lk, N):
    """jmt_small_attn_fwd / _bwd (small_attn.hip) on q/k/v slices of packed projections in a
    (N, L, *) memory layout (seq-first strided views, as the SELF_ATTEN head and intra-modal
    fusion hand them over), against an fp32 torch reference on the same (16-bit-exact) inputs:
    the kernels compute in fp32, so the only 16-bit error is the final rounding (<= 1 ulp)."""
    cd = TD[dt]
    E = 512
    g = torch.Generator(device=DEV).manual_seed(100 + H + Lq * 8 + Lk)
    pad = 64                                     # columns nobody may touch
    if Lq == Lk:                                 # self-attention: one packed qkv
        x = (2 * torch.randn(N, Lq, 3 * E + pad, device=DEV, generator=g)).to(cd)
        qsrc, ksrc, vsrc, qc, kc, vc = x, x, x, 0, E, 2 * E
    else:                                        # separate q, packed kv
        qsrc = (2 * torch.randn(N, Lq, E + pad, device=DEV, generator=g)).to(cd)
        ksrc = (2 * torch.randn(N, Lk, 2 * E + pad, device=DEV, generator=g)).to(cd)
        vsrc, qc, kc, vc = ksrc, 0, 0, E
    sf = lambda t: (t.stride(1), t.stride(0))    # (row stride, batch stride) of (N, L, *)
    q = qsrc[..., qc:qc + E].permute(1, 0, 2)
    k = ksrc[..., kc:kc + E].permute(1, 0, 2)
    v = vsrc[..., vc:vc + E].permute(1, 0, 2)
    scale = 1.0 / math.sqrt(E // H)
    o = torch.full((N, Lq, E), float("nan"), dtype=cd, device=DEV)
    P = torch.empty(N * H * Lq * Lk, dtype=torch.float32, device=DEV)
    ops.small_attn_fwd(dt, N, H, Lq, Lk, E, q.data_ptr(), sf(qsrc), k.data_ptr(), sf(ksrc),
                       v.data_ptr(), sf(vsrc), o.data_ptr(), sf(o), scale, P)
    go = torch.randn(N, Lq, E, device=DEV, generator=g).to(cd)
    gq = torch.full_like(qsrc, float("nan"))
    gk = gq if ksrc is qsrc else torch.full_like(ksrc, float("nan"))
    ops.small_attn_bwd(dt, N, H, Lq, Lk, E, go.data_ptr(), sf(go), q.data_ptr(), sf(qsrc),
                       k.data_ptr(), sf(ksrc), v.data_ptr(), sf(vsrc), P,
                       gq[..., qc:].data_ptr(), sf(gq), gk[..., kc:].data_ptr(), sf(gk),
                       gk[..., vc:].data_ptr(), sf(gk), scale)
    torch.cuda.synchronize()
    qr, kr, vr = (t.float().requires_grad_(True) for t in (q, k, v))
    ref, pref = _small_ref(qr, kr, vr, H, scale)
    ref.backward(go.float().permute(1, 0, 2))
    u = {F32: 2e-6, BF16: 2.0 ** -8, F16: 2.0 ** -11}[dt]
    assert (P.view(N, H, Lq, Lk) - pref).abs().max().item() <= 2e-6
    pairs = [(o.permute(1, 0, 2), ref), (gq[..., qc:qc + E].permute(1, 0, 2), qr.grad),
             (gk[..., kc:kc + E].permute(1, 0, 2), kr.grad),
             (gk[..., vc:vc + E].permute(1, 0, 2), vr.grad)]
    for i, (got, want) in enumerate(pairs):
        err = (got.float() - want).abs().max().item()
        assert err <= 2 * u * want.abs().max().item() + 1e-6, (i, err)
    # padding columns are never written
    assert bool(torch.isnan(gq[..., -pad:]).all()) and bool(torch.isnan(gk[..., -pad:]).all())


def test_small_attn_rejects_unsupported():
    from jmt._lib import JMTError
    x = torch.zeros(4, 9, 512, dtype=torch.bfloat16, device=DEV)
    P = torch.empty(4 * 9 * 9, dtype=torch.float32, device=DEV)
    args = (x.data_ptr(), (512, 9 * 512))
    with pytest.raises(JMTError):                 # Lk = 9 > 8
        ops.small_attn_fwd(BF16, 4, 1, 9, 9, 512, *args, *args, *args, *args, 1.0, P)
    with pytest.raises(JMTError):                 # E != 512
        ops.small_attn_fwd(BF16, 4, 1, 2, 2, 256, *args, *args, *args, *args, 1.0, P)
    with pytest.raises(JMTError):                 # misaligned row start
        ops.small_attn_fwd(BF16, 4, 1, 2, 2, 512, x.data_ptr() + 2, (512, 9 * 512), *args,
                           *args, *args, 1.0, P)


@pytest.mark.parametrize("cd", [torch.float32, torch.bfloat16])
def test_short_sequences_dispatch_to_small_attn(cd):
    """AttnCoreFn routes Lk <= 8 to the small kernels (SELF_ATTEN head shapes: packed qkv over 6
    tokens, then the last-token query over them) and matches the GEMM + softmax path."""
    fams = []
    ops.set_launch_hook(lambda info, launch: (fams.append(info.get("family")), launch())[1])
    g = torch.Generator(device=DEV).manual_seed(5)
    N, E = 257, 512
    x = torch.randn(N, 6, 3 * E, device=DEV, generator=g).to(cd).permute(1, 0, 2)
    outs = []
    try:
        for fused in (True, False):
            ops._attn_fused["on"] = fused
            fams.clear()
            xx = x.detach().clone().requires_grad_(True)
            with JF.compute_mode(cd):
                o = JF.AttnCoreFn.apply(xx, xx, xx, E, 1, 0, E, 2 * E)
                o2 = JF.AttnCoreFn.apply(o[-1:], xx, xx, E, 1, 0, E, 2 * E)
            (o2.float().square().sum() + o.float().sum()).backward()
            outs.append((o.float(), o2.float(), xx.grad.float()))
            if fused:
                assert fams.count("small_attn_fwd") == 2 and fams.count("small_attn_bwd") == 2
            else:
                assert "small_attn_fwd" not in fams
    finally:
        ops._attn_fused["on"] = True
        ops.set_launch_hook(None)
    tol = 1e-5 if cd == torch.float32 else 2e-2
    for a, b in zip(*outs):
        assert (a - b).abs().max().item() <= tol * b.abs().max().item()


@pytest.mark.parametrize("D", [512, 768])
def test_layernorm_bwd_dsum_matches_colsum(D):
    """jmt_layernorm_bwd_dsum: dx, dgamma, dbeta as jmt_layernorm_bwd and dsum (+)= the
    fp32 column sums of dx (the residual branch's bias gradient), accumulated onto dsum."""
    cd = torch.bfloat16
    g = torch.Generator(device=DEV).manual_seed(31)
    rows = 1000
    x = torch.randn(rows, D, device=DEV, generator=g).to(cd)
    r = torch.randn(rows, D, device=DEV, generator=g).to(cd)
    dy = torch.randn(rows, D, device=DEV, generator=g).to(cd)
    gamma = torch.randn(D, device=DEV, generator=g)
    beta = torch.randn(D, device=DEV, generator=g)
    y = torch.empty(rows, D, dtype=cd, device=DEV)
    mean = torch.empty(rows, device=DEV)
    rstd = torch.empty(rows, device=DEV)
    ops.layernorm_fwd(x, D, r, D, gamma, beta, 1e-5, y, D, mean, rstd, rows, D)
    outs = []
    for fused in (False, True):
        dx = torch.empty(rows, D, dtype=cd, device=DEV)
        dg = torch.full((D,), 0.5, device=DEV)
        db = torch.full((D,), 0.25, device=DEV)
        ds = torch.full((D,), 1.0, device=DEV)
        if fused:
            assert ops.layernorm_bwd_dsum(x, D, r, D, dy, D, mean, rstd, gamma, dx, D, dg, db, ds,
                                          True, rows, D) is not None
        else:
            ops.layernorm_bwd(x, D, r, D, dy, D, mean, rstd, gamma, dx, D, dg, db, True, rows, D)
        torch.cuda.synchronize()
        outs.append((dx, dg, db, ds))
    (dx0, dg0, db0, _), (dx1, dg1, db1, ds1) = outs
    # the two instantiations may contract the dx arithmetic differently: 1 bf16 ulp apart at most
    assert (dx0.float() - dx1.float()).abs().max().item() <= 2.0 ** -7 * dx0.float().abs().max().item()
    assert torch.allclose(dg0, dg1, rtol=1e-5, atol=1e-4) and torch.allclose(db0, db1, rtol=1e-5,
                                                                              atol=1e-4)
    want = 1.0 + dx0.float().sum(0)
    assert (ds1 - want).abs().max().item() <= 1e-2 * want.abs().max().item() + 1e-3


_BOUNDS_LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                           "joint-multimodal-transformer-6th-abaw_amd", "jmt",
                           "libjmt_hip_bounds.so")

_BOUNDS_SCRIPT = r"""
import sys, torch
sys.path[:0] = [sys.argv[1], sys.argv[2]]
from jmt import _lib, functional as JF
from models.two_transformers import Two_transformers
from models.fc_layer import FcLayer
from losses.loss import CCCLoss
try:
    lib = _lib.load()
except AttributeError as e:        # a bounds build older than the library's ABI
    print("stale", e)
    sys.exit(5)
assert lib.jmt_bounds_violations(1) == 0
for jm, fmt, B, T in (("TRANSFORMER", "FC", 4, 300), ("TRANSFORMER", "SELF_ATTEN", 2, 37),
                      ("NONE", "FC", 8, 61)):
    torch.manual_seed(0)
    m = Two_transformers(0.0, 0.0, 1, 1, jm, fmt, 2048).cuda()
    fc = FcLayer(1024, 512).cuda()
    a = torch.randn(B, T, 1024, device="cuda"); v = torch.randn(B, T, 2048, device="cuda")
    y = torch.rand(1, B * T, device="cuda") * 2 - 1
    crit = CCCLoss(1)
    for cd in (torch.bfloat16, torch.float32):
        with JF.compute_mode(cd):
            vo, ao = m(fc(a), v)
            (crit(vo.reshape(1, -1), y) + crit(ao.reshape(1, -1), y)).backward()
n = lib.jmt_bounds_violations(1)
print("violations", n)
sys.exit(0 if n == 0 else 3)
"""


@pytest.mark.skipif(not os.path.exists(_BOUNDS_LIB), reason="bounds build not present")
def test_bounds_build_reports_no_violations():
    """the device-side index-check build (csrc `make bounds`, JMT_DCHECK counters)
    runs the TRANSFORMER/FC (T=300 tails), SELF_ATTEN and NONE models forward + backward in bf16
    and fp32 with zero failed checks.  Runs in a child process with JMT_LIB pointing at it."""
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    pkg = os.path.join(repo, "joint-multimodal-transformer-6th-abaw_amd")
    r = subprocess.run([sys.executable, "-c", _BOUNDS_SCRIPT, repo, pkg], capture_output=True,
                       text=True, timeout=240, env=dict(os.environ, JMT_LIB=_BOUNDS_LIB))
    if r.returncode == 5:
        pytest.skip("bounds build predates the library ABI (rebuild: make -C csrc bounds)")
    print(r.stdout)                     # the checker's report (committed under profiles/ with -s)
    assert r.returncode == 0 and "violations 0" in r.stdout, (r.stdout, r.stderr[-3000:])


@pytest.mark.parametrize("k", [1, 20])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_head_kernels_vs_torch(k, dt):
    """csrc/head.hip: both regressors' output layers (Linear(128, k) on the halves of one
    ReLU'd hidden buffer, two_transformers.py:104-114) forward, ReLU-masked input gradient and
    fp32 weight / bias gradients (+= into the buffers) vs torch fp32 on the same 16-bit h and
    W2; ragged row count, padded row strides."""
    from jmt import ops
    g = torch.Generator(device=DEV).manual_seed(11)
    rows, ldh = 1237, 264
    h = torch.relu(torch.randn(rows, ldh, device=DEV, generator=g)).to(dt)
    W2 = [(torch.randn(k, 128, device=DEV, generator=g) * 0.1).to(dt) for _ in range(2)]
    b2 = [torch.randn(k, device=DEV, generator=g) for _ in range(2)]
    ldy = k + 3
    ys = [torch.full((rows, ldy), float("nan"), device=DEV) for _ in range(2)]
    ops.head_fwd(h, ldh, rows, k, W2, b2, ys, ldy)
    for i in range(2):
        ref = h[:, 128 * i:128 * (i + 1)].float() @ W2[i].float().t() + b2[i]
        err = (ys[i][:, :k] - ref).abs().max().item()
        assert err <= 1e-5 * max(1.0, ref.abs().max().item()), (i, err)
        assert torch.isnan(ys[i][:, k:]).all()
    gy = [torch.randn(rows, ldy, device=DEV, generator=g) for _ in range(2)]
    dh = torch.full((rows, ldh), float("nan"), device=DEV).to(dt)
    dw = [torch.ones(k, 128, device=DEV) for _ in range(2)]      # accumulated into
    db = [torch.ones(k, device=DEV) for _ in range(2)]
    ops.head_bwd(h, ldh, rows, k, W2, gy, ldy, dh, ldh, dw, db)
    tol = 2 ** -7 if dt == torch.bfloat16 else 2 ** -10
    for i in range(2):
        hh = h[:, 128 * i:128 * (i + 1)].float()
        G = gy[i][:, :k]
        ref_dh = (G @ W2[i].float()) * (hh > 0)
        err = (dh[:, 128 * i:128 * (i + 1)].float() - ref_dh).abs().max().item()
        assert err <= tol * max(1.0, ref_dh.abs().max().item()), (i, err)
        rw = 1.0 + G.t() @ hh
        assert (dw[i] - rw).abs().max().item() <= 1e-4 * rw.abs().max().item()
        rb = 1.0 + G.sum(0)
        assert (db[i] - rb).abs().max().item() <= 1e-4 * max(1.0, rb.abs().max().item())
    assert torch.isnan(dh[:, 256:].float()).all(), "wrote past the two heads"


@pytest.mark.parametrize("dsum", [False, True])
@pytest.mark.parametrize("cd", [torch.bfloat16, torch.float32])
def test_layernorm_grouped_equals_per_group(dsum, cd):
    """jmt_layernorm_{fwd,bwd}_grouped (G groups, one launch each + one reduce) give the per-group
    jmt_layernorm_fwd / _bwd(_dsum) results: forward and dx bitwise (same row math), the column
    sums (dgamma, dbeta, dsum) to fp32 reassociation."""
    G, rows, D = 3, 1900, 512
    g = torch.Generator(device=DEV).manual_seed(37)
    X = torch.randn(G, rows, D, device=DEV, generator=g).to(cd)
    Rr = torch.randn(G, rows, D, device=DEV, generator=g).to(cd)
    dY = torch.randn(G, rows, D, device=DEV, generator=g).to(cd)
    gam = [torch.randn(D, device=DEV, generator=g) for _ in range(G)]
    bet = [torch.randn(D, device=DEV, generator=g) for _ in range(G)]
    Y1, Y2 = torch.empty_like(X), torch.empty_like(X)
    st1 = torch.empty(2, G * rows, device=DEV)
    st2 = torch.empty(2, G * rows, device=DEV)
    for i in range(G):
        ops.layernorm_fwd(X[i], D, Rr[i], D, gam[i], bet[i], 1e-5, Y1[i], D, st1[0, i * rows:],
                          st1[1, i * rows:], rows, D)
    assert ops.layernorm_fwd_grouped(X, Rr, gam, bet, 1e-5, Y2, st2[0], st2[1])
    torch.cuda.synchronize()
    assert torch.equal(Y1, Y2) and torch.equal(st1, st2)
    outs = []
    for grouped in (False, True):
        dX = torch.empty_like(X)
        dg = [torch.full((D,), 0.5, device=DEV) for _ in range(G)]
        db = [torch.full((D,), 0.25, device=DEV) for _ in range(G)]
        ds = [torch.full((D,), 1.0, device=DEV) for _ in range(G)] if dsum else None
        if grouped:
            assert ops.layernorm_bwd_grouped(X, Rr, dY, st1[0], st1[1], gam, dX, dg, db, ds,
                                             True) is not None
        else:
            for i in range(G):
                a = (X[i], D, Rr[i], D, dY[i], D, st1[0, i * rows:], st1[1, i * rows:], gam[i],
                     dX[i], D, dg[i], db[i])
                if dsum:
                    assert ops.layernorm_bwd_dsum(*a, ds[i], True, rows, D) is not None
                else:
                    ops.layernorm_bwd(*a, True, rows, D)
        torch.cuda.synchronize()
        outs.append((dX, dg, db, ds))
    (a, b) = outs
    assert torch.equal(a[0], b[0])
    # the grouped launch folds 32 rows per partial (one group: 16): the same fp32 sums in a
    # different association
    close = lambda u, v: torch.allclose(u, v, rtol=1e-5, atol=1e-4)
    for i in range(G):
        assert close(a[1][i], b[1][i]) and close(a[2][i], b[2][i])
        if dsum:
            assert close(a[3][i], b[3][i])


@pytest.mark.parametrize("ak,bk", [(False, False), (True, True), (True, False), (False, True)])
def test_gemm_pp_split_k(ak, bk):
    """Split-K ping-pong kernel (cfg 44, gemm_persist.hip gemm_pp_split_kernel): items are
    (256 x 256 tile, split) with balanced K-tile ranges, fp32 partial slabs reduced by
    splitk_reduce_kernel.  vs torch fp32 with beta = 1 accumulation into C, for the planner's own
    split count (the weight-gradient shapes) and forced uneven splits; the A row sums (dbias,
    TN layout only) within fp32 accumulation noise and C bit-identical with and without them."""
    from jmt import _lib
    lib = _lib.load()
    g = torch.Generator(device=DEV).manual_seed(44)
    bf = torch.bfloat16
    cases = [(1024, 512, 19200, 3, None), (1024, 1536, 4096, 1, None), (512, 256, 1344, 2, 7)]
    for (M, N, K, nb, splits) in cases:
        if splits is None:
            assert ops.auto_splits(M, N, K, nb, BF16) >= 2
        A, Al, lda, sa = _operand(M, K, ak, BF16, batch=nb, gen=g)
        Bs, Bl_t, ldb, sb = _operand(N, K, bk, BF16, batch=nb, gen=g)
        Bl = Bl_t.transpose(1, 2)
        C0 = torch.randn(nb, M, N, device=DEV, generator=g)
        outs = []
        for cfg in (44, 5):                 # 5: the one-block-per-tile split-K kernel
            for rs in ((False, True) if (not ak and not bk and cfg == 44) else (False,)):
                C = C0.clone()
                db = [torch.zeros(M, device=DEV) for _ in range(nb)] if rs else None
                lib.jmt_gemm_set_debug(cfg << 8)
                try:
                    ops.gemm(M=M, N=N, K=K, ab_dtype=BF16, c_dtype=F32,
                             a=[A[i].data_ptr() for i in range(nb)], lda=lda, a_kmajor=ak,
                             a_mode=1, b=[Bs[i].data_ptr() for i in range(nb)], ldb=ldb,
                             b_kmajor=bk, b_mode=1, c=[C[i].data_ptr() for i in range(nb)],
                             ldc=N, c_mode=1, batch0=nb, beta=1.0, splits=splits,
                             dbias_tab=db, device=DEV)
                finally:
                    lib.jmt_gemm_set_debug(0)
                torch.cuda.synchronize()
                outs.append(C)
                for i in range(nb):
                    ref = C0[i] + Al[i] @ Bl[i]
                    err = (C[i] - ref).abs().max().item()
                    assert err <= 2e-3 * (Al[i].abs() @ Bl[i].abs()).max().item(), (M, N, K, cfg, err)
                    if rs:
                        rref = Al[i].sum(1)
                        rerr = (db[i] - rref).abs().max().item()
                        assert rerr <= 1e-6 * Al[i].abs().sum(1).max().item() + 1e-5, (M, K, rerr)
        if not ak and not bk:
            assert torch.equal(outs[0], outs[1]), "row sums changed C"


@pytest.mark.parametrize("mode", [2, 3])
@pytest.mark.parametrize("ak,bk", [(False, False), (False, True)])
def test_gemm_kconcat_split_k(mode, ak, bk):
    """K-concatenated operands on the split-K kernels: mode 2 (segments shared by
    every batch entry) and mode 3 (ABI 7: each batch entry's own segments, base[b0 * nseg + s] —
    the two uses of a cross-attention module in one weight-gradient entry).  The split ranges
    start partway through a segment (K-tiles per split not dividing the segment); cfg 44 (split-K
    ping-pong, the planner's choice for the merged wgrads), cfg 5 and the planner's default vs
    the fp32 sum of the per-segment products, with beta = 1 and (TN) the A row sums over all
    segments."""
    from jmt import _lib
    lib = _lib.load()
    g = torch.Generator(device=DEV).manual_seed(45)
    cases = [(512, 512, 19200, 2, 3, None), (512, 256, 1344, 2, 2, 7), (256, 512, 2240, 3, 2, 5)]
    for (M, N, kseg, nseg, nb, splits) in cases:
        if mode == 2 and nb > 1 and splits is None:
            nb = 1
        A, B = [], []
        for i in range(nb if mode == 3 else 1):
            for _ in range(nseg):
                A.append(_operand(M, kseg, ak, BF16, gen=g))
                B.append(_operand(N, kseg, bk, BF16, gen=g))
        lda, ldb = A[0][2], B[0][2]
        C0 = torch.randn(nb, M, N, device=DEV, generator=g)
        refs, rrefs = [], []
        for i in range(nb):
            ss = range(i * nseg, (i + 1) * nseg) if mode == 3 else range(nseg)
            refs.append(C0[i] + sum(A[s][1][0] @ B[s][1][0].transpose(0, 1) for s in ss))
            rrefs.append(sum(A[s][1][0].sum(1) for s in ss))
        if splits is None:
            assert ops.auto_splits(M, N, nseg * kseg, nb, BF16) >= 2
        for cfg in (44, 5, 0):
            rs = not ak and not bk
            C = C0.clone()
            db = [torch.zeros(M, device=DEV) for _ in range(nb)] if rs else None
            lib.jmt_gemm_set_debug(cfg << 8)
            try:
                ops.gemm(M=M, N=N, K=nseg * kseg, ab_dtype=BF16, c_dtype=F32,
                         a=[t[0].data_ptr() for t in A], lda=lda, a_kmajor=ak, a_mode=mode,
                         a_kseg=kseg, b=[t[0].data_ptr() for t in B], ldb=ldb, b_kmajor=bk,
                         b_mode=mode, b_kseg=kseg, c=[C[i].data_ptr() for i in range(nb)],
                         ldc=N, c_mode=1, batch0=nb, beta=1.0, splits=splits, dbias_tab=db,
                         device=DEV)
            finally:
                lib.jmt_gemm_set_debug(0)
            torch.cuda.synchronize()
            for i in range(nb):
                scale = sum((A[s][1][0].abs() @ B[s][1][0].abs().transpose(0, 1)).max().item()
                            for s in range(nseg))
                err = (C[i] - refs[i]).abs().max().item()
                assert err <= 2e-3 * scale, (mode, M, N, kseg, cfg, i, err)
                if rs:
                    rerr = (db[i] - rrefs[i]).abs().max().item()
                    assert rerr <= 1e-5 * nseg * kseg, (mode, cfg, i, rerr)


def test_gemm_kconcat_per_batch_rejects_short_table():
    """Mode 3 needs batch0 x ceil(K / kseg) pointers and a kseg of whole K-tiles."""
    from jmt import _lib
    x = torch.zeros(64, 64, device=DEV, dtype=torch.bfloat16)
    c = torch.zeros(2, 64, 64, device=DEV)
    for kseg, na in ((64, 3), (48, 4)):
        with pytest.raises(RuntimeError, match="per-batch K-concat"):
            ops.gemm(M=64, N=64, K=128, ab_dtype=BF16, c_dtype=F32, a=[x.data_ptr()] * na,
                     lda=64, a_kmajor=False, a_mode=3, a_kseg=kseg, b=[x.data_ptr()] * 4,
                     ldb=64, b_kmajor=False, b_mode=3, b_kseg=64,
                     c=[c[0].data_ptr(), c[1].data_ptr()], ldc=64, c_mode=1, batch0=2,
                     device=DEV)
    assert _lib.load() is not None


@pytest.mark.parametrize("cfg", [0, 1, 5, 10, 11, 20, 21])
@pytest.mark.parametrize("dt", [BF16, F16])
def test_gemm_wgrad_row_sums_bias_grad(cfg, dt):
    """jmt_gemm's A row sums (dbias_tab, ABI 4): a weight-gradient GEMM dW = dY^T X also writes
    the bias gradient db = column sums of dY from the A fragments it already holds.  vs the fp32
    column sums of the same rounded dY, with and without split-K, accumulate and overwrite,
    ragged M / K, pointer-table batch; C is bit-identical to the same launch without row sums."""
    from jmt import _lib
    lib = _lib.load()
    t = TD[dt]
    g = torch.Generator(device=DEV).manual_seed(41)
    lib.jmt_gemm_set_debug(cfg << 8)
    try:
        for (n, Kin, rows, batch, splits, acc) in [(300, 520, 1000, 2, 1, True),
                                                   (512, 512, 19200, 3, None, True),
                                                   (257, 129, 333, 1, 3, False),
                                                   (1536, 512, 4800, 1, None, True),
                                                   (40, 64, 4096, 2, 8, False)]:
            ldn, ldk = _rup(n, 8) + 8, _rup(Kin, 8) + 8
            dY = torch.randn(batch, rows, ldn, device=DEV, generator=g).to(t)
            X = torch.randn(batch, rows, ldk, device=DEV, generator=g).to(t)
            C0 = torch.randn(batch, n, Kin, device=DEV, generator=g)
            C1 = C0.clone()
            db = [torch.randn(n, device=DEV, generator=g) for _ in range(batch)]
            db0 = [d.clone() for d in db]
            kw = dict(M=n, N=Kin, K=rows, ab_dtype=dt, c_dtype=F32,
                      a=[dY[i].data_ptr() for i in range(batch)], lda=ldn, a_kmajor=False,
                      a_mode=1, b=[X[i].data_ptr() for i in range(batch)], ldb=ldk,
                      b_kmajor=False, b_mode=1, ldc=Kin, c_mode=1, batch0=batch, beta=1.0,
                      splits=splits, device=DEV)
            ops.gemm(c=[C0[i].data_ptr() for i in range(batch)], **kw)
            ops.gemm(c=[C1[i].data_ptr() for i in range(batch)], dbias_tab=db, dbias_acc=acc,
                     **kw)
            torch.cuda.synchronize()
            assert torch.equal(C0, C1), (cfg, n, Kin, rows, "C changed by the row sums")
            for i in range(batch):
                ref = dY[i, :, :n].float().sum(0) + (db0[i] if acc else 0.0)
                err = (db[i] - ref).abs().max().item()
                scale = dY[i, :, :n].float().abs().sum(0).max().item()
                assert err <= 1e-6 * scale + 1e-5, (cfg, n, Kin, rows, splits, i, err)
        # K-concatenated wgrad: the segments share dY (sA = 0), only segment 0 takes the sums
        n, Kin, rows = 512, 256, 3000
        dY = torch.randn(rows, n, device=DEV, generator=g).to(t)
        X = torch.randn(2, rows, Kin, device=DEV, generator=g).to(t)
        C = torch.zeros(n, 2 * Kin, device=DEV)
        db = torch.randn(n, device=DEV, generator=g)
        db0 = db.clone()
        ops.gemm(M=n, N=Kin, K=rows, ab_dtype=dt, c_dtype=F32, a=[dY.data_ptr()], lda=n,
                 a_kmajor=False, sA=(0, 0), b=[X.data_ptr()], ldb=Kin, b_kmajor=False,
                 sB=(rows * Kin, 0), c=[C.data_ptr()], ldc=2 * Kin, sC=(Kin, 0), batch0=2,
                 beta=1.0, dbias_tab=[db, None], device=DEV)
        torch.cuda.synchronize()
        ref = db0 + dY.float().sum(0)
        assert (db - ref).abs().max().item() <= 1e-6 * dY.float().abs().sum(0).max().item() + 1e-5
        with pytest.raises(_lib.JMTError):    # K-major A: not a weight-gradient launch
            A = torch.randn(64, 64, device=DEV).to(t)
            C = torch.empty(64, 64, device=DEV)
            ops.gemm(M=64, N=64, K=64, ab_dtype=dt, c_dtype=F32, a=[A.data_ptr()], lda=64,
                     a_kmajor=True, b=[A.data_ptr()], ldb=64, b_kmajor=False, c=[C.data_ptr()],
                     ldc=64, dbias_tab=[torch.zeros(64, device=DEV)], device=DEV)
    finally:
        lib.jmt_gemm_set_debug(0)
