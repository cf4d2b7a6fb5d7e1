"""Data parallelism through the PRODUCT path: two ranks sharing cuda:0 over gloo,
each running the HIP drop-ins on its contiguous batch shard (jmt.dist.shard_range), the
reference's losses with the process group registered (jmt.dist.set_loss_group: the CCC
statistics all-gathered, the global-batch CCC on every rank) and the gradients summed over one
flat buffer (jmt.dist.FlatGrads) — against the DataParallel semantics the reference trains with
(main.py:487-491: replicas on dim-0 shards, outputs gathered on dim 0; train.py:303-311: the loss
on the gathered batch), restated on the CPU oracle (oracle/jmt_ref.py)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

B, T, VIN = 4, 16, 512


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _inputs():
    from oracle.hashinit import features, labels
    return (torch.from_numpy(features("dp.audio", (B, T, 512))),
            torch.from_numpy(features("dp.video", (B, T, VIN))),
            torch.from_numpy(labels("dp.lv", (B, T))), torch.from_numpy(labels("dp.la", (B, T))))


def _model(hashed=True, jm="TRANSFORMER"):
    """hashed: the discriminative counter-hash init of the goldens (sharp attention: 16-bit runs
    of it differ by O(10 %) in the gradients from any reordering, tests/parity.py); otherwise
    torch's default init under a fixed seed (smooth: 16-bit differences stay O(1e-3)).
    jm: joint_modalities ("NONE" = MultimodalTransformer_wo_JR, bench config c2, whose encoder
    and cross-attention backwards run on the run_parallel branch streams)."""
    from models.two_transformers import Two_transformers
    from oracle.hashinit import init_module_
    torch.manual_seed(0)
    m = Two_transformers(0.0, 0.0, 1, 1, jm, "FC", VIN)
    if hashed:
        init_module_(m, "")
    return m


def _spawn(target, args, world=2, timeout=240):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q) + args) for r in range(world)]
    for p in procs:
        p.start()
    try:
        out = sorted([q.get(timeout=timeout) for _ in range(world)], key=lambda r: r[0])
    finally:
        for p in procs:
            p.join(timeout=60)
        for p in procs:             # a rank left waiting in a collective for a dead peer
            if p.is_alive():
                p.kill()
                p.join(timeout=10)
    for p in procs:
        assert p.exitcode == 0, p.exitcode
    return out


def _init(rank, world, port):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      HSA_ENABLE_IPC_MODE_LEGACY="0")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    torch.set_num_threads(2)
    from jmt import dist as jdist
    jdist.set_loss_group(dist.group.WORLD)
    return dist, jdist


def _train_step_worker(rank, world, port, q, cd_name):
    dist, jdist = _init(rank, world, port)
    try:
        from jmt import functional as JF
        from losses.loss import CCCLoss
        cd = getattr(torch, cd_name)
        audio, video, lv, la = _inputs()
        lo, hi = jdist.shard_range(B, rank, world)
        m = _model(hashed=cd == torch.float32).cuda()
        fg = jdist.FlatGrads(list(m.parameters()), "cuda")
        fg.zero_()
        crit = CCCLoss(1)
        with JF.compute_mode(cd):
            vo, ao = m(audio[lo:hi].cuda(), video[lo:hi].cuda())
            # train.py:303-307 on the replica's (T, b) outputs and the shard's (b, T) labels
            vout = vo.view(-1, vo.shape[0] * vo.shape[1])
            aout = ao.view(-1, ao.shape[0] * ao.shape[1])
            n = (hi - lo) * T
            loss = crit(vout, lv[lo:hi].cuda().view(-1, n)) + crit(aout, la[lo:hi].cuda().view(-1, n))
            loss.backward()
        fg.allreduce_()
        torch.cuda.synchronize()
        grads = {k: p.grad.detach().float().cpu().numpy() for k, p in m.named_parameters()
                 if p.grad is not None}
        q.put((rank, float(loss.detach()), grads))
    finally:
        dist.destroy_process_group()


def _dp_oracle(jm="TRANSFORMER"):
    """nn.DataParallel on 2 replicas, restated on the CPU oracle: per-replica forward on the
    dim-0 shard, outputs gathered on dim 0, CCC on the gathered (1, B*T) view, grads."""
    from oracle import jmt_ref as R
    m = _model(jm=jm)
    p = {k: v.detach().clone().float().requires_grad_(True) for k, v in m.state_dict().items()}
    audio, video, lv, la = _inputs()
    vos, aos = [], []
    for r in range(2):
        sl = slice(r * B // 2, (r + 1) * B // 2)
        vo, ao = R.two_transformers_forward(audio[sl], video[sl], p, 1, 1, jm, "FC", VIN)
        vos.append(vo)
        aos.append(ao)
    vo, ao = torch.cat(vos, 0), torch.cat(aos, 0)
    loss = R.ccc_loss(vo.reshape(1, -1), lv.reshape(1, -1)) + \
        R.ccc_loss(ao.reshape(1, -1), la.reshape(1, -1))
    loss.backward()
    return float(loss.detach()), {k: t.grad for k, t in p.items() if t.grad is not None}


def _single_gpu(cd):
    """The same full batch in ONE process (the 1-GPU product path), its (T, B) outputs regrouped
    as DataParallel's dim-0 gather of the two replicas' (T, B/2) chunks before the flatten."""
    from jmt import dist as jdist
    from jmt import functional as JF
    from losses.loss import CCCLoss
    audio, video, lv, la = _inputs()
    m = _model(hashed=False).cuda()
    crit = CCCLoss(1)
    gather = lambda o: torch.cat([o[:, slice(*jdist.shard_range(B, r, 2))] for r in range(2)], 0)
    with JF.compute_mode(cd):
        vo, ao = m(audio.cuda(), video.cuda())
        loss = crit(gather(vo).reshape(1, -1), lv.cuda().view(1, -1)) + \
            crit(gather(ao).reshape(1, -1), la.cuda().view(1, -1))
        loss.backward()
    return float(loss), {k: p.grad.detach().float().cpu() for k, p in m.named_parameters()
                         if p.grad is not None}


def test_two_rank_product_path_fp32_matches_dataparallel_oracle():
    out = _spawn(_train_step_worker, ("float32",))
    ref_loss, ref_grads = _dp_oracle()
    gmax = max(float(g.abs().max()) for g in ref_grads.values())
    (_, l0, g0), (_, l1, g1) = out
    assert l0 == l1, (l0, l1)                                  # global-batch loss on every rank
    assert abs(l0 - ref_loss) <= 1e-5, (l0, ref_loss)
    assert set(ref_grads) <= set(g0), set(ref_grads) - set(g0)
    for k in g0:
        assert np.array_equal(g0[k], g1[k]), k                 # all-reduced: identical replicas
        if k not in ref_grads:                                 # never used by the forward
            assert not g0[k].any(), k                          # (final_encoder): zero in FlatGrads
            continue
        r = ref_grads[k]
        err = float((torch.from_numpy(g0[k]) - r).abs().max())
        assert err <= 1e-4 * max(float(r.abs().max()), 0.01 * gmax), (k, err)


def test_two_rank_product_path_bf16_matches_single_gpu():
    """bf16 (torch default init): the 2-rank run equals the one-process full-batch run up to
    the GEMM accumulation orders that differ with the per-rank row count and the order in which
    the per-rank gradient halves are summed."""
    out = _spawn(_train_step_worker, ("bfloat16",))
    ref_loss, ref_grads = _single_gpu(torch.bfloat16)
    gmax = max(float(g.abs().max()) for g in ref_grads.values())
    (_, l0, g0), (_, l1, g1) = out
    assert l0 == l1
    assert abs(l0 - ref_loss) <= 2e-3, (l0, ref_loss)
    for k in ref_grads:
        r = ref_grads[k]
        err = float((torch.from_numpy(g0[k]) - r).abs().max())
        # floor: near-cancelling sums (the regressor bias) carry bf16 noise of the summands
        assert err <= 2e-2 * max(float(r.abs().max()), 0.05 * gmax), (k, err)


SIZES = (7, 12)     # unequal per-rank batches


def _loss_worker(rank, world, port, q, kind):
    dist, jdist = _init(rank, world, port)
    try:
        from oracle.hashinit import features, labels
        n = SIZES[rank]
        off = sum(SIZES[:rank])
        tot = sum(SIZES)
        if kind == "ignore":
            from losses.CCCLoss import CCCLoss
            x = torch.from_numpy(features("dpl.x", (tot,)))[off:off + n]
            y = torch.from_numpy(labels("dpl.y", (tot,), ignore_frac=0.3))[off:off + n]
            crit = CCCLoss(-5.0)
        else:                               # digitized expectation CCC, k = 5 bins
            from losses.loss import CCCLoss
            x = torch.from_numpy(features("dpl.logits", (tot, 5)))[off:off + n] * 3
            y = torch.from_numpy(labels("dpl.y5", (tot,)))[off:off + n].view(1, -1)
            crit = CCCLoss(5)
        xg = x.cuda().requires_grad_(True)
        loss = crit(xg, y.cuda())
        loss.backward()
        torch.cuda.synchronize()
        q.put((rank, float(loss.detach()), xg.grad.cpu().numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("kind", ["ignore", "digitized"])
def test_two_rank_losses_unequal_shards_match_gathered_batch(kind):
    """losses/CCCLoss.py (ignore-masked, 1-D: the gathered size(0) is the SUM of the ranks'
    sizes) and losses/loss.py CCCLoss(digitize_num=5) on 7 + 12 elements: every rank's loss
    equals the loss of the gathered batch and its gradient the matching slice of that loss's."""
    from oracle import jmt_ref as R
    from oracle.hashinit import features, labels
    out = _spawn(_loss_worker, (kind,))
    tot = sum(SIZES)
    if kind == "ignore":
        x = torch.from_numpy(features("dpl.x", (tot,))).double().requires_grad_(True)
        y = torch.from_numpy(labels("dpl.y", (tot,), ignore_frac=0.3)).double()
        ref = R.ccc_loss_ignore(x, y, -5.0)
    else:
        x = (torch.from_numpy(features("dpl.logits", (tot, 5))) * 3).double().requires_grad_(True)
        y = torch.from_numpy(labels("dpl.y5", (tot,))).double()
        ref = R.ccc_loss(x, y.view(1, -1), digitize_num=5)
    ref.backward()
    off = 0
    for rank, loss, g in out:
        assert abs(loss - float(ref)) <= 1e-5, (rank, loss, float(ref))
        gr = x.grad[off:off + SIZES[rank]].numpy()
        assert np.abs(g - gr).max() <= 1e-5 * max(1.0, np.abs(gr).max()), (rank, g, gr)
        off += SIZES[rank]


def _bucketed_worker(rank, world, port, q, jm="TRANSFORMER", side=True):
    """bench.py's N>1 step: FusedSGD's flat gradients in write-completion order and the
    all-reduce issued bucket by bucket during the backward (jmt.dist.GradBucketer).  side=False
    turns the weight-gradient side stream off (JMT_SIDE_STREAM=0, bench.py's probe steps)."""
    dist, jdist = _init(rank, world, port)
    try:
        from jmt import functional as JF
        from jmt import streams
        from jmt.optim import FusedSGD
        from losses.loss import CCCLoss
        streams.set_side_enabled(side)
        audio, video, lv, la = _inputs()
        lo, hi = jdist.shard_range(B, rank, world)
        m = _model(jm=jm).cuda()
        crit = CCCLoss(1)
        a, v = audio[lo:hi].cuda(), video[lo:hi].cuda()
        n = (hi - lo) * T
        yv, ya = lv[lo:hi].cuda().view(-1, n), la[lo:hi].cuda().view(-1, n)

        def fwd_bwd():
            with JF.compute_mode(torch.float32):
                vo, ao = m(a, v)
                loss = crit(vo.view(-1, n), yv) + crit(ao.view(-1, n), ya)
                loss.backward()
            return loss

        params, counts = jdist.grad_write_profile(fwd_bwd, list(m.parameters()))
        opt = FusedSGD(params, lr=0.0)
        bk = jdist.GradBucketer(opt, counts, bucket_bytes=1 << 20, group=dist.group.WORLD)
        opt.zero_grad()
        bk.begin()
        loss = fwd_bwd()
        early = len(bk.launch_log)             # buckets issued before the backward returned
        bk.finish()
        torch.cuda.synchronize()
        names = {id(p): k for k, p in m.named_parameters()}
        grads = {names[id(p)]: p.grad.detach().cpu().numpy() for p in params}
        q.put((rank, float(loss.detach()), grads, early, len(bk.buckets)))
        bk.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("jm,side", [("TRANSFORMER", True), ("NONE", True),
                                     ("TRANSFORMER", False)])
def test_two_rank_overlapped_bucket_allreduce_matches_dataparallel_oracle(jm, side):
    """the bucket gating must cover gradient writes on every stream —
    the grouped w_JR model (side stream on / off) and the wo_JR model (c2), whose branch
    backwards run on the run_parallel streams."""
    out = sorted(_spawn_raw(_bucketed_worker, args=(jm, side)), key=lambda r: r[0])
    ref_loss, ref_grads = _dp_oracle(jm)
    gmax = max(float(g.abs().max()) for g in ref_grads.values())
    (_, l0, g0, early0, nb), (_, l1, g1, _, _) = out
    assert nb > 2 and early0 >= 1, (nb, early0)   # several buckets, some issued mid-backward
    assert abs(l0 - ref_loss) <= 1e-5, (l0, ref_loss)
    assert set(g0) == set(ref_grads), set(g0) ^ set(ref_grads)
    for k in g0:
        assert np.array_equal(g0[k], g1[k]), k
        r = ref_grads[k]
        err = float((torch.from_numpy(g0[k]) - r).abs().max())
        assert err <= 1e-4 * max(float(r.abs().max()), 0.01 * gmax), (k, err)


def _spawn_raw(target, world=2, args=()):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q) + args) for r in range(world)]
    for p in procs:
        p.start()
    try:
        out = [q.get(timeout=240) for _ in range(world)]
    finally:
        for p in procs:
            p.join(timeout=60)
    for p in procs:
        assert p.exitcode == 0, p.exitcode
    return out


def _rccl1_worker(rank, world, port, q, mode):
    """One rank with the nccl (RCCL) backend and the bucketer's collectives forced on at world
    size 1 (GradBucketer.world1): the real RCCL launch path of bench.py's N>1 step on a 1-GPU box.
    mode 'sync': one bucketed step under torch.cuda.set_sync_debug_mode('error') — the step
    (forward, backward, bucket gating, all-reduces, fused SGD) must not synchronise the device.
    mode 'graph': the same step captured into a hipGraph with the RCCL all-reduces inside
    (bench.py's N>1 default), replayed; its parameters must equal eager steps' bit for bit."""
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      HSA_ENABLE_IPC_MODE_LEGACY="0")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=rank, world_size=world,
                            device_id=torch.device("cuda", 0))
    try:
        from jmt import dist as jdist
        from jmt import functional as JF
        from jmt.graph import GraphedStep
        from jmt.optim import FusedSGD
        from losses.loss import CCCLoss
        jdist.set_loss_group(dist.group.WORLD)
        audio, video, lv, la = _inputs()
        m = _model(hashed=False).cuda()
        crit = CCCLoss(1)
        a, v = audio.cuda(), video.cuda()
        n = B * T
        yv, ya = lv.cuda().view(-1, n), la.cuda().view(-1, n)

        def fwd_bwd():
            with JF.compute_mode(torch.bfloat16):
                vo, ao = m(a, v)
                loss = crit(vo.view(-1, n), yv) + crit(ao.view(-1, n), ya)
                loss.backward()
            return loss

        params, counts = jdist.grad_write_profile(fwd_bwd, list(m.parameters()))
        opt = FusedSGD(params, lr=1e-3, momentum=0.9, weight_decay=1e-4, nesterov=True,
                       shadow_dtype=torch.bfloat16)
        bk = jdist.GradBucketer(opt, counts, bucket_bytes=1 << 20, group=dist.group.WORLD)
        bk.world1 = True

        def step():
            opt.zero_grad()
            bk.begin()
            loss = fwd_bwd()
            bk.finish()
            opt.step()
            return loss

        for _ in range(2):                              # first-step branches, allocator warm
            step()
        torch.cuda.synchronize()
        if mode == "sync":
            torch.cuda.set_sync_debug_mode("error")
            try:
                step()
            finally:
                torch.cuda.set_sync_debug_mode(0)
            torch.cuda.synchronize()
            q.put((rank, len(bk.buckets), len(bk.launch_log), None))
        else:
            bufs = [t for t in (opt.flat_p, opt.buf, opt.shadow) if t is not None]
            snap = [t.clone() for t in bufs]

            def rewind():
                with torch.no_grad():
                    for t, s in zip(bufs, snap):
                        t.copy_(s)

            for _ in range(3):
                step()
            torch.cuda.synchronize()
            eager = opt.flat_p.clone()
            rewind()
            g = GraphedStep(step).capture(warmup=1)
            rewind()
            for _ in range(3):
                g.replay()
            torch.cuda.synchronize()
            same = bool(torch.equal(opt.flat_p, eager))
            q.put((rank, len(bk.buckets), len(bk.launch_log), same))
        bk.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["sync"])
def test_rccl_bucketed_step_sync_free_and_capturable(mode):
    """a bucketed step issues no device synchronisation.  (Its 'graph' mode —
    the RCCL all-reduces captured into one whole-step hipGraph — is retired with that path in
    round 6: ProcessGroupNCCL's watchdog thread intermittently queried a work event recorded
    inside the capture and aborted the rank, hipErrorCapturedEvent; the N>1 step is now the
    segmented graph with eager collectives, test_segmented_graph_step_matches_eager.)"""
    out = _spawn(_rccl1_worker, (mode,), world=1)
    (_, nb, launched, same), = out
    assert nb > 2 and launched == nb, (nb, launched)
    if mode == "graph":
        assert same


def _segmented_worker(rank, world, port, q, backend, bucket_mb=1):
    """bench.py's N>1 default: the bucketed step captured as hipGraph
    segments with the collectives (CCC all-gather, bucket all-reduces, the final join) issued on
    the host between them (jmt.graph.SegmentedStep).  Three replayed steps must leave the
    parameters bit-identical to three eager steps from the same state, and the host time to issue
    one replayed step is reported."""
    import time
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      HSA_ENABLE_IPC_MODE_LEGACY="0")
    torch.cuda.set_device(0)
    if backend == "nccl":
        dist.init_process_group("nccl", rank=rank, world_size=world,
                                device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from jmt import dist as jdist
        from jmt import functional as JF
        from jmt.graph import SegmentedStep
        from jmt.optim import FusedSGD
        from losses.loss import CCCLoss
        jdist.set_loss_group(dist.group.WORLD)
        audio, video, lv, la = _inputs()
        lo, hi = jdist.shard_range(B, rank, world)
        m = _model(hashed=False).cuda()
        crit = CCCLoss(1)
        a, v = audio[lo:hi].cuda(), video[lo:hi].cuda()
        n = (hi - lo) * T
        yv, ya = lv[lo:hi].cuda().view(-1, n), la[lo:hi].cuda().view(-1, n)

        def fwd_bwd():
            with JF.compute_mode(torch.bfloat16):
                vo, ao = m(a, v)
                loss = crit(vo.view(-1, n), yv) + crit(ao.view(-1, n), ya)
                loss.backward()
            return loss

        params, counts = jdist.grad_write_profile(fwd_bwd, list(m.parameters()))
        opt = FusedSGD(params, lr=1e-3, momentum=0.9, weight_decay=1e-4, nesterov=True,
                       shadow_dtype=torch.bfloat16, fuse_zero_grad=True)
        bk = jdist.GradBucketer(opt, counts, bucket_bytes=bucket_mb << 20,
                                group=dist.group.WORLD)
        bk.world1 = world == 1

        def step():
            opt.zero_grad()
            bk.begin()
            loss = fwd_bwd()
            bk.finish()
            opt.step()
            return loss

        for _ in range(2):                              # first-step branches, allocator warm
            step()
        torch.cuda.synchronize()
        bufs = [t for t in (opt.flat_p, opt.buf, opt.shadow, opt.flat_g) if t is not None]
        snap = [t.clone() for t in bufs]

        def rewind():
            with torch.no_grad():
                for t, s in zip(bufs, snap):
                    t.copy_(s)

        losses_e = [float(step()) for _ in range(3)]
        torch.cuda.synchronize()
        eager = opt.flat_p.clone()
        rewind()
        g = SegmentedStep(step).capture(warmup=1)
        rewind()
        losses_g = []
        issue = []
        for _ in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            out = g.replay()
            issue.append(time.perf_counter() - t0)
            losses_g.append(float(out))
        torch.cuda.synchronize()
        same = bool(torch.equal(opt.flat_p, eager))
        q.put((rank, len(bk.buckets), len(g.segments), same, losses_e, losses_g,
               min(issue) * 1e3))
        bk.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("backend,world,bucket_mb", [("gloo", 2, 1), ("nccl", 1, 1),
                                                    ("nccl", 1, 8)])
def test_segmented_graph_step_matches_eager(backend, world, bucket_mb):
    """the piecewise-captured N>1 step (two gloo ranks sharing cuda:0, and
    one RCCL rank with the bucket collectives forced on) replays bit-identical to the eager
    bucketed step; every bucket all-reduce and the CCC all-gather cut the capture (segments >=
    buckets + 2)."""
    out = _spawn(_segmented_worker, (backend, bucket_mb), world=world, timeout=100)
    for (_, nb, nseg, same, le, lg, issue_ms) in out:
        assert same, (backend, le, lg)
        assert le == lg
        assert nseg >= nb + 2, (nseg, nb)
        print(f"{backend} ws {world}: {nseg} segments, {nb} buckets, host issue "
              f"{issue_ms:.3f} ms per replayed step")
