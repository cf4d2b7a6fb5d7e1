"""The N>1 data-parallel algorithm on CPU with world_size=2 (gloo): contiguous batch sharding
(jmt.dist.shard_range), all-gathered CCC statistics combined in rank order (the algorithm of
jmt_ccc_stats / jmt_ccc_finish, restated in oracle/dist_ref.py), and the SUM all-reduce of the
flat gradient buffer (jmt.dist.FlatGrads) — checked against the reference's DataParallel
semantics: replicas on dim-0 shards, outputs gathered on dim 0, loss on the gathered batch
(main.py:487-491, train.py:303-311)."""
import os

import numpy as np
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import dist_ref as D
from oracle import jmt_ref as R
from tests.golden import spec

B, T = 4, 16


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _setup():
    p = R.hash_params(R.two_transformers_shapes(1, "TRANSFORMER", "FC", 512), "")
    audio, video, lv, la = spec.tt_inputs("dist", B, T, 512)
    return p, torch.from_numpy(audio[..., :512].copy()), torch.from_numpy(video), \
        torch.from_numpy(lv), torch.from_numpy(la)


def _dataparallel_reference():
    """Replicas on dim-0 shards -> (T, B/g) outputs -> gather on dim 0 -> (1, B*T) view ->
    CCCLoss on the gathered batch -> grads (what nn.DataParallel computes)."""
    p, audio, video, lv, la = _setup()
    for t in p.values():
        t.requires_grad_(True)
    outs_v, outs_a = [], []
    for r in range(2):
        sl = slice(r * B // 2, (r + 1) * B // 2)
        vo, ao = R.two_transformers_forward(audio[sl], video[sl], p, 1, 1, "TRANSFORMER", "FC",
                                            512)
        outs_v.append(vo)
        outs_a.append(ao)
    vo = torch.cat(outs_v, 0)
    ao = torch.cat(outs_a, 0)
    loss = R.ccc_loss(vo.reshape(1, -1), lv.reshape(1, -1)) + \
        R.ccc_loss(ao.reshape(1, -1), la.reshape(1, -1))
    loss.backward()
    return float(loss), {k: t.grad.clone() for k, t in p.items() if t.grad is not None}


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(2)
    try:
        from jmt import dist as jdist
        p, audio, video, lv, la = _setup()
        lo, hi = jdist.shard_range(B, rank, world)
        params = [torch.nn.Parameter(t.clone()) for t in p.values()]
        names = list(p.keys())
        pd = dict(zip(names, params))
        vo, ao = R.two_transformers_forward(audio[lo:hi], video[lo:hi], pd, 1, 1, "TRANSFORMER",
                                            "FC", 512)
        # local (T, B/g) predictions paired with local (B/g, T) labels, as each DP replica
        xs = [vo.reshape(-1), ao.reshape(-1)]
        ys = [lv[lo:hi].reshape(-1), la[lo:hi].reshape(-1)]
        loss = 0.0
        for x, y in zip(xs, ys):
            st = D.local_stats(x.detach(), y)
            allst = [torch.empty(6, dtype=torch.float64) for _ in range(world)]
            dist.all_gather(allst, st)
            loss = loss + D.global_ccc_loss_local(x, y, torch.stack(allst), rank)
        loss.backward()
        # FlatGrads re-homes .grad into one zeroed flat buffer: snapshot the local grads first
        gsnap = {n: t.grad.clone() for n, t in zip(names, params) if t.grad is not None}
        fg = jdist.FlatGrads([t for t in params if t.grad is not None], "cpu")
        fg_params = fg.params
        fg.zero_()
        off = 0
        for t in fg_params:
            n_ = [k for k, v in pd.items() if v is t][0]
            fg.flat[off:off + t.numel()].copy_(gsnap[n_].reshape(-1))
            off += t.numel()
        fg.allreduce_()
        res = {}
        off = 0
        for t in fg_params:
            n_ = [k for k, v in pd.items() if v is t][0]
            res[n_] = fg.flat[off:off + t.numel()].view_as(t).clone()
            off += t.numel()
        q.put((rank, float(loss), {k: v.numpy() for k, v in res.items()}))
    finally:
        dist.destroy_process_group()


def test_two_rank_global_ccc_and_grad_allreduce_match_dataparallel():
    ref_loss, ref_grads = _dataparallel_reference()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    out = [q.get(timeout=300) for _ in range(2)]
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    gmax = max(float(r.abs().max()) for r in ref_grads.values())
    for rank, loss, grads in out:
        assert abs(loss - ref_loss) < 1e-6, (rank, loss, ref_loss)
        assert set(grads) == set(ref_grads)
        for k, g in grads.items():
            r = ref_grads[k]
            err = float((torch.from_numpy(g) - r).abs().max())
            # fp32 summation-order noise; the floor covers cancellation-dominated bias grads
            assert err <= 1e-3 * max(float(r.abs().max()), 0.01 * gmax), (k, err)


def test_shard_pairing_equals_dataparallel_gather():
    """Per-rank (T, B/g) flatten + local (B/g, T) labels == DataParallel's dim-0 gather of the
    (T, B/g) chunks paired with the global (B, T) labels."""
    from jmt import dist as jdist
    T_, B_, g = 5, 6, 3
    preds = torch.arange(B_ * T_).reshape(B_, T_).t().float()     # (T, B) values = b*T + t
    labels = torch.arange(B_ * T_).reshape(B_, T_).float()
    gathered = torch.cat([preds[:, jdist.shard_range(B_, r, g)[0]:jdist.shard_range(B_, r, g)[1]]
                          for r in range(g)], 0).reshape(-1)
    pairs_dp = set(zip(gathered.tolist(), labels.reshape(-1).tolist()))
    pairs_rank = set()
    for r in range(g):
        lo, hi = jdist.shard_range(B_, r, g)
        pairs_rank |= set(zip(preds[:, lo:hi].reshape(-1).tolist(),
                              labels[lo:hi].reshape(-1).tolist()))
    assert pairs_dp == pairs_rank


class _FakeOpt:
    """The slice of FusedSGD that GradBucketer reads: params, their flat offsets, flat_g."""

    def __init__(self, sizes):
        self.params = [torch.nn.Parameter(torch.zeros(n)) for n in sizes]
        self.offsets, n = [], 0
        for p in self.params:
            self.offsets.append(n)
            n += -(-p.numel() // 64) * 64
        self.flat_g = torch.zeros(n)


def _bucket_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from jmt import dist as jdist
        from jmt import functional as JF
        sizes = [300, 70, 1000, 5, 64, 2000]
        opt = _FakeOpt(sizes)
        counts = {id(p): c for p, c in zip(opt.params, [1, 2, 1, 3, 1, 1])}
        b = jdist.GradBucketer(opt, counts, bucket_bytes=1200 * 4)
        logs = []
        for step in range(2):
            opt.flat_g.zero_()
            b.begin()
            # a backward's writes, in the layout order, some parameters written several times
            for i, p in enumerate(opt.params):
                off = opt.offsets[i]
                for w in range(counts[id(p)]):
                    opt.flat_g[off:off + p.numel()] += (rank + 1) * (i + 1) * (w + 1)
                    JF._grad_done(p)
                logs.append((step, i, list(b.launch_log)))
            b.finish()
            q.put((rank, step, opt.flat_g.clone().numpy(), b.buckets, logs))
        b.close()
    finally:
        dist.destroy_process_group()


def test_grad_bucketer_launches_each_bucket_when_complete_and_sums():
    """jmt.dist.GradBucketer on two gloo ranks: buckets are contiguous and >= the byte size, a
    bucket is issued exactly when the last write of its last parameter is notified (never
    before: that would reduce a half-written gradient), and after finish() every rank holds
    the SUM over ranks."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bucket_worker, args=(r, 2, port, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    out = [q.get(timeout=300) for _ in range(4)]
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    sizes = [300, 70, 1000, 5, 64, 2000]
    counts = [1, 2, 1, 3, 1, 1]
    for rank, step, flat, buckets, logs in out:
        # params 0-2 (1370 floats) close bucket 0, 3-5 the last one
        assert [(b[2]) for b in buckets] == [3, 3]
        assert buckets[0][0] == 0 and buckets[0][1] == buckets[1][0]
        for st, i, launched in logs:
            if st != step:
                continue
            assert launched == ([] if i < 2 else [0] if i < 5 else [0, 1]), (i, launched)
        off = 0
        for i, n in enumerate(sizes):
            want = sum((r + 1) * (i + 1) * (w + 1) for r in range(2) for w in range(counts[i]))
            assert np.all(flat[off:off + n] == want), (i, flat[off], want)
            off += -(-n // 64) * 64
