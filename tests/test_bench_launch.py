"""bench.py as its own multi-rank launcher (the reference scales to every
visible GPU by itself, main.py:487-491, tools.py:16-21): `python bench.py --gpus N` without
torchrun's environment starts N ranks, relays rank 0's JSON line and fails if a rank fails.
CPU tests drive the launcher with a stand-in worker (tests/_fake_rank.py) and the real bench.py
up to its first GPU call; the GPU test runs the real 2-rank bench over gloo on one GPU."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FAKE = os.path.join(REPO, "tests", "_fake_rank.py")
BENCH = os.path.join(REPO, "bench.py")


def _bench():
    sys.path.insert(0, REPO)
    import bench
    return bench


def test_launcher_relays_rank0_json_and_rank_logs(capsys, monkeypatch):
    b = _bench()
    monkeypatch.delenv("FAKE_RANK_FAIL", raising=False)
    monkeypatch.delenv("FAKE_RANK_NGPUS", raising=False)
    rc = b.launch_ranks(3, ["--steps", "2"], script=FAKE, backend="gloo")
    out, err = capsys.readouterr()
    assert rc == 0
    lines = [ln for ln in out.splitlines() if ln.strip()]
    assert len(lines) == 1                                   # ONE JSON line on stdout
    j = json.loads(lines[0])
    assert j["n_gpus"] == 3 and j["launcher"] == "bench.py" and j["backend"] == "gloo"
    for r in range(3):                                       # every rank's log, prefixed
        assert f"[rank {r}] rank {r}/3 local {r} master 127.0.0.1:" in err
    assert "['--steps', '2']" in err
    assert "[rank 0] plain text on rank 0's stdout" in err


@pytest.mark.parametrize("bad_rank", [0, 1])
def test_launcher_fails_when_a_rank_fails(capsys, monkeypatch, bad_rank):
    b = _bench()
    monkeypatch.setenv("FAKE_RANK_FAIL", str(bad_rank))
    rc = b.launch_ranks(2, [], script=FAKE, backend="gloo")
    out, err = capsys.readouterr()
    assert rc == 3
    assert out.strip() == ""                                 # no bench line from a failed job
    assert f"rank {bad_rank} exited with status 3" in err


def test_launcher_rejects_wrong_n_gpus(capsys, monkeypatch):
    b = _bench()
    monkeypatch.delenv("FAKE_RANK_FAIL", raising=False)
    monkeypatch.setenv("FAKE_RANK_NGPUS", "1")
    rc = b.launch_ranks(2, [], script=FAKE, backend="gloo")
    out, err = capsys.readouterr()
    assert rc == 1 and out.strip() == "" and "n_gpus=1" in err


def test_launcher_needs_one_gpu_per_rccl_rank(capsys, monkeypatch):
    b = _bench()
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,1")
    assert b.visible_gpus() == 2
    assert b.launch_ranks(3, [], script=FAKE, backend="nccl") == 2
    assert "RCCL needs one rank per GPU" in capsys.readouterr().err


def test_visible_gpus_reads_env_before_sysfs(monkeypatch):
    b = _bench()
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(var, raising=False)
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "3,5,7")
    assert b.visible_gpus() == 3
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "")
    assert b.visible_gpus() == 0
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "-1")
    assert b.visible_gpus() == 0


def test_launcher_parent_never_initialises_hip():
    """the parent that starts the ranks must not be able to initialise HIP
    (on ROCm torch.cuda.device_count() falls back to hipGetDeviceCount when amdsmi fails).  In a
    child interpreter every torch.cuda entry that could reach HIP raises; launch_ranks with the
    stand-in worker still succeeds and torch.cuda was never initialised."""
    code = f"""
import sys, torch
def boom(*a, **k):
    raise AssertionError("launcher parent touched torch.cuda")
for name in ("device_count", "is_available", "init", "_lazy_init", "current_device",
             "set_device", "synchronize", "get_device_properties"):
    setattr(torch.cuda, name, boom)
sys.path.insert(0, {REPO!r})
import bench
rc = bench.launch_ranks(2, [], script={FAKE!r}, backend="nccl")
assert not torch.cuda.is_initialized()
sys.exit(rc)
"""
    env = dict(os.environ, HIP_VISIBLE_DEVICES="0,1")
    env.pop("FAKE_RANK_FAIL", None)
    env.pop("FAKE_RANK_NGPUS", None)
    r = subprocess.run([sys.executable, "-c", code], env=env, text=True, capture_output=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert json.loads(r.stdout.strip().splitlines()[-1])["n_gpus"] == 2


def test_launcher_deadline_terminates_hung_ranks(capsys, monkeypatch):
    """ranks that hang without exiting (e.g. in a collective) are terminated at the
    job deadline and the launcher exits 124 with no bench line."""
    b = _bench()
    monkeypatch.delenv("FAKE_RANK_FAIL", raising=False)
    monkeypatch.setenv("FAKE_RANK_HANG", "1")
    rc = b.launch_ranks(2, [], script=FAKE, backend="gloo", deadline_s=3.0)
    out, err = capsys.readouterr()
    assert rc == 124 and out.strip() == ""
    assert "still running after 3 s" in err


def _run_bench(args, env_extra, timeout=240):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra)
    return subprocess.run([sys.executable, BENCH] + args, cwd=REPO, env=env, text=True,
                          capture_output=True, timeout=timeout)


def test_bench_world_size_must_match_gpus():
    r = _run_bench(["--gpus", "4"], {"WORLD_SIZE": "2", "RANK": "0"}, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=2 but --gpus 4" in r.stderr


@pytest.mark.skipif(__import__("torch").cuda.is_available(), reason="CPU-only: ranks must fail")
def test_bench_gpus2_on_cpu_box_launches_two_ranks_and_fails_loudly():
    # the real bench.py: without a GPU both ranks fail at their first GPU call; the launcher
    # shows both ranks' logs and exits non-zero with no bench line
    r = _run_bench(["--gpus", "2", "--steps", "1", "--warmup", "0"],
                   {"JMT_DIST_BACKEND": "gloo"})
    assert r.returncode != 0
    assert r.stdout.strip() == ""
    assert "[rank 0]" in r.stderr and "[rank 1]" in r.stderr


@pytest.mark.gpu
def test_bench_gpus2_gloo_on_one_gpu():
    """`python bench.py --gpus 2` (no torchrun): two gloo ranks on cuda:0 run the eager bucketed
    step, rank 0 relays n_gpus 2 with parity passing, both ranks log."""
    r = _run_bench(["--gpus", "2", "--steps", "3", "--warmup", "1", "--batch", "4",
                    "--probe-steps", "1", "--no-cpu-baseline"],
                   {"JMT_DIST_BACKEND": "gloo"}, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1
    j = json.loads(lines[0])
    assert j["n_gpus"] == 2 and j["launcher"] == "bench.py" and j["dist_backend"] == "gloo"
    assert j["graph"] is True and "segments" in j["graph_kind"]   # N > 1: segmented graph
    assert j["config"]["global_batch"] == 8
    assert j["parity"]["pass"], j["parity"]
    assert "[rank 0] rank 0/2" in r.stderr and "[rank 1] rank 1/2" in r.stderr


class _Ev:
    def __init__(self, t):
        self.t = t

    def elapsed_time(self, other):
        return other.t - self.t


def _probe_with(seq_per_step):
    b = _bench()
    pr = b.FamilyProbe()
    for step, seq in enumerate(seq_per_step):
        for fam, ms in seq:
            pr.rec.append((fam, 1e9, None, (_Ev(0.0), _Ev(ms))))
            pr.cal.append(((_Ev(0.0), _Ev(0.010)), (_Ev(0.0), _Ev(0.020))))
    return pr


def test_family_probe_per_position_medians_need_identical_sequences():
    """the per-position medians are taken only when every probe step issued the same
    (family, flops) sequence; a different sequence with the same length falls back to the
    per-launch sum (flagged in the summary)."""
    same = [[("gemm_nt", 0.1), ("gemm_nn", 0.2)]] * 3
    s = _probe_with(same).summary(3)
    assert s["per_position_medians"] is True
    fam = {f["family"]: f for f in s["families"]}
    assert fam["gemm_nt"]["launches_per_step"] == 1 and fam["gemm_nn"]["launches_per_step"] == 1
    diff = [[("gemm_nt", 0.1), ("gemm_nn", 0.2)], [("gemm_nn", 0.2), ("gemm_nt", 0.1)],
            [("gemm_nt", 0.1), ("gemm_nn", 0.2)]]
    s = _probe_with(diff).summary(3)
    assert s["per_position_medians"] is False
    fam = {f["family"]: f for f in s["families"]}
    assert fam["gemm_nt"]["launches_per_step"] == 1 and fam["gemm_nn"]["launches_per_step"] == 1
    assert abs(fam["gemm_nn"]["avg_launch_us_raw"] - 200.0) < 1e-6
