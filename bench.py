"""Training-step throughput of the JMT fusion hot path on MI355X (BASELINE.json metric:
"train windows/sec + CCC parity, B=64 T=300 A/V fusion, 1/2/4/8 MI355X").

Workload (BASELINE.json configs[2], the one the metric is quoted on): per GPU B=64 windows of
T=300 synthetic backbone features (audio D_a=1024, video D_v=2048, N(0,1), resident in HBM),
FcLayer(1024,512) on the audio (main.py:379) -> Two_transformers(0,0,H=1,L=1,'TRANSFORMER','FC',
vision_in_ft=2048) -> 2x losses.loss.CCCLoss(1) (global-batch statistics) -> backward -> RCCL
all-reduce of the flat gradient (N>1) -> fused SGD-nesterov step (config_file.json:73-80).
Random-init weights.  bf16 MFMA compute, fp32 master weights / statistics.

    python bench.py [--gpus N] [--steps K] [--warmup W]      (N > 1: starts N ranks itself)
    torchrun --nproc-per-node N bench.py --gpus N ...        (or one rank per GPU via torchrun)

One process per GPU either way (RCCL).  The reference scales to every visible GPU by itself
(main.py:487-491 wraps the model in DataParallel, tools.py:16-21); `--gpus N` without torchrun's
environment makes this script the launcher: it starts N worker processes of itself before any
GPU call, relays rank 0's JSON line and fails if any rank fails.

Prints ONE JSON line (rank 0).  `value` = windows/s of the whole job (weak scaling: B=64 per GPU).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "joint-multimodal-transformer-6th-abaw_amd")
for _p in (REPO, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

PROFILE_TAG = "r06"            # profiles/<tag>_pmc_bench/ (PMC traffic), <tag>_family_trace.json
PEAK_BF16_TFLOPS = 2516.6      # 256 CU x 4 SIMD x 1024 flop/clk (16x16x32 bf16 / 16 cyc) x 2.4 GHz
PEAK_HBM_GBS = 8000.0
D_A, D_V, E = 1024, 2048, 512


# workloads (BASELINE.json configs): the metric is quoted on c3; the others are parity /
# profiling cases (`--config`)
CONFIGS = {
    "c3": dict(B=64, T=300, Da=1024, Dv=2048, fc=True, jm="TRANSFORMER", fmt="FC", dtype="bf16",
               desc="configs[2]: FcLayer(1024,512) + Two_transformers(TRANSFORMER,FC,H=1,L=1,"
                    "vision_in_ft=2048) + 2x CCCLoss + SGD-nesterov"),
    "c3sa": dict(B=64, T=300, Da=1024, Dv=2048, fc=True, jm="TRANSFORMER", fmt="SELF_ATTEN",
                 dtype="bf16", desc="configs[2] with output_format=SELF_ATTEN"),
    "c2": dict(B=32, T=300, Da=1024, Dv=2048, fc=True, jm="NONE", fmt="FC", dtype="bf16",
               desc="configs[1]: FcLayer(1024,512) + Two_transformers(NONE,FC) (mm_transformers)"),
    "c4": dict(B=16, T=1024, Da=1024, Dv=2048, fc=True, jm="TRANSFORMER", fmt="FC", dtype="bf16",
               desc="configs[3]: long window T=1024, TRANSFORMER/FC"),
    "c5": dict(B=128, T=300, Da=1024, Dv=2048, fc=True, jm="TRANSFORMER", fmt="FC", dtype="fp16",
               digitize=20,
               desc="configs[4]: B=128 fp16 TRANSFORMER/FC, expression-style head: 20-bin V/A "
                    "logits + losses.loss.CCCLoss(digitize_num=20) (loss.py:14-22)"),
    "realdata": dict(B=64, T=16, Da=512, Dv=512, fc=False, jm="TRANSFORMER", fmt="FC",
                     dtype="bf16", desc="shipped config_file.json: T=16 clips (512/32), R2D1 + "
                                        "ResNet18 features (512), Two_transformers(TRANSFORMER,"
                                        "FC,vision_in_ft=512)"),
}


def synthetic_batch(B: int, T: int, Da: int, Dv: int, rank: int, dev):
    """Rank `rank`'s B windows of synthetic data: audio / video ~ N(0,1), labels ~ U(-1,1), one
    generator per GLOBAL window index, so rank r holds windows [r*B, (r+1)*B)
    and the 1/2/4/8-GPU runs see identical global batches.  Labels come as the (1, B*T) views
    train.py:303-307 makes."""
    audio = torch.empty(B, T, Da, device=dev)
    video = torch.empty(B, T, Dv, device=dev)
    lv = torch.empty(B, T, device=dev)
    la = torch.empty(B, T, device=dev)
    for i in range(B):
        g = torch.Generator(device=dev).manual_seed(1000 + rank * B + i)
        audio[i].normal_(generator=g)
        video[i].normal_(generator=g)
        lv[i].uniform_(-1.0, 1.0, generator=g)
        la[i].uniform_(-1.0, 1.0, generator=g)
    return audio, video, lv.view(-1, B * T), la.view(-1, B * T)


def step_flops(B: int, T: int, Da: int = D_A, Dv: int = D_V, fc: bool = True,
               jm: str = "TRANSFORMER", fmt: str = "FC", k: int = 1):
    """Algorithmic matmul FLOPs of one training step (SURVEY.md §8d closed form for
    TRANSFORMER/FC, L=1, h=d): F per window = input projections + out_layer_pv + 3 encoders +
    6 cross-attentions + out_layer1 + regressors; W = 3F minus the input gradients of the
    projections that act on leaf inputs.  SELF_ATTEN swaps out_layer1 for its head.
    NONE (MultimodalTransformer_wo_JR, mm_transformers.py:119-146): 2 encoders whose
    self-attention runs over the BATCH axis (a length-B sequence per time step: 4 B d FLOP per
    token), 2 cross-attentions over T, final_layer 1024->512, regressors over 512.
    FC (FeatureConcatFC, mm_multi_transformers.py:217-224): one 1024->512 linear + regressors."""
    d = E
    proj = (2 * T * d * Da if fc else 0) + (2 * T * d * Dv if Dv != 512 else 0)
    reg = lambda dim: 4 * T * dim * 128 + 4 * T * 128 * k          # V and A regressors
    if jm == "NONE" and fmt == "FC":
        F = (proj + 2 * (12 * T * d * d + 4 * T * B * d) + 2 * (8 * T * d * d + 4 * T * T * d)
             + 4 * T * d * d + reg(512))
        leaf = proj if proj else 12 * T * d * d       # else: the encoders' qkv input gradients
        return (3 * F - leaf) * B
    if jm == "FC" and fmt == "FC":
        F = proj + 4 * T * d * d + reg(512)
        leaf = proj if proj else 4 * T * d * d
        return (3 * F - leaf) * B
    if jm != "TRANSFORMER" or fmt not in ("FC", "SELF_ATTEN"):
        return None
    F = (proj + 4 * T * d * d + 3 * (12 * T * d * d + 4 * T * T * d)
         + 6 * (8 * T * d * d + 4 * T * T * d))
    if fmt == "FC":
        F += 24 * T * d * d + reg(1024)               # out_layer1 + regressors (1024)
    else:
        # SELF_ATTEN head (mm_multi_transformers.py:169-199): an encoder layer over the 6
        # cross-attention outputs of every clip, then MHA with the last token as the only query
        # row that is kept (q: 1 token, k/v: 6 tokens, out_proj: 1 token); regressors over 512
        F += 6 * T * (12 * d * d + 4 * 6 * d) + T * (2 * d * d + 24 * d * d + 4 * 6 * d
                                                    + 2 * d * d) + reg(512)
    leaf = proj if proj else 4 * T * d * d + 2 * 6 * T * d * d
    return (3 * F - leaf) * B


class FamilyProbe:
    """In-step timing of the step's kernel families over eager probe steps (right after the
    timed region, same data and weights): one HIP event pair around EVERY launch of a family
    (GEMM NT / NN / TN by operand majorness, fused attention forward / backward), recorded on
    the stream the launch goes to (torch's current stream: the grouped path launches everything
    there).  An event pair reads above the kernel's own duration (the dispatch after the start
    marker and the end-of-kernel flush fall inside it: profiles/r01_event_check.txt), so each
    launch is followed by two calibration pairs around empty launches (jmt_noop): one around a
    single empty launch, one around two back to back.  overhead = pair(1) - (pair(2) - pair(1))
    (the pair's fixed cost without the empty kernel's own execution) is subtracted from every
    launch's reading.  Every pair is preceded by a GPU spin (torch.cuda._sleep), so the start
    marker is stamped only after the host has queued the launch behind it: without it an
    issue-bound step (small shapes, eager Python) puts the host's issue gap inside the pair."""

    def __init__(self):
        self.on = False
        self.rec = []
        self.cal = []
        self.info = []

    SLEEP_CYCLES = 200000     # ~80 us spin ahead of each pair (torch.cuda._sleep)

    @staticmethod
    def _pair(fn):
        # the GPU is kept busy while the host issues marker + launch + marker, so the pair
        # times the kernel and not the host's issue latency (small launches are issue-bound)
        torch.cuda._sleep(FamilyProbe.SLEEP_CYCLES)
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        r = fn()
        e.record()
        return r, (s, e)

    def __call__(self, info, launch):
        if not self.on:
            return launch()
        from jmt import ops
        r, ev = self._pair(launch)
        self.rec.append((info["family"], info["flops"], info.get("bytes"), ev))
        self.info.append({k: v for k, v in info.items() if isinstance(v, (int, float, str, bool))})
        _, e1 = self._pair(ops.noop)
        _, e2 = self._pair(lambda: (ops.noop(), ops.noop()))
        self.cal.append((e1, e2))
        return r

    def summary(self, probe_steps: int):
        if not self.rec:
            return None
        import statistics
        ms = lambda ev: ev[0].elapsed_time(ev[1])
        one = statistics.median(ms(a) for a, _ in self.cal)
        two = statistics.median(ms(b) for _, b in self.cal)
        over = max(0.0, one - (two - one))
        fam = {}
        # every probe step launches the same sequence: each launch position is timed by the
        # median over the probe steps (one disturbed launch does not move its family), then
        # summed per family as if each step had run at those medians.  Checked: the family and
        # flop count of every position agree across the steps; otherwise the per-launch sum
        n = len(self.rec) // probe_steps if len(self.rec) % probe_steps == 0 else 0
        if n and any(self.rec[k * n + i][:2] != self.rec[i][:2]
                     for k in range(1, probe_steps) for i in range(n)):
            n = 0
        same_sequence = bool(n)
        med = [statistics.median(ms(self.rec[k * n + i][3]) for k in range(probe_steps))
               for i in range(n)] if n else [ms(r[3]) for r in self.rec]
        for i, (f, fl, by, ev) in enumerate(self.rec[:n] if n else self.rec):
            d = fam.setdefault(f, {"launches": 0, "ms": 0.0, "ms_raw": 0.0, "flops": 0.0,
                                   "bytes": 0.0})
            w = probe_steps if n else 1                # per-step medians stand for every step
            d["launches"] += w
            d["ms_raw"] += w * med[i]
            d["ms"] += w * max(med[i] - over, 1e-6)
            d["flops"] += w * fl
            d["bytes"] += w * (by or 0.0)
        out = []
        for f, d in fam.items():
            tf = d["flops"] / (d["ms"] * 1e-3) / 1e12
            out.append({"family": f, "launches_per_step": d["launches"] / probe_steps,
                        "ms_per_step": round(d["ms"] / probe_steps, 4),
                        "avg_launch_us": round(d["ms"] / d["launches"] * 1e3, 2),
                        "avg_launch_us_raw": round(d["ms_raw"] / d["launches"] * 1e3, 2),
                        "gflop_per_launch": round(d["flops"] / d["launches"] / 1e9, 3),
                        "algorithmic_bytes_per_launch": round(d["bytes"] / d["launches"]),
                        "tflops": round(tf, 1), "frac": round(tf / PEAK_BF16_TFLOPS, 4)})
            if f.startswith(("small_attn", "attn_short", "attn_bwd", "attn_dkdv")):
                # HBM-bound families: algorithmic bytes per launch (jmt.ops hooks).  The attention
                # backward pair at dh = 512 moves ~92 FLOP per byte (Q, dO, O, K, V read, P / dS
                # handed over) against a machine balance of ~400: its roofline is HBM, the MFMA
                # fraction beside it is the secondary view
                gbs = d["bytes"] / (d["ms"] * 1e-3) / 1e9
                out[-1].update({"bound": "hbm", "gbps": round(gbs, 1),
                                "hbm_frac": round(gbs / PEAK_HBM_GBS, 4)})
        out.sort(key=lambda r: -r["ms_per_step"])
        return {"families": out, "event_pair_overhead_us": round(over * 1e3, 2),
                "per_position_medians": same_sequence}

    def dump(self, path: str, probe_steps: int):
        """Per-launch records of the last probe step (shape, family, overhead-corrected us)."""
        import statistics
        ms = lambda ev: ev[0].elapsed_time(ev[1])
        one = statistics.median(ms(a) for a, _ in self.cal)
        two = statistics.median(ms(b) for _, b in self.cal)
        over = max(0.0, one - (two - one))
        n = len(self.rec) // probe_steps
        with open(path, "w") as f:
            for (fam, fl, by, ev), info in zip(self.rec[-n:], self.info[-n:]):
                us = max(ms(ev) - over, 1e-6) * 1e3
                info = dict(info, us=round(us, 2), tflops=round(fl / us / 1e6, 1))
                f.write(json.dumps(info) + "\n")


def parity_check(model, fc, audio, video, lv, la, cd, jm, fmt, Dv, nwin=2, k=1, H=1, L=1):
    """BASELINE.json's '+ CCC parity': the GPU predictions and CCC losses in the compute dtype
    vs the CPU oracle (oracle/jmt_ref.py, fp32, pinned by the reference goldens) on the first
    `nwin` windows of the bench batch with the trained weights (north_star: 1e-2 bf16)."""
    from oracle import jmt_ref as R
    from jmt import functional as JF
    from losses.loss import CCCLoss
    crit = CCCLoss(k)
    flat = (lambda o: o.reshape(-1, k)) if k > 1 else (lambda o: o.reshape(1, -1))
    from jmt import dist as jdist
    a, v = audio[:nwin], video[:nwin]
    T = a.shape[1]
    group = jdist.loss_group()
    jdist.set_loss_group(None)       # rank 0 alone: local statistics, no collective
    yv = lv.view(audio.shape[0], T)[:nwin]
    ya = la.view(audio.shape[0], T)[:nwin]
    with torch.no_grad(), JF.compute_mode(cd):
        vo, ao = model(fc(a) if fc is not None else a, v)
        gl1 = float(crit(flat(vo), yv.reshape(1, -1)))
        gl2 = float(crit(flat(ao), ya.reshape(1, -1)))
    jdist.set_loss_group(group)
    p = {k: t.detach().float().cpu() for k, t in model.state_dict().items()}
    with torch.no_grad():
        ac = a.float().cpu()
        if fc is not None:
            fp = {k: t.detach().float().cpu() for k, t in fc.state_dict().items()}
            ac = R.linear(ac, fp["fc_layer.weight"], fp["fc_layer.bias"])
        rvo, rao = R.two_transformers_forward(ac, v.float().cpu(), p, H, L, jm, fmt, Dv)
        rl1 = float(R.ccc_loss(flat(rvo), yv.cpu().reshape(1, -1), digitize_num=k))
        rl2 = float(R.ccc_loss(flat(rao), ya.cpu().reshape(1, -1), digitize_num=k))
    err = max(float((vo.float().cpu() - rvo).abs().max()), float((ao.float().cpu() - rao).abs().max()))
    lerr = max(abs(gl1 - rl1), abs(gl2 - rl2))
    return {"reference": "oracle/jmt_ref.py fp32 CPU, same weights (after the timed steps) and "
                         f"windows 0..{nwin - 1} of the bench batch",
            "pred_max_abs_err": float(f"{err:.3g}"), "loss_max_abs_err": float(f"{lerr:.3g}"),
            "pred_abs_max": float(f"{float(max(rvo.abs().max(), rao.abs().max())):.3g}"),
            "tolerance": 1e-2, "pass": bool(err <= 1e-2 and lerr <= 1e-2)}


NORTH_STAR_TOL = {torch.float32: 1e-4, torch.bfloat16: 1e-2, torch.float16: 1e-2}
RATIO_TO_EMULATED_BOUND = 1.25


def north_star_key(cd) -> str:
    name = {torch.float32: "fp32", torch.bfloat16: "bf16", torch.float16: "fp16"}[cd]
    return f"north_star_{name}_{NORTH_STAR_TOL[cd]:g}"


def north_star_verdict(own: dict, cd, strict: dict = None) -> dict:
    """BASELINE.json north_star: "logits/VA predictions that match the reference CPU path within
    1e-4 fp32 / 1e-2 bf16 on fixed seeds".  The measure is the ABSOLUTE prediction error on the
    bench's fixed-seed batch (windows 0-1, the bench model's weights after the timed steps) vs the
    fp32 oracle; the spread-relative error of the discriminative check (conditioned weights whose
    predictions spread O(1), every gradient under its own strict bound) is reported beside it
    against the same number, as its own verdict."""
    tol = NORTH_STAR_TOL[cd]
    out = {"verdict": "pass" if own["pred_max_abs_err"] <= tol else "fail",
           "measure": "max |pred_gpu - pred_oracle| over the V and A predictions (absolute), "
                      "bench batch windows 0-1, fixed seeds, the bench model's weights",
           "value": own["pred_max_abs_err"], "tolerance": tol,
           "pred_abs_max": own["pred_abs_max"]}
    if strict is not None and "pred_max_abs_err" in strict:
        ab = strict["pred_max_abs_err"]
        out["conditioned"] = {
            "verdict": "pass" if ab <= tol else "fail", "value": ab, "tolerance": tol,
            "measure": "the same absolute error on the windows of the strict window-subset "
                       "check (conditioned hash-init weights, predictions spread O(0.1))",
            "rel_to_spread": strict["pred_abs_err_rel_to_spread"],
            "rounding_emulating_oracle_rel_to_spread": strict.get("pred_emulated_rel_to_spread"),
            "note": "relative to the spread no bf16 path is within 1e-2 on these weights: the "
                    "oracle with only its storage rounded to bf16 is at the value above"}
        emu = strict.get("pred_emulated_rel_to_spread")
        if emu:
            # the GPU's spread-relative error over the rounding-emulating
            # oracle's, tracked every round (bound 1.25: kernel changes must not drift it up)
            ratio = strict["pred_abs_err_rel_to_spread"] / emu
            out["conditioned"]["ratio_to_emulated"] = round(ratio, 3)
            out["conditioned"]["ratio_bound"] = RATIO_TO_EMULATED_BOUND
            out["conditioned"]["ratio_verdict"] = \
                "pass" if ratio <= RATIO_TO_EMULATED_BOUND else "fail"
            out["verdict_spread_relative"] = out["conditioned"]["ratio_verdict"]
    return out


def cpu_threads():
    """Threads for the CPU baseline: the box's CPU share (OMP_NUM_THREADS, 16 per GPU on the
    GPU pool, whose nproc shows the whole machine) or the affinity set."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    env = os.environ.get("OMP_NUM_THREADS")
    return (max(1, min(int(env), aff)) if env and env.isdigit() else aff), aff


def cpu_baseline(model_sd, fc_sd, audio, video, lv, la, steps=2):
    """The oracle (CPU restatement, oracle/jmt_ref.py) timed on this host: fp32 torch-CPU
    forward+backward+SGD of the SAME training step (rank 0's batch, the initial weights),
    1 warm-up + `steps` timed steps."""
    from oracle import jmt_ref as R
    threads, aff = cpu_threads()
    torch.set_num_threads(threads)
    B, T = audio.shape[0], audio.shape[1]
    a, v = audio.float().cpu(), video.float().cpu()
    yv, ya = lv.float().cpu().view(B, T), la.float().cpu().view(B, T)
    p = {k: t.detach().float().cpu().clone() for k, t in model_sd.items()}
    fp = {k: t.detach().float().cpu().clone() for k, t in fc_sd.items()}
    bufs = {}
    times = []
    for i in range(steps + 1):
        t0 = time.perf_counter()
        R.train_step(p, fp, a, v, yv, ya, 1, 1, "TRANSFORMER", "FC", v.shape[-1], bufs)
        times.append(time.perf_counter() - t0)
    t = sum(times[1:]) / steps
    return {"value": round(B / t, 3), "unit": "windows/s", "cores": threads, "kind": "port",
            "sample": f"oracle/jmt_ref.py train_step on the bench batch (B={B} T={T}, rank 0's "
                      f"data, initial weights), fp32 torch-CPU, {threads} threads, 1 warm-up + "
                      f"{steps} timed steps ({t * 1e3:.0f} ms/step)",
            "threads_policy": f"{threads} = OMP_NUM_THREADS, the CPU share the GPU pool gives one "
                              f"GPU's job; the affinity mask ({aff} CPUs) is the whole host, "
                              "shared with the other GPU slots, so it is not used"}


def visible_gpus():
    """GPUs this process may use, WITHOUT initialising HIP (the launcher parent must not touch the
    GPU before it starts its ranks): the first of HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES /
    CUDA_VISIBLE_DEVICES that is set, else the GPU nodes of the KFD topology in sysfs (nodes with
    a non-zero gpu_id; CPU nodes have 0).  None when neither says (the ranks then check)."""
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            return len([d for d in v.split(",") if d.strip() not in ("", "-1")])
    root = "/sys/class/kfd/kfd/topology/nodes"
    try:
        n = 0
        for node in os.listdir(root):
            with open(os.path.join(root, node, "gpu_id")) as f:
                n += int(f.read().strip() or 0) != 0
        return n
    except (OSError, ValueError):
        return None


def launch_ranks(n: int, argv, script: str = None, backend: str = None,
                 deadline_s: float = None) -> int:
    """Start `n` worker processes of `script` (this file) with torchrun's environment (RANK,
    LOCAL_RANK, WORLD_SIZE, MASTER_ADDR=127.0.0.1, a free MASTER_PORT), one per GPU, and wait.
    Called before anything touches the GPU (torch.cuda.device_count() does not initialise it on
    ROCm), and the workers are children, never an exec of this process.  Rank 0's stdout lines
    that are JSON objects are held back and printed on stdout once every rank has exited 0 (the
    ONE bench line); every other line of every rank goes to stderr prefixed "[rank r]", as it
    comes (the ranks' logs, and a sign of life for long runs).  Returns the exit status: 0 only
    if every rank exited 0 and rank 0 printed a JSON line whose n_gpus is `n`; when one rank
    fails the others are terminated (their own PIDs) after a grace period, and so are all of them
    when the job outlives `deadline_s` (a rank hung in a collective; exit status 124).  The
    parent never initialises HIP: the GPU count comes from visible_gpus()."""
    import socket
    import subprocess
    import threading
    backend = backend or os.environ.get("JMT_DIST_BACKEND", "nccl")
    ndev = visible_gpus()
    if backend == "nccl" and ndev is not None and ndev < n:
        print(f"bench.py --gpus {n}: only {ndev} GPU(s) visible; RCCL needs one rank per GPU "
              "(JMT_DIST_BACKEND=gloo rehearses N ranks on fewer GPUs)", file=sys.stderr)
        return 2
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    script = script or os.path.abspath(__file__)
    procs, lines = [], []
    lock = threading.Lock()

    def pump(r, stream):
        for line in stream:
            if r == 0 and line.lstrip().startswith("{"):
                with lock:
                    lines.append(line.rstrip("\n"))
                continue
            sys.stderr.write(f"[rank {r}] {line}")
            sys.stderr.flush()

    threads = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), JMT_DIST_BACKEND=backend, JMT_LAUNCHER="bench.py")
        p = subprocess.Popen([sys.executable, "-u", script] + list(argv), env=env,
                             stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                             bufsize=1)
        procs.append(p)
        t = threading.Thread(target=pump, args=(r, p.stdout), daemon=True)
        t.start()
        threads.append(t)
    failed = None
    t_end = None if deadline_s is None else time.time() + deadline_s
    while True:
        codes = [p.poll() for p in procs]
        bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
        if bad:
            failed = bad[0]
            break
        if all(c == 0 for c in codes):
            break
        if t_end is not None and time.time() > t_end:
            failed = (next(r for r, c in enumerate(codes) if c is None), 124)
            print(f"bench.py --gpus {n}: ranks still running after {deadline_s:.0f} s; "
                  "terminating them", file=sys.stderr)
            break
        time.sleep(0.2)
    if failed is not None:
        deadline = time.time() + (0.0 if failed[1] == 124 else 30.0)
        while time.time() < deadline and any(p.poll() is None for p in procs):
            time.sleep(0.2)
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=15)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    for t in threads:
        t.join(timeout=5)
    if failed is not None:
        print(f"bench.py --gpus {n}: rank {failed[0]} exited with status {failed[1]}",
              file=sys.stderr)
        return failed[1] if failed[1] > 0 else 1
    if not lines:
        print(f"bench.py --gpus {n}: rank 0 printed no JSON line", file=sys.stderr)
        return 1
    try:
        got = json.loads(lines[-1]).get("n_gpus")
    except ValueError:
        got = None
    if got != n:
        print(f"bench.py --gpus {n}: rank 0 reported n_gpus={got}", file=sys.stderr)
        return 1
    print(lines[-1], flush=True)
    return 0


def _rank0_legs(args, cfg, cd, k, heads, layers, B, T, Da, Dv, model, fc, audio, video, lv, la,
                rank, world, jcfg, model_sd0, fc_sd0):
    """Rank 0's parity check and CPU baseline after the timed region (local CCC statistics: the
    caller has taken the loss group away and restores it even if these raise)."""
    parity = None
    if rank == 0:
        if (cfg["jm"], cfg["fmt"], cfg["fc"], k, heads, layers, Dv, Da) == \
                ("TRANSFORMER", "FC", True, 1, 1, 1, 2048, 1024) and cd != torch.float32 and \
                T == 300 and B >= 4:
            # discriminative form: conditioned weights, the bench shape,
            # every parameter gradient under the strict 16-bit bound (tests/parity.py)
            from tests.parity import window_subset_check
            torch.set_num_threads(cpu_threads()[0])
            win = (0, B // 3, (2 * B) // 3, B - 1)
            parity = window_subset_check(cd, B=B, T=T, win=win, perturb=args.parity_perturb)
            parity["reference"] = ("oracle/jmt_ref.py fp32 CPU on windows %s of a B=%d T=%d batch "
                                   "(whole batch on the GPU), conditioned hash-init weights, "
                                   "objective zero outside those windows" % (list(win), B, T))
            parity["tolerance"] = ("min(5 %, 4 x the rounding-emulating oracle's error, floor "
                                   "2u) per prediction set / parameter gradient")
            if args.parity_perturb:
                parity["perturbed"] = ("cross_attention_v.out_proj.weight x %g on the GPU"
                                       % (1 + args.parity_perturb))
            # north_star's own number on the bench's fixed-seed batch and its trained weights
            own = parity_check(model, fc, audio, video, lv, la, cd, cfg["jm"], cfg["fmt"], Dv,
                               k=k, H=heads, L=layers)
            parity["bench_weights"] = own
            parity[north_star_key(cd)] = north_star_verdict(own, cd, parity)
        else:
            parity = parity_check(model, fc, audio, video, lv, la, cd, cfg["jm"], cfg["fmt"], Dv,
                                  k=k, H=heads, L=layers)
            parity[north_star_key(cd)] = north_star_verdict(parity, cd)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.config == "c3" and \
            jcfg is None:
        cpu = cpu_baseline(model_sd0, fc_sd0, audio, video, lv, la)

    return parity, cpu


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); without torchrun's environment and N > 1 this "
                         "script starts them itself (default: WORLD_SIZE, else 1)")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS),
                    help="workload (c3 = the one BASELINE.json's metric is quoted on)")
    ap.add_argument("--batch", type=int, default=None, help="windows per GPU (config default)")
    ap.add_argument("--seq", type=int, default=None, help="T (config default)")
    ap.add_argument("--dtype", default=None, choices=["bf16", "fp16", "fp32"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--parity-perturb", type=float, default=0.0,
                    help="scale cross_attention_v.out_proj.weight by 1+x before the parity check "
                         "(shows that the check fails)")
    ap.add_argument("--no-probe", action="store_true", help="no per-launch events (profiling)")
    ap.add_argument("--graph", dest="graph", action="store_true", default=True,
                    help="replay the whole step as one hipGraph (default)")
    ap.add_argument("--no-graph", dest="graph", action="store_false",
                    help="eager launches from Python every step")
    ap.add_argument("--probe-steps", type=int, default=3)
    ap.add_argument("--launch-log", default=None, help="write per-launch records (jsonl)")
    ap.add_argument("--scaling", choices=["weak", "strong"], default="weak",
                    help="weak: B windows per GPU (headline); strong: B windows in total")
    ap.add_argument("--bucket-mb", type=int, default=8,
                    help="gradient all-reduce bucket size (MiB) for N > 1")
    ap.add_argument("--no-overlap", action="store_true",
                    help="N > 1: all-reduce after the whole backward instead of per bucket "
                         "as soon as its gradients are complete")
    ap.add_argument("--config-file", default=None,
                    help="a config_file.json (the reference's schema): model_params, the train "
                         "batch / window and the opt__* SGD settings define the workload; further "
                         "--key value pairs override it as parseit.py does (e.g. --num_heads 2 "
                         "--opt__lr 1e-3 --train_params__batch_size 32)")
    args, extra = ap.parse_known_args()
    jcfg = None
    if args.config_file:
        from jmt import config as jconfig
        jcfg = jconfig.override(jconfig.load(args.config_file), extra)
    elif extra:
        ap.error(f"unrecognized arguments: {' '.join(extra)}")

    if "WORLD_SIZE" not in os.environ:
        if (args.gpus or 1) > 1:
            # no torchrun around us: be the launcher (nothing has touched the GPU yet); a job
            # that outlives a generous bound on its own work (hung ranks) is terminated
            budget = 600.0 + 2.0 * (args.steps + args.warmup + args.probe_steps)
            raise SystemExit(launch_ranks(args.gpus, sys.argv[1:], deadline_s=budget))
    elif args.gpus is not None and int(os.environ["WORLD_SIZE"]) != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={os.environ['WORLD_SIZE']} but --gpus "
                         f"{args.gpus}: one rank per GPU")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one process per GPU; JMT_DIST_BACKEND=gloo and the modulo only serve the rehearsal of the
    # N>1 path with several ranks on a 1-GPU box (the driver's runs use RCCL, one rank per GPU)
    backend = os.environ.get("JMT_DIST_BACKEND", "nccl")
    local = local % max(1, torch.cuda.device_count())
    if world > 1:
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from jmt import functional as JF
    from jmt import ops
    from jmt import dist as jdist
    from jmt import streams
    from jmt.optim import FusedSGD, GradScaler
    from jmt.graph import GraphedStep
    from models.two_transformers import Two_transformers
    from models.fc_layer import FcLayer
    from losses.loss import CCCLoss

    cfg = dict(CONFIGS[args.config])
    heads, layers, drop = 1, 1, (0.0, 0.0)
    sgd_kw = dict(lr=1e-4, momentum=0.9, dampening=0.0, weight_decay=1e-4, nesterov=True)
    if jcfg is not None:
        # the shipped schema: R2D1 + ResNet18 features (512 each), no FcLayer (main.py:469-481)
        mp = jcfg["model_params"]
        jb, jt = jconfig.window(jcfg)
        cfg = dict(B=jb, T=jt, Da=512, Dv=512, fc=False, jm=mp["joint_modalities"],
                   fmt=mp["output_format"], dtype="bf16",
                   desc=f"config file {os.path.basename(args.config_file)}"
                        + (f" + {' '.join(extra)}" if extra else "")
                        + f": T={jt} clips, batch {jb}, Two_transformers({mp['joint_modalities']},"
                          f"{mp['output_format']},H={mp['num_heads']},L={mp['num_layers']})")
        heads, layers = int(mp["num_heads"]), int(mp["num_layers"])
        drop = (float(mp["v_dropout"]), float(mp["a_dropout"]))
        sgd_kw = jconfig.sgd_kwargs(jcfg)
    k = int(cfg.get("digitize", 1))
    args.dtype = args.dtype or cfg["dtype"]
    cd = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}[args.dtype]
    B = args.batch or cfg["B"]
    if args.scaling == "strong":
        # fixed GLOBAL batch (SURVEY.md §8e strong scaling): each rank takes its contiguous share
        if B % world:
            raise SystemExit(f"--scaling strong: global batch {B} not divisible by {world} ranks")
        B //= world
    T = args.seq or cfg["T"]
    Da, Dv = cfg["Da"], cfg["Dv"]
    fl_kw = dict(Da=Da, Dv=Dv, fc=cfg["fc"], jm=cfg["jm"], fmt=cfg["fmt"], k=k)
    torch.manual_seed(0)
    model = Two_transformers(drop[0], drop[1], heads, layers, cfg["jm"], cfg["fmt"], Dv,
                             digitize_num=k).to(dev)
    fc = FcLayer(Da, E).to(dev) if cfg["fc"] else None
    model_sd0 = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()} \
        if rank == 0 else None
    fc_sd0 = {k: v.detach().cpu().clone() for k, v in fc.state_dict().items()} \
        if rank == 0 and fc is not None else None
    if world > 1:
        jdist.set_loss_group(dist.group.WORLD)

    # synthetic inputs resident in HBM, disjoint per rank (global batch = world * B)
    audio, video, lv, la = synthetic_batch(B, T, Da, Dv, rank, dev)
    crit = CCCLoss(k)
    # k = 1: train.py:303-307's (1, T*B) views; k > 1 (c5's expression-style head): the (T, B, k)
    # logits as the (N, k) rows loss.py:18-22 takes, labels (N,)
    flat = (lambda o: o.reshape(-1, k)) if k > 1 else (lambda o: o.view(-1, o.shape[0] * o.shape[1]))

    # fp16 trains under loss scaling as the reference does (train.py:89,314-316); the scaler's
    # state lives on the device, so the step stays one graph replay
    scaler = GradScaler(device=dev) if cd == torch.float16 else None

    # train.py:309-314: v_loss + a_loss summed by the second criterion's finish kernel
    # (CCCLoss.forward_add), backward seeded with a persistent 1 — the step runs no torch kernel
    one = torch.ones((), dtype=torch.float32, device=dev)

    def fwd_bwd():
        with JF.compute_mode(cd):
            vo, ao = model(fc(audio) if fc is not None else audio, video)
            l1 = crit(flat(vo), lv)
            loss = crit.forward_add(flat(ao), la, l1)
            if scaler is not None:
                scaler.scale(loss).backward()
            else:
                loss.backward(one)
        return loss

    # the parameters that get a gradient, laid out in the order their gradients complete, so
    # that the all-reduce buckets become ready one after another during the backward
    params, wcounts = jdist.grad_write_profile(fwd_bwd, list(model.parameters()) +
                                               (list(fc.parameters()) if fc is not None else []))
    opt = FusedSGD(params, **sgd_kw, shadow_dtype=cd if cd != torch.float32 else None,
                   fuse_zero_grad=True)
    bucketer = None
    if world > 1 and not args.no_overlap:
        bucketer = jdist.GradBucketer(opt, wcounts, bucket_bytes=args.bucket_mb << 20,
                                      group=dist.group.WORLD)

    def step():
        opt.zero_grad()
        if bucketer is not None:
            bucketer.begin()                     # buckets all-reduce during the backward
        loss = fwd_bwd()
        if bucketer is not None:
            bucketer.finish()
        elif world > 1:
            bucket = 16 << 20   # elements per all-reduce bucket, after the whole backward
            for off in range(0, opt.numel, bucket):
                dist.all_reduce(opt.flat_g[off:off + bucket])
        if scaler is not None:
            scaler.step(opt)
            scaler.update()
        else:
            opt.step()
        return loss

    probe = FamilyProbe()
    for _ in range(args.warmup):
        loss = step()
    torch.cuda.synchronize()
    # host issue time of one eager step (how long Python + autograd + ctypes take to enqueue it)
    t_issue = time.perf_counter()
    loss = step()
    host_issue_ms = (time.perf_counter() - t_issue) * 1e3
    torch.cuda.synchronize()

    run = step
    graphed = None
    # N > 1: the step as hipGraph SEGMENTS with the collectives (CCC
    # all-gather, per-bucket RCCL all-reduces, the final join) issued eagerly between them
    # (jmt.graph.SegmentedStep): host issue is one graph launch per segment instead of the
    # eager step's ~300 launches (host_issue_ms_per_eager_step, ~3 ms at c3), which a
    # strong-scaling B = 8 per GPU step would not hide.  JMT_GRAPH_DIST=0: eager.  (Round 5's
    # JMT_GRAPH_DIST=1 — RCCL captured into one whole-step graph — is retired: ProcessGroupNCCL's
    # watchdog intermittently aborted a rank on a work event recorded inside the capture.)
    gmode = os.environ.get("JMT_GRAPH_DIST", "segmented")
    use_graph = args.graph and (world == 1 or gmode != "0")
    graph_kind = None
    if use_graph:
        if world == 1:
            # the whole step as one hipGraph (jmt/graph.py): replay issues ~300 launches at once
            graphed = GraphedStep(step).capture(warmup=1)
            graph_kind = "whole step"
        else:
            from jmt.graph import SegmentedStep
            loss = None         # no eager step's autograd graph may outlive into the capture
            graphed = SegmentedStep(step).capture(warmup=1)
            graph_kind = f"{len(graphed.segments)} segments, collectives eager between them"
        run = graphed.replay
        torch.cuda.synchronize()
        t_issue = time.perf_counter()
        loss = run()                                # host time to issue one replayed step
        host_issue_graph_ms = (time.perf_counter() - t_issue) * 1e3
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = run()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    last_loss = float(loss.detach())
    if not args.no_probe:
        # per-launch HIP events cannot sit inside the replayed graph (and would add host work to
        # an eager timed region): the dominant kernel is timed over `probe_steps` eager steps
        # right after the timed region, on the stream its launches go to.  The weight-gradient
        # side stream (jmt.streams.run_side) is off for them: every launch then runs alone on the
        # compute stream, so its event pair times the kernel itself, not the kernel plus the
        # other stream's kernels sharing the CUs (profiles/r02_bench_family_check_s3.txt)
        ops.set_launch_hook(probe)
        streams.set_side_enabled(False)
        probe.on = True
        for _ in range(args.probe_steps):
            step()
        torch.cuda.synchronize()
        probe.on = False
        streams.set_side_enabled(os.environ.get("JMT_SIDE_STREAM", "0") == "1")
        ops.set_launch_hook(None)
    if world > 1:
        tt = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    ms_per_step = elapsed / args.steps * 1e3
    windows = B * world * args.steps
    value = windows / elapsed

    psum = probe.summary(args.probe_steps)
    if args.launch_log and rank == 0 and probe.rec:
        probe.dump(args.launch_log, args.probe_steps)
    roofline = None
    if psum:
        dom = psum["families"][0]                  # the family with the most in-step time
        # HBM bytes per launch of that family from the committed PMC passes
        # (scripts/pmc_bench.sh: FETCH_SIZE / WRITE_SIZE, separate rocprofv3 passes, gfx950
        # FETCH_SIZE x2 correction), when one exists for this workload
        traffic, traffic_src, traffic_commit = None, None, None
        tpath = os.path.join(REPO, "profiles", f"{PROFILE_TAG}_pmc_bench",
                             f"traffic_{dom['family']}.json")
        if args.config == "c3" and cd == torch.bfloat16 and os.path.exists(tpath):
            tj = json.load(open(tpath))
            traffic = round(tj["hbm_bytes_per_launch"])
            traffic_src = os.path.relpath(tpath, REPO)
            traffic_commit = tj.get("commit")
        # the in-step view: each family's kernel time inside the
        # graph-replayed timed region (side stream on, launches overlapping) from the committed
        # rocprofv3 trace of the default command (scripts/family_from_trace.py --json), beside
        # the isolated probe figure; same FLOPs per launch
        in_step, trace_commit = None, None
        ipath = os.path.join(REPO, "profiles", f"{PROFILE_TAG}_family_trace.json")
        if args.config == "c3" and cd == torch.bfloat16 and world == 1 and \
                os.path.exists(ipath):
            ij = json.load(open(ipath))
            trace_commit = ij.get("commit")
            for f in psum["families"]:
                t = ij["families"].get(f["family"])
                if t and t.get("avg_launch_us"):
                    tf = f["gflop_per_launch"] * 1e9 / (t["avg_launch_us"] * 1e-6) / 1e12
                    f["in_step"] = {"avg_launch_us": t["avg_launch_us"],
                                    "ms_per_step": t["ms_per_step"],
                                    "tflops": round(tf, 1),
                                    "frac": round(tf / PEAK_BF16_TFLOPS, 4)}
            in_step = os.path.relpath(ipath, REPO)
        roofline = {"bound": "mfma", "kernel": dom["family"], "achieved": dom["tflops"],
                    "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s", "frac": dom["frac"],
                    "traffic": traffic, "traffic_unit": "HBM bytes per launch (PMC)",
                    "traffic_source": traffic_src, "traffic_commit": traffic_commit,
                    "in_step": dom.get("in_step"), "in_step_source": in_step,
                    "in_step_commit": trace_commit,
                    "algorithmic_bytes_per_launch": dom["algorithmic_bytes_per_launch"] or None,
                    "avg_launch_us": dom["avg_launch_us"],
                    "launches_per_step": dom["launches_per_step"],
                    "timed_over": f"{args.probe_steps} eager probe steps after the timed region "
                                  "(side stream off: each launch alone on the compute stream), "
                                  "one event pair per launch minus the empty-launch pair "
                                  f"overhead ({psum['event_pair_overhead_us']} us), each "
                                  "launch position at its median over the probe steps",
                    "families": psum["families"]}
    sfl = step_flops(B, T, **fl_kw)
    step_mfma = None
    if sfl is not None:
        step_tf = sfl * world / (elapsed / args.steps) / 1e12
        step_mfma = {"algorithmic_tflop_per_step": round(sfl * world / 1e12, 4),
                     "achieved_tflops": round(step_tf, 1),
                     "frac_of_peak": round(step_tf / (PEAK_BF16_TFLOPS * world), 4)}

    if world > 1:
        print(f"rank {rank}/{world}: cuda:{local} backend {backend}, {B} windows, "
              f"{elapsed / args.steps * 1e3:.3f} ms/step (max over ranks), graph {use_graph}, "
              f"final loss {last_loss:.6f}", file=sys.stderr, flush=True)
    # the parity and CPU legs run on rank 0 alone: the CCC losses inside them must use local
    # statistics (a loss group would all-gather with ranks that are not there)
    group = jdist.loss_group()
    jdist.set_loss_group(None)
    try:
        parity, cpu = _rank0_legs(args, cfg, cd, k, heads, layers, B, T, Da, Dv, model, fc, audio,
                                  video, lv, la, rank, world, jcfg, model_sd0, fc_sd0)
    finally:
        jdist.set_loss_group(group)
    if rank == 0:
        out = {
            "metric": "train windows/sec + CCC parity, B=64 T=300 A/V fusion, 1/2/4/8 MI355X",
            "value": round(value, 2), "unit": "windows/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True, "scaling": args.scaling, "vs_baseline": None,
            "dtype": args.dtype, "data": "synthetic (N(0,1) features, U(-1,1) labels, "
                                         "random-init weights)",
            "config": {"workload": cfg["desc"],
                       "name": "config_file" if jcfg is not None else args.config,
                       "global_batch": B * world, "per_gpu_batch": B, "seq_len": T,
                       "D_a": Da, "D_v": Dv, "parallelism": f"dp{world}",
                       "grad_allreduce": (None if world == 1 else
                                          "after backward" if bucketer is None else
                                          f"{len(bucketer.buckets)} buckets of >= "
                                          f"{args.bucket_mb} MiB, each as soon as its "
                                          "gradients are written (overlaps the backward)"),
                       "loss_scaling": "device GradScaler" if scaler is not None else None},
            "roofline": roofline,
            "step_mfma": step_mfma,
            "parity": parity,
            "cpu_baseline": cpu,
            "final_loss": round(last_loss, 6),
            "graph": bool(use_graph),
            "graph_kind": graph_kind,
            "host_issue_ms_per_graphed_step": (round(host_issue_graph_ms, 3) if use_graph
                                               else None),
            "launcher": (os.environ.get("JMT_LAUNCHER", "torchrun") if world > 1 else None),
            "dist_backend": backend if world > 1 else None,
            "host_issue_ms_per_eager_step": round(host_issue_ms, 3),
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
