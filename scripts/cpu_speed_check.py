"""The CPU restatement's speed against the reference's own CPU path (within ±15 %
on the same cores), in this container (the reference is importable here; it never travels to
the GPU box).  One training step of configs[2]'s model (FcLayer(1024,512) + Two_transformers(
TRANSFORMER, FC, H=1, L=1, vision_in_ft=2048) + 2x CCCLoss(1) + SGD-nesterov, train.py:283-316)
on the same batch and weights, fp32 torch-CPU, the same thread count for both:

    python scripts/cpu_speed_check.py [--B 2] [--T 300] [--threads 8] [--steps 3]

The reference's losses/loss.py builds its bins with .cuda(): Tensor.cuda is the identity while
it is constructed (tests/golden/make_golden.py:make_loss)."""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO]

import torch  # noqa: E402

from oracle import jmt_ref as R  # noqa: E402
from tests.golden.make_golden import import_reference, make_loss  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=2)
    ap.add_argument("--T", type=int, default=300)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--steps", type=int, default=10)
    args = ap.parse_args()
    torch.set_num_threads(args.threads)
    mods = import_reference()
    torch.manual_seed(0)
    model = mods["models.two_transformers"].Two_transformers(0.0, 0.0, 1, 1, "TRANSFORMER", "FC",
                                                            2048)
    fc = mods["models.fc_layer"].FcLayer(1024, 512)
    crit = make_loss(mods, "CCCLoss", 1)
    g = torch.Generator().manual_seed(1)
    B, T = args.B, args.T
    audio = torch.randn(B, T, 1024, generator=g)
    video = torch.randn(B, T, 2048, generator=g)
    lv = torch.rand(B, T, generator=g) * 2 - 1
    la = torch.rand(B, T, generator=g) * 2 - 1
    p0 = {k: v.detach().clone() for k, v in model.state_dict().items()}
    f0 = {k: v.detach().clone() for k, v in fc.state_dict().items()}
    params = list(model.parameters()) + list(fc.parameters())
    opt = torch.optim.SGD(params, lr=1e-4, momentum=0.9, dampening=0.0, weight_decay=1e-4,
                          nesterov=True)

    def ref_step():
        opt.zero_grad()
        vo, ao = model(fc(audio), video)
        vo = vo.reshape(-1, vo.shape[0] * vo.shape[1])
        ao = ao.reshape(-1, ao.shape[0] * ao.shape[1])
        loss = crit(vo, lv.view(-1, B * T)) + crit(ao, la.view(-1, B * T))
        loss.backward()
        opt.step()
        return float(loss)

    p = {k: v.clone() for k, v in p0.items()}
    f = {k: v.clone() for k, v in f0.items()}
    bufs = {}

    def oracle_step():
        lv_, la_, _ = R.train_step(p, f, audio, video, lv, la, 1, 1, "TRANSFORMER", "FC", 2048,
                                   bufs)
        return float(lv_ + la_)

    # interleaved (reference step, oracle step) pairs, median per side: the container's other
    # load drifts over seconds, and interleaving exposes both sides to the same drift
    import statistics
    res = {"reference": ([], []), "oracle": ([], [])}
    for i in range(args.steps + 1):
        for name, fn in (("reference", ref_step), ("oracle", oracle_step)):
            t0 = time.perf_counter()
            res[name][0].append(fn())
            res[name][1].append(time.perf_counter() - t0)
    lr_, tr = res["reference"][0], statistics.median(res["reference"][1][1:])
    lo, to = res["oracle"][0], statistics.median(res["oracle"][1][1:])
    print(f"configs[2] model, B={B} T={T}, fp32 torch-CPU, {args.threads} threads, "
          f"1 warm-up + {args.steps} timed steps each, interleaved, median")
    print(f"reference (models/*.py + losses/loss.py + torch SGD): {tr * 1e3:.1f} ms/step "
          f"-> {B / tr:.3f} windows/s; losses {[round(x, 6) for x in lr_]}")
    print(f"oracle    (oracle/jmt_ref.py train_step):            {to * 1e3:.1f} ms/step "
          f"-> {B / to:.3f} windows/s; losses {[round(x, 6) for x in lo]}")
    print(f"oracle / reference time = {to / tr:.3f}  (bar: within 0.85 .. 1.15)")
    print(f"max |loss difference| over the trajectory = "
          f"{max(abs(a - b) for a, b in zip(lr_, lo)):.2e}")


if __name__ == "__main__":
    main()
