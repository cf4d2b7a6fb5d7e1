"""Whole-step hipGraph capture (jmt/graph.py): replaying the captured training step must give
exactly the eager step's results (same kernels, same order per stream, deterministic reductions
-> bit-identical losses and parameters)."""
import pytest
import torch

from jmt import functional as JF
from jmt.graph import GraphedStep
from jmt.optim import FusedSGD, used_parameters
from oracle.hashinit import init_module_

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _setup(cd, B=4, T=37):
    from models.two_transformers import Two_transformers
    from models.fc_layer import FcLayer
    from losses.loss import CCCLoss
    m = Two_transformers(0.0, 0.0, 1, 1, "TRANSFORMER", "FC", 2048)
    fc = FcLayer(1024, 512)
    init_module_(m, "")
    init_module_(fc, "fc.")
    m, fc = m.to(DEV), fc.to(DEV)
    g = torch.Generator(device=DEV).manual_seed(7)
    audio = torch.randn(B, T, 1024, device=DEV, generator=g)
    video = torch.randn(B, T, 2048, device=DEV, generator=g)
    lv = (torch.rand(B, T, device=DEV, generator=g) * 2 - 1).view(-1, B * T)
    la = (torch.rand(B, T, device=DEV, generator=g) * 2 - 1).view(-1, B * T)
    crit = CCCLoss(1)

    def fwd_bwd():
        with JF.compute_mode(cd):
            vo, ao = m(fc(audio), video)
            loss = crit(vo.view(-1, B * T), lv) + crit(ao.view(-1, B * T), la)
            loss.backward()
        return loss

    params = used_parameters(fwd_bwd, list(m.parameters()) + list(fc.parameters()))
    opt = FusedSGD(params, lr=1e-2, momentum=0.9, dampening=0.0, weight_decay=1e-4,
                   nesterov=True, shadow_dtype=cd if cd != torch.float32 else None)

    def step():
        opt.zero_grad()
        loss = fwd_bwd()
        opt.step()
        return loss.detach()

    return step, opt, (audio, video)


@pytest.mark.parametrize("cd", [torch.float32, torch.bfloat16], ids=["fp32", "bf16"])
def test_graph_replay_matches_eager(cd):
    # eager: 2 warm-up steps + 3 steps
    step_e, opt_e, _ = _setup(cd)
    for _ in range(2):
        step_e()
    eager = [float(step_e()) for _ in range(3)]
    torch.cuda.synchronize()
    pe = opt_e.flat_p.clone()

    # graphed: the capture's own warm-up step + 1 eager step (= 2 warm-up steps), then 3 replays
    step_g, opt_g, _ = _setup(cd)
    step_g()
    gs = GraphedStep(step_g).capture(warmup=1)
    graphed = [float(gs.replay()) for _ in range(3)]
    torch.cuda.synchronize()
    assert graphed == eager, (graphed, eager)
    assert torch.equal(opt_g.flat_p, pe)
