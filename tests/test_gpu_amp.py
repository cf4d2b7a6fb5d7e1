"""Device-side GradScaler (train.py:89,314-316) + FusedSGD vs torch.amp.GradScaler +
torch.optim.SGD on the same scaled gradients, including overflow steps (skip + backoff) and scale
growth after growth_interval clean steps.  fp32 parameters: bit-level agreement is expected up to
the fused multiply-add in the update (tolerance 1e-6 relative, written below)."""
import pytest
import torch

from jmt.optim import FusedSGD, GradScaler

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")
TOL = 1e-6


def _scenario(shapes, steps, bad_steps, init_scale, interval, seed=0):
    g = torch.Generator().manual_seed(seed)
    p0 = [torch.randn(s, generator=g) for s in shapes]
    grads = [[torch.randn(s, generator=g) for s in shapes] for _ in range(steps)]
    # torch reference
    ref = [torch.nn.Parameter(p.clone().to(DEV)) for p in p0]
    ropt = torch.optim.SGD(ref, lr=1e-2, momentum=0.9, dampening=0.0, weight_decay=1e-4,
                           nesterov=True)
    rsc = torch.amp.GradScaler("cuda", init_scale=init_scale, growth_interval=interval)
    # ours
    mine = [torch.nn.Parameter(p.clone().to(DEV)) for p in p0]
    opt = FusedSGD(mine, lr=1e-2, momentum=0.9, dampening=0.0, weight_decay=1e-4, nesterov=True)
    sc = GradScaler(init_scale=init_scale, growth_interval=interval, device=DEV)
    scales = []
    for k in range(steps):
        rsc.scale(torch.zeros((), device=DEV))      # torch creates its scale tensor lazily here
        s_ref = rsc.get_scale()
        s_mine = sc.get_scale()
        assert s_ref == s_mine, (k, s_ref, s_mine)
        scales.append(s_mine)
        for i, (pr, pm) in enumerate(zip(ref, mine)):
            gk = grads[k][i].to(DEV) * s_ref
            if k in bad_steps and i == len(ref) - 1:
                gk[0] = float("inf") if k % 2 else float("nan")
            pr.grad = gk.clone()
            pm.grad.copy_(gk)
        rsc.step(ropt)
        rsc.update()
        sc.step(opt)
        sc.update()
        for pr, pm in zip(ref, mine):
            err = ((pr.detach() - pm.detach()).abs().max() /
                   pr.detach().abs().max().clamp_min(1e-30)).item()
            assert err <= TOL, (k, err)
    assert rsc.get_scale() == sc.get_scale()
    return scales


def test_scaler_matches_torch_with_overflows_and_growth():
    scales = _scenario([(37, 5), (1000,), (3, 129)], steps=9, bad_steps={0, 4, 5},
                       init_scale=1024.0, interval=2)
    assert min(scales) < 1024.0 and max(scales) > 512.0     # backed off and grew again


def test_scaler_first_step_skipped_keeps_momentum_fresh():
    # an overflow on the first step must leave the momentum buffer uninitialised: the next
    # clean step is the optimizer's first (torch creates the buffer there)
    _scenario([(4096,)], steps=4, bad_steps={0, 1}, init_scale=2.0 ** 16, interval=2000)


def test_scaler_non_power_of_two_scale():
    _scenario([(513,)], steps=5, bad_steps={2}, init_scale=1000.0, interval=3)


def test_scaler_state_is_device_only_and_capturable():
    p = [torch.nn.Parameter(torch.randn(2048, device=DEV))]
    opt = FusedSGD(p, lr=1e-2, momentum=0.9, nesterov=True)
    sc = GradScaler(init_scale=8.0, growth_interval=1, device=DEV)
    gsrc = torch.randn(2048, device=DEV)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            opt.flat_g[:2048].copy_(gsrc * sc.state[0])
            sc.step(opt)
            sc.update()
    torch.cuda.current_stream().wait_stream(s)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    assert sc.get_scale() == 8.0 * 2 ** 3                  # grew once per clean replay
    assert int(sc.state[4].item()) == 3


def test_plain_step_after_scaled_step_raises():
    p = [torch.nn.Parameter(torch.randn(64, device=DEV))]
    opt = FusedSGD(p, lr=1e-2, momentum=0.9)
    sc = GradScaler(device=DEV)
    sc.step(opt)
    with pytest.raises(RuntimeError):
        opt.step()
