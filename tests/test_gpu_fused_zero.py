"""The ABI-5 paths the default bench step runs: the SGD step that zeroes the
gradients it consumes (jmt_sgd_step_zero, jmt_sgd_step_amp_zero), FusedSGD(fuse_zero_grad=True)
and the CCC finish kernel that adds the other loss (jmt_ccc_finish_add, CCCLoss.forward_add,
train.py:309-311's v_loss + a_loss).  Each is checked bit for bit against the form without the
fusion."""
import pytest
import torch

from jmt import functional as JF
from jmt import ops
from jmt.optim import FusedSGD, GradScaler

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")
SGD_KW = dict(lr=1e-2, momentum=0.9, dampening=0.0, weight_decay=1e-4, nesterov=True)


def _flat(n, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    return torch.randn(n, generator=g, device=DEV)


@pytest.mark.parametrize("shadow", [None, torch.bfloat16], ids=["no_shadow", "bf16_shadow"])
@pytest.mark.parametrize("first", [True, False])
def test_sgd_step_zero_bit_identical_and_zeroes_grad(shadow, first):
    n = 3 * 4096 + 77
    p0, g0, b0 = _flat(n, 1), _flat(n, 2), _flat(n, 3)
    outs = []
    for zero in (False, True):
        p, g, b = p0.clone(), g0.clone(), b0.clone()
        sh = torch.empty(n, dtype=shadow, device=DEV) if shadow is not None else None
        ops.sgd_step(p, g, b, SGD_KW["lr"], SGD_KW["momentum"], 0.0, SGD_KW["weight_decay"],
                     True, first, 1.0, sh, zero_grad=zero)
        outs.append((p, g, b, sh))
    (p1, g1, b1, s1), (p2, g2, b2, s2) = outs
    assert torch.equal(p1, p2) and torch.equal(b1, b2)
    if shadow is not None:
        assert torch.equal(s1, s2)
    assert torch.equal(g1, g0)                       # the plain step leaves the gradient
    assert int((g2 != 0).sum()) == 0                 # the fused one zeroes all of it


@pytest.mark.parametrize("found_inf", [False, True])
def test_sgd_step_amp_zero_bit_identical(found_inf):
    """jmt_sgd_step_amp_zero == jmt_sgd_step_amp on params / momentum / shadow / scaler state; an
    overflow step leaves params, momentum and shadow untouched and still zeroes the gradient."""
    n = 8192 + 5
    p0, g0 = _flat(n, 11), _flat(n, 12) * 1024.0
    if found_inf:
        g0[n // 2] = float("inf")
    res = []
    for fuse in (False, True):
        prm = [torch.nn.Parameter(p0.clone())]
        opt = FusedSGD(prm, **SGD_KW, shadow_dtype=torch.bfloat16, fuse_zero_grad=fuse)
        sc = GradScaler(init_scale=1024.0, growth_interval=1, device=DEV)
        # a clean first step initialises the momentum, the second is the one under test
        opt.flat_g[:n].copy_(_flat(n, 13) * 1024.0)
        sc.step(opt)
        sc.update()
        before = (opt.flat_p.clone(), opt.buf.clone(), opt.shadow.clone())
        opt.flat_g[:n].copy_(g0)
        sc.step(opt)
        sc.update()
        res.append((opt.flat_p.clone(), opt.buf.clone(), opt.shadow.clone(),
                    opt.flat_g.clone(), sc.state.clone(), before))
    (p1, b1, s1, g1, st1, _), (p2, b2, s2, g2, st2, before2) = res
    assert torch.equal(p1, p2) and torch.equal(b1, b2) and torch.equal(s1, s2)
    assert torch.equal(st1, st2)
    assert int((g2 != 0).sum()) == 0
    if found_inf:
        assert torch.equal(p2, before2[0]) and torch.equal(b2, before2[1])
        assert torch.equal(s2, before2[2])
        assert torch.equal(g1[:n], g0)               # unfused: the skipped step leaves .grad
    else:
        assert not torch.equal(p2, before2[0])


def test_fused_sgd_zero_grad_on_off_three_steps_bit_identical():
    """3 steps of FusedSGD with fuse_zero_grad on vs off: identical parameters, momentum and
    shadows after each step, with gradients written by HIP linears (functional._grad_gen) in
    steps 1 and 3 and by torch autograd accumulating into .grad (post-accumulate hooks) in
    step 2 — the skipped fill must never leave a stale gradient behind."""
    from models.fc_layer import FcLayer
    torch.manual_seed(0)
    base = FcLayer(96, 64).to(DEV)
    x = torch.randn(40, 96, device=DEV)
    runs = []
    for fuse in (False, True):
        m = FcLayer(96, 64).to(DEV)
        m.load_state_dict(base.state_dict())
        opt = FusedSGD(list(m.parameters()), **SGD_KW, fuse_zero_grad=fuse)
        states = []
        for step in range(3):
            opt.zero_grad()
            if step == 1:
                # plain torch autograd into the same .grad views
                loss = (torch.nn.functional.linear(x, m.fc_layer.weight, m.fc_layer.bias) ** 2
                        ).mean()
            else:
                with JF.compute_mode(torch.float32):
                    loss = (m(x) ** 2).mean()
            loss.backward()
            opt.step()
            states.append((opt.flat_p.clone(), opt.buf.clone()))
        runs.append(states)
    for (pa, ba), (pb, bb) in zip(*runs):
        assert torch.equal(pa, pb) and torch.equal(ba, bb)


def test_fused_sgd_untracked_grad_write_check_force_and_close(monkeypatch):
    """The skipped fill's contract: an in-place .grad write outside the tracked writers is caught
    by JMT_CHECK_ZERO_GRAD=1, zero_grad(force=True) clears it, close() removes the hooks."""
    from models.fc_layer import FcLayer
    m = FcLayer(32, 16).to(DEV)
    opt = FusedSGD(list(m.parameters()), **SGD_KW, fuse_zero_grad=True)
    x = torch.randn(8, 32, device=DEV)
    with JF.compute_mode(torch.float32):
        (m(x) ** 2).mean().backward()
    opt.step()
    assert int(torch.count_nonzero(opt.flat_g)) == 0
    m.fc_layer.weight.grad.add_(1.0)                    # untracked write
    monkeypatch.setenv("JMT_CHECK_ZERO_GRAD", "1")
    with pytest.raises(RuntimeError, match="outside the tracked writers"):
        opt.zero_grad()
    opt.zero_grad(force=True)
    assert int(torch.count_nonzero(opt.flat_g)) == 0
    opt.zero_grad()                                     # clean: the check passes
    n_hooks = len(opt._hooks)
    assert n_hooks == len(opt.params)
    opt.close()
    assert opt._hooks == []


@pytest.mark.parametrize("add_shape", [(), (1,)])
def test_ccc_finish_add_bit_identical(add_shape):
    """CCCLoss.forward_add(x2, y2, l1) == l1 + CCCLoss(x2, y2) bit for bit (one fp32 add either
    way), d/d(add) = 1 in add's own shape, and the x2 gradient equals the unfused one."""
    from losses.loss import CCCLoss
    g = torch.Generator(device=DEV).manual_seed(5)
    x1 = torch.randn(1, 600, generator=g, device=DEV)
    y1 = torch.rand(1, 600, generator=g, device=DEV) * 2 - 1
    x2 = torch.randn(1, 600, generator=g, device=DEV).requires_grad_(True)
    y2 = torch.rand(1, 600, generator=g, device=DEV) * 2 - 1
    crit = CCCLoss(1)
    l1 = crit(x1, y1).detach().reshape(add_shape).requires_grad_(True)
    fused = crit.forward_add(x2, y2, l1)
    fused.backward()
    ga, gx_fused = l1.grad.clone(), x2.grad.clone()
    x2.grad = None
    plain = l1.detach() + crit(x2, y2)
    plain.sum().backward()
    assert torch.equal(fused.reshape(()), plain.reshape(()))
    assert ga.shape == l1.shape and float(ga.reshape(())) == 1.0
    assert torch.equal(gx_fused, x2.grad)
