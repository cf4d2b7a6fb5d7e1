"""The training entry points a reference user drives (train.py:89-101,283-316, main.py:105-177,
515-518) on the HIP drop-ins:

* FusedSGD (flat fp32 master + bf16 shadow rewritten in the same kernel) vs torch.optim.SGD in
  bf16 compute, with and without a shadow, and across a mid-training `load_state_dict` (the
  shadow-staleness hazard of ADVICE r1: an in-place parameter write must reach the 16-bit copy
  the forward reads);
* a `fusion_w.pt` checkpoint (torch.save of the state_dict, main.py:105-177) loaded into a fresh
  module (main.py:515-518) gives identical predictions;
* train.py unchanged: `torch.cuda.amp.autocast()` selects the 16-bit HIP path by itself and
  torch's own GradScaler + SGD train it exactly like the explicit compute_mode path."""
import os

import numpy as np
import pytest
import torch

from jmt import functional as JF
from jmt.optim import FusedSGD, used_parameters
from tests.golden import spec
from tests.parity import build_tt

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")
CASE = [c for c in spec.TT_CASES if c["tag"] == "tr_fc"][0]
SGD_KW = dict(lr=1e-2, momentum=0.9, dampening=0.0, weight_decay=1e-4, nesterov=True)


def _data(c=CASE):
    B, T = c["B"], c["T"]
    audio, video, lv, la = spec.tt_inputs(c["tag"], B, T, c["vin"])
    return (torch.from_numpy(audio).to(DEV), torch.from_numpy(video).to(DEV),
            torch.from_numpy(lv).to(DEV).view(-1, B * T),
            torch.from_numpy(la).to(DEV).view(-1, B * T))


def _loss(m, fc, data, crit):
    a, v, vt, at = data
    vo, ao = m(fc(a), v)
    return crit(vo.view(-1, vo.numel()), vt) + crit(ao.view(-1, ao.numel()), at)


def _params(m, fc, data, crit, cd):
    with JF.compute_mode(cd):
        return used_parameters(lambda: _loss(m, fc, data, crit).backward(),
                               list(m.parameters()) + list(fc.parameters()))


def _state(m, fc):
    return {**{k: v.detach().clone() for k, v in m.state_dict().items()},
            **{"fc." + k: v.detach().clone() for k, v in fc.state_dict().items()}}


@pytest.mark.parametrize("shadow", [True, False], ids=["bf16_shadow", "no_shadow"])
@pytest.mark.parametrize("reload", [False, True], ids=["plain", "load_state_dict_mid_run"])
def test_fused_sgd_bf16_matches_torch_sgd(shadow, reload):
    from losses.loss import CCCLoss
    cd = torch.bfloat16
    crit = CCCLoss(1)
    data = _data()
    ma, fa = build_tt(CASE)           # FusedSGD
    mb, fb = build_tt(CASE)           # torch.optim.SGD
    pa = _params(ma, fa, data, crit, cd)
    pb = _params(mb, fb, data, crit, cd)
    opt_a = FusedSGD(pa, shadow_dtype=cd if shadow else None, **SGD_KW)
    opt_b = torch.optim.SGD(pb, **SGD_KW)
    snapshot = None
    for step in range(4):
        if reload and step == 2:
            # both models jump back to the step-1 weights (momentum buffers stay)
            ma.load_state_dict({k: v for k, v in snapshot.items() if not k.startswith("fc.")})
            mb.load_state_dict({k: v for k, v in snapshot.items() if not k.startswith("fc.")})
        losses = []
        for m, fc, opt in ((ma, fa, opt_a), (mb, fb, opt_b)):
            opt.zero_grad()
            with JF.compute_mode(cd):
                loss = _loss(m, fc, data, crit)
                loss.backward()
            opt.step()
            losses.append(float(loss))
        assert abs(losses[0] - losses[1]) <= 1e-5, (step, losses)
        if step == 0:
            snapshot = _state(ma, fa)
    sa, sb = _state(ma, fa), _state(mb, fb)
    for k in sa:
        err = float((sa[k] - sb[k]).abs().max() / sb[k].abs().max().clamp_min(1e-30))
        assert err <= 1e-5, (k, err)


def test_fusion_w_checkpoint_roundtrip(tmp_path):
    """torch.save(model.state_dict()) as main.py:105-177 dumps it (CPU tensors), loaded into a
    freshly built drop-in (main.py:515-518): identical keys, values and predictions, also after
    FusedSGD moved the parameters into its flat buffer."""
    from losses.loss import CCCLoss
    from models.two_transformers import Two_transformers
    crit = CCCLoss(1)
    data = _data()
    m, fc = build_tt(CASE)
    params = _params(m, fc, data, crit, torch.bfloat16)
    opt = FusedSGD(params, shadow_dtype=torch.bfloat16, **SGD_KW)
    for _ in range(2):
        opt.zero_grad()
        with JF.compute_mode(torch.bfloat16):
            _loss(m, fc, data, crit).backward()
        opt.step()
    path = os.path.join(tmp_path, "fusion_w.pt")
    torch.save({k: v.cpu() for k, v in m.state_dict().items()}, path)
    sd = torch.load(path, weights_only=True)
    m2 = Two_transformers(0.0, 0.0, CASE["H"], CASE["L"], CASE["jm"], CASE["fmt"], CASE["vin"])
    assert list(sd.keys()) == list(m2.state_dict().keys())
    m2.load_state_dict(sd)
    m2 = m2.to(DEV)
    a, v, _, _ = data
    with torch.no_grad():
        for cd in (torch.float32, torch.bfloat16):
            with JF.compute_mode(cd):
                o1 = m(fc(a), v)
                o2 = m2(fc(a), v)
            for x, y in zip(o1, o2):
                assert torch.equal(x, y), cd


def test_train_py_autocast_entry_unchanged():
    """train.py:89,101,283-316 verbatim in spirit: torch.cuda.amp.GradScaler(), the forward under
    torch.cuda.amp.autocast(), scaler.scale(loss).backward(), scaler.step(optimizer),
    scaler.update() with torch.optim.SGD.  The drop-ins pick fp16 from autocast on their own and
    the three-step trajectory equals the explicit compute_mode(fp16) run bit for bit, and the
    fp32 reference trajectory (golden) within the fp16 error model."""
    import warnings
    from losses.loss import CCCLoss
    crit = CCCLoss(1)
    data = _data()
    runs = []
    for mode in ("autocast", "explicit"):
        m, fc = build_tt(CASE)
        params = list(m.parameters()) + list(fc.parameters())
        opt = torch.optim.SGD(params, lr=1e-4, momentum=0.9, dampening=0.0, weight_decay=1e-4,
                              nesterov=True)
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            scaler = torch.cuda.amp.GradScaler()
        losses = []
        for _ in range(CASE["train_steps"]):
            opt.zero_grad()
            if mode == "autocast":
                with warnings.catch_warnings():
                    warnings.simplefilter("ignore")
                    ctx = torch.cuda.amp.autocast()
                with ctx:
                    assert JF.compute_dtype() == torch.float16
                    a, v, vt, at = data
                    vo, ao = m(fc(a), v)
                    vout = vo.view(-1, vo.shape[0] * vo.shape[1])
                    aout = ao.view(-1, ao.shape[0] * ao.shape[1])
                    loss = crit(vout, vt) + crit(aout, at)
            else:
                with JF.compute_mode(torch.float16):
                    loss = _loss(m, fc, data, crit)
            scaler.scale(loss).backward()
            scaler.step(opt)
            scaler.update()
            losses.append(float(loss))
        runs.append(losses)
    assert runs[0] == runs[1], runs
    np.testing.assert_allclose(np.array(runs[0]), _golden_sum(), atol=5e-3)


def _golden_sum():
    import os as _os
    path = _os.path.join(_os.path.dirname(__file__), "golden", "golden.npz")
    with np.load(path, allow_pickle=False) as z:
        return z[CASE["tag"] + "/train_losses"].sum(axis=1)
