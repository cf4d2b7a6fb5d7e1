"""Run the golden cases through the CPU oracle and compare results with the golden fixtures.
Shared by tests/test_oracle.py (oracle vs reference-generated goldens)."""
from __future__ import annotations

import numpy as np
import torch

from oracle import jmt_ref as R
from tests.golden import spec


def rel_err(a, b) -> float:
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    den = max(np.abs(b).max(), 1e-30)
    return float(np.abs(a - b).max() / den)


def canon(t, seq_first: bool):
    """(T, B, F) -> (B, T, F) when seq_first (the goldens' canonical intermediate layout)."""
    if t is None:
        return None
    return t.permute(1, 0, 2) if seq_first else t


def oracle_tt(c: dict, emulate=None, loss_scale: float = 1.0) -> dict:
    """The golden case through the oracle; `emulate` = 16-bit storage emulation dtype
    (R.emulate_storage), `loss_scale` = GradScaler-style scaling of the backward (grads are
    returned unscaled)."""
    with R.emulate_storage(emulate):
        return _oracle_tt(c, loss_scale)


def case_losses(c: dict, vo, ao, lv, la, ccc):
    """The two losses of a golden case: train.py:303-311's CCC on the (1, B*T) views, or the
    conditioned cases' mean(w * outputs) (spec.COND_CASES)."""
    if c.get("loss") == "proj":
        wv, wa = (torch.from_numpy(w).to(vo.device) for w in spec.proj_inputs(c))
        return (vo.float() * wv).mean(), (ao.float() * wa).mean()
    n = vo.shape[0] * vo.shape[1]
    return (ccc(vo.reshape(1, n), lv.reshape(1, n).to(vo.device)),
            ccc(ao.reshape(1, n), la.reshape(1, n).to(ao.device)))


def _oracle_tt(c: dict, loss_scale: float) -> dict:
    tag = c["tag"]
    shapes = R.two_transformers_shapes(c["L"], c["jm"], c["fmt"], c["vin"])
    p = R.hash_params(shapes, "", c.get("gains"))
    fcp = R.hash_params({"fc_layer.weight": (512, 1024), "fc_layer.bias": (512,)}, "fc.",
                        c.get("gains"))
    B, T = c["B"], c["T"]
    audio, video, lv, la = spec.tt_inputs(tag, B, T, c["vin"])
    for t in list(p.values()) + list(fcp.values()):
        t.requires_grad_(True)
    a = torch.from_numpy(audio).requires_grad_(True)
    v = torch.from_numpy(video).requires_grad_(True)
    aud = R.linear(a, fcp["fc_layer.weight"], fcp["fc_layer.bias"])
    taps = {}
    vo, ao = R.two_transformers_forward(aud, v, p, c["H"], c["L"], c["jm"], c["fmt"], c["vin"],
                                        taps=taps)
    for t, _ in taps.values():
        t.retain_grad()
    l1, l2 = case_losses(c, vo, ao, torch.from_numpy(lv), torch.from_numpy(la), R.ccc_loss)
    ((l1 + l2) * loss_scale).backward()
    uns = lambda g: None if g is None else g / loss_scale
    res = {"vouts": vo.detach().numpy(), "aouts": ao.detach().numpy(),
           "v_loss": float(l1), "a_loss": float(l2), "grads": {},
           "taps": {k: {"val": canon(t.detach(), sf), "grad": uns(canon(t.grad, sf))}
                    for k, (t, sf) in taps.items()}}
    for k, t in p.items():
        res["grads"][k] = uns(t.grad)
    for k, t in fcp.items():
        res["grads"]["fc." + k] = uns(t.grad)
    res["grads"]["input.audio"] = uns(a.grad)
    res["grads"]["input.video"] = uns(v.grad)
    return res


def compare_grads(golden: dict, tag: str, grads: dict, tol: float):
    """Every parameter: relative L2-norm error and the strided sample; None grads must be None."""
    bad = []
    scale = max(float(v) for k, v in golden.items()
                if k.startswith(tag + "/") and k.endswith(":norm"))
    atol = 0.1 * tol * scale   # cancellation-dominated sums (e.g. last-layer bias grads)
    for name, g in grads.items():
        key = f"{tag}/{name}"
        gn = float(golden[key + ":norm"])
        if gn < 0:
            if g is not None and float(torch.as_tensor(g).abs().max()) != 0.0:
                bad.append((name, "expected no grad"))
            continue
        if g is None:
            bad.append((name, "missing grad"))
            continue
        g = torch.as_tensor(g).detach().double().cpu().reshape(-1)
        n = float(g.norm())
        if abs(n - gn) > tol * gn + atol:
            bad.append((name, f"norm {n} vs {gn}"))
            continue
        stride = max(1, g.numel() // spec.N_SAMPLE)
        s = g[::stride][:spec.N_SAMPLE].numpy()
        ref = golden[key + ":sample"]
        err = np.abs(s - ref).max()
        if err > 10 * tol * max(np.abs(ref).max(), gn / np.sqrt(g.numel())) + atol:
            bad.append((name, f"sample rel err {err}"))
    return bad


def inter_errors(golden: dict, tag: str, taps: dict):
    """Relative Frobenius error of the recorded intermediates (and of their gradients) on the
    golden's sampled (b, t) rows: {name:kind: err}.  taps[name] = {"val": (B,T,F), "grad": ...}
    (canonical layout, any device / dtype).  Every golden intermediate must be present."""
    idx = torch.from_numpy(golden[tag + "/inter_rows"])
    names = sorted({k.split("/inter/")[1].split(":")[0] for k in golden
                    if k.startswith(tag + "/inter/")})
    errs = {}
    for name in names:
        for kind in ("val", "grad"):
            ref = golden[f"{tag}/inter/{name}:{kind}_rows"].astype(np.float64)
            t = taps.get(name, {}).get(kind)
            if t is None:
                errs[f"{name}:{kind}"] = float("inf")
                continue
            got = t.detach().double().cpu().reshape(-1, ref.shape[1])[idx].numpy()
            errs[f"{name}:{kind}"] = float(np.linalg.norm(got - ref) /
                                           max(np.linalg.norm(ref), 1e-30))
    return errs


def oracle_intra(c: dict, emulate=None) -> dict:
    with R.emulate_storage(emulate):
        return _oracle_intra(c)


def _oracle_intra(c: dict) -> dict:
    tag = c["tag"]
    p = R.hash_params(R.intra_modal_shapes(512, c["L"]), "intra.")
    for t in p.values():
        t.requires_grad_(True)
    fa_np, fb_np, w_np = spec.intra_inputs(tag, c["B"], c["T"], c["Da"], c["Db"])
    fa = torch.from_numpy(fa_np).requires_grad_(True)
    fb = torch.from_numpy(fb_np).requires_grad_(True)
    o = R.intra_modal_forward(fa, fb, p, "", c["H"], c["L"])
    (o * torch.from_numpy(w_np)).sum().backward()
    grads = {k: t.grad for k, t in p.items()}
    grads["input.a"] = fa.grad
    grads["input.b"] = fb.grad
    return {"out": o.detach().numpy(), "grads": grads}


def oracle_loss(case: dict):
    x_np, y_np = spec.loss_inputs(case)
    x = torch.from_numpy(x_np).requires_grad_(True)
    y = torch.from_numpy(y_np)
    if case["kind"] == "ccc":
        l = R.ccc_loss(x, y, digitize_num=case["k"])
    elif case["kind"] == "ccc_ignore":
        l = R.ccc_loss_ignore(x, y)
    else:
        l = R.ce_loss(x, y, case["k"])
    if l.requires_grad:
        l.backward()
    g = x.grad.numpy() if x.grad is not None else np.zeros_like(x_np)
    return float(l), g
