"""Model-level parity measurement shared by the GPU tests (tests/test_gpu_models.py) and
scripts/parity_report.py: run a golden case through the HIP drop-in modules in a compute dtype
and measure every error the 16-bit tests bound (predictions, losses, intermediates and their
gradients, parameter gradients)."""
from __future__ import annotations

import os

import numpy as np
import torch

from jmt import functional as JF  # noqa
from jmt import taps
from oracle.hashinit import init_module_
from tests.golden import spec
from tests.oracle_cases import inter_errors

DEV = torch.device("cuda")


def build_tt(c):
    from models.two_transformers import Two_transformers
    from models.fc_layer import FcLayer
    m = Two_transformers(0.0, 0.0, c["H"], c["L"], c["jm"], c["fmt"], c["vin"])
    fc = FcLayer(1024, 512)
    init_module_(m, "")
    init_module_(fc, "fc.")
    return m.to(DEV), fc.to(DEV)


def run_tt(c, cd, record=False, loss_scale: float = 1.0, model=None):
    """-> (vouts, aouts, v_loss, a_loss, grads{name: tensor}, taps{name: {val, grad}}).
    The backward runs on loss * loss_scale (GradScaler style); grads come back unscaled."""
    from losses.loss import CCCLoss
    m, fc = build_tt(c) if model is None else model
    B, T = c["B"], c["T"]
    audio, video, lv, la = spec.tt_inputs(c["tag"], B, T, c["vin"])
    a = torch.from_numpy(audio).to(DEV).requires_grad_(True)
    v = torch.from_numpy(video).to(DEV).requires_grad_(True)
    crit = CCCLoss(1)
    store = {}
    if record:
        taps.enable(store)
    try:
        with JF.compute_mode(cd):
            vo, ao = m(fc(a), v)
            vout = vo.view(-1, vo.shape[0] * vo.shape[1])
            aout = ao.view(-1, ao.shape[0] * ao.shape[1])
            l1 = crit(vout, torch.from_numpy(lv).to(DEV).view(-1, B * T))
            l2 = crit(aout, torch.from_numpy(la).to(DEV).view(-1, B * T))
            ((l1 + l2) * loss_scale).backward()
    finally:
        taps.disable()
    uns = (lambda g: g) if loss_scale == 1.0 else (lambda g: None if g is None else g / loss_scale)
    grads = {k: uns(p.grad) for k, p in m.named_parameters()}
    grads.update({"fc." + k: uns(p.grad) for k, p in fc.named_parameters()})
    grads["input.audio"] = uns(a.grad)
    grads["input.video"] = uns(v.grad)
    for d in store.values():
        if "grad" in d:
            d["grad"] = uns(d["grad"])
    return vo, ao, float(l1.detach()), float(l2.detach()), grads, store


def grad_errors(golden: dict, tag: str, grads: dict) -> dict:
    """Relative L2 error of every parameter / input gradient vs the golden norm and sample:
    {name: max(|n - n_ref| / n_ref, |sample - ref| / |ref|)}; inf if a grad is missing or
    present where the reference has none."""
    out = {}
    for name, g in grads.items():
        key = f"{tag}/{name}"
        gn = float(golden[key + ":norm"])
        if gn < 0:
            out[name] = 0.0 if g is None or float(g.abs().max()) == 0.0 else float("inf")
            continue
        if g is None:
            out[name] = float("inf")
            continue
        gg = g.detach().double().cpu().reshape(-1)
        stride = max(1, gg.numel() // spec.N_SAMPLE)
        s = gg[::stride][:spec.N_SAMPLE].numpy()
        ref = golden[key + ":sample"].astype(np.float64)
        out[name] = max(abs(float(gg.norm()) - gn) / gn,
                        float(np.linalg.norm(s - ref) / max(np.linalg.norm(ref), 1e-30)))
    return out


# fp16 runs under loss scaling, as the reference trains fp16 (train.py:89,314-316: GradScaler):
# without it the attention-score gradients (~1e-6) fall below fp16's normal range
LOSS_SCALE = {torch.float32: 1.0, torch.bfloat16: 1.0, torch.float16: 1024.0}


def errors(golden: dict, c: dict, vo, ao, l1, l2, grads, store) -> dict:
    """Every error of one run (GPU or emulating oracle) of a golden case."""
    tag = c["tag"]
    r = {"case": tag}
    for k, o in (("vouts", vo), ("aouts", ao)):
        a = np.asarray(o.detach().float().cpu().numpy() if torch.is_tensor(o) else o)
        b = golden[f"{tag}/{k}"]
        assert a.shape == b.shape, (k, a.shape, b.shape)
        r[k + "_abs"] = float(np.abs(a - b).max())
        r[k + "_of_spread"] = float(np.abs(a - b).max() / (b.max() - b.min()))
    r["loss_abs"] = max(abs(float(l1) - float(golden[f"{tag}/v_loss"])),
                        abs(float(l2) - float(golden[f"{tag}/a_loss"])))
    ge = grad_errors(golden, tag, grads)
    r["pgrad_max"] = max(ge.values())
    r["pgrad_worst"] = max(ge, key=ge.get)
    if c.get("inter"):
        ie = inter_errors(golden, tag, store)
        r["inter_val_max"] = max(v for k, v in ie.items() if k.endswith(":val"))
        r["inter_grad_max"] = max(v for k, v in ie.items() if k.endswith(":grad"))
        r["inter"] = ie
    r["pgrad"] = ge
    return r


def measure(golden: dict, c: dict, cd) -> dict:
    """Every error of one (case, dtype) GPU run."""
    res = run_tt(c, cd, record=bool(c.get("inter")), loss_scale=LOSS_SCALE[cd])
    r = errors(golden, c, *res)
    r["dtype"] = str(cd).replace("torch.", "")
    return r


def emulated(golden: dict, c: dict, cd) -> dict:
    """The same errors for the CPU oracle with 16-bit storage emulated (the error model)."""
    from tests.oracle_cases import oracle_tt
    torch.set_num_threads(min(16, max(1, len(os.sched_getaffinity(0)))))
    o = oracle_tt(c, cd, LOSS_SCALE[cd])
    return errors(golden, c, o["vouts"], o["aouts"], o["v_loss"], o["a_loss"], o["grads"],
                  o["taps"])


# 16-bit error model (tests/test_gpu_models.py): every error of the HIP run must stay within
# K16 x the error of the rounding-emulating oracle on the same case, with floors: u = 2^-8 (bf16)
# / 2^-11 (fp16) unit roundoff of 16-bit storage, and — because a single quantity's emulated error
# can be small by luck of cancellation while its neighbours' is not — the largest emulated error
# of its group: intermediates by (kind of tap, value/gradient), parameter gradients by layer.
# Measured GPU / emulated ratios (profiles/r02_parity_error_model.txt): median 1.0, p99 ~3.
K16 = 4.0
UNIT = {torch.bfloat16: 2.0 ** -8, torch.float16: 2.0 ** -11}


def _inter_group(k: str) -> str:
    name, kind = k.split(":")
    return name.split(".")[0] + ":" + kind


def _param_group(k: str) -> str:
    parts = k.split(".")
    if "layers" in parts:
        return ".".join(parts[:parts.index("layers") + 2])
    return ".".join(parts[:-1]) or k


def check16(gpu: dict, emu: dict, cd) -> list:
    """-> list of (quantity, gpu_err, bound) that break the error model."""
    u = UNIT[cd]
    bad = []

    def chk(name, g, e, floor):
        bound = K16 * max(e, floor)
        if not (g <= bound):
            bad.append((name, g, bound))

    for k in ("vouts_of_spread", "aouts_of_spread"):
        chk(k, gpu[k], emu[k], u)
    chk("loss_abs", gpu["loss_abs"], emu["loss_abs"], u)
    if "inter" in gpu:
        gmax = {}
        for k, e in emu["inter"].items():
            gmax[_inter_group(k)] = max(gmax.get(_inter_group(k), 0.0), e)
        for k, g in gpu["inter"].items():
            chk("inter:" + k, g, emu["inter"][k], max(2 * u, gmax[_inter_group(k)]))
    med = float(np.median(list(emu["pgrad"].values())))
    pmax = {}
    for k, e in emu["pgrad"].items():
        pmax[_param_group(k)] = max(pmax.get(_param_group(k), 0.0), e)
    for k, g in gpu["pgrad"].items():
        chk("pgrad:" + k, g, emu["pgrad"][k], max(med, 2 * u, pmax[_param_group(k)]))
    return bad
