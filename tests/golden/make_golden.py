"""Generate the golden vectors under tests/golden/ by running the REFERENCE itself on CPU.

Run in the build container (where /root/reference exists):
    python tests/golden/make_golden.py

Recipe: put /root/reference on sys.path with bytecode writing disabled, stub the
unused `comet_ml` / `torchvision` imports of models/mm_transformers.py:2-3,14-15, patch
Tensor.cuda to identity while losses/loss.py:16 builds its bins, overwrite every parameter with
the counter-hash values of oracle/hashinit.py, run forward + backward, save small .npz fixtures.
Inputs are NOT stored: they are regenerated from the same hash (oracle/hashinit.features/labels);
a checksum of each input is stored so a drifting generator is caught.

The reference's sources never leave this script: the fixtures are data (outputs, losses, grad
norms and strided grad samples).
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
from oracle import hashinit as hi  # noqa: E402
from tests.golden import spec  # noqa: E402

REF = "/root/reference"
N_SAMPLE = spec.N_SAMPLE


def import_reference():
    sys.dont_write_bytecode = True
    for name in ("comet_ml",):
        m = types.ModuleType(name)
        m.Experiment = object
        sys.modules[name] = m
    tv = types.ModuleType("torchvision")
    tv.transforms = types.ModuleType("torchvision.transforms")
    tv.models = types.ModuleType("torchvision.models")
    tv.models.video = types.ModuleType("torchvision.models.video")
    tv.models.video.r3d_18 = None
    for k, v in {"torchvision": tv, "torchvision.transforms": tv.transforms,
                 "torchvision.models": tv.models,
                 "torchvision.models.video": tv.models.video}.items():
        sys.modules[k] = v
    sys.path.insert(0, REF)
    import importlib
    mods = {}
    for name in ("models.two_transformers", "models.fc_layer", "models.mm_multi_transformers",
                 "models.mm_transformers", "models.intra_modal_transformer_fusion",
                 "losses.loss", "losses.CCCLoss"):
        mods[name] = importlib.import_module(name)
    return mods


def make_loss(mods, cls, *a, **k):
    orig = torch.Tensor.cuda
    torch.Tensor.cuda = lambda self, *x, **y: self
    try:
        return getattr(mods["losses.loss"], cls)(*a, **k)
    finally:
        torch.Tensor.cuda = orig


def grad_record(out: dict, tag: str, named, rsample: bool = False):
    for name, t in named:
        g = t.grad
        key = f"{tag}/{name}"
        if g is None:
            out[key + ":norm"] = np.array(-1.0)
            continue
        g = g.detach().double().reshape(-1)
        out[key + ":norm"] = np.array(float(g.norm()))
        stride = max(1, g.numel() // N_SAMPLE)
        out[key + ":sample"] = g[::stride][:N_SAMPLE].float().numpy()
        if rsample:
            out[key + ":rsample"] = g[torch.from_numpy(spec.rsample_idx(name, g.numel()))].numpy()


def checksum(x: np.ndarray) -> float:
    return float(np.float64(x).sum() + (np.float64(x) ** 2).sum())


def tap_intermediates(model, c, taps):
    """Forward hooks on the reference's own submodules: each encoder block's output, the six
    cross-attention outputs in call order (mm_multi_transformers.py:142-167 /
    mm_transformers.py:125-135) and the regressors' input (the fusion output); a tensor hook on
    each records dL/d(that tensor).  Everything is stored canonically as (B, T, F) rows."""
    mm = model.mm_transformer
    handles = []

    def add(name, seq_first):
        def store(t):
            taps[name] = {"val": (t.permute(1, 0, 2) if seq_first else t).detach().clone()}

            def ghook(g):
                taps[name]["grad"] = (g.permute(1, 0, 2) if seq_first else g).detach().clone()
            t.register_hook(ghook)
        return store

    if c["jm"] in ("TRANSFORMER", "NONE"):
        encs = ["visual_encoder", "physiological_encoder"]
        if c["jm"] == "TRANSFORMER":
            encs.append("joint_representation_encoder")
        for e in encs:
            st = add("enc." + e, c["jm"] == "TRANSFORMER")
            handles.append(getattr(mm, e).register_forward_hook(
                lambda mod, inp, o, st=st: st(o)))
        calls = []
        cas = ["cross_attention_v", "cross_attention_p"] + (
            ["cross_attention_pv"] if c["jm"] == "TRANSFORMER" else [])
        for ca in cas:
            def h(mod, inp, o):
                add(f"ca.{len(calls)}", True)(o[0])
                calls.append(1)
            handles.append(getattr(mm, ca).register_forward_hook(h))
    head_sf = c["jm"] == "TRANSFORMER" and c["fmt"] == "FC"
    st_head = add("head", head_sf)
    handles.append(model.vregressor.register_forward_hook(lambda mod, inp, o: st_head(inp[0])))
    return handles


def record_intermediates(out: dict, tag: str, taps: dict, B: int, T: int):
    idx = np.unique(np.linspace(0, B * T - 1, spec.N_INTER_ROWS).round().astype(np.int64))
    out[f"{tag}/inter_rows"] = idx
    for name, d in taps.items():
        for kind in ("val", "grad"):
            x = d[kind].reshape(B * T, -1).double()
            out[f"{tag}/inter/{name}:{kind}_norm"] = np.array(float(x.norm()))
            out[f"{tag}/inter/{name}:{kind}_rows"] = x[torch.from_numpy(idx)].float().numpy()


def run_two_transformers(mods, out, c):
    tag = c["tag"]
    torch.manual_seed(0)
    model = mods["models.two_transformers"].Two_transformers(
        0.0, 0.0, c["H"], c["L"], c["jm"], c["fmt"], c["vin"])
    fc = mods["models.fc_layer"].FcLayer(1024, 512)
    hi.init_module_(model, "", c.get("gains"))
    hi.init_module_(fc, "fc.", c.get("gains"))
    model.train()
    B, T = c["B"], c["T"]
    audio, video, lv, la = spec.tt_inputs(tag, B, T, c["vin"])
    out[f"{tag}/in_checksum"] = np.array([checksum(audio), checksum(video), checksum(lv),
                                          checksum(la)])
    a = torch.from_numpy(audio).requires_grad_(True)
    v = torch.from_numpy(video).requires_grad_(True)
    crit = make_loss(mods, "CCCLoss", 1)
    taps = {}
    handles = tap_intermediates(model, c, taps) if c.get("inter") else []
    aud = fc(a)
    vo, ao = model(aud, v)
    out[f"{tag}/vouts"] = vo.detach().numpy()
    out[f"{tag}/aouts"] = ao.detach().numpy()
    vout = vo.view(-1, vo.shape[0] * vo.shape[1])
    aout = ao.view(-1, ao.shape[0] * ao.shape[1])
    vt = torch.from_numpy(lv).view(-1, B * T)
    at = torch.from_numpy(la).view(-1, B * T)
    if c.get("loss") == "proj":          # conditioned cases: mean(w * outputs), spec.COND_CASES
        wv, wa = (torch.from_numpy(w) for w in spec.proj_inputs(c))
        l1 = (vo * wv).mean()
        l2 = (ao * wa).mean()
    else:
        l1 = crit(vout, vt)
        l2 = crit(aout, at)
    out[f"{tag}/v_loss"] = np.array(float(l1))
    out[f"{tag}/a_loss"] = np.array(float(l2))
    (l1 + l2).backward()
    for h in handles:
        h.remove()
    if taps:
        record_intermediates(out, tag, taps, B, T)
    rs = c.get("loss") == "proj"
    grad_record(out, tag, list(model.named_parameters()), rs)
    grad_record(out, tag, [("fc." + n, p) for n, p in fc.named_parameters()], rs)
    grad_record(out, tag, [("input.audio", a), ("input.video", v)], rs)

    if c.get("train_steps"):
        # 3-step training trajectory (SURVEY.md §8c last paragraph): SGD nesterov, config lr etc.
        params = list(model.parameters()) + list(fc.parameters())
        opt = torch.optim.SGD(params, lr=1e-4, momentum=0.9, dampening=0.0, weight_decay=1e-4,
                              nesterov=True)
        losses = []
        for step in range(c["train_steps"]):
            opt.zero_grad(set_to_none=True)
            vo, ao = model(fc(torch.from_numpy(audio)), torch.from_numpy(video))
            l1 = crit(vo.view(-1, B * T), vt)
            l2 = crit(ao.view(-1, B * T), at)
            (l1 + l2).backward()
            opt.step()
            losses.append([float(l1), float(l2)])
        out[f"{tag}/train_losses"] = np.array(losses)
        out[f"{tag}/train_final_out_layer1_w_sample"] = (
            model.mm_transformer.out_layer1.weight.detach().reshape(-1)[:N_SAMPLE].numpy())


def _tt_once(mods, c, ac_dtype):
    """(vouts, aouts, v_loss, a_loss, {param: grad}) of one case through the reference, fp32 or
    under CPU autocast in `ac_dtype` (the reference's own 16-bit path: train.py:101 runs the
    model under autocast; fp16 under loss scaling 1024 as its GradScaler, train.py:89)."""
    torch.manual_seed(0)
    model = mods["models.two_transformers"].Two_transformers(
        0.0, 0.0, c["H"], c["L"], c["jm"], c["fmt"], c["vin"])
    fc = mods["models.fc_layer"].FcLayer(1024, 512)
    hi.init_module_(model, "", c.get("gains"))
    hi.init_module_(fc, "fc.", c.get("gains"))
    B, T = c["B"], c["T"]
    audio, video, lv, la = spec.tt_inputs(c["tag"], B, T, c["vin"])
    crit = make_loss(mods, "CCCLoss", 1)
    ctx = (torch.autocast("cpu", dtype=ac_dtype) if ac_dtype is not None
           else torch.autocast("cpu", enabled=False))
    with ctx:
        vo, ao = model(fc(torch.from_numpy(audio)), torch.from_numpy(video))
    vo, ao = vo.float(), ao.float()
    if c.get("loss") == "proj":
        wv, wa = (torch.from_numpy(w) for w in spec.proj_inputs(c))
        l1, l2 = (vo * wv).mean(), (ao * wa).mean()
    else:
        l1 = crit(vo.reshape(1, -1), torch.from_numpy(lv).view(1, -1))
        l2 = crit(ao.reshape(1, -1), torch.from_numpy(la).view(1, -1))
    scale = 1024.0 if ac_dtype == torch.float16 else 1.0
    ((l1 + l2) * scale).backward()
    named = list(model.named_parameters()) + [("fc." + n, p) for n, p in fc.named_parameters()]
    grads = {n: p.grad.detach().double() / scale for n, p in named if p.grad is not None}
    return vo.detach().double(), ao.detach().double(), float(l1), float(l2), grads


def ref16_errors(mods, out, c):
    """The reference's OWN 16-bit error on the case: its CPU autocast bf16 / fp16 run vs its
    fp32 run — prediction error over the prediction spread, loss error, and the relative L2
    error of every parameter gradient (names in `{tag}/ref16_param_names`).  Context for the
    16-bit tests: what the reference itself achieves in 16 bits on the same weights and inputs."""
    tag = c["tag"]
    rvo, rao, rl1, rl2, rg = _tt_once(mods, c, None)
    names = sorted(rg)
    out[f"{tag}/ref16_param_names"] = np.array(names)
    for dt, key in ((torch.bfloat16, "bf16"), (torch.float16, "fp16")):
        vo, ao, l1, l2, g = _tt_once(mods, c, dt)
        spread = max(float(rvo.max() - rvo.min()), float(rao.max() - rao.min()), 1e-30)
        out[f"{tag}/ref16_{key}/out_of_spread"] = np.array(
            max(float((vo - rvo).abs().max()), float((ao - rao).abs().max())) / spread)
        out[f"{tag}/ref16_{key}/loss_abs"] = np.array(max(abs(l1 - rl1), abs(l2 - rl2)))
        out[f"{tag}/ref16_{key}/pgrad"] = np.array(
            [float((g[n] - rg[n]).norm() / max(float(rg[n].norm()), 1e-30)) for n in names])


def run_intra(mods, out, c):
    tag = c["tag"]
    m = mods["models.intra_modal_transformer_fusion"].Intra_modal_transformer_fusion(
        512, c["H"], 512, c["L"])
    hi.init_module_(m, "intra.")
    fa_np, fb_np, w_np = spec.intra_inputs(tag, c["B"], c["T"], c["Da"], c["Db"])
    fa = torch.from_numpy(fa_np).requires_grad_(True)
    fb = torch.from_numpy(fb_np).requires_grad_(True)
    o = m(fa, fb)
    out[f"{tag}/out"] = o.detach().numpy()
    (o * torch.from_numpy(w_np)).sum().backward()
    grad_record(out, tag, list(m.named_parameters()))
    grad_record(out, tag, [("input.a", fa), ("input.b", fb)])


def run_losses(mods, out):
    CCCi = mods["losses.CCCLoss"].CCCLoss
    for case in spec.LOSS_CASES:
        tag = case["tag"]
        x_np, y_np = spec.loss_inputs(case)
        x = torch.from_numpy(x_np).requires_grad_(True)
        y = torch.from_numpy(y_np)
        if case["kind"] == "ccc":
            crit = make_loss(mods, "CCCLoss", case["k"])
            l = crit(x, y)
        elif case["kind"] == "ccc_ignore":
            l = CCCi(ignore=-5.0)(x, y)
            out[f"{tag}/mask_idx"] = np.nonzero(y_np.reshape(-1) != -5.0)[0].astype(np.int64)
        elif case["kind"] == "ce":
            crit = make_loss(mods, "CELoss", case["k"])
            orig = torch.cuda.LongTensor
            try:
                torch.cuda.LongTensor = lambda a: torch.as_tensor(a, dtype=torch.long)
                l = crit(x, y)
            finally:
                torch.cuda.LongTensor = orig
        out[f"{tag}/loss"] = np.array(float(l))
        if l.requires_grad:
            l.backward()
        out[f"{tag}/grad"] = (x.grad.numpy() if x.grad is not None
                              else np.zeros_like(x_np))


def main():
    mods = import_reference()
    torch.set_num_threads(8)
    out = {}
    for c in spec.ALL_TT_CASES:
        print("case", c["tag"], flush=True)
        run_two_transformers(mods, out, c)
        ref16_errors(mods, out, c)
    for c in spec.INTRA_CASES:
        print("case", c["tag"], flush=True)
        run_intra(mods, out, c)
    run_losses(mods, out)
    path = os.path.join(HERE, "golden.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes,", len(out), "arrays")


if __name__ == "__main__":
    main()
