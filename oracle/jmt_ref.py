"""CPU restatement (oracle) of the reference's JMT fusion hot path.  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module, and
only as the checker / CPU baseline.  The product path (joint-multimodal-transformer-6th-abaw_amd/)
never imports it and fails loudly when the HIP library is missing.

It is written from the formulas of SURVEY.md §8(a) as plain torch-CPU fp32 tensor algebra (no
nn.Module from the reference, no nn.MultiheadAttention): every function cites the reference
file:line it restates.  Parameters are passed as a flat dict keyed by the reference's state_dict
names, so the same dict drives the oracle, the reference (golden generator) and the HIP modules.
Autograd gives the backward pass, which the CPU baseline in bench.py times.

Pinned: tests/test_oracle.py checks every function against the golden vectors produced by
running the reference itself (tests/golden/make_golden.py).
"""
from __future__ import annotations

import math
from typing import Dict

import torch

P = Dict[str, torch.Tensor]


# ---------------------------------------------------------------- 16-bit storage emulation ----
# emulate_storage(torch.bfloat16 / torch.float16) makes the restatement round every tensor the HIP
# path stores in the compute dtype (GEMM operands and outputs, LayerNorm / L2-norm outputs,
# attention probabilities) — in the forward value AND in the gradient flowing back through that
# point — while all arithmetic stays fp32 (fp32 MFMA accumulation, fp32 statistics).  It is the
# error model of the 16-bit parity tests: it measures what plain 16-bit storage of the reference's
# math costs on a given input, independently of the HIP kernels (tests/test_gpu_models.py).
_EMU = {"dtype": None}


class _Round(torch.autograd.Function):
    @staticmethod
    def forward(ctx, t, dtype):
        ctx.dtype = dtype
        return t.to(dtype).to(t.dtype)

    @staticmethod
    def backward(ctx, g):
        return g.to(ctx.dtype).to(g.dtype), None


class _AttnCore16(torch.autograd.Function):
    """softmax(scale Q K^T) V with 16-bit storage emulated the way a flash-style kernel stores
    it: scores / softmax in fp32, P rounded for P V, O rounded; backward with
    Delta = rowsum(dO o O) from the 16-bit dO and O, dS = P o (dP - Delta) in fp32 then rounded,
    P rounded for dV = P^T dO (the standard flash-attention backward formula)."""

    @staticmethod
    def forward(ctx, q, k, v, scale, dtype):
        r = lambda t: t.to(dtype).to(torch.float32)
        P = torch.softmax(torch.bmm(q, k.transpose(1, 2)) * scale, dim=-1)
        o = r(torch.bmm(r(P), v))
        ctx.save_for_backward(q, k, v, P, o)
        ctx.scale, ctx.dtype = scale, dtype
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, P, o = ctx.saved_tensors
        r = lambda t: t.to(ctx.dtype).to(torch.float32)
        do = r(do)
        dP = torch.bmm(do, v.transpose(1, 2))
        delta = (do * o).sum(-1, keepdim=True)
        dS = r(P * (dP - delta) * ctx.scale)
        return (r(torch.bmm(dS, k)), r(torch.bmm(dS.transpose(1, 2), q)),
                r(torch.bmm(r(P).transpose(1, 2), do)), None, None)


def rnd(t):
    d = _EMU["dtype"]
    return t if d is None else _Round.apply(t, d)


class emulate_storage:
    """`with emulate_storage(torch.bfloat16): ...` (None = exact fp32)."""

    def __init__(self, dtype):
        self.dtype = dtype

    def __enter__(self):
        self.prev = _EMU["dtype"]
        _EMU["dtype"] = self.dtype
        return self

    def __exit__(self, *a):
        _EMU["dtype"] = self.prev


# ---------------------------------------------------------------- primitives ------------------

def linear(x, W, b, out_round: bool = True):
    """nn.Linear: y = x W^T + b (models/fc_layer.py:6-12, two_transformers.py:56).  fp32: the
    same fused addmm nn.Linear runs (torch.nn.functional.linear)."""
    if _EMU["dtype"] is None:
        return torch.nn.functional.linear(x, W, b)
    y = torch.matmul(rnd(x), rnd(W).t()) + b
    return rnd(y) if out_round else y


def l2_normalize(x, eps: float = 1e-12):
    """F.normalize(x, p=2, dim=-1, eps=1e-12) (models/two_transformers.py:118-119)."""
    n = torch.sqrt((x * x).sum(-1, keepdim=True))
    return rnd(x / torch.clamp(n, min=eps))


def layer_norm(x, g, b, eps: float = 1e-5):
    """nn.LayerNorm(E) with affine params, biased variance (mm_multi_transformers.py:57-58).
    fp32: torch's layer_norm primitive (what nn.LayerNorm calls); emulated 16-bit storage: the
    explicit formula with its rounded output."""
    if _EMU["dtype"] is None:
        return torch.nn.functional.layer_norm(x, (x.shape[-1],), g, b, eps)
    mu = x.mean(-1, keepdim=True)
    xc = x - mu
    var = (xc * xc).mean(-1, keepdim=True)
    return rnd(xc * torch.rsqrt(var + eps) * g + b)


def mha(q_in, k_in, v_in, p: P, pre: str, num_heads: int):
    """nn.MultiheadAttention(E, H) forward, seq-first (L, N, E) inputs, dropout 0.

    Packed in_proj (3E, E) / (3E,): q = q_in Wq^T + bq, k = k_in Wk^T + bk, v = v_in Wv^T + bv,
    q scaled by head_dim^-1/2, S = q k^T, P = softmax(S), O = P v, out_proj.  The averaged
    attention weights the module also returns are discarded at every reference call site
    (mm_multi_transformers.py:62,142-167,186; mm_transformers.py:125-135;
    intra_modal_transformer_fusion.py:104).
    """
    E = q_in.shape[-1]
    W = p[pre + "in_proj_weight"]
    bi = p[pre + "in_proj_bias"]
    q = linear(q_in, W[:E], bi[:E])
    k = linear(k_in, W[E:2 * E], bi[E:2 * E])
    v = linear(v_in, W[2 * E:], bi[2 * E:])
    L, N, _ = q.shape
    S = k.shape[0]
    H = num_heads
    dh = E // H
    q = q.reshape(L, N * H, dh).transpose(0, 1)
    k = k.reshape(S, N * H, dh).transpose(0, 1)
    v = v.reshape(S, N * H, dh).transpose(0, 1)
    if _EMU["dtype"] is None:
        a = torch.softmax(torch.bmm(q * (1.0 / math.sqrt(dh)), k.transpose(1, 2)), dim=-1)
        o = torch.bmm(a, v)
    else:
        o = _AttnCore16.apply(q, k, v, 1.0 / math.sqrt(dh), _EMU["dtype"])
    o = o.transpose(0, 1).reshape(L, N, E)
    return linear(o, p[pre + "out_proj.weight"], p[pre + "out_proj.bias"])


def encoder_layer(x, p: P, pre: str, num_heads: int):
    """Post-LN TransformerEncoderLayer.forward (mm_multi_transformers.py:61-70; identical copies
    in mm_transformers.py:74-84 and intra_modal_transformer_fusion.py:207-217)."""
    a = mha(x, x, x, p, pre + "attention.", num_heads)
    x = layer_norm(x + a, p[pre + "layer_norm1.weight"], p[pre + "layer_norm1.bias"])
    h = torch.relu(linear(x, p[pre + "feed_forward.0.weight"], p[pre + "feed_forward.0.bias"]))
    f = linear(h, p[pre + "feed_forward.2.weight"], p[pre + "feed_forward.2.bias"])
    return layer_norm(x + f, p[pre + "layer_norm2.weight"], p[pre + "layer_norm2.bias"])


def encoder_block(x, p: P, pre: str, num_heads: int, num_layers: int):
    """TransformerEncoderBlock / SequentialEncoder (mm_multi_transformers.py:29-45)."""
    for i in range(num_layers):
        x = encoder_layer(x, p, f"{pre}layers.{i}.", num_heads)
    return x


# ---------------------------------------------------------------- fusion models --------------

def _tap(taps, name, t, seq_first):
    """Record an intermediate as (tensor, seq_first); (B, T, F) is the canonical layout (test
    infrastructure: the golden generator taps the same points of the reference with hooks)."""
    if taps is not None:
        taps[name] = (t, seq_first)


def w_jr_forward(visual, phys, p: P, pre: str, H: int, L: int, output_format: str, taps=None):
    """MultimodalTransformer_w_JR.forward (models/mm_multi_transformers.py:118-214).
    visual/phys: (B, T, 512).  FC -> (T, B, 1024); SELF_ATTEN -> (B, T, 512)."""
    jr = linear(torch.cat((visual, phys), dim=2), p[pre + "out_layer_pv.weight"],
                p[pre + "out_layer_pv.bias"])                                   # :120-124
    v = visual.permute(1, 0, 2)                                                 # :127-129
    a = phys.permute(1, 0, 2)
    j = jr.permute(1, 0, 2)
    v = encoder_block(v, p, pre + "visual_encoder.", H, L)                      # :132-136
    a = encoder_block(a, p, pre + "physiological_encoder.", H, L)
    j = encoder_block(j, p, pre + "joint_representation_encoder.", H, L)
    _tap(taps, "enc.visual_encoder", v, True)
    _tap(taps, "enc.physiological_encoder", a, True)
    _tap(taps, "enc.joint_representation_encoder", j, True)
    cv, cp, cpv = pre + "cross_attention_v.", pre + "cross_attention_p.", pre + "cross_attention_pv."
    outs = [mha(v, a, a, p, cv, H),                                             # :142-167
            mha(a, v, v, p, cp, H),
            mha(j, v, v, p, cpv, H),
            mha(v, j, j, p, cv, H),
            mha(j, a, a, p, cpv, H),
            mha(a, j, j, p, cp, H)]
    for i, o in enumerate(outs):
        _tap(taps, f"ca.{i}", o, True)
    if output_format == "SELF_ATTEN":                                           # :169-199
        st = torch.stack(outs, dim=2)                     # (T, B, 6, E)
        st = st.permute(1, 0, 2, 3)                       # (B, T, 6, E)
        Bsz, Tsz = st.shape[0], st.shape[1]
        flat = st.flatten(0, 1).permute(1, 0, 2)          # (6, B*T, E)
        enc = encoder_block(flat, p, pre + "final_visual_encoder.", H, L)
        fa = mha(enc, enc, enc, p, pre + "final_self_attention.", H)
        fa = fa.permute(1, 0, 2).unflatten(0, (Bsz, Tsz))
        return fa[:, :, -1, :]
    cat = torch.cat(outs, dim=2)                                                # :201-211
    return linear(cat, p[pre + "out_layer1.weight"], p[pre + "out_layer1.bias"])


def wo_jr_forward(visual, phys, p: P, pre: str, H: int, L: int, taps=None):
    """MultimodalTransformer_wo_JR.forward (models/mm_transformers.py:119-146).  The encoders are
    applied to (B, T, D) directly, i.e. self-attention runs over the batch axis (:120-122)."""
    v = encoder_block(visual, p, pre + "visual_encoder.", H, L)
    a = encoder_block(phys, p, pre + "physiological_encoder.", H, L)
    _tap(taps, "enc.visual_encoder", v, False)
    _tap(taps, "enc.physiological_encoder", a, False)
    ov = mha(v.permute(1, 0, 2), a.permute(1, 0, 2), a.permute(1, 0, 2), p,
             pre + "cross_attention_v.", H)
    op = mha(a.permute(1, 0, 2), v.permute(1, 0, 2), v.permute(1, 0, 2), p,
             pre + "cross_attention_p.", H)
    ov, op = ov.permute(1, 0, 2), op.permute(1, 0, 2)
    _tap(taps, "ca.0", ov, False)
    _tap(taps, "ca.1", op, False)
    return linear(torch.cat((ov, op), dim=2), p[pre + "final_layer.weight"],
                  p[pre + "final_layer.bias"])


def feature_concat_fc(visual, audio, p: P, pre: str):
    """FeatureConcatFC.forward (models/mm_multi_transformers.py:221-224)."""
    return linear(torch.cat((visual, audio), dim=2), p[pre + "fc.weight"], p[pre + "fc.bias"])


def intra_modal_forward(fa, fb, p: P, pre: str, H: int, L: int):
    """Intra_modal_transformer_fusion.forward (models/intra_modal_transformer_fusion.py:84-111)."""
    if fa.shape[-1] == 768:
        fa = linear(fa, p[pre + "fc.weight"], p[pre + "fc.bias"])
    if fb.shape[-1] == 768:
        fb = linear(fb, p[pre + "fc.weight"], p[pre + "fc.bias"])
    st = torch.stack((fa, fb), dim=2)                   # (B, T, 2, E)
    Bsz, Tsz = st.shape[0], st.shape[1]
    flat = st.flatten(0, 1).permute(1, 0, 2)            # (2, B*T, E)
    enc = encoder_block(flat, p, pre + "final_visual_encoder.", H, L)
    fa_ = mha(enc, enc, enc, p, pre + "final_self_attention.", H)
    fa_ = fa_.permute(1, 0, 2).unflatten(0, (Bsz, Tsz))
    return fa_[:, :, -1, :]


def regressor(x, p: P, pre: str):
    """Linear(dim,128)-ReLU-Dropout(p)-Linear(128,1) (two_transformers.py:104-114); dropout is
    identity at p=0 (config_file.json:69-70) and in eval."""
    h = torch.relu(linear(x, p[pre + "0.weight"], p[pre + "0.bias"]))
    return linear(h, p[pre + "3.weight"], p[pre + "3.bias"], out_round=False)   # fp32 out


def two_transformers_forward(audio, video, p: P, H: int, L: int, joint_modalities: str,
                             output_format: str = "FC", vision_in_ft: int = 512, taps=None):
    """Two_transformers.forward (models/two_transformers.py:116-128).  Argument order is
    (f1_norm=audio, f2_norm=video).  `taps` (optional dict) receives the intermediates the golden
    generator records (encoder outputs, the cross-attention outputs, the regressors' input)."""
    vid = l2_normalize(video)
    aud = l2_normalize(audio)
    if vision_in_ft != 512:
        vid = linear(vid, p["linear.weight"], p["linear.bias"])
    if joint_modalities == "TRANSFORMER":
        av = w_jr_forward(vid, aud, p, "mm_transformer.", H, L, output_format, taps)
    elif joint_modalities == "FC":
        av = feature_concat_fc(vid, aud, p, "mm_transformer.")
    elif joint_modalities == "NONE":
        av = wo_jr_forward(vid, aud, p, "mm_transformer.", H, L, taps)
    else:
        raise NotImplementedError(joint_modalities)
    _tap(taps, "head", av, joint_modalities == "TRANSFORMER" and output_format == "FC")
    vo = regressor(av, p, "vregressor.")
    ao = regressor(av, p, "aregressor.")
    return vo.squeeze(2), ao.squeeze(2)


# ---------------------------------------------------------------- losses ---------------------

def ccc_loss(x, y, eps: float = 1e-8, digitize_num: int = 1, rng=(-1, 1)):
    """losses/loss.py:18-32 CCCLoss.forward.  x (1,N) preds or (N,k) logits, y (1,N) labels."""
    y = y.reshape(-1)
    if digitize_num != 1:
        bins = torch.linspace(rng[0], rng[1], digitize_num, dtype=torch.float64).float().view(1, -1)
        x = (torch.softmax(x, dim=-1) * bins).sum(-1)
    x = x.reshape(-1)
    vx = x - x.mean()
    vy = y - y.mean()
    rho = (vx * vy).sum() / (torch.sqrt((vx * vx).sum()) * torch.sqrt((vy * vy).sum()) + eps)
    xm, ym = x.mean(), y.mean()
    xs, ys = x.std(), y.std()          # unbiased
    ccc = 2 * rho * xs * ys / (xs * xs + ys * ys + (xm - ym) ** 2)
    return 1 - ccc


def ccc_loss_ignore(y_pred, y_true, ignore: float = -5.0):
    """losses/CCCLoss.py:15-43 CCCLoss.forward (ignore-masked; note the swapped std names and the
    division by the pre-mask size(0))."""
    bs = y_pred.shape[0]
    idx = y_true != ignore
    t = y_true[idx]
    pr = y_pred[idx]
    if t.shape[0] <= 1:
        return torch.zeros((), dtype=torch.float32)
    xm, ym = pr.mean(), t.mean()
    x_std, y_std = t.std(), pr.std()
    s_xy = ((pr - xm) * (t - ym)).sum()
    den = x_std ** 2 + y_std ** 2 + (xm - ym) ** 2 + 1e-8
    return torch.mean(1 - 2 * s_xy / (den * bs))


def ce_loss(x, y, digitize_num: int, rng=(-1, 1), weights=None):
    """losses/loss.py:34-51 CELoss.forward: labels digitized into `digitize_num` bins."""
    import numpy as np
    y = y.reshape(-1)
    edges = np.linspace(rng[0], rng[1], num=digitize_num + 1)
    yd = np.digitize(y.detach().cpu().numpy(), edges) - 1
    yd[yd == digitize_num] = digitize_num - 1
    w = None if weights is None else torch.as_tensor(weights, dtype=torch.float32)
    return torch.nn.functional.cross_entropy(x, torch.as_tensor(yd, dtype=torch.long), weight=w)


# ---------------------------------------------------------------- train step -----------------

def sgd_nesterov_(params: P, grads: P, bufs: P, lr=1e-4, momentum=0.9, weight_decay=1e-4,
                  dampening=0.0):
    """torch.optim.SGD(nesterov=True) as configured by config_file.json:73-80 and
    instantiator.py:32-38.  Params with no grad (final_encoder) are skipped."""
    keys = [k for k, p in params.items() if grads.get(k) is not None]
    if not keys:
        return
    with torch.no_grad():
        ps = [params[k] for k in keys]
        # d = g + wd p; buf = d (first step) or momentum buf + (1 - dampening) d;
        # d += momentum buf; p -= lr d  (multi-tensor form of the same per-tensor updates)
        ds = torch._foreach_add([grads[k] for k in keys], ps, alpha=weight_decay)
        if keys[0] not in bufs:
            for k, d in zip(keys, ds):
                bufs[k] = d.clone()
        else:
            bs = [bufs[k] for k in keys]
            torch._foreach_mul_(bs, momentum)
            torch._foreach_add_(bs, ds, alpha=1 - dampening)
        torch._foreach_add_(ds, [bufs[k] for k in keys], alpha=momentum)
        torch._foreach_add_(ps, ds, alpha=-lr)


def train_step(params: P, fc_params: P, audio_raw, video, labels_v, labels_a, H, L, jm, fmt,
               vision_in_ft, bufs: P):
    """One reference training step (train.py:283-316): FcLayer on the audio, fusion model,
    (1, B*T) flatten of preds and labels, CCCLoss(1) on V and A, sum, backward, SGD.
    Returns (v_loss, a_loss, grads)."""
    allp = dict(params)
    allp.update({"fc." + k: v for k, v in fc_params.items()})
    for v in allp.values():
        v.requires_grad_(True)
        v.grad = None
    aud = linear(audio_raw, fc_params["fc_layer.weight"], fc_params["fc_layer.bias"])
    vo, ao = two_transformers_forward(aud, video, params, H, L, jm, fmt, vision_in_ft)
    vout = vo.reshape(-1, vo.shape[0] * vo.shape[1])
    aout = ao.reshape(-1, ao.shape[0] * ao.shape[1])
    vt = labels_v.reshape(-1, labels_v.shape[0] * labels_v.shape[1])
    at = labels_a.reshape(-1, labels_a.shape[0] * labels_a.shape[1])
    lv = ccc_loss(vout, vt)
    la = ccc_loss(aout, at)
    (lv + la).backward()
    grads = {k: (v.grad.detach().clone() if v.grad is not None else None) for k, v in allp.items()}
    for v in allp.values():
        v.requires_grad_(False)
    sgd_nesterov_(allp, grads, bufs)
    return lv.detach(), la.detach(), grads


# ---------------------------------------------------------------- shapes ---------------------

def _enc_layer_shapes(pre: str, E: int, Hd: int) -> dict:
    return {
        pre + "attention.in_proj_weight": (3 * E, E),
        pre + "attention.in_proj_bias": (3 * E,),
        pre + "attention.out_proj.weight": (E, E),
        pre + "attention.out_proj.bias": (E,),
        pre + "feed_forward.0.weight": (Hd, E),
        pre + "feed_forward.0.bias": (Hd,),
        pre + "feed_forward.2.weight": (E, Hd),
        pre + "feed_forward.2.bias": (E,),
        pre + "layer_norm1.weight": (E,),
        pre + "layer_norm1.bias": (E,),
        pre + "layer_norm2.weight": (E,),
        pre + "layer_norm2.bias": (E,),
    }


def _mha_shapes(pre: str, E: int) -> dict:
    return {pre + "in_proj_weight": (3 * E, E), pre + "in_proj_bias": (3 * E,),
            pre + "out_proj.weight": (E, E), pre + "out_proj.bias": (E,)}


def _block_shapes(pre: str, E: int, Hd: int, L: int) -> dict:
    d = {}
    for i in range(L):
        d.update(_enc_layer_shapes(f"{pre}layers.{i}.", E, Hd))
    return d


def two_transformers_shapes(L: int, joint_modalities: str, output_format: str = "FC",
                            vision_in_ft: int = 512, digitize_num: int = 1) -> dict:
    """state_dict key -> shape of Two_transformers (SURVEY.md §8a 'state_dict keys')."""
    d = {}
    if vision_in_ft != 512:
        d.update({"linear.weight": (512, vision_in_ft), "linear.bias": (512,)})
    m = "mm_transformer."
    if joint_modalities == "TRANSFORMER":
        for enc in ("visual_encoder.", "physiological_encoder.", "joint_representation_encoder."):
            d.update(_block_shapes(m + enc, 512, 512, L))
        d.update(_block_shapes(m + "final_encoder.", 3072, 512, L))
        for ca in ("cross_attention_v.", "cross_attention_p.", "cross_attention_pv."):
            d.update(_mha_shapes(m + ca, 512))
        d.update({m + "out_layer_pv.weight": (512, 1024), m + "out_layer_pv.bias": (512,)})
        if output_format == "FC":
            d.update({m + "out_layer1.weight": (1024, 3072), m + "out_layer1.bias": (1024,)})
            dim = 1024
        else:
            d.update(_block_shapes(m + "final_visual_encoder.", 512, 512, L))
            d.update(_mha_shapes(m + "final_self_attention.", 512))
            dim = 512
    elif joint_modalities == "FC":
        d.update({m + "fc.weight": (512, 1024), m + "fc.bias": (512,)})
        dim = 512
    else:
        for enc in ("visual_encoder.", "physiological_encoder."):
            d.update(_block_shapes(m + enc, 512, 512, L))
        for ca in ("cross_attention_v.", "cross_attention_p."):
            d.update(_mha_shapes(m + ca, 512))
        d.update({m + "gated_attention.weight": (1, 1024), m + "gated_attention.bias": (1,),
                  m + "final_layer.weight": (512, 1024), m + "final_layer.bias": (512,)})
        dim = 512
    for r in ("vregressor.", "aregressor."):
        d.update({r + "0.weight": (128, dim), r + "0.bias": (128,),
                  r + "3.weight": (digitize_num, 128), r + "3.bias": (digitize_num,)})
    return d


def intra_modal_shapes(feat_dim: int, L: int, hidden_dim: int = 512) -> dict:
    d = _block_shapes("final_visual_encoder.", feat_dim, hidden_dim, L)
    d.update(_mha_shapes("final_self_attention.", 512))
    d.update({"fc.weight": (512, 768), "fc.bias": (512,)})
    return d


def hash_params(shapes: dict, prefix: str = "", gains=None) -> P:
    from oracle.hashinit import param_value
    return {k: torch.from_numpy(param_value(prefix + k, s, gains)) for k, s in shapes.items()}
