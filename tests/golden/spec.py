"""Golden case definitions and input generators (shared by make_golden.py, the oracle tests and
the GPU parity tests).  Inputs are pure functions of the case tag (oracle/hashinit.py)."""
from __future__ import annotations

import numpy as np

from oracle import hashinit as hi

N_SAMPLE = 64
N_RSAMPLE = 512       # hash-chosen elements per gradient (conditioned cases, rsample_idx)
N_INTER_ROWS = 8      # (b, t) rows sampled from each recorded intermediate (make_golden.py)

# Two_transformers (+ FcLayer(1024,512) on the audio, as main.py:379 / train.py:265) cases.
TT_CASES = [
    dict(tag="none_fc", jm="NONE", fmt="FC", H=1, L=1, B=2, T=37, vin=2048, inter=True),
    dict(tag="tr_fc", jm="TRANSFORMER", fmt="FC", H=1, L=1, B=2, T=37, vin=2048, train_steps=3,
         inter=True),
    dict(tag="tr_fc_h8l2", jm="TRANSFORMER", fmt="FC", H=8, L=2, B=2, T=16, vin=2048),
    dict(tag="tr_sa", jm="TRANSFORMER", fmt="SELF_ATTEN", H=1, L=1, B=2, T=16, vin=2048,
         inter=True),
    dict(tag="tr_fc_t300", jm="TRANSFORMER", fmt="FC", H=1, L=1, B=2, T=300, vin=2048,
         inter=True),
    dict(tag="fcjoint", jm="FC", fmt="FC", H=1, L=1, B=3, T=37, vin=512),
]

# Conditioned cases (round 3): the STRICT 16-bit suite (tests/parity.py check16_strict: every
# error <= min(ceiling, K_STRICT x the rounding-emulating oracle's), ceilings 5 % bf16 / 2 % fp16 on
# predictions, losses and every parameter gradient).  Gains only on in_proj (oracle/hashinit.py
# GAINS_COND: attention peaked enough to carry signal) and the objective
# mean(w_v * vouts) + mean(w_a * aouts) with w in [0.5, 1.5] (hashinit.proj_weights): each
# parameter gradient is then a well-conditioned sum.  The CCC-trained GAINS cases above are kept
# for fp32 and for the comparison with the reference's own 16-bit autocast path.
COND_CASES = [
    dict(tag="cond_tr_fc", jm="TRANSFORMER", fmt="FC", H=1, L=1, B=4, T=61, vin=2048,
         inter=True, gains=hi.GAINS_COND, loss="proj", score_path=True),
    dict(tag="cond_tr_fc_t300", jm="TRANSFORMER", fmt="FC", H=1, L=1, B=2, T=300, vin=2048,
         inter=True, gains=hi.GAINS_COND_T300, loss="proj", score_path=True),
    dict(tag="cond_none_fc", jm="NONE", fmt="FC", H=1, L=1, B=4, T=61, vin=2048, inter=True,
         gains=hi.GAINS_COND, loss="proj"),
    dict(tag="cond_tr_sa", jm="TRANSFORMER", fmt="SELF_ATTEN", H=1, L=1, B=2, T=37, vin=2048,
         inter=True, gains=(), loss="proj"),
    dict(tag="cond_tr_fc_h8l2", jm="TRANSFORMER", fmt="FC", H=8, L=2, B=2, T=37, vin=2048,
         gains=hi.GAINS_COND, loss="proj"),
    dict(tag="cond_fcjoint", jm="FC", fmt="FC", H=1, L=1, B=16, T=61, vin=512,
         gains=hi.GAINS_COND, loss="proj"),
]
ALL_TT_CASES = TT_CASES + COND_CASES


def out_shape(c: dict):
    """Shape of each regressor output: (T, B) for TRANSFORMER/FC (seq-first), else (B, T)."""
    return (c["T"], c["B"]) if c["jm"] == "TRANSFORMER" and c["fmt"] == "FC" else (c["B"], c["T"])


def proj_inputs(c: dict):
    """(w_v, w_a) of a conditioned case's objective, shaped like the outputs."""
    return (hi.proj_weights(c["tag"] + ".wv", out_shape(c)),
            hi.proj_weights(c["tag"] + ".wa", out_shape(c)))


# Intra_modal_transformer_fusion cases: config 1 exactly (B=2,T=64,D=512), plus the 768 path.
INTRA_CASES = [
    dict(tag="intra", H=1, L=1, B=2, T=64, Da=512, Db=512),
    dict(tag="intra768_h8l2", H=8, L=2, B=2, T=16, Da=768, Db=512),
]

LOSS_CASES = [
    dict(tag="ccc_n600", kind="ccc", k=1, N=600),
    dict(tag="ccc_n2", kind="ccc", k=1, N=2),
    dict(tag="ccc_dig5", kind="ccc", k=5, N=300),
    dict(tag="ccci_5pct", kind="ccc_ignore", N=600, frac=0.05),
    dict(tag="ccci_all", kind="ccc_ignore", N=50, frac=1.01),
    dict(tag="ccci_one", kind="ccc_ignore", N=50, frac=-1.0),
    dict(tag="ccci_1d", kind="ccc_ignore", N=97, frac=0.3, oned=True),
    dict(tag="ce_k5", kind="ce", k=5, N=300),
]


def tt_inputs(tag: str, B: int, T: int, vin: int):
    audio = hi.features(tag + ".audio", (B, T, 1024))
    video = hi.features(tag + ".video", (B, T, vin))
    lv = hi.labels(tag + ".lv", (B, T))
    la = hi.labels(tag + ".la", (B, T))
    return audio, video, lv, la


def intra_inputs(tag: str, B: int, T: int, Da: int, Db: int):
    fa = hi.features(tag + ".a", (B, T, Da))
    fb = hi.features(tag + ".b", (B, T, Db))
    w = hi.features(tag + ".w", (B, T, 512))
    return fa, fb, w


def loss_inputs(case: dict):
    tag, N = case["tag"], case["N"]
    if case["kind"] == "ccc":
        if case["k"] == 1:
            x = hi.features(tag + ".x", (1, N)) * 0.5
        else:
            x = hi.features(tag + ".x", (N, case["k"])) * 2.0
        y = hi.labels(tag + ".y", (1, N))
        return x.astype(np.float32), y
    if case["kind"] == "ccc_ignore":
        shape = (N,) if case.get("oned") else (1, N)
        x = (hi.features(tag + ".x", shape) * 0.5).astype(np.float32)
        frac = case["frac"]
        if frac < 0:   # exactly one surviving label
            y = np.full(shape, -5.0, np.float32)
            y.reshape(-1)[3] = 0.25
        else:
            y = hi.labels(tag + ".y", shape, ignore_frac=frac)
        return x, y
    if case["kind"] == "ce":
        x = hi.features(tag + ".x", (N, case["k"])) * 2.0
        y = hi.labels(tag + ".y", (1, N))
        return x.astype(np.float32), y
    raise ValueError(case)


def rsample_idx(name: str, numel: int) -> np.ndarray:
    """Indices of the gradient elements the conditioned cases store (`{tag}/{name}:rsample`):
    every element when numel <= N_RSAMPLE, else N_RSAMPLE distinct hash-chosen positions spread
    over all rows and columns (the strided `:sample` of 64 hits one column of a 512-wide
    weight, too narrow for a relative-error estimate)."""
    if numel <= N_RSAMPLE:
        return np.arange(numel, dtype=np.int64)
    u = hi.uniform01("ridx:" + name, 4 * N_RSAMPLE)
    idx = np.unique((u * numel).astype(np.int64))
    return idx[:N_RSAMPLE]

