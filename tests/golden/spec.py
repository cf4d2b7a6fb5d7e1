"""Golden case definitions and input generators (shared by make_golden.py, the oracle tests and
the GPU parity tests).  Inputs are pure functions of the case tag (oracle/hashinit.py)."""
from __future__ import annotations

import numpy as np

from oracle import hashinit as hi

N_SAMPLE = 64
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
