"""The FC head's out_layer1 forward as the step launches it (grouped.ConcatLinearFn: A = six
K-concatenated (B T, 512) segments, bias) against the same GEMM on a plain strided A, forced
configs interleaved in one process: which part of the launch costs what.

    python scripts/gemm_kcat_probe.py [--cfg 32 45] [--reps 30] [--rounds 5]
Reference point only: nothing here is on the product path."""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "joint-multimodal-transformer-6th-abaw_amd")]

import torch  # noqa: E402

from jmt import _lib, ops  # noqa: E402
from jmt._lib import BF16  # noqa: E402


def timed(fn, reps):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", type=int, nargs="*", default=[32, 45])
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--rounds", type=int, default=5)
    args = ap.parse_args()
    lib = _lib.load()
    dev = "cuda"
    R, E, S, N = 19200, 512, 6, 1024
    g = torch.Generator(device=dev).manual_seed(3)
    X = (torch.rand(S, R, E, device=dev, generator=g) * 2 - 1).bfloat16()
    Xp = torch.cat([X[s] for s in range(S)], 1).contiguous()
    W = (torch.rand(N, S * E, device=dev, generator=g) * 2 - 1).bfloat16()
    b = torch.rand(N, device=dev, generator=g)
    y = torch.empty(R, N, device=dev, dtype=torch.bfloat16)
    forms = {
        "kcat_bias": dict(a=[X[s].data_ptr() for s in range(S)], lda=E, a_mode=2, a_kseg=E,
                          bias=b, bias_mode=1),
        "kcat": dict(a=[X[s].data_ptr() for s in range(S)], lda=E, a_mode=2, a_kseg=E),
        "plain_bias": dict(a=[Xp.data_ptr()], lda=S * E, bias=b, bias_mode=1),
        "plain": dict(a=[Xp.data_ptr()], lda=S * E),
    }
    arms = {}
    for name, kw in forms.items():
        for cfg in args.cfg:
            def f(kw=kw, cfg=cfg):
                lib.jmt_gemm_set_debug(cfg << 8)
                ops.gemm(M=R, N=N, K=S * E, ab_dtype=BF16, c_dtype=BF16, a_kmajor=True,
                         b=[W.data_ptr()], ldb=S * E, b_kmajor=True, c=[y.data_ptr()], ldc=N,
                         device=dev, **kw)
            arms[f"{name}_cfg{cfg}"] = f
    ref = (Xp.float() @ W.float().t())
    for k, f in arms.items():
        f()
        torch.cuda.synchronize()
        want = ref + b if "bias" in k else ref
        err = float((y.float() - want).abs().max() / want.abs().max())
        assert err < 1e-2, (k, err)
    res = {k: [] for k in arms}
    for _ in range(args.rounds):
        for k, f in arms.items():
            res[k].append(timed(f, args.reps))
    lib.jmt_gemm_set_debug(0)
    out = {}
    for k, v in res.items():
        v.sort()
        out[k] = {"us_med": round(v[len(v) // 2], 2), "us_min": round(v[0], 2)}
    print(json.dumps({"shape": "NT 19200x1024x3072 out_layer1", **out}), flush=True)


if __name__ == "__main__":
    main()
