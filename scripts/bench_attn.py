"""Attention-core micro-benchmark at the bench workload (N=64 windows, L=300, E=512, H=1, bf16):
fused jmt_attn_fwd vs the score-GEMM + softmax + PV-GEMM path, forward and forward+backward
through AttnCoreFn (self-attention on a packed qkv projection)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "joint-multimodal-transformer-6th-abaw_amd")]

import torch  # noqa: E402

from jmt import functional as JF, ops  # noqa: E402


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    N, L, E = 64, 300, 512
    cd = torch.bfloat16
    x = torch.randn(N, L, 3 * E, device="cuda").to(cd).permute(1, 0, 2).requires_grad_(True)
    go = torch.randn(L, N, E, device="cuda").to(cd)
    for fused in (True, False):
        ops._attn_fused["on"] = fused

        def fwd():
            with torch.no_grad(), JF.compute_mode(cd):
                JF.AttnCoreFn.apply(x, x, x, E, 1, 0, E, 2 * E)

        def fwdbwd():
            with JF.compute_mode(cd):
                o = JF.AttnCoreFn.apply(x, x, x, E, 1, 0, E, 2 * E)
            o.backward(go)

        fl = 4.0 * N * L * L * E
        tf = timeit(fwd)
        tb = timeit(fwdbwd)
        print(json.dumps({"fused": fused, "fwd_us": round(tf, 1), "fwd_tflops": round(fl / tf / 1e6, 1),
                          "fwd_bwd_us": round(tb, 1)}), flush=True)
    ops._attn_fused["on"] = True


if __name__ == "__main__":
    main()
