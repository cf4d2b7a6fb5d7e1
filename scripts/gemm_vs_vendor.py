"""gemm.hip against the vendor BLAS (torch.bmm -> hipBLASLt) on the JMT step's GEMM shapes, same
random bf16 operands, interleaved in one process (cdna_hip_programming.md §5.4 rule 24).

    python scripts/gemm_vs_vendor.py [--reps 30] [--rounds 3] [--only NT] [--cfg 0 5 30]

Layouts as the step launches them (M = B*T rows):
  NT  y = x W^T          (forward)      x (b, M, K) K-major, W (b, N, K) K-major
  NN  dx = dy W          (dgrad)        dy (b, M, K) K-major, W (b, K, N) N-major
  TN  dW = dy^T x        (wgrad)        dy (b, K, M) M-major, x (b, K, N) N-major, fp32 out
Reference point only: nothing here is on the product path."""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "joint-multimodal-transformer-6th-abaw_amd")]

import torch  # noqa: E402

from jmt import _lib, ops  # noqa: E402
from jmt._lib import BF16, F32  # noqa: E402

R = 19200
# (name, layout, batch, M, N, K)
SHAPES = [
    ("NT b3 19200x512x512", "NT", 3, R, 512, 512),
    ("NT b6 19200x1024x512", "NT", 6, R, 1024, 512),
    ("NT b3 19200x1536x512", "NT", 3, R, 1536, 512),
    ("NT b1 19200x512x2048", "NT", 1, R, 512, 2048),
    ("NT b1 19200x512x1024", "NT", 1, R, 512, 1024),
    ("NT b1 19200x1024x3072", "NT", 1, R, 1024, 3072),
    ("NN b1 19200x512x3072", "NN", 1, R, 512, 3072),
    ("NN b1 19200x1024x256", "NN", 1, R, 1024, 256),
    ("NT b2 19200x128x1024", "NT", 2, R, 128, 1024),
    ("NN b2 19200x512x512", "NN", 2, R, 512, 512),      # out_layer_pv's stacked-stream dgrad
    ("NN b3 19200x512x512", "NN", 3, R, 512, 512),
    ("NN b6 19200x512x1024", "NN", 6, R, 512, 1024),
    ("NN b3 19200x512x1536", "NN", 3, R, 512, 1536),
    ("TN b3 512x512x19200", "TN", 3, 512, 512, R),
    ("TN b3 1536x512x19200", "TN", 3, 1536, 512, R),
    ("TN b6 1024x512x19200", "TN", 6, 1024, 512, R),
    # round 6: the merged weight gradients (encoder W1 + W2 as b6; a cross-attention module's
    # two uses as one K = 2 B T entry, timed here as a plain long-K TN)
    ("TN b6 512x512x19200", "TN", 6, 512, 512, R),
    ("TN b3 512x512x38400", "TN", 3, 512, 512, 2 * R),
    ("TN b3 1024x512x38400", "TN", 3, 1024, 512, 2 * R),
]


def make(layout, b, M, N, K, dev, pad=0):
    """pad: extra elements on every operand row (row strides off the power of two)."""
    g = torch.Generator(device=dev).manual_seed(1)
    r = lambda rows, cols: (torch.rand(b, rows, cols + pad, device=dev, generator=g) * 2 - 1
                            ).bfloat16()[:, :, :cols]
    if layout == "NT":
        a, w = r(M, K), r(N, K)
        ref = lambda: torch.bmm(a, w.transpose(1, 2))
        kw = dict(a_kmajor=True, b_kmajor=True, lda=K + pad, ldb=K + pad,
                  sA=(M * (K + pad), 0), sB=(N * (K + pad), 0))
        cdt = BF16
    elif layout == "NN":
        a, w = r(M, K), r(K, N)
        ref = lambda: torch.bmm(a, w)
        kw = dict(a_kmajor=True, b_kmajor=False, lda=K + pad, ldb=N + pad,
                  sA=(M * (K + pad), 0), sB=(K * (N + pad), 0))
        cdt = BF16
    else:
        a, w = r(K, M), r(K, N)
        ref = lambda: torch.bmm(a.transpose(1, 2), w)     # (vendor writes bf16, ours fp32)
        kw = dict(a_kmajor=False, b_kmajor=False, lda=M + pad, ldb=N + pad,
                  sA=(K * (M + pad), 0), sB=(K * (N + pad), 0))
        cdt = F32
    c = torch.empty(b, M, N, device=dev, dtype=torch.float32 if cdt == F32 else torch.bfloat16)
    kw.update(M=M, N=N, K=K, ab_dtype=BF16, c_dtype=cdt, a=[a.data_ptr()], b=[w.data_ptr()],
              c=[c.data_ptr()], ldc=N, batch0=b, sC=(M * N, 0), splits=None, device=dev)
    return a, w, c, ref, kw


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
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--only", default="")
    ap.add_argument("--cfg", type=int, nargs="*", default=[0])
    ap.add_argument("--no-vendor", action="store_true")
    ap.add_argument("--pad", type=int, nargs="*", default=[0],
                    help="operand row padding (elements) per pass")
    ap.add_argument("--dbg", type=int, nargs="*", default=[0],
                    help="ablation flags per arm (1 skip MFMA, 2 skip epilogue, 32 drain stores)")
    args = ap.parse_args()
    lib = _lib.load()
    dev = "cuda"
    for name, layout, b, M, N, K, pad in [s + (pd,) for s in SHAPES for pd in args.pad]:
        if args.only and not any(s in name for s in args.only.split(",")):
            continue
        a, w, c, ref, kw = make(layout, b, M, N, K, dev, pad)
        name = name + (f" pad{pad}" if pad else "")
        arms = {}
        if not args.no_vendor:
            arms["vendor"] = ref
        for cfg in args.cfg:
            for dbg in args.dbg:
                def ours(cfg=cfg, dbg=dbg):
                    lib.jmt_gemm_set_debug((cfg << 8) | dbg)
                    ops.gemm(**kw)
                arms[f"ours_cfg{cfg}" + (f"_dbg{dbg}" if dbg else "")] = ours
        # correctness of ours vs vendor (fp32 compare)
        lib.jmt_gemm_set_debug(args.cfg[0] << 8)
        ops.gemm(**kw)
        if not args.no_vendor:
            rv = ref().float()
            err = float((c.float() - rv).abs().max() / rv.abs().max())
        else:
            err = None
        for f in arms.values():
            for _ in range(3):
                f()
        torch.cuda.synchronize()
        res = {k: [] for k in arms}
        for _ in range(args.rounds):
            for k, f in arms.items():
                res[k].append(timed(f, args.reps))
        fl = 2.0 * b * M * N * K
        out = {"shape": name, "rel_err_vs_vendor": err}
        for k, v in res.items():
            v.sort()
            out[k] = {"us_med": round(v[len(v) // 2], 2), "us_min": round(v[0], 2),
                      "tflops": round(fl / v[len(v) // 2] / 1e6, 1)}
        print(json.dumps(out), flush=True)
    lib.jmt_gemm_set_debug(0)


if __name__ == "__main__":
    main()
