"""Per-block timeline of one GEMM launch (debug flag 8: s_memrealtime stamps at entry, first K-tile
landed, main loop end, epilogue end; 100 MHz = 10 ns ticks):
    python scripts/gemm_timeline.py --only "fwd NT 512" --cfg 5"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "scripts"), os.path.join(REPO, "joint-multimodal-transformer-6th-abaw_amd")]

import torch  # noqa: E402

import bench_gemm_step as B  # noqa: E402
from jmt import _lib  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--only", default="fwd NT 512")
ap.add_argument("--cfg", type=int, nargs="*", default=[5])
ap.add_argument("--rows", type=int, default=B.R)
args = ap.parse_args()
B.SHAPES[:] = [s for s in B.make_shapes(args.rows) if args.only in s[0]]
lib = _lib.load()
for cfg in args.cfg:
    B.run(3, cfg, 8)      # last launch leaves its stamps
    n = 8192
    buf = (ctypes.c_uint64 * (4 * n))()
    got = lib.jmt_gemm_trace_read(buf, n)
    t = np.frombuffer(buf, dtype=np.uint64).reshape(n, 4).astype(np.int64)
    t = t[(t[:, 0] > 0) & (t[:, 3] >= t[:, 0])]
    last = t[:, 0].max()
    t = t[t[:, 0] > last - 100000]          # the final launch only (stamps are overwritten)
    t0 = t[:, 0].min()
    rel = (t - t0) * 0.01                   # us
    d = np.diff(t, axis=1) * 0.01
    tot = (t[:, 3] - t[:, 0]) * 0.01
    starts = np.sort(rel[:, 0])
    print(json.dumps({
        "cfg": cfg, "blocks": int(len(t)), "launch_span_us": round(float(rel[:, 3].max()), 2),
        "block_us_median": round(float(np.median(tot)), 2),
        "first_tile_us": round(float(np.median(d[:, 0])), 2),
        "loop_us": round(float(np.median(d[:, 1])), 2),
        "epilogue_us": round(float(np.median(d[:, 2])), 2),
        "start_quantiles_us": [round(float(np.quantile(starts, q)), 2) for q in (0, .25, .5, .57, .6, .75, 1)],
        "end_quantiles_us": [round(float(np.quantile(rel[:, 3], q)), 2) for q in (0, .25, .5, .75, 1)],
    }), flush=True)
