"""Per-family kernel time from a rocprofv3 --kernel-trace database, in bench.py's families
(GEMM by operand majorness NT / NN / TN / TT, attention fwd / bwd, small attention fwd / bwd),
next to the in-step figures bench.py printed in the same command:

    python scripts/family_from_trace.py gpurun_out/prof/run_results.db gpurun_out/bench.log \
        [--steps 200]

A GEMM launch with split-K is two kernels (the tile kernel and splitk_reduce_kernel); bench.py's
event pair brackets both, so the reduce kernels are attributed to the family of the GEMM
dispatched right before them.  Trace time per step = family kernel time in the timed region
(the last `--steps` graph replays: the kernels between the first and last dispatch of the timed
steps are selected by count) ÷ steps."""
import argparse
import json
import re
import sqlite3
from collections import defaultdict

MANGLED = re.compile(r"gemm_(?:persist3?_|pp_split_|pp2?_)?kernel.*?Lb([01])ELb([01])E")
DEMANGLED = re.compile(r"gemm_(?:persist3?_|pp_split_|pp2?_)?kernel<.*?(true|false), (true|false),")


# ROCm 7.2's demangler prints gemm_persist_kernel<__bf16, AK, BK, ...> as
# "gemm_persist_kernel<bool _Accum, bool, E, BK, ..." — the A majorness is lost.  Every
# persistent launch has a K-major A in practice (the weight gradients, A MN-major, are split-K,
# which the persistent kernel does not take: gemm_persist.hip persist_choice), so BK decides.
BROKEN_PERSIST = re.compile(r"gemm_(?:persist3?|pp2?)_kernel<bool _Accum, bool, E, (true|false),")
# the split-K ping-pong kernel (cfg 44) takes the weight gradients (A MN-major): B decides too
BROKEN_SPLIT = re.compile(r"gemm_pp_split_kernel<bool _Accum, bool, E, (true|false),")


def family(name: str):
    if "gemm_kernel" in name or "gemm_persist" in name or "gemm_pp" in name:
        bs = BROKEN_SPLIT.search(name)
        if bs:
            return "gemm_TT" if bs.group(1) == "true" else "gemm_TN"
        bp = BROKEN_PERSIST.search(name)
        if bp:
            return "gemm_NT" if bp.group(1) == "true" else "gemm_NN"
        m = MANGLED.search(name)
        if m:
            ak, bk = m.group(1) == "1", m.group(2) == "1"
        else:
            m = DEMANGLED.search(name)
            if not m:
                return "gemm_?"
            ak, bk = m.group(1) == "true", m.group(2) == "true"
        return {(True, True): "gemm_NT", (True, False): "gemm_NN", (False, False): "gemm_TN",
                (False, True): "gemm_TT"}[(ak, bk)]
    if "splitk_reduce" in name:
        return "reduce"
    if "small_attn_fwd" in name:
        return "small_attn_fwd"
    if "small_attn_bwd" in name:
        return "small_attn_bwd"
    if "attn_short_fwd" in name:
        return "attn_short_fwd"
    if "attn_short_bwd" in name:
        return "attn_short_bwd"
    if "attn_fwd_kernel" in name:
        return "attn_fwd"
    if "attn_bwd_kernel" in name or "attn_bwd_pds_kernel" in name:
        return "attn_bwd"
    if "attn_dkdv_kernel" in name:
        return "attn_dkdv"
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("bench_log")
    ap.add_argument("--json", default=None,
                    help="also write the timed-region figures per family (bench.py reads them "
                         "as the in-step view of its roofline)")
    args = ap.parse_args()
    line = [l for l in open(args.bench_log) if l.startswith("{")][-1]
    bench = json.loads(line)
    steps = bench["steps"]
    fams = {f["family"]: f for f in bench["roofline"]["families"]}
    c = sqlite3.connect(args.db)
    rows = c.execute("select name, start, end, duration from kernels order by start").fetchall()
    # the timed region: bench.py's probe steps come after it and launch jmt_noop / the torch
    # sleep kernel around every hooked launch; the graph replays before them carry none
    first_probe = next((i for i, r in enumerate(rows) if "noop_kernel" in r[0]), len(rows))
    per_step_n = None
    timed = rows[:first_probe]
    # dispatches per step = those of one replay: count launches of the CCC finish kernel
    finish = [i for i, r in enumerate(timed) if "ccc_finish_kernel" in r[0]]
    per_loss = 2
    if len(finish) >= per_loss * (steps + 1):
        lo = finish[-per_loss * steps - 1] + 1
        timed = timed[lo:]
        per_step_n = len(timed) / steps
    agg = defaultdict(float)
    last = None
    for name, s, e, d in timed:
        f = family(name)
        if f == "reduce":
            f = last
        if f is not None:
            agg[f] += d
            if not f.startswith("reduce"):
                last = f
    # the probe steps themselves (eager launches between the first and the last empty launch):
    # the same kernels bench.py's event pairs bracketed
    last_probe = max((i for i, r in enumerate(rows) if "noop_kernel" in r[0]), default=-1)
    pagg, pn = defaultdict(float), defaultdict(int)
    last = None
    for name, s, e, d in rows[first_probe:last_probe + 1]:
        f = family(name)
        if f == "reduce":
            if last is not None:
                pagg[last] += d
            continue
        if f is not None:
            pagg[f] += d
            pn[f] += 1
            last = f
    print(f"bench: {bench['metric']}  {bench['value']} {bench['unit']}, {bench['ms_per_step']} "
          f"ms/step; trace: {len(timed)} dispatches in the timed region "
          f"({per_step_n} per step)" if per_step_n else "(timed region not isolated)")
    print(f"{'family':16s} {'timed region':>13s} {'probe':>9s} {'ratio':>6s} | "
          f"{'probe-step trace':>17s} {'probe events':>13s} {'ratio':>6s}")
    print(f"{'':16s} {'ms/step':>13s} {'ms/step':>9s} {'':>6s} | {'us/launch':>17s} "
          f"{'us/launch':>13s}")
    # launches of each family in the timed region (split-K reduces ride with their GEMM)
    tn = defaultdict(int)
    for name, s, e, d in timed:
        f = family(name)
        if f is not None and f != "reduce":
            tn[f] += 1
    if args.json:
        import os
        rec = {"commit": os.environ.get("JMT_COMMIT"), "steps": steps,
               "ms_per_step": bench["ms_per_step"],
               "method": "rocprofv3 --kernel-trace over the default bench command; kernels of "
                         "the last `steps` graph replays (the timed region; the weight-gradient side "
                         "stream as bench.py's default: off since round 4), "
                         "split-K reduce kernels added to their GEMM (scripts/family_from_trace.py)",
               "families": {}}
        for f in agg:
            n = tn[f] / steps
            ms = agg[f] / 1e6 / steps
            rec["families"][f] = {"ms_per_step": round(ms, 4), "launches_per_step": n,
                                  "avg_launch_us": round(ms / n * 1e3, 2) if n else None}
        json.dump(rec, open(args.json, "w"), indent=1)
    for f in sorted(set(agg) | set(fams), key=lambda k: -agg.get(k, 0.0)):
        t = agg.get(f, 0.0) / 1e6 / steps
        pb = fams.get(f, {}).get("ms_per_step")
        ratio = f"{pb / t:6.3f}" if pb and t else "     -"
        tu = pagg[f] / pn[f] / 1e3 if pn.get(f) else None
        eu = fams.get(f, {}).get("avg_launch_us")
        r2 = f"{eu / tu:6.3f}" if tu and eu else "     -"
        print(f"{f:16s} {t:13.4f} {pb if pb is not None else '-':>9} {ratio} | "
              f"{(f'{tu:.2f}' if tu else '-'):>17s} {eu if eu is not None else '-':>13} {r2}")


if __name__ == "__main__":
    main()
