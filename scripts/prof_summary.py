"""Summarise a rocprofv3 --kernel-trace database (rocpd sqlite, `-d DIR -o run`):
per-kernel count / total / average duration, and the busy fraction of the GPU over the
dispatch window (sum of kernel durations vs. first-start-to-last-end) of the last `--tail`
dispatches (the timed steps).
    python scripts/prof_summary.py gpurun_out/prof_real/run_results.db [--tail 3000] [--top 30]"""
import argparse
import re
import sqlite3
from collections import defaultdict


def short(name: str) -> str:
    name = re.sub(r"\(.*", "", name)
    name = re.sub(r"^void ", "", name)
    return name[:90]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--tail", type=int, default=0, help="only the last N dispatches")
    ap.add_argument("--top", type=int, default=40)
    args = ap.parse_args()
    c = sqlite3.connect(args.db)
    rows = c.execute("select name, start, end, duration, grid_x, workgroup_x from kernels "
                     "order by start").fetchall()
    if args.tail:
        rows = rows[-args.tail:]
    agg = defaultdict(lambda: [0, 0])
    for name, s, e, d, gx, wx in rows:
        a = agg[short(name)]
        a[0] += 1
        a[1] += d
    tot = sum(a[1] for a in agg.values())
    span = rows[-1][2] - rows[0][1]
    print(f"dispatches {len(rows)}  kernel time {tot / 1e6:.3f} ms  span {span / 1e6:.3f} ms  "
          f"busy {tot / span:.3f}")
    print(f"{'kernel':90s} {'count':>7s} {'total_ms':>9s} {'avg_us':>8s} {'share':>6s}")
    for k, (n, d) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:args.top]:
        print(f"{k:90s} {n:7d} {d / 1e6:9.3f} {d / n / 1e3:8.2f} {d / tot:6.3f}")


if __name__ == "__main__":
    main()
