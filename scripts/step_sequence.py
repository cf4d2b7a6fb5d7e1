"""Ordered kernel sequence of one eager training step from a rocprofv3 kernel-trace CSV.

usage: python scripts/step_sequence.py run_kernel_trace.csv [marker]
The step is the dispatches after the second-to-last `marker` kernel (default: the fused SGD
kernel, the last launch of a step) up to and including the last one.
"""
import csv
import sys


def main():
    path = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else "sgd_kernel"
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    if len(ends) < 2:
        sys.exit("fewer than two step markers")
    step = rows[ends[-2] + 1:ends[-1] + 1]
    t0 = int(step[0]["Start_Timestamp"])
    tot = 0.0
    for r in step:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        us = (e - s) / 1e3
        tot += us
        grid = f'{r["Grid_Size_X"]}x{r["Grid_Size_Y"]}x{r["Grid_Size_Z"]}/{r["Workgroup_Size_X"]}'
        print(f'{(s - t0) / 1e3:9.1f} {us:8.2f}  {grid:>22}  {r["Kernel_Name"][:110]}')
    span = (int(step[-1]["End_Timestamp"]) - t0) / 1e3
    print(f"# {len(step)} dispatches, kernel time {tot:.1f} us, span {span:.1f} us")


if __name__ == "__main__":
    main()
