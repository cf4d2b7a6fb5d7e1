"""Kernels of the timed region of a `rocprofv3 --kernel-trace` run of bench.py: the last
`--steps` training steps (each ends with the fused SGD launch), per-kernel-kind time per step,
concurrency (sum of kernel time / wall) and any torch (at::native) kernel inside.
    python scripts/step_trace.py <run_kernel_trace.csv> [steps] [--seq]
--seq also lists the last step's launches in order (start offset, duration, grid, kind)."""
import csv
import re
import sys
from collections import defaultdict


def kind(n):
    m = re.search(r"jmt::(\w+)", n) or re.search(r"_ZN3jmt\d+(\w+?)I", n)
    k = m.group(1) if m else n[:60]
    t = re.search(r"TileCfgILi(\d+)ELi(\d+)ELi\d+ELi\d+ELi(\d+)ELi(\d+)", n)
    if t:
        k += f" {t.group(1)}x{t.group(2)}/KB{t.group(3)}/S{t.group(4)}"
    lay = re.search(r"DF16\w?Lb(\d)ELb(\d)E", n)
    if lay:
        k += " " + {("1", "1"): "NT", ("1", "0"): "NN", ("0", "0"): "TN", ("0", "1"): "TT"}[lay.groups()]
    return k


def main(path, steps=10, seq=False):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    sgd = [i for i, r in enumerate(rows) if "sgd" in r["Kernel_Name"]]
    first = sgd[-steps - 1] + 1
    last = sgd[-1]
    reg = rows[first:last + 1]
    t0, t1 = int(reg[0]["Start_Timestamp"]), int(reg[-1]["End_Timestamp"])
    acc = defaultdict(lambda: [0.0, 0])
    for r in reg:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        acc[kind(r["Kernel_Name"])][0] += d / steps
        acc[kind(r["Kernel_Name"])][1] += 1
    tot = sum(v[0] for v in acc.values())
    print(f"wall {((t1 - t0) / 1e3 / steps):.1f} us/step, kernel sum {tot:.1f} us/step, "
          f"launches/step {len(reg) / steps:.1f}")
    for k, (us, n) in sorted(acc.items(), key=lambda kv: -kv[1][0]):
        print(f"{us:9.1f} us/step {n / steps:6.1f} launches  {k}")
    torch_k = [r["Kernel_Name"][:90] for r in reg if "at::native" in r["Kernel_Name"]]
    print("torch kernels in the timed region:", len(torch_k), sorted(set(torch_k))[:5])
    if seq:
        s0 = sgd[-2] + 1
        b = int(rows[s0]["Start_Timestamp"])
        print("last step, in launch order: start_us dur_us grid kind")
        for r in rows[s0:last + 1]:
            st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            print(f"{(st - b) / 1e3:9.1f} {(en - st) / 1e3:8.1f} {r.get('Grid_Size', '?'):>9} "
                  f"{kind(r['Kernel_Name'])}")


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if a != "--seq"]
    main(args[0], int(args[1]) if len(args) > 1 else 10, "--seq" in sys.argv)
