"""Summarise a rocprofv3 kernel_stats.csv: per-kernel total / calls / average, per-step share."""
import csv
import sys

path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total kernel time {tot/1e6:.2f} ms  = {tot/1e6/steps:.3f} ms/step over {steps:g} steps")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
    n = r["Name"]
    n = n.replace("jmt::", "").replace("_ZN3jmt", "")[:95]
    print(f"{float(r['TotalDurationNs'])/1e6/steps:8.3f} ms/step {int(r['Calls'])/steps:6.1f}/step "
          f"{float(r['AverageNs'])/1e3:8.1f} us  {n}")
