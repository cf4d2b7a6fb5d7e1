"""GPU busy time (union of kernel intervals) vs wall span over the last N steps of a rocprofv3
kernel trace: tells whether a step is GPU-bound or host-issue-bound.  Also per (kernel, grid)
average durations."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
key = sys.argv[2] if len(sys.argv) > 2 else "sgd_kernel"
nsteps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r) for r in rows)
marks = [i for i, (s, e, r) in enumerate(iv) if key in r["Kernel_Name"]]
a, b = marks[-nsteps - 1], marks[-1]
seg = iv[a + 1:b + 1]
t0, t1 = iv[a][1], seg[-1][1]
busy, cur_s, cur_e = 0, None, None
for s, e, _ in seg:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
print(f"{nsteps} steps: wall {(t1-t0)/1e6/nsteps:.3f} ms/step, GPU busy {busy/1e6/nsteps:.3f} ms/step, "
      f"kernels/step {len(seg)/nsteps:.0f}, sum of durations {sum(e-s for s,e,_ in seg)/1e6/nsteps:.3f}")
g = defaultdict(list)
for s, e, r in seg:
    n = r["Kernel_Name"].replace("jmt::", "").replace("_ZN3jmt", "")[:60]
    g[(n, r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"], r["Workgroup_Size_X"])].append(e - s)
tops = sorted(g.items(), key=lambda kv: -sum(kv[1]))[:int(sys.argv[4]) if len(sys.argv) > 4 else 40]
for k, v in tops:
    print(f"{sum(v)/1e3/nsteps:8.1f} us/step {len(v)/nsteps:5.1f}x {sum(v)/len(v)/1e3:7.1f} us  grid={k[1]}x{k[2]}x{k[3]} wg={k[4]} {k[0]}")
