"""Per-kernel HBM traffic from the PMC passes of scripts/pmc_bench.sh (rocprofv3 counter CSVs).
FETCH_SIZE (KB, from TCC_EA0_RDREQ x 64 B) reports half the bytes of wide streaming reads on
gfx950 (MI355X_MICROARCH.md, HBM section): doubled here; WRITE_SIZE (KB) is taken as is.
Prints one JSON line per kernel name (+ grid): dispatches, mean read / write bytes per launch."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

out = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for i, counter in ((1, "FETCH_SIZE"), (2, "WRITE_SIZE")):
    files = glob.glob(os.path.join(out, f"p{i}", "**", "*counter_collection.csv"), recursive=True)
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            key = (r["Kernel_Name"], r.get("Grid_Size", r.get("Grid_Size_X", "")))
            acc[key][counter].append(float(r["Counter_Value"]))
rows = []
for (name, grid), d in acc.items():
    fs = d.get("FETCH_SIZE", [])
    ws = d.get("WRITE_SIZE", [])
    rd = 2.0 * 1024 * sum(fs) / len(fs) if fs else None
    wr = 1024 * sum(ws) / len(ws) if ws else None
    rows.append({"kernel": name[:120], "grid": grid, "dispatches": max(len(fs), len(ws)),
                 "hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr,
                 "total_bytes_per_launch": (rd or 0) + (wr or 0)})
rows.sort(key=lambda r: -(r["total_bytes_per_launch"] * r["dispatches"]))
for r in rows:
    print(json.dumps(r))
