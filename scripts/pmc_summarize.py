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


def family_traffic(out: str, dest: str):
    """Per bench.py family (scripts/family_from_trace.family): mean HBM bytes per hooked launch,
    a split-K GEMM's reduce kernel counted with the GEMM dispatched before it (bench.py's event
    pair brackets both).  Writes dest/traffic_<family>.json."""
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from family_from_trace import family
    per = {}
    for i, counter in ((1, "FETCH_SIZE"), (2, "WRITE_SIZE")):
        files = glob.glob(os.path.join(out, f"p{i}", "**", "*counter_collection.csv"),
                          recursive=True)
        recs = []
        for f in files:
            for r in csv.DictReader(open(f)):
                if r.get("Counter_Name") == counter:
                    recs.append((int(r.get("Dispatch_Id", 0)), r["Kernel_Name"],
                                 float(r["Counter_Value"])))
        recs.sort()
        fam_bytes = defaultdict(float)
        fam_launches = defaultdict(int)
        last = None
        for _, name, v in recs:
            f = family(name)
            b = (2.0 if counter == "FETCH_SIZE" else 1.0) * 1024 * v
            if f == "reduce":
                if last is not None:
                    fam_bytes[last] += b
                continue
            if f is None:
                continue
            fam_bytes[f] += b
            fam_launches[f] += 1
            last = f
        per[counter] = (fam_bytes, fam_launches)
    os.makedirs(dest, exist_ok=True)
    fb_r, fl_r = per["FETCH_SIZE"]
    fb_w, fl_w = per["WRITE_SIZE"]
    for f in sorted(set(fl_r) | set(fl_w)):
        rd = fb_r[f] / fl_r[f] if fl_r.get(f) else None
        wr = fb_w[f] / fl_w[f] if fl_w.get(f) else None
        rec = {"family": f, "dispatches": max(fl_r.get(f, 0), fl_w.get(f, 0)),
               "hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr,
               "hbm_bytes_per_launch": (rd or 0) + (wr or 0),
               "commit": os.environ.get("JMT_COMMIT"),
               "method": "rocprofv3 --kernel-trace --pmc FETCH_SIZE / WRITE_SIZE in separate "
                         "passes over `bench.py --steps 2 --warmup 1 --no-probe "
                         "--no-cpu-baseline` (scripts/pmc_bench.sh); FETCH_SIZE doubled (gfx950 "
                         "wide-read correction, MI355X_MICROARCH.md HBM section); split-K reduce "
                         "kernels counted with their GEMM launch"}
        json.dump(rec, open(os.path.join(dest, f"traffic_{f}.json"), "w"), indent=1)
        print(json.dumps(rec))


if len(sys.argv) > 2:
    family_traffic(sys.argv[1], sys.argv[2])
