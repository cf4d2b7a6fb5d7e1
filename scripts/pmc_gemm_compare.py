"""Per-kernel PMC summary of a scripts/gemm_vs_vendor.py run under the rocprofv3 passes of
scratch-style pmc scripts: gemm.hip kernels vs hipBLASLt (Cijk_*) kernels, counter means per
dispatch and the wait / active fractions of SQ_WAVE_CYCLES."""
import csv, glob, os, sys, collections, re
out = sys.argv[1]
data = collections.defaultdict(lambda: collections.defaultdict(list))
meta = {}
dur = collections.defaultdict(list)
for f in glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if "gemm_kernel" in n:
            m = re.search(r"Lb(\d)ELb(\d)ENS_7TileCfgILi(\d+)ELi(\d+)ELi\d+ELi\d+ELi(\d+)", n)
            short = f"ours AK{m.group(1)} BK{m.group(2)} {m.group(3)}x{m.group(4)} KB{m.group(5)}"
        elif "Cijk" in n:
            short = "vendor " + re.search(r"MT\w+?_", n).group(0) + n[5:16]
        else: continue
        key = (short, r["Grid_Size"])
        data[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
        meta[key] = (r["Workgroup_Size"], r["LDS_Block_Size"], r["VGPR_Count"], r["Accum_VGPR_Count"], r["SGPR_Count"])
        if r["Counter_Name"] in ("SQ_WAVE_CYCLES",):
            dur[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for key, d in sorted(data.items()):
    print(key, "wg,lds,vgpr,agpr,sgpr=", meta[key], "dur_us(profiled)=%.1f" % (sum(dur[key])/max(1,len(dur[key]))))
    g = {c: sum(v)/len(v) for c, v in d.items()}
    for c, v in sorted(g.items()):
        print(f"   {c:24s} {v:14.4g}")
    if "SQ_WAVE_CYCLES" in g:
        w = g["SQ_WAVE_CYCLES"]
        print("   -> wait_any %.2f wait_inst %.2f active %.2f | lds_bank_conf/idx %.3f | MB rd %.1f wr %.1f" % (
            g.get("SQ_WAIT_ANY",0)/w, g.get("SQ_WAIT_INST_ANY",0)/w, g.get("SQ_ACTIVE_INST_ANY",0)/w,
            g.get("SQ_LDS_BANK_CONFLICT",0)/max(1,g.get("SQ_LDS_IDX_ACTIVE",1)), 2*1024*g.get("FETCH_SIZE",0)/1e6, 1024*g.get("WRITE_SIZE",0)/1e6))
