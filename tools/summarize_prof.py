"""Summarise a tools/gpu_prof.sh output directory into profiles/<tag>_*.

kernel_stats:    rocprofv3 --kernel-trace --stats summary (copied; its averages mix
                 launch sizes, e.g. the one-off IMHK initial-draw Klein launch).
kernel_launches: per kernel and grid size: launches and average duration from the
                 kernel trace -- the full-size rows are what bench.py times.
pmc:             per kernel and grid size: average FETCH_SIZE / WRITE_SIZE (KB, as
                 reported) and the corrected HBM bytes per launch (FETCH_SIZE x 2 on
                 gfx950 for wide coalesced reads, MI355X_MICROARCH.md §HBM).
"""
import csv
import os
import shutil
import sys

src, tag = sys.argv[1], sys.argv[2]
dst = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles")
shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, f"{tag}_kernel_stats.csv"))
trace = os.path.join(src, "trace", "run_kernel_trace.csv")
if os.path.exists(trace):
    launches = {}
    for r in csv.DictReader(open(trace)):
        if not r["Kernel_Name"].startswith(("void lgs::", "lgs::")):
            continue
        g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        k = (r["Kernel_Name"].split("(")[0].replace("void ", ""), g)
        launches.setdefault(k, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    with open(os.path.join(dst, f"{tag}_kernel_launches.csv"), "w") as f:
        f.write("kernel,grid_size,launches,avg_ms,min_ms,max_ms\n")
        for (k, g), v in sorted(launches.items()):
            f.write(f"\"{k}\",{g},{len(v)},{sum(v) / len(v):.4f},{min(v):.4f},{max(v):.4f}\n")
rows_out = []
agg = {}
for sub, ctr in (("pmc_fetch", "FETCH_SIZE"), ("pmc_write", "WRITE_SIZE")):
    p = os.path.join(src, sub, "run_counter_collection.csv")
    if not os.path.exists(p):
        continue
    for r in csv.DictReader(open(p)):
        if not r["Kernel_Name"].startswith(("void lgs::", "lgs::")):
            continue
        k = r["Kernel_Name"].split("(")[0].replace("void ", "") + "|" + r["Grid_Size"]
        agg.setdefault(k, {}).setdefault(ctr, []).append(float(r["Counter_Value"]))
        if "klein" in k:
            rows_out.append(r)
with open(os.path.join(dst, f"{tag}_pmc_summary.csv"), "w") as f:
    f.write("kernel,grid_size,launches,FETCH_SIZE_KB_avg,WRITE_SIZE_KB_avg,hbm_bytes_per_launch_corrected\n")
    for k, v in sorted(agg.items()):
        fe = sum(v.get("FETCH_SIZE", [0])) / max(len(v.get("FETCH_SIZE", [])), 1)
        wr = sum(v.get("WRITE_SIZE", [0])) / max(len(v.get("WRITE_SIZE", [])), 1)
        n = max(len(v.get("FETCH_SIZE", [])), len(v.get("WRITE_SIZE", [])))
        name, grid = k.rsplit("|", 1)
        f.write(f"\"{name}\",{grid},{n},{fe:.1f},{wr:.1f},{(2 * fe + wr) * 1024:.0f}\n")
if rows_out:
    with open(os.path.join(dst, f"{tag}_pmc_klein.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(rows_out[0].keys()))
        w.writeheader()
        w.writerows(rows_out)
print(open(os.path.join(dst, f"{tag}_pmc_summary.csv")).read())
if os.path.exists(os.path.join(dst, f"{tag}_kernel_launches.csv")):
    print(open(os.path.join(dst, f"{tag}_kernel_launches.csv")).read())
