"""Summarise SQ counter passes (tools/gpu_sqpmc.sh): per-wave instruction mix of the Klein kernel."""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
kname = sys.argv[2] if len(sys.argv) > 2 else "klein"
for var in sorted(os.listdir(root)):
    d = os.path.join(root, var)
    if not os.path.isdir(d):
        continue
    tot = defaultdict(float)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        rows = [r for r in csv.DictReader(open(f)) if kname in r.get("Kernel_Name", "")]
        if not rows:
            continue
        # last dispatch of the Klein kernel (the timed rep)
        last = max(int(r["Dispatch_Id"]) for r in rows)
        for r in rows:
            if int(r["Dispatch_Id"]) == last:
                tot[r["Counter_Name"]] += float(r["Counter_Value"])
    waves = tot.get("SQ_WAVES", 0) or 1
    print(f"== {var}: waves {waves:.0f}")
    for k in sorted(tot):
        print(f"  {k:28s} {tot[k]:16.4g}   per wave {tot[k] / waves:12.1f}")
