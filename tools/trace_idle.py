"""GPU idle per bench step from a rocprofv3 kernel trace: the span between
consecutive 2^20-proposal Klein launches minus the union of all kernels' busy time.
usage: python tools/trace_idle.py <run_kernel_trace.csv>"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
big = [i for i, r in enumerate(rows) if "klein_mfma" in r["Kernel_Name"] and int(r["Grid_Size_X"]) >= 1 << 20]
for a, b in zip(big, big[1:]):
    t0, t1 = int(rows[a]["Start_Timestamp"]), int(rows[b]["Start_Timestamp"])
    busy, last, gaps = 0, t0, []
    for r in rows[a:b]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if s > last:
            gaps.append((s - last, r["Kernel_Name"][:48]))
        s = max(s, last)
        if e > s:
            busy += e - s
            last = max(last, e)
    if t1 > last:
        gaps.append((t1 - last, "(next Klein launch)"))
    top = ", ".join("%.3f before %s" % (g / 1e6, n) for g, n in sorted(gaps, reverse=True)[:3])
    print("step %.3f ms  busy %.3f  idle %.3f  | largest gaps: %s" % ((t1 - t0) / 1e6, busy / 1e6, (t1 - t0 - busy) / 1e6, top))
