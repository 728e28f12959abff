"""Timeline of the pipelined bench from a rocprofv3 kernel trace: for the last steps,
every kernel longer than 0.05 ms with its start / end relative to the Klein launch
of that step (ms), to see what runs beside the Klein launch and what runs behind it.
usage: python tools/trace_timeline.py <run_kernel_trace.csv> [steps]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
nlast = int(sys.argv[2]) if len(sys.argv) > 2 else 3
big = [i for i, r in enumerate(rows) if "klein_mfma" in r["Kernel_Name"] and int(r["Grid_Size_X"]) >= 1 << 20]
for a, b in list(zip(big, big[1:]))[-nlast:]:
    t0 = int(rows[a]["Start_Timestamp"])
    print("-- step %.3f ms" % ((int(rows[b]["Start_Timestamp"]) - t0) / 1e6))
    for r in rows[max(0, a - 8):b]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if e - s < 50_000 or e < t0:
            continue
        print("  %8.3f %8.3f %8.3f  %s" % ((s - t0) / 1e6, (e - t0) / 1e6, (e - s) / 1e6, r["Kernel_Name"][:60]))
