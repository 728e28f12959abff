"""Per-launch Klein-kernel counters of a rocprofv3 profile of bench.py -> JSON for
bench.py's roofline (tools/gpu_roofline.sh).

usage: roofline_counters.py <profile dir> <config> <units_per_launch> <d> <out.json> [bench_trace.log]
                            [co_resources.json]

The build id of the library the profiled bench loaded (its JSON line's
roofline.build_id, from the optional log) is stored with the counters: bench.py
uses a counters file only for that same build.

Every counter_collection.csv under the profile dir is read; rows of the Klein
kernel's largest dispatches (the bench's 2^20-proposal launches) are averaged per
counter.  Executed fp64 flops = 64 lanes x (2 FMA + MUL + ADD) fp64 VALU
instructions + 2048 flops per v_mfma_f64_16x16x4 (the near-field coupling: 16 per
32-row panel per wave; the far field runs on int8); int8 ops = 32768 per
v_mfma_i32_16x16x64_i8 (all other MFMA instructions).  HBM bytes = FETCH_SIZE x 2
+ WRITE_SIZE (KB; gfx950 correction, MI355X_MICROARCH.md).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

root, config, units, d, out = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), sys.argv[5]
build_id = None
if len(sys.argv) > 6 and os.path.exists(sys.argv[6]):
    lines = [x for x in open(sys.argv[6]) if x.startswith("{")]
    if lines:
        build_id = json.loads(lines[-1]).get("roofline", {}).get("build_id")
vals = defaultdict(list)
grid_max = 0
rows_all = []
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if "klein_mfma_kernel" in r.get("Kernel_Name", ""):
            rows_all.append(r)
            grid_max = max(grid_max, int(r["Grid_Size"]))
disp = defaultdict(lambda: defaultdict(float))
for r in rows_all:
    if int(r["Grid_Size"]) == grid_max:
        disp[(r["Counter_Name"], r["Dispatch_Id"], r.get("Agent_Id", ""))]["v"] += float(r["Counter_Value"])
for (name, _, _), v in disp.items():
    vals[name].append(v["v"])
avg = {k: sum(v) / len(v) for k, v in vals.items()}
waves = avg.get("SQ_WAVES")
n_panels = (d + 31) // 32
f64_mfma = (waves or 0) * 16 * max(n_panels - 1, 0)
res = {"config": config, "units_per_launch": units, "grid_size": grid_max, "build_id": build_id,
       "counters_per_launch": avg,
       "fp64_flops": 64 * (2 * avg.get("SQ_INSTS_VALU_FMA_F64", 0) + avg.get("SQ_INSTS_VALU_MUL_F64", 0)
                           + avg.get("SQ_INSTS_VALU_ADD_F64", 0)) + 2048 * f64_mfma,
       "i8_ops": 32768 * max(avg.get("SQ_INSTS_MFMA", 0) - f64_mfma, 0),
       "hbm_bytes": 1024 * (2 * avg.get("FETCH_SIZE", 0) + avg.get("WRITE_SIZE", 0)),
       "compulsory_bytes": units * d * 2 + 8 * d * (d + 1) // 2}
# the profiled run's own duration of those launches (kernel trace of the same
# command): bench.py divides the counters by THIS time, so every fraction is of one
# run; its HIP-event time of the timed run is reported beside it
durs = []
for f in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if "klein_mfma_kernel" not in r.get("Kernel_Name", ""):
            continue
        g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        if g == grid_max:
            durs.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
if durs:
    res["kernel_ms_rocprof"] = sum(durs) / len(durs)
    res["kernel_launches_rocprof"] = len(durs)
wc = avg.get("SQ_WAVE_CYCLES")
if wc:
    res["issue"] = {"valu_active_per_wave_cycle": round(avg.get("SQ_ACTIVE_INST_VALU", 0) / wc, 4),
                    "any_active_per_wave_cycle": round(avg.get("SQ_ACTIVE_INST_ANY", 0) / wc, 4),
                    "waiting_on_memory_or_barrier": round(avg.get("SQ_WAIT_ANY", 0) / wc, 4),
                    "waiting_on_issue": round(avg.get("SQ_WAIT_INST_ANY", 0) / wc, 4),
                    "valu_insts_per_wave": round(avg.get("SQ_INSTS_VALU", 0) / (waves or 1), 1)}
if len(sys.argv) > 7 and os.path.exists(sys.argv[7]):  # code-object resources of the profiled build
    co = json.load(open(sys.argv[7]))
    res["code_object"] = {k["name"]: {f: k.get(f) for f in ("vgpr_count", "agpr_count", "sgpr_count",
                                                               "vgpr_spill_count", "sgpr_spill_count",
                                                               "private_segment_fixed_size",
                                                               "group_segment_fixed_size", "waves_per_simd")}
                          for k in co["kernels"] if "klein_mfma_kernel" in k["name"] or "bz_i8" in k["name"]}
    res["code_object_build_id"] = co.get("build_id")
# the profiled command's library switches (tools/gpu_roofline.sh profiles isolated
# launches: LGS_NO_PIPE=1, see there)
res["profile_env"] = {k: os.environ[k] for k in ("LGS_NO_PIPE", "LGS_NO_LOOKAHEAD", "LGS_NO_BZ_MOMENTS")
                      if k in os.environ}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps({k: v for k, v in res.items() if k != "counters_per_launch"}))
