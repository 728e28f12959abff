"""Benchmark: Klein samples/sec at NTRU n=512 (d=1024), IMHK, one process per GPU.

Workload (BASELINE.json configs[2], the config the metric is quoted on):
NTRU n=512, q=12289 basis [[qI,0],[H,I]] (d = 1024, Philox-generated h),
sigma = 165.7, IMHK with 2^14 chains per GPU.  One bench step = one
``lgs_imhk`` call advancing every chain by --imhk-steps steps: 2^14 x 64 =
2^20 Klein proposals (back-substitution + SampleZ + importance weight), the
Metropolis scan, exact integer moments, and the lattice points v = B z of every
kept state (thin = 1), all resident in HBM.  value = Klein proposals per second
over all ranks (weak scaling: chains per GPU fixed).

Multi-GPU: launched by torch.distributed.run; rank r owns chains
[r * 2^14, (r+1) * 2^14) (global chain ids -> Philox counters), so the union of
all ranks' chains is bit-identical for any GPU count.  The only collective is
one RCCL all-reduce of the moment / acceptance accumulators per step.

Also reported: roofline of the dominant kernel (the Klein sampler, HIP-event
timed on its launch stream), IMHK acceptance next to the CPU reference's, and
the CPU baseline (the C oracle, OpenMP over the host cores, bounded sample).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "lattice-gaussian-mcmc_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP64_PEAK_TFLOPS = 78.6    # MI355X FP64 vector / matrix dense peak (spec)


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def b_alg(d):
    """Algorithmic bytes per Klein sample: fp64 upper triangle of R + int32 z."""
    return 8 * d * (d + 1) // 2 + 4 * d


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="C3_ntru512")
    ap.add_argument("--chains", type=int, default=1 << 14, help="IMHK chains per GPU")
    ap.add_argument("--imhk-steps", type=int, default=64, help="IMHK steps per bench step (one lgs_imhk call)")
    ap.add_argument("--no-v", action="store_true", help="skip lattice points (coefficients only)")
    ap.add_argument("--exact-order", action="store_true")
    ap.add_argument("--cpu-samples", type=int, default=16384, help="IMHK proposals for the CPU baseline")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--traffic-csv", default=os.environ.get(
                        "LGS_TRAFFIC_CSV", os.path.join(REPO, "profiles", "r01n_pmc_klein.csv")),
                    help="rocprofv3 --pmc counter_collection.csv with FETCH_SIZE/WRITE_SIZE")
    return ap.parse_args()


def pmc_traffic(path, kernel_substr="klein_"):
    """Per-launch HBM bytes of the Klein kernel from rocprofv3 --pmc CSVs.

    `path` is a counter_collection.csv holding FETCH_SIZE and/or WRITE_SIZE rows
    (tools/gpu_prof.sh collects them in separate passes and tools/summarize_prof.py
    merges the Klein-kernel rows).  Only the largest dispatches (the bench's main
    launches) are averaged.  FETCH_SIZE / WRITE_SIZE are in KB; on gfx950
    FETCH_SIZE reports half of a wide coalesced read (MI355X_MICROARCH.md §HBM),
    so it is doubled."""
    import csv
    if not path or not os.path.exists(path):
        return None
    rows = [r for r in csv.DictReader(open(path)) if kernel_substr in r.get("Kernel_Name", "")]
    if not rows:
        return None
    gmax = max(int(r["Grid_Size"]) for r in rows)
    vals = {}
    for r in rows:
        if int(r["Grid_Size"]) == gmax:
            vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    if "FETCH_SIZE" not in vals:
        return None
    fetch = 2.0 * 1024 * sum(vals["FETCH_SIZE"]) / len(vals["FETCH_SIZE"])
    write = 1024 * sum(vals["WRITE_SIZE"]) / len(vals["WRITE_SIZE"]) if "WRITE_SIZE" in vals else 0.0
    return fetch + write


def main():
    args = parse()
    import torch
    import torch.distributed as dist
    from lgs_amd import _capi
    from lgs_amd.lattices import CONFIGS, build_config

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("LGS_ONE_DEVICE") == "1":  # rehearsal: every rank on device 0 (gloo)
        local = 0
    if world > 1:
        torch.cuda.set_device(local)
        backend = os.environ.get("LGS_DIST_BACKEND", "nccl")  # nccl = RCCL on ROCm
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)

    lat, sigma = build_config(args.config)
    B = lat.basis
    d = B.shape[0]
    # host QR set-up of klein.py:56-79 (identical to the drop-in)
    Q, R = np.linalg.qr(B, mode="full")
    sgn = np.where(np.diag(R) < 0, -1.0, 1.0)
    R = np.ascontiguousarray(R * sgn[:, None])
    cp = np.zeros(d)

    ctx = _capi.Context(local)
    ctx.set_basis(R, cp, B, sigma)
    nc, T = args.chains, args.imhk_steps
    first_chain = rank * nc
    seed = 0x5EED_0001
    flags = _capi.LGS_DEVICE_PTRS | _capi.LGS_COORD_MAJOR
    if args.exact_order:
        flags |= _capi.LGS_EXACT_ORDER
    z_state = torch.zeros((d, nc), dtype=torch.int32, device=dev)
    lw = torch.zeros(nc, dtype=torch.float64, device=dev)
    init = torch.zeros(nc, dtype=torch.int32, device=dev)
    acc = torch.zeros(nc, dtype=torch.int64, device=dev)
    mom = torch.zeros(2 * d, dtype=torch.int64, device=dev)
    v_samples = None if args.no_v else torch.empty((nc, T, d), dtype=torch.float64, device=dev)
    torch.cuda.synchronize()

    step_counter = [1]

    def one_step():
        ctx.imhk(seed, first_chain, nc, step_counter[0], T, 1, z_state, lw, init, acc,
                 v_samples=v_samples, moments=mom, flags=flags)
        step_counter[0] += T

    def reduce_stats():
        stats = torch.cat([acc.sum().reshape(1), mom])  # per-rank accumulators
        if world > 1:
            dist.all_reduce(stats)  # the single RCCL collective over xGMI
        return stats

    for _ in range(args.warmup):
        one_step()
    reduce_stats()  # warm torch's lazily loaded kernels and the communicator
    acc.zero_()
    mom.zero_()
    ctx.resolved(reset=True)
    ctx.timing_enable(True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        one_step()
    stats = reduce_stats()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    proposals = args.steps * nc * T * world
    value = proposals / elapsed
    k_ms, k_n = ctx.timing_get(_capi.KERNEL_KLEIN)
    g_ms, g_n = ctx.timing_get(_capi.KERNEL_BZ)
    a_ms, a_n = ctx.timing_get(_capi.KERNEL_ACCEPT)
    m_ms, m_n = ctx.timing_get(_capi.KERNEL_MOMENTS)
    acceptance = float(stats[0].item()) / proposals
    redos = ctx.resolved()

    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return

    # ---- roofline of the dominant kernel (the Klein sampler), HIP-event timed on its
    # launch stream.  It is FP64-compute bound: algorithmic work = d^2 flops per
    # sample (the d^2/2 multiply-adds of klein.py:191-193), peak = FP64 dense
    # (vector = matrix = 78.6 TF spec on MI355X).  The north_star's HBM view
    # (B_alg bytes per sample) is reported beside it.
    units = nc * T
    k_avg_s = (k_ms / max(k_n, 1)) / 1e3
    tflops = units * float(d) * d / k_avg_s / 1e12
    traffic = pmc_traffic(args.traffic_csv, kernel_substr="klein_")
    roofline = {"bound": "mfma", "achieved": round(tflops, 3), "peak": FP64_PEAK_TFLOPS,
                "unit": "TFLOP/s", "frac": round(tflops / FP64_PEAK_TFLOPS, 4),
                "traffic": None if traffic is None else round(traffic),
                "traffic_unit": "bytes/launch (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE)",
                "kernel": "klein_exact_kernel" if args.exact_order else "klein_mfma_kernel",
                "kernel_ms_avg": round(k_avg_s * 1e3, 3), "units_per_launch": units,
                "flops_per_unit": d * d,
                "hbm_algorithmic": {"bytes_per_unit": b_alg(d),
                                    "achieved_GBs": round(units * b_alg(d) / k_avg_s / 1e9, 1),
                                    "frac_of_8TBs": round(units * b_alg(d) / k_avg_s / 1e9 / HBM_PEAK_GBS, 3)}}
    gemm = None
    if g_n:
        # B z over all proposals + the carried states: 2 d^2 flops per vector
        gemm = {"kernel": "bz_gemm_kernel" if os.environ.get("LGS_BZ_FP64") == "1" else "bz_i8_kernel", "ms_per_step": round(g_ms / args.steps, 3),
                "tflops": round(2.0 * d * d * (units + nc) * args.steps / (g_ms / 1e3) / 1e12, 2)}

    # ---- parity spot check of this run's first proposals against the oracle
    import lgs_oracle
    n_chk = 8
    zc = torch.empty((d, n_chk), dtype=torch.int32, device=dev)
    ctx.klein(seed, 0, n_chk, zc, None, None, flags)
    o = lgs_oracle.klein(R, cp, sigma, n_chk, seed=seed, first_sample=0)
    parity = int((zc.cpu().numpy().T == o["z"]).all(1).sum())

    # ---- CPU baseline: the C oracle (IMHK reference mode), OpenMP over host cores
    cpu = None
    if world == 1 and not args.no_cpu:
        threads = args.cpu_threads or min(16, os.cpu_count() or 1)
        n_ch = max(threads, 1)
        steps_cpu = max(1, args.cpu_samples // n_ch)
        t1 = time.perf_counter()
        zc_, lwc, accc = lgs_oracle.imhk_parallel(R, cp, B, sigma, n_ch, steps_cpu, seed=seed,
                                                  first_step=1, threads=threads)
        tc = time.perf_counter() - t1
        props = n_ch * (steps_cpu + 1)  # + the initial draw of every chain
        cpu = {"value": round(props / tc, 2), "unit": "Klein samples/s", "cores": threads,
               "kind": "port",
               "sample": f"{n_ch} IMHK chains x {steps_cpu} steps (+1 initial draw), same NTRU "
                         f"d={d} basis, reference-mode weights, {tc:.1f} s wall on {threads} threads",
               "acceptance": float(accc.sum() / (n_ch * steps_cpu)),
               "per_core": round(props / tc / threads, 2), "host_cpus": os.cpu_count(),
               "cpu_model": _cpu_model()}

    dinfo = ctx.device_info()
    out = {
        "metric": "Klein samples/sec at n=512 NTRU (IMHK proposals, d=1024)",
        "value": round(value, 1),
        "unit": "samples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (Philox-generated NTRU public key h, seed 1)",
        "config": {"workload": f"{args.config}: NTRU n=512 q=12289 d={d} sigma={sigma} IMHK",
                   "chains_per_gpu": nc, "imhk_steps_per_step": T, "thin": 1,
                   "lattice_points": not args.no_v, "kernel_order": "exact" if args.exact_order else "panel",
                   "parallelism": f"chains sharded over {world} GPU(s), 1 RCCL all-reduce per step"},
        "imhk_acceptance": round(acceptance, 6),
        "imhk_acceptance_cpu_reference": 1.0,
        "parity_check": f"{parity}/{n_chk} proposals bit-exact vs oracle",
        "certificate_redos": {"coordinates": redos, "per_proposal": redos / (args.steps * nc * T)},
        "roofline": roofline,
        "gemm": gemm,
        "kernel_ms": {"klein": round(k_ms / max(k_n, 1), 3), "bz": round(g_ms / max(g_n, 1), 3),
                      "accept": round(a_ms / max(a_n, 1), 3), "moments": round(m_ms / max(m_n, 1), 3)},
        "cpu_baseline": cpu,
        "device": dinfo["name"],
    }
    print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
