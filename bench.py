"""Benchmark: Klein samples/sec at NTRU n=512 (d=1024), IMHK, one process per GPU.

Workload (BASELINE.json configs[2], the config the metric is quoted on):
NTRU n=512, q=12289 basis [[qI,0],[H,I]] (d = 1024, Philox-generated h),
sigma = 165.7, IMHK with 2^14 chains per GPU.  One bench step = one
``lgs_imhk`` call advancing every chain by --imhk-steps steps: 2^14 x 256 =
2^22 Klein proposals in one block (back-substitution + SampleZ + importance weight), the
Metropolis scan, exact integer moments, and the lattice points v = B z of every
kept state (thin = 1), all resident in HBM; then the lag-L autocovariance sums
of two scalar functionals of the first 1024 chains' kept states (a coefficient and
||v||^2) are continued on the device inside the same library call
(lgs_imhk_ex: ||v||^2 in the B z epilogue for those chains, the coefficient from
the proposal store, the lag sums before the call's synchronisation), and the
exact sum z z^T of the chains' states after the step (lgs_gram;
the job's empirical covariance, base.py:154-160, comes back from the same single
all-reduce).  The coefficient is z_{d-1}, the first one Klein decides (for the
NTRU / q-ary bases z_0 is a q-coordinate with sigma_0 ~ 0.01, identically 0).
value = Klein proposals per second over all ranks (weak scaling: chains per GPU
fixed).

Multi-GPU: ``python bench.py --gpus N`` (no WORLD_SIZE in the environment)
starts ``torch.distributed.run`` with N ranks as a child process and exits with
its status; rank r owns chains [r * C, (r+1) * C) (global chain ids -> Philox
counters), so the union of all ranks' chains is bit-identical for any GPU
count.  The one exchange is a single RCCL all-reduce after the timed steps of
every accumulator (acceptance, exact moments, the lag sums), inside the timed
region.  The 8-GPU workload of BASELINE configs[3] is
``--gpus 8 --config C4_qary1024`` (2^15 chains per GPU, 2^18 in all).

Also reported: the dominant kernel's roofline (the Klein sampler: executed-work
and HBM counters and the launch's rocprof duration from the committed rocprofv3
profile of this command, profiles/r0*_klein_counters.json, used only when its
build_id is the loaded library's; the HIP-event time of the same kernel in this
run beside it), the
certificate's redo count, a parity check of the timed run's final chain states
against the oracle, and the CPU baselines (the C oracle over the host cores and
the NumPy restatement of the reference's loop, one process per core).
"""
import argparse
import glob
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "lattice-gaussian-mcmc_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP64_PEAK_TFLOPS = 78.6    # MI355X FP64 vector / matrix dense peak (spec)
I8_PEAK_TOPS = 5000.0      # MI355X int8 MFMA dense (2x BF16 per clock, MI355X_MICROARCH.md)
ACF_LAGS = 16              # lag-L autocovariance of z_{d-1} and ||v||^2
ACF_CHAINS = 1024          # chains per rank whose states feed the lag sums

WORKLOADS = {
    "C3_ntru512": dict(chains=1 << 14, text="NTRU n=512 q=12289 d=1024 sigma=165.7 IMHK"),
    "C4_qary1024": dict(chains=1 << 15, text="q-ary d=1024 k=512 q=3329 sigma=165.7 IMHK (8 GPUs: 2^18 chains)"),
    "C2_qary128": dict(chains=1 << 16, text="q-ary d=128 q=3329 sigma=165.7 IMHK"),
    "C5_ntru2048": dict(chains=1 << 12, text="NTRU n=2048 q=12289 d=4096 sigma=165.7 IMHK (fp64 throughout)"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="C3_ntru512", choices=sorted(WORKLOADS))
    ap.add_argument("--chains", type=int, default=0, help="IMHK chains per GPU (default per config)")
    # (round 5: 256 -- one 2^22-proposal block per call at the library's default cap --
    # 111 vs 105 M samples/s at 64, profiles/r05aa_*, r05ab_*)
    ap.add_argument("--imhk-steps", type=int, default=256, help="IMHK steps per bench step (one lgs_imhk call)")
    ap.add_argument("--no-v", action="store_true", help="skip lattice points (coefficients only)")
    ap.add_argument("--exact-order", action="store_true")
    ap.add_argument("--cpu-samples", type=int, default=0,
                    help="IMHK proposals for the C-port baseline (0: 512 per core, < 0: skip it)")
    ap.add_argument("--wl-steps", type=int, default=3,
                    help="timed bench steps of the Wang-Ling leg after the headline (0: skip)")
    ap.add_argument("--wl-check-chains", type=int, default=8,
                    help="chains of the Wang-Ling leg replayed by the C oracle")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--numpy-samples", type=int, default=24, help="Klein samples per process, NumPy baseline")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-dist", action="store_true", help="N = 1 without the one-rank RCCL group")
    ap.add_argument("--gram-every", type=int, default=1,
                    help="exact sum z z^T of the chains' states after every k-th bench step (0: off)")
    ap.add_argument("--counters", default=os.environ.get("LGS_COUNTERS_JSON", ""),
                    help="klein_counters.json of a rocprofv3 profile of this command (default: newest in profiles/)")
    return ap.parse_args()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(n):
    """--gpus N without a torch.distributed launcher: N ranks as a child process
    (never an exec: nothing here has touched the GPU yet); rank 0 prints the line."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return subprocess.call(cmd, env=env)


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_share():
    """CPUs this process may use: its affinity set, capped by OMP_NUM_THREADS (the
    GPU box exports its per-GPU CPU share there)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(n, 1)


def b_alg(d):
    """SURVEY §8d algorithmic bytes per Klein sample: fp64 upper triangle of R + int32 z
    (R counted once per sample -- it is shared by every chain, see roofline notes)."""
    return 8 * d * (d + 1) // 2 + 4 * d


def build_id(path):
    """sha256 (first 16 hex digits) of the HIP library file this process loaded."""
    import hashlib
    try:
        with open(path, "rb") as f:
            return hashlib.sha256(f.read()).hexdigest()[:16]
    except OSError:
        return None


def load_counters(path, config, bid):
    """Per-launch Klein-kernel counters of a rocprofv3 profile of this bench command
    (tools/gpu_roofline.sh -> profiles/<tag>_klein_counters.json), used only when
    the profile was taken of the same library build (its build_id); returns
    (counters or None, path or None, "current" | "stale" | None)."""
    if not path:
        cands = sorted(glob.glob(os.path.join(REPO, "profiles", "r0*_klein_counters.json")))
        cands = [c for c in cands if json.load(open(c)).get("config") == config]
        same = [c for c in cands if json.load(open(c)).get("build_id") == bid]
        path = (same or cands or [""])[-1]
    if not path or not os.path.exists(path):
        return None, None, None
    cnt = json.load(open(path))
    rel = os.path.relpath(path, REPO)
    if bid is None or cnt.get("build_id") != bid:
        return None, rel, "stale"
    return cnt, rel, "current"


def wang_ling_leg(args, ctx, D, _capi, lgs_oracle, R, cp, B, sigma, d, nc, T, seed, dev, binv_k):
    """The headline pipeline (StreamingShard over lgs_imhk_ex: Klein proposals, the
    certified Wang-Ling accept kernel, moments, B z, lag sums, Gram) with Wang-Ling
    weights (LGS_WANG_LING), 1 untimed + args.wl_steps timed steps; the first
    args.wl_check_chains chains replayed by the C oracle (same Philox counters):
    per-chain accept counts and final states must be equal."""
    import torch
    flags = _capi.LGS_WANG_LING | (_capi.LGS_EXACT_ORDER if args.exact_order else 0)
    adv = D.gpu_advance(ctx, seed, 0, nc, d, dev, flags=flags, block_steps=T, want_v=not args.no_v,
                        fn_chains=ACF_CHAINS)
    shard = D.StreamingShard(adv, nc, d, binv_row=binv_k, device=dev, lag_chains=ACF_CHAINS, lags=ACF_LAGS,
                             gram_every=args.gram_every)
    ctx.counter(_capi.LGS_COUNTER_ACCEPT_RESOLVED, reset=True)
    ctx.counter(_capi.LGS_COUNTER_WL_MISMATCH, reset=True)
    shard.step(T)  # warm-up block (initial draws + T steps)
    torch.cuda.synchronize()
    acc0 = shard.acc.clone()
    t0 = time.perf_counter()
    for _ in range(args.wl_steps):
        shard.step(T)
    shard.reduce()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    props = args.wl_steps * nc * T
    acc = shard.acc.cpu().numpy()
    acc_timed = int((shard.acc - acc0).sum().item())
    m = min(args.wl_check_chains, nc)
    steps_all = (1 + args.wl_steps) * T
    t1 = time.perf_counter()
    zo, lwo, acco = lgs_oracle.imhk_parallel(R, cp, B, sigma, m, steps_all, seed=seed, first_step=1,
                                             mode=lgs_oracle.IMHK_WANG_LING, threads=min(m, cpu_share()))
    tcpu = time.perf_counter() - t1
    zg = adv.state["z"][:, :m].cpu().numpy().T
    same_acc = int(sum(int(acc[c]) == int(acco[c]) for c in range(m)))
    same_z = int(sum(np.array_equal(zg[c], zo[c]) for c in range(m)))
    return {"value": round(props / el, 1), "unit": "samples/s", "ms_per_step": round(1e3 * el / args.wl_steps, 3),
            "steps": args.wl_steps, "imhk_steps_per_step": T, "chains": nc,
            "acceptance": round(acc_timed / props, 6),
            "acceptance_gpu_subset": round(float(acc[:m].sum()) / (m * steps_all), 6),
            "acceptance_cpu_subset": round(float(acco.sum()) / (m * steps_all), 6),
            "flags_equal_oracle": f"{same_acc}/{m} chains' accept counts and {same_z}/{m} final states equal "
                                  f"to the C oracle over {steps_all} Wang-Ling steps ({tcpu:.1f} s CPU)",
            "decisions_at_reference_order_weights": ctx.counter(_capi.LGS_COUNTER_ACCEPT_RESOLVED),
            "wl_mismatch": ctx.counter(_capi.LGS_COUNTER_WL_MISMATCH),
            "note": "imhk.py:141-177 with the Wang-Ling weight; the q-panel skip does not apply (every mean "
                    "enters the weight); not part of `value`"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    import torch
    import torch.distributed as dist
    from lgs_amd import _capi
    from lgs_amd import distributed as D
    from lgs_amd.lattices import build_config

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("LGS_ONE_DEVICE") == "1":  # rehearsal: every rank on device 0 (gloo)
        local = 0
    torch.cuda.set_device(local)
    backend = os.environ.get("LGS_DIST_BACKEND", "nccl")  # nccl = RCCL on ROCm
    collective = "none"
    if world > 1:
        D.init_process_group(backend, local, world)
        collective = backend
    elif not args.no_dist:
        # N = 1 runs the same collective as N > 1: a one-rank RCCL group (set up
        # outside the timed region); if the box cannot form it, say so and go on
        try:
            D.init_process_group(backend, local, 1)
            collective = backend
        except Exception as e:  # noqa: BLE001
            collective = f"none ({type(e).__name__}: {str(e)[:120]})"
    dev = torch.device("cuda", local)

    lat, sigma = build_config(args.config)
    B = lat.basis
    d = B.shape[0]
    # host QR set-up of klein.py:56-79 (identical to the drop-in)
    Q, R = np.linalg.qr(B, mode="complete")
    sgn = np.where(np.diag(R) < 0, -1.0, 1.0)
    R = np.ascontiguousarray(R * sgn[:, None])
    cp = np.zeros(d)
    binv_k = np.linalg.inv(B)[d - 1]  # z_{d-1} = row d-1 of B^-1 times v (rounded: v, z integral)

    # LGS_NO_PIPE=1 (read here, passed as lgs_create_ex's LGS_CTX_NO_PIPELINE): isolated
    # launches, for the rocprof roofline passes (tools/gpu_roofline.sh)
    pipelined = os.environ.get("LGS_NO_PIPE") != "1"
    # LGS_NO_CU_SPLIT=1 (lgs_create_ex's LGS_CTX_NO_CU_SPLIT): the Klein stream on every CU, A/B
    ctx = _capi.Context(local, pipeline=pipelined, cu_split=os.environ.get("LGS_NO_CU_SPLIT") != "1")
    ctx.set_basis(R, cp, B, sigma)
    nc = args.chains or WORKLOADS[args.config]["chains"]
    T = args.imhk_steps
    first_chain = rank * nc
    seed = 0x5EED_0001
    flags = _capi.LGS_EXACT_ORDER if args.exact_order else 0
    # the timed path is lgs_amd.distributed's StreamingShard: one lgs_imhk call per
    # bench step, lag sums on the device, one all-reduce (tests/test_distributed.py
    # drives the same class with the oracle over gloo, world 2); all of it on one
    # work stream, which the library then uses as its own (no cross-stream waits)
    torch.cuda.synchronize()
    if os.environ.get("LGS_BENCH_DEFAULT_STREAM") != "1":  # (=1: the A/B switch)
        torch.cuda.set_stream(torch.cuda.Stream(device=dev))
    advance = D.gpu_advance(ctx, seed, first_chain, nc, d, dev, flags=flags, block_steps=T, want_v=not args.no_v,
                            fn_chains=ACF_CHAINS)
    shard = D.StreamingShard(advance, nc, d, binv_row=binv_k, device=dev, lag_chains=ACF_CHAINS, lags=ACF_LAGS,
                             gram_every=args.gram_every)
    z_state = advance.state["z"]
    nacf = shard.lag_chains
    torch.cuda.synchronize()

    for _ in range(args.warmup):
        shard.step(T)
    shard.reduce()  # warm torch's lazily loaded kernels and the communicator
    shard.reset_stats()
    ctx.resolved(reset=True)
    ctx.timing_enable(True)
    torch.cuda.synchronize()
    if D.collective_active():
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        shard.step(T)
    stats = shard.reduce()
    torch.cuda.synchronize()
    if D.collective_active():
        dist.barrier()
    elapsed = time.perf_counter() - t0
    # device memory at the end of the timed region: the whole device's use (library
    # buffers are hipMalloc'd outside torch's allocator; with LGS_ONE_DEVICE=1 every
    # rank's buffers are on one device) and torch's own peak, max over ranks
    free_b, total_b = torch.cuda.mem_get_info(dev)
    mem_t = [(total_b - free_b) / 2**30, torch.cuda.max_memory_reserved(dev) / 2**30]
    if world > 1:
        t = torch.tensor([elapsed] + mem_t, dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t[0].item())
        mem_t = [float(t[1].item()), float(t[2].item())]
    memory = {"device_used_gib": round(mem_t[0], 1), "device_total_gib": round(total_b / 2**30, 1),
              "torch_peak_reserved_gib_per_rank": round(mem_t[1], 1),
              "ranks_on_device": world if os.environ.get("LGS_ONE_DEVICE") == "1" else 1}
    step_counter = [shard.next_step]

    proposals = args.steps * nc * T * world
    value = proposals / elapsed
    k_ms, k_n = ctx.timing_get(_capi.KERNEL_KLEIN)
    g_ms, g_n = ctx.timing_get(_capi.KERNEL_BZ)
    a_ms, a_n = ctx.timing_get(_capi.KERNEL_ACCEPT)
    m_ms, m_n = ctx.timing_get(_capi.KERNEL_MOMENTS)
    redos = ctx.resolved()
    s_acc = int(stats["accepts"][0].item())
    acceptance = s_acc / proposals
    acf = {"lags": ACF_LAGS, "chains": nacf * world,
           "z_last": D.StreamingShard.acf(stats["lag_z"]), "norm_v_sq": D.StreamingShard.acf(stats["lag_v"])}
    covariance = None
    if args.gram_every:
        # empirical covariance of the thinned kept states (base.py:154-160) from the
        # exact all-reduced sums; the checksum is of the int64 sum z z^T itself
        import hashlib
        G = stats["gram"][0].cpu().numpy()
        cov = D.StreamingShard.covariance(stats["gram"])
        covariance = {"states": int(stats["gram"][2][0].item()), "every_steps": args.gram_every * T,
                      "sum_zzT_sha256": hashlib.sha256(np.ascontiguousarray(G).tobytes()).hexdigest()[:16],
                      "trace": float(np.trace(cov)), "offdiag_abs_max": float(np.abs(cov - np.diag(np.diag(cov))).max()),
                      "diag_min": float(np.diag(cov).min()), "diag_max": float(np.diag(cov).max())}

    # ---- parity: the timed run's final chain states against the oracle.  In the
    # reference's IMHK mode every proposal is accepted (the weight is a constant up to
    # rounding, imhk.py:102-124), so chain c's state is its last proposal: the Klein
    # sample at counter (chain first_chain + c, step step_counter - 1).
    import lgs_oracle
    parity = None
    if rank == 0:
        zs = z_state.cpu().numpy()
        last = step_counter[0] - 1
        chk = [int(c) for c in np.linspace(0, nc - 1, 8)]
        if acceptance == 1.0:
            ok = 0
            for c in chk:
                o = lgs_oracle.klein(R, cp, sigma, 1, seed=seed, first_sample=(last << 32) | (first_chain + c))
                ok += int(np.array_equal(zs[:, c], o["z"][0]))
            parity = f"{ok}/{len(chk)} final chain states (after {step_counter[0] - 1} IMHK steps) bit-exact vs oracle"
        else:
            parity = "skipped: acceptance < 1 (final state is not the last proposal)"

    if rank != 0:
        if D.collective_active():
            dist.destroy_process_group()
        return

    # ---- roofline of the dominant kernel (the Klein sampler), HIP-event timed on
    # its launch stream.  The kernel is bound by neither pipe nor HBM: it issues the
    # near-field fp64 FMAs and SampleZ's fp64 polynomials on the VALU (the FP64
    # datapath it shares with fp64 MFMA), the far field on int8 MFMA, and waits on
    # latency.  Executed work comes from SQ counters of the committed profile of this
    # command (per launch), so every fraction is of work actually issued.
    units = nc * T
    k_avg_s = (k_ms / max(k_n, 1)) / 1e3
    bid = build_id(_capi.LIB_PATH)
    cnt, cnt_path, cnt_state = load_counters(args.counters, args.config, bid)
    roofline = {"bound": "mfma", "unit": "TFLOP/s", "peak": FP64_PEAK_TFLOPS, "achieved": None, "frac": None,
                "traffic": None, "kernel": "klein_exact_kernel" if args.exact_order else "klein_mfma_kernel",
                "kernel_ms_avg": round(k_avg_s * 1e3, 3), "units_per_launch": units, "build_id": bid,
                "counters": cnt_state if cnt_state != "current" else cnt_path}
    if cnt_state == "stale":
        roofline["counters_note"] = f"newest profile {cnt_path} is of another library build: not used"
    if cnt and cnt.get("units_per_launch") == units:
        f64 = cnt["fp64_flops"]
        # every fraction divides the profiled run's counters by THAT run's own kernel
        # duration (rocprofv3 kernel trace of the same command); this run's HIP-event
        # time is reported beside it (kernel_ms_avg)
        p_s = cnt.get("kernel_ms_rocprof", k_avg_s * 1e3) / 1e3
        roofline.update({
            "achieved": round(f64 / p_s / 1e12, 3), "frac": round(f64 / p_s / 1e12 / FP64_PEAK_TFLOPS, 4),
            "what": "executed fp64 flops (VALU FMA x2 + ADD/MUL + fp64 MFMA) per launch / the profiled launch's "
                    "rocprof duration; FP64 pipe peak",
            "kernel_ms_rocprof": round(p_s * 1e3, 3),
            "profile_env": cnt.get("profile_env", {}),
            "profile_note": "counters and rocprof duration of the same bench command with isolated launches "
                            "(LGS_NO_PIPE=1: under the profiler the pipelined launches overlap differently); "
                            "kernel_ms_avg is this run's HIP-event time of the pipelined launches",
            "traffic": int(cnt["hbm_bytes"]),
            "traffic_note": "FETCH_SIZE x2 + WRITE_SIZE per launch (gfx950 correction), profile of this command",
            "hbm": {"achieved_GBs": round(cnt["hbm_bytes"] / p_s / 1e9, 1),
                    "frac_of_8TBs": round(cnt["hbm_bytes"] / p_s / 1e9 / HBM_PEAK_GBS, 4),
                    "compulsory_bytes": int(cnt["compulsory_bytes"]),
                    "traffic_over_compulsory": round(cnt["hbm_bytes"] / cnt["compulsory_bytes"], 2)},
            "int8_mfma": {"achieved_TOPS": round(cnt["i8_ops"] / p_s / 1e12, 2),
                          "frac_of_5POPS": round(cnt["i8_ops"] / p_s / 1e12 / I8_PEAK_TOPS, 4)},
            "issue": cnt["issue"]})
        if "code_object" in cnt:
            roofline["code_object"] = {k: v for k, v in cnt["code_object"].items() if "klein" in k and "Lb0ELb1ELb0E" in k}
    roofline["hbm_algorithmic_note"] = (
        f"SURVEY 8d B_alg = {b_alg(d)} B/sample counts R once per sample, but R is shared by every "
        f"chain (read once per 256-sample block from L2), so B_alg x rate is not an HBM quantity")
    gemm = None
    if g_n:
        gemm = {"kernel": "bz_i8_kernel", "ms_per_step": round(g_ms / args.steps, 3)}
        if pipelined:
            gemm["note"] = ("HIP-event span on the work stream, beside the next block's Klein launch (pipelined "
                            "blocks): it stretches over that launch; LGS_NO_PIPE=1 times it alone")

    # ---- Wang-Ling leg (after the headline's timed region; not part of `value`):
    # the one IMHK mode whose acceptance is not identically 1 (imhk.py:102-124 gives a
    # constant weight), run through the same StreamingShard pipeline, its acceptance
    # checked against the C oracle on a chain subset (imhk.py:141-177)
    wang_ling = None
    if rank == 0 and world == 1 and args.wl_steps > 0:
        wang_ling = wang_ling_leg(args, ctx, D, _capi, lgs_oracle, R, cp, B, sigma, d, nc, T, seed, dev, binv_k)

    # ---- CPU baselines (bounded samples; rank 0 at N=1 only).  `value` is the
    # reference's own path: the NumPy restatement of klein.py:101-220 (the
    # reference's statements and indexing, one process per core), calibrated at
    # 1.05x the imported reference's per-core rate on the same C3 basis
    # (profiles/r03_cpu_baseline_calibration.log); the C port (lgs_oracle.c,
    # OpenMP) is reported beside it as c_port.
    cpu = None
    if world == 1 and not args.no_cpu:
        threads = args.cpu_threads or cpu_share()
        c_port = None
        if args.cpu_samples >= 0:
            n_ch = threads
            cpu_props = args.cpu_samples or 512 * threads
            steps_cpu = max(1, cpu_props // n_ch)
            t1 = time.perf_counter()
            zc_, lwc, accc = lgs_oracle.imhk_parallel(R, cp, B, sigma, n_ch, steps_cpu, seed=seed,
                                                      first_step=1, threads=threads)
            tc = time.perf_counter() - t1
            props = n_ch * (steps_cpu + 1)  # + the initial draw of every chain
            c_port = {"value": round(props / tc, 2), "unit": "Klein samples/s", "cores": threads, "kind": "port",
                      "sample": f"C oracle (lgs_oracle.c, OpenMP): {n_ch} IMHK chains x {steps_cpu} steps "
                                f"(+1 initial draw), same basis, reference-mode weights, {tc:.1f} s wall on "
                                f"{threads} threads",
                      "acceptance": float(accc.sum() / (n_ch * steps_cpu)),
                      "per_core": round(props / tc / threads, 2)}
        cpu = {"value": None, "unit": "Klein samples/s", "cores": threads, "kind": "reference-restatement",
               "host_cpus": os.cpu_count(), "cpu_model": _cpu_model(), "c_port": c_port,
               "acceptance": None if c_port is None else c_port["acceptance"]}
        if args.numpy_samples > 0:
            import lgs_numpy_restatement as NR
            rate, tot, wall = NR.timed_run(R, cp, B, sigma, processes=threads,
                                           samples_per_process=args.numpy_samples, seed=seed)
            cpu.update({
                "value": round(rate, 2), "per_core": round(rate / threads, 3),
                "sample": f"{tot} Klein samples of the reference's NumPy loop (klein.py:101-220, "
                          f"oracle/lgs_numpy_restatement.py), {threads} processes x {args.numpy_samples} "
                          f"samples, one BLAS thread each, {wall:.1f} s per process",
                "calibration": "restatement / imported reference = 1.051 per core on the same C3 basis and "
                               "samples (profiles/r03_cpu_baseline_calibration.log)"})

    dinfo = ctx.device_info()
    out = {
        "metric": "Klein samples/sec at n=512 NTRU (IMHK proposals, d=1024)" if args.config == "C3_ntru512"
        else f"Klein samples/sec, {args.config} (IMHK proposals, d={d})",
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
        "data": "synthetic (Philox-generated basis, seed 1)",
        "config": {"workload": f"{args.config}: {WORKLOADS[args.config]['text']}",
                   "chains_per_gpu": nc, "chains_total": nc * world, "imhk_steps_per_step": T, "thin": 1,
                   "lattice_points": not args.no_v, "kernel_order": "exact" if args.exact_order else "certified-blocked",
                   "parallelism": f"chains sharded over {world} GPU(s); one all-reduce of every accumulator "
                                  f"after the timed steps (inside the timed region)",
                   "collective": collective},
        "imhk_acceptance": round(acceptance, 6),
        "imhk_acceptance_cpu_reference": None if cpu is None else cpu["acceptance"],
        # (reference mode: the weight is a constant up to rounding, acceptance 1; the
        # Wang-Ling leg below carries the acceptance that can differ)
        "parity_check": parity,
        "certificate_redos": {"verified_subpanels": redos, "per_proposal": redos / (args.steps * nc * T)},
        "autocorrelation": acf,
        "covariance": covariance,
        "roofline": roofline,
        "gemm": gemm,
        "memory": memory,
        "kernel_ms": {"klein": round(k_ms / max(k_n, 1), 3), "bz": round(g_ms / max(g_n, 1), 3),
                      "accept": round(a_ms / max(a_n, 1), 3), "moments": round(m_ms / max(m_n, 1), 3),
                      "blocks_pipelined": pipelined,
                      "klein_stream_cus": ctx.counter(_capi.LGS_COUNTER_KLEIN_CUS) or dinfo.get("n_cu"),
                      "note": "pipelined blocks: each lgs_imhk block's Klein launch runs on the library's Klein "
                              "stream beside the previous block's accept / moments / B z on the work stream, so "
                              "these launch times overlap (their sum exceeds ms_per_step) and each is stretched by "
                              "sharing the CUs; the Klein stream's queue is masked to klein_stream_cus CUs "
                              "(1/8 of them left to B z); LGS_NO_PIPE=1 gives isolated launches"},
        "cpu_baseline": cpu,
        "wang_ling": wang_ling,
        "device": dinfo["name"],
    }
    print(json.dumps(out))
    if D.collective_active():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
