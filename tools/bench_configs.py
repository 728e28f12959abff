"""Per-config throughput of the GPU path (BASELINE.json configs):
Klein samples/s (coefficients + lattice points B z, device-resident) for
C1 Z^64, C2 q-ary 128, C3 NTRU n=512 (d=1024), C4 q-ary 1024, C5 NTRU n=2048
(d=4096), plus the component kernels built after the hot path (exact sum z z^T
on int8 MFMA, series statistics, Babai nearest plane) at the C3 shape.

Wall time of whole lgs_klein calls (torch-synchronised), and device time of the
Klein kernel from HIP events on its stream.  One JSON line per measurement.

usage: python tools/bench_configs.py [--configs C1_Z64,C2_qary128,...] [--reps 3]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lattice-gaussian-mcmc_amd"))

N_DEFAULT = {"C1_Z64": 1 << 20, "C2_qary128": 1 << 20, "C3_ntru512": 1 << 18,
             "C4_qary1024": 1 << 18, "C5_ntru2048": 1 << 17}
F64_PEAK, I8_PEAK = 78.6, 5000.0   # TFLOP/s, TOPS dense (MI355X_MICROARCH.md)


def prep(name):
    import numpy as np
    from lgs_amd.lattices import build_config
    lat, sigma = build_config(name)
    B = lat.basis
    Q, R = np.linalg.qr(B)
    sg = np.where(np.diag(R) < 0, -1.0, 1.0)
    return B, np.ascontiguousarray(R * sg[:, None]), np.ascontiguousarray(Q * sg[None, :]), sigma


def bench_klein(name, reps):
    import numpy as np
    import torch
    from lgs_amd import _capi
    B, R, Q, sigma = prep(name)
    d = B.shape[0]
    t0 = time.perf_counter()
    ctx = _capi.Context(0)
    ctx.set_basis(R, np.zeros(d), B, sigma)
    setup = time.perf_counter() - t0
    n = N_DEFAULT[name]
    z = torch.empty((d, n), dtype=torch.int32, device="cuda")
    v = torch.empty((n, d), dtype=torch.float64, device="cuda")
    f = _capi.LGS_DEVICE_PTRS | _capi.LGS_COORD_MAJOR
    ctx.klein(1, 0, n, z, v, None, f)                       # warm-up
    torch.cuda.synchronize()
    ctx.timing_enable(True)
    t0 = time.perf_counter()
    for r in range(reps):
        ctx.klein(1, (r + 1) * n, n, z, v, None, f)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / reps
    k_ms, k_n = ctx.timing_get(_capi.KERNEL_KLEIN)
    b_ms, b_n = ctx.timing_get(_capi.KERNEL_BZ)
    per_call_k = k_ms / reps
    # the reference-order kernel (LGS_EXACT_ORDER: sequential unfused mu, one
    # coordinate at a time) on a smaller sample, beside the default certified one
    ne = min(n, 65536 if d <= 1024 else 8192)
    ze = torch.empty((d, ne), dtype=torch.int32, device="cuda")
    ctx.klein(1, 0, ne, ze, None, None, f | _capi.LGS_EXACT_ORDER)  # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ctx.klein(1, ne, ne, ze, None, None, f | _capi.LGS_EXACT_ORDER)
    torch.cuda.synchronize()
    exact_s = time.perf_counter() - t0
    return {"bench": "klein", "config": name, "d": d, "samples_per_call": n,
            "samples_per_s": round(n / wall, 1), "ms_per_call": round(wall * 1e3, 3),
            "klein_kernel_ms_per_call": round(per_call_k, 3), "bz_ms_per_call": round(b_ms / reps, 3),
            # algorithmic back-substitution multiply-adds (d(d-1)/2 per sample) per
            # second: a rate, not a hardware bound (the far field runs on int8 MFMA
            # and skips all-zero chunks; bench.py's roofline reports executed work
            # per unit from PMC counters)
            "klein_backsub_gmacs_per_s": round(n * d * (d - 1) / 2 / (per_call_k / 1e3) / 1e9, 1),
            "exact_order_samples_per_s": round(ne / exact_s, 1), "exact_order_samples": ne,
            "basis_setup_s": round(setup, 2)}


def bench_components(reps):
    import numpy as np
    import torch
    from lgs_amd import _capi
    from lgs_amd.diagnostics import _gpu
    name = "C3_ntru512"
    B, R, Q, sigma = prep(name)
    d = B.shape[0]
    ctx = _capi.Context(0)
    ctx.set_basis(R, np.zeros(d), B, sigma)
    n = 1 << 18
    z = torch.empty((n, d), dtype=torch.int32, device="cuda")
    ctx.klein(3, 0, n, z, None, None, _capi.LGS_DEVICE_PTRS)
    out = []
    # exact sum z z^T (int8 MFMA, 2 digits -> 4 int8 products per MAC)
    s = torch.zeros(d, dtype=torch.int64, device="cuda")
    G = torch.zeros((d, d), dtype=torch.int64, device="cuda")
    ctx.gram(z, sum_out=s, gram_out=G, flags=_capi.LGS_DEVICE_PTRS)
    ctx.timing_enable(True)
    for _ in range(reps):
        ctx.gram(z, sum_out=s, gram_out=G, flags=_capi.LGS_DEVICE_PTRS)
    ms, k = ctx.timing_get(_capi.KERNEL_GRAM)
    ms /= reps                                  # per call: digit packing + MFMA Gram + mirror
    macs = float(n) * d * (d + 1) / 2          # upper tile pairs (diagonal tiles computed in full)
    out.append({"bench": "gram_i8", "config": name, "d": d, "n": n, "kernel_ms": round(ms, 3),
                "int8_tops_algorithmic": round(4 * 2 * macs / (ms / 1e3) / 1e12, 1),
                "frac_int8_peak": round(4 * 2 * macs / (ms / 1e3) / 1e12 / I8_PEAK, 4),
                "note": "per call: digit-plane packing (reads the n x d int32 samples once) + MFMA Gram"})
    # series statistics: tau_int of every coordinate of an IMHK-like trace (n steps x d)
    T = 4096
    x = z[:T].contiguous()
    tau = torch.empty(d, dtype=torch.float64, device="cuda")
    acf = torch.empty((d, 101), dtype=torch.float64, device="cuda")
    for want_acf in (False, True):
        ctx.timing_enable(True)
        for _ in range(reps):
            ctx.series_stats(x, d, T, d, 0, 1, d, max_lag=100, tau=tau, acf=acf if want_acf else None,
                             flags=_capi.LGS_DEVICE_PTRS)
        ms, k = ctx.timing_get(_capi.KERNEL_SERIES)
        ms /= reps
        out.append({"bench": "series_stats", "mode": "acf_101_lags" if want_acf else "tau_early_exit",
                    "series": d, "n": T, "kernel_ms": round(ms, 4),
                    "gbytes_per_s_input": round(d * T * 4 / (ms / 1e3) / 1e9, 1)})
    # Babai nearest plane (fp64 frame GEMM + panel walk + B z)
    ctx.set_decoder(Q, None)
    m = 1 << 16
    t = torch.randn((m, d), dtype=torch.float64, device="cuda") * 4000.0
    zo = torch.empty((m, d), dtype=torch.int32, device="cuda")
    vo = torch.empty((m, d), dtype=torch.float64, device="cuda")
    ctx.decode(t, "plane", zo, vo, _capi.LGS_DEVICE_PTRS)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        ctx.decode(t, "plane", zo, vo, _capi.LGS_DEVICE_PTRS)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / reps
    out.append({"bench": "nearest_plane", "config": name, "d": d, "targets": m,
                "targets_per_s": round(m / wall, 1), "ms_per_call": round(wall * 1e3, 3)})
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="C1_Z64,C2_qary128,C3_ntru512,C4_qary1024,C5_ntru2048")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--no-components", action="store_true")
    a = ap.parse_args()
    for name in a.configs.split(","):
        print(json.dumps(bench_klein(name, a.reps)), flush=True)
    if not a.no_components:
        for r in bench_components(a.reps):
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
