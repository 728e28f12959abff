"""Klein-kernel micro-benchmark: device time of lgs_klein at a BASELINE config.

usage: python tools/kbench.py [--config C3_ntru512] [--n 262144] [--reps 3] [--exact]
Prints one JSON line per library in $LGS_LIBS (colon-separated .so paths) or the
default library."""
import argparse
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lattice-gaussian-mcmc_amd"))


def run_one(args):
    import numpy as np
    import torch
    from lgs_amd import _capi
    from lgs_amd.lattices import build_config
    lat, sigma = build_config(args.config)
    B = lat.basis
    d = B.shape[0]
    Q, R = np.linalg.qr(B)
    sg = np.where(np.diag(R) < 0, -1.0, 1.0)
    R = np.ascontiguousarray(R * sg[:, None])
    cp = np.zeros(d)
    if args.center:  # c' = Q^T c of a uniform random center of that scale (seed 5)
        c = np.random.default_rng(5).uniform(-args.center, args.center, d)
        cp = np.ascontiguousarray((Q * sg[None, :]).T @ c)
    ctx = _capi.Context(0)
    ctx.set_basis(R, cp, B, sigma)
    n = args.n
    z = torch.empty((d, n), dtype=torch.int32, device="cuda:0")
    lw = torch.empty(n, dtype=torch.float64, device="cuda:0")
    flags = _capi.LGS_DEVICE_PTRS | _capi.LGS_COORD_MAJOR | (_capi.LGS_EXACT_ORDER if args.exact else 0)
    flags |= _capi.LGS_WANG_LING if args.wl else 0
    v = torch.empty((n, d), dtype=torch.float64, device="cuda:0") if args.bz else None
    ctx.klein(1, 0, n, z, v, lw, flags)
    import ctypes
    diag = getattr(_capi.load_library(), "lgs_diag_cycles_read", None)
    dbuf = (ctypes.c_ulonglong * 16)()
    if diag is not None:
        diag(dbuf)  # reset after the warm-up launch
    if getattr(_capi.load_library(), "lgs_diag_far_read", None) is not None:
        _capi.load_library().lgs_diag_far_read((ctypes.c_ulonglong * 8)())
    ctx.timing_enable(True)
    for r in range(args.reps):
        ctx.klein(1, (r + 1) * n, n, z, v, lw, flags)
    ms, k = ctx.timing_get(_capi.KERNEL_KLEIN)
    avg = ms / k
    out = {"lib": os.environ.get("LGS_LIB", "default"), "config": args.config, "d": d, "n": n,
           "wl": args.wl, "center": args.center,
           "kernel_ms": round(avg, 3), "samples_per_s": round(n / avg * 1e3, 1)}
    if args.hash:  # outputs of the last launch, for A/B equality of library variants
        import hashlib
        torch.cuda.synchronize()
        out["z_sha"] = hashlib.sha256(z.cpu().numpy().tobytes()).hexdigest()[:16]
        out["lw_sha"] = hashlib.sha256(lw.cpu().numpy().tobytes()).hexdigest()[:16]
        if v is not None:
            out["v_sha"] = hashlib.sha256(v.cpu().numpy().tobytes()).hexdigest()[:16]
    if args.bz:
        ms, k = ctx.timing_get(_capi.KERNEL_BZ)
        out["bz_ms"] = round(ms / k, 3)
        out["bz_write_GBps"] = round(n * d * 8 / (ms / k) * 1e-6, 1)
    if diag is not None:
        diag(dbuf)
        waves = args.reps * n // 64
        names = ["stage", "far", "near", "sz_round", "sz_small", "sz_closed", "sz_capped", "sz_generic"]
        out["cycles_per_wave"] = {nm: round(dbuf[i] / waves) for i, nm in enumerate(names)}
        out["cycles_per_wave"]["kernel"] = round(dbuf[13] / waves)
        out["decisions_per_wave"] = {names[3 + k]: round(dbuf[8 + k] / waves, 1) for k in range(5)}
        out["cycles_per_decision"] = {names[3 + k]: round(dbuf[3 + k] / max(dbuf[8 + k], 1), 1)
                                      for k in range(5)}
    dfar = getattr(_capi.load_library(), "lgs_diag_far_read", None)
    if dfar is not None:
        fb = (ctypes.c_ulonglong * 8)()
        dfar(fb)
        waves = args.reps * n // 64
        out["far_cycles_per_wave"] = {nm: round(fb[i] / waves) for i, nm in enumerate(
            ["hist_wait", "slab_store", "mfma_issue", "barrier", "prologue", "epilogue"])}
        out["far_chunk_visits_per_wave"] = round(fb[6] / waves, 1)
        out["far_calls_per_wave"] = round(fb[7] / waves, 1)
    capq = getattr(_capi.load_library(), "lgs_diag_capq_read", None)
    if capq is not None:
        qb = (ctypes.c_ulonglong * 8)()
        capq(qb)
        out["capq"] = {"lanes": qb[0], "tol": qb[1], "range": qb[2], "v": qb[3], "rint": qb[4],
                       "waves_with_fail": qb[5], "waves": qb[6], "max_dmu": qb[7] * 1e-15}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3_ntru512")
    ap.add_argument("--n", type=int, default=1 << 18)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--exact", action="store_true")
    ap.add_argument("--one", action="store_true")
    ap.add_argument("--bz", action="store_true", help="also compute v = Bz and time bz_i8")
    ap.add_argument("--hash", action="store_true", help="print sha256 prefixes of the last launch's z (and v)")
    ap.add_argument("--wl", action="store_true", help="Wang-Ling weights")
    ap.add_argument("--center", type=float, default=0.0, help="scale of a random center (0: the origin)")
    args = ap.parse_args()
    libs = os.environ.get("LGS_LIBS")
    if args.one or not libs:
        run_one(args)
    else:
        for lib in libs.split(":"):
            env = dict(os.environ, LGS_LIB=lib)
            subprocess.run([sys.executable, __file__, "--one"] + sys.argv[1:], env=env, check=True, timeout=600)
