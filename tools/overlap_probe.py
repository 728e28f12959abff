"""Concurrency probe: does a Klein launch tolerate a memory-bound B z kernel on
another stream?  Two contexts on two streams: A runs lgs_klein (2^20 C3
proposals, no lattice points), B runs lgs_lattice_points (v = B z of 2^20
coordinate-major coefficients, the int8-digit kernel from the coefficient
store).  Wall time of A alone, B alone, and both enqueued together.

usage: python tools/overlap_probe.py [--n 1048576] [--reps 3]"""
import argparse
import json
import os
import sys
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lattice-gaussian-mcmc_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3_ntru512")
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--prio", action="store_true", help="A's stream at high priority")
    args = ap.parse_args()
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
    n = args.n
    sA, sB = torch.cuda.Stream(priority=-1 if args.prio else 0), torch.cuda.Stream()
    A, Bc = _capi.Context(0), _capi.Context(0)
    A.set_stream(sA.cuda_stream)
    Bc.set_stream(sB.cuda_stream)
    A.set_basis(R, cp, B, sigma)
    Bc.set_basis(R, cp, B, sigma)
    fl = _capi.LGS_DEVICE_PTRS | _capi.LGS_COORD_MAJOR
    zA = torch.empty((d, n), dtype=torch.int32, device="cuda:0")
    lwA = torch.empty(n, dtype=torch.float64, device="cuda:0")
    zB = torch.empty((d, n), dtype=torch.int32, device="cuda:0")
    lwB = torch.empty(n, dtype=torch.float64, device="cuda:0")
    vB = torch.empty((n, d), dtype=torch.float64, device="cuda:0")
    Bc.klein(2, 0, n, zB, None, lwB, fl)  # B's coefficients (a Klein draw)
    torch.cuda.synchronize()

    def runA(r):
        torch.cuda.set_device(0)
        A.klein(1, (r + 1) * n, n, zA, None, lwA, fl)

    def runB(r):
        torch.cuda.set_device(0)
        Bc.lattice_points(zB, vB, fl)

    runA(0)
    runB(0)
    torch.cuda.synchronize()
    out = {"config": args.config, "n": n, "prio": args.prio}
    for name, fns in (("klein", (runA,)), ("bz", (runB,)), ("both", (runA, runB)), ("klein", (runA,)),
                      ("bz", (runB,)), ("both", (runA, runB))):
        ts = []
        for r in range(args.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            # one host thread per call (each call waits for its own stream's flags;
            # ctypes releases the GIL), so the two launches are in flight together
            th = [threading.Thread(target=f, args=(r,)) for f in fns]
            for t in th:
                t.start()
            for t in th:
                t.join()
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        out.setdefault(name, []).append(round(min(ts), 3))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
