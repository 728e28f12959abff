"""Calibrate bench.py's CPU baseline: the NumPy restatement of the reference's
Klein loop (oracle/lgs_numpy_restatement.py, timed on the GPU box) against the
reference itself (src/samplers/klein.py:181-220, imported read-only from
/root/reference -- build container only), same C3 basis (NTRU n = 512,
sigma = 165.7), one core (BLAS limited to one thread), alternating rounds in one process.

usage: python3 -B tools/calibrate_cpu_baseline.py [--n 12] [--rounds 5]
Prints one line per round and a JSON summary (median rates, ratio)."""
import argparse
import json
import logging
import os
import statistics
import sys
import time

sys.dont_write_bytecode = True
for _v in ("OPENBLAS_NUM_THREADS", "OMP_NUM_THREADS", "MKL_NUM_THREADS"):
    os.environ[_v] = "1"  # one core: B @ x must not fan out over BLAS threads
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "lattice-gaussian-mcmc_amd"), os.path.join(REPO, "oracle"), "/root/reference"]

import numpy as np  # noqa: E402

import lgs_numpy_restatement as NR  # noqa: E402
import lgs_oracle  # noqa: E402
from lgs_amd.lattices import build_config  # noqa: E402


class Duck:
    """The attributes RefinedKleinSampler reads (simple.py:74-82)."""

    def __init__(self, B):
        self.basis = B
        self.dimension = B.shape[0]
        self.name = "C3_ntru512"
        self.min_gram_schmidt_norm = float(np.min(np.abs(np.diag(np.linalg.qr(B, mode="r")))))

    def smoothing_parameter(self):
        return 0.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=12)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--config", default="C3_ntru512")
    args = ap.parse_args()
    from src.samplers.klein import RefinedKleinSampler
    logging.disable(logging.WARNING)
    lat, sigma = build_config(args.config)
    B = lat.basis
    ref = RefinedKleinSampler(Duck(B), sigma)
    R, cp = lgs_oracle.qr_prepare(B)
    rst = NR.NumpyKlein(R, cp, B, sigma)
    np.random.seed(1)
    rr, rn = [], []
    for r in range(args.rounds):
        t0 = time.perf_counter()
        for _ in range(args.n):
            ref.sample_single()
        rr.append(args.n / (time.perf_counter() - t0))
        t0 = time.perf_counter()
        for s in range(args.n):
            k = r * args.n + s
            rst.sample_single(lambda slot, k=k: NR._philox_uniform(lgs_oracle, 1, slot, k, 0))
        rn.append(args.n / (time.perf_counter() - t0))
        print(f"round {r}: reference {rr[-1]:.3f}/s  restatement {rn[-1]:.3f}/s", flush=True)
    out = {"config": args.config, "d": int(B.shape[0]), "samples_per_round": args.n, "rounds": args.rounds,
           "cores": 1, "cpu": os.uname().machine, "load_avg": os.getloadavg(),
           "reference_per_core": round(statistics.median(rr), 3),
           "restatement_per_core": round(statistics.median(rn), 3)}
    out["restatement_over_reference"] = round(out["restatement_per_core"] / out["reference_per_core"], 3)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
