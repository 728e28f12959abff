"""Default (certified blocked-order) Klein kernel vs LGS_EXACT_ORDER at scale.

usage: python tools/cert_mismatch.py [--config C3_ntru512] [--total 16777216] [--chunk 262144]
Draws `total` Klein samples (counter-addressed: samples 0 .. total-1) with both
kernels in chunks, compares every coefficient vector on the device and prints one
JSON line: samples compared, samples that differ, certificate verifications, and
both kernels' device time / samples per second."""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lattice-gaussian-mcmc_amd"))

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="C3_ntru512")
ap.add_argument("--total", type=int, default=1 << 24)
ap.add_argument("--chunk", type=int, default=1 << 18)
args = ap.parse_args()

import numpy as np
import torch
from lgs_amd import _capi
from lgs_amd.lattices import build_config

lat, sigma = build_config(args.config)
B = lat.basis
d = B.shape[0]
Q, R = np.linalg.qr(B)
R = np.ascontiguousarray(R * np.where(np.diag(R) < 0, -1.0, 1.0)[:, None])
ctx = _capi.Context(0)
ctx.set_basis(R, np.zeros(d), B, sigma)
n = args.chunk
za = torch.empty((d, n), dtype=torch.int32, device="cuda:0")
zb = torch.empty_like(za)
f = _capi.LGS_DEVICE_PTRS | _capi.LGS_COORD_MAJOR
ctx.klein(5, 0, n, za, None, None, f)  # warm-up
ctx.klein(5, 0, n, zb, None, None, f | _capi.LGS_EXACT_ORDER)
ctx.resolved(reset=True)
ctx.fallbacks(reset=True)
bad = 0
t_fast = t_exact = 0.0
for c in range(args.total // n):
    ctx.timing_enable(True)
    ctx.klein(5, c * n, n, za, None, None, f)
    t_fast += ctx.timing_get(_capi.KERNEL_KLEIN)[0]
    ctx.timing_enable(True)
    ctx.klein(5, c * n, n, zb, None, None, f | _capi.LGS_EXACT_ORDER)
    t_exact += ctx.timing_get(_capi.KERNEL_KLEIN)[0]
    bad += int((za != zb).any(dim=0).sum())
    print(json.dumps({"chunk": c, "differ_so_far": bad, "verified_so_far": ctx.resolved()}), flush=True)
total = (args.total // n) * n
print(json.dumps({"config": args.config, "d": d, "samples": total, "samples_differ": bad,
                  "certificate_verifications": ctx.resolved(), "fallback_launches": ctx.fallbacks(),
                  "default_kernel_ms_per_chunk": round(t_fast / (total // n), 3),
                  "exact_kernel_ms_per_chunk": round(t_exact / (total // n), 3),
                  "default_samples_per_s": round(total / (t_fast / 1e3), 1),
                  "exact_samples_per_s": round(total / (t_exact / 1e3), 1)}), flush=True)
