"""Localise panel-kernel mismatches on ragged dimensions (diagnostic)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "lattice-gaussian-mcmc_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import lgs_oracle as oracle  # noqa: E402
from lgs_amd import _capi  # noqa: E402
from test_gpu_edges import _ill_basis as _int_basis  # noqa: E402

ctx = _capi.Context(0)
for d in [int(x) for x in os.environ.get("DS", "33 64 65 66 96 97 100 129").split()]:
    for n in (129, 128, 64):
        B = _int_basis(d, d)
        R, cp = oracle.qr_prepare(B)
        ctx.set_basis(R, cp, B, 3.5)
        r = ctx.klein_host(777 + d, 31, n, want_z=True, want_v=False, flags=0)
        o = oracle.klein(R, cp, 3.5, n, seed=777 + d, first_sample=31)
        bad = ~(r["z"] == o["z"])
        rows = np.nonzero(bad.any(1))[0]
        cols = np.nonzero(bad.any(0))[0]
        print(f"d={d} n={n} env={os.environ.get('LGS_FAR', '')}/{os.environ.get('LGS_PANEL', '')}: "
              f"{len(rows)} bad samples {rows[:8]} cols {cols[-8:]}", flush=True)

if os.environ.get("DETAIL"):
    d, n = 64, 64
    B = _int_basis(d, d)
    R, cp = oracle.qr_prepare(B)
    ctx.set_basis(R, cp, B, 3.5)
    r = ctx.klein_host(777 + d, 31, n, want_z=True, want_v=False, flags=0)
    o = oracle.klein(R, cp, 3.5, n, seed=777 + d, first_sample=31, want_mu=True)
    sig_i = 3.5 / np.abs(np.diag(R))
    print("sigma_i:", np.array2string(sig_i, precision=3, max_line_width=200))
    for s in range(n):
        bad = np.nonzero(r["z"][s] != o["z"][s])[0]
        if len(bad) == 0:
            continue
        i = bad.max()  # first coordinate sampled that differs (order d-1 -> 0)
        print(f"sample {s}: first diff coord {i}: gpu {r['z'][s][i]} oracle {o['z'][s][i]} "
              f"mu {o['mu'][s][i]!r} sigma_i {sig_i[i]:.6g}", flush=True)
