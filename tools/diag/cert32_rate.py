"""Where does the fp32 SampleZ certificate decline?  (diagnostic)"""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "lattice-gaussian-mcmc_amd"))
import numpy as np
from lgs_amd import _capi
ctx = _capi.Context(0)
rng = np.random.default_rng(78)
n = 400000
sig = np.exp(rng.uniform(np.log(4.0), np.log(1e6), n))
mu = rng.uniform(-1, 1, n) * rng.choice([1.0, 30.0, 1e4, 1e9], n)
u = rng.random(n)
z_c, _ = ctx.sample_z(mu, sig, u, mode="cert32")
z_t, _ = ctx.sample_z(mu, sig, u, table=True)
bad = z_c == np.iinfo(np.int64).min
print("decline rate", bad.mean())
for lo, hi in [(4, 10), (10, 50), (50, 100), (100, 1e3), (1e3, 1e4), (1e4, 1e5), (1e5, 1e6)]:
    m = (sig >= lo) & (sig < hi)
    print(f"sigma [{lo:g},{hi:g}) n={m.sum()} decline={bad[m].mean():.4f}")
for lo, hi in [(0, 0.01), (0.01, 0.1), (0.1, 0.9), (0.9, 0.99), (0.99, 1)]:
    m = (u >= lo) & (u < hi)
    print(f"u [{lo},{hi}) decline={bad[m].mean():.4f}")
idx = np.flatnonzero(bad)[:20]
for i in idx:
    print(f"mu={mu[i]!r} sig={sig[i]!r} u={u[i]!r} z_t={z_t[i]}")
