"""1-D window normalisers log sum_k exp(-(k - mu)^2 / (2 sigma^2)) computed by the
REFERENCE itself, for the (mu, sigma) pairs of samplez_table.npz.

The Wang-Ling weight / delta multiplies these normalisers.
The reference's Jacobi theta (src/samplers/utils.py:141-206) cannot pin them: its
direct sum starts at n = -max_iterations and stops at the first summand below
`precision` (utils.py:168-178), i.e. immediately, so it returns 0 for every
argument (probe below).  The reference's own window normaliser is the logsumexp
of klein.py:132-134 inside RefinedKleinSampler._compute_1d_probabilities; it is
recovered here from that method's output at the window's heaviest point:
lse = raw[k*] - log_probs[k*], raw = -0.5 ((support - mean) / sigma)^2.

Usage:  python3 -B tests/golden/make_golden_normalisers.py   (writes samplez_lognorm.npz)
"""
import os
import sys

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402

import make_golden as mg  # noqa: E402
from src.samplers.utils import DiscreteGaussianUtils  # noqa: E402


def main():
    g = np.load(os.path.join(HERE, "samplez_table.npz"))
    s = mg.RefinedKleinSampler(mg.DuckLattice(np.eye(2), "norm"), 1.0)
    mu, sig = g["mu"], g["sigma"]
    lse = np.empty(mu.size)
    lo = np.empty(mu.size, dtype=np.int64)
    hi = np.empty(mu.size, dtype=np.int64)
    for i in range(mu.size):
        sup, lp = s._compute_1d_probabilities(float(mu[i]), float(sig[i]), 10)
        raw = -0.5 * ((sup - mu[i]) / sig[i]) ** 2
        k = int(np.argmax(raw))
        lse[i] = raw[k] - lp[k]
        lo[i], hi[i] = sup[0], sup[-1]
    # the reference's theta_3 on the same quantities (rho = exp(-mu^2/2s^2) theta_3(z|tau))
    u = DiscreteGaussianUtils()
    probe = []
    for i in range(0, mu.size, 500):
        tau = 1j / (2 * np.pi * sig[i] ** 2)
        z = -1j * mu[i] / (2 * np.pi * sig[i] ** 2)
        probe.append(complex(u.jacobi_theta_3(z, tau)))
    np.savez_compressed(os.path.join(HERE, "samplez_lognorm.npz"), mu=mu, sigma=sig, log_norm=lse,
                        lo=lo, hi=hi, theta3_probe=np.array(probe), theta3_probe_index=np.arange(0, mu.size, 500))
    print(f"samplez_lognorm: {mu.size} normalisers; reference theta_3 probe values: {set(probe)}")


if __name__ == "__main__":
    main()
