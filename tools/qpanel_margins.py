"""Margins of the q-panel z = 0 certificate (klein_mfma_kernel, reference mode) per
32-row panel, against the ||z_W|| of actual Klein samples.

For a row i of a panel made of speculative sub-panels (small kind, q[7] = 0), with
every speculative z decided so far equal to 0, the reference's mean obeys
|mu_i| <= (|c'_i| + (1 + g) sum_j |R_ij z_j|) / R_ii, and z_i = rint(mu_i) = 0 is
certain for |mu_i| < theta_i (lgs_capi.hip, lgs_set_basis).  The tests compared:

  cs      sum_j |R_ij z_j| <= G_i ||z_W||            (the shipped test: one number per
                                                      sample, ||z_W||^2 tracked exactly)
  cs64    sum over 64-coordinate blocks b of ||R_i,b|| ||z_b||   (blockwise Cauchy-Schwarz)
  l1      sum_j |R_ij| |z_j|                          (exact absolute sum: what any test
                                                      built on |z| alone can reach)
  true    |sum_j R_ij z_j| / R_ii = |mu_i|            (what the far field computes)

For each panel: the fraction of samples for which every row passes each test, the
largest bound / theta ratio over rows and samples, and for the digit-truncated far
field (R rounded to k base-256 digits of each row's maximum, the kernel's coarse
far field) the largest rounding bound 2^(E - 8k + 1) sum |z_j| / R_ii, E the row's
exponent.  Samples: the C oracle's Klein draws (test infrastructure only).

usage: python tools/qpanel_margins.py [--config C4_qary1024] [--n 2048]
"""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lattice-gaussian-mcmc_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C4_qary1024")
    ap.add_argument("--n", type=int, default=2048)
    ap.add_argument("--threads", type=int, default=8)
    args = ap.parse_args()
    import lgs_oracle
    from lgs_amd.lattices import build_config
    lat, sigma = build_config(args.config)
    B = lat.basis
    d = B.shape[0]
    R, cp = lgs_oracle.qr_prepare(B)
    rii = np.diag(R).copy()
    sig_i = sigma / rii
    small = sig_i < 4.0
    isv = np.where(small, 1.0 / np.where(small, sig_i, 1.0), 0.0)
    theta = np.where(small, 0.5 - 745.2 / np.maximum(isv ** 2 * (1 - 1e-12), 1e-300) - 1e-9, 0.0)
    W = ~small
    Z = lgs_oracle.klein_parallel(R, cp, sigma, args.n, seed=777, threads=args.threads)  # n x d
    Z = np.asarray(Z, dtype=np.float64)
    zW = Z * W[None, :]
    nzW = np.sqrt((zW ** 2).sum(1))
    g = 1.1 * d * 2.0 ** -53
    print(f"{args.config}: d {d}, sigma {sigma}, {int(small.sum())} small-kind rows, {args.n} oracle samples; "
          f"||z_W||: median {np.median(nzW):.4g}, max {nzW.max():.4g}")
    print("panel rows       pass: cs   cs64     l1   true | max bound/theta: cs     cs64       l1      true | "
          "coarse-digit rounding / theta (k=1, 2, 4)")
    nblk = (d + 63) // 64
    for pk in range(d // 32):
        hi = d - 32 * pk
        rows = np.arange(hi - 32, hi)
        if not small[rows].all():
            continue
        cs_r, cs64_r, l1_r, tr_r, dig = [], [], [], [], {1: [], 2: [], 4: []}
        for i in rows:
            Ri = R[i].copy()
            Ri[: i + 1] = 0.0
            RiW = Ri * W
            Gi = np.linalg.norm(RiW)
            blk = np.array([np.linalg.norm(RiW[64 * b:64 * b + 64]) for b in range(nblk)])
            zb = np.sqrt(np.add.reduceat(zW ** 2, np.arange(0, d, 64), axis=1))  # n x nblk
            num = theta[i] * rii[i] * (1 - 1e-12) - abs(cp[i])
            cs = (1 + g) * Gi * nzW
            cs64 = (1 + g) * (zb * blk[None, :]).sum(1)
            l1 = (1 + g) * np.abs(zW) @ np.abs(RiW)
            tr = np.abs(zW @ RiW)
            cs_r.append(cs / num)
            cs64_r.append(cs64 / num)
            l1_r.append(l1 / num)
            tr_r.append(tr / num)
            E = np.ceil(np.log2(np.abs(RiW).max() * 4)) if np.abs(RiW).max() > 0 else 0.0  # |R 2^-E| < 1/4
            for k in dig:
                dig[k].append((2.0 ** (E - 8 * k + 1)) * np.abs(zW).sum(1) / num)
        cs_r, cs64_r, l1_r, tr_r = (np.array(x) for x in (cs_r, cs64_r, l1_r, tr_r))  # rows x n
        frac = [float(((x < 1.0).all(0)).mean()) for x in (cs_r, cs64_r, l1_r, tr_r)]
        mx = [float(x.max()) for x in (cs_r, cs64_r, l1_r, tr_r)]
        dg = [float(np.array(dig[k]).max()) for k in (1, 2, 4)]
        print(f"{pk:5d} {hi - 32:4d}-{hi - 1:4d} {frac[0]:6.3f} {frac[1]:6.3f} {frac[2]:6.3f} {frac[3]:6.3f} | "
              f"{mx[0]:9.3g} {mx[1]:9.3g} {mx[2]:9.3g} {mx[3]:9.3g} | {dg[0]:9.3g} {dg[1]:9.3g} {dg[2]:9.3g}")


if __name__ == "__main__":
    main()
