"""ORACLE / TEST INFRASTRUCTURE ONLY -- ctypes front-end of oracle/lgs_oracle.c.

CPU restatement of the reference's Klein/IMHK hot path
(``src/samplers/klein.py``, ``src/samplers/imhk.py``, ``src/samplers/base.py``
of NickQrumpton/lattice-gaussian-mcmc).  Imported only by ``tests/``,
``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of ``bench.py``; the
product package (``lattice-gaussian-mcmc_amd/lgs_amd``) never imports it.

Parity is pinned by the reference's published seed-42 artifacts (MT19937 mode)
and by golden vectors generated from the reference itself (Philox mode); see
``tests/golden/make_golden.py`` and DESIGN.md.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# LGS_ORACLE_LIB: another build of the same source (the ASan/UBSan one, `make sanitize`)
_LIB_PATH = os.environ.get("LGS_ORACLE_LIB") or os.path.join(_HERE, "_build", "liblgs_oracle.so")
_lib = None

RNG_MT = 0
RNG_PHILOX = 1
IMHK_REFERENCE = 0
IMHK_WANG_LING = 1

_i64p = ctypes.POINTER(ctypes.c_int64)
_i32p = ctypes.POINTER(ctypes.c_int32)
_dp = ctypes.POINTER(ctypes.c_double)


def build():
    """Compile the oracle with its Makefile (gcc, no GPU needed)."""
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.lgso_mt_new.restype = ctypes.c_void_p
        L.lgso_mt_new.argtypes = [ctypes.c_uint32]
        L.lgso_mt_free.argtypes = [ctypes.c_void_p]
        L.lgso_mt_double.restype = ctypes.c_double
        L.lgso_mt_double.argtypes = [ctypes.c_void_p]
        L.lgso_philox.argtypes = [ctypes.POINTER(ctypes.c_uint32)] * 3
        L.lgso_philox_u.restype = ctypes.c_double
        L.lgso_philox_u.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                                    ctypes.c_uint32, ctypes.c_uint32]
        L.lgso_pairwise_sum.restype = ctypes.c_double
        L.lgso_pairwise_sum.argtypes = [_dp, ctypes.c_int64]
        L.lgso_logsumexp.restype = ctypes.c_double
        L.lgso_logsumexp.argtypes = [_dp, ctypes.c_int64, _dp]
        L.lgso_sample_z.restype = ctypes.c_int64
        L.lgso_sample_z.argtypes = [ctypes.c_double, ctypes.c_double, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_double, _dp, ctypes.POINTER(ctypes.c_int)]
        L.lgso_support.restype = ctypes.c_int64
        L.lgso_support.argtypes = [ctypes.c_double, ctypes.c_double, ctypes.c_int, _i64p]
        L.lgso_klein.restype = ctypes.c_int
        L.lgso_klein.argtypes = [ctypes.c_int64, _dp, _dp, ctypes.c_double, ctypes.c_int,
                                 ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64,
                                 ctypes.c_uint64, ctypes.c_int64, _dp, _i64p, _dp, _dp, _i64p]
        L.lgso_klein_parallel.restype = ctypes.c_int
        L.lgso_klein_parallel.argtypes = [ctypes.c_int64, _dp, _dp, ctypes.c_double, ctypes.c_int,
                                          ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64,
                                          ctypes.c_int64, _i64p, ctypes.c_int]
        L.lgso_imhk_parallel.restype = ctypes.c_int
        L.lgso_imhk_parallel.argtypes = [ctypes.c_int64, _dp, _dp, _dp, _dp, ctypes.c_double,
                                         ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint64,
                                         ctypes.c_uint64, ctypes.c_int64, ctypes.c_uint64,
                                         ctypes.c_int64, _i64p, _dp, _i32p, _i64p, ctypes.c_int]
        L.lgso_log_weight.restype = ctypes.c_double
        L.lgso_log_weight.argtypes = [ctypes.c_int64, _dp, _dp, _dp, _dp, ctypes.c_double,
                                      ctypes.c_int, ctypes.c_int, ctypes.c_int, _i64p]
        L.lgso_imhk.restype = ctypes.c_int
        L.lgso_imhk.argtypes = [ctypes.c_int64, _dp, _dp, _dp, _dp, ctypes.c_double, ctypes.c_int,
                                ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int64, ctypes.c_uint64,
                                ctypes.c_int64, _i64p, _dp, _i32p, _i64p, _i64p]
        _lib = L
    return _lib


def _p(a, t):
    return None if a is None else a.ctypes.data_as(t)


def qr_prepare(basis, center=None):
    """Host setup of klein.py:56-79: full QR, sign fix so R_ii > 0, c' = Q^T c.

    Returns (R, cprime) as C-contiguous float64 arrays.
    """
    B = np.asarray(basis, dtype=np.float64)
    d = B.shape[0]
    Q, R = np.linalg.qr(B, mode="full")
    for i in range(d):
        if R[i, i] < 0:
            R[i, :] *= -1
            Q[:, i] *= -1
    c = np.zeros(d) if center is None else np.asarray(center, dtype=np.float64)
    return np.ascontiguousarray(R), np.ascontiguousarray(Q.T @ c)


class MT19937:
    """NumPy legacy RandomState stream (seeded like ``np.random.seed(int)``)."""

    def __init__(self, seed: int):
        self.h = lib().lgso_mt_new(ctypes.c_uint32(seed))

    def double(self) -> float:
        return lib().lgso_mt_double(self.h)

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.lgso_mt_free(self.h)
            self.h = None


def philox(ctr, key):
    c = (ctypes.c_uint32 * 4)(*[int(x) & 0xFFFFFFFF for x in ctr])
    k = (ctypes.c_uint32 * 2)(*[int(x) & 0xFFFFFFFF for x in key])
    o = (ctypes.c_uint32 * 4)()
    lib().lgso_philox(c, k, o)
    return tuple(o)


def philox_u(seed, slot, step, chain, tag):
    return lib().lgso_philox_u(seed, slot, step, chain, tag)


def pairwise_sum(a):
    a = np.ascontiguousarray(a, dtype=np.float64)
    return lib().lgso_pairwise_sum(_p(a, _dp), a.size)


def logsumexp(a):
    a = np.ascontiguousarray(a, dtype=np.float64)
    tmp = np.empty(max(a.size, 1))
    return lib().lgso_logsumexp(_p(a, _dp), a.size, _p(tmp, _dp))


def sample_z(mean, sigma, u, precision=10, use_log_space=True):
    """SampleZ decision of klein.py:143-179 for a given uniform u."""
    work = np.empty(3 * 1024)
    fb = ctypes.c_int(0)
    k = lib().lgso_sample_z(mean, sigma, precision, int(use_log_space), u, _p(work, _dp),
                            ctypes.byref(fb))
    return int(k), bool(fb.value)


def support(mean, sigma, precision=10):
    lo = ctypes.c_int64(0)
    n = lib().lgso_support(mean, sigma, precision, ctypes.byref(lo))
    return int(lo.value), int(n)


def klein(R, cprime, sigma, n, *, seed=0, first_sample=0, rng="philox", mt=None, B=None,
          precision=10, use_log_space=True, want_mu=False):
    """n Klein samples (klein.py:181-220).  Returns dict(z, v, mu, fallbacks)."""
    R = np.ascontiguousarray(R, dtype=np.float64)
    cp = np.ascontiguousarray(cprime, dtype=np.float64)
    d = R.shape[0]
    z = np.zeros((n, d), dtype=np.int64)
    v = np.zeros((n, d)) if B is not None else None
    mu = np.zeros((n, d)) if want_mu else None
    Bc = None if B is None else np.ascontiguousarray(B, dtype=np.float64)
    nfb = ctypes.c_int64(0)
    kind = RNG_MT if rng == "mt" else RNG_PHILOX
    if kind == RNG_MT and mt is None:
        raise ValueError("mt stream required")
    rc = lib().lgso_klein(d, _p(R, _dp), _p(cp, _dp), sigma, precision, int(use_log_space), kind,
                          mt.h if mt is not None else None, seed, first_sample, n, _p(Bc, _dp),
                          _p(z, _i64p), _p(v, _dp), _p(mu, _dp), ctypes.byref(nfb))
    if rc != 0:
        raise RuntimeError(f"lgso_klein failed rc={rc}")
    return {"z": z, "v": v, "mu": mu, "fallbacks": int(nfb.value)}


def klein_parallel(R, cprime, sigma, n, *, seed=0, first_sample=0, precision=10,
                   use_log_space=True, threads=1):
    R = np.ascontiguousarray(R, dtype=np.float64)
    cp = np.ascontiguousarray(cprime, dtype=np.float64)
    d = R.shape[0]
    z = np.zeros((n, d), dtype=np.int64)
    rc = lib().lgso_klein_parallel(d, _p(R, _dp), _p(cp, _dp), sigma, precision,
                                   int(use_log_space), seed, first_sample, n, _p(z, _i64p), threads)
    if rc != 0:
        raise RuntimeError(f"lgso_klein_parallel failed rc={rc}")
    return z


def log_weight(R, cprime, B, sigma, z, *, center=None, mode=IMHK_REFERENCE, precision=10,
               use_log_space=True):
    R = np.ascontiguousarray(R, dtype=np.float64)
    cp = np.ascontiguousarray(cprime, dtype=np.float64)
    Bc = np.ascontiguousarray(B, dtype=np.float64)
    c = None if center is None else np.ascontiguousarray(center, dtype=np.float64)
    zz = np.ascontiguousarray(z, dtype=np.int64)
    return lib().lgso_log_weight(R.shape[0], _p(R, _dp), _p(cp, _dp), _p(Bc, _dp), _p(c, _dp),
                                 sigma, precision, int(use_log_space), mode, _p(zz, _i64p))


def imhk(R, cprime, B, sigma, n_chains, n_steps, *, center=None, seed=0, first_chain=0,
         first_step=1, state=None, mode=IMHK_REFERENCE, rng="philox", mt=None, precision=10,
         use_log_space=True, trace=False):
    """IMHK chains (imhk.py:126-177).  `state` = dict(z, lw, init, accepts) to resume."""
    R = np.ascontiguousarray(R, dtype=np.float64)
    cp = np.ascontiguousarray(cprime, dtype=np.float64)
    Bc = np.ascontiguousarray(B, dtype=np.float64)
    c = None if center is None else np.ascontiguousarray(center, dtype=np.float64)
    d = R.shape[0]
    if state is None:
        state = {"z": np.zeros((n_chains, d), dtype=np.int64), "lw": np.zeros(n_chains),
                 "init": np.zeros(n_chains, dtype=np.int32),
                 "accepts": np.zeros(n_chains, dtype=np.int64)}
    ztr = np.zeros((n_chains, n_steps, d), dtype=np.int64) if trace else None
    kind = RNG_MT if rng == "mt" else RNG_PHILOX
    rc = lib().lgso_imhk(d, _p(R, _dp), _p(cp, _dp), _p(Bc, _dp), _p(c, _dp), sigma, precision,
                         int(use_log_space), mode, kind, mt.h if mt is not None else None, seed,
                         first_chain, n_chains, first_step, n_steps, _p(state["z"], _i64p),
                         _p(state["lw"], _dp), _p(state["init"], _i32p),
                         _p(state["accepts"], _i64p), _p(ztr, _i64p))
    if rc != 0:
        raise RuntimeError(f"lgso_imhk failed rc={rc}")
    state["trace"] = ztr
    return state


def imhk_parallel(R, cprime, B, sigma, n_chains, n_steps, *, center=None, seed=0, first_chain=0,
                  first_step=1, mode=IMHK_REFERENCE, precision=10, use_log_space=True, threads=1):
    """Philox-mode IMHK chains in parallel (OpenMP); returns (z_state, lw, accepts)."""
    R = np.ascontiguousarray(R, dtype=np.float64)
    cp = np.ascontiguousarray(cprime, dtype=np.float64)
    Bc = np.ascontiguousarray(B, dtype=np.float64)
    c = None if center is None else np.ascontiguousarray(center, dtype=np.float64)
    d = R.shape[0]
    z = np.zeros((n_chains, d), dtype=np.int64)
    lw = np.zeros(n_chains)
    init = np.zeros(n_chains, dtype=np.int32)
    acc = np.zeros(n_chains, dtype=np.int64)
    rc = lib().lgso_imhk_parallel(d, _p(R, _dp), _p(cp, _dp), _p(Bc, _dp), _p(c, _dp), sigma,
                                  precision, int(use_log_space), mode, seed, first_chain, n_chains,
                                  first_step, n_steps, _p(z, _i64p), _p(lw, _dp), _p(init, _i32p),
                                  _p(acc, _i64p), threads)
    if rc != 0:
        raise RuntimeError(f"lgso_imhk_parallel failed rc={rc}")
    return z, lw, acc
