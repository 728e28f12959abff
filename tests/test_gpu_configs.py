"""GPU parity at BASELINE configs C4 (q-ary d=1024, k=512) and C5 (NTRU n=2048, d=4096).

* Klein coefficients and lattice points of the default (certified blocked-order)
  kernels on a 256-sample launch -- whole 256-sample blocks, so the int8-digit far
  field runs, over the most panels at d = 4096 -- are bit-exact against the C
  oracle on a subset and against LGS_EXACT_ORDER on every sample; the
  reference-order kernel itself is bit-exact against the oracle.
* Wang-Ling IMHK (acceptance < 1): the accept decisions and states of a chain
  subset are bit-exact against the oracle on the same counters, so the
  acceptance is the CPU reference's (north_star: "acceptance validated vs CPU").

C5 runs in full fp64 (BASELINE configs[4] names fp32 sampling; the int8-digit far
field keeps the fp64 semantics at int8 MFMA rates).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CASES = [("C4_qary1024", 64, 8), ("C5_ntru2048", 16, 4)]
_cache = {}


def _setup(cfg, oracle):
    if cfg not in _cache:
        from lgs_amd.lattices import build_config
        lat, sigma = build_config(cfg)
        B = lat.basis
        R, cp = oracle.qr_prepare(B)
        _cache[cfg] = (B, R, cp, sigma)
    return _cache[cfg]


@pytest.mark.parametrize("cfg,n_oracle,_", CASES)
def test_klein_bit_exact(oracle, cfg, n_oracle, _):
    import torch
    from lgs_amd import _capi
    B, R, cp, sigma = _setup(cfg, oracle)
    d = B.shape[0]
    ctx = _capi.Context(0)
    ctx.set_basis(R, cp, B, sigma)
    n, seed, first = 256, 1234, 7 << 20
    f = _capi.LGS_DEVICE_PTRS | _capi.LGS_COORD_MAJOR
    za = torch.empty((d, n), dtype=torch.int32, device="cuda")
    zb = torch.empty_like(za)
    va = torch.empty((n, d), dtype=torch.float64, device="cuda")
    ctx.klein(seed, first, n, za, va, None, f)
    assert ctx.fallbacks() == 0  # the int8-digit far field path itself
    ctx.klein(seed, first, n, zb, None, None, f | _capi.LGS_EXACT_ORDER)
    assert torch.equal(za, zb)  # certified blocked order == reference order, every sample
    sub = list(range(n_oracle // 2)) + list(range(n - n_oracle // 2, n))
    zo = np.concatenate([oracle.klein_parallel(R, cp, sigma, n_oracle // 2, seed=seed, first_sample=first + s0,
                                               threads=16) for s0 in (0, n - n_oracle // 2)])
    z = za.cpu().numpy().T
    assert np.array_equal(z[sub], zo)
    np.testing.assert_array_equal(va.cpu().numpy()[sub], zo.astype(np.float64) @ B.T)


@pytest.mark.parametrize("cfg,_,m", CASES)
def test_wang_ling_imhk_subset_bit_exact(oracle, cfg, _, m):
    import torch
    from lgs_amd import _capi
    B, R, cp, sigma = _setup(cfg, oracle)
    d = B.shape[0]
    ctx = _capi.Context(0)
    ctx.set_basis(R, cp, B, sigma)
    nc, T, seed = 256, 2, 77
    z = torch.zeros((d, nc), dtype=torch.int32, device="cuda")
    lw = torch.zeros(nc, dtype=torch.float64, device="cuda")
    init = torch.zeros(nc, dtype=torch.int32, device="cuda")
    acc = torch.zeros(nc, dtype=torch.int64, device="cuda")
    ctx.imhk(seed, 0, nc, 1, T, 1, z, lw, init, acc,
             flags=_capi.LGS_DEVICE_PTRS | _capi.LGS_COORD_MAJOR | _capi.LGS_WANG_LING)
    zo, lwo, acco = oracle.imhk_parallel(R, cp, B, sigma, m, T, seed=seed, first_step=1,
                                         mode=oracle.IMHK_WANG_LING, threads=16)
    assert np.array_equal(acc.cpu().numpy()[:m], acco)
    assert np.array_equal(z.cpu().numpy().T[:m], zo)
    np.testing.assert_allclose(lw.cpu().numpy()[:m], lwo, rtol=1e-9, atol=1e-9)
    rate = acc.sum().item() / (nc * T)
    assert 0.0 < rate <= 1.0


ACC_CASES = [("C3_ntru512", 1 << 14, 1024), ("C4_qary1024", 1 << 14, 1024), ("C5_ntru2048", 1 << 11, 256)]


@pytest.mark.parametrize("cfg,nc,m", ACC_CASES)
def test_imhk_acceptance_vs_cpu(oracle, cfg, nc, m):
    """IMHK acceptance against the CPU reference (imhk.py:141-177), north_star
    'acceptance within +-1 % of CPU reference', at C3, C4 and C5:
    * reference-mode weights: every proposal accepted on the GPU (1.0 exactly),
      as in the reference (its weight is a constant up to rounding), and the first m
      chains' accept counts, final states and log weights equal to the oracle's in
      reference mode -- the coarse q-panel far field and the q-panel skip move the
      weights' rounding only;
    * Wang-Ling weights: the oracle runs the first m chains x 4 steps on the same
      counters -- every accept decision and final state is bit-equal -- and the
      GPU's acceptance over all nc chains is within 1 % (absolute) of the oracle's
      (or 4 standard errors of the oracle estimate, whichever is larger)."""
    import torch
    from lgs_amd import _capi
    B, R, cp, sigma = _setup(cfg, oracle)
    d = B.shape[0]
    ctx = _capi.Context(0)
    ctx.set_basis(R, cp, B, sigma)
    T, seed = 4, 2027
    res = {}
    for wl in (False, True):
        z = torch.zeros((d, nc), dtype=torch.int32, device="cuda")
        lw = torch.zeros(nc, dtype=torch.float64, device="cuda")
        init = torch.zeros(nc, dtype=torch.int32, device="cuda")
        acc = torch.zeros(nc, dtype=torch.int64, device="cuda")
        f = _capi.LGS_DEVICE_PTRS | _capi.LGS_COORD_MAJOR | (_capi.LGS_WANG_LING if wl else 0)
        ctx.imhk(seed, 0, nc, 1, T, 1, z, lw, init, acc, flags=f)
        res[wl] = (acc.cpu().numpy(), z[:, :m].cpu().numpy().T, lw[:m].cpu().numpy())
    assert res[False][0].sum() == nc * T  # reference mode: acceptance 1.0
    zr, lwr, accr = oracle.imhk_parallel(R, cp, B, sigma, m, T, seed=seed, first_step=1,
                                         mode=oracle.IMHK_REFERENCE, threads=16)
    assert np.array_equal(res[False][0][:m], accr)
    assert np.array_equal(res[False][1], zr)
    np.testing.assert_allclose(res[False][2], lwr, rtol=1e-12, atol=1e-9)
    acc_wl, z_wl, _ = res[True]
    zo, _, acco = oracle.imhk_parallel(R, cp, B, sigma, m, T, seed=seed, first_step=1,
                                       mode=oracle.IMHK_WANG_LING, threads=16)
    assert np.array_equal(acc_wl[:m], acco)  # bit-equal decisions on the CPU subset
    assert np.array_equal(z_wl, zo)
    gpu, cpu = acc_wl.sum() / (nc * T), acco.sum() / (m * T)
    se = np.sqrt(max(cpu * (1 - cpu), 1e-4) / (m * T))
    assert abs(gpu - cpu) < max(0.01, 4 * se), (gpu, cpu, se)
    print(f"{cfg}: Wang-Ling acceptance GPU {gpu:.4f} ({nc} chains) vs CPU oracle {cpu:.4f} ({m} chains), "
          f"se {se:.4f}; reference mode 1.0")
