"""Certified decisions of the default (blocked-order) Klein kernels at BASELINE scale.

The default kernels form each conditional mean in blocked order (int8-digit /
fp64 MFMA far field, FMA near field, reciprocal of R_ii); every SampleZ decision is
certified against a rigorous bound on its distance to the reference-order mean
(klein.py:191-195) or replayed in that order (lgs_device.h, certified decisions).
Their coefficients must therefore equal LGS_EXACT_ORDER's -- which follows the
reference's arithmetic order and is bit-exact against the oracle
(test_gpu_parity.py) -- on every sample, at the sizes the bench runs.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def capi():
    from lgs_amd import _capi
    return _capi


@pytest.mark.parametrize("cfg,n", [("C3_ntru512", 1 << 16), ("C2_qary128", 1 << 18),
                                   ("C4_qary1024", 1 << 15)])
def test_default_order_equals_exact_order_at_scale(capi, oracle, cfg, n):
    import torch
    from lgs_amd.lattices import build_config
    lat, sigma = build_config(cfg)
    B = lat.basis
    R, cp = oracle.qr_prepare(B)
    ctx = capi.Context(0)
    ctx.set_basis(R, cp, B, sigma)
    d = B.shape[0]
    za = torch.empty((d, n), dtype=torch.int32, device="cuda")
    zb = torch.empty_like(za)
    f = capi.LGS_DEVICE_PTRS | capi.LGS_COORD_MAJOR
    ctx.resolved(reset=True)
    ctx.klein(77, 0, n, za, None, None, f)
    redos = ctx.resolved()
    assert ctx.fallbacks() == 0  # the int8-digit far field / 16-bit store path itself was checked
    ctx.klein(77, 0, n, zb, None, None, f | capi.LGS_EXACT_ORDER)
    torch.cuda.synchronize()
    bad = int((za != zb).any(dim=0).sum())
    print(f"{cfg}: {n} samples, {redos} certificate replays, {bad} samples differ")
    assert bad == 0
