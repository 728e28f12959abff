"""Certified Wang-Ling IMHK accept decisions (imhk.py:158-167).

The default (blocked-order) kernels' Wang-Ling weights are within a derived bound
of the reference-order ones (lgs_kernels.hip wl_bound_*); imhk_accept_cert_kernel
takes a decision only when it is the same for every pair of weights within the
bounds, and otherwise recomputes both weights in the reference's order on the wave
(wl_exact_wave).  So the accept flags of every chain-step must equal those of
LGS_EXACT_ORDER (whose weights are the reference's), and a chain subset must equal
the C oracle.  LGS_TEST_WL_BOUND_SCALE widens the bounds so that thousands of
decisions take the recomputation path."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def capi():
    from lgs_amd import _capi
    return _capi


def _run(capi, ctx, d, nc, T, seed, flags, calls=1):
    """T Wang-Ling steps of nc chains from their initial draws, in `calls` equal
    lgs_imhk calls (calls > 1: the chain states, their weights and bounds and their
    state_init words cross call boundaries)."""
    import torch
    z = torch.zeros((d, nc), dtype=torch.int32, device="cuda")
    lw = torch.zeros(nc, dtype=torch.float64, device="cuda")
    init = torch.zeros(nc, dtype=torch.int32, device="cuda")
    acc = torch.zeros(nc, dtype=torch.int64, device="cuda")
    flags_t = torch.zeros((nc, T), dtype=torch.uint8, device="cuda")
    tb = T // calls
    for k in range(calls):
        ft = torch.zeros((nc, tb), dtype=torch.uint8, device="cuda")
        ctx.imhk(seed, 0, nc, 1 + k * tb, tb, 1, z, lw, init, acc, accepted=ft,
                 flags=capi.LGS_DEVICE_PTRS | capi.LGS_COORD_MAJOR | capi.LGS_WANG_LING | flags)
        flags_t[:, k * tb:(k + 1) * tb] = ft
    torch.cuda.synchronize()
    return z.cpu().numpy(), lw.cpu().numpy(), acc.cpu().numpy(), flags_t.cpu().numpy(), init.cpu().numpy()


@pytest.fixture(scope="module")
def c3(oracle):
    from lgs_amd.lattices import build_config
    lat, sigma = build_config("C3_ntru512")
    B = lat.basis
    R, cp = oracle.qr_prepare(B)
    return B, R, cp, sigma


@pytest.mark.parametrize("scale,calls", [(1.0, 1), (3e3, 1), (3e3, 2)])
def test_wl_accept_flags_equal_exact_order(capi, oracle, c3, scale, calls, monkeypatch):
    """C3 (NTRU n=512), 2^14 chains x 64 Wang-Ling steps: default-kernel accept flags
    identical to LGS_EXACT_ORDER's on every chain-step; 64 chains bit-equal to the
    oracle (accept counts, final states), so the subset's acceptance is the CPU
    reference's exactly.  scale > 1 widens every bound (test hook) so the
    reference-order recomputation decides thousands of steps; calls = 2 splits the
    64 steps over two lgs_imhk calls, so carried-in chain states are recomputed too
    -- with their own counters, from the draw step their state_init word records."""
    B, R, cp, sigma = c3
    d = B.shape[0]
    nc, T, seed = 1 << 14, 64, 4099
    ctx = capi.Context(0, hooks=scale != 1.0)  # (the bound scale is a test hook of liblgs_hip_hooks.so)
    ctx.set_basis(R, cp, B, sigma)
    zx, lwx, accx, fx, ix = _run(capi, ctx, d, nc, T, seed, capi.LGS_EXACT_ORDER)
    if scale != 1.0:
        monkeypatch.setenv("LGS_TEST_WL_BOUND_SCALE", str(scale))
    ctx.counter(capi.LGS_COUNTER_ACCEPT_RESOLVED, reset=True)
    ctx.counter(capi.LGS_COUNTER_WL_MISMATCH, reset=True)
    zd, lwd, accd, fd, idd = _run(capi, ctx, d, nc, T, seed, 0, calls=calls)
    nres = ctx.counter(capi.LGS_COUNTER_ACCEPT_RESOLVED)
    nbad = ctx.counter(capi.LGS_COUNTER_WL_MISMATCH)
    rate = accd.sum() / (nc * T)
    print(f"scale {scale}, {calls} call(s): acceptance {rate:.4f}, {nres} decisions at reference-order "
          f"weights, {int((fd != fx).sum())} of {nc * T} flags differ")
    assert nbad == 0  # every recomputed draw (carried states included) reproduced its z
    assert np.array_equal(fd, fx)  # every chain-step
    assert np.array_equal(accd, accx)
    assert np.array_equal(zd, zx)
    # state_init: the step each chain's state was drawn at (+2), the same in both
    assert np.array_equal(idd, ix) and int(idd.min()) >= 2
    if scale != 1.0:
        assert nres > 1000
    # final weights: the reference's wherever the state's weight was recomputed, else
    # within the bounds (largest bound at C3 ~1e-5)
    assert float(np.abs(lwd - lwx).max()) < 1e-4
    m = 64
    zo, lwo, acco = oracle.imhk_parallel(R, cp, B, sigma, m, T, seed=seed, first_step=1,
                                         mode=oracle.IMHK_WANG_LING, threads=8)
    assert np.array_equal(accd[:m], acco)
    assert np.array_equal(zd.T[:m], zo)
    sub_gpu, sub_cpu = accd[:m].sum() / (m * T), acco.sum() / (m * T)
    print(f"64-chain subset: GPU acceptance {sub_gpu:.5f}, C oracle {sub_cpu:.5f}")
    assert sub_gpu == sub_cpu and 0.0 < sub_cpu < 1.0
