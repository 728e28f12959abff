"""IMHKSampler.step() served from look-ahead blocks (lgs_imhk_trace) equals one
launch per step -- states, accept decisions, current_log_weight and counters
(imhk.py:141-177) -- including interleaving with sample()/run_chain() and block
refills, in the reference weight mode and the Wang-Ling mode (rejections)."""
import numpy as np
import pytest

from conftest import load_golden

pytestmark = pytest.mark.gpu


def _one_launch_step(s):
    """The unbuffered path: one lgs_imhk call per step."""
    _, a = s._run(1, 1, keep=False)
    return s.current_state.copy(), bool(a)


@pytest.mark.parametrize("wang_ling", [False, True])
def test_buffered_step_equals_single_launches(wang_ling):
    from lgs_amd.lattices import SimpleLattice
    from lgs_amd.samplers import IMHKSampler
    g = load_golden("imhk_B2.npz")
    # sigma 1.2: sigma_i = 0.29, 0.45, where the Wang-Ling normalisers vary with mu
    # enough for frequent rejections
    mk = lambda: IMHKSampler(SimpleLattice(g["B"]), 1.2, burn_in=0, seed=123,
                             chain_id=3, wang_ling=wang_ling)
    a, b = mk(), mk()
    acc_a, acc_b = [], []

    def both(k):
        for _ in range(k):
            va, fa = a.step()
            vb, fb = _one_launch_step(b)
            assert np.array_equal(va, vb)
            assert fa == fb
            assert a.current_log_weight == b.current_log_weight
            assert np.array_equal(a.current_coeffs, b.current_coeffs)
            acc_a.append(fa)
            acc_b.append(fb)

    both(5)
    assert np.array_equal(a.sample(7, thin=2), b.sample(7, thin=2))
    both(40)  # crosses a refill (16, then 32 steps)
    ca, cb = a.run_chain(9, save_every=2), b.run_chain(9, save_every=2)
    assert all(np.array_equal(x, y) for x, y in zip(ca, cb))
    both(3)
    assert a.total_proposals == b.total_proposals
    assert a.accepted_proposals == b.accepted_proposals
    if wang_ling:
        assert not all(acc_a), "expected rejections with the Wang-Ling weight"
    # changing the counters between steps drops the look-ahead block:
    # the next steps use the new seed / chain id, as an unbuffered launch does
    a.seed = b.seed = 777
    both(4)
    a.chain_id = b.chain_id = 11
    both(4)


def test_imhk_trace_matches_oracle(oracle):
    """Per-step accept flags and kept log weights of lgs_imhk_trace against the CPU
    oracle's IMHK trace (same counters)."""
    from lgs_amd import _capi
    from lgs_amd.lattices import build_config
    lat, sigma = build_config("C2_qary128")
    B = lat.basis
    R, cp = oracle.qr_prepare(B)
    ctx = _capi.Context(0)
    ctx.set_basis(R, cp, B, sigma)
    d = R.shape[0]
    nc, steps = 3, 20
    z = np.zeros((nc, d), dtype=np.int32)
    lw = np.zeros(nc)
    init = np.zeros(nc, dtype=np.int32)
    acc = np.zeros(nc, dtype=np.int64)
    zs = np.zeros((nc, steps, d), dtype=np.int32)
    lws = np.zeros((nc, steps))
    accd = np.zeros((nc, steps), dtype=np.uint8)
    ctx.imhk(11, 0, nc, 1, steps, 1, z, lw, init, acc, z_samples=zs, logw_samples=lws, accepted=accd,
             flags=_capi.LGS_WANG_LING)
    st = oracle.imhk(R, cp, B, sigma, nc, steps, seed=11, first_step=1, trace=True,
                     mode=oracle.IMHK_WANG_LING)
    assert np.array_equal(zs, st["trace"])
    assert np.array_equal(acc, st["accepts"])
    assert np.array_equal(accd.sum(axis=1), acc)
    assert np.array_equal(lws[:, -1], lw)
    # a state that changed was accepted; the kept weight follows the state
    changed = np.any(zs[:, 1:] != zs[:, :-1], axis=2)
    assert np.all(accd[:, 1:][changed] == 1)
    assert np.all(lws[:, 1:][~accd[:, 1:].astype(bool)] == lws[:, :-1][~accd[:, 1:].astype(bool)])
