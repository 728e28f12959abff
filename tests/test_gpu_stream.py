"""StreamingShard's per-block lag-sum update replayed as a captured HIP graph (the
bench's timed path) equals the eager update, block by block, on the same inputs."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(__file__)), "lattice-gaussian-mcmc_amd"))

pytestmark = pytest.mark.gpu


def _run(graph: bool, blocks: int = 5):
    import torch
    from lgs_amd import distributed as D
    old = os.environ.get("LGS_NO_GRAPH")
    os.environ["LGS_NO_GRAPH"] = "0" if graph else "1"
    try:
        nc, T, d = 96, 8, 24
        buf = torch.empty((nc, T, d), dtype=torch.float64, device="cuda:0")
        rng = np.random.default_rng(5)
        data = [rng.integers(-300, 300, size=(nc, T, d)).astype(np.float64) for _ in range(blocks)]
        it = iter(data)

        def advance(first_step, n_steps, acc, mom):
            buf.copy_(torch.from_numpy(next(it)))  # same buffer every block, as gpu_advance
            acc += 1
            return buf

        binv = rng.standard_normal(d) * 0.01
        sh = D.StreamingShard(advance, nc, d, binv_row=binv, device="cuda:0", lag_chains=64, lags=5)
        for _ in range(blocks):
            sh.step(T)
        torch.cuda.synchronize()
        return ([x.cpu().numpy().copy() for x in sh.lag_z.parts()], [x.cpu().numpy().copy() for x in sh.lag_v.parts()],
                sh._graph is not None)
    finally:
        if old is None:
            os.environ.pop("LGS_NO_GRAPH", None)
        else:
            os.environ["LGS_NO_GRAPH"] = old


def test_lag_sums_graph_replay_equals_eager():
    z_g, v_g, captured = _run(True)
    z_e, v_e, eager_captured = _run(False)
    assert captured and not eager_captured
    for a, b in zip(z_g, z_e):
        assert np.array_equal(a, b)
    for a, b in zip(v_g, v_e):
        assert np.array_equal(a, b)
