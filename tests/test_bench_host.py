"""Host logic of bench.py's timed path (CPU), which lives in lgs_amd.distributed:
the lag-L autocovariance sums carried across bench steps, the exact
int64-in-fp64 packing of the single all-reduce, a gloo world-2 reduction that
equals the single-process statistics, and the counters' build-id check."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
from lgs_amd import distributed as D  # noqa: E402


def _direct(x, L):
    """sum_t x_t x_{t-k} and pair counts over whole series (n_chains x T)."""
    S = [float((x[:, k:] * x[:, :x.shape[1] - k]).sum()) for k in range(L + 1)]
    N = [x.shape[0] * (x.shape[1] - k) for k in range(L + 1)]
    return np.array(S), np.array(N)


@pytest.mark.parametrize("T,L", [(64, 16), (5, 16), (16, 16), (1, 3)])
def test_lag_sums_across_blocks_equal_whole_series(T, L):
    rng = np.random.default_rng(T + L)
    x = rng.integers(-50, 50, (7, 6 * T)).astype(np.int64)
    acc = D.LagSums(torch, 7, L, torch.int64, "cpu")
    for b in range(6):
        acc.update(torch.from_numpy(x[:, b * T:(b + 1) * T]))
    S, N = _direct(x, L)
    np.testing.assert_array_equal(acc.S.numpy(), S)
    np.testing.assert_array_equal(acc.N, N)
    assert int(acc.S1) == x.sum() and int(acc.n) == x.size
    a = D.LagSums.acf(S, N, float(x.sum()), float(x.size))
    assert a[0] == pytest.approx(1.0)


def test_pack_unpack_exact_int64():
    ints = torch.tensor([0, 1, -1, 2**62 - 5, -(2**61) + 3], dtype=torch.int64)
    f = torch.tensor([1.5, -2.25])
    flat, layout = D.pack_f64(torch, [ints, f])
    a, b = D.unpack_f64(torch, flat, layout)
    assert torch.equal(a, ints) and torch.equal(b, f)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, x, out):
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "lattice-gaussian-mcmc_amd"))
    import torch.distributed as dist
    from lgs_amd import distributed as bm
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    half = x.shape[0] // world
    mine = x[rank * half:(rank + 1) * half]
    acc = bm.LagSums(torch, half, 8, torch.int64, "cpu")
    for b in range(4):
        acc.update(torch.from_numpy(mine[:, b * 10:(b + 1) * 10]))
    out[rank] = [t.numpy().tolist() for t in bm.allreduce_parts(acc.parts())]
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_gloo_world2_lag_sums_match_single_process():
    x = np.random.default_rng(3).integers(-9, 9, (8, 40)).astype(np.int64)
    mgr = mp.Manager()
    out = mgr.dict()
    mp.start_processes(_worker, args=(2, _free_port(), x, out), nprocs=2, join=True, start_method="spawn")
    single = D.LagSums(torch, 8, 8, torch.int64, "cpu")
    for b in range(4):
        single.update(torch.from_numpy(x[:, b * 10:(b + 1) * 10]))
    for r in (0, 1):
        S, N, S1, n = out[r]
        assert S == single.S.tolist() and N == single.N.tolist()
        assert S1 == single.S1.tolist() and n == [single.n]


def test_counters_used_only_for_the_same_build(tmp_path):
    import json
    p = tmp_path / "x_klein_counters.json"
    p.write_text(json.dumps({"config": "C3_ntru512", "build_id": "abc", "fp64_flops": 1.0}))
    cnt, path, state = bench.load_counters(str(p), "C3_ntru512", "abc")
    assert state == "current" and cnt["fp64_flops"] == 1.0
    cnt, path, state = bench.load_counters(str(p), "C3_ntru512", "def")
    assert state == "stale" and cnt is None
    lib = tmp_path / "lib.so"
    lib.write_bytes(b"\x7fELF...")
    assert bench.build_id(str(lib)) == bench.build_id(str(lib)) and len(bench.build_id(str(lib))) == 16
