"""Child process of tests/test_gpu_rccl.py: a one-rank RCCL process group next to
liblgs_hip.so's HIP runtime, driving the benchmark's aggregation
(StreamingShard.reduce -> allreduce_parts) and imhk_sharded (all-reduce +
all-gather) with device tensors.  Prints one JSON line; exits non-zero on a
mismatch."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path[:0] = [os.path.join(REPO, "lattice-gaussian-mcmc_amd"), HERE]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from lgs_amd import _capi, distributed as D  # noqa: E402
from lgs_amd.lattices import build_config  # noqa: E402


def main():
    D.init_process_group("nccl", 0, 1)
    assert dist.get_backend() == "nccl" and D.collective_active()
    dev = torch.device("cuda", 0)
    lat, sigma = build_config("C2_qary128")
    B = lat.basis
    d = B.shape[0]
    Q, R = np.linalg.qr(B)
    R = np.ascontiguousarray(R * np.where(np.diag(R) < 0, -1.0, 1.0)[:, None])
    ctx = _capi.Context(0)
    ctx.set_basis(R, np.zeros(d), B, sigma)
    out = {}
    # 1. the bench's timed path: StreamingShard over the C-ABI, reduced through RCCL
    nc, T = 512, 8
    adv = D.gpu_advance(ctx, 77, 0, nc, d, dev, flags=_capi.LGS_WANG_LING, block_steps=T)
    sh = D.StreamingShard(adv, nc, d, binv_row=np.linalg.inv(B)[d - 1], device=dev, lag_chains=256, lags=6)
    for _ in range(3):
        sh.step(T)
    local = [sh.acc.sum().reshape(1), sh.mom] + sh.lag_z.parts() + sh.lag_v.parts()
    local = [x.clone() for x in local]
    red = sh.reduce()
    got = [red["accepts"], red["moments"]] + red["lag_z"] + red["lag_v"]
    assert all(g.device.type == "cuda" for g in got)
    for a, b in zip(local, got):
        assert torch.equal(a.to(b.dtype), b), "StreamingShard.reduce through RCCL changed the values"
    out["stream_accepts"] = int(red["accepts"][0])
    # 2. imhk_sharded with device tensors: all-reduce of accepts / moments / gram,
    #    all-gather of per-chain statistics
    comp = D.gpu_compute(ctx, 91, d, thin=2, flags=_capi.LGS_WANG_LING, device=dev, want_gram=True, gr_coord=d - 1)
    direct = D.gpu_compute(ctx, 91, d, thin=2, flags=_capi.LGS_WANG_LING, device=dev, want_gram=True,
                           gr_coord=d - 1)(first_chain=0, n_chains=64, first_step=1, n_steps=6)
    js = D.imhk_sharded(comp, 64, 6, rank=0, world=1, device=dev)
    assert js.accepts == direct.accepts and js.kept == direct.kept == 64 * 3
    assert np.array_equal(js.moments, direct.moments)
    assert np.array_equal(js.gram, direct.gram)
    assert np.array_equal(js.chain_stats, direct.chain_stats)
    out["sharded_accepts"] = js.accepts
    maps = open("/proc/self/maps").read()
    out["liblgs_hip_loaded"] = "liblgs_hip.so" in maps
    out["rccl_loaded"] = "librccl" in maps
    out["backend"] = dist.get_backend()
    dist.destroy_process_group()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
