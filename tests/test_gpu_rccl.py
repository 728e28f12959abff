"""GPU: RCCL next to liblgs_hip.so in one process.

A fresh child process initialises a one-rank "nccl" (= RCCL) process group on
cuda:0, loads the HIP library, and runs the benchmark's aggregation
(lgs_amd.distributed.StreamingShard.reduce -> allreduce_parts, the exact code
bench.py times) and imhk_sharded with device tensors (all-reduce + all-gather);
the reduced values must equal the local ones (tests/_rccl_child.py)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def test_rccl_one_rank_aggregation_equals_local():
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    env.pop("MASTER_ADDR", None)
    env.pop("RANK", None)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(HERE, "_rccl_child.py")], env=env, capture_output=True,
                       text=True, timeout=100)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["backend"] == "nccl" and out["liblgs_hip_loaded"] and out["rccl_loaded"], out
    assert out["stream_accepts"] > 0 and out["sharded_accepts"] > 0
