"""The C restatement (oracle/lgs_oracle.c) under AddressSanitizer + UndefinedBehavior-
Sanitizer (race detection / sanitizers): `make -C oracle sanitize`
builds the same source with -fsanitize=address,undefined -fno-sanitize-recover=all,
and tests/test_oracle.py -- the published seed-42 KATs, the reference-generated
golden vectors, the OpenMP-parallel IMHK -- runs against it in a child Python with
libasan preloaded.  Any out-of-bounds access, use-after-free or undefined
behaviour aborts the child.  CPU only."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _libasan():
    try:
        p = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True, check=True)
    except (OSError, subprocess.CalledProcessError):
        return None
    path = p.stdout.strip()
    return path if os.path.isabs(path) and os.path.exists(path) else None


def test_oracle_suite_under_asan_ubsan():
    asan = _libasan()
    if asan is None:
        pytest.skip("gcc's libasan is not available")
    subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "oracle"), "sanitize"])
    san = os.path.join(REPO, "oracle", "_build", "liblgs_oracle_san.so")
    env = dict(os.environ, LD_PRELOAD=asan, LGS_ORACLE_LIB=san,
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1", OMP_NUM_THREADS="4")
    # the child really runs the instrumented library
    probe = ("import ctypes, sys; sys.path.insert(0, 'oracle'); import lgs_oracle as o; o.lib(); "
             "assert o._LIB_PATH.endswith('_san.so'); "
             "assert hasattr(ctypes.CDLL(None), '__asan_init'); print('asan active')")
    out = subprocess.run([sys.executable, "-c", probe], cwd=REPO, env=env, capture_output=True, text=True,
                         timeout=120)
    assert out.returncode == 0 and "asan active" in out.stdout, out.stderr[-2000:]
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider",
                        os.path.join(REPO, "tests", "test_oracle.py")],
                       cwd=REPO, env=env, capture_output=True, text=True, timeout=900)
    tail = (r.stdout + r.stderr)[-3000:]
    assert r.returncode == 0, tail
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error:" not in r.stderr, tail
