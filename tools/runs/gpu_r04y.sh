# B z: the ||v||^2 rows in a launch of their own (bzsplit); moments: the zero flags
# decided per workgroup (momwg); against the current library (base)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
V=lattice-gaussian-mcmc_amd/build/var
for lib in bzsplit momwg; do
  echo "== stream/parity tests $lib" && LGS_LIB=$V/$lib.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_stream.py tests/test_gpu_parity.py 2>&1 | tail -1 || exit 1
done
for r in 1 2; do for lib in $V/bzsplit.so $V/momwg.so lattice-gaussian-mcmc_amd/lgs_amd/_lib/liblgs_hip.so; do
echo "== $lib" && LGS_LIB=$lib timeout -k 10 300 python bench.py --no-cpu > gpurun_out/r04y_b.log 2>&1 || { tail -5 gpurun_out/r04y_b.log; exit 1; }
tail -1 gpurun_out/r04y_b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['kernel_ms'], d['parity_check'][:12], d['covariance']['sum_zzT_sha256'], d['autocorrelation']['z_last'][1])"
done; done
